#!/bin/bash
set -o pipefail
for cfg in "TAG=default" "TAG=hostclear LC_FXQ_HOSTCLEAR=1" "TAG=g1 LC_FXQ_G=1" "TAG=g8 LC_FXQ_G=8" "TAG=level LC_FX_QUEUE=0"; do
  env LC_FX_QUEUE=1 $cfg timeout -k 10 120 python tools/fxq_debug.py || exit $?
done
