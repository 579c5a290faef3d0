#!/bin/bash
# Dev: crash_leg call time per variant in tools/variants, interleaved.
set -o pipefail
for rep in 1 2; do
  for v in $(ls tools/variants); do
    echo "$v $(LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 120 python tools/crash_call.py 3 2>/dev/null | tr '\n' ' ')" || exit 1
  done
done
