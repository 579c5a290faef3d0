#!/bin/bash
# Dev: the crash-leg / C2 variant A/B alone.
set -o pipefail
bash tools/crash_var.sh
