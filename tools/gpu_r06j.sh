#!/bin/bash
# round 6 call j: long-run soak of the final build (tools/soak.py)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06j; mkdir -p $out
timeout -k 10 600 python -u tools/soak.py 3000 > $out/soak.log 2>&1
echo soak exit $?
