#!/bin/bash
# round 5 call x: report cost per env step (stamps build): C3 semi-implicit, C3 RK budgeted, C4
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r05x; mkdir -p $out
timeout -k 10 200 python -u tools/stamps.py 64 MuscleWalkingImitation2D-v0 > $out/stamps_2d.log 2>&1 &&
timeout -k 10 200 python -u tools/stamps.py 64 MuscleWalkingImitation2D-v0 --rk > $out/stamps_2d_rk.log 2>&1 &&
timeout -k 10 200 python -u tools/stamps.py 64 MuscleRunningImitation3D-v0 > $out/stamps_3d.log 2>&1
echo exit $?
