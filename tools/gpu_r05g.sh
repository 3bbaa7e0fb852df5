#!/bin/bash
# Round 5, GPU call g: GPU suite on the build with the planar RK reset table,
# then the reference-integrator leg A/B (reset table on / off) on C3.
set -e
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
bash tools/ab_flags.sh $O/ab 3 "MuscleWalkingImitation2D-v0" "tab=--integrator rk-merson --rk-budget 6" "notab=--integrator rk-merson --rk-budget 6 --no-reset-table" > $O/ab.log 2>&1
echo done
