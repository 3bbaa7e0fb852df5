#!/bin/bash
# round 5 call v: RK leg probe (ready-count overhead, budget sweep incl. B < 6)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r05v; mkdir -p $out
timeout -k 10 280 python -u tools/rk_probe.py MuscleWalkingImitation2D-v0 --budgets 4,5,6,7 --rounds 2 > $out/rk_probe_c3.log 2>&1 &&
timeout -k 10 400 python -u tools/rk_probe.py MuscleRunningImitation3D-v0 --budgets 4,5,6,7 --rounds 2 > $out/rk_probe_c4.log 2>&1
echo exit $?
