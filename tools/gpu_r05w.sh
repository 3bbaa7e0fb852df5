#!/bin/bash
# round 5 call w: bioim_finished_count (RK budget tests), per-wave durations of the budgeted RK
# launches (C3, C4) and of the semi-implicit C3 launch, the default bench line
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r05w; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rk_budget.py > $out/test_rk_budget.log 2>&1 &&
timeout -k 10 200 python -u tools/wavetime.py MuscleWalkingImitation2D-v0 --rk > $out/wavetime_rk_c3.log 2>&1 &&
timeout -k 10 300 python -u tools/wavetime.py MuscleRunningImitation3D-v0 --rk > $out/wavetime_rk_c4.log 2>&1 &&
timeout -k 10 200 python -u tools/wavetime.py MuscleWalkingImitation2D-v0 > $out/wavetime_c3.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $out/bench_c3.json 2> $out/bench_c3.err &&
timeout -k 10 400 python -u bench.py --env-id MuscleRunningImitation3D-v0 > $out/bench_c4.json 2> $out/bench_c4.err
echo exit $?
