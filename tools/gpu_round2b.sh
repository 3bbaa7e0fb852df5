#!/bin/bash
# Round-2 evidence on one GPU box for the current build: GPU tests, smoke,
# the headline bench line (CPU baseline, reference integrator) and the other
# configs' lines.   bash tools/gpu_round2b.sh <out-dir>
set -e
out=$1; mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python bench.py > "$out/bench_fp64.json" 2> "$out/bench_fp64.err"
timeout -k 10 120 python bench.py --no-cpu-baseline --env-id TorqueWalkingImitation2D-v0 > "$out/bench_torque2d.json"
timeout -k 10 120 python bench.py --no-cpu-baseline --env-id MuscleRunningImitation3D-v0 > "$out/bench_3d.json"
timeout -k 10 120 python bench.py --no-cpu-baseline --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 > "$out/bench_mixed.json"
timeout -k 10 120 python bench.py --no-cpu-baseline --precision 32 > "$out/bench_fp32.json"
timeout -k 10 300 python bench.py --no-cpu-baseline --env-id MuscleRunningImitation3D-v0 --integrator rk-merson --rk-budget 6 > "$out/bench_rk3d_budget6.json"
timeout -k 10 300 python bench.py --no-cpu-baseline --env-id TorqueWalkingImitation2D-v0 --integrator rk-merson --rk-budget 6 > "$out/bench_rkt2d_budget6.json"
echo done
