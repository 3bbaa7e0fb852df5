#!/bin/bash
# Budgeted RK-Merson steps (bioim_set_rk_budget) on one GPU box: the parity
# tests, then bench lines per budget for 2D and 3D, then the default-kernel
# A/B against a baseline library (no regression from the new state arrays).
#   bash tools/gpu_rk_budget.sh <out-dir> [baseline.so]
set -e
out=$1; base=$2; mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_rk_budget.py -x -v --timeout 240 --timeout-method thread > "$out/gpu_rk_budget_tests.log" 2>&1
for id in MuscleWalkingImitation2D-v0 MuscleRunningImitation3D-v0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --env-id $id --integrator rk-merson --steps 40 --warmup 5 --burn-in 20 > "$out/bench_rk_sync_$id.json"
  for b in 16 32 64; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --env-id $id --integrator rk-merson --rk-budget $b --steps 100 --warmup 10 --burn-in 40 > "$out/bench_rk_b${b}_$id.json"
  done
done
if [ -n "$base" ]; then bash tools/ab.sh "$out/ab" 2 MuscleWalkingImitation2D-v0,MuscleRunningImitation3D-v0 tree "$base"; fi
echo done
