#!/bin/bash
# Finished env steps/s of budgeted RK-Merson launches over a range of
# budgets, and the unbudgeted line, at the default burn-in (150 + 20 env
# steps; budgeted runs burn in by finished steps).  GPU box:
#   bash tools/rk_budget_sweep.sh <out-dir>
set -e
out=$1; mkdir -p "$out"
for id in MuscleWalkingImitation2D-v0 MuscleRunningImitation3D-v0 TorqueWalkingImitation2D-v0; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --env-id $id --integrator rk-merson --steps 40 > "$out/bench_rk_sync_$id.json"
  for b in 6 8 12 16 32; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --env-id $id --integrator rk-merson --rk-budget $b --steps 200 > "$out/bench_rk_b${b}_$id.json"
  done
done
echo done
