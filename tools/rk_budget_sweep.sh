#!/bin/bash
# Finished env steps/s of budgeted RK-Merson launches over a range of
# budgets (attempt-equivalents of 5 dynamics evaluations per launch) at the
# default burn-in (150 + 20 env steps; budgeted runs burn in by finished
# steps).  GPU box:
#   bash tools/rk_budget_sweep.sh <out-dir> [budgets...] 
set -e
out=$1; shift; mkdir -p "$out"
budgets=${@:-"2 3 4 5 6 8"}
for id in MuscleWalkingImitation2D-v0 MuscleRunningImitation3D-v0 TorqueWalkingImitation2D-v0; do
  for b in $budgets; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --env-id $id --integrator rk-merson --rk-budget $b --steps 200 > "$out/bench_rk_b${b}_$id.json"
  done
done
echo done
