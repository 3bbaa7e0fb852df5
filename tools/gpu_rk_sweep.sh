#!/bin/bash
# Reference-integrator launch budget sweep on the shipped build (finished env
# steps/s at 4096 envs, RK-Merson 1e-3) for C3, C2 and C4; plus the fp32 RK
# budget tests.
set -e
O=gpurun_out/${1:-r04i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rk_budget.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $O/rk_budget_tests.log 2>&1
for E in MuscleWalkingImitation2D-v0 TorqueWalkingImitation2D-v0 MuscleRunningImitation3D-v0; do
  for B in 3 4 5 6 8; do
    timeout -k 10 120 python bench.py --env-id $E --integrator rk-merson --rk-budget $B --steps 100 --no-cpu-baseline --no-single-env --no-reference-integrator > $O/sweep_${E}_B$B.json 2>> $O/sweep.err
  done
done
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], 'sweep_*.json'))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), f"{d['value'] / 1e6:.3f} M finished/s", f"{d['roofline']['kernel_ms']:.4f} ms/launch",
          f"evals/step {d.get('evals_per_env_step', 0):.1f}")
PY
