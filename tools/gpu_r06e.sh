#!/bin/bash
# round 6 call e: the reset table in the spatial RK kernels (-DBIOIM_RESET_TAB_RK_SPATIAL=1, build/ab/rktab3d):
# its GPU tests, then a same-box A/B of the reference-integrator legs (C4, LockedKnee3D, Palsy3D, C5)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06e; mkdir -p $out
V=$PWD/bioimitation-gym_amd/build/ab/rktab3d/libbioim.so
BIOIM_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "reset_table or rk_merson or rk_budget or mixed_batch_rk or realize_report" > $out/gpu_tests_rktab3d.log 2>&1
echo tests exit $?
BENCH_ARGS="--integrator rk-merson --rk-budget 6 --steps 100" timeout -k 10 900 bash tools/ab.sh $out/ab_rk 3 \
  MuscleRunningImitation3D-v0,MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 tree $V > $out/ab_rk.txt 2>&1 || exit 1
for r in 1 2; do
  for v in tree rktab3d; do
    if [ $v = tree ]; then unset BIOIM_LIB; else export BIOIM_LIB=$V; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-reference-integrator --no-single-env --integrator rk-merson --rk-budget 6 \
      --steps 100 --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 > $out/c5rk_${v}_$r.json 2>> $out/c5.err || exit 1
  done
done
echo done
