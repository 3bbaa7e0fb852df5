#!/bin/bash
# round 6 call i: the final round-6 build against the final round-5 build (16658a1e25677762, rebuilt
# from its commit into build/ab/r05), same box: semi-implicit lines of C3 / C2 / C4 / LockedKnee3D /
# Palsy3D, the reference-integrator legs of C3 and C4, and C5 fused (bench --mixed)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06i; mkdir -p $out
R05=$PWD/bioimitation-gym_amd/build/ab/r05/libbioim.so
timeout -k 10 900 bash tools/ab.sh $out/ab 3 MuscleWalkingImitation2D-v0,TorqueWalkingImitation2D-v0,MuscleRunningImitation3D-v0,MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 \
  tree $R05 > $out/ab.txt 2>&1 || exit 1
BENCH_ARGS="--integrator rk-merson --rk-budget 6 --steps 100" timeout -k 10 600 bash tools/ab.sh $out/ab_rk 2 \
  MuscleWalkingImitation2D-v0,MuscleRunningImitation3D-v0 tree $R05 > $out/ab_rk.txt 2>&1 || exit 1
for r in 1 2; do
  for v in tree r05; do
    if [ $v = tree ]; then unset BIOIM_LIB; else export BIOIM_LIB=$R05; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-reference-integrator --no-single-env \
      --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 > $out/c5_${v}_$r.json 2>> $out/c5.err || exit 1
  done
done
echo done
