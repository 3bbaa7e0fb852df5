#!/bin/bash
# round 6 call c: the realize cache in every muscle model (planar and spatial, C5 fused) — GPU suite,
# same-box A/B against -DBIOIM_REALIZE_CACHE=0 on C3 / C4 / LockedKnee3D / Palsy3D / C5, the Palsy3D diagnosis
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06c; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
echo tests exit $?
timeout -k 10 900 bash tools/ab.sh $out/ab_cache 3 MuscleWalkingImitation2D-v0,MuscleRunningImitation3D-v0,MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 \
  tree bioimitation-gym_amd/build/ab/nocache/libbioim.so > $out/ab_cache.txt 2>&1 || exit 1
for r in 1 2 3; do
  for v in tree nocache; do
    if [ $v = tree ]; then unset BIOIM_LIB; else export BIOIM_LIB=$PWD/bioimitation-gym_amd/build/ab/$v/libbioim.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-reference-integrator --no-single-env \
      --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 > $out/c5_${v}_$r.json 2>> $out/c5.err || exit 1
  done
done
unset BIOIM_LIB
timeout -k 10 300 python tools/diag_palsy_ratio.py > $out/diag_palsy.txt 2>&1
echo diag exit $?
echo done
