#!/bin/bash
# round 6 call l: the report after an inner integrate-and-realize loop
# (-DBIOIM_RK_BATCH=1, build/ab/rkb: every kernel but the fused C5 pair, which
# is the tree's object — the hazard gate flags one copy in it under the flag):
# the GPU suite on it, then same-box A/Bs of the semi-implicit lines (C3, C2,
# C4, C5 as concurrent per-segment launches) and the reference-integrator legs
# (C3, C2, C4).  Not shipped: the variant is
# profiles/r06/r06l/rk_batch_nested_loops.patch applied to the tree, then
# python tools/build_variants.py --units abi,topo0,...,topo6 rkb=-DBIOIM_RK_BATCH=1
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06l; mkdir -p $out
V=$PWD/bioimitation-gym_amd/build/ab/rkb/libbioim.so
BIOIM_LIB=$V timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > $out/gpu_tests_rkb.log 2>&1
echo tests exit $?
tail -3 $out/gpu_tests_rkb.log
timeout -k 10 900 bash tools/ab.sh $out/ab_semi 4 \
  MuscleWalkingImitation2D-v0,TorqueWalkingImitation2D-v0,MuscleRunningImitation3D-v0 tree $V > $out/ab_semi.txt 2>&1 || exit 1
cat $out/ab_semi.txt
BENCH_ARGS="--integrator rk-merson --rk-budget 6 --steps 200" timeout -k 10 900 bash tools/ab.sh $out/ab_rk 3 \
  MuscleWalkingImitation2D-v0,TorqueWalkingImitation2D-v0,MuscleRunningImitation3D-v0 tree $V > $out/ab_rk.txt 2>&1 || exit 1
cat $out/ab_rk.txt
for r in 1 2 3; do
  for v in tree rkb; do
    if [ $v = tree ]; then unset BIOIM_LIB; else export BIOIM_LIB=$V; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-reference-integrator --no-single-env \
      --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 --no-fuse > $out/c5_${v}_$r.json 2>> $out/c5.err || exit 1
  done
done
unset BIOIM_LIB
python3 - $out <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + '/c5_*.json')):
    j = json.load(open(f)); print(f.split('/')[-1], j['ms_per_step'], j['value'] / 1e6)
PY
echo done
