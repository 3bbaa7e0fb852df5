#!/bin/bash
# round 6 call k: the RK-Merson finished envs of a wave report together
# (-DBIOIM_RK_BATCH=1, planar kernels, build/ab/rkb): its RK GPU tests, then a
# same-box A/B of the reference-integrator legs (C3, C2).  Not shipped: the
# variant is profiles/r06/r06k/rk_batch_ballot_hold.patch applied to the tree,
# then python tools/build_variants.py --units topo0,topo1,topo4 rkb=-DBIOIM_RK_BATCH=1
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06k; mkdir -p $out
V=$PWD/bioimitation-gym_amd/build/ab/rkb/libbioim.so
BIOIM_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "reset_table or rk_merson or rk_budget or rk_counters or mixed_batch_rk or realize_report or rllib" > $out/gpu_tests_rkb.log 2>&1
echo tests exit $?
tail -3 $out/gpu_tests_rkb.log
BENCH_ARGS="--integrator rk-merson --rk-budget 6 --steps 200" timeout -k 10 900 bash tools/ab.sh $out/ab_rk 3 \
  MuscleWalkingImitation2D-v0,TorqueWalkingImitation2D-v0 tree $V > $out/ab_rk.txt 2>&1 || exit 1
cat $out/ab_rk.txt
echo done
