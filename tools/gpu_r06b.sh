#!/bin/bash
# round 6 call b: the realize cache — whole GPU suite, then a same-box A/B against the
# build without it (-DBIOIM_REALIZE_CACHE=0) and the SQ VALU/LDS pass of the C3 kernel
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06b; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
echo tests exit $?
timeout -k 10 600 bash tools/ab.sh $out/ab_cache 3 MuscleWalkingImitation2D-v0 tree bioimitation-gym_amd/build/ab/nocache/libbioim.so > $out/ab_cache.txt 2>&1 || exit 1
for v in tree nocache; do
  if [ $v = tree ]; then unset BIOIM_LIB; else export BIOIM_LIB=$PWD/bioimitation-gym_amd/build/ab/$v/libbioim.so; fi
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
     --output-format csv -d $GRAFT_REPO_ROOT/$out/pmc_$v -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline \
     --no-reference-integrator --no-single-env > $GRAFT_REPO_ROOT/$out/pmc_$v.log 2>&1) || exit 1
done
unset BIOIM_LIB

# the Palsy3D drive's GPU/twin ratio on builds with the oracle's operations
for v in exactrcp nocontract exactnc; do
  BIOIM_LIB=$PWD/bioimitation-gym_amd/build/ab/$v/libbioim.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 380 --timeout-method thread \
    -k "muscle_tracking_drive and Palsy" > $out/palsy_$v.log 2>&1
  echo palsy $v exit $?
done
echo done
