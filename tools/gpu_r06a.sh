#!/bin/bash
# round 6 call a: the new reset-table / RK-counter / storage tests
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06a; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "reset_table or c4_auto_reset or rk_counters or storage_overflow or rk_budget_equals" > $out/gpu_tests.log 2>&1
echo tests exit $?
# odd-double per-env LDS strides (the two envs of a 32-lane group on opposite bank pairs)
timeout -k 10 900 bash tools/ab.sh $out/ab_envmod 3 MuscleWalkingImitation2D-v0,TorqueWalkingImitation2D-v0 tree \
  bioimitation-gym_amd/build/ab/envmod17/libbioim.so bioimitation-gym_amd/build/ab/envmod15/libbioim.so > $out/ab_envmod.txt 2>&1
echo ab exit $?
for v in tree envmod17; do
  if [ $v = tree ]; then unset BIOIM_LIB; else export BIOIM_LIB=$PWD/bioimitation-gym_amd/build/ab/$v/libbioim.so; fi
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU \
     --output-format csv -d $GRAFT_REPO_ROOT/$out/pmc_$v -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline \
     --no-reference-integrator --no-single-env > $GRAFT_REPO_ROOT/$out/pmc_$v.log 2>&1) || exit 1
done
unset BIOIM_LIB
echo done
