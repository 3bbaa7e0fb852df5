#!/bin/bash
# SQ instruction-mix / stall counters for the env kernel, one rocprofv3 pass
# per counter group (no tracing domains combined with --pmc).
#   bash tools/pmc_sq.sh <tag> [precision] [env id]
TAG=${1:-sq}; PREC=${2:-64}; ENV=${3:-MuscleWalkingImitation2D-v0}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_fp${PREC}
[ -z "$GRAFT_REPO_ROOT" ] && OUT=$(pwd)/gpurun_out/pmc_${TAG}_fp${PREC}
mkdir -p $OUT
export BIOIM_PRECISION=$PREC
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-reference-integrator --no-single-env --env-id $ENV"
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY" \
         "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU"; do
    i=$((i+1))
    (cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o p$i -- \
        python3 $OLDPWD/bench.py $ARGS > $OUT/p$i.log 2>&1)
    rc=$?
    echo "pass $i ($G): rc=$rc"
    if [ $rc -ge 124 ]; then exit $rc; fi
done
