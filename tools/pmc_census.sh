#!/bin/bash
# VALU instruction census by class for the env kernel (round 5): one
# rocprofv3 --pmc pass per counter group, no tracing domains combined.
#   bash tools/pmc_census.sh <tag> [env id]
# Summarise with: python tools/pmc_summary.py gpurun_out/pmc_<tag>
TAG=${1:-census}; ENV=${2:-MuscleWalkingImitation2D-v0}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${TAG}
mkdir -p $OUT
ARGS="--steps 5 --warmup 2 --burn-in 20 --no-cpu-baseline --no-reference-integrator --no-single-env --env-id $ENV"
i=0
for G in "SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT" \
         "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o p$i -- \
        python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1)
    rc=$?
    echo "pass $i: rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
done
