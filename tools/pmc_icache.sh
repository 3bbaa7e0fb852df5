#!/bin/bash
# Instruction-cache / wait counters for the env kernel (one pass per group).
TAG=${1:-ic}; PREC=${2:-64}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pmc_${TAG}_fp${PREC}
mkdir -p $OUT
export BIOIM_PRECISION=$PREC
ARGS="--steps 5 --warmup 2 --no-cpu-baseline"
i=0
for G in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" \
         "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_ANY SQ_INSTS" \
         "SQC_TC_INST_REQ SQC_TC_STALL SQC_DCACHE_HITS SQC_DCACHE_MISSES"; do
    i=$((i+1))
    (cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o p$i -- \
        python3 $OLDPWD/bench.py $ARGS > $OUT/p$i.log 2>&1)
    rc=$?
    echo "pass $i ($G): rc=$rc"
    if [ $rc -ge 124 ]; then exit $rc; fi
done
