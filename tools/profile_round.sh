#!/bin/bash
# Profile the bench kernel: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE
# in separate PMC passes (MI355X_MICROARCH.md rocprofv3 section).  Run on the
# GPU box from the repo root:  bash tools/profile_round.sh <tag> [precision]
# (EXTRA="--env-id ..." profiles another config)
set -e
TAG=${1:-r01}; PREC=${2:-64}
OUT=gpurun_out/prof_${TAG}_fp${PREC}
mkdir -p $OUT
export TMPDIR=/tmp BIOIM_PRECISION=$PREC
ARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-reference-integrator $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1
find $OUT -name "*.csv"
