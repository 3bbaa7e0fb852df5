#!/bin/bash
# One GPU-box evidence pass (run from the repo root on the box):
#   bench lines (2D fp64 headline with CPU baseline, 2D fp32, 3D Running, C5 mixed),
#   rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes (separate
#   runs, MI355X_MICROARCH.md rocprofv3 section) for the 2D and 3D kernels.
# Every GPU step has its own time limit; the script stops at the first failure.
#   bash tools/gpu_evidence.sh <tag>
set -e
TAG=${1:-r01}
O=gpurun_out/ev_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench_fp64.json 2> $O/bench.err
timeout -k 10 200 python bench.py --precision 32 --no-cpu-baseline > $O/bench_fp32.json 2>> $O/bench.err
timeout -k 10 200 python bench.py --env-id MuscleRunningImitation3D-v0 --no-cpu-baseline > $O/bench_3d_fp64.json 2>> $O/bench.err
timeout -k 10 200 python bench.py --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 > $O/bench_mixed_fp64.json 2>> $O/bench.err
for CFG in "2d:--env-id MuscleWalkingImitation2D-v0" "3d:--env-id MuscleRunningImitation3D-v0"; do
    K=${CFG%%:*}; A="${CFG#*:} --steps 20 --warmup 3 --no-cpu-baseline"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${K}_trace -o trace -- python3 bench.py $A > $O/${K}_trace.log 2>&1
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${K}_fetch -o fetch -- python3 bench.py $A > $O/${K}_fetch.log 2>&1
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${K}_write -o write -- python3 bench.py $A > $O/${K}_write.log 2>&1
done
find $O -name "*.csv" | sort
