#!/bin/bash
# One GPU-box pass: parity tests, smoke, default bench (with CPU baseline),
# fp32 bench, kernel trace + HBM traffic passes, SQ counter passes.
# Each GPU step under its own time limit; stop at the first failure.
set -e
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -rA > gpurun_out/${TAG}_gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
BIOIM_PRECISION=32 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_fp32.json 2>> gpurun_out/${TAG}_bench.err
bash tools/profile_round.sh $TAG 64
bash tools/pmc_sq.sh $TAG 64
