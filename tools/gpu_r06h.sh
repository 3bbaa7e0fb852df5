#!/bin/bash
# round 6 call h: the realize-cache first-substep test; the driver's command with the counter read
# moved 20 burn-in steps ahead (bench.py) against the previous bench.py, alternating, 3 each
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06h; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "realize_cache" > $out/gpu_tests.log 2>&1
echo tests exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-env > $out/new_$i.json 2>> $out/bench.err || exit 1
  timeout -k 10 300 python bench_prev.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-single-env > $out/prev_$i.json 2>> $out/bench.err || exit 1
done
echo done
