#!/bin/bash
# round 5 call z: the driver's command after moving the counter reads before the warm-up (3 runs),
# a 200-step line, and the --rk-budget main path
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r05z; mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/driver_$i.json 2>> $out/bench.err || exit 1
done
timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --no-single-env > $out/s200.json 2>> $out/bench.err &&
timeout -k 10 300 python bench.py --integrator rk-merson --rk-budget 6 --steps 50 --no-cpu-baseline --no-single-env > $out/rkb.json 2>> $out/bench.err
echo exit $?
