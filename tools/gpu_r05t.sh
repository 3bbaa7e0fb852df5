#!/bin/bash
# Round 5, GPU call t: kernel time / termination rate by window after the
# fresh start; planar past-end exit A/B in the driver's 20-step window and
# in the 200-step window.
set -e
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 200 python tools/window_probe.py MuscleWalkingImitation2D-v0 600 > $O/window_2d.log 2>&1
B=$PWD/bioimitation-gym_amd/build/ab
BENCH_ARGS="--steps 20 --warmup 5" bash tools/ab.sh $O/ab20 3 MuscleWalkingImitation2D-v0 tree $B/pe2d/libbioim.so > $O/ab20.log 2>&1
bash tools/ab.sh $O/ab200 3 MuscleWalkingImitation2D-v0 tree $B/pe2d/libbioim.so > $O/ab200.log 2>&1
echo done
