#!/bin/bash
# round 5: per-wave durations of the C3 and C4 semi-implicit launches split by the wave's done envs
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r05ab2; mkdir -p $out
timeout -k 10 200 python -u tools/wavetime.py MuscleWalkingImitation2D-v0 > $out/wavetime_done_c3.log 2>&1 &&
timeout -k 10 300 python -u tools/wavetime.py MuscleRunningImitation3D-v0 > $out/wavetime_done_c4.log 2>&1
echo exit $?
