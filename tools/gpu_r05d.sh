#!/bin/bash
# Round 5, GPU call d: the whole GPU suite on the reset-table build, then a
# same-box A/B of the reset table (on / off) on C3, C4 and C5.
set -e
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
bash tools/ab_flags.sh $O/ab 3 "MuscleWalkingImitation2D-v0;MuscleRunningImitation3D-v0;mixed:MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0" tab= notab=--no-reset-table > $O/ab.log 2>&1
echo done
