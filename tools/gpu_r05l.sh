#!/bin/bash
# Round 5, GPU call l: GPU suite with the torque models' reset table, then
# the reset table A/B on the torque configs and bench lines of C3/C4/C5.
set -e
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
bash tools/ab_flags.sh $O/ab 3 "TorqueWalkingImitation2D-v0;TorqueWalkingImitation3D-v0;MuscleWalkingImitation2D-v0;mixed:MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0" tab= notab=--no-reset-table > $O/ab.log 2>&1
echo done
