#!/bin/bash
# round 6 call g: fiber-velocity predictor (BIOIM_FV_PRED=1: linear extrapolation of the previous two
# substeps' roots) re-measured now that every substep of a launch is warm-started (the realize cache)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06g; mkdir -p $out
timeout -k 10 600 bash tools/ab.sh $out/ab_fvpred 3 MuscleWalkingImitation2D-v0 tree \
  bioimitation-gym_amd/build/ab/fvpred/libbioim.so > $out/ab_fvpred.txt 2>&1
echo ab exit $?
