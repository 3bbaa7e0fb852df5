#!/bin/bash
# Round 5, GPU call p: GPU suite with the substep update through fast_rcp,
# then a same-box A/B against the IEEE division (variant -DBIOIM_SUBSTEP_RCP=0).
set -e
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
B=$PWD/bioimitation-gym_amd/build/ab
bash tools/ab.sh $O/ab 3 MuscleWalkingImitation2D-v0,MuscleRunningImitation3D-v0 tree $B/div/libbioim.so > $O/ab.log 2>&1
echo done
