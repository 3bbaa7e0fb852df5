#!/bin/bash
# Round 5, GPU call o: phase stamps of the current kernels (diagnostic build),
# then a same-box A/B of two sched_group_barrier pipelines in the muscle eval.
set -e
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 200 python tools/stamps.py 64 MuscleWalkingImitation2D-v0 > $O/stamps_2d.log 2>&1
timeout -k 10 200 python tools/stamps.py 64 MuscleRunningImitation3D-v0 > $O/stamps_3d.log 2>&1
B=$PWD/bioimitation-gym_amd/build/ab
bash tools/ab.sh $O/ab 3 MuscleWalkingImitation2D-v0 tree $B/sgb1/libbioim.so $B/sgb2/libbioim.so > $O/ab.log 2>&1
echo done
