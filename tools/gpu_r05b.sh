#!/bin/bash
# Round 5, GPU call b: instruction-cost microbenchmark, VALU census by class,
# fiber-velocity warm-start variants A/B, the new GPU tests.
set -e
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 60 tools/ubench/lat2 > $O/lat2.log 2>&1
bash tools/pmc_census.sh r05b_census > $O/census.log 2>&1
python tools/pmc_summary.py gpurun_out/pmc_r05b_census > $O/census_summary.txt
B=$PWD/bioimitation-gym_amd/build/ab
bash tools/ab.sh $O/ab 3 MuscleWalkingImitation2D-v0,MuscleRunningImitation3D-v0 tree $B/fvh/libbioim.so $B/fvp/libbioim.so $B/fvhp/libbioim.so > $O/ab.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "c5_fused or fp32_free_running or mixed_batch or rk_analyses or storage_overflow" > $O/tests.log 2>&1
echo done
