#!/bin/bash
# The 32-lanes-per-env spatial muscle build on the GPU
# box: its parity on the spatial muscle IDs, a same-box A/B against the tree
# build (16 lanes), and its SQ counters.  Build it first (CPU):
#   python -c "import __graft_entry__ as g; g.build_lib(out='bioimitation-gym_amd/build/ab/g32/libbioim.so',
#              extra=['-DBIOIM_G_SPATIAL_MUSCLE=32'])"
#   bash tools/gpu_g32.sh <tag>
set -e
TAG=${1:-r04d}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
G32=$PWD/bioimitation-gym_amd/build/ab/g32/libbioim.so
BIOIM_LIB=$G32 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -v \
    --timeout 300 --timeout-method thread -k "MuscleRunningImitation3D or MuscleLockedKneeImitation3D or MusclePalsyImitation3D" \
    > $O/g32_parity.log 2>&1
bash tools/ab.sh $O/ab 3 MuscleRunningImitation3D-v0,MuscleLockedKneeImitation3D-v0 tree $G32 > $O/ab.log 2>&1
BIOIM_LIB=$G32 bash tools/pmc_sq.sh ${TAG}_g32_3d 64 MuscleRunningImitation3D-v0 > $O/pmc_g32.log 2>&1
bash tools/pmc_sq.sh ${TAG}_g16_3d 64 MuscleRunningImitation3D-v0 > $O/pmc_g16.log 2>&1
echo done
