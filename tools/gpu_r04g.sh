#!/bin/bash
# Round-4 GPU pass: full GPU suite on the tree build and on the BIOIM_CHECK
# build, smoke, the headline bench, and a same-box A/B of the RK kernels with
# the spatial branch-free pieces (build/ab/rkbf, -DBIOIM_BF3_RK=1).
set -e
O=gpurun_out/${1:-r04g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
BIOIM_LIB=$PWD/bioimitation-gym_amd/build/check/libbioim.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_check.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
BENCH_ARGS="--integrator rk-merson --rk-budget 6 --steps 100" bash tools/ab.sh $O/ab_rk 3 MuscleRunningImitation3D-v0,MuscleLockedKneeImitation3D-v0 tree $PWD/bioimitation-gym_amd/build/ab/rkbf/libbioim.so > $O/ab_rk.log 2>&1
echo done
