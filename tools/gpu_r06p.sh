#!/bin/bash
# round 6 call p: the C3 kernel with the post-RA machine scheduler run
# bottom-up (p1) or bidirectionally (p2) instead of top-down
# (python tools/build_variants.py --units topo1 p1=-mllvm,-misched-postra-direction=bottomup
#  p2=-mllvm,-misched-postra-direction=bidirectional; -misched-limit=1024 and
# -misched-cyclicpath compile to the tree's instructions): C3 parity tests,
# then a same-box A/B against the tree
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06p; mkdir -p $out
B=$PWD/bioimitation-gym_amd/build/ab
for v in p1 p2; do
  BIOIM_LIB=$B/$v/libbioim.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "MuscleWalkingImitation2D" > $out/tests_$v.log 2>&1 || { echo "tests $v failed"; exit 1; }
  tail -1 $out/tests_$v.log
done
timeout -k 10 900 bash tools/ab.sh $out/ab_c3 4 MuscleWalkingImitation2D-v0 tree $B/p1/libbioim.so $B/p2/libbioim.so \
  > $out/ab_c3.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/ab_c3.txt
echo done
