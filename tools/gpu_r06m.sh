#!/bin/bash
# round 6 call m: register-allocator flags on the C3 kernel (topology 1 only;
# build/ab/f*, python tools/build_variants.py --units topo1 f2=-mllvm,... ):
# f2 -greedy-regclass-priority-trumps-globalness, f3 -greedy-reverse-local-assignment,
# f5 -split-spill-mode=size, f9 f5+f3, f10 f5+f2.  Same-box A/B of C3 and its
# RK-Merson leg; the variants' realize/parity tests first
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06m; mkdir -p $out
B=$PWD/bioimitation-gym_amd/build/ab
for v in f2 f3 f5 f9 f10; do
  BIOIM_LIB=$B/$v/libbioim.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "MuscleWalkingImitation2D" > $out/tests_$v.log 2>&1 || { echo "tests $v failed"; exit 1; }
  tail -1 $out/tests_$v.log
done
timeout -k 10 900 bash tools/ab.sh $out/ab_c3 4 MuscleWalkingImitation2D-v0 tree $B/f2/libbioim.so $B/f3/libbioim.so \
  $B/f5/libbioim.so $B/f9/libbioim.so $B/f10/libbioim.so > $out/ab_c3.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/ab_c3.txt
echo done
