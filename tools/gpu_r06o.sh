#!/bin/bash
# round 6 call o: the C3 kernel under LLVM's default and max-ilp machine
# schedulers (python tools/sched_variants.py; the memory-clause,
# iterative-minreg and iterative-maxocc builds fail the hazard gate and are not
# run): C3 parity tests, then a same-box A/B against the tree (iterative-ilp)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06o; mkdir -p $out
B=$PWD/bioimitation-gym_amd/build/ab
for v in s_default s_maxilp; do
  BIOIM_LIB=$B/$v/libbioim.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "MuscleWalkingImitation2D" > $out/tests_$v.log 2>&1 || { echo "tests $v failed"; exit 1; }
  tail -1 $out/tests_$v.log
done
timeout -k 10 900 bash tools/ab.sh $out/ab_c3 4 MuscleWalkingImitation2D-v0 tree $B/s_default/libbioim.so $B/s_maxilp/libbioim.so \
  > $out/ab_c3.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/ab_c3.txt
echo done
