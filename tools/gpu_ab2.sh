#!/bin/bash
# Two variant libraries (build/ab/<a>, build/ab/<b>): GPU tests on each, then
# a same-box A/B of both against the tree build.
#   bash tools/gpu_ab2.sh <tag> <a> <b> <ids>
set -e
O=gpurun_out/$1
mkdir -p $O
for V in $2 $3; do
  BIOIM_LIB=$PWD/bioimitation-gym_amd/build/ab/$V/libbioim.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q \
      --timeout 300 --timeout-method thread > $O/gpu_tests_$V.log 2>&1
done
bash tools/ab.sh $O/ab 3 $4 tree $PWD/bioimitation-gym_amd/build/ab/$2/libbioim.so $PWD/bioimitation-gym_amd/build/ab/$3/libbioim.so > $O/ab.log 2>&1
echo done
