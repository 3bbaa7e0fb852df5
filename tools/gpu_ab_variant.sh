#!/bin/bash
# GPU tests on a variant library, then a same-box A/B against the tree build.
#   bash tools/gpu_ab_variant.sh <tag> <variant dir under build/ab> <ids>
set -e
O=gpurun_out/$1
mkdir -p $O
V=$PWD/bioimitation-gym_amd/build/ab/$2/libbioim.so
BIOIM_LIB=$V timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$2.log 2>&1
bash tools/ab.sh $O/ab 3 $3 tree $V > $O/ab.log 2>&1
echo done
