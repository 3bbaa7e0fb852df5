#!/bin/bash
# round 6 call n: the VALU census (tools/pmc_census.sh) of the C3 kernel for
# the tree build and the -split-spill-mode=size variant of call m (build/ab/f5:
# python tools/build_variants.py --units topo1 f5=-mllvm,-split-spill-mode=size)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06n; mkdir -p $out
timeout -k 10 400 bash tools/pmc_census.sh r06n_tree > $out/census_tree.log 2>&1 || exit 1
BIOIM_LIB=$PWD/bioimitation-gym_amd/build/ab/f5/libbioim.so timeout -k 10 400 bash tools/pmc_census.sh r06n_f5 > $out/census_f5.log 2>&1 || exit 1
for t in tree f5; do python3 tools/pmc_summary.py gpurun_out/pmc_r06n_$t > $out/summary_$t.txt 2>&1; done
cat $out/census_*.log
echo done
