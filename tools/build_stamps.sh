#!/bin/bash
# Diagnostic build with per-phase s_memtime stamps (tools/stamps.py reads them).
set -e
cd "$(dirname "$0")/.."
C=bioimitation-gym_amd/csrc
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DBIOIM_STAMPS -mllvm -amdgpu-sched-strategy=iterative-ilp -Iinclude -I$C -Wno-unused-result \
    -Wno-unused-value -o bioimitation-gym_amd/build/libbioim_stamps.so $C/bioim_step.hip
