# evidence pass on the tree build (spatial branch-free pieces BIOIM_BF3=26):
# GPU tests, smoke, bench lines, rocprof passes; then same-box A/B of further
# BIOIM_BF3 variants against it
set -o pipefail
mkdir -p gpurun_out/r03s
bash tools/gpu_r03.sh r03s && \
bash tools/ab.sh gpurun_out/r03s/ab3 3 MuscleRunningImitation3D-v0 bioimitation-gym_amd/build/ab/bf58/libbioim.so bioimitation-gym_amd/build/ab/bf122/libbioim.so tree > gpurun_out/r03s/ab3.log 2>&1
