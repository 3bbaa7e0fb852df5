# GPU tests of the BIOIM_BF3=122 variant library (spatial phase-3 rows and
# h-free implicit terms on top of the default's pieces) through BIOIM_LIB
set -o pipefail
mkdir -p gpurun_out/r03t
BIOIM_LIB=bioimitation-gym_amd/build/ab/bf122/libbioim.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03t/gpu_tests_bf122.log 2>&1
