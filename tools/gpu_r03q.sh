set -o pipefail
mkdir -p gpurun_out/r03q
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03q/tests.log 2>&1 && \
bash tools/ab.sh gpurun_out/r03q/ab 3 MuscleRunningImitation3D-v0,MuscleWalkingImitation2D-v0 bioimitation-gym_amd/build/ab/fr32/libbioim.so tree > gpurun_out/r03q/ab.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -s -q --timeout 300 --timeout-method thread -k "c3_tracking or kept_up" > gpurun_out/r03q/parity_print.log 2>&1
