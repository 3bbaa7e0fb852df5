#!/bin/bash
# round 6 call s: RLlibVectorEnv.vector_step and RLlibBaseEnv.poll through pinned buffers and
# asynchronous copies: the adapter / env GPU tests, then its host time per
# step against the blocking form (tools/rllib_step_time.py)
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06s; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "rllib or adapter or gym_vector or facade or golden or base_env or rk_budget or poll" > $out/gpu_tests.log 2>&1
rc=$?; echo tests exit $rc; tail -1 $out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/rllib_step_time.py > $out/rllib_step_time.txt 2>&1 || exit 1
grep -v amdgpu.ids $out/rllib_step_time.txt
echo done
