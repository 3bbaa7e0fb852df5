#!/bin/bash
# round 6 call q: the single-env facade's packed output buffer, pinned
# action/output copies (envs.py _bind_packed) and the recorder's deferred rows
# (simulation_io.TrajectoryRecorder): the GPU suite, then the
# facade parts of the old path (tools/facade_parts.py) and the step times of
# the new one (tools/single_env_breakdown.py), C1 and the Muscle2D single env
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06q; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; echo tests exit $rc; tail -1 $out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for id in TorqueWalkingImitation2D-v0 MuscleWalkingImitation2D-v0; do
  timeout -k 10 200 python tools/facade_parts.py $id >> $out/facade_parts.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/single_env_breakdown.py $id >> $out/single_env.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $out/facade_parts.txt $out/single_env.txt
echo done
