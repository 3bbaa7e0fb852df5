#!/bin/bash
# round 6 call d: realize cache in the torque models too + the reset equilibrium's residual stop (oracle's rule);
# GPU suite, same-box A/B of the torque cache, the Palsy3D diagnosis again, single-env breakdown
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r06d; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
echo tests exit $?
timeout -k 10 600 bash tools/ab.sh $out/ab_torque 3 TorqueWalkingImitation2D-v0,TorqueWalkingImitation3D-v0 \
  tree bioimitation-gym_amd/build/ab/notorque/libbioim.so > $out/ab_torque.txt 2>&1 || exit 1
timeout -k 10 300 python tools/diag_palsy_ratio.py > $out/diag_palsy.txt 2>&1 || exit 1
for id in TorqueWalkingImitation2D-v0 MuscleWalkingImitation2D-v0; do
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_single_$id -o s -- \
     python3 $GRAFT_REPO_ROOT/tools/single_env_breakdown.py $id > $GRAFT_REPO_ROOT/$out/single_$id.txt 2>&1) || exit 1
done
echo done
