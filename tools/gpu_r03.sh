#!/bin/bash
# Round-3 GPU evidence pass on the build in the tree (run from the repo root on
# the box): GPU tests, smoke, bench lines (C3 headline with CPU baselines, C4,
# C2, C5), rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes for
# the 2D and 3D kernels, and the SQ counter passes for both (tools/pmc_sq.sh).
# Every GPU step has its own time limit; the script stops at the first failure.
#   bash tools/gpu_r03.sh <tag> [skip-tests]
set -e
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "$2" != skip-tests ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 200 python bench.py --env-id MuscleRunningImitation3D-v0 --no-cpu-baseline --no-single-env > $O/bench_3d.json 2>> $O/bench.err
timeout -k 10 200 python bench.py --env-id TorqueWalkingImitation2D-v0 --no-cpu-baseline --no-single-env > $O/bench_torque2d.json 2>> $O/bench.err
timeout -k 10 200 python bench.py --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 --no-cpu-baseline > $O/bench_mixed.json 2>> $O/bench.err
for CFG in "2d:--env-id MuscleWalkingImitation2D-v0" "3d:--env-id MuscleRunningImitation3D-v0"; do
    K=${CFG%%:*}; A="${CFG#*:} --steps 20 --warmup 3 --no-cpu-baseline --no-reference-integrator --no-single-env"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/${K}_trace -o trace -- python3 $OLDPWD/bench.py $A > $OLDPWD/$O/${K}_trace.log 2>&1)
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OLDPWD/$O/${K}_fetch -o fetch -- python3 $OLDPWD/bench.py $A > $OLDPWD/$O/${K}_fetch.log 2>&1)
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OLDPWD/$O/${K}_write -o write -- python3 $OLDPWD/bench.py $A > $OLDPWD/$O/${K}_write.log 2>&1)
done
bash tools/pmc_sq.sh ${TAG}_2d 64 MuscleWalkingImitation2D-v0
bash tools/pmc_sq.sh ${TAG}_3d 64 MuscleRunningImitation3D-v0
find $O gpurun_out/pmc_${TAG}_* -name "*.csv" | sort
