# One GPU check of the current tree: GPU tests, smoke, the default bench line,
# and the C4 / C2 bench lines (no CPU baseline).
# usage: bash tools/gpu_check.sh TAG
set -e
TAG=${1:-r03}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
timeout -k 10 200 python bench.py --env-id MuscleRunningImitation3D-v0 --no-cpu-baseline --no-single-env > gpurun_out/$TAG/bench_3d.json 2>> gpurun_out/$TAG/bench.err
timeout -k 10 200 python bench.py --env-id TorqueWalkingImitation2D-v0 --no-cpu-baseline --no-single-env > gpurun_out/$TAG/bench_torque2d.json 2>> gpurun_out/$TAG/bench.err
