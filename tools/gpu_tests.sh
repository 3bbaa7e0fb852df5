# GPU test suite only (one process), then smoke.  usage: bash tools/gpu_tests.sh TAG [pytest args]
set -e
TAG=${1:-r03}; shift || true
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/$TAG/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1
