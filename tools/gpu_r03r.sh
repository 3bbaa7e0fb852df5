# final check of the tree build (BIOIM_BF3=122): GPU tests, smoke, C4 and C3 bench lines
set -o pipefail
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --env-id MuscleRunningImitation3D-v0 --no-cpu-baseline --no-single-env > $O/bench_3d.json 2> $O/bench.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-single-env --no-reference-integrator > $O/bench_2d.json 2>> $O/bench.err
