set -e
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 900 bash tools/gpu_evidence.sh ${TAG} > gpurun_out/${TAG}_evidence.log 2>&1
timeout -k 10 120 python bench.py --env-id TorqueWalkingImitation2D-v0 --no-cpu-baseline > gpurun_out/ev_${TAG}/bench_torque2d_fp64.json
timeout -k 10 120 python bench.py --env-id TorqueWalkingImitation3D-v0 --no-cpu-baseline > gpurun_out/ev_${TAG}/bench_torque3d_fp64.json
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 50 --warmup 5 > gpurun_out/ev_${TAG}/bench_torchrun_n1.json 2> gpurun_out/ev_${TAG}/torchrun.err
timeout -k 10 400 python tools/error_curve.py --out gpurun_out/ev_${TAG}/error_curve.json > gpurun_out/ev_${TAG}/error_curve.log 2>&1
