#!/bin/bash
# Round 5, GPU call k: GPU suite on the build whose fiber-velocity Newton
# lets a past-the-curve-end lane leave after one step, then a same-box A/B
# against the previous behaviour (variant build -DBIOIM_FV_PAST_END=0).
set -e
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
B=$PWD/bioimitation-gym_amd/build/ab
bash tools/ab.sh $O/ab 3 MusclePalsyImitation3D-v0,MuscleLockedKneeImitation3D-v0,MuscleRunningImitation3D-v0,MuscleWalkingImitation2D-v0 tree $B/nope/libbioim.so > $O/ab.log 2>&1
for r in 1 2 3; do
  for V in tree nope; do
    if [ $V = tree ]; then L=""; else L="BIOIM_LIB=$B/$V/libbioim.so"; fi
    env $L timeout -k 10 120 python bench.py --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 --no-cpu-baseline --no-reference-integrator > $O/mixed_${V}_$r.json
  done
done
python3 - <<'PY' >> $O/ab.log
import glob, json
for V in ('tree', 'nope'):
    ms = [json.load(open(f))['roofline']['kernel_ms'] for f in sorted(glob.glob(f'gpurun_out/r05k/mixed_{V}_*.json'))]
    print(f'mixed C5 {V:6s} kernel ms ' + ' '.join(f'{x:.4f}' for x in ms) + f'  min {min(ms):.4f}')
PY
echo done
