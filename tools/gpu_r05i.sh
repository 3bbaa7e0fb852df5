#!/bin/bash
# Round 5, GPU call i: fiber-velocity warm-start variants on the raw-action
# Palsy3D model and the C5 mixed batch (its slower segment), plus per-wave
# durations of Palsy3D.
set -e
O=gpurun_out/r05i
mkdir -p $O
B=$PWD/bioimitation-gym_amd/build/ab
timeout -k 10 200 python tools/wavetime.py MusclePalsyImitation3D-v0 > $O/wavetime.log 2>&1
bash tools/ab.sh $O/ab 3 MusclePalsyImitation3D-v0,MuscleRunningImitation3D-v0,MuscleWalkingImitation2D-v0 tree $B/fvp/libbioim.so $B/fvhp/libbioim.so > $O/ab.log 2>&1
for r in 1 2 3; do
  for V in tree fvp fvhp; do
    if [ $V = tree ]; then L=""; else L="BIOIM_LIB=$B/$V/libbioim.so"; fi
    env $L timeout -k 10 120 python bench.py --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 --no-cpu-baseline --no-reference-integrator > $O/mixed_${V}_$r.json
  done
done
python3 - <<'PY' >> $O/ab.log
import glob, json
for V in ('tree', 'fvp', 'fvhp'):
    ms = [json.load(open(f))['roofline']['kernel_ms'] for f in sorted(glob.glob(f'gpurun_out/r05i/mixed_{V}_*.json'))]
    print(f'mixed C5 {V:6s} kernel ms ' + ' '.join(f'{x:.4f}' for x in ms) + f'  min {min(ms):.4f}')
PY
echo done
