#!/bin/bash
# C5 (mixed LockedKnee3D + Palsy3D batch): parity of the fused launch, then a
# same-box A/B of the fused two-topology kernel against concurrent
# per-segment launches.
set -e
O=gpurun_out/${1:-r04m}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k mixed > $O/mixed_tests.log 2>&1
for r in 1 2 3; do
  for F in "" "--no-fuse"; do
    tag=fused; [ -n "$F" ] && tag=concurrent
    timeout -k 10 200 python bench.py --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 --no-cpu-baseline $F > $O/c5_${tag}_$r.json 2>> $O/bench.err
  done
done
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], 'c5_*.json'))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), f"{d['value'] / 1e6:.3f} M env-steps/s", f"{d['ms_per_step']:.4f} ms/step",
          f"kernel {d['roofline']['kernel_ms']:.4f} ms", 'fusion', d['config'].get('group_fusion'))
PY
