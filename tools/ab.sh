#!/bin/bash
# Same-box A/B of two builds of libbioim.so (GPU box): alternates the
# candidate (the in-tree build) and a baseline library (BIOIM_LIB=...) over
# R rounds of bench.py, per env ID, and prints ms_per_step of each.
#   bash tools/ab.sh <baseline.so> <out-dir> [rounds] [env ids...]
set -e
base=$1; out=$2; rounds=${3:-3}; shift 3 || true
ids=${@:-MuscleWalkingImitation2D-v0 MuscleRunningImitation3D-v0}
mkdir -p "$out"
for id in $ids; do
  for r in $(seq 1 "$rounds"); do
    timeout -k 10 120 python bench.py --no-cpu-baseline --env-id "$id" > "$out/new_${id}_$r.json"
    BIOIM_LIB="$base" timeout -k 10 120 python bench.py --no-cpu-baseline --env-id "$id" > "$out/old_${id}_$r.json"
  done
done
python3 - "$out" <<'PY'
import glob, json, os, sys, collections
d = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], '*.json'))):
    tag, rest = os.path.basename(f).split('_', 1)
    env = rest.rsplit('_', 1)[0]
    d[(env, tag)].append(json.load(open(f))['roofline']['kernel_ms'])
for (env, tag), v in sorted(d.items()):
    print(f'{env:34s} {tag}: kernel ms ' + ' '.join(f'{x:.4f}' for x in v) + f'  min {min(v):.4f}')
PY
