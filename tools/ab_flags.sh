#!/bin/bash
# Same-box A/B of bench.py flag sets on the tree build: alternates the
# variants over R rounds per env ID (or mixed batch) and prints kernel ms.
#   bash tools/ab_flags.sh <out-dir> <rounds> <id|mixed:a,b>[;...] <tag>=<flags> [<tag>=<flags> ...]
set -e
out=$1; rounds=$2; ids=$3; shift 3
mkdir -p "$out"
IFS=';' read -ra IDS <<< "$ids"
for id in "${IDS[@]}"; do
  if [[ $id == mixed:* ]]; then sel="--mixed ${id#mixed:}"; tagid=mixed; else sel="--env-id $id"; tagid=$id; fi
  for r in $(seq 1 "$rounds"); do
    for v in "$@"; do
      tag=${v%%=*}; flags=${v#*=}
      timeout -k 10 120 python bench.py --no-cpu-baseline --no-reference-integrator --no-single-env $sel $flags \
          > "$out/${tag}__${tagid}__$r.json"
    done
  done
done
python3 - "$out" <<'PY'
import glob, json, os, sys, collections
d = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], '*.json'))):
    tag, env, _ = os.path.basename(f).split('__')
    j = json.load(open(f))
    d[(env, tag)].append((j['roofline']['kernel_ms'], j.get('done_rate'), j['value']))
for (env, tag), v in sorted(d.items()):
    ms = [x for x, _, _ in v]
    val = [x for _, _, x in v]
    print(f'{env:30s} {tag:14s} kernel ms ' + ' '.join(f'{x:.4f}' for x in ms) + f'  min {min(ms):.4f}'
          f'  done_rate {v[0][1]}  value ' + ' '.join(f'{x / 1e6:.3f}' for x in val) + f'  max {max(val) / 1e6:.3f} M')
PY
