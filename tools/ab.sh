#!/bin/bash
# Same-box A/B of builds of libbioim.so (GPU box).  Alternates the libraries
# over R rounds of bench.py per env ID and prints each one's kernel ms per
# step (HIP events on the launch stream); "tree" is the in-tree build.
#   bash tools/ab.sh <out-dir> <rounds> <id,id,...> <lib|tree> [<lib|tree> ...]
# BENCH_ARGS adds bench.py arguments (e.g. "--integrator rk-merson --rk-budget 6 --steps 200";
# the table then also shows the line's value, finished env steps/s)
set -e
out=$1; rounds=$2; ids=$3; shift 3
mkdir -p "$out"
for id in ${ids//,/ }; do
  for r in $(seq 1 "$rounds"); do
    for lib in "$@"; do
      tag=$(basename "$lib" .so)
      [ "$tag" = libbioim ] && tag=$(basename "$(dirname "$lib")")   # build/ab/<variant>/libbioim.so
      if [ "$lib" = tree ]; then
        timeout -k 10 120 python bench.py --no-cpu-baseline --no-reference-integrator --no-single-env --env-id "$id" $BENCH_ARGS > "$out/${tag}__${id}__$r.json"
      else
        BIOIM_LIB="$lib" timeout -k 10 120 python bench.py --no-cpu-baseline --no-reference-integrator --no-single-env --env-id "$id" $BENCH_ARGS > "$out/${tag}__${id}__$r.json"
      fi
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
    print(f'{env:30s} {tag:22s} kernel ms ' + ' '.join(f'{x:.4f}' for x in ms) + f'  min {min(ms):.4f}'
          f'  done_rate {v[0][1]}  value ' + ' '.join(f'{x / 1e6:.3f}' for x in val) + f'  max {max(val) / 1e6:.3f} M')
PY
