#!/bin/bash
# Round 5, GPU call u: the bench's timed-window length (--steps) and burn-in
# against the kernel time it reports (is the driver's 20-step window biased?).
set -e
O=gpurun_out/r05u
mkdir -p $O
for r in 1 2 3; do
  for S in 20 40 100 200; do
    timeout -k 10 120 python bench.py --steps $S --warmup 5 --no-cpu-baseline --no-reference-integrator --no-single-env > $O/s${S}_b150_$r.json
  done
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --burn-in 400 --no-cpu-baseline --no-reference-integrator --no-single-env > $O/s20_b400_$r.json
  timeout -k 10 120 python bench.py --steps 20 --warmup 100 --no-cpu-baseline --no-reference-integrator --no-single-env > $O/s20_w100_$r.json
done
python3 - <<'PY' > $O/summary.txt
import glob, json, collections
d = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/r05u/s*.json')):
    tag = f.split('/')[-1].rsplit('_', 1)[0]
    j = json.load(open(f))
    d[tag].append((j['roofline']['kernel_ms'], j['ms_per_step'], j['value'], j['done_rate']))
for tag, v in sorted(d.items()):
    print(f'{tag:10s} kernel ms ' + ' '.join(f'{x[0]:.4f}' for x in v) + '  ms/step ' + ' '.join(f'{x[1]:.4f}' for x in v) +
          '  M/s ' + ' '.join(f'{x[2] / 1e6:.3f}' for x in v) + f'  done {v[0][3]:.4f}')
PY
echo done
