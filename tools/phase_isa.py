"""Static instruction mix between consecutive s_memtime stamps of the
diagnostic (-DBIOIM_STAMPS) build, for one kernel.

    hipcc $(cd bioimitation-gym_amd && python3 -m bioimitation._buildinfo flags) \
        -DBIOIM_STAMPS --offload-device-only -S bioim_step.hip -o ks.s
    python tools/phase_isa.py ks.s MuscleWalkingImitation2D_v0dE
"""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
lines = open(path).read().split('\n')
start = next(i for i, l in enumerate(lines) if l.startswith('_Z') and sym in l.split(':')[0] and ':' in l)
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
seg, segs = collections.Counter(), []
for l in lines[start:end]:
    t = l.strip()
    if not t or t[0] in '.;' or t.endswith(':'):
        continue
    op = t.split()[0]
    if op == 's_memtime':
        segs.append(seg)
        seg = collections.Counter()
        continue
    if op.startswith('v_') and '_f64' in op:
        seg['valu_f64'] += 1
        if any(x in op for x in ('rcp', 'rsq', 'sqrt', 'div', 'sin', 'cos', 'frexp', 'ldexp')):
            seg['f64_special'] += 1
    elif op.startswith('v_accvgpr'):
        seg['accvgpr'] += 1
    elif op.startswith('v_'):
        seg['valu_other'] += 1
    elif op.startswith('ds_'):
        seg['ds'] += 1
    elif op.startswith('s_waitcnt'):
        seg['waitcnt'] += 1
    elif op.startswith('s_cbranch') or op.startswith('s_branch'):
        seg['branch'] += 1
    elif op.startswith('s_'):
        seg['salu'] += 1
    elif op.startswith('global_') or op.startswith('buffer_') or op.startswith('scratch_') or op.startswith('flat_'):
        seg['vmem'] += 1
    seg['total'] += 1
segs.append(seg)
for i, s in enumerate(segs):
    print(i, dict(s))
