"""Basic-block profile of one kernel in a gfx950 assembly file: per block its
instruction count, LDS / fp64 / waitcnt / EXEC-writing instructions and the
terminator.  The machine scheduler works within a basic block, so the blocks
inside the substep loop bound how far independent dependency chains can be
interleaved.

    hipcc $(cd bioimitation-gym_amd && python3 -m bioimitation._buildinfo flags) \
        -DBIOIM_TOPO_ONLY=1 --offload-device-only -S bioim_step.hip -o t1.s
    python tools/bb_profile.py t1.s MuscleWalkingImitation2D_v0dLb0ELb0ELb0E [min-insts]
"""
import sys


def blocks(path, sym):
    lines = open(path).read().split('\n')
    st = next(i for i, l in enumerate(lines) if l.startswith('_Z') and sym in l.split(':')[0])
    en = next(i for i in range(st, len(lines)) if lines[i].startswith('.Lfunc_end'))
    out, cur, loc = [], None, None
    for l in lines[st:en]:
        t = l.split(';')[0].strip()
        if not t:
            continue
        if t.endswith(':') and not t.startswith('.Ltmp') and not t.startswith('.Lfunc_begin'):   # debug labels are not blocks
            cur = [t[:-1], [], []]
            out.append(cur)
            continue
        if t.startswith('.loc\t') or t.startswith('.loc '):   # -gline-tables-only builds: source line of what follows
            f = t.split()
            loc = int(f[2]) if f[1] == '0' else None   # file 0: bioim_step.hip
            continue
        if t[0] == '.' or t.endswith(':'):
            continue
        cur[1].append(t)
        cur[2].append(loc or 0)
        if t.startswith('s_cbranch') or t.startswith('s_branch'):   # a fall-through successor has no label
            cur = [cur[0].split('+')[0] + '+', [], []]
            out.append(cur)
    return [b for b in out if b[1]]


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    bbs = blocks(path, sym)
    tot = sum(len(b[1]) for b in bbs)
    print(f'{len(bbs)} blocks, {tot} instructions')
    for name, ins, locs in bbs:
        ops = [i.split()[0] for i in ins]
        if len(ops) < lo:
            continue
        ds = sum(o.startswith('ds_') for o in ops)
        f64 = sum(o.startswith('v_') and 'f64' in o for o in ops)
        wc = sum(o == 's_waitcnt' for o in ops)
        ex = sum(1 for i in ins if ' exec' in i and i.split()[0].startswith('s_'))
        last = ins[-1] if ins else ''
        src = ''
        if any(locs):   # the three most frequent source lines of the block
            cnt = {}
            for x in (x for x in locs if x):
                cnt[x] = cnt.get(x, 0) + 1
            src = ' L' + ','.join(str(k) for k, _ in sorted(cnt.items(), key=lambda kv: -kv[1])[:3])
        print(f'{name:24s} n={len(ops):5d} ds={ds:4d} f64={f64:5d} wait={wc:4d} exec={ex:3d}{src} | {last[:48]}')


if __name__ == '__main__':
    main()
