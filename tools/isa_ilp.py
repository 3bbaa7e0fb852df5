"""Static ILP view of one kernel in a gfx950 assembly file (round 5).

For every basic block: VALU instruction count, the issue-bound cycles
(per-class issue costs) and the cycles of an in-order, one-wave issue model
in which an instruction waits for the registers it reads (VALU result
latency, LDS latency, s_waitcnt) — calibrated on tools/ubench/lat2.hip
(gfx950, one wave per SIMD: dependent VALU issue-to-issue 9.2 cycles, fp64
FMA issue 5.8, 32-bit VALU 4.5, fp64 transcendental 16.5, ds_read latency
~53 cycles (dependent chain incl. the wait), SALU / s_nop 4).  The ratio
model / issue-bound says how much of a block's time is dependency latency
the schedule leaves exposed.

    python tools/isa_ilp.py t1g.s <kernel-symbol-substring> [top]
"""
import collections
import re
import sys

LAT_VALU = 9.2       # issue-to-issue of a dependent VALU instruction
LAT_LDS = 53.0       # ds_read issue to data use
ISSUE_LDS = 8.0
ISSUE_SALU = 4.0


def valu_issue(op):
    if any(k in op for k in ('rcp', 'rsq', 'sqrt', 'sin', 'cos', 'exp', 'log', 'frexp', 'ldexp', 'div_fixup', 'div_scale', 'div_fmas')) and op.startswith('v_'):
        return 16.5 if 'f64' in op else 8.0
    if '_f64' in op or op.startswith('v_mov_b64') or op.startswith('v_lshl_add_u64') or op.startswith('v_mad_u64'):
        return 5.8
    return 4.5


REG = re.compile(r'\b([vsa])\[(\d+):(\d+)\]|\b([vsa])(\d+)\b|\b(vcc|exec|scc)\b')


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            for r in range(int(m.group(2)), int(m.group(3)) + 1):
                out.add(f'{m.group(1)}{r}')
        elif m.group(4):
            out.add(f'{m.group(4)}{m.group(5)}')
        else:
            out.add(m.group(6))
    return out


def split_ops(t):
    """destination / source register sets of one instruction"""
    parts = t.split(None, 1)
    op = parts[0]
    if len(parts) == 1:
        return op, set(), set()
    args = [a.strip() for a in parts[1].split(',')]
    if op.startswith('ds_read') or op.startswith('ds_bpermute') or op.startswith('ds_swizzle'):
        return op, regs(args[0]), regs(','.join(args[1:]))
    if op.startswith('ds_write') or op.startswith('global_store') or op.startswith('buffer_store') or op.startswith('s_cbranch') \
            or op.startswith('s_branch') or op.startswith('s_waitcnt') or op.startswith('v_cmpx'):
        return op, set(), regs(','.join(args))
    if op.startswith('v_cmp'):
        return op, regs(args[0]), regs(','.join(args[1:]))
    d = regs(args[0])
    s = regs(','.join(args[1:]))
    if op.startswith('v_fmac') or op.startswith('v_mac'):
        s |= d
    if op.startswith('v_cndmask') or op.startswith('v_addc') or op.startswith('v_subb'):
        s |= {'vcc'} if len(args) < 4 else set()
    return op, d, s


def blocks(path, sym):
    lines = open(path).read().split('\n')
    st = next(i for i, l in enumerate(lines) if l.startswith('_Z') and sym in l.split(':')[0] and ':' in l)
    en = next(i for i in range(st, len(lines)) if lines[i].startswith('.Lfunc_end'))
    out, cur, loc, depth = [], None, 0, 0
    for l in lines[st:en]:
        if l.startswith('.LBB') or l.startswith('; %bb'):
            m = re.search(r'Depth=(\d+)', l)
            depth = int(m.group(1)) if m else 0
            cur = [l.split()[0].rstrip(':'), depth, []]
            out.append(cur)
            continue
        t = l.split(';')[0].strip()
        if not t:
            continue
        if t.startswith('.loc'):
            f = t.split()
            loc = int(f[2]) if f[1] == '0' else 0
            continue
        if t[0] == '.' or t.endswith(':'):
            continue
        if cur is None:
            cur = ['entry', 0, []]
            out.append(cur)
        cur[2].append((t, loc))
    return out


def simulate(ins):
    """cycles of one pass through a block: in-order issue, register-ready
    times, lgkmcnt-tracked LDS completions"""
    ready = collections.defaultdict(float)
    t = 0.0
    issue_bound = 0.0
    lds_q = []   # completion times of outstanding LDS ops (oldest first)
    nvalu = 0
    for text, _ in ins:
        op, d, s = split_ops(text)
        if op.startswith('s_waitcnt'):
            m = re.search(r'lgkmcnt\((\d+)\)', text)
            if m:
                keep = int(m.group(1))
                while len(lds_q) > keep:
                    t = max(t, lds_q.pop(0))
            continue
        start = max([t] + [ready[r] for r in s if not r.startswith('s') and r not in ('scc',)])
        if op.startswith('v_'):
            c = valu_issue(op)
            nvalu += 1
            lat = LAT_VALU if c < 16 else c + 4
            issue_bound += c
        elif op.startswith('ds_'):
            c, lat = ISSUE_LDS, LAT_LDS
            issue_bound += c
            lds_q.append(start + lat)
        else:
            c, lat = ISSUE_SALU, ISSUE_SALU
            issue_bound += c
        for r in d:
            ready[r] = start + lat
        t = start + c
    return t, issue_bound, nvalu


if __name__ == '__main__':
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = []
    for name, depth, ins in blocks(path, sym):
        if not ins:
            continue
        cyc, ib, nv = simulate(ins)
        lines = collections.Counter(l for _, l in ins if l)
        rows.append((name, depth, len(ins), nv, ib, cyc, lines.most_common(3)))
    tot_ib = sum(r[4] for r in rows if r[1] >= 1)
    tot_c = sum(r[5] for r in rows if r[1] >= 1)
    print(f'blocks in loops: issue-bound {tot_ib:.0f} cyc, modelled {tot_c:.0f} cyc, ratio {tot_c / max(tot_ib, 1):.2f}')
    print('block depth insts valu issue-bound model ratio excess  top source lines')
    for r in sorted(rows, key=lambda r: -(r[5] - r[4]))[:top]:
        print(f'{r[0]:12s} {r[1]} {r[2]:5d} {r[3]:5d} {r[4]:8.0f} {r[5]:8.0f} {r[5] / max(r[4], 1):5.2f} {r[5] - r[4]:7.0f}  {r[6]}')
