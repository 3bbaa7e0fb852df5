"""Scan gfx950 assembly for register copies executed under a narrowed EXEC
that move a value defined before the divergent region into a register read
after the region joins (the wrong-lane / fault incidents).

A structured `if` in the ISA is
    s_and_saveexec_b64 s[a:b], vcc     ; EXEC narrowed to the taken lanes
    ...                                 ; region
    s_or_b64 exec, exec, s[a:b]        ; join: EXEC restored
A VGPR <-> AGPR copy (v_accvgpr_write / v_accvgpr_read / v_mov_b32) inside
the region writes only the active lanes.  If its source was defined before
the region (the value is live in every lane) and its destination is read
after the join before being rewritten, the inactive lanes read whatever the
destination held before: a value silently lost in those lanes.  The scan is
linear over each kernel (loop back-edges are ignored), so it reports
candidates, each classified:

  phi-merge   the destination's last write before the region was made with
              EXEC at least as wide as the region's parent (a well-defined
              value in the lanes the region leaves out): the copy is the
              ISA form of `x = cond ? new : x_old` — what the source code asks
              for, not an allocator split; benign;
  masked-use  no such earlier write, but every read after the join until
              the next full write happens inside a narrowed region again
              (the lanes that skipped the copy may be masked off there too:
              check that the two conditions select the same lanes);
  undefined   no earlier write and a read under wider EXEC: lanes outside
              the region read a register nothing wrote — the hazard.

A candidate whose value reaches a memory instruction's address operand
(linear taint through VALU results), copied at a deeper EXEC nesting than the
read after the join (the nesting is tracked linearly: if/else pairs and loop
exits make it approximate, so this prunes candidates heuristically), gets
"+addr"; "masked-use+addr" and
"undefined" are reported as risky: a lane that skipped the copy would load or
store through a stale address — the fault incident class.  The fault of the
r03i build (an RK kernel storing through an env offset copied to an AGPR
only in the resume branch's lanes) scans as masked-use+addr.

    python tools/exec_hazard.py <file.s> [kernel-substring]
"""
import re
import sys

REG = re.compile(r'\b([va])(\d+)\b|\b([va])\[(\d+):(\d+)\]')


def regs(text):
    out = []
    for m in REG.finditer(text):
        if m.group(1):
            out.append(f'{m.group(1)}{m.group(2)}')
        else:
            out += [f'{m.group(3)}{i}' for i in range(int(m.group(4)), int(m.group(5)) + 1)]
    return out


def parse(lines):
    """[(op, dst regs, src regs, raw)] for the instructions of one kernel."""
    ins = []
    for ln in lines:
        t = ln.split(';')[0].strip()
        if not t or t.startswith('.') or t.endswith(':'):
            continue
        parts = t.split(None, 1)
        op = parts[0]
        args = parts[1] if len(parts) > 1 else ''
        a = [x.strip() for x in args.split(',')] if args else []
        stores = op.startswith(('global_store', 'buffer_store', 'ds_write', 'scratch_store', 'flat_store', 's_'))
        dst = [] if stores or not a else regs(a[0])
        src = regs(','.join(a if stores else a[1:]))
        ins.append((op, dst, src, t))
    return ins


def is_join(op, raw):
    return op == 's_or_b64' and raw.split(None, 1)[1].startswith('exec, exec,')


def writes_exec(op, raw):
    parts = raw.split(None, 1)
    return op.startswith('s_') and len(parts) > 1 and parts[1].startswith('exec,') and not is_join(op, raw)


def depths(ins):
    """EXEC nesting depth at each instruction (0: the kernel's full EXEC).
    A save by plain move (s_mov_b64 sX, exec: a loop, or an if whose
    narrowing comes later) opens the region only at the instruction that
    then narrows EXEC; until then the kernel still runs at the parent depth."""
    out, stack, pending = [], [], None
    for op, dst, src, raw in ins:
        if op in ('s_and_saveexec_b64', 's_or_saveexec_b64', 's_andn2_saveexec_b64'):
            out.append(len(stack))
            stack.append(raw.split(None, 1)[1].split(',')[0].strip())
            pending = None
            continue
        if op == 's_mov_b64' and raw.split(None, 1)[1].endswith(', exec'):
            pending = raw.split(None, 1)[1].split(',')[0].strip()
            out.append(len(stack))
            continue
        if pending and writes_exec(op, raw):
            out.append(len(stack))
            stack.append(pending)
            pending = None
            continue
        if is_join(op, raw):
            sv = raw.split(',')[-1].strip()
            if sv == pending:
                pending = None
            if sv in stack:        # a restore of a mask this scan did not see saved is not a join
                while stack.pop() != sv:
                    pass
        out.append(len(stack))
    return out


def classify(ins, dep, i, start, dst, join_read):
    """phi-merge / masked-use / undefined for the candidate copy at i in the
    region opened at `start` (module docstring)"""
    parent = dep[start]
    for j in range(start - 1, -1, -1):
        if any(d in ins[j][1] for d in dst):
            return 'phi-merge' if dep[j] <= parent else 'masked-use'
    return 'masked-use' if dep[join_read] > 0 else 'undefined'


MEM_ADDR_FIRST = ('global_store', 'flat_store', 'ds_write', 'scratch_store', 'buffer_store')
MEM_ADDR_SECOND = ('global_load', 'flat_load', 'ds_read', 'scratch_load', 'buffer_load', 'global_atomic', 'ds_bpermute')


def addr_operands(op, raw):
    """the vector registers a memory instruction uses as its address"""
    parts = raw.split(None, 1)
    if len(parts) < 2:
        return []
    a = [x.strip() for x in parts[1].split(',')]
    if op.startswith(MEM_ADDR_FIRST):
        return regs(a[0]) if a else []
    if op.startswith(MEM_ADDR_SECOND):
        return regs(a[1]) if len(a) > 1 else []
    return []


def feeds_address(ins, j, reg, horizon=600, lds=False):
    """does the value read at j into `reg` (and anything computed from it)
    reach the address operand of a global / flat / scratch / buffer access
    (lds=True: of an LDS access) before being overwritten?  Linear,
    conservative taint propagation through VALU results.  A wrong lane value
    in a global address is a memory fault; in an LDS address a wrong value."""
    taint = {reg} if isinstance(reg, str) else set(reg)
    for k in range(j + 1, min(len(ins), j + horizon)):
        op, dd, ss, raw = ins[k]
        if op.startswith('ds_') == lds and any(r in taint for r in addr_operands(op, raw)):
            return True
        if op.startswith(('s_', 'global_store', 'ds_write', 'buffer_store', 'flat_store', 'scratch_store')):
            continue
        hit = any(r in taint for r in ss)
        for d in dd:
            if hit:
                taint.add(d)
            else:
                taint.discard(d)
        if not taint:
            return False
    return False


def scan(ins):
    hits = []
    dep = depths(ins)
    stack = []   # open regions: (saved-exec sgpr text, start index)
    pending = None
    for i, (op, dst, src, raw) in enumerate(ins):
        if op in ('s_and_saveexec_b64', 's_or_saveexec_b64', 's_andn2_saveexec_b64'):
            stack.append((raw.split(None, 1)[1].split(',')[0].strip(), i))
            pending = None
            continue
        if op == 's_mov_b64' and raw.split(None, 1)[1].endswith(', exec'):
            pending = raw.split(None, 1)[1].split(',')[0].strip()   # the region opens where EXEC narrows
            continue
        if pending and writes_exec(op, raw):
            stack.append((pending, i))
            pending = None
            continue
        if is_join(op, raw):
            sv = raw.split(',')[-1].strip()
            if sv == pending:
                pending = None
            if any(s == sv for s, _ in stack):
                while stack.pop()[0] != sv:
                    pass
            continue
        if not stack or op not in ('v_accvgpr_write_b32', 'v_accvgpr_read_b32', 'v_mov_b32', 'v_mov_b64'):
            continue
        if not dst or not src:
            continue
        inner_sv, start = stack[-1]
        # source defined before the innermost open region (not written inside it before i)
        if any(sr in ins[j][1] for j in range(start, i) for sr in src):
            continue
        # the destination already holds the value in every lane: its last write before the
        # region is the same copy and the source was not rewritten since (a redundant re-copy)
        lw = next((j for j in range(start - 1, -1, -1) if any(d in ins[j][1] for d in dst)), None)
        if lw is not None and ins[lw][0] == op and ins[lw][2] == src and \
                not any(sr in ins[j][1] for j in range(lw + 1, start) for sr in src):
            continue
        # destination read after THIS region's join (s_or_b64 exec, exec, <its saved mask>)
        # before being rewritten
        j = i + 1
        closed = False
        verdict = None
        while j < len(ins) and verdict is None:
            o, dd, ss, rr = ins[j]
            if is_join(o, rr) and rr.split(',')[-1].strip() == inner_sv:
                closed = True
            if any(x in ss for x in dst):
                verdict = 'read-after-join' if closed else 'read-inside'
            elif any(x in dd for x in dst):
                verdict = 'overwritten'
            j += 1
        if verdict == 'read-after-join':
            kind = classify(ins, dep, i, start, dst, j - 1)
            o, dd, ss, rr = ins[j - 1]
            # the value read after the join reaches an address (a wrong lane value
            # there is an out-of-range access: the fault incidents)
            tainted = dd if o.startswith(('v_accvgpr_read', 'v_mov', 'v_accvgpr_write')) else [x for x in dst]
            # ... and the copy sits deeper in the EXEC nesting than that read: lanes
            # active at the read were not all active at the copy (a copy at the read's
            # own depth, e.g. after the kernel's early-return regions, covers them)
            direct = any(x in addr_operands(o, rr) for x in dst)
            if dep[i] > dep[j - 1]:
                if feeds_address(ins, j - 1, tainted) or (direct and not o.startswith('ds_')):
                    kind += '+addr'
                elif feeds_address(ins, j - 1, tainted, lds=True) or direct:
                    kind += '+ldsaddr'
            hits.append((i, raw, j - 1, ins[j - 1][3], kind))
    return hits


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ''
    text = open(path).read().split('\n')
    starts = [i for i, l in enumerate(text) if re.match(r'^_Z\S+:', l)]
    for k, s in enumerate(starts):
        name = text[s].split(':')[0]
        if want not in name:
            continue
        e = next(i for i in range(s, len(text)) if text[i].startswith('.Lfunc_end'))
        ins = parse(text[s:e])
        hits = scan(ins)
        kinds = {k: sum(1 for h in hits if h[4].split('+')[0] == k) for k in ('phi-merge', 'masked-use', 'undefined')}
        risky = sum(1 for h in hits if h[4] in ('masked-use+addr', 'undefined', 'undefined+addr'))
        print(f'{name[:90]}: {len(ins)} instructions, {len(hits)} candidate copies {kinds}, '
              f'{risky} risky (masked-use into an address, or undefined)')
        for i, raw, j, use, kind in hits:
            print(f'    [{i}] {raw:50s} -> read after join at [{j}] {use:45s} {kind}')


if __name__ == '__main__':
    main()
