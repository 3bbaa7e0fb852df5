"""VALU instruction census of the Muscle2D fp64 step kernel by class
(VERDICT r04 item 1a).

Dynamic counts per launch come from the SQ counter passes of
tools/pmc_census.sh (SQ_INSTS_VALU and its FMA/MUL/ADD/TRANS F64, INT32,
INT64, CVT and F32 sub-counters, summarised by tools/pmc_summary.py).  The
remainder — VALU instructions no sub-counter claims (selects, moves,
compares, AGPR copies, lane reads/writes, bit operations) — is split by the
static shares of those opcodes in the basic blocks of the substep loop
(loop depth >= 1 in the assembly: the dynamics call, the substep update and
the report; an approximation, the blocks' execution counts are not known).
Issue costs per class from tools/ubench/lat2.hip / lat3.hip (one wave per
SIMD, shader cycles): fp64 FMA/MUL/ADD 5.8 (dependent back-to-back 10.3),
32-bit VALU 4.5 (dependent 9.2), fp64 transcendental 16.5, AGPR copy 4.8.

    python tools/census.py <census_summary.txt> <kernel .s> <symbol substring>
"""
import collections
import re
import sys

sys.path.insert(0, __file__.rsplit('/', 1)[0])
from isa_ilp import blocks  # noqa: E402

COST = {'fp64 FMA/MUL/ADD': 5.8, 'fp64 transcendental': 16.5, 'int32': 4.5, 'int64': 5.8, 'cvt': 4.5,
        'v_cndmask (select)': 4.5, 'v_mov / v_mov_b64': 4.5, 'v_cmp (compare)': 5.7, 'v_accvgpr (AGPR copy)': 4.8,
        'v_readlane / v_writelane': 4.5, 'bit ops / other': 4.5}


def other_class(op):
    if op.startswith('v_cndmask'):
        return 'v_cndmask (select)'
    if op.startswith('v_mov'):
        return 'v_mov / v_mov_b64'
    if op.startswith('v_cmp'):
        return 'v_cmp (compare)'
    if op.startswith('v_accvgpr'):
        return 'v_accvgpr (AGPR copy)'
    if op.startswith(('v_readlane', 'v_writelane', 'v_readfirstlane')):
        return 'v_readlane / v_writelane'
    return 'bit ops / other'


def counted(op):
    """opcodes an SQ sub-counter claims (approximately, by name)"""
    if not op.startswith('v_') or op.startswith(('v_cndmask', 'v_mov', 'v_cmp', 'v_accvgpr', 'v_readlane',
                                                 'v_writelane', 'v_readfirstlane')):
        return False
    return bool(re.search(r'_f64|_u32|_i32|_u64|_i64|_cvt_|_f32', op)) and not op.startswith(('v_and', 'v_or', 'v_xor', 'v_not', 'v_bfe', 'v_bfi', 'v_lsh', 'v_ash'))


def main():
    summ, asm, sym = sys.argv[1:4]
    c = {}
    for line in open(summ):
        f = line.split()
        if len(f) >= 2:
            c[f[0]] = float(f[1])
    f64 = c['SQ_INSTS_VALU_FMA_F64'] + c['SQ_INSTS_VALU_MUL_F64'] + c['SQ_INSTS_VALU_ADD_F64']
    dyn = collections.OrderedDict([
        ('fp64 FMA/MUL/ADD', f64), ('fp64 transcendental', c['SQ_INSTS_VALU_TRANS_F64']),
        ('int32', c['SQ_INSTS_VALU_INT32']), ('int64', c['SQ_INSTS_VALU_INT64']), ('cvt', c['SQ_INSTS_VALU_CVT'])])
    rest = c['SQ_INSTS_VALU'] - sum(dyn.values())
    st = collections.Counter()
    for name, depth, ins in blocks(asm, sym):
        if depth < 1:
            continue
        for t, _ in ins:
            op = t.split()[0]
            if op.startswith('v_') and not counted(op):
                st[other_class(op)] += 1
    tot = sum(st.values())
    for k in ('v_cndmask (select)', 'v_mov / v_mov_b64', 'v_cmp (compare)', 'v_accvgpr (AGPR copy)',
              'v_readlane / v_writelane', 'bit ops / other'):
        dyn[k + ' *'] = rest * st[k] / tot
    total = c['SQ_INSTS_VALU']
    cyc = {k: v * COST[k.rstrip(' *')] for k, v in dyn.items()}
    ctot = sum(cyc.values())
    print(f'VALU instructions per launch {total:.3e} (1024 waves); * = remainder {rest:.3e} split by static loop-block shares')
    print(f'{"class":32s} {"per launch":>11s} {"share":>7s} {"per wave":>9s} {"issue cyc/wave":>14s} {"of issue":>8s}')
    for k, v in dyn.items():
        print(f'{k:32s} {v:11.3e} {v / total:7.1%} {v / 1024:9.0f} {cyc[k] / 1024:14.0f} {cyc[k] / ctot:8.1%}')
    wave = c['SQ_WAVE_CYCLES'] * 4 / 1024 if 'SQ_WAVE_CYCLES' in c else None
    print(f'issue-bound VALU cycles per wave {ctot / 1024:.0f}' + (f' of {wave:.0f} wave cycles ({ctot / 1024 / wave:.0%})' if wave else ''))


if __name__ == '__main__':
    main()
