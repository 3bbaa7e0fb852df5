"""Where does a kernel spill?  Reads `hipcc -g -S --offload-device-only`
output and tallies scratch loads/stores, AGPR moves and instruction counts
per source line (.loc), for one kernel symbol (substring match).

    python tools/spills.py k.s MuscleWalkingImitation2D_v0dE [file_substring]
"""
import collections
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    want_file = sys.argv[3] if len(sys.argv) > 3 else 'bioim_step.hip'
    lines = open(path).read().split('\n')
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2))
    start = next(i for i, l in enumerate(lines) if l.startswith('_Z') and sym in l.split(':')[0] and ':' in l)
    end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
    loc = None
    st, ld, agpr, ninst = (collections.Counter() for _ in range(4))
    for l in lines[start:end]:
        m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)\s+(\d+)', l)
        if m:
            f = files.get(int(m.group(1)), '?')
            loc = int(m.group(2)) if want_file in f else f'{f.split("/")[-1]}:{m.group(2)}'
            continue
        t = l.strip()
        if not t or t.startswith('.') or t.startswith(';') or t.endswith(':'):
            continue
        ninst[loc] += 1
        if t.startswith('scratch_store'):
            st[loc] += 1
        elif t.startswith('scratch_load'):
            ld[loc] += 1
        elif t.startswith('v_accvgpr'):
            agpr[loc] += 1
    print(f'instructions {sum(ninst.values())}  scratch stores {sum(st.values())}  loads {sum(ld.values())}  '
          f'accvgpr moves {sum(agpr.values())}')
    for name, c in (('scratch_store', st), ('scratch_load', ld), ('v_accvgpr', agpr), ('instructions', ninst)):
        print(name, c.most_common(12))


if __name__ == '__main__':
    main()
