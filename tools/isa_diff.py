"""Compare the device ISA of two builds' unit objects, kernel by kernel
(labels and addresses normalised): shows that a source change left the
shipped kernels instruction-identical.

    python tools/isa_diff.py <build dir A> <build dir B> [unit ...]
"""
import glob
import os
import re
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import hazard_gate  # noqa: E402


def kernels(obj):
    with tempfile.TemporaryDirectory() as tmp:
        out = {}
        for name, body in hazard_gate.kernels(hazard_gate.disassemble(obj, tmp)):
            out[name] = [re.sub(r'<[^>]*>|0x[0-9a-f]+|\b[0-9a-f]{8,}\b', '#', ln) for ln in body]
        return out


def main():
    a, b = sys.argv[1:3]
    units = sys.argv[3:] or sorted(os.path.basename(f) for f in glob.glob(os.path.join(a, 'bioim_topo*.o')) +
                                   glob.glob(os.path.join(a, 'bioim_fused.o')))
    same = diff = 0
    for u in units:
        ka, kb = kernels(os.path.join(a, u)), kernels(os.path.join(b, u))
        for k in sorted(set(ka) | set(kb)):
            if ka.get(k) == kb.get(k):
                same += 1
            else:
                diff += 1
                print(f'{u}: {k[:90]} differs ({len(ka.get(k, []))} vs {len(kb.get(k, []))} instructions)')
    print(f'{same} kernels instruction-identical, {diff} differ')
    return 1 if diff else 0


if __name__ == '__main__':
    sys.exit(main())
