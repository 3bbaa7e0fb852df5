"""Register-hazard gate over the BUILT kernels (CPU, seconds): the device code
object of every libbioim.so unit (bioimitation-gym_amd/build/bioim_topo*.o) is
unbundled and disassembled, and tools/exec_hazard.py scans every env / ID
kernel for VGPR<->AGPR copies made under a narrowed EXEC whose value a later
read uses as a memory address ("masked-use+addr") or that no lane wrote
("undefined").  Either is the wrong-lane / fault incident class of DESIGN.md
5.5: the r03i build faulted in such a kernel.

    python tools/hazard_gate.py [build-dir] [-v]     # list risky copies; exit 1 if any
    python tools/hazard_gate.py [build-dir] --baseline   # record the per-kernel counts (profiles/r04)

The scan is conservative (it cannot tell that a later region selects a subset
of the copy's lanes); the shipped build carries none in any of its 128
kernels, and tests/test_hazard_gate.py requires exactly that.
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import exec_hazard as E  # noqa: E402

LLVM = '/opt/rocm/lib/llvm/bin'
TARGET = 'hipv4-amdgcn-amd-amdhsa--gfx950'


def disassemble(obj: str, tmp: str) -> list[str]:
    fb = os.path.join(tmp, os.path.basename(obj) + '.fatbin')
    co = os.path.join(tmp, os.path.basename(obj) + '.co')
    subprocess.check_call(['objcopy', '-O', 'binary', '--only-section=.hip_fatbin', obj, fb])
    subprocess.check_call([os.path.join(LLVM, 'clang-offload-bundler'), '--unbundle', f'--input={fb}', '--type=o',
                           f'--targets={TARGET}', f'--output={co}'])
    out = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--no-show-raw-insn', co],
                         check=True, capture_output=True, text=True).stdout
    return out.split('\n')


def kernels(lines: list[str]):
    """(name, [instruction lines in the scanner's syntax]) per kernel symbol"""
    cur, body = None, []
    for ln in lines:
        m = re.match(r'^[0-9a-f]+ <(_Z\S+)>:', ln)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur is None or not ln.startswith('\t'):
            continue
        body.append(ln.split('//')[0].strip())
    if cur:
        yield cur, body


RISKY = ('masked-use+addr', 'undefined', 'undefined+addr')


def _scan_unit(obj):
    out = []
    with tempfile.TemporaryDirectory() as tmp:
        for name, body in kernels(disassemble(obj, tmp)):
            if 'env_kernel' not in name and 'id_kernel' not in name:
                continue
            ins = E.parse(body)
            hits = E.scan(ins)
            out.append((name, len(ins), hits))
    return out


def scan_build(build_dir: str):
    """[(kernel, instructions, hits)] over every unit, units scanned in parallel"""
    from concurrent.futures import ProcessPoolExecutor
    objs = sorted(glob.glob(os.path.join(build_dir, 'bioim_topo*.o')) + glob.glob(os.path.join(build_dir, 'bioim_fused.o')))
    if not objs:
        raise FileNotFoundError(f'no bioim_topo*.o under {build_dir}')
    with ProcessPoolExecutor(min(8, len(objs))) as ex:
        return [k for unit in ex.map(_scan_unit, objs) for k in unit]


def _unit_resources(obj):
    """{kernel: (scratch bytes/lane, registers, AGPRs)} from the code object's
    metadata notes (.private_segment_fixed_size; .vgpr_count, which on gfx950
    is the unified VGPR + AGPR allocation; .agpr_count)"""
    out, cur = {}, {}
    with tempfile.TemporaryDirectory() as tmp:
        disassemble(obj, tmp)   # leaves the unbundled code object in tmp
        co = os.path.join(tmp, os.path.basename(obj) + '.co')
        notes = subprocess.run([os.path.join(LLVM, 'llvm-readelf'), '--notes', co],
                               check=True, capture_output=True, text=True).stdout
    for ln in notes.split('\n'):
        m = re.match(r'\s*(?:- )?\.(name|private_segment_fixed_size|vgpr_count|agpr_count):\s+(\S+)', ln)
        if not m:
            continue
        if ln.lstrip().startswith('- '):   # a new kernel record
            cur = {}
        cur[m.group(1)] = m.group(2)
        if {'name', 'private_segment_fixed_size', 'vgpr_count', 'agpr_count'} <= cur.keys():
            n = cur['name']
            if 'env_kernel' in n or 'id_kernel' in n:
                out[n] = (int(cur['private_segment_fixed_size']), int(cur['vgpr_count']), int(cur['agpr_count']))
            cur = {}
    return out


def resources(build_dir: str) -> dict:
    """{kernel: (scratch bytes/lane, registers, AGPRs)} over every unit of a build"""
    from concurrent.futures import ProcessPoolExecutor
    objs = sorted(glob.glob(os.path.join(build_dir, 'bioim_topo*.o')) + glob.glob(os.path.join(build_dir, 'bioim_fused.o')))
    if not objs:
        raise FileNotFoundError(f'no bioim_topo*.o under {build_dir}')
    res = {}
    with ProcessPoolExecutor(min(8, len(objs))) as ex:
        for unit in ex.map(_unit_resources, objs):
            res.update(unit)
    return res


def per_kernel(build_dir: str) -> dict:
    """risky copies per kernel symbol"""
    return {name: sum(1 for h in hits if h[4] in RISKY) for name, _, hits in scan_build(build_dir)}


def gate(build_dir: str, verbose: bool = False) -> int:
    risky_total = 0
    res = scan_build(build_dir)
    for name, n, hits in res:
        risky = [h for h in hits if h[4] in RISKY]
        risky_total += len(risky)
        if risky or verbose:
            print(f'{name[:96]}: {n} instructions, {len(hits)} candidate copies, {len(risky)} risky')
        for i, raw, j, use, kind in risky:
            print(f'    [{i}] {raw:50s} -> read after join at [{j}] {use:45s} {kind}')
    print(f'hazard gate: {risky_total} risky copies in {len(res)} kernels')
    return risky_total


if __name__ == '__main__':
    args = [a for a in sys.argv[1:] if not a.startswith('-')]
    d = args[0] if args else os.path.join(os.path.dirname(HERE), 'bioimitation-gym_amd', 'build')
    if '--baseline' in sys.argv:   # record the per-kernel counts of a GPU-verified build
        import json
        out = os.path.join(os.path.dirname(HERE), 'profiles', 'r04', 'hazard_baseline.json')
        json.dump({'build': os.path.relpath(d, os.path.dirname(HERE)), 'risky': per_kernel(d)},
                  open(out, 'w'), indent=1, sort_keys=True)
        print('wrote', out)
        sys.exit(0)
    sys.exit(1 if gate(d, verbose='-v' in sys.argv) else 0)
