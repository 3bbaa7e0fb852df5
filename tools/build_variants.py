"""Build variant libraries of libbioim.so for same-box A/B runs
(tools/ab.sh): build/ab/<name>/libbioim.so with extra hipcc flags.

    python tools/build_variants.py [--units topo1,topo2] name=-DFLAG=1,-DOTHER=2 [name2=...]

The tree library (default flags) is built first if its id is stale.  With
``--units`` only those objects (abi, fused, topo0..topo6) are compiled with
the variant's flags and the rest are linked from the tree build's objects —
enough when the flags change kernel code only (the C-ABI and the launchers of
the other topologies are the tree's); about a minute per variant instead of
four."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402
from bioimitation import _buildinfo  # noqa: E402


def build_partial(name, extra, units):
    bdir = os.path.join(g.PKG_ROOT, 'build', 'ab', name)
    os.makedirs(bdir, exist_ok=True)
    tree = os.path.join(g.PKG_ROOT, 'build')
    bid = _buildinfo.build_id(extra)
    base = ['hipcc'] + _buildinfo.hipcc_flags(extra) + [f'-DBIOIM_BUILD_ID="{bid}"']
    allu = [('abi', ['-DBIOIM_ABI_ONLY']), ('fused', ['-DBIOIM_FUSED_ONLY'])] + \
        [(f'topo{k}', [f'-DBIOIM_TOPO_ONLY={k}']) for k in range(g._ntopologies())]

    def unit(u):
        uname, flags = u
        if uname not in units:
            return os.path.join(tree, f'bioim_{uname}.o')
        obj = os.path.join(bdir, f'bioim_{uname}.o')
        subprocess.check_call(base + flags + ['-c', '-o', obj + '.tmp', g.SOURCES[0]])
        os.replace(obj + '.tmp', obj)
        return obj
    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(unit, allu))
    lib = os.path.join(bdir, 'libbioim.so')
    subprocess.check_call(['hipcc'] + _buildinfo.ARCH + ['-shared', '-fPIC', '-o', lib + '.tmp'] + objs)
    os.replace(lib + '.tmp', lib)
    return lib


if __name__ == '__main__':
    args = sys.argv[1:]
    units = None
    if args and args[0] == '--units':
        units = set(args[1].split(','))
        args = args[2:]
    g.build_lib()
    jobs = []
    for arg in args:
        name, flags = arg.split('=', 1)
        jobs.append((name, [f for f in flags.split(',') if f]))
    if units:
        # variants in parallel (each compiles only its units)
        with ThreadPoolExecutor(max(1, 8 // max(1, len(units)))) as ex:
            for (name, extra), lib in zip(jobs, ex.map(lambda j: build_partial(j[0], j[1], units), jobs)):
                print(name, extra, '->', lib, flush=True)
    else:
        for name, extra in jobs:
            out = os.path.join(g.PKG_ROOT, 'build', 'ab', name, 'libbioim.so')
            g.build_lib(out=out, extra=extra, jobs=8)
            print(name, extra, '->', out, flush=True)
