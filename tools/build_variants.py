"""Build variant libraries of libbioim.so for same-box A/B runs
(tools/ab.sh): build/ab/<name>/libbioim.so with extra hipcc flags.
    python tools/build_variants.py name=-DFLAG=1,-DOTHER=2 [name2=...]
The tree library (default flags) is built first if its id is stale."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as g  # noqa: E402

g.build_lib()
for arg in sys.argv[1:]:
    name, flags = arg.split('=', 1)
    extra = [f for f in flags.split(',') if f]
    out = os.path.join(g.PKG_ROOT, 'build', 'ab', name, 'libbioim.so')
    g.build_lib(out=out, extra=extra, jobs=8)
    print(name, extra, '->', out, flush=True)
