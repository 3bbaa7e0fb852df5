"""Round 6 call o: the C3 kernel (topology 1) under other LLVM machine
schedulers, linked with the tree's other objects into build/ab/s_*/libbioim.so
(the shipped flags minus -amdgpu-sched-strategy=iterative-ilp, plus the
variant's strategy; s_default: none)."""
import os, subprocess, sys
from concurrent.futures import ThreadPoolExecutor
REPO = '/root/repo'
sys.path.insert(0, REPO)
import __graft_entry__ as g
from bioimitation import _buildinfo as B
tree = os.path.join(g.PKG_ROOT, 'build')
def build(name, strat):
    bdir = os.path.join(tree, 'ab', name); os.makedirs(bdir, exist_ok=True)
    fl = B.ARCH + ['-O3', '-std=c++17', '-fPIC', '-I' + B.INCLUDE, '-I' + B.CSRC, '-Wno-unused-result', '-Wno-unused-value']
    if strat:
        fl += ['-mllvm', '-amdgpu-sched-strategy=' + strat]
    obj = os.path.join(bdir, 'bioim_topo1.o')
    subprocess.check_call(['hipcc'] + fl + ['-DBIOIM_BUILD_ID="' + name + '"', '-DBIOIM_TOPO_ONLY=1', '-c', '-o', obj, B.SOURCES[0]])
    objs = [os.path.join(tree, f'bioim_{u}.o') for u in ['abi', 'fused'] + [f'topo{k}' for k in range(g._ntopologies())]]
    objs = [obj if o.endswith('bioim_topo1.o') else o for o in objs]
    lib = os.path.join(bdir, 'libbioim.so')
    subprocess.check_call(['hipcc'] + B.ARCH + ['-shared', '-fPIC', '-o', lib] + objs)
    return lib
V = {'s_default': None, 's_maxilp': 'max-ilp', 's_clause': 'max-memory-clause', 's_minreg': 'iterative-minreg', 's_maxocc': 'iterative-maxocc'}
with ThreadPoolExecutor(5) as ex:
    for r in ex.map(lambda kv: build(*kv), V.items()): print(r)
