"""Register-hazard regression guard over the built kernels (CPU).

tools/hazard_gate.py disassembles the in-tree build's device code objects and
counts, per kernel, the "risky" VGPR<->AGPR copies: made under a narrowed
EXEC, read after the join into a memory address (or never written in the
other lanes).  That is the pattern of the r03i fault (an RK kernel stored
through an env offset that only the resume branch's lanes had copied into an
AGPR).  The scan is linear and conservative, so GPU-verified
kernels carry some such candidates too; the guard is that no kernel has MORE
of them than in the last GPU-verified build (profiles/r03/hazard_baseline.json),
so an edit that makes the allocator introduce a new one is caught here, before
the GPU.  Runs only where the unit objects exist (the build container).
"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, 'bioimitation-gym_amd', 'build')
BASELINE = os.path.join(REPO, 'profiles', 'r03', 'hazard_baseline.json')


def _objects_current():
    import glob
    objs = glob.glob(os.path.join(BUILD, 'bioim_topo*.o'))
    lib = os.path.join(BUILD, 'libbioim.so')
    return objs and os.path.exists(lib) and all(os.path.getmtime(o) <= os.path.getmtime(lib) + 1 for o in objs)


@pytest.mark.skipif(not _objects_current(), reason='needs the in-tree build objects (build container)')
def test_no_new_risky_register_copies():
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    import hazard_gate
    counts = hazard_gate.per_kernel(BUILD)
    base = json.load(open(BASELINE))['risky']
    worse = {k: (base.get(k, 0), v) for k, v in counts.items() if v > base.get(k, 0)}
    assert not worse, f'kernels with more risky copies than the GPU-verified build (baseline, now): {worse}'
