"""Register-hazard regression guard over the built kernels (CPU).

tools/hazard_gate.py disassembles the in-tree build's device code objects and
counts, per kernel, the "risky" VGPR<->AGPR copies: made under a narrowed
EXEC, read after the join into a memory address (or never written in the
other lanes).  That is the pattern of the r03i fault (an RK kernel stored
through an env offset that only the resume branch's lanes had copied into an
AGPR).  Every built kernel is scanned — the env kernels in all
push / RK / force-report (REP) variants and the ID kernels, both precisions,
128 kernels — and the shipped build must have NONE (round 4; round 3 allowed
the counts of a GPU-verified build, which let 6 flagged copies stand in the
fp32 Muscle2D RK kernel).  An edit that makes the allocator introduce one is
caught here, before the GPU.  Runs only where the unit objects exist (the
build container).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, 'bioimitation-gym_amd', 'build')


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
    assert len(counts) >= 126, sorted(counts)
    assert any('Lb1EEv10LaunchArgs' in k for k in counts)        # the REP (force-report) variants are scanned
    risky = {k: v for k, v in counts.items() if v}
    assert not risky, f'kernels with risky VGPR<->AGPR copies: {risky}'


@pytest.mark.skipif(not _objects_current(), reason='needs the in-tree build objects (build container)')
def test_no_kernel_uses_scratch():
    """Every built kernel — step, RK, push, force-report (REP), fused, ID —
    runs out of registers and LDS alone: no scratch (private segment) in the
    code-object metadata.  Round 3 had 46 REP kernels spilling 0.6-2.9 KB per
    lane; round 4's first cut still 10."""
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    import hazard_gate
    res = hazard_gate.resources(BUILD)
    assert len(res) >= 126, sorted(res)
    spill = {k: v[0] for k, v in res.items() if v[0]}
    assert not spill, f'kernels with scratch (bytes/lane): {spill}'
    assert all(v[1] <= 512 for v in res.values())
