"""One place for the hipcc flags of libbioim.so and the build id that ties a
built library to its sources.

Used by ``__graft_entry__.build_lib`` (the product build), by the tools that
must see the same binary (``tools/resources.sh``, ``tools/build_stamps.sh``,
``tools/phase_isa.py`` via ``python -m bioimitation._buildinfo flags``), and
by ``_lib.load()``, which refuses a library whose exported
``bioim_build_id()`` differs from the id of the sources next to it.
"""
from __future__ import annotations

import hashlib
import os
import sys

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, 'csrc')
INCLUDE = os.path.join(REPO, 'include')
SOURCES = [os.path.join(CSRC, f) for f in ('bioim_step.hip', 'bioim_device.h', 'topologies.h')] + \
    [os.path.join(INCLUDE, f) for f in ('bioim.h', 'bioim_modelpack.h')] + \
    [os.path.join(REPO, '__graft_entry__.py')]   # the per-object -D unit selectors and the link line live there

# LLVM's iterative ILP machine scheduler for gfx950: the step kernel runs one
# wave per SIMD and is latency-bound, and this schedule shortens its dependent
# chains (same-box A/B: 2D 0.4411 -> 0.4084 ms, 3D 0.6741 -> 0.6359 ms per
# step; profiles/r01i/ab_sched*.log; the default, max-occupancy-oriented
# iterative, min-register and memory-clause strategies were all slower).
SCHED = ['-mllvm', '-amdgpu-sched-strategy=iterative-ilp']

ARCH = ['--offload-arch=gfx950']


def hipcc_flags(extra=()):
    """Compile flags of every libbioim.so object (the -D unit selectors and
    the build id define are added per object by the build)."""
    return ARCH + ['-O3', '-std=c++17', '-fPIC', '-I' + INCLUDE, '-I' + CSRC,
                   '-Wno-unused-result', '-Wno-unused-value'] + SCHED + list(extra)


def sources_present():
    return all(os.path.exists(f) for f in SOURCES)


def build_id(extra=()):
    """sha256 over the kernel sources, the build recipe and the compile
    flags, 16 hex digits."""
    h = hashlib.sha256()
    for f in SOURCES:
        h.update(os.path.basename(f).encode())
        with open(f, 'rb') as fh:
            h.update(fh.read())
    h.update(' '.join(hipcc_flags(extra)).replace(REPO, '<repo>').encode())
    return h.hexdigest()[:16]


if __name__ == '__main__':
    cmd = sys.argv[1] if len(sys.argv) > 1 else 'flags'
    if cmd == 'flags':
        print(' '.join(hipcc_flags()))
    elif cmd == 'id':
        print(build_id())
    else:
        raise SystemExit(f'usage: python -m bioimitation._buildinfo [flags|id]')
