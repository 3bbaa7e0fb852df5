"""The product library exports every entry point include/bioim.h declares
(no compute calls: this runs without a GPU)."""
import ctypes as C
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    txt = open(os.path.join(REPO, 'include', 'bioim.h')).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(bioim_[a-z_]+)\s*\(', txt)))


def test_header_lists_the_boundary():
    names = declared_functions()
    for n in ('bioim_create', 'bioim_reset', 'bioim_step', 'bioim_get_state', 'bioim_set_state', 'bioim_destroy',
              'bioim_last_error'):
        assert n in names


def test_library_exports_every_declared_symbol():
    from bioimitation import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip('libbioim.so not built (run __graft_entry__.build())')
    lib = C.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared_functions()) <= set(_lib.EXPORTS) | {'bioim_debug_stamps'}


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from bioimitation import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip('libbioim.so not built')
    from bioimitation.vector_env import VectorEnv
    with pytest.raises(_lib.BioimError):
        VectorEnv('MuscleWalkingImitation2D-v0', 4)
