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


def _lib_or_skip():
    from bioimitation import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip('libbioim.so not built')
    return _lib, _lib.load()


def test_entry_points_reject_bad_arguments_without_touching_a_gpu():
    """Argument checks run before any device call: null handles and bad
    sizes return BIOIM_E_ARG (-1) with a message (include/bioim.h error
    convention), on a machine without a GPU too."""
    _lib, L = _lib_or_skip()
    from bioimitation.registry import load_pack
    vp = C.c_void_p
    h = vp()
    pk = load_pack('MuscleWalkingImitation2D-v0')
    assert L.bioim_create(None, 4, 0, 64, 0, C.byref(h)) == -1
    assert b'bad arguments' in L.bioim_last_error()
    assert L.bioim_create(C.byref(pk), 0, 0, 64, 0, C.byref(h)) == -1
    assert L.bioim_create(C.byref(pk), 4, 0, 16, 0, C.byref(h)) == -1
    assert b'precision' in L.bioim_last_error()
    assert L.bioim_reset(None, None, None, 1, None) == -1
    assert L.bioim_step(None, None, None, None, None, None) == -1
    assert L.bioim_set_auto_reset(None, 1) == -1
    assert L.bioim_set_env_offset(None, 0) == -1
    assert L.bioim_set_io_strides(None, 1, 1, 1) == -1
    assert L.bioim_step_group(None, 0, None, None, None, None, None) == -1
    assert L.bioim_set_perturbation(None, 0, 0, None, None) == -1
    assert L.bioim_id_eval(None, 0, 1, None, None, None, None) == -1
    assert L.bioim_get_state(None, None) == -1 and L.bioim_set_state(None, None) == -1
    assert L.bioim_query(None, None) == -1 and L.bioim_query_launch(None, None) == -1
    assert L.bioim_sync(None) == -1 and L.bioim_destroy(None) == 0
    assert L.bioim_modelpack_size() == C.sizeof(pk)


def test_create_rejects_a_pack_with_a_bad_magic():
    _lib, L = _lib_or_skip()
    from bioimitation.registry import load_pack
    pk = load_pack('TorqueWalkingImitation2D-v0')
    pk.magic = 0
    h = C.c_void_p()
    assert L.bioim_create(C.byref(pk), 4, 0, 64, 0, C.byref(h)) == -3     # BIOIM_E_PACK
    assert b'magic' in L.bioim_last_error()


def test_env_mask_validation_refuses_what_the_kernel_cannot_read():
    """VectorEnv.set_active_mask hands the mask's pointer to the step kernel,
    which reads one byte per env: a wrong dtype, device, length, shape or a
    non-contiguous view is refused before it reaches the library."""
    import torch
    from bioimitation.vector_env import check_env_mask
    dev = torch.device('cuda', 0)
    check_env_mask(None, 8, dev)
    with pytest.raises(ValueError, match='dtype'):
        check_env_mask(torch.zeros(8, dtype=torch.int64), 8, dev)
    with pytest.raises(ValueError, match='dtype'):
        check_env_mask(torch.zeros(8, dtype=torch.float32), 8, dev)
    with pytest.raises(ValueError, match='must be on'):
        check_env_mask(torch.zeros(8, dtype=torch.uint8), 8, dev)            # a CPU tensor
    with pytest.raises(ValueError, match='torch tensor'):
        check_env_mask([1] * 8, 8, dev)
    cpu = torch.device('cpu')      # the remaining checks, on a device this machine has
    with pytest.raises(ValueError, match='shape'):
        check_env_mask(torch.zeros(7, dtype=torch.uint8), 8, cpu)
    with pytest.raises(ValueError, match='shape'):
        check_env_mask(torch.zeros((2, 4), dtype=torch.bool), 8, cpu)
    with pytest.raises(ValueError, match='contiguous'):
        check_env_mask(torch.zeros(16, dtype=torch.uint8)[::2], 8, cpu)
    check_env_mask(torch.zeros(8, dtype=torch.bool), 8, cpu)


def test_set_active_mask_refuses_a_host_pointer():
    """The raw C entry refuses host memory (hipPointerGetAttributes) instead
    of letting the kernel read it; a null handle is an argument error."""
    _lib, L = _lib_or_skip()
    assert L.bioim_set_active_mask(None, None) == -1


def test_build_id_covers_the_build_recipe():
    """The per-object -D unit selectors and the link line live in
    __graft_entry__.py, so it is part of the build id."""
    from bioimitation import _buildinfo
    assert any(p.endswith('__graft_entry__.py') for p in _buildinfo.SOURCES)
    assert _buildinfo.sources_present()
