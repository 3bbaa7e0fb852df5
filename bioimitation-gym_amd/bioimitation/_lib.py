"""ctypes binding of libbioim.so (include/bioim.h), the HIP product path.

The library is built in-tree by ``__graft_entry__.build()`` (hipcc,
--offload-arch=gfx950) into ``bioimitation-gym_amd/build/libbioim.so``.  There
is no CPU fallback: if the library or a GPU is missing, every constructor
raises.
"""
from __future__ import annotations

import ctypes as C
import os

from . import packdef as P

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get('BIOIM_LIB', os.path.join(PKG_ROOT, 'build', 'libbioim.so'))

EXPORTS = ['bioim_create', 'bioim_destroy', 'bioim_reset', 'bioim_step', 'bioim_set_auto_reset', 'bioim_set_env_offset', 'bioim_set_io_strides', 'bioim_step_group', 'bioim_set_group_fusion', 'bioim_group_fused', 'bioim_set_reset_table', 'bioim_reset_table_rows', 'bioim_set_perturbation', 'bioim_id_eval', 'bioim_state_dim',
           'bioim_get_state', 'bioim_set_state', 'bioim_query', 'bioim_query_launch', 'bioim_stream', 'bioim_set_stream', 'bioim_sync',
           'bioim_last_error', 'bioim_modelpack_size', 'bioim_build_id', 'bioim_reset_count', 'bioim_set_final_obs', 'bioim_set_integrator', 'bioim_force_report_dim', 'bioim_set_force_report',
           'bioim_set_rk_budget', 'bioim_pending_count', 'bioim_set_active_mask', 'bioim_osim', 'bioim_osim_report_dim', 'bioim_eval_count', 'bioim_set_state_storage',
           'bioim_finished_count', 'bioim_set_rk_counters', 'bioim_copy_state']

_lib = None


class BioimError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BioimError(f'libbioim.so not found at {LIB_PATH}; run __graft_entry__.build()')
    L = C.CDLL(LIB_PATH)
    vp, i32p, dp = C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_double)
    sig = {
        'bioim_create': (C.c_int, [C.POINTER(P.ModelPack), C.c_int, C.c_int, C.c_int, C.c_uint64, C.POINTER(vp)]),
        'bioim_destroy': (C.c_int, [vp]),
        'bioim_reset': (C.c_int, [vp, vp, vp, C.c_int, vp]),
        'bioim_step': (C.c_int, [vp, vp, vp, vp, vp, vp]),
        'bioim_set_auto_reset': (C.c_int, [vp, C.c_int]),
        'bioim_set_env_offset': (C.c_int, [vp, C.c_int]),
        'bioim_set_io_strides': (C.c_int, [vp, C.c_int, C.c_int, C.c_int]),
        'bioim_step_group': (C.c_int, [C.POINTER(vp), C.c_int, vp, vp, vp, vp, vp]),
        'bioim_set_group_fusion': (C.c_int, [C.c_int]),
        'bioim_group_fused': (C.c_int, [C.c_void_p]),
        'bioim_set_reset_table': (C.c_int, [C.c_void_p, C.c_int]),
        'bioim_reset_table_rows': (C.c_int, [C.c_void_p]),
        'bioim_set_perturbation': (C.c_int, [vp, C.c_int, C.c_int, dp, dp]),
        'bioim_id_eval': (C.c_int, [vp, C.c_int, C.c_int, vp, vp, vp, vp]),
        'bioim_state_dim': (C.c_int, [vp]),
        'bioim_get_state': (C.c_int, [vp, dp]),
        'bioim_set_state': (C.c_int, [vp, dp]),
        'bioim_query': (C.c_int, [vp, i32p]),
        'bioim_query_launch': (C.c_int, [vp, i32p]),
        'bioim_stream': (vp, [vp]),
        'bioim_set_stream': (C.c_int, [vp, vp]),
        'bioim_sync': (C.c_int, [vp]),
        'bioim_last_error': (C.c_char_p, []),
        'bioim_modelpack_size': (C.c_uint64, []),
        'bioim_build_id': (C.c_char_p, []),
        'bioim_reset_count': (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        'bioim_set_final_obs': (C.c_int, [vp, vp]),
        'bioim_set_integrator': (C.c_int, [vp, C.c_int, C.c_double]),
        'bioim_force_report_dim': (C.c_int, [vp]),
        'bioim_set_rk_budget': (C.c_int, [vp, C.c_int, vp]),
        'bioim_pending_count': (C.c_int, [vp]),
        'bioim_set_active_mask': (C.c_int, [vp, vp]),
        'bioim_set_force_report': (C.c_int, [vp, vp]),
        'bioim_osim': (C.c_int, [vp, C.c_int, vp, C.c_int, vp, vp, vp]),
        'bioim_osim_report_dim': (C.c_int, [vp]),
        'bioim_eval_count': (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        'bioim_finished_count': (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        'bioim_set_rk_counters': (C.c_int, [vp, C.c_uint32, C.c_uint32]),
        'bioim_copy_state': (C.c_int, [vp, vp]),
        'bioim_set_state_storage': (C.c_int, [vp, vp, C.c_int, vp]),
    }
    for name, (res, args) in sig.items():
        if 'BIOIM_LIB' in os.environ and not hasattr(L, name):
            continue   # an older variant build for a same-box A/B (tools/ab.sh): entry points it lacks stay unbound
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    if L.bioim_modelpack_size() != C.sizeof(P.ModelPack):
        raise BioimError('ModelPack layout mismatch between libbioim.so and packdef.py')
    check_build_id(L)
    _lib = L
    return L


def check_build_id(L):
    """A library built from other sources or flags than the tree it sits in
    is refused (set BIOIM_LIB to load a variant build on purpose)."""
    from . import _buildinfo
    if 'BIOIM_LIB' in os.environ:
        return
    if not _buildinfo.sources_present():
        # a library shipped without its sources (installed elsewhere): nothing to compare against
        import warnings
        warnings.warn(f'{LIB_PATH}: kernel sources not found next to the library; build id not checked')
        return
    got = L.bioim_build_id().decode()
    want = _buildinfo.build_id()
    if got != want:
        raise BioimError(f'{LIB_PATH} was built from other sources/flags (build id {got}, tree {want}); '
                         'run __graft_entry__.build()')


def check(rc):
    if rc < 0:
        raise BioimError(_lib.bioim_last_error().decode())
    return rc
