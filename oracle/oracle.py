"""ctypes loader for the fp64 CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: importable from tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product path never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'liboracle.so')

_dp = C.POINTER(C.c_double)


def build(force=False):
    if force or not os.path.exists(LIB):
        subprocess.check_call(['make', '-s', '-C', HERE])
    return LIB


def _ptr(a):
    return a.ctypes.data_as(_dp)


class Oracle:
    def __init__(self, pack):
        build()
        self.lib = C.CDLL(LIB)
        L = self.lib
        for name, res, args in [
            ('orc_env_size', C.c_size_t, []), ('orc_pack_size', C.c_size_t, []),
            ('orc_state_dim', C.c_int, [C.c_void_p]),
            ('orc_env_reset', C.c_int, [C.c_void_p, C.c_void_p, C.c_int, _dp]),
            ('orc_env_step', C.c_int, [C.c_void_p, C.c_void_p, _dp, _dp, _dp, C.POINTER(C.c_int), _dp]),
            ('orc_get_state', None, [C.c_void_p, C.c_void_p, _dp]),
            ('orc_set_state', None, [C.c_void_p, C.c_void_p, _dp]),
            ('orc_env_init', None, [C.c_void_p]),
            ('orc_id_eval', C.c_int, [C.c_void_p, C.c_int, _dp, _dp, _dp, _dp]),
            ('orc_env_set_perturbation', C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, _dp, _dp]),
            ('orc_forward_kinematics', None, [C.c_void_p, _dp, _dp, _dp, _dp]),
            ('orc_mass_matrix_bias', None, [C.c_void_p, _dp, _dp, _dp, _dp]),
            ('orc_forward_dynamics', C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, _dp, _dp, _dp]),
            ('orc_muscle_path', None, [C.c_void_p, _dp, _dp, C.c_int, _dp, _dp, _dp]),
            ('orc_muscle_paths', None, [C.c_void_p, _dp, _dp, _dp, _dp, _dp]),
            ('orc_curve', C.c_double, [C.c_void_p, C.c_int, C.c_int, C.c_double, _dp]),
            ('orc_fn', C.c_double, [C.c_void_p, C.c_int, C.c_double, _dp, _dp]),
            ('orc_muscle_equilibrium', C.c_double, [C.c_void_p, C.c_int, C.c_double, C.c_double]),
            ('orc_contact', None, [C.c_void_p, _dp, _dp, _dp, _dp]),
            ('orc_batch_step', C.c_int, [C.c_void_p, C.c_int, C.c_void_p, _dp, _dp, _dp,
                                         C.POINTER(C.c_int32), _dp, C.c_int]),
            ('orc_env_set_integrator', C.c_int, [C.c_void_p, C.c_int, C.c_double]),
            ('orc_env_rk_stats', None, [C.c_void_p, _dp]),
            ('orc_force_report', C.c_int, [C.c_void_p, C.c_void_p, _dp]),
            ('orc_osim_reset', None, [C.c_void_p, C.c_void_p]),
            ('orc_osim_set_time', None, [C.c_void_p, C.c_void_p, C.c_double]),
            ('orc_osim_set_coords', None, [C.c_void_p, C.c_void_p, _dp, C.c_int]),
            ('orc_osim_actuate', None, [C.c_void_p, C.c_void_p, _dp]),
            ('orc_osim_integrate', None, [C.c_void_p, C.c_void_p]),
            ('orc_osim_reset_manager', None, [C.c_void_p, C.c_void_p]),
            ('orc_osim_full_report_dim', C.c_int, [C.c_void_p]),
            ('orc_osim_full_report', None, [C.c_void_p, C.c_void_p, _dp]),
            ('orc_env_observe', None, [C.c_void_p, C.c_void_p, _dp]),
            ('orc_env_set_state_storage', None, [C.c_void_p, _dp, C.c_int]),
            ('orc_env_state_storage_count', C.c_int, [C.c_void_p]),
        ]:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.orc_pack_size() != C.sizeof(pack):
            raise RuntimeError('ModelPack layout mismatch between oracle and packdef.py')
        self.pack = pack
        self.pk = C.byref(pack)
        self.env_size = L.orc_env_size()

    # ------------------------------------------------------------ env
    def new_envs(self, n):
        buf = C.create_string_buffer(self.env_size * n)
        for i in range(n):
            self.lib.orc_env_init(C.byref(buf, i * self.env_size))
        return buf

    def env_ptr(self, envs, i):
        return C.byref(envs, i * self.env_size)

    def reset(self, envs, i, index):
        obs = np.zeros(self.pack.obs_dim)
        self.lib.orc_env_reset(self.pk, self.env_ptr(envs, i), int(index), _ptr(obs))
        return obs

    def step(self, envs, i, action):
        a = np.ascontiguousarray(action, dtype=np.float64)
        obs = np.zeros(self.pack.obs_dim)
        rew = np.zeros(1)
        info = np.zeros(self.pack.info_dim)
        done = C.c_int(0)
        self.lib.orc_env_step(self.pk, self.env_ptr(envs, i), _ptr(a), _ptr(obs), _ptr(rew), C.byref(done),
                              _ptr(info))
        return obs, float(rew[0]), bool(done.value), info

    def set_perturbation(self, envs, i, os_body, x, y):
        """Zero-order-hold torso force table of env i (see orc_env_t)"""
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.ascontiguousarray(y, dtype=np.float64)
        rc = self.lib.orc_env_set_perturbation(self.pk, self.env_ptr(envs, i), int(os_body), len(x), _ptr(x), _ptr(y))
        if rc:
            raise ValueError('orc_env_set_perturbation: bad table')

    def set_integrator(self, envs, i, kind, accuracy=1e-3):
        """kind 'euler' (the kernel's fixed-substep semi-implicit scheme) or
        'rk-merson' (the reference's adaptive integrator at `accuracy`)."""
        k = {'euler': 0, 'rk-merson': 1, 'extrap2': 2, 'extrap3': 3, 'extrap-adaptive': 4}[kind]
        if self.lib.orc_env_set_integrator(self.env_ptr(envs, i), k, float(accuracy)):
            raise ValueError('orc_env_set_integrator: bad arguments')

    def rk_stats(self, envs, i):
        """(accepted steps, rejected steps, smallest step, next step, dynamics
        evaluations) since set_integrator"""
        out = np.zeros(5)
        self.lib.orc_env_rk_stats(self.env_ptr(envs, i), _ptr(out))
        return out

    def force_report(self, envs, i):
        """per-force-element values of env i's realized state (bioim_set_force_report layout)"""
        pk = self.pack
        out = np.zeros(pk.nact + 6 * pk.ncforce + pk.nlimit + 6 * pk.nsphere)
        self.lib.orc_force_report(self.pk, self.env_ptr(envs, i), _ptr(out))
        return out

    # ------------------------------------------------------------ OsimModel calls
    # (opensim_wrapper.py:92-332 restated; the HIP path's bioim_osim)
    def osim_reset(self, envs, i):
        self.lib.orc_osim_reset(self.pk, self.env_ptr(envs, i))

    def osim_set_time(self, envs, i, t):
        self.lib.orc_osim_set_time(self.pk, self.env_ptr(envs, i), float(t))

    def osim_set_coords(self, envs, i, qfull, speeds=False):
        """all coordinates in CoordinateSet order (locked ones are ignored)"""
        v = np.ascontiguousarray(qfull, dtype=np.float64)
        self.lib.orc_osim_set_coords(self.pk, self.env_ptr(envs, i), _ptr(v), int(bool(speeds)))

    def osim_actuate(self, envs, i, action):
        a = np.ascontiguousarray(action, dtype=np.float64)
        self.lib.orc_osim_actuate(self.pk, self.env_ptr(envs, i), _ptr(a))

    def osim_integrate(self, envs, i):
        self.lib.orc_osim_integrate(self.pk, self.env_ptr(envs, i))

    def osim_reset_manager(self, envs, i):
        self.lib.orc_osim_reset_manager(self.pk, self.env_ptr(envs, i))

    def osim_report(self, envs, i):
        """the realized state of env i, include/bioim.h bioim_osim report layout"""
        out = np.zeros(self.lib.orc_osim_full_report_dim(self.pk))
        self.lib.orc_osim_full_report(self.pk, self.env_ptr(envs, i), _ptr(out))
        return out

    def set_state_storage(self, envs, i, buf):
        """buf: float64 array (capacity, 1 + 2 ndof + 2 nm) kept alive by the
        caller, or None"""
        if buf is None:
            self.lib.orc_env_set_state_storage(self.env_ptr(envs, i), None, 0)
        else:
            assert buf.dtype == np.float64 and buf.flags.c_contiguous
            self.lib.orc_env_set_state_storage(self.env_ptr(envs, i), _ptr(buf), buf.shape[0])

    def state_storage_count(self, envs, i):
        return self.lib.orc_env_state_storage_count(self.env_ptr(envs, i))

    def observe(self, envs, i):
        """env i's observation at its current state"""
        obs = np.zeros(self.pack.obs_dim)
        self.lib.orc_env_observe(self.pk, self.env_ptr(envs, i), _ptr(obs))
        return obs

    def state_dim(self):
        return self.lib.orc_state_dim(self.pk)

    def get_state(self, envs, i):
        s = np.zeros(self.state_dim())
        self.lib.orc_get_state(self.pk, self.env_ptr(envs, i), _ptr(s))
        return s

    def set_state(self, envs, i, s):
        s = np.ascontiguousarray(s, dtype=np.float64)
        self.lib.orc_set_state(self.pk, self.env_ptr(envs, i), _ptr(s))

    def batch_step(self, envs, n, actions, nthreads=1, want_obs=True):
        actions = np.ascontiguousarray(actions, dtype=np.float64)
        obs = np.zeros((n, self.pack.obs_dim)) if want_obs else None
        rew = np.zeros(n)
        info = np.zeros((n, self.pack.info_dim))
        done = np.zeros(n, dtype=np.int32)
        self.lib.orc_batch_step(self.pk, n, envs, _ptr(actions), _ptr(obs) if want_obs else None, _ptr(rew),
                                done.ctypes.data_as(C.POINTER(C.c_int32)), _ptr(info), int(nthreads))
        return obs, rew, done.astype(bool), info

    # ------------------------------------------------------------ physics probes
    def fk(self, qfull_dofs):
        n = self.pack.nosbody
        R = np.zeros((n, 9))
        p = np.zeros((n, 3))
        com = np.zeros(3)
        q = np.ascontiguousarray(qfull_dofs, dtype=np.float64)
        self.lib.orc_forward_kinematics(self.pk, _ptr(q), _ptr(R), _ptr(p), _ptr(com))
        return R.reshape(n, 3, 3), p, com

    def mass_bias(self, q, u):
        nd = self.pack.ndof
        M = np.zeros((nd, nd))
        b = np.zeros(nd)
        q = np.ascontiguousarray(q, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        self.lib.orc_mass_matrix_bias(self.pk, _ptr(q), _ptr(u), _ptr(M), _ptr(b))
        return M, b

    def forward_dynamics(self, q, u, act, lce, controls):
        nd, nm = self.pack.ndof, max(1, self.pack.nmuscle)
        qdd = np.zeros(nd)
        mo = np.zeros((nm, 8))
        args = [np.ascontiguousarray(x, dtype=np.float64) for x in (q, u, act, lce, controls)]
        rc = self.lib.orc_forward_dynamics(self.pk, *[_ptr(x) for x in args], _ptr(qdd), _ptr(mo))
        return qdd, mo, rc

    def id_eval(self, op, q, u=None, v=None):
        """inverse-dynamics primitive op (include/bioim.h BIOIM_ID_*), per-dof vectors"""
        nd = self.pack.ndof
        z = np.zeros(nd)
        q, u, v = (np.ascontiguousarray(z if x is None else x, dtype=np.float64) for x in (q, u, v))
        out = np.zeros(nd)
        if self.lib.orc_id_eval(self.pk, int(op), _ptr(q), _ptr(u), _ptr(v), _ptr(out)):
            raise ValueError('orc_id_eval failed (M not SPD?)')
        return out

    def muscle_path(self, q, u, m):
        L, Ld = C.c_double(), C.c_double()
        d = np.zeros(self.pack.ndof)
        q = np.ascontiguousarray(q, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        self.lib.orc_muscle_path(self.pk, _ptr(q), _ptr(u), int(m), C.byref(L), C.byref(Ld), _ptr(d))
        return L.value, Ld.value, d

    def muscle_paths(self, q, u):
        """(L[nm], dL/dt[nm], dL/dq[nm][nd]) of every muscle from one kinematics pass"""
        nm, nd = self.pack.nmuscle, self.pack.ndof
        L, Ld, d = np.zeros(nm), np.zeros(nm), np.zeros((nm, nd))
        q = np.ascontiguousarray(q, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        self.lib.orc_muscle_paths(self.pk, _ptr(q), _ptr(u), _ptr(L), _ptr(Ld), _ptr(d))
        return L, Ld, d

    def curve(self, m, which, x):
        d = C.c_double()
        y = self.lib.orc_curve(self.pk, int(m), int(which), float(x), C.byref(d))
        return y, d.value

    def fn(self, fi, q):
        d1, d2 = C.c_double(), C.c_double()
        v = self.lib.orc_fn(self.pk, int(fi), float(q), C.byref(d1), C.byref(d2))
        return v, d1.value, d2.value

    def muscle_equilibrium(self, m, a, L):
        return self.lib.orc_muscle_equilibrium(self.pk, int(m), float(a), float(L))

    def contact(self, q, u):
        tau = np.zeros(self.pack.ndof)
        w = np.zeros(6 * max(1, self.pack.ncforce))
        q = np.ascontiguousarray(q, dtype=np.float64)
        u = np.ascontiguousarray(u, dtype=np.float64)
        self.lib.orc_contact(self.pk, _ptr(q), _ptr(u), _ptr(tau), _ptr(w))
        return tau, w
