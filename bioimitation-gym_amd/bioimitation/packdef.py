"""ctypes mirror of include/bioim_modelpack.h (keep the two in lock-step;
tests/test_modelpack.py checks sizeof against both shared libraries)."""
import ctypes as C

MAGIC = 0x4D4F4942
VERSION = 3   # include/bioim_modelpack.h BIOIM_PACK_VERSION

MAX_COORD = 24
MAX_CBODY = 12
MAX_OSBODY = 24
MAX_FN = 96
MAX_KNOTS = 1536
MAX_MUSCLE = 24
MAX_PATHPT = 160
MAX_SPHERE = 8
MAX_CFORCE = 4
MAX_LIMIT = 12
MAX_ACT = 24
MAX_CURVESEG = 6
MAX_OBSBODY = 12
MAX_REFROWS = 512
NREFBODY = 9
MAX_HORIZON = 8

FN_CONST, FN_LINEAR, FN_SPLINE = 0, 1, 2
PT_FIXED, PT_COND, PT_MOVING = 0, 1, 2

ENV_MUSCLE = 1 << 0
ENV_HAS_TZ = 1 << 1
ENV_REWARD_FEET = 1 << 2
ENV_DONE_CROSS = 1 << 3
ENV_RAW_ACTION = 1 << 4
ENV_TARGET_OBS = 1 << 5
ENV_GRF_OBS = 1 << 6
ENV_PD = 1 << 7
ENV_PHASE_ISTEP = 1 << 8

D = C.c_double
I = C.c_int32


class Fn(C.Structure):
    _fields_ = [('type', I), ('coord', I), ('knot_off', I), ('nknots', I), ('a', D), ('b', D)]


class CBody(C.Structure):
    _fields_ = [('parent', I), ('fn', I * 6), ('pad', I),
                ('R_pf', D * 9), ('p_pf', D * 3), ('R_mb', D * 9), ('p_mb', D * 3),
                ('axis', (D * 3) * 6), ('mass', D), ('com', D * 3), ('inertia', D * 6)]


class Coord(C.Structure):
    _fields_ = [('motion', I), ('locked', I), ('dof', I), ('cbody', I),
                ('default_value', D), ('range_min', D), ('range_max', D)]


class OsBody(C.Structure):
    _fields_ = [('cbody', I), ('pad', I), ('R', D * 9), ('p', D * 3), ('mass', D), ('com', D * 3)]


class PathPt(C.Structure):
    _fields_ = [('cbody', I), ('type', I), ('cond_coord', I), ('fn', I * 3),
                ('loc', D * 3), ('R', D * 9), ('p', D * 3), ('range_lo', D), ('range_hi', D)]


class Curve(C.Structure):
    _fields_ = [('nseg', I), ('pad', I),
                ('x', (D * 6) * MAX_CURVESEG), ('y', (D * 6) * MAX_CURVESEG),
                ('x0', D), ('y0', D), ('dydx0', D), ('x1', D), ('y1', D), ('dydx1', D)]


class Muscle(C.Structure):
    _fields_ = [('pt_off', I), ('npt', I),
                ('fiso', D), ('lopt', D), ('lts', D), ('alpha_opt', D), ('vmax', D),
                ('tau_act', D), ('tau_deact', D), ('amin', D), ('damping', D), ('default_act', D),
                ('width', D), ('lmin', D), ('slow_twitch', D), ('mass', D),
                ('fal', Curve), ('fv', Curve), ('fpe', Curve), ('fse', Curve)]


class Sphere(C.Structure):
    _fields_ = [('cbody', I), ('force', I), ('loc', D * 3), ('radius', D), ('obody', I), ('pad_', I)]


class CForce(C.Structure):
    _fields_ = [('stiffness', D), ('dissipation', D), ('static_friction', D), ('dynamic_friction', D),
                ('viscous_friction', D), ('transition_velocity', D)]


class Limit(C.Structure):
    _fields_ = [('coord', I), ('dof', I), ('qup', D), ('qlow', D), ('kup', D), ('klow', D),
                ('damping', D), ('trans', D)]


class CoordAct(C.Structure):
    _fields_ = [('coord', I), ('dof', I), ('optimal_force', D), ('min_control', D), ('max_control', D)]


class ModelPack(C.Structure):
    _fields_ = [
        ('magic', C.c_uint32), ('version', C.c_uint32), ('env_id', C.c_char * 48),
        ('ncoord', I), ('ndof', I), ('ncbody', I), ('nosbody', I),
        ('nfn', I), ('nknots', I), ('nmuscle', I), ('npathpt', I),
        ('nsphere', I), ('ncforce', I), ('nlimit', I), ('ncoordact', I),
        ('env_flags', C.c_uint32), ('nact', I), ('obs_dim', I), ('info_dim', I),
        ('nsub', I), ('horizon', I), ('cycle', I), ('n_episode', I), ('reset_hi', I),
        ('coord_tx', I), ('coord_ty', I), ('coord_tz', I),
        ('torso_body', I), ('calcn_r_body', I), ('calcn_l_body', I),
        ('n_obs_bpos', I), ('n_obs_bvel', I),
        ('obs_bpos', I * MAX_OBSBODY), ('obs_bvel', I * MAX_OBSBODY),
        ('rw_body', I * NREFBODY), ('pd_coord', I * MAX_ACT), ('pd_vcoord', I * MAX_ACT), ('pad0', I),
        ('step_size', D), ('w_imitate', D), ('w_effort', D), ('w_action', D),
        ('action_r_scale', D), ('max_actuation', D),
        ('total_mass', D), ('gravity', D * 3), ('height', D),
        ('torso_y_min', D), ('limit_force_max', D), ('acc_max', D),
        ('kp', D * MAX_ACT), ('kv', D * MAX_ACT),
        ('coord', Coord * MAX_COORD), ('cbody', CBody * MAX_CBODY), ('osbody', OsBody * MAX_OSBODY),
        ('fn', Fn * MAX_FN),
        ('knot_x', D * MAX_KNOTS), ('knot_y', D * MAX_KNOTS), ('knot_b', D * MAX_KNOTS),
        ('knot_c', D * MAX_KNOTS), ('knot_d', D * MAX_KNOTS),
        ('muscle', Muscle * MAX_MUSCLE), ('pathpt', PathPt * MAX_PATHPT),
        ('sphere', Sphere * MAX_SPHERE), ('cforce', CForce * MAX_CFORCE),
        ('limit', Limit * MAX_LIMIT), ('coordact', CoordAct * MAX_ACT),
        ('nrows', I), ('pad1', I),
        ('ref_istep', I * MAX_REFROWS), ('ref_time', D * MAX_REFROWS),
        ('ref_q', (D * MAX_COORD) * MAX_REFROWS), ('ref_u', (D * MAX_COORD) * MAX_REFROWS),
        ('ref_x', ((D * 3) * NREFBODY) * MAX_REFROWS),
    ]
