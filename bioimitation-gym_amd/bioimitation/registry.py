"""Registered environment IDs and their compile recipes.

Mirrors ``bioimitation/__init__.py:23-143`` (gym ``register`` + Ray
``register_env``): every ID maps to (model source, load-time transforms, env
semantics).  The env semantics are read off each reference env class, cited
per entry.  Compiled packs live in ``bioimitation/data/packs/<ID>.npz``.
"""
from __future__ import annotations

from .modelpack import EnvSpec

SLOW_TWITCH_2D = [0.499, 0.55, 0.5, 0.484, 0.546, 0.759, 0.721, 0.499, 0.55, 0.5, 0.484, 0.546, 0.759, 0.721]
SLOW_TWITCH_3D = [0.499, 0.55, 0.5, 0.484, 0.546, 0.759, 0.721, 0.484, 0.546, 0.759, 0.721, 0.499, 0.55, 0.5,
                  0.484, 0.546, 0.759, 0.721, 0.484, 0.546, 0.759, 0.721]

PD_COORDS_2D = ['pelvis_tilt', 'hip_flexion_r', 'knee_angle_r', 'ankle_angle_r',
                'hip_flexion_l', 'knee_angle_l', 'ankle_angle_l']

_PD_2D = dict(pd=True, pd_coords=PD_COORDS_2D, kp=[100, 100, 100, 50, 100, 100, 50], kv=[5, 5, 5, 2, 5, 5, 2])

# env id -> (model file relative to the reference data dir, transforms, spec kwargs)
RECIPES = {
    # torque_walking_imitation_env2D.py:18-366 (PD :117-149, done :249-277, reward :279-366)
    'TorqueWalkingImitation2D-v0': dict(
        model='2D/scale/model_scaled.osim', transforms=('predictive', 'torque'),
        reference='2D/walking_reference_data',
        spec=dict(muscle=False, three_d=False, cycle=132, n_episode=264, reset_hi=132,
                  acc_max=1e5, **_PD_2D)),
    # muscle_walking_imitation_env2D.py:17-403 (done :237-265, reward :267-358, COT :360-403)
    'MuscleWalkingImitation2D-v0': dict(
        model='2D/scale/model_scaled.osim', transforms=('predictive',),
        reference='2D/walking_reference_data',
        spec=dict(muscle=True, three_d=False, cycle=132, n_episode=264, reset_hi=132,
                  acc_max=1e4, slow_twitch=SLOW_TWITCH_2D)),
}

# muscle_{walking,running,locked_knee,palsy}_imitation_env3D.py share: done thresholds (limit force 1e4,
# |qdd| 1e6, calcn_r.z < calcn_l.z; :240-275), reward x (foot_l + foot_r) and exp(-0.5|da|) (:345-351)
_SPEC_3D = dict(muscle=True, three_d=True, acc_max=1e6, limit_force_max=1e4, action_r_scale=0.5,
                reward_feet=True, done_cross=True, slow_twitch=SLOW_TWITCH_3D)
_IK_3D = '3D/inverse_kinematics/task_InverseKinematics.mot'
_IK_PALSY = '02905/02905_PRE/inverse_kinematics/task_InverseKinematics.mot'

RECIPES.update({
    # muscle_walking_imitation_env3D.py: cycle 50 (:73), N = rows - 2 (:75), reset randint(0, cycle) (:144)
    'MuscleWalkingImitation3D-v0': dict(
        model='3D/scale/model_scaled.osim', transforms=('predictive',),
        reference='3D/walking_reference_data', ik=_IK_3D,
        spec=dict(cycle=50, n_episode='rows-2', reset_hi=50, **_SPEC_3D)),
    # muscle_running_imitation_env3D.py: cycle 70 (:177), N = rows - 2 (:76), reset randint(0, N/2) (:144).
    # Its running_reference_data/ is absent from the reference (no recipe, no IK): the only shipped 3D
    # trial (walking) is used, so Running3D differs from Walking3D in cycle/reset range only.
    'MuscleRunningImitation3D-v0': dict(
        model='3D/scale/model_scaled.osim', transforms=('predictive',),
        reference='3D/walking_reference_data', ik=_IK_3D,
        spec=dict(cycle=70, n_episode='rows-2', reset_hi='N/2', **_SPEC_3D)),
    # muscle_locked_knee_imitation_env3D.py: prosthetic transform (:104-126), cycle 50 (:75),
    # N = rows - 2 (:77), reset randint(0, cycle) (:169)
    'MuscleLockedKneeImitation3D-v0': dict(
        model='3D/scale/model_scaled.osim', transforms=('predictive', 'prosthetic'),
        reference='3D/walking_reference_data', ik=_IK_3D,
        spec=dict(cycle=50, n_episode='rows-2', reset_hi=50, **_SPEC_3D)),
    # muscle_palsy_imitation_env3D.py: the shipped, already-transformed 02905_PRE model_predictive.osim
    # (:45, :55-59), physics gets the raw action (:131), cycle 50 (:73), N = rows - 2 (:75), reset
    # randint(0, cycle) (:144)
    'MusclePalsyImitation3D-v0': dict(
        model='02905/02905_PRE/scale/model_predictive.osim', transforms=(),
        reference='02905/walking_reference_data', ik=_IK_PALSY,
        spec=dict(cycle=50, n_episode='rows-2', reset_hi=50, raw_action=True, **_SPEC_3D)),
})

# torque_*_imitation_env3D.py:128-139: PD on x = coordinate_pos (pelvis translations deleted)[0:11] and
# v = coordinate_vel (all 17)[[0, 4, 5, 6, 8, 8, 9, 10, 11, 12, 13]] — the speed indices do not match the
# position ones (pelvis_ty/tz, hip_rotation_r twice); reproduced as written
PD_COORDS_3D = ['pelvis_tilt', 'pelvis_list', 'pelvis_rotation', 'hip_flexion_r', 'hip_adduction_r',
                'hip_rotation_r', 'knee_angle_r', 'ankle_angle_r', 'hip_flexion_l', 'hip_adduction_l', 'hip_rotation_l']
PD_VCOORDS_3D = ['pelvis_tilt', 'pelvis_ty', 'pelvis_tz', 'hip_flexion_r', 'hip_rotation_r', 'hip_rotation_r',
                 'knee_angle_r', 'ankle_angle_r', 'hip_flexion_l', 'hip_adduction_l', 'hip_rotation_l']
_PD_3D = dict(pd=True, pd_coords=PD_COORDS_3D, pd_vcoords=PD_VCOORDS_3D,
              kp=[100, 100, 100, 100, 100, 50, 100, 100, 100, 100, 50], kv=[5, 5, 5, 5, 5, 2, 5, 5, 5, 5, 2])
# limit force 1e4, |qdd| 1e6 (the variants' is_done), exp(-|da|) action reward
_LOOSE = dict(limit_force_max=1e4, acc_max=1e6)
_IK_2D = '3D/inverse_kinematics/task_InverseKinematics.mot'

RECIPES.update({
    # muscle_locked_knee_imitation_env2D.py: never calls its convert_model_to_prosthetic (:102, no call
    # site), so the simulated model is the 2D muscle model; cycle 132, N = 2*cycle (:73-77), reset
    # randint(0, N/2) (:167), done limit 1e4 / qdd 1e6 (:281-283)
    'MuscleLockedKneeImitation2D-v0': dict(
        model='2D/scale/model_scaled.osim', transforms=('predictive',),
        reference='2D/walking_reference_data',
        spec=dict(muscle=True, three_d=False, cycle=132, n_episode=264, reset_hi=132, slow_twitch=SLOW_TWITCH_2D,
                  raw_action=True, **_LOOSE)),   # physics gets the raw action (:154)
    # muscle_running_imitation_env2D.py: cycle 70 (:176), N = rows - 2 (:73-75), reset randint(0, N/2)
    # (:142).  The reference never sets self.w_effort (:30-31) and raises AttributeError in get_reward
    # (:341); here w_effort = r_weights[1] as in every other env.  running_reference_data/ is absent:
    # the 2D walking tables are used.
    'MuscleRunningImitation2D-v0': dict(
        model='2D/scale/model_scaled.osim', transforms=('predictive',),
        reference='2D/walking_reference_data',
        spec=dict(muscle=True, three_d=False, cycle=70, n_episode='rows-2', reset_hi='N/2',
                  slow_twitch=SLOW_TWITCH_2D, raw_action=True, **_LOOSE)),   # raw action to physics (:129)
    # torque_running_imitation_env2D.py: cycle 70 (:195), N = rows - 2 (:76-78), reset N/2 (:161)
    'TorqueRunningImitation2D-v0': dict(
        model='2D/scale/model_scaled.osim', transforms=('predictive', 'torque'),
        reference='2D/walking_reference_data',
        spec=dict(muscle=False, three_d=False, cycle=70, n_episode='rows-2', reset_hi='N/2', **_PD_2D, **_LOOSE)),
    # torque_locked_knee_imitation_env2D.py: torque model, then knee_l/ankle_l locked (:61-62, :105-123);
    # their actuators stay (no effect on a locked coordinate); cycle 132, N = 2*cycle, reset N/2
    'TorqueLockedKneeImitation2D-v0': dict(
        model='2D/scale/model_scaled.osim', transforms=('predictive', 'torque', 'prosthetic'),
        reference='2D/walking_reference_data',
        spec=dict(muscle=False, three_d=False, cycle=132, n_episode=264, reset_hi=132, **_PD_2D, **_LOOSE)),
    # torque_walking_imitation_env3D.py: cycle 132 (:75), N = 2*cycle (:79), reset N/2 (:162),
    # effort |a|/(max_actuation*11^2) (:353), exp(-|da|) (:355), feet in the reward (:357)
    'TorqueWalkingImitation3D-v0': dict(
        model='3D/scale/model_scaled.osim', transforms=('predictive', 'torque'),
        reference='3D/walking_reference_data', ik=_IK_3D,
        spec=dict(muscle=False, three_d=True, cycle=132, n_episode=264, reset_hi=132, reward_feet=True,
                  done_cross=True, **_PD_3D, **_LOOSE)),
    # torque_running_imitation_env3D.py: cycle 70 (:195), N = rows - 2 (:76-78), reset N/2 (:161)
    'TorqueRunningImitation3D-v0': dict(
        model='3D/scale/model_scaled.osim', transforms=('predictive', 'torque'),
        reference='3D/walking_reference_data', ik=_IK_3D,
        spec=dict(muscle=False, three_d=True, cycle=70, n_episode='rows-2', reset_hi='N/2', reward_feet=True,
                  done_cross=True, **_PD_3D, **_LOOSE)),
    # torque_locked_knee_imitation_env3D.py: torque model, then prosthetic (:61-62); cycle 132, N = 2*cycle
    'TorqueLockedKneeImitation3D-v0': dict(
        model='3D/scale/model_scaled.osim', transforms=('predictive', 'torque', 'prosthetic'),
        reference='3D/walking_reference_data', ik=_IK_3D,
        spec=dict(muscle=False, three_d=True, cycle=132, n_episode=264, reset_hi=132, reward_feet=True,
                  done_cross=True, **_PD_3D, **_LOOSE)),
})

# mixed-topology batches (BASELINE.json config C5, bench.py --mixed): the prosthetic (12 dof,
# 19 muscles) next to the palsy model (14 dof, 22 muscles)
MIXED_BATCHES = [('MuscleLockedKneeImitation3D-v0', 'MusclePalsyImitation3D-v0')]

REGISTERED_IDS = [
    'TorqueWalkingImitation2D-v0', 'TorqueRunningImitation2D-v0', 'TorqueJumpingImitation2D-v0',
    'TorqueLockedKneeImitation2D-v0', 'TorqueWalkingImitation3D-v0', 'TorqueRunningImitation3D-v0',
    'TorqueJumpingImitation3D-v0', 'TorqueLockedKneeImitation3D-v0',
    'MuscleWalkingImitation2D-v0', 'MuscleRunningImitation2D-v0', 'MuscleJumpingImitation2D-v0',
    'MuscleLockedKneeImitation2D-v0', 'MuscleWalkingImitation3D-v0', 'MuscleRunningImitation3D-v0',
    'MuscleJumpingImitation3D-v0', 'MuscleLockedKneeImitation3D-v0', 'MusclePalsyImitation3D-v0',
]


# registered by the reference, not built here (why)
_NO_JUMP_DATA = ('its reference motion ({}_reference_data/task_Kinematics_q.sto etc.) is absent from the '
                 'reference and no jump IK trial ships to regenerate it from')
NOT_BUILT = {
    'MuscleJumpingImitation2D-v0': _NO_JUMP_DATA.format('2D/highjump'),
    'TorqueJumpingImitation2D-v0': _NO_JUMP_DATA.format('2D/highjump'),
    'TorqueJumpingImitation3D-v0': _NO_JUMP_DATA.format('3D/jumping'),
    'MuscleJumpingImitation3D-v0': _NO_JUMP_DATA.format('3D/jumping') +
    '; the reference class also fails at construction (self.cycle = self.N/2 before N is set, '
    'muscle_jumping_imitation_env3D.py:73)',
}
assert set(NOT_BUILT) | set(RECIPES) == set(REGISTERED_IDS)


def build_model(env_id: str, ref_data: str, transforms: tuple = None):
    """The simulated model of ``env_id``: its .osim under the reference's data
    dir with the recipe's load-time transforms applied (dev container only)."""
    import os
    from . import transforms as T
    from .osim import load_osim
    r = RECIPES[env_id]
    m = load_osim(os.path.join(ref_data, r['model']))
    for t in (r['transforms'] if transforms is None else transforms):
        if t == 'predictive':
            m = T.construct_predictive_model(m)
        elif t == 'torque':
            m = T.convert_model_to_torque_actuated(m, 200.0)
        elif t == 'prosthetic':
            m = T.convert_model_to_prosthetic(m)
        else:
            raise ValueError(t)
    return m


def env_spec(env_id: str, config: dict = None) -> EnvSpec:
    """EnvSpec for an ID with the user's env config (configs/env_default.py:7-15)."""
    cfg = dict(config or {})
    r = RECIPES[env_id]
    kw = dict(r['spec'])
    if 'r_weights' in cfg:
        kw['w_imitate'], kw['w_effort'], kw['w_action'] = [float(v) for v in cfg['r_weights']]
    if 'horizon' in cfg:
        kw['horizon'] = int(cfg['horizon'])
    if 'use_target_obs' in cfg:
        kw['use_target_obs'] = bool(cfg['use_target_obs'])
    if 'use_GRF' in cfg:
        kw['use_grf'] = bool(cfg['use_GRF'])
    if 'max_actuation' in cfg:
        kw['max_actuation'] = float(cfg['max_actuation'])
    return EnvSpec(env_id=env_id, **kw)


def _pack_path(env_id: str) -> str:
    import os
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'packs', env_id + '.npz')


def load_pack(env_id: str, config: dict = None):
    """The committed ModelPack of ``env_id`` with the user's env config
    applied (reward weights, horizon, obs switches, test mode)."""
    import numpy as np
    from . import packdef as P
    from .modelpack import pack_from_bytes
    if env_id not in RECIPES:
        if env_id in NOT_BUILT:
            raise NotImplementedError(f'{env_id}: {NOT_BUILT[env_id]}')
        raise KeyError(env_id)
    with np.load(_pack_path(env_id), allow_pickle=False) as z:
        pk = pack_from_bytes(z['pack'].tobytes())
    cfg = dict(config or {})
    spec = env_spec(env_id, cfg)
    pk.w_imitate, pk.w_effort, pk.w_action = spec.w_imitate, spec.w_effort, spec.w_action
    if spec.horizon < 1 or spec.horizon > P.MAX_HORIZON:
        raise ValueError(f'horizon must be in [1, {P.MAX_HORIZON}]')
    pk.horizon = spec.horizon
    pk.max_actuation = spec.max_actuation
    flags = pk.env_flags & ~(P.ENV_TARGET_OBS | P.ENV_GRF_OBS)
    flags |= P.ENV_TARGET_OBS if spec.use_target_obs else 0
    flags |= P.ENV_GRF_OBS if spec.use_grf else 0
    pk.env_flags = flags
    ntrans = sum(1 for c in (pk.coord_tx, pk.coord_ty, pk.coord_tz) if c >= 0)
    n = 1 + (pk.ncoord - ntrans) + 2 * pk.ncoord
    n += 2 * (pk.ncoord - 1) if spec.use_target_obs else 0
    n += 3 * pk.n_obs_bpos + 3 * pk.n_obs_bvel + 3 * pk.nmuscle
    n += 6 * pk.ncforce if spec.use_grf else 0
    pk.obs_dim = n
    if cfg.get('mode') == 'test':
        pk.n_episode = pk.nrows - 2   # muscle_walking_imitation_env2D.py:74-75
        pk.reset_hi = 0               # reset index 0 in test mode (:141-142)
    if 'nsub' in cfg:
        pk.nsub = int(cfg['nsub'])
    return pk
