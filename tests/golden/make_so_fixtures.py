"""Fixtures that pin the model's dynamics to OpenSim's own output: the
reference ships OpenSim StaticOptimization results (task_StaticOptimization_
controls.xml: every muscle activation and every reserve / residual actuator
control, 0.01 s apart) together with all their inputs — the IK solution, the
measured ground reaction forces (task_grf.mot + setup_grf.xml), the reserve
actuators (model/reserve_actuators.xml) and the setup (setup_so.xml).
Static optimization enforces, at every frame, that the actuators reproduce
the inverse-dynamics generalized forces of the model under those loads; so
the same balance evaluated on OUR model (tests/test_so_pin.py) pins masses,
inertias, gravity, joint kinematics, moment arms and the Millard curves.

Runs in the dev container only (reads /root/reference); the committed npz is
data (inputs and outputs of the reference's OpenSim runs).

    python tests/golden/make_so_fixtures.py
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DATA = '/root/reference/bioimitation/imitation_envs/data'
sys.path.insert(0, os.path.join(REPO, 'bioimitation-gym_amd'))

from bioimitation.obslayout import load_names  # noqa: E402
from bioimitation.storage import read_sto  # noqa: E402

TRIALS = {'3D': ('3D', 'MuscleRunningImitation3D-v0'),
          # the palsy subject's model family: explicit Millard curve parameters (model_predictive.osim:1851-1870)
          '02905': ('02905/02905_PRE', 'MusclePalsyImitation3D-v0')}


def _vec(txt):
    return np.array([float(x) for x in txt.split()])


def read_controls(path):
    x = open(path).read()
    names, series = [], []
    for m in re.finditer(r'<ControlLinear name="([^"]+)">(.*?)</ControlLinear>', x, re.S):
        nodes = re.findall(r'<t>([^<]+)</t>\s*<value>([^<]+)</value>', m.group(2))
        names.append(m.group(1))
        series.append(np.array([[float(t), float(v)] for t, v in nodes]))
    t = series[0][:, 0]
    assert all(np.array_equal(s[:, 0], t) for s in series)
    return t, names, np.stack([s[:, 1] for s in series], axis=1)


def read_reserves(path):
    x = open(path).read()
    x = re.sub(r'<!--.*?-->', '', x, flags=re.S)
    out = {}
    for kind in ('CoordinateActuator', 'PointActuator', 'TorqueActuator'):
        for m in re.finditer(rf'<{kind} name="([^"]+)">(.*?)</{kind}>', x, re.S):
            if m.group(1) == 'default':
                continue
            b = m.group(2)

            def tag(t, d=None):
                r = re.search(rf'<{t}>([^<]*)</{t}>', b)
                return r.group(1).strip() if r else d
            out[m.group(1)] = dict(kind=kind, coord=tag('coordinate', ''), body=tag('body', tag('bodyA', '')),
                                   point=_vec(tag('point', '0 0 0')), direction=_vec(tag('direction', tag('axis', '0 0 0'))),
                                   optimal_force=float(tag('optimal_force', '1')),
                                   point_global=tag('point_is_global', 'false') == 'true',
                                   vec_global=(tag('force_is_global', tag('torque_is_global', 'false')) == 'true'))
    return out


def main():
    for tag_, (sub, env_id) in TRIALS.items():
        d = os.path.join(DATA, sub)
        setup = re.sub(r'<!--.*?-->', '', open(os.path.join(d, 'static_optimization', 'setup_so.xml')).read(), flags=re.S)
        assert re.search(r'<use_muscle_physiology>true', setup) and re.search(r'<activation_exponent>2', setup)
        cutoff = float(re.search(r'<lowpass_cutoff_frequency_for_coordinates>([^<]+)<', setup).group(1))
        names = load_names(env_id)
        hdr, labels, ik = read_sto(os.path.join(d, 'inverse_kinematics', 'task_InverseKinematics.mot'))
        coords = [c for c in labels if c != 'time']
        assert coords == names['coords']
        q = ik[:, 1:].copy()
        rot = np.array(names['coord_rotational'], dtype=bool)
        if hdr.get('inDegrees', 'no').lower() == 'yes':
            q[:, rot] = np.deg2rad(q[:, rot])
        gpath = os.path.join(d, 'experimental_data', 'setup_grf.xml')
        if not os.path.exists(gpath):
            # 02905_PRE's setup_so.xml names ../experimental_data/setup_grf.xml, which the
            # reference does not ship; its task_grf.mot has the 3D trial's columns
            # (left_/right_ground_force_v*, _p*, left_/right_ground_torque_*), so the 3D
            # trial's ExternalLoads mapping (same lab pipeline: right -> calcn_r, left -> calcn_l,
            # force and point in ground) is used
            gpath = os.path.join(DATA, '3D', 'experimental_data', 'setup_grf.xml')
        grf_setup = re.sub(r'<!--.*?-->', '', open(gpath).read(), flags=re.S)
        ext = []
        for m in re.finditer(r'<ExternalForce name="([^"]+)">(.*?)</ExternalForce>', grf_setup, re.S):
            b = m.group(2)

            def tg(t):
                return re.search(rf'<{t}>([^<]*)</{t}>', b).group(1).strip()
            assert tg('force_expressed_in_body') == 'ground' and tg('point_expressed_in_body') == 'ground'
            ext.append((tg('applied_to_body'), tg('force_identifier'), tg('point_identifier'), tg('torque_identifier')))
        # setup_grf.xml's <lowpass_cutoff_frequency> filters the load KINEMATICS (used only to
        # re-express points given in a body frame); these points are in ground, so the GRF data
        # enter unfiltered.
        _, glabels, grf = read_sto(os.path.join(d, 'experimental_data', 'task_grf.mot'))
        cols = []
        for body, fi, pi, ti in ext:
            cols.append([glabels.index(f'{fi}{a}') for a in 'xyz'] + [glabels.index(f'{pi}{a}') for a in 'xyz'] +
                        [glabels.index(f'{ti}{a}') for a in 'xyz'])
        so_t, so_names, so_v = read_controls(os.path.join(d, 'static_optimization',
                                                         'task_StaticOptimization_controls.xml'))
        res = read_reserves(os.path.normpath(os.path.join(d, 'static_optimization',
                                                          re.search(r'<force_set_files>([^<]+)<', setup).group(1).strip())))
        kinds, rcoord, rbody, rpoint, rdir, ropt, rpg, rvg = [], [], [], [], [], [], [], []
        for n in so_names:
            if n in names['muscles']:
                kinds.append('muscle'); rcoord.append(-1); rbody.append(''); rpoint.append(np.zeros(3))
                rdir.append(np.zeros(3)); ropt.append(0.0); rpg.append(False); rvg.append(False)
                continue
            r = res[n]
            kinds.append(r['kind']); rcoord.append(coords.index(r['coord']) if r['coord'] else -1)
            rbody.append(r['body']); rpoint.append(r['point']); rdir.append(r['direction'])
            ropt.append(r['optimal_force']); rpg.append(r['point_global']); rvg.append(r['vec_global'])
        out = dict(env_id=env_id, coords=np.array(coords), ik_time=ik[:, 0], ik_q=q, coord_cutoff=cutoff,
                   grf_time=grf[:, 0], grf=grf[:, np.array(cols).ravel()].reshape(len(grf), len(ext), 9),
                   grf_bodies=np.array([e[0] for e in ext]),
                   so_time=so_t, so_names=np.array(so_names), so_values=so_v, act_kind=np.array(kinds),
                   act_coord=np.array(rcoord), act_body=np.array(rbody), act_point=np.array(rpoint),
                   act_dir=np.array(rdir), act_opt=np.array(ropt), act_point_global=np.array(rpg),
                   act_vec_global=np.array(rvg))
        path = os.path.join(HERE, f'so_{tag_}.npz')
        np.savez_compressed(path, **out)
        print(tag_, env_id, 'IK rows', len(q), 'GRF rows', len(grf), 'SO frames', len(so_t), so_t[0], so_t[-1],
              'actuators', len(so_names), 'kinds', {k: kinds.count(k) for k in set(kinds)}, '->', path)


if __name__ == '__main__':
    main()
