"""Fixtures that pin the model compiler's kinematics to OpenSim's own output:
the reference ships OpenSim InverseKinematicsTool solutions together with
their inputs, so our forward kinematics can be checked against them
(tests/test_ik_pin.py).

Per trial (data/3D and data/02905/02905_PRE):
  - setup_ik.xml: the IKMarkerTasks (apply, weight) and the accuracy;
  - experimental_data/task.trc: measured marker positions (mm -> m), the task
    markers only, at the frames of the IK output;
  - inverse_kinematics/task_InverseKinematics.mot: the IK solution (deg -> rad
    for rotational coordinates);
  - the model's MarkerSet (body, location) and coordinate ranges / clamped
    flags, read from the model the IK ran on (setup_ik.xml model_file).

Runs in the dev container only (reads /root/reference); the committed npz
files are data (inputs and outputs of the reference's IK runs).

    python tests/golden/make_ik_fixtures.py
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DATA = '/root/reference/bioimitation/imitation_envs/data'
sys.path.insert(0, os.path.join(REPO, 'bioimitation-gym_amd'))

from bioimitation.osim import load_osim  # noqa: E402
from bioimitation.obslayout import load_names  # noqa: E402
from bioimitation.storage import read_sto  # noqa: E402

TRIALS = {'3D': ('3D', 'MuscleRunningImitation3D-v0'),
          '02905': ('02905/02905_PRE', 'MusclePalsyImitation3D-v0')}
STRIDE = 2          # every 2nd IK frame (0.02 s)


def read_trc(path):
    lines = open(path).read().split('\n')
    units = lines[2].split('\t')[4].strip()
    names = [x.strip() for x in lines[3].split('\t')[2:] if x.strip()]
    rows = []
    for ln in lines[5:]:
        if not ln.strip():
            continue
        f = ln.split('\t')
        vals = [float(x) if x.strip() else np.nan for x in f[2:2 + 3 * len(names)]]
        vals += [np.nan] * (3 * len(names) - len(vals))
        rows.append((float(f[1]), vals))
    t = np.array([r[0] for r in rows])
    X = np.array([r[1] for r in rows]).reshape(len(rows), len(names), 3)
    scale = {'mm': 1e-3, 'm': 1.0, 'cm': 1e-2}[units]
    return t, names, X * scale


def main():
    for tag, (sub, env_id) in TRIALS.items():
        d = os.path.join(DATA, sub)
        setup = open(os.path.join(d, 'inverse_kinematics', 'setup_ik.xml')).read()
        model_rel = re.search(r'<model_file>(.*?)</model_file>', setup).group(1).strip()
        marker_rel = re.search(r'<marker_file>(.*?)</marker_file>', setup).group(1).strip()
        accuracy = float(re.search(r'<accuracy>(.*?)</accuracy>', setup).group(1))
        tasks = re.findall(r'<IKMarkerTask name="(\w+)">.*?<apply>(\w+)</apply>.*?<weight>([\d.eE+-]+)</weight>',
                           setup, re.S)
        assert not re.search(r'<IKCoordinateTask', setup), 'coordinate tasks would change the objective'
        model_path = os.path.normpath(os.path.join(d, 'inverse_kinematics', model_rel))
        model = load_osim(model_path)
        mk = {m.name: m for m in model.markers}
        t_trc, names, X = read_trc(os.path.normpath(os.path.join(d, 'inverse_kinematics', marker_rel)))
        hdr, labels, data = read_sto(os.path.join(d, 'inverse_kinematics', 'task_InverseKinematics.mot'))
        coords = [c for c in labels if c != 'time']
        assert coords == list(model.coord_order), (coords, model.coord_order)
        qd = data[:, 1:].copy()
        in_deg = hdr.get('inDegrees', 'no').lower() == 'yes'
        # motion type from the CustomJoint transform axes (4.x files carry no motion_type)
        rot = np.array(load_names(env_id)['coord_rotational'], dtype=bool)
        assert list(load_names(env_id)['coords']) == coords
        if in_deg:
            qd[:, rot] = np.deg2rad(qd[:, rot])
        tm = data[:, 0]
        sel = np.arange(0, len(tm), STRIDE)
        use = [(n, float(w)) for n, a, w in tasks if a == 'true' and n in mk and n in names]
        frame = [int(np.argmin(np.abs(t_trc - tm[i]))) for i in sel]
        assert np.abs(t_trc[frame] - tm[sel]).max() < 1e-6
        Xsel = np.stack([X[frame, names.index(n)] for n, _ in use], axis=1)
        ranges = np.array([list(model.coords[c].range) for c in coords])
        xml = open(model_path).read()
        clamped = np.array([bool(re.search(rf'<Coordinate name="{c}">(?:(?!</Coordinate>).)*<clamped>true</clamped>',
                                           xml, re.S)) for c in coords])
        out = dict(env_id=env_id, model=os.path.relpath(model_path, DATA), accuracy=accuracy,
                   coords=np.array(coords), q=qd[sel], time=tm[sel], ranges=ranges, clamped=clamped,
                   markers=np.array([n for n, _ in use]), weights=np.array([w for _, w in use]),
                   bodies=np.array([mk[n].body for n, _ in use]),
                   locations=np.stack([mk[n].location for n, _ in use]), x_exp=Xsel)
        path = os.path.join(HERE, f'ik_{tag}.npz')
        np.savez_compressed(path, **out)
        print(tag, env_id, out['model'], 'frames', len(sel), 'markers', len(use), 'of', len(tasks), 'tasks;',
              'missing', [n for n, a, w in tasks if a == 'true' and (n not in mk or n not in names)],
              'nan', int(np.isnan(Xsel).any(axis=2).sum()), '->', path)


if __name__ == '__main__':
    main()
