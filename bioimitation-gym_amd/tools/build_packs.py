"""Compile the committed ModelPacks (and synthesize the 2D reference motion)
from the reference's shipped data.  Runs in the dev container only (needs
/root/reference); the GPU box uses the committed outputs.

    python bioimitation-gym_amd/tools/build_packs.py [--ref /root/reference]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
sys.path.insert(0, PKG_ROOT)

from bioimitation import modelpack, refmotion, registry, transforms  # noqa: E402
from bioimitation.osim import load_osim  # noqa: E402

DATA = os.path.join(PKG_ROOT, 'bioimitation', 'data')


def load_model(ref_data, recipe):
    m = load_osim(os.path.join(ref_data, recipe['model']))
    for t in recipe['transforms']:
        if t == 'predictive':
            m = transforms.construct_predictive_model(m)
        elif t == 'torque':
            m = transforms.convert_model_to_torque_actuated(m, 200.0)
        elif t == 'prosthetic':
            m = transforms.convert_model_to_prosthetic(m)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/root/reference')
    ap.add_argument('--ids', nargs='*', default=list(registry.RECIPES))
    ap.add_argument('--resynth', action='store_true')
    a = ap.parse_args()
    ref_data = os.path.join(a.ref, 'bioimitation', 'imitation_envs', 'data')
    os.makedirs(os.path.join(DATA, 'packs'), exist_ok=True)
    for env_id in a.ids:
        recipe = registry.RECIPES[env_id]
        model = load_model(ref_data, recipe)
        ref_dir = os.path.join(DATA, recipe['reference'])
        if recipe['reference'].startswith('2D') and (a.resynth or not os.path.exists(
                os.path.join(ref_dir, 'task_Kinematics_q.sto'))):
            base = transforms.construct_predictive_model(load_osim(os.path.join(ref_data, '2D/scale/model_scaled.osim')))
            refmotion.synthesize_2d_walking(base, os.path.join(ref_data, '3D/inverse_kinematics/task_InverseKinematics.mot'),
                                            ref_dir)
        ref = refmotion.load_reference_tables(ref_dir, model.coord_order)
        spec = registry.env_spec(env_id)
        pk = modelpack.compile_pack(model, spec, ref)
        out = os.path.join(DATA, 'packs', env_id + '.npz')
        np.savez_compressed(out, pack=np.frombuffer(modelpack.pack_bytes(pk), dtype=np.uint8))
        print(f'{env_id}: ncoord={pk.ncoord} ndof={pk.ndof} ncbody={pk.ncbody} muscles={pk.nmuscle} '
              f'spheres={pk.nsphere} limits={pk.nlimit} act={pk.nact} obs={pk.obs_dim} rows={pk.nrows} -> {out}')


if __name__ == '__main__':
    main()
