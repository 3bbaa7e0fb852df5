"""Compile the committed ModelPacks (and synthesize the 2D reference motion)
from the reference's shipped data.  Runs in the dev container only (needs
/root/reference); the GPU box uses the committed outputs.

    python bioimitation-gym_amd/tools/build_packs.py [--ref /root/reference]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
sys.path.insert(0, PKG_ROOT)

from bioimitation import modelpack, refmotion, registry, transforms  # noqa: E402
from bioimitation.osim import load_osim  # noqa: E402

DATA = os.path.join(PKG_ROOT, 'bioimitation', 'data')
# env flags baked into a kernel (MUSCLE, HAS_TZ, REWARD_FEET, DONE_CROSS, PD); the others
# (RAW_ACTION, TARGET_OBS, GRF_OBS) are read at run time — csrc/bioim_step.hip: BIOIM_STRUCT_FLAGS
STRUCT_FLAGS = 0x8f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ref', default='/root/reference')
    ap.add_argument('--ids', nargs='*', default=list(registry.RECIPES))
    ap.add_argument('--resynth', action='store_true')
    a = ap.parse_args()
    ref_data = os.path.join(a.ref, 'bioimitation', 'imitation_envs', 'data')
    os.makedirs(os.path.join(DATA, 'packs'), exist_ok=True)
    built = []
    for env_id in a.ids:
        recipe = registry.RECIPES[env_id]
        model = registry.build_model(env_id, ref_data)
        ref_dir = os.path.join(DATA, recipe['reference'])
        if a.resynth or not os.path.exists(os.path.join(ref_dir, 'task_Kinematics_q.sto')):
            if recipe['reference'].startswith('2D'):
                base = transforms.construct_predictive_model(
                    load_osim(os.path.join(ref_data, '2D/scale/model_scaled.osim')))
                refmotion.synthesize_2d_walking(base, os.path.join(ref_data, '3D/inverse_kinematics/task_InverseKinematics.mot'),
                                                ref_dir)
            else:
                # the un-prosthetic model of the same subject drives the recipe (shared tables)
                base = registry.build_model(env_id, ref_data, tuple(t for t in recipe['transforms']
                                                                    if t != 'prosthetic'))
                refmotion.synthesize_reference(base, os.path.join(ref_data, recipe['ik']), ref_dir)
        ref = refmotion.load_reference_tables(ref_dir, model.coord_order)
        spec = registry.env_spec(env_id)
        pk = modelpack.compile_pack(model, spec, ref)
        out = os.path.join(DATA, 'packs', env_id + '.npz')
        names = dict(coords=list(model.coord_order), bodies=list(model.body_order),
                     muscles=[mu.name for mu in model.muscles] if pk.nmuscle else [],
                     cforces=[h.name for h in model.hc_forces], limits=[l.name for l in model.limits],
                     coord_joints=[model.coords[c].joint for c in model.coord_order],
                     coord_rotational=[c not in _translational(model) for c in model.coord_order],
                     coord_locked=[bool(model.coords[c].locked) for c in model.coord_order])
        np.savez_compressed(out, pack=np.frombuffer(modelpack.pack_bytes(pk), dtype=np.uint8),
                            names=np.array(json.dumps(names)))
        built.append((env_id, pk))
        print(f'{env_id}: ncoord={pk.ncoord} ndof={pk.ndof} ncbody={pk.ncbody} muscles={pk.nmuscle} '
              f'spheres={pk.nsphere} limits={pk.nlimit} act={pk.nact} obs={pk.obs_dim} rows={pk.nrows} -> {out}')
    write_topologies(built)




# --------------------------------------------------------------------------
# compile-time topology descriptors for the HIP kernels (csrc/topologies.h)
def _carr(name, vals, ctype='int'):
    vals = list(vals) or [0]
    return f'    static constexpr {ctype} {name}[{len(vals)}] = {{{", ".join(str(int(v)) for v in vals)}}};\n'


def _translational(model):
    """Coordinates that drive a CustomJoint translation axis and no rotation
    axis (OpenSim 4 derives the motion type from the spatial transform; 3.x
    files also state it)."""
    out = {c for c, co in model.coords.items() if co.motion == 'translational'}
    rot = set()
    for j in model.joints:
        for ax in (j.axes or []):
            if ax.coord and ax.name.startswith('rotation'):
                rot.add(ax.coord)
            elif ax.coord and ax.name.startswith('translation'):
                out.add(ax.coord)
    return out - rot


def unique_curves(pk):
    """Distinct muscle curves (byte-equal bioim_curve_t), first-appearance
    order over (fal, fv, fpe, fse) of each muscle — the order the device
    model image stores them in (bioim_step.hip: build_smodel)."""
    seen = []
    for i in range(pk.nmuscle):
        m = pk.muscle[i]
        for name in ('fal', 'fv', 'fpe', 'fse'):
            b = bytes(getattr(m, name))
            if b not in seen:
                seen.append(b)
    return seen


def is_planar(pk):
    """Every motion stays in the x-y plane: joint and body frames rotate
    about z only, rotation axes that move are about z, translation axes that
    move have no z component, gravity has none.  The kernels then carry the
    structural zeros of planar frames (R13 R23 R31 R32 = 0, R33 = 1; angular
    velocity/acceleration along z only; linear ones in the plane) as
    constants (bioim_step.hip: Planar)."""
    def zrot(R):
        return R[2] == 0 and R[5] == 0 and R[6] == 0 and R[7] == 0 and R[8] == 1
    for c in range(pk.ncbody):
        b = pk.cbody[c]
        if not (zrot(list(b.R_pf)) and zrot(list(b.R_mb))):
            return False
        for a in range(6):
            fi = b.fn[a]
            if fi < 0:
                continue
            ax = list(b.axis[a])
            if a < 3 and not (ax[0] == 0 and ax[1] == 0):
                return False
            if a >= 3 and pk.fn[fi].type != 0 and ax[2] != 0:
                return False
    return pk.gravity[2] == 0


def emit_topology(struct, pk, lanes, lanes_expr=None):  # noqa: C901
    nb, nd, nc, nm = pk.ncbody, pk.ndof, pk.ncoord, pk.nmuscle
    parent = [pk.cbody[c].parent for c in range(nb)]
    anc = []
    for c in range(nb):
        m, p = 1 << c, parent[c]
        while p >= 0:
            m |= 1 << p
            p = parent[p]
        anc.append(m)
    dof_cb = [0] * max(nd, 1)
    dof_coord = [0] * max(nd, 1)
    for c in range(nc):
        d = pk.coord[c].dof
        if d >= 0:
            dof_cb[d] = pk.coord[c].cbody
            dof_coord[d] = c
    dofmask = []
    for c in range(nb):
        m = 0
        for d in range(nd):
            if anc[c] >> dof_cb[d] & 1:
                m |= 1 << d
        dofmask.append(m)
    axis_coord, axis_kind = [], []
    for c in range(nb):
        for a in range(6):
            fi = pk.cbody[c].fn[a]
            axis_kind.append(-1 if fi < 0 else pk.fn[fi].type)
            axis_coord.append(-1 if fi < 0 else pk.fn[fi].coord)
    s = f'struct {struct} {{\n'
    s += f'    static constexpr int NB = {nb}, ND = {nd}, NC = {nc}, NM = {nm}, NA = {pk.nact}, NS = {pk.nsphere},' \
         f' NF = {pk.ncforce}, NL = {pk.nlimit}, NOS = {pk.nosbody}, G = {lanes_expr or lanes};\n'
    s += f'    static constexpr int NOBP = {pk.n_obs_bpos}, NOBV = {pk.n_obs_bvel};\n'
    s += f'    static constexpr int NPT = {pk.npathpt}, NFN = {pk.nfn}, NKNOT = {pk.nknots},' \
         f' NCURVE = {len(unique_curves(pk))},' \
         f' NKMAX = {max([pk.fn[i].nknots for i in range(pk.nfn)] + [2])};\n'
    maxpt, cond, move = 0, 0, 0
    for i in range(pk.nmuscle):
        m = pk.muscle[i]
        maxpt = max(maxpt, m.npt)
        for j in range(m.npt):
            t = pk.pathpt[m.pt_off + j].type
            cond |= (1 << j) if t == 1 else 0
            move |= (1 << j) if t == 2 else 0
    root = (1 << nd) - 1
    for c in range(nb):
        root &= dofmask[c]
    maxspan, arms = 1, [0] * max(nd, 1)
    for i in range(pk.nmuscle):
        m = pk.muscle[i]
        u = 0
        for j in range(m.npt):
            u |= dofmask[pk.pathpt[m.pt_off + j].cbody]
        maxspan = max(maxspan, bin(u & ~root).count('1'))
        for d in range(nd):
            arms[d] += (u & ~root) >> d & 1
    if pk.nmuscle == 0:
        for a in range(pk.nact):
            if pk.coordact[a].dof >= 0:
                arms[pk.coordact[a].dof] += 1
    s += f'    static constexpr int MAXPT = {maxpt}; /* path points per muscle (max) */\n'
    s += f'    static constexpr int MAXSPAN = {maxspan}; /* non-root dofs a muscle path moves (max) */\n'
    s += f'    static constexpr int MAXARM = {max(arms + [1])}; /* muscles (actuators) acting on one dof (max) */\n'
    # muscle slot -> muscle: when muscles take two passes over the lanes (NM > G), the second,
    # partly idle pass gets the cheapest paths (fewest points, no moving/conditional points)
    def cost(i):
        m = pk.muscle[i]
        t = [pk.pathpt[m.pt_off + j].type for j in range(m.npt)]
        return m.npt + 3 * t.count(2) + t.count(1)
    if nm > lanes:
        order = sorted(range(nm), key=lambda i: (-cost(i), i))
        mperm = sorted(order[:lanes]) + sorted(order[lanes:], key=lambda i: (cost(i), i))
    else:
        mperm = list(range(nm))
    s += _carr('mperm', mperm or [0])
    nmf = sum(1 for j in range(pk.npathpt) if pk.pathpt[j].type == 2 for a in range(3) if pk.pathpt[j].fn[a] >= 0)
    s += f'    static constexpr int NMF = {nmf}; /* moving-point location functions (one lane each, per dynamics call) */\n'
    s += f'    static constexpr unsigned PT_COND = {cond}u, PT_MOVING = {move}u; /* point indices that can be conditional / moving */\n'
    s += f'    static constexpr int TX = {pk.coord_tx}, TY = {pk.coord_ty}, TZ = {pk.coord_tz};\n'
    s += f'    static constexpr int TORSO = {pk.torso_body}, CALCN_R = {pk.calcn_r_body}, CALCN_L = {pk.calcn_l_body};\n'
    s += f'    static constexpr unsigned FLAGS = {pk.env_flags & STRUCT_FLAGS}u; /* structural env flags */\n'
    s += f'    static constexpr bool PLANAR = {"true" if is_planar(pk) else "false"}; /* motion in the x-y plane (is_planar) */\n'
    s += _carr('parent', parent) + _carr('anc', anc, 'unsigned') + _carr('dofmask', dofmask, 'unsigned')
    s += _carr('coord_dof', [pk.coord[c].dof for c in range(nc)])
    s += _carr('dof_cb', dof_cb) + _carr('dof_coord', dof_coord)
    s += _carr('axis_kind', axis_kind) + _carr('axis_coord', axis_coord)
    s += _carr('sphere_cb', [pk.sphere[i].cbody for i in range(pk.nsphere)])
    s += _carr('sphere_force', [pk.sphere[i].force for i in range(pk.nsphere)])
    s += _carr('os_cb', [pk.osbody[i].cbody for i in range(pk.nosbody)])
    s += _carr('limit_dof', [pk.limit[i].dof for i in range(pk.nlimit)])
    s += _carr('limit_coord', [pk.limit[i].coord for i in range(pk.nlimit)])
    s += _carr('act_dof', [pk.coordact[i].dof for i in range(pk.ncoordact)] if pk.ncoordact else [-1])
    s += _carr('pd_coord', [pk.pd_coord[i] for i in range(pk.nact)])
    s += _carr('pd_vcoord', [pk.pd_vcoord[i] for i in range(pk.nact)])
    s += _carr('obs_bpos', [pk.obs_bpos[i] for i in range(pk.n_obs_bpos)])
    s += _carr('obs_bvel', [pk.obs_bvel[i] for i in range(pk.n_obs_bvel)])
    s += _carr('rw_body', [pk.rw_body[i] for i in range(9)])
    s += '};\n'
    return s


def topology_signature(pk):
    """Everything the compiled kernels bake in; bioim_create() recomputes it
    from the pack and refuses a pack whose signature has no kernel."""
    import hashlib
    return hashlib.sha1(emit_topology('T', pk, 0).encode()).hexdigest()[:16]


def write_topologies(packs):
    out = ['/* GENERATED by tools/build_packs.py — compile-time topology of each env family. */',
           '#pragma once', '',
           '/* lanes per env of the spatial muscle topologies (16; 32 in the diagnostic G32 build) */',
           '#ifndef BIOIM_G_SPATIAL_MUSCLE', '#define BIOIM_G_SPATIAL_MUSCLE 16', '#endif', '']
    names, seen = [], {}
    for env_id, pk in packs:
        # env IDs that differ only in env constants (e.g. Walking3D / Running3D) share one kernel
        sig = topology_signature(pk)
        if sig in seen:
            out.append(f'/* {env_id}: same topology as {seen[sig]} */')
            continue
        struct = 'Topo_' + env_id.replace('-', '_')
        seen[sig] = struct
        # 16 lanes per env (4 envs per wave): one lane per body, dof and reported body; muscles,
        # actions and coordinates beyond 16 take a second pass on the same lanes
        lanes = 16 if pk.ncbody < 16 and pk.ndof <= 16 and pk.nosbody < 16 else 32
        expr = None
        if lanes == 16 and not is_planar(pk) and pk.nmuscle > 16:
            # spatial muscle models (22 / 19 muscles: two muscle passes at 16 lanes); a diagnostic
            # build sets BIOIM_G_SPATIAL_MUSCLE=32 (one muscle per lane, 512-thread workgroups)
            expr = 'BIOIM_G_SPATIAL_MUSCLE'
        out.append(emit_topology(struct, pk, lanes, expr))
        names.append((env_id, struct))
    out.append('#define BIOIM_FOR_EACH_TOPOLOGY(X) \\')
    out.append(' \\\n'.join(f'    X({s}, "{e}")' for e, s in names))
    out.append('')
    # one topology by index: the per-topology objects of the library build (__graft_entry__.py)
    out.append(f'#define BIOIM_NTOPOLOGIES {len(names)}')
    out.append('#define BIOIM_TOPOLOGY_AT(k, X) BIOIM_TOPOLOGY_AT_I(k, X)')
    out.append('#define BIOIM_TOPOLOGY_AT_I(k, X) BIOIM_TOPOLOGY_AT_##k(X)')
    for k, (e, s_) in enumerate(names):
        out.append(f'#define BIOIM_TOPOLOGY_AT_{k}(X) X({s_}, "{e}")')
    out.append('')
    path = os.path.join(PKG_ROOT, 'csrc', 'topologies.h')
    with open(path, 'w') as fh:
        fh.write('\n'.join(out))
    print('wrote', path)


if __name__ == '__main__':
    main()
