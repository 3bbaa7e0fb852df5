"""Minimal OpenSim ``.osim`` reader for the models bioimitation-gym ships.

Reads the subset of the OpenSim 3.0 (``Version="30000"``, joints nested in
bodies — ``data/2D/scale/model_scaled.osim``) and 4.0 (``Version="40000"``,
``JointSet`` + ``PhysicalOffsetFrame`` sockets — ``data/3D/scale/model_scaled.osim``,
``data/02905/02905_PRE/scale/model_predictive.osim``) formats that the
reference's envs load through ``opensim.Model(model_path)``
(``bioimitation/imitation_envs/utils/opensim_wrapper.py:9``).

The result is a plain-Python :class:`OsimModel` description; it is compiled into
a flat ModelPack by :mod:`bioimitation.modelpack`.  Nothing here simulates.
"""
from __future__ import annotations

import math
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np


# ---------------------------------------------------------------- functions
@dataclass
class Function:
    """OpenSim Function subset: Constant, LinearFunction, SimmSpline,
    NaturalCubicSpline (treated as SimmSpline), MultiplierFunction(SimmSpline)."""
    kind: str                     # 'const' | 'linear' | 'spline'
    a: float = 0.0                # linear slope | spline scale
    b: float = 0.0                # linear offset | constant value
    x: Optional[np.ndarray] = None
    y: Optional[np.ndarray] = None
    coord: Optional[str] = None   # independent coordinate name

    def value(self, q: float) -> float:
        if self.kind == 'const':
            return self.b
        if self.kind == 'linear':
            return self.a * q + self.b
        from .splines import simm_spline_coeffs, simm_spline_eval
        b, c, d = simm_spline_coeffs(self.x, self.y)
        return self.a * simm_spline_eval(self.x, self.y, b, c, d, q, 0)


def _floats(text) -> np.ndarray:
    return np.array([float(t) for t in (text or '').split()], dtype=np.float64)


_FUNCTION_TAGS = ('Constant', 'LinearFunction', 'SimmSpline', 'NaturalCubicSpline', 'MultiplierFunction',
                  'GCVSpline', 'PiecewiseLinearFunction', 'PolynomialFunction', 'PiecewiseConstantFunction')


def _parse_function(elem) -> Function:
    """``elem`` is the element holding one function child (e.g. <function>)."""
    if elem is None:
        return Function('const', b=0.0)
    kids = [k for k in elem if isinstance(k.tag, str) and k.tag in _FUNCTION_TAGS]
    if not kids:
        return Function('const', b=0.0)
    f = kids[0]
    tag = f.tag
    if tag == 'Constant':
        return Function('const', b=float(f.findtext('value')))
    if tag == 'LinearFunction':
        c = _floats(f.findtext('coefficients'))
        return Function('linear', a=float(c[0]), b=float(c[1]))
    if tag in ('SimmSpline', 'NaturalCubicSpline'):
        return Function('spline', a=1.0, x=_floats(f.findtext('x')), y=_floats(f.findtext('y')))
    if tag == 'MultiplierFunction':
        scale = float(f.findtext('scale') or 1.0)
        inner = _parse_function(f.find('function'))
        if inner.kind == 'spline':
            inner.a *= scale
        elif inner.kind == 'linear':
            inner.a *= scale
            inner.b *= scale
        else:
            inner.b *= scale
        return inner
    raise NotImplementedError(f'unsupported OpenSim function {tag}')


# ---------------------------------------------------------------- model parts
@dataclass
class Body:
    name: str
    mass: float
    com: np.ndarray
    inertia: np.ndarray           # xx yy zz xy xz yz


@dataclass
class Coordinate:
    name: str
    motion: str                   # 'rotational' | 'translational'
    default_value: float
    range: tuple
    locked: bool
    joint: str = ''


@dataclass
class TransformAxis:
    name: str                     # rotation1..3 / translation1..3
    axis: np.ndarray
    func: Function
    coord: Optional[str]


@dataclass
class Joint:
    name: str
    kind: str                     # CustomJoint | PinJoint | WeldJoint
    parent: str                   # parent body name ('ground')
    child: str
    R_pf: np.ndarray              # F frame in parent body frame
    p_pf: np.ndarray
    R_cm: np.ndarray              # M frame in child body frame
    p_cm: np.ndarray
    coords: List[str]
    axes: List[TransformAxis] = field(default_factory=list)


@dataclass
class PathPoint:
    name: str
    body: str
    kind: str                     # 'fixed' | 'cond' | 'moving'
    loc: np.ndarray
    cond_coord: Optional[str] = None
    cond_range: tuple = (0.0, 0.0)
    move: Optional[List[Optional[Function]]] = None   # x, y, z functions


@dataclass
class Muscle:
    name: str
    kind: str
    fiso: float
    lopt: float
    lts: float
    alpha_opt: float
    vmax: float
    tau_act: float
    tau_deact: float
    path: List[PathPoint]
    props: Dict[str, str] = field(default_factory=dict)
    curves: Dict[str, Dict[str, float]] = field(default_factory=dict)


@dataclass
class ContactSphere:
    name: str
    body: str
    loc: np.ndarray
    radius: float


@dataclass
class ContactHalfSpace:
    name: str
    body: str
    loc: np.ndarray
    orientation: np.ndarray


@dataclass
class HuntCrossley:
    name: str
    geometries: List[str]
    stiffness: float
    dissipation: float
    static_friction: float
    dynamic_friction: float
    viscous_friction: float
    transition_velocity: float


@dataclass
class CoordinateLimit:
    name: str
    coord: str
    upper_stiffness: float
    upper_limit: float
    lower_stiffness: float
    lower_limit: float
    damping: float
    transition: float


@dataclass
class CoordinateActuator:
    name: str
    coord: str
    optimal_force: float
    min_control: float
    max_control: float


@dataclass
class Marker:
    """MarkerSet station: a point fixed in a body frame (used by OpenSim's
    InverseKinematicsTool; tests/test_ik_pin.py pins our kinematics with it)."""
    name: str
    body: str
    location: np.ndarray


@dataclass
class OsimModel:
    name: str
    gravity: np.ndarray
    bodies: Dict[str, Body]
    body_order: List[str]                     # BodySet order (ground excluded)
    joints: List[Joint]
    coords: Dict[str, Coordinate]
    coord_order: List[str]                    # CoordinateSet order
    muscles: List[Muscle] = field(default_factory=list)
    spheres: List[ContactSphere] = field(default_factory=list)
    halfspaces: List[ContactHalfSpace] = field(default_factory=list)
    hc_forces: List[HuntCrossley] = field(default_factory=list)
    limits: List[CoordinateLimit] = field(default_factory=list)
    coord_actuators: List[CoordinateActuator] = field(default_factory=list)
    markers: List[Marker] = field(default_factory=list)

    def total_mass(self) -> float:
        return float(sum(b.mass for b in self.bodies.values()))


# ---------------------------------------------------------------- helpers
def rot_body_xyz(angles) -> np.ndarray:
    """OpenSim body-fixed XYZ Euler angles -> rotation matrix (Rx Ry Rz)."""
    a, b, c = angles
    ca, sa, cb, sb, cc, sc = math.cos(a), math.sin(a), math.cos(b), math.sin(b), math.cos(c), math.sin(c)
    rx = np.array([[1, 0, 0], [0, ca, -sa], [0, sa, ca]])
    ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
    rz = np.array([[cc, -sc, 0], [sc, cc, 0], [0, 0, 1]])
    return rx @ ry @ rz


def _vec3(text, default=(0.0, 0.0, 0.0)) -> np.ndarray:
    if text is None or not text.strip():
        return np.array(default, dtype=np.float64)
    v = _floats(text)
    return v[:3]


def _text(e, tag, default=None):
    t = e.findtext(tag)
    return default if t is None else t.strip()


def _read_xml(path: str) -> ET.Element:
    with open(path, 'r', encoding='utf-8', errors='replace') as fh:
        text = fh.read()
    # OpenSim 4 serializes "HuntCrossleyForce::ContactParametersSet" and
    # "HuntCrossleyForce::ContactParameters" element names (not well-formed
    # for ElementTree: ':' is a namespace separator).
    text = text.replace('HuntCrossleyForce::', 'HuntCrossleyForce__')
    return ET.fromstring(text)


# ---------------------------------------------------------------- parsing
def _parse_coordinates(joint_elem, joint_name, coords, order):
    names = []
    for c in joint_elem.iter('Coordinate'):
        name = c.get('name')
        rng = _floats(c.findtext('range'))
        motion = _text(c, 'motion_type', 'rotational')
        coords[name] = Coordinate(
            name=name, motion=motion,
            default_value=float(_text(c, 'default_value', '0')),
            range=(float(rng[0]), float(rng[1])) if rng.size >= 2 else (-math.inf, math.inf),
            locked=_text(c, 'locked', 'false').lower() == 'true',
            joint=joint_name)
        order.append(name)
        names.append(name)
    return names


def _parse_spatial_transform(st, coord_names):
    axes = []
    for ta in st.findall('TransformAxis'):
        cname = (ta.findtext('coordinates') or '').strip() or None
        fe = ta.find('function')      # 3.x: <function><LinearFunction>…; 4.x: <LinearFunction name="function">
        if fe is None:
            fe = ta
        axes.append(TransformAxis(name=ta.get('name'), axis=_vec3(ta.findtext('axis')),
                                  func=_parse_function(fe), coord=cname))
    return axes


def _default_axes(kind, coord_names):
    """PinJoint: rotation about the joint frame Z; WeldJoint: no motion."""
    ident = Function('linear', a=1.0, b=0.0)
    zero = Function('const', b=0.0)
    ax = [np.array([0., 0., 1.]), np.array([1., 0., 0.]), np.array([0., 1., 0.]),
          np.array([1., 0., 0.]), np.array([0., 1., 0.]), np.array([0., 0., 1.])]
    names = ['rotation1', 'rotation2', 'rotation3', 'translation1', 'translation2', 'translation3']
    out = []
    for i in range(6):
        if kind == 'PinJoint' and i == 0:
            out.append(TransformAxis(names[i], ax[i], ident, coord_names[0]))
        else:
            out.append(TransformAxis(names[i], ax[i], zero, None))
    return out


def _parse_path(gp) -> List[PathPoint]:
    pts = []
    pps = gp.find('PathPointSet/objects')
    if pps is None:
        return pts
    for pp in pps:
        name = pp.get('name')
        body = (pp.findtext('body') or pp.findtext('socket_parent_frame') or '').strip()
        body = body.split('/')[-1]
        loc = _vec3(pp.findtext('location'))
        if pp.tag == 'PathPoint':
            pts.append(PathPoint(name, body, 'fixed', loc))
        elif pp.tag == 'ConditionalPathPoint':
            rng = _floats(pp.findtext('range'))
            coord = (pp.findtext('coordinate') or pp.findtext('socket_coordinate') or '').strip().split('/')[-1]
            pts.append(PathPoint(name, body, 'cond', loc, cond_coord=coord,
                                 cond_range=(float(rng[0]), float(rng[1]))))
        elif pp.tag == 'MovingPathPoint':
            move = []
            for ax in 'xyz':
                fe = pp.find(f'{ax}_location')
                if fe is None or not len(fe):
                    move.append(None)
                    continue
                f = _parse_function(fe)
                cn = (pp.findtext(f'{ax}_coordinate') or pp.findtext(f'socket_{ax}_coordinate') or '').strip()
                f.coord = cn.split('/')[-1] if cn else None
                move.append(f)
            pts.append(PathPoint(name, body, 'moving', loc, move=move))
        else:
            raise NotImplementedError(f'path point kind {pp.tag}')
    return pts


_CURVE_TAGS = ('ActiveForceLengthCurve', 'ForceVelocityCurve', 'FiberForceLengthCurve',
               'TendonForceLengthCurve', 'ForceVelocityInverseCurve')


def _parse_muscle(m) -> Muscle:
    props = {ch.tag: (ch.text or '').strip() for ch in m if isinstance(ch.tag, str) and len(ch) == 0}
    curves = {}
    for tag in _CURVE_TAGS:
        ce = m.find(tag)
        if ce is not None:
            curves[tag] = {ch.tag: float(ch.text) for ch in ce
                           if isinstance(ch.tag, str) and len(ch) == 0 and ch.text and ch.text.strip()}
    if m.tag != 'Millard2012EquilibriumMuscle':
        raise NotImplementedError(f'muscle model {m.tag}')
    return Muscle(
        name=m.get('name'), kind=m.tag,
        fiso=float(props['max_isometric_force']),
        lopt=float(props['optimal_fiber_length']),
        lts=float(props['tendon_slack_length']),
        alpha_opt=float(props.get('pennation_angle_at_optimal', '0')),
        vmax=float(props.get('max_contraction_velocity', '10')),
        tau_act=float(props.get('activation_time_constant', '0.01')),
        tau_deact=float(props.get('deactivation_time_constant', '0.04')),
        path=_parse_path(m.find('GeometryPath')), props=props, curves=curves)


def _parse_forces(model_elem, model: OsimModel):
    fs = model_elem.find('ForceSet/objects')
    if fs is None:
        return
    for f in fs:
        if not isinstance(f.tag, str):
            continue
        if f.tag == 'Millard2012EquilibriumMuscle':
            if _text(f, 'isDisabled', 'false').lower() == 'true' or _text(f, 'appliesForce', 'true').lower() == 'false':
                continue
            model.muscles.append(_parse_muscle(f))
        elif f.tag == 'HuntCrossleyForce':
            cp = f.find('HuntCrossleyForce__ContactParametersSet/objects/HuntCrossleyForce__ContactParameters')
            model.hc_forces.append(HuntCrossley(
                name=f.get('name'), geometries=(cp.findtext('geometry') or '').split(),
                stiffness=float(cp.findtext('stiffness')), dissipation=float(cp.findtext('dissipation')),
                static_friction=float(cp.findtext('static_friction')),
                dynamic_friction=float(cp.findtext('dynamic_friction')),
                viscous_friction=float(cp.findtext('viscous_friction')),
                transition_velocity=float(f.findtext('transition_velocity') or 0.1)))
        elif f.tag == 'CoordinateLimitForce':
            model.limits.append(CoordinateLimit(
                name=f.get('name'), coord=_text(f, 'coordinate'),
                upper_stiffness=float(_text(f, 'upper_stiffness')), upper_limit=float(_text(f, 'upper_limit')),
                lower_stiffness=float(_text(f, 'lower_stiffness')), lower_limit=float(_text(f, 'lower_limit')),
                damping=float(_text(f, 'damping')), transition=float(_text(f, 'transition'))))
        elif f.tag == 'CoordinateActuator':
            model.coord_actuators.append(CoordinateActuator(
                name=f.get('name'), coord=_text(f, 'coordinate'),
                optimal_force=float(_text(f, 'optimal_force', '1')),
                min_control=float(_text(f, 'min_control', '-inf')),
                max_control=float(_text(f, 'max_control', 'inf'))))
        # other forces (e.g. disabled reserve actuators) are not part of the step


def _parse_contact_geometry(model_elem, model: OsimModel):
    cg = model_elem.find('ContactGeometrySet/objects')
    if cg is None:
        return
    for g in cg:
        body = (g.findtext('body_name') or g.findtext('socket_frame') or '').strip().split('/')[-1]
        loc = _vec3(g.findtext('location'))
        ori = _vec3(g.findtext('orientation'))
        if g.tag == 'ContactSphere':
            model.spheres.append(ContactSphere(g.get('name'), body, loc, float(g.findtext('radius'))))
        elif g.tag == 'ContactHalfSpace':
            model.halfspaces.append(ContactHalfSpace(g.get('name'), body, loc, ori))


def _parse_v3(model_elem) -> OsimModel:
    bodies, order, joints, coords, corder = {}, [], [], {}, []
    for b in model_elem.find('BodySet/objects'):
        name = b.get('name')
        if name == 'ground':
            continue
        bodies[name] = Body(name, float(b.findtext('mass')), _vec3(b.findtext('mass_center')),
                            np.array([float(b.findtext(k) or 0) for k in
                                      ('inertia_xx', 'inertia_yy', 'inertia_zz', 'inertia_xy', 'inertia_xz', 'inertia_yz')]))
        order.append(name)
        jw = b.find('Joint')
        for j in jw:
            cnames = _parse_coordinates(j, j.get('name'), coords, corder)
            st = j.find('SpatialTransform')
            axes = _parse_spatial_transform(st, cnames) if st is not None else _default_axes(j.tag, cnames)
            joints.append(Joint(
                name=j.get('name'), kind=j.tag, parent=j.findtext('parent_body').strip(), child=name,
                R_pf=rot_body_xyz(_vec3(j.findtext('orientation_in_parent'))),
                p_pf=_vec3(j.findtext('location_in_parent')),
                R_cm=rot_body_xyz(_vec3(j.findtext('orientation'))),
                p_cm=_vec3(j.findtext('location')), coords=cnames, axes=axes))
    return OsimModel(model_elem.get('name'), _vec3(model_elem.findtext('gravity')), bodies, order,
                     joints, coords, corder)


def _parse_v4(model_elem) -> OsimModel:
    bodies, order, joints, coords, corder = {}, [], [], {}, []
    for b in model_elem.find('BodySet/objects'):
        name = b.get('name')
        inertia = _floats(b.findtext('inertia'))
        bodies[name] = Body(name, float(b.findtext('mass')), _vec3(b.findtext('mass_center')), inertia[:6])
        order.append(name)
    for j in model_elem.find('JointSet/objects'):
        frames = {}
        fr = j.find('frames')
        if fr is not None:
            for pof in fr.findall('PhysicalOffsetFrame'):
                frames[pof.get('name')] = (
                    (pof.findtext('socket_parent') or '').strip().split('/')[-1],
                    rot_body_xyz(_vec3(pof.findtext('orientation'))), _vec3(pof.findtext('translation')))

        def resolve(sock):
            nm = sock.strip().split('/')[-1]
            if nm in frames:
                body, R, p = frames[nm]
                return body, R, p
            return nm, np.eye(3), np.zeros(3)
        pb, R_pf, p_pf = resolve(j.findtext('socket_parent_frame'))
        cb, R_cm, p_cm = resolve(j.findtext('socket_child_frame'))
        cnames = _parse_coordinates(j, j.get('name'), coords, corder)
        st = j.find('SpatialTransform')
        axes = _parse_spatial_transform(st, cnames) if st is not None else _default_axes(j.tag, cnames)
        joints.append(Joint(j.get('name'), j.tag, pb, cb, R_pf, p_pf, R_cm, p_cm, cnames, axes))
    return OsimModel(model_elem.get('name'), _vec3(model_elem.findtext('gravity')), bodies, order,
                     joints, coords, corder)


def _parse_markers(model_elem, model: OsimModel):
    """MarkerSet (4.x: socket_parent_frame '/bodyset/<body>'; 3.x: <body>)."""
    ms = model_elem.find('MarkerSet/objects')
    if ms is None:
        return
    for m in ms.findall('Marker'):
        frame = m.findtext('socket_parent_frame') or m.findtext('body') or ''
        model.markers.append(Marker(m.get('name'), frame.strip().split('/')[-1], _vec3(m.findtext('location'))))


def load_osim(path: str) -> OsimModel:
    root = _read_xml(path)
    version = int(root.get('Version', '30000'))
    me = root.find('Model')
    model = _parse_v3(me) if version < 40000 else _parse_v4(me)
    _parse_forces(me, model)
    _parse_contact_geometry(me, model)
    _parse_markers(me, model)
    # PinJoint/WeldJoint coordinate lists follow the SpatialTransform defaults
    for j in model.joints:
        for c in j.coords:
            model.coords[c].joint = j.name
    return model
