"""Load-time model transforms, restated on the parsed model description.

Each function mirrors one reference routine that edits an ``opensim.Model``
before the env builds its ``OsimModel``; here they edit the
:class:`bioimitation.osim.OsimModel` description instead (no OpenSim).
"""
from __future__ import annotations

import copy
import math

import numpy as np

from .osim import (ContactHalfSpace, ContactSphere, CoordinateActuator,
                   CoordinateLimit, HuntCrossley, OsimModel)


def default_contact_sphere_parameters():
    """opensim_utils.py:14-53"""
    return {
        'heel_r': dict(body='calcn_r', location=[0.03, 0.02, 0], orientation=[0, 0, 0], radius=0.05),
        'toe1_r': dict(body='toes_r', location=[0.02, -0.005, -0.026], orientation=[0, 0, 0], radius=0.025),
        'toe2_r': dict(body='toes_r', location=[0.02, -0.005, 0.026], orientation=[0, 0, 0], radius=0.025),
        'heel_l': dict(body='calcn_l', location=[0.03, 0.02, 0], orientation=[0, 0, 0], radius=0.05),
        'toe1_l': dict(body='toes_l', location=[0.02, -0.005, -0.026], orientation=[0, 0, 0], radius=0.025),
        'toe2_l': dict(body='toes_l', location=[0.02, -0.005, 0.026], orientation=[0, 0, 0], radius=0.025),
    }


def default_contact_force_parameters():
    """opensim_utils.py:56-81"""
    common = dict(stiffness=2000000, dissipation=1.0, static_friction=0.8, dynamic_friction=0.8,
                  viscous_friction=0.6, transition_velocity=0.1)
    return {'foot_r': dict(geometries=['platform', 'heel_r', 'toe1_r', 'toe2_r'], **common),
            'foot_l': dict(geometries=['platform', 'heel_l', 'toe1_l', 'toe2_l'], **common)}


def default_coordinate_limit_force_parameters():
    """opensim_utils.py:84-141"""
    p = {}
    for side in ('r', 'l'):
        p[f'hip_flexion_limit_{side}'] = dict(coordinate=f'hip_flexion_{side}', upper_stiffness=20, upper_limit=120,
                                             lower_stiffness=20, lower_limit=-30, damping=0.25, transition=10)
    for side in ('r', 'l'):
        p[f'knee_limit_{side}'] = dict(coordinate=f'knee_angle_{side}', upper_stiffness=20, upper_limit=0,
                                      lower_stiffness=20, lower_limit=-140, damping=0.25, transition=10)
    for side in ('r', 'l'):
        p[f'ankle_limit_{side}'] = dict(coordinate=f'ankle_angle_{side}', upper_stiffness=20, upper_limit=20,
                                       lower_stiffness=20, lower_limit=-40, damping=0.25, transition=10)
    return p


def add_contact_model(model: OsimModel, spheres, forces):
    """opensim_utils.py:144-182 — ground half-space 'platform' (orientation
    (0,0,-pi/2): the plane y=0 with the solid below) plus spheres and one
    HuntCrossleyForce per foot."""
    model.halfspaces.append(ContactHalfSpace('platform', 'ground', np.zeros(3),
                                             np.array([0.0, 0.0, -math.pi / 2])))
    for name, v in spheres.items():
        model.spheres.append(ContactSphere(name, v['body'], np.array(v['location'], float), float(v['radius'])))
    for name, v in forces.items():
        model.hc_forces.append(HuntCrossley(name, list(v['geometries']), float(v['stiffness']),
                                            float(v['dissipation']), float(v['static_friction']),
                                            float(v['dynamic_friction']), float(v['viscous_friction']),
                                            float(v['transition_velocity'])))


def add_coordinate_limit_forces(model: OsimModel, params):
    """opensim_utils.py:185-201"""
    for name, v in params.items():
        model.limits.append(CoordinateLimit(name, v['coordinate'], float(v['upper_stiffness']),
                                            float(v['upper_limit']), float(v['lower_stiffness']),
                                            float(v['lower_limit']), float(v['damping']), float(v['transition'])))


def construct_predictive_model(model: OsimModel) -> OsimModel:
    """opensim_utils.py:204-222: contact + coordinate limits, pelvis_ty default 1.02."""
    m = copy.deepcopy(model)
    add_contact_model(m, default_contact_sphere_parameters(), default_contact_force_parameters())
    add_coordinate_limit_forces(m, default_coordinate_limit_force_parameters())
    m.coords['pelvis_ty'].default_value = 1.02
    m.name = 'model_predictive'
    return m


def convert_model_to_torque_actuated(model: OsimModel, max_actuation: float,
                                     remove_floating_base: bool = True) -> OsimModel:
    """opensim_utils.py:238-270: drop muscles, one CoordinateActuator
    (optimal force 1, controls +-max_actuation) per unlocked coordinate except
    pelvis_tx/ty/tz."""
    m = copy.deepcopy(model)
    m.muscles = []
    for cname in m.coord_order:
        c = m.coords[cname]
        if (remove_floating_base and cname in ('pelvis_tx', 'pelvis_ty', 'pelvis_tz')) or c.locked:
            continue
        m.coord_actuators.append(CoordinateActuator(cname + '_actuator', cname, 1.0,
                                                    -float(max_actuation), float(max_actuation)))
    m.name = 'model_predictive_no_muscles'
    return m


def convert_model_to_prosthetic(model: OsimModel) -> OsimModel:
    """muscle_locked_knee_imitation_env3D.py:104-126: remove gastroc_l,
    soleus_l, tib_ant_l; lock knee_angle_l and ankle_angle_l at 0."""
    m = copy.deepcopy(model)
    m.muscles = [mu for mu in m.muscles if mu.name not in ('gastroc_l', 'soleus_l', 'tib_ant_l')]
    for cname in ('knee_angle_l', 'ankle_angle_l'):
        m.coords[cname].default_value = 0.0
        m.coords[cname].locked = True
    m.name = 'model_predictive_prosthetic'
    return m
