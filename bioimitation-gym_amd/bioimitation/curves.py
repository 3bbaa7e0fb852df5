"""Millard2012EquilibriumMuscle curve construction (host side).

The reference's muscles are ``Millard2012EquilibriumMuscle``
(``data/2D/scale/model_scaled.osim`` ForceSet); their four characteristic
curves are OpenSim ``SmoothSegmentedFunction`` objects: C2-continuous chains of
quintic Bezier "corner" segments with linear extrapolation.  This module
restates the upstream construction [upstream: OpenSim 4.1
SmoothSegmentedFunctionFactory / SegmentedQuinticBezierToolkit, not vendored in
the reference, parity unpinned] and emits the control points that the
ModelPack stores (bioim_curve_t).

Curve defaults are the OpenSim 4.1 property defaults; the palsy model
(``data/02905/02905_PRE/scale/model_predictive.osim:1851-1870``) overrides
some of them per muscle, which ``muscle_curves()`` honours.
"""
from __future__ import annotations

import math

import numpy as np

DEFAULTS = {
    'ActiveForceLengthCurve': dict(min_norm_active_fiber_length=0.4441, transition_norm_fiber_length=0.73,
                                   max_norm_active_fiber_length=1.8123, shallow_ascending_slope=0.8616,
                                   minimum_value=0.1),
    'ForceVelocityCurve': dict(concentric_slope_at_vmax=0.0, concentric_slope_near_vmax=0.25,
                               isometric_slope=5.0, eccentric_slope_at_vmax=0.0,
                               eccentric_slope_near_vmax=0.15, max_eccentric_velocity_force_multiplier=1.4,
                               concentric_curviness=0.6, eccentric_curviness=0.9),
    'FiberForceLengthCurve': dict(strain_at_zero_force=0.0, strain_at_one_norm_force=0.7,
                                  stiffness_at_low_force=0.2, stiffness_at_one_norm_force=2.0 / 0.7,
                                  curviness=0.75),
    'TendonForceLengthCurve': dict(strain_at_one_norm_force=0.049, stiffness_at_one_norm_force=1.375 / 0.049,
                                   norm_force_at_toe_end=2.0 / 3.0, curviness=0.5),
}


def scale_curviness(c):
    return 0.1 + 0.8 * c


def corner_control_points(x0, y0, dydx0, x1, y1, dydx1, c):
    """SegmentedQuinticBezierToolkit::calcQuinticBezierCornerControlPoints."""
    root_eps = math.sqrt(np.finfo(float).eps)
    if abs(dydx0 - dydx1) > root_eps:
        xc = (y1 - y0 - x1 * dydx1 + x0 * dydx0) / (dydx0 - dydx1)
    else:
        xc = 0.5 * (x1 + x0)
    yc = (xc - x1) * dydx1 + y1
    px = np.empty(6)
    py = np.empty(6)
    px[0], py[0] = x0, y0
    px[5], py[5] = x1, y1
    px[1] = x0 + c * (xc - x0)
    py[1] = y0 + c * (yc - y0)
    px[2], py[2] = px[1], py[1]
    px[3] = x1 + c * (xc - x1)
    py[3] = y1 + c * (yc - y1)
    px[4], py[4] = px[3], py[3]
    return px, py


class Curve:
    """Chain of quintic Bezier segments with linear extrapolation."""

    def __init__(self, segs):
        self.x = np.array([s[0] for s in segs])
        self.y = np.array([s[1] for s in segs])
        self.x0, self.y0 = self.x[0, 0], self.y[0, 0]
        self.x1, self.y1 = self.x[-1, 5], self.y[-1, 5]
        self.dydx0 = (self.y[0, 1] - self.y[0, 0]) / (self.x[0, 1] - self.x[0, 0])
        self.dydx1 = (self.y[-1, 5] - self.y[-1, 4]) / (self.x[-1, 5] - self.x[-1, 4])

    @property
    def nseg(self):
        return self.x.shape[0]

    # --- Bezier helpers -------------------------------------------------
    @staticmethod
    def _bern(p, u):
        v = 1.0 - u
        return (p[0] * v ** 5 + 5 * p[1] * u * v ** 4 + 10 * p[2] * u ** 2 * v ** 3
                + 10 * p[3] * u ** 3 * v ** 2 + 5 * p[4] * u ** 4 * v + p[5] * u ** 5)

    @staticmethod
    def _dbern(p, u):
        v = 1.0 - u
        return 5 * ((p[1] - p[0]) * v ** 4 + 4 * (p[2] - p[1]) * u * v ** 3
                    + 6 * (p[3] - p[2]) * u ** 2 * v ** 2 + 4 * (p[4] - p[3]) * u ** 3 * v
                    + (p[5] - p[4]) * u ** 4)

    def value(self, x, deriv=0):
        if x <= self.x0:
            return self.y0 + self.dydx0 * (x - self.x0) if deriv == 0 else self.dydx0
        if x >= self.x1:
            return self.y1 + self.dydx1 * (x - self.x1) if deriv == 0 else self.dydx1
        k = 0
        while k < self.nseg - 1 and x > self.x[k, 5]:
            k += 1
        px, py = self.x[k], self.y[k]
        # bisection-safeguarded Newton on x(u) = x
        lo, hi, u = 0.0, 1.0, (x - px[0]) / (px[5] - px[0])
        for _ in range(100):
            f = self._bern(px, u) - x
            if abs(f) < 1e-14:
                break
            if f > 0:
                hi = u
            else:
                lo = u
            d = self._dbern(px, u)
            un = u - f / d if d != 0 else 0.5 * (lo + hi)
            u = un if lo < un < hi else 0.5 * (lo + hi)
        if deriv == 0:
            return self._bern(py, u)
        return self._dbern(py, u) / self._dbern(px, u)


def active_force_length(p):
    x0, x1, x2, x3 = (p['min_norm_active_fiber_length'], p['transition_norm_fiber_length'], 1.0,
                      p['max_norm_active_fiber_length'])
    ylow, dydx, curv = p['minimum_value'], p['shallow_ascending_slope'], 1.0
    c = scale_curviness(curv)
    x_delta = 0.05 * x2
    xs = x2 - x_delta
    y0, dydx0 = 0.0, 0.0
    y1 = 1.0 - dydx * (xs - x1)
    dydx01 = 1.25 * (y1 - y0) / (x1 - x0)
    x01 = x0 + 0.5 * (x1 - x0)
    y01 = y0 + 0.5 * (y1 - y0)
    x1s = x1 + 0.5 * (xs - x1)
    y1s = y1 + 0.5 * (1.0 - y1)
    dydx1s = dydx
    y2, dydx2 = 1.0, 0.0
    y3, dydx3 = 0.0, 0.0
    x23 = (x2 + x_delta) + 0.5 * (x3 - (x2 + x_delta))
    y23 = y2 + 0.5 * (y3 - y2)
    dydx23 = (y3 - y2) / ((x3 - x_delta) - (x2 + x_delta))
    segs = [corner_control_points(x0, ylow, dydx0, x01, y01, dydx01, c),
            corner_control_points(x01, y01, dydx01, x1s, y1s, dydx1s, c),
            corner_control_points(x1s, y1s, dydx1s, x2, y2, dydx2, c),
            corner_control_points(x2, y2, dydx2, x23, y23, dydx23, c),
            corner_control_points(x23, y23, dydx23, x3, ylow, dydx3, c)]
    return Curve(segs)


def force_velocity(p):
    dydx_c, dydx_near_c = p['concentric_slope_at_vmax'], p['concentric_slope_near_vmax']
    dydx_iso = p['isometric_slope']
    dydx_e, dydx_near_e = p['eccentric_slope_at_vmax'], p['eccentric_slope_near_vmax']
    fmax_e = p['max_eccentric_velocity_force_multiplier']
    cc = scale_curviness(p['concentric_curviness'])
    ce = scale_curviness(p['eccentric_curviness'])
    xc, yc = -1.0, 0.0
    xnc = -0.9
    ync = yc + 0.5 * dydx_near_c * (xnc - xc) + 0.5 * dydx_c * (xnc - xc)
    xiso, yiso = 0.0, 1.0
    xe, ye = 1.0, fmax_e
    xne = 0.9
    yne = ye + 0.5 * dydx_near_e * (xne - xe) + 0.5 * dydx_e * (xne - xe)
    segs = [corner_control_points(xc, yc, dydx_c, xnc, ync, dydx_near_c, cc),
            corner_control_points(xnc, ync, dydx_near_c, xiso, yiso, dydx_iso, cc),
            corner_control_points(xiso, yiso, dydx_iso, xne, yne, dydx_near_e, ce),
            corner_control_points(xne, yne, dydx_near_e, xe, ye, dydx_e, ce)]
    return Curve(segs)


def fiber_force_length(p):
    e_zero, e_iso = p['strain_at_zero_force'], p['strain_at_one_norm_force']
    k_low, k_iso = p['stiffness_at_low_force'], p['stiffness_at_one_norm_force']
    c = scale_curviness(p['curviness'])
    x_zero, y_zero = 1.0 + e_zero, 0.0
    x_iso, y_iso = 1.0 + e_iso, 1.0
    delta_x = min(0.1 * (1.0 / k_iso), 0.1 * (x_iso - x_zero))
    x_low = x_zero + delta_x
    x_foot = x_zero + 0.5 * (x_low - x_zero)
    y_foot = 0.0
    y_low = y_foot + k_low * (x_low - x_foot)
    segs = [corner_control_points(x_zero, y_zero, 0.0, x_low, y_low, k_low, c),
            corner_control_points(x_low, y_low, k_low, x_iso, y_iso, k_iso, c)]
    return Curve(segs)


def tendon_force_length(p):
    e_iso, k_iso, f_toe = p['strain_at_one_norm_force'], p['stiffness_at_one_norm_force'], p['norm_force_at_toe_end']
    c = scale_curviness(p['curviness'])
    x0, y0, dydx0 = 1.0, 0.0, 0.0
    x_iso, y_iso = 1.0 + e_iso, 1.0
    y_toe = f_toe
    x_toe = (y_toe - 1.0) / k_iso + x_iso
    x_foot = 1.0 + (x_toe - 1.0) / 10.0
    y_foot = 0.0
    y_toe_mid = y_toe * 0.5
    x_toe_mid = (y_toe_mid - y_iso) / k_iso + x_iso
    dydx_toe_mid = (y_toe_mid - y_foot) / (x_toe_mid - x_foot)
    x_toe_ctrl = x_foot + 0.5 * (x_toe_mid - x_foot)
    y_toe_ctrl = y_foot + dydx_toe_mid * (x_toe_ctrl - x_foot)
    segs = [corner_control_points(x0, y0, dydx0, x_toe_ctrl, y_toe_ctrl, dydx_toe_mid, c),
            corner_control_points(x_toe_ctrl, y_toe_ctrl, dydx_toe_mid, x_toe, y_toe, k_iso, c)]
    return Curve(segs)


def muscle_curves(overrides=None):
    """Return (fal, fv, fpe, fse) for a muscle; ``overrides`` maps curve tag ->
    {property: value} as parsed from the .osim file."""
    overrides = overrides or {}

    def params(tag):
        p = dict(DEFAULTS[tag])
        for k, v in overrides.get(tag, {}).items():
            if k in p:
                p[k] = v
        return p
    return (active_force_length(params('ActiveForceLengthCurve')),
            force_velocity(params('ForceVelocityCurve')),
            fiber_force_length(params('FiberForceLengthCurve')),
            tendon_force_length(params('TendonForceLengthCurve')))
