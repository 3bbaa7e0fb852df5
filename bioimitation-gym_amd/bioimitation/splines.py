"""SimmSpline (OpenSim) coefficient fit and evaluation, host side.

OpenSim's ``SimmSpline`` is the Forsythe-Malcolm-Moler cubic spline: the
tridiagonal system is closed by matching the third derivative at each end to
the third divided difference of the four end knots, and values outside the
knot range are extrapolated linearly with the end slope.  The knee
translations (``data/2D/scale/model_scaled.osim`` knee_r TransformAxis
translation1/2) and the quadriceps MovingPathPoint locations use it.

The coefficients (b, c, d) are fitted once here and stored in the ModelPack;
both the C oracle and the HIP kernels evaluate
``y + dx*(b + dx*(c + dx*d))`` on the knot interval containing ``q``.
"""
from __future__ import annotations

import numpy as np


def simm_spline_coeffs(x, y):
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n = x.size
    b = np.zeros(n)
    c = np.zeros(n)
    d = np.zeros(n)
    if n < 2:
        return b, c, d
    if n < 3:
        b[0] = (y[1] - y[0]) / (x[1] - x[0])
        b[1] = b[0]
        return b, c, d
    nm1 = n - 1
    d[0] = x[1] - x[0]
    c[1] = (y[1] - y[0]) / d[0]
    for i in range(1, nm1):
        d[i] = x[i + 1] - x[i]
        b[i] = 2.0 * (d[i - 1] + d[i])
        c[i + 1] = (y[i + 1] - y[i]) / d[i]
        c[i] = c[i + 1] - c[i]
    b[0] = -d[0]
    b[nm1] = -d[n - 2]
    c[0] = 0.0
    c[nm1] = 0.0
    if n > 3:
        d31 = x[3] - x[1]
        d20 = x[2] - x[0]
        d1 = x[nm1] - x[n - 3]
        d2 = x[nm1 - 1] - x[n - 4]
        d30 = x[3] - x[0]
        d3 = x[nm1] - x[n - 4]
        c[0] = c[2] / d31 - c[1] / d20
        c[nm1] = c[n - 2] / d1 - c[n - 3] / d2
        c[0] = c[0] * d[0] * d[0] / d30
        c[nm1] = -c[nm1] * d[n - 2] * d[n - 2] / d3
    for i in range(1, n):
        t = d[i - 1] / b[i - 1]
        b[i] -= t * d[i - 1]
        c[i] -= t * c[i - 1]
    c[nm1] /= b[nm1]
    for j in range(nm1):
        i = nm1 - j - 1
        c[i] = (c[i] - d[i] * c[i + 1]) / b[i]
    b[nm1] = (y[nm1] - y[n - 2]) / d[n - 2] + d[n - 2] * (c[n - 2] + 2.0 * c[nm1])
    for i in range(nm1):
        b[i] = (y[i + 1] - y[i]) / d[i] - d[i] * (c[i + 1] + 2.0 * c[i])
        d[i] = (c[i + 1] - c[i]) / d[i]
        c[i] *= 3.0
    c[nm1] *= 3.0
    d[nm1] = d[n - 2]
    return b, c, d


def simm_spline_eval(x, y, b, c, d, q, deriv=0):
    """Value (deriv=0), slope (1) or curvature (2) of the fitted spline."""
    n = len(x)
    if q < x[0]:
        return (y[0] + (q - x[0]) * b[0]) if deriv == 0 else (b[0] if deriv == 1 else 0.0)
    if q > x[n - 1]:
        return (y[n - 1] + (q - x[n - 1]) * b[n - 1]) if deriv == 0 else (b[n - 1] if deriv == 1 else 0.0)
    k = 0
    while k < n - 2 and q > x[k + 1]:
        k += 1
    dx = q - x[k]
    if deriv == 0:
        return y[k] + dx * (b[k] + dx * (c[k] + dx * d[k]))
    if deriv == 1:
        return b[k] + dx * (2.0 * c[k] + 3.0 * dx * d[k])
    return 2.0 * c[k] + 6.0 * dx * d[k]
