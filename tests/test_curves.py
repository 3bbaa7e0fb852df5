"""The device path inverts x(u) of each quintic Bezier segment from a
32-interval u(x) table (node values and slopes, cubic Hermite start) and a
fixed number of Newton steps: two in fp64, one in fp32 (bioim_step.hip
curve_eval).  Verify that this scheme reaches machine precision in fp64 and
stays below fp32 rounding in one step, on every segment of every curve of
every built pack (host restatement of the scheme)."""
import numpy as np

from bioimitation import registry
from bioimitation.curves import Curve

B, dB = Curve._bern, Curve._dbern


def _exact(px, x):
    lo, hi = 0.0, 1.0
    for _ in range(200):
        m = 0.5 * (lo + hi)
        if B(px, m) > x:
            hi = m
        else:
            lo = m
    return 0.5 * (lo + hi)


def test_hermite_table_plus_newton_steps_converges():
    worst = 0.0
    worst1 = 0.0
    for env_id in registry.RECIPES:
        pk = registry.load_pack(env_id)
        seen = set()
        for m in range(pk.nmuscle):
            for cv in (pk.muscle[m].fal, pk.muscle[m].fv, pk.muscle[m].fpe, pk.muscle[m].fse):
                for s in range(cv.nseg):
                    px = np.array(cv.x[s][:])
                    if tuple(px) in seen:
                        continue
                    seen.add(tuple(px))
                    a, b = px[0], px[5]
                    ut = np.array([_exact(px, a + (b - a) * i / 32) for i in range(33)])
                    mt = (b - a) / 32 / dB(px, ut)
                    xt = np.linspace(a, b, 997)
                    tt = (xt - a) * (32 / (b - a))
                    i0 = np.clip(tt.astype(int), 0, 31)
                    f = tt - i0
                    u0, u1, m0, m1 = ut[i0], ut[i0 + 1], mt[i0], mt[i0 + 1]
                    c2 = 3 * (u1 - u0) - 2 * m0 - m1
                    c3 = m0 + m1 - 2 * (u1 - u0)
                    u = u0 + f * (m0 + f * (c2 + f * c3))
                    for it in range(2):
                        u = u - (B(px, u) - xt) / dB(px, u)
                        if it == 0:
                            worst1 = max(worst1, np.abs(B(px, u) - xt).max() / max(1.0, np.abs(xt).max()))
                    worst = max(worst, np.abs(B(px, u) - xt).max())
    assert worst < 5e-15, worst
    assert worst1 < 6e-8, worst1
