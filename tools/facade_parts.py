"""Where the single-env facade's host time goes beyond the step launch (C1,
TorqueWalkingImitation2D-v0, one env, fp64, recorder on): ImitationEnv.step's
parts replayed with a clock around each, 300 steps after 30 warm-up steps,
medians.  The synchronizing part (the output transfer) includes the wait for
the step kernel, so the kernel's duration is subtracted from it in the
printout (rocprofv3 gives that).

    python tools/facade_parts.py [env id]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'bioimitation-gym_amd')]
import torch  # noqa: E402
from bioimitation import envs  # noqa: E402

ENV = sys.argv[1] if len(sys.argv) > 1 else 'TorqueWalkingImitation2D-v0'
W, K = 30, 300


def main():
    e = envs.make(ENV, config={'record_trajectory': True, 'mode': 'test'})
    e.reset()
    rng = np.random.default_rng(0)
    lo, hi = np.asarray(e.action_space.low), np.asarray(e.action_space.high)
    parts = {}

    def clk(name, t0):
        t1 = time.perf_counter()
        parts.setdefault(name, []).append(t1 - t0)
        return t1

    full = []
    for k in range(W + K):
        action = lo + (hi - lo) * rng.uniform(0.3, 0.7, size=lo.shape)
        t0 = time.perf_counter()
        t = t0
        a = torch.as_tensor(np.asarray(action, dtype=np.float64).reshape(1, -1), dtype=e._env.dtype, device=e._env.device)
        t = clk('action to device (as_tensor)', t)
        obs, rew, done, info = e._env.step(a)
        t = clk('step launch', t)
        e.osim_model._dirty()
        parts_ = [obs[0], rew[:1], info[0], done[:1].to(obs.dtype)]
        t = clk('done to float (a kernel)', t)
        parts_.append(e._env.force_report[0])
        parts_.append(e._env.state_rows(e._state_buf)[0])
        t = clk('state rows (a kernel)', t)
        cat = torch.cat(parts_)
        t = clk('cat (a kernel)', t)
        out = cat.double().cpu().numpy()
        t = clk('to host (waits for the step)', t)
        nobs, ninf = obs.shape[1], info.shape[1]
        o = out[:nobs]
        nfr = e._env.force_report.shape[1]
        f0 = nobs + 1 + ninf + 1
        e._record_row(o, fr=out[f0:f0 + nfr], state=out[f0 + nfr:])
        t = clk('record row', t)
        inf = [float(v) for v in out[nobs + 1:nobs + 1 + ninf]]
        e._last = (float(out[nobs]), inf, bool(out[nobs + 1 + ninf]))
        r = [e._out(o[None, :], False), e._last[0], e._last[2], {'all_rewards': inf}]
        t = clk('return values', t)
        full.append(t - t0)
        if k % 50 == 49:
            e.reset()
        del r
    print(f'{ENV}: facade step parts, host wall clock, median of {K} steps')
    for n, v in parts.items():
        print(f'  {n:32s} {1e6 * np.median(v[W:]):8.1f} us')
    print(f'  {"whole step":32s} {1e6 * np.median(full[W:]):8.1f} us')


if __name__ == '__main__':
    main()
