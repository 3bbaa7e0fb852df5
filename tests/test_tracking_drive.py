"""The C3 tracking drive (tests/tracking.py) on the fp64 oracle: from the
rows listed as ROWS_UP it keeps MuscleWalkingImitation2D-v0 up for 200 steps,
from ROWS_FALL the model falls, and the dynamics under it are not chaotic
(a one-ulp twin stays within 1e-8) — the premises of the GPU test
test_gpu_parity.py::test_parity_200_steps_c3_tracking_drive.  CPU only."""
import numpy as np


def test_tracking_drive_keeps_the_listed_rows_up():
    import oracle
    from tracking import ROWS_FALL, ROWS_UP, TrackingDrive
    from bioimitation.obslayout import load_names
    from bioimitation.registry import load_pack
    env_id = 'MuscleWalkingImitation2D-v0'
    pk = load_pack(env_id)
    orc = oracle.Oracle(pk)
    drive = TrackingDrive(orc, pk, load_names(env_id))
    rows = ROWS_UP + ROWS_FALL[:4]
    n, T = len(rows), 200
    bufs, twin = orc.new_envs(n), orc.new_envs(n)
    for i, r in enumerate(rows):
        orc.reset(bufs, i, r)
        orc.reset(twin, i, r)
        s = orc.get_state(twin, i)
        s[5] = np.nextafter(s[5], np.inf)
        orc.set_state(twin, i, s)
    alive = np.ones(n, bool)
    worst = 0.0
    for t in range(T):
        for i in np.where(alive)[0]:
            a = drive(orc.get_state(bufs, i))
            o, r, d, _ = orc.step(bufs, i, a)
            o2, r2, d2, _ = orc.step(twin, i, a)
            worst = max(worst, (np.abs(o2 - o) / np.maximum(1.0, np.abs(o))).max())
            assert d == d2
            alive[i] = not d
    assert alive[:len(ROWS_UP)].all() and not alive[len(ROWS_UP):].any(), alive
    assert worst < 1e-8, worst
