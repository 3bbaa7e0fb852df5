"""The C3 tracking drive (tests/tracking.py) on the fp64 oracle: from the
rows listed as ROWS_UP it keeps MuscleWalkingImitation2D-v0 up for 200 steps,
from ROWS_FALL the model falls, and the dynamics under it are not chaotic
(a one-ulp twin stays within 1e-8) — the premises of the GPU test
test_gpu_parity.py::test_parity_200_steps_c3_tracking_drive.  CPU only."""
import numpy as np
import pytest


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


@pytest.mark.parametrize('env_id', ['MuscleRunningImitation3D-v0', 'MuscleLockedKneeImitation3D-v0',
                                    'MusclePalsyImitation3D-v0', 'MuscleWalkingImitation2D-v0'])
def test_scheduled_drive_premises(env_id):
    """The premises of test_gpu_parity.py::test_parity_200_steps_muscle_tracking_drive
    on the oracle: the committed schedule (tests/golden/drive_<ID>.npz) was
    found for reset rows drawn by the reference's rule (random.seed(0) +
    random.randint(0, reset_hi), tools/drive_search.py) and keeps >= 50 % of
    the 32 envs alive for 200 steps or to the episode limit (istep >= N,
    which rows drawn near reset_hi reach first); under it the dynamics are mostly not
    chaotic: on >= 3/4 of the envs a one-ulp twin stays within 1e-6 while
    both are alive (the GPU test bounds each env by its own twins)."""
    import random
    import oracle
    from tracking import TrackingDrive, load_schedule, make_twin
    from bioimitation.obslayout import load_names
    from bioimitation.registry import load_pack
    rows, sched, P, gains = load_schedule(env_id)
    pk = load_pack(env_id)
    random.seed(0)
    assert list(rows) == [random.randint(0, pk.reset_hi) for _ in range(len(rows))]
    orc = oracle.Oracle(pk)
    drive = TrackingDrive(orc, pk, load_names(env_id), gains)
    n, T = len(rows), 200
    bufs, twin = orc.new_envs(n), orc.new_envs(n)
    for i, r in enumerate(rows):
        orc.reset(bufs, i, int(r))
        orc.reset(twin, i, int(r))
        make_twin(orc, twin, i, 5)
    alive, live, limit = np.ones(n, bool), np.ones(n, bool), np.zeros(n, bool)
    worst = np.zeros(n)
    for t in range(T):
        for i in np.where(alive)[0]:
            a = drive(orc.get_state(bufs, i), sched[i, t // P])
            o, r, d, _ = orc.step(bufs, i, a)
            o2, r2, d2, _ = orc.step(twin, i, a)
            if live[i]:
                worst[i] = max(worst[i], (np.abs(o2 - o) / np.maximum(1.0, np.abs(o))).max())
            alive[i] = not d
            limit[i] = d and orc.get_state(bufs, i)[1] >= pk.n_episode
            live[i] = live[i] and not (d or d2)
    assert (alive | limit).sum() >= n // 2, (alive.sum(), limit.sum())
    assert (worst < 1e-6).sum() >= 3 * n // 4, worst
