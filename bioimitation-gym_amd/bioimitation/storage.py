"""OpenSim Storage (.sto / .mot) text IO and ``read_from_storage``.

Restates ``read_from_storage`` (``bioimitation/imitation_envs/utils/opensim_utils.py:283-315``):
read the table, convert degrees to radians when the header says
``inDegrees=yes`` (rotational coordinate columns only, as
``SimbodyEngine::convertDegreesToRadians`` does), then ``resampleLinear(dt)``
(rows at ``t0 + dt*i``), returning a pandas DataFrame indexed by time.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Optional

import numpy as np


def read_sto(path: str):
    """Return (header dict, column labels, data array (rows, cols))."""
    header = {}
    with open(path, 'r') as fh:
        lines = fh.read().splitlines()
    i = 0
    while i < len(lines):
        ln = lines[i].strip()
        i += 1
        if ln.lower() == 'endheader':
            break
        if '=' in ln:
            k, v = ln.split('=', 1)
            header[k.strip()] = v.strip()
    labels = lines[i].split('\t') if '\t' in lines[i] else lines[i].split()
    labels = [l.strip() for l in labels if l.strip()]
    rows = [[float(t) for t in ln.split()] for ln in lines[i + 1:] if ln.strip()]
    return header, labels, np.array(rows, dtype=np.float64)


def write_sto(path: str, labels: List[str], data: np.ndarray, name: str = 'Storage', in_degrees: bool = False):
    with open(path, 'w') as fh:
        fh.write(f'{name}\nversion=1\nnRows={data.shape[0]}\nnColumns={data.shape[1]}\n')
        fh.write(f'inDegrees={"yes" if in_degrees else "no"}\nendheader\n')
        fh.write('\t'.join(labels) + '\n')
        for row in data:
            fh.write('\t'.join(f'{v:.10f}' for v in row) + '\n')


def resample_linear(time: np.ndarray, data: np.ndarray, dt: float):
    """Storage::resampleLinear: uniform rows t0 + dt*i up to the last time."""
    t0, tf = float(time[0]), float(time[-1])
    n = int((tf - t0) / dt + 1e-9) + 1
    t = np.array([t0 + dt * float(i) for i in range(n)])
    out = np.empty((n, data.shape[1]))
    for c in range(data.shape[1]):
        out[:, c] = np.interp(t, time, data[:, c])
    return t, out


def read_from_storage(path: str, sampling_interval: float, rotational: Optional[Iterable[str]] = None):
    """opensim_utils.py:283-315 restated; returns a pandas DataFrame with a
    'time' column, indexed by time."""
    import pandas as pd
    header, labels, arr = read_sto(path)
    time, data = arr[:, 0], arr[:, 1:]
    cols = labels[1:]
    if header.get('inDegrees', 'no').lower() == 'yes' and rotational is not None:
        rot = set(rotational)
        for j, c in enumerate(cols):
            if c in rot:
                data[:, j] *= math.pi / 180.0
    t, d = resample_linear(time, data, sampling_interval)
    df = pd.DataFrame(np.column_stack([t, d]), columns=['time'] + cols)
    df.index = df.time
    return df
