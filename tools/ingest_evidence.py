"""Turn one GPU evidence pass (tools/gpu_evidence_r04.sh) into the records
bench.py reads: profiles/traffic.json (HBM bytes per launch from the
FETCH_SIZE / WRITE_SIZE passes) and profiles/valu.json (the VALU-side
record from the SQ passes), each stamped with the build id of the library
the pass profiled (``build_id``, the evidence dir's libbioim.so.buildid),
so bench.py can tell whether a record describes the binary it benchmarks.

    python tools/ingest_evidence.py <evidence dir> [<copy to: profiles/rNN/...>]

Per MI355X_MICROARCH.md (HBM/rocprofv3 section): FETCH_SIZE counts half the
bytes of the kernel's 128-B coalesced read requests, so bytes = 2 x
FETCH_SIZE + WRITE_SIZE (tools/traffic.py).  The kernel time the VALU record
divides by is the kernel-trace average of the same build's step dispatches.
"""
import csv
import glob
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)

import valu  # noqa: E402

CONFIGS = {'2d': 'MuscleWalkingImitation2D-v0', '3d': 'MuscleRunningImitation3D-v0'}
DEFAULT_KERNEL = 'false, false, false>'   # env_kernel<T, double, PERT=false, RK=false, REP=false>


def _step_rows(path, counter=False):
    rows = [r for r in csv.DictReader(open(path)) if 'env_kernel' in r['Kernel_Name']
            and 'double' in r['Kernel_Name'] and DEFAULT_KERNEL in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Dispatch_Id']))
    # the step launches' grid (4096 envs); round 5: the reset-table build adds one
    # smaller mode-1 dispatch of the same kernel (one scratch env per reference row)
    gkey = 'Grid_Size' if 'Grid_Size' in rows[0] else 'Grid_Size_X'
    grids = [r[gkey] for r in rows]
    step_grid = max(set(grids), key=grids.count)
    rows = [r for r in rows if r[gkey] == step_grid]
    return rows[1:]        # the first dispatch is the reset realize of bench.py's start


def kernel_ms(trace_dir):
    f = glob.glob(os.path.join(trace_dir, '**', '*kernel_trace.csv'), recursive=True)[0]
    rows = _step_rows(f)
    return sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rows) / len(rows) / 1e6, len(rows)


def counter_mean(pass_dir):
    f = glob.glob(os.path.join(pass_dir, '**', '*counter_collection.csv'), recursive=True)[0]
    rows = _step_rows(f, True)
    vals = {}
    for r in rows:
        vals.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def sq_summary(pmc_dir):
    vals = {}
    for p in sorted(glob.glob(os.path.join(pmc_dir, 'p*'))):
        if os.path.isdir(p):
            vals.update(counter_mean(p))
    return vals


def main():
    ev = sys.argv[1]
    copy_to = sys.argv[2] if len(sys.argv) > 2 else None
    bid = open(os.path.join(ev, 'libbioim.so.buildid')).read().strip()
    src = os.path.relpath(copy_to or ev, REPO)
    tpath, vpath = (os.path.join(REPO, 'profiles', n) for n in ('traffic.json', 'valu.json'))
    tdb = json.load(open(tpath)) if os.path.exists(tpath) else {}
    vdb = json.load(open(vpath)) if os.path.exists(vpath) else {}
    summary = {'build_id': bid}
    for k, env_id in CONFIGS.items():
        if not os.path.isdir(os.path.join(ev, f'{k}_trace')):
            continue
        key = f'{env_id}/fp64/4096'
        ms, nd = kernel_ms(os.path.join(ev, f'{k}_trace'))
        fetch = counter_mean(os.path.join(ev, f'{k}_fetch'))['FETCH_SIZE'] * 1024.0   # KB -> bytes
        write = counter_mean(os.path.join(ev, f'{k}_write'))['WRITE_SIZE'] * 1024.0
        tdb[key] = {'bytes': 2 * fetch + write, 'fetch_bytes_raw': fetch, 'fetch_bytes_x2': 2 * fetch,
                    'write_bytes': write, 'kernel_ms_trace': ms, 'dispatches': nd, 'source': src, 'build_id': bid}
        sq = sq_summary(os.path.join(ev, f'pmc_{k}'))
        if sq:
            rec = valu.record(sq, ms, src)
            rec.update(valu.issue_analysis(sq, ms))
            rec['build_id'] = bid
            vdb[key] = rec
            with open(os.path.join(ev, f'{k}_fp64_pmc_sq_summary.txt'), 'w') as fh:
                for c, v in sorted(sq.items()):
                    fh.write(f'{c:28s} {v:16.4g}\n')
        summary[key] = {'kernel_ms_trace': ms, 'traffic': tdb[key], 'valu': vdb.get(key)}
    json.dump(tdb, open(tpath, 'w'), indent=1, sort_keys=True)
    json.dump(vdb, open(vpath, 'w'), indent=1, sort_keys=True)
    if copy_to:
        os.makedirs(copy_to, exist_ok=True)
        for pat in ('*.json', '*.log', '*.txt', '*.buildid'):
            for f in glob.glob(os.path.join(ev, pat)):
                shutil.copy(f, copy_to)
        for k in CONFIGS:
            for f in glob.glob(os.path.join(ev, f'{k}_trace', '**', '*kernel_stats.csv'), recursive=True):
                shutil.copy(f, os.path.join(copy_to, f'{k}_fp64_kernel_stats.csv'))
        with open(os.path.join(copy_to, 'ingest_summary.json'), 'w') as fh:
            json.dump(summary, fh, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


if __name__ == '__main__':
    main()
