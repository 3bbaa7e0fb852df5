"""Per-launch HBM traffic of the env kernel from rocprofv3 FETCH_SIZE /
WRITE_SIZE passes (KB per dispatch) -> profiles/traffic.json, keyed like
bench.py's lookup: '<env_id>/fp<precision>/<envs>'.

Per MI355X_MICROARCH.md (HBM/rocprofv3 section): FETCH_SIZE counts 64 B per
memory-side read request and reads exactly 1/2 of the bytes of wide (16 B/lane)
coalesced streams; the env kernel's loads are 8 B/lane SoA rows, an
uncalibrated width, so the raw value is recorded next to the doubled one and
bench.py reports the raw FETCH + WRITE sum (a lower bound on bytes moved).
The reset dispatch (first, much shorter) is excluded.

    python tools/traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <env_id> <precision> <envs>
"""
import csv
import json
import os
import sys


def per_launch(path):
    rows = [r for r in csv.DictReader(open(path)) if 'env_kernel' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Dispatch_Id']))
    v = [float(r['Counter_Value']) * 1024.0 for r in rows[1:]]   # KB -> bytes, skip the reset launch
    return sum(v) / len(v)


def main():
    fcsv, wcsv, env_id, prec, n = sys.argv[1:6]
    fetch = per_launch(fcsv)
    write = per_launch(wcsv)
    d = os.path.dirname(os.path.dirname(fcsv))
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles', 'traffic.json')
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[f'{env_id}/fp{prec}/{n}'] = {'bytes': fetch + write, 'fetch_bytes_raw': fetch, 'fetch_bytes_x2': 2 * fetch,
                                    'write_bytes': write, 'source': d}
    json.dump(db, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps(db[f'{env_id}/fp{prec}/{n}']))


if __name__ == '__main__':
    main()
