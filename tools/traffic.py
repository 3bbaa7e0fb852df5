"""Per-launch HBM traffic of the env kernel from rocprofv3 FETCH_SIZE /
WRITE_SIZE passes (KB per dispatch) -> profiles/traffic.json, keyed like
bench.py's lookup: '<env_id>/fp<precision>/<envs>'.

Per MI355X_MICROARCH.md (HBM/rocprofv3 section): FETCH_SIZE counts 64 B per
memory-side read request and reads exactly 1/2 of the bytes of wide (16 B/lane)
coalesced streams.  The env kernel's loads are 8 B/lane SoA rows of 16
consecutive envs (128 B per workgroup row), i.e. whole 128-B requests, so the
doubled value is the byte count: ``bytes`` = 2 x FETCH_SIZE + WRITE_SIZE
(the raw counter is kept next to it).  WRITE_SIZE matches the algorithmic
write bytes to 0.1 %, which supports reading the counters this way.
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
    db[f'{env_id}/fp{prec}/{n}'] = {'bytes': 2 * fetch + write, 'fetch_bytes_raw': fetch, 'fetch_bytes_x2': 2 * fetch,
                                    'write_bytes': write, 'source': d}
    json.dump(db, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps(db[f'{env_id}/fp{prec}/{n}']))


if __name__ == '__main__':
    main()
