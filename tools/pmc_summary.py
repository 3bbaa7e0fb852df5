"""Summarise tools/pmc_sq.sh output: per-dispatch average of each counter
over the env-kernel step dispatches (the first, reset, dispatch skipped)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
vals = {}
for f in sorted(glob.glob(os.path.join(d, 'p*', '*counter_collection.csv'))):
    rows = [r for r in csv.DictReader(open(f)) if 'env_kernel' in r['Kernel_Name'] and 'false, false>' in r['Kernel_Name']]   # the default (no push, semi-implicit) kernel
    # the step launches' grid only (round 5: the reset-table build adds one smaller dispatch)
    grids = [r['Grid_Size'] for r in rows]
    rows = [r for r in rows if r['Grid_Size'] == max(set(grids), key=grids.count)]
    disp = sorted({int(r['Dispatch_Id']) for r in rows})[1:]
    for r in rows:
        if int(r['Dispatch_Id']) in disp:
            vals.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
for k, v in vals.items():
    n = len(v) and len({0})
    print(f'{k:28s} {sum(v) / max(1, len(v)):16.4g}  (n={len(v)})')
