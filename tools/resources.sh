#!/bin/bash
# Per-kernel register / scratch / LDS usage of libbioim's kernels (gfx950),
# from the compiler's kernel-resource-usage remarks.  CPU only.
#   bash tools/resources.sh [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
# the shipped library's flags (bioimitation/_buildinfo.py: one place for them)
FLAGS=$(cd bioimitation-gym_amd && python3 -m bioimitation._buildinfo flags)
hipcc $FLAGS -c --offload-device-only \
    -Rpass-analysis=kernel-resource-usage "$@" -o /tmp/bioim_res.o bioimitation-gym_amd/csrc/bioim_step.hip 2>&1 |
    python3 -c "
import re, sys
cur = None
rows = []
for l in sys.stdin:
    m = re.search(r'Function Name: (\S+)', l)
    if m:
        cur = {'name': m.group(1)}; rows.append(cur); continue
    m = re.search(r'remark: (?:.*?)(VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)', l)
    if m and cur is not None:
        cur[m.group(1).split(' ')[0]] = int(m.group(2))
for r in rows:
    n = re.sub(r'^_Z\d+', '', r['name'])[:60]
    print(f\"{n:60s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>4} SGPR {r.get('SGPRs','?'):>4} scratch {r.get('ScratchSize','?'):>5}\")
"
