#!/bin/bash
# Per-kernel register / scratch / LDS usage of libbioim's kernels (gfx950),
# from the compiler's kernel-resource-usage remarks, one topology per job
# (the shipped per-topology units, in parallel).  CPU only.
#   bash tools/resources.sh [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
# the shipped library's flags (bioimitation/_buildinfo.py: one place for them)
FLAGS=$(cd bioimitation-gym_amd && python3 -m bioimitation._buildinfo flags)
NT=$(sed -n 's/#define BIOIM_NTOPOLOGIES \([0-9]*\)/\1/p' bioimitation-gym_amd/csrc/topologies.h)
tmp=$(mktemp -d)
for k in $(seq 0 $((NT - 1))); do
  hipcc $FLAGS -DBIOIM_TOPO_ONLY=$k -c --offload-device-only \
      -Rpass-analysis=kernel-resource-usage "$@" -o $tmp/res$k.o bioimitation-gym_amd/csrc/bioim_step.hip > $tmp/res$k.txt 2>&1 &
done
hipcc $FLAGS -DBIOIM_FUSED_ONLY -c --offload-device-only \
    -Rpass-analysis=kernel-resource-usage "$@" -o $tmp/resF.o bioimitation-gym_amd/csrc/bioim_step.hip > $tmp/resF.txt 2>&1 &
wait
cat $tmp/res*.txt |
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
    n = re.sub(r'^_Z\d+', '', r['name'])[:64]
    v, a = r.get('VGPRs', 0), r.get('AGPRs', 0)
    print(f\"{n:64s} VGPR {v:>4} AGPR {a:>4} total {v + a:>4} SGPR {r.get('SGPRs','?'):>4} scratch {r.get('ScratchSize','?'):>5}\")
"
rm -rf $tmp
