#!/bin/bash
# Same-box A/B of library builds with LDS bank-conflict counters (GPU box).
#   bash tools/ab_lds.sh <out-dir> <rounds> <env_id> <lib|tree> [<lib|tree> ...]
# Per library: R alternating bench.py rounds (kernel ms per step), then one
# rocprofv3 pass of SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS / SQ_INSTS_LDS /
# SQ_INSTS_VALU over 5 steps (summed per dispatch by tools/pmc_summary.py).
set -e
out=$(realpath -m "$1"); rounds=$2; id=$3; shift 3
mkdir -p "$out"
bash tools/ab.sh "$out/time" "$rounds" "$id" "$@"
REPO=$(pwd)
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  d="$out/pmc_$tag"
  mkdir -p "$d"
  if [ "$lib" = tree ]; then unset BIOIM_LIB; else export BIOIM_LIB=$(realpath "$lib"); fi
  (cd /tmp && TMPDIR=/tmp timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU \
      --output-format csv -d "$d/p1" -o p1 -- python3 "$REPO/bench.py" --steps 5 --warmup 2 --burn-in 0 \
      --no-cpu-baseline --env-id "$id" > "$d/p1.log" 2>&1)
  unset BIOIM_LIB
  echo "== $tag"
  python3 "$REPO/tools/pmc_summary.py" "$d"
done
