#!/bin/bash
# round 5 call y: the first timed window of a process (bench.py times one) against later ones
set -o pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/r05y; mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/first_window.py >> $out/first_window3.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/first_window.py --dry-window 5 >> $out/first_window3.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/first_window.py --dry-window 20 >> $out/first_window3.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/first_window.py --idle-ms 20 >> $out/first_window3.log 2>&1 || exit 1
done
echo exit 0
