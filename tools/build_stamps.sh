#!/bin/bash
# Diagnostic build with per-phase s_memtime stamps (tools/stamps.py reads them).
set -e
cd "$(dirname "$0")/.."
C=bioimitation-gym_amd/csrc
# the shipped library's flags (bioimitation/_buildinfo.py: one place for them)
FLAGS=$(cd bioimitation-gym_amd && python3 -m bioimitation._buildinfo flags)
hipcc $FLAGS -shared -DBIOIM_STAMPS -o bioimitation-gym_amd/build/libbioim_stamps.so $C/bioim_step.hip
