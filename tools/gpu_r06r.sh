#!/bin/bash
# Round 6, GPU call r (final build 5ff29d07decbd052): the multi-rank bench path on the final build, ranks
# sharing the one GPU (rehearsal only, marked in the line): C3 with 2 ranks,
# C4 with 4 ranks, C5 with 2 ranks; and the driver's own default command.
set -e
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --steps 50 --warmup 5 --no-cpu-baseline --no-single-env > $O/rehearsal_n2.json 2> $O/rehearsal_n2.err
timeout -k 10 300 python bench.py --gpus 4 --share-gpu --steps 50 --warmup 5 --no-cpu-baseline --no-single-env --env-id MuscleRunningImitation3D-v0 > $O/rehearsal_n4_c4.json 2> $O/rehearsal_n4_c4.err
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --steps 50 --warmup 5 --no-cpu-baseline --no-single-env --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 > $O/rehearsal_n2_c5.json 2> $O/rehearsal_n2_c5.err
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
echo done
