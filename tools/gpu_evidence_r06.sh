#!/bin/bash
# Round 6 GPU evidence on the build in the tree (run from the repo root on the box), in two calls:
#   bash tools/gpu_evidence_r06.sh <tag> A   GPU tests (default and bounds-checked builds), smoke, bench lines
#                                            (C3 headline with CPU baselines, C4, C2, C5 fused / concurrent,
#                                            LockedKnee3D, Palsy3D), the driver's command x3, the single-env
#                                            breakdown with and without the kernel trace
#   bash tools/gpu_evidence_r06.sh <tag> B   rocprofv3 kernel-trace stats, FETCH_SIZE / WRITE_SIZE and the SQ
#                                            counter passes of the 2D and 3D kernels, the VALU census
# Each writes into gpurun_out/<tag> with the build id of the library it measured; then, in the dev container:
#     python tools/ingest_evidence.py gpurun_out/<tag> profiles/r06/<tag>
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
TAG=${1:-r06ev}; PART=${2:-A}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cp bioimitation-gym_amd/build/libbioim.so.buildid $O/
if [ "$PART" == A ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
  if [ -f bioimitation-gym_amd/build/ab/check/libbioim.so ]; then   # the bounds-checked build (BIOIM_CHECK=1)
    BIOIM_LIB=$PWD/bioimitation-gym_amd/build/ab/check/libbioim.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
        --timeout 300 --timeout-method thread > $O/gpu_tests_check.log 2>&1
  fi
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
  timeout -k 10 300 python bench.py --env-id MuscleRunningImitation3D-v0 --no-cpu-baseline --no-single-env > $O/bench_3d.json 2>> $O/bench.err
  timeout -k 10 300 python bench.py --env-id TorqueWalkingImitation2D-v0 --no-cpu-baseline --no-single-env > $O/bench_torque2d.json 2>> $O/bench.err
  timeout -k 10 300 python bench.py --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 --no-cpu-baseline > $O/bench_mixed.json 2>> $O/bench.err
  timeout -k 10 300 python bench.py --mixed MuscleLockedKneeImitation3D-v0,MusclePalsyImitation3D-v0 --no-cpu-baseline --no-fuse --no-reference-integrator > $O/bench_mixed_nofuse.json 2>> $O/bench.err
  for E in MuscleLockedKneeImitation3D-v0 MusclePalsyImitation3D-v0; do
    timeout -k 10 300 python bench.py --env-id $E --no-cpu-baseline --no-single-env > $O/bench_$E.json 2>> $O/bench.err
  done
  for i in 1 2 3; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_$i.json 2>> $O/bench.err
  done
  for E in TorqueWalkingImitation2D-v0 MuscleWalkingImitation2D-v0; do
    timeout -k 10 300 python tools/single_env_breakdown.py $E > $O/single_$E.txt 2>&1
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/single_trace_$E -o s -- \
       python3 $OLDPWD/tools/single_env_breakdown.py $E > $OLDPWD/$O/single_trace_$E.txt 2>&1)
  done
  echo evidence A done
else
  for CFG in "2d:MuscleWalkingImitation2D-v0" "3d:MuscleRunningImitation3D-v0"; do
    K=${CFG%%:*}; E=${CFG#*:}
    A="--env-id $E --steps 20 --warmup 3 --no-cpu-baseline --no-reference-integrator --no-single-env"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/${K}_trace -o trace -- python3 $OLDPWD/bench.py $A > $OLDPWD/$O/${K}_trace.log 2>&1)
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OLDPWD/$O/${K}_fetch -o fetch -- python3 $OLDPWD/bench.py $A > $OLDPWD/$O/${K}_fetch.log 2>&1)
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OLDPWD/$O/${K}_write -o write -- python3 $OLDPWD/bench.py $A > $OLDPWD/$O/${K}_write.log 2>&1)
    i=0
    for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
             "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" \
             "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY" \
             "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU"; do
      i=$((i+1))
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $OLDPWD/$O/pmc_${K}/p$i -o p$i -- \
          python3 $OLDPWD/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-reference-integrator --no-single-env --env-id $E \
          > $OLDPWD/$O/pmc_${K}_p$i.log 2>&1)
    done
  done
  bash tools/pmc_census.sh ${TAG}_census > $O/census.log 2>&1
  cp -r gpurun_out/pmc_${TAG}_census $O/pmc_census
  echo evidence B done
fi
