#!/bin/bash
# round 5: SQ counters of the scan decodes and the AsType widening cast
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
for cfg in "D_i2 dec" "C4 dec" "DF4_LE dec" "ASTYPE enc" "C5 dec"; do
  set -- $cfg
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES -d gpurun_out/sq/$1_$2 -o run -- python3 tools/prof_configs.py $1 $2 > gpurun_out/sq/$1_$2.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
