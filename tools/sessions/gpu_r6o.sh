#!/bin/bash
# round 6: SQ counters of the one-launch checksum verifies and CRC encodes
# one kernel-trace pass and one PMC pass (8 SQ + 2 GRBM) per config
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r6o
export TMPDIR=/tmp
for cfg in "CRC32 dec" "CRC32C dec" "ADLER32 dec" "F32 dec" "CRC32 enc" "CRC32C enc"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6o/kt_$1_$2 -o run -- python3 tools/prof_configs.py $1 $2 > gpurun_out/r6o/kt_$1_$2.log 2>&1
  rc=$?; echo "kt $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r6o/pmc_$1_$2 -o run -- python3 tools/prof_configs.py $1 $2 > gpurun_out/r6o/pmc_$1_$2.log 2>&1
  rc=$?; echo "pmc $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
