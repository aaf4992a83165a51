#!/bin/bash
# round 5: SQ counters of the verify kernels and the Shuffle(8)/C3 encodes
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
for cfg in "ADLER32 dec" "CRC32 dec" "F32 dec" "C2_f64 enc" "C3 enc" "C2_f32 enc" "PACKBITS enc"; do
  set -- $cfg
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES -d gpurun_out/sq/$1_$2 -o run -- python3 tools/prof_configs.py $1 $2 > gpurun_out/sq/$1_$2.log 2>&1
  rc=$?; echo "$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
