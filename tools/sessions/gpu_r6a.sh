#!/bin/bash
# round 6: effective clock + SQ counters of the Shuffle(4) / BitRound+Shuffle(4) / Shuffle(8) encodes
# (VERDICT r5 item 3): one kernel-trace pass and one PMC pass (8 SQ + 2 GRBM) per config
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r6a
export TMPDIR=/tmp
for cfg in "C2_f32 enc" "C3 enc" "C2_f64 enc"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6a/kt_$1_$2 -o run -- python3 tools/prof_configs.py $1 $2 > gpurun_out/r6a/kt_$1_$2.log 2>&1
  rc=$?; echo "kt $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r6a/pmc_$1_$2 -o run -- python3 tools/prof_configs.py $1 $2 > gpurun_out/r6a/pmc_$1_$2.log 2>&1
  rc=$?; echo "pmc $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
