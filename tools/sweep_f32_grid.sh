#!/usr/bin/env bash
# One-launch Fletcher32 verify: sweep its knobs (MCODEC_F32_FUSED_GRID,
# MCODEC_F32_NTLD, MCODEC_F32_UNROLL, MCODEC_F32_SLICE_KB) with
# tools/probe_verify_overhead.py; one JSON line per setting.
# the MCODEC_* schedule variables act on the lab library only (tools/lab/lab_sched.hip)
export NUMCODECS_AMD_LIB="$(cd "$(dirname "$0")" && pwd)/_build/libmcodec_lab.so"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sweep_f32_knobs.jsonl
for cfg in "2048 1 4 32" "2048 0 4 32" "2048 1 8 32" "4096 1 4 32" "4096 1 8 32" "8192 1 4 32" "8192 1 8 32" "1024 1 8 64"; do
  set -- $cfg
  echo "{\"grid\": $1, \"ntld\": $2, \"unroll\": $3, \"slice_kb\": $4}" >> $out
  MCODEC_F32_FUSED_GRID=$1 MCODEC_F32_NTLD=$2 MCODEC_F32_UNROLL=$3 MCODEC_F32_SLICE_KB=$4 \
    timeout -k 10 120 python tools/probe_verify_overhead.py >> $out 2> gpurun_out/sweep_f32_knobs.err || exit $?
done
cat $out
