#!/usr/bin/env bash
# One-launch Fletcher32 verify: sweep the block cap (MCODEC_F32_FUSED_GRID)
# with tools/probe_verify_overhead.py; one JSON line per setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for g in 1024 2048 4096 8192; do
  MCODEC_F32_FUSED_GRID=$g timeout -k 10 120 python tools/probe_verify_overhead.py >> gpurun_out/sweep_f32_grid.jsonl 2> gpurun_out/sweep_f32_grid.err || exit $?
done
tail -4 gpurun_out/sweep_f32_grid.jsonl
