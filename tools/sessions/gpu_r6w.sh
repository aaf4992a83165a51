#!/bin/bash
# round 6: one-launch CRC encode: 16 vs 32 KiB tiles x grid (lab)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6w
export TMPDIR=/tmp
CK_SWEEP_K4=1 timeout -k 10 400 python3 tools/probe_ck_encode.py > gpurun_out/r6w/probe_ck_encode_sweep.jsonl 2> gpurun_out/r6w/enc.err || { tail gpurun_out/r6w/enc.err; exit 1; }
cat gpurun_out/r6w/probe_ck_encode_sweep.jsonl
