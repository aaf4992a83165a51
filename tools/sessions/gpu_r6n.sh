#!/bin/bash
# round 6: one-launch CRC encode: tile size x grid sweep (lab)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6n
export TMPDIR=/tmp
CK_SWEEP=1 timeout -k 10 400 python3 tools/probe_ck_encode.py > gpurun_out/r6n/probe_ck_encode_sweep.jsonl 2> gpurun_out/r6n/enc.err || { tail gpurun_out/r6n/enc.err; exit 1; }
cat gpurun_out/r6n/probe_ck_encode_sweep.jsonl
