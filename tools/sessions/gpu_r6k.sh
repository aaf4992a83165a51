#!/bin/bash
# round 6: the one-launch CRC verify's cost of bytes outside the whole tiles
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6k
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/probe_ck_tail.py > gpurun_out/r6k/probe_ck_tail.jsonl 2> gpurun_out/r6k/tail.err || { tail gpurun_out/r6k/tail.err; exit 1; }
cat gpurun_out/r6k/probe_ck_tail.jsonl
