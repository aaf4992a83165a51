#!/bin/bash
# round 6: CRC verify, 16 / 32 / 64 KiB tiles over the grid (lab)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6u
export TMPDIR=/tmp
CK_KSWEEP=1 timeout -k 10 400 python3 tools/probe_ck_verify_grid6.py > gpurun_out/r6u/probe_crc_verify_k.jsonl 2> gpurun_out/r6u/grid.err || { tail gpurun_out/r6u/grid.err; exit 1; }
cat gpurun_out/r6u/probe_crc_verify_k.jsonl
