#!/bin/bash
# round 6: Adler32 one-launch verify, 32 vs 64 KiB tiles x grid (lab)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6x
export TMPDIR=/tmp
CK_ADLER=1 CK_KSWEEP=1 timeout -k 10 400 python3 tools/probe_ck_verify_grid6.py > gpurun_out/r6x/probe_adler_verify_k.jsonl 2> gpurun_out/r6x/grid.err || { tail gpurun_out/r6x/grid.err; exit 1; }
cat gpurun_out/r6x/probe_adler_verify_k.jsonl
