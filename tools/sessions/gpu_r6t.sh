#!/bin/bash
# round 6: Adler32 one-launch verify over the grid cap (lab)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6t
export TMPDIR=/tmp
CK_ADLER=1 timeout -k 10 400 python3 tools/probe_ck_verify_grid6.py > gpurun_out/r6t/probe_adler_verify_grid.jsonl 2> gpurun_out/r6t/grid.err || { tail gpurun_out/r6t/grid.err; exit 1; }
cat gpurun_out/r6t/probe_adler_verify_grid.jsonl
