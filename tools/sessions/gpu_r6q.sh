#!/bin/bash
# round 6: one-launch CRC verify (ride finish) over the grid cap, back-to-back and single launches (lab)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6q
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/probe_ck_verify_grid6.py > gpurun_out/r6q/probe_ck_verify_grid6.jsonl 2> gpurun_out/r6q/grid.err || { tail gpurun_out/r6q/grid.err; exit 1; }
cat gpurun_out/r6q/probe_ck_verify_grid6.jsonl
