#!/bin/bash
# round 6: int16 Delta reduce pass, per-group workgroups against a persistent prefetching grid (lab)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6zb
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/probe_dscan_reduce.py > gpurun_out/r6zb/probe_dscan_reduce.jsonl 2> gpurun_out/r6zb/dsr.err || { tail gpurun_out/r6zb/dsr.err; exit 1; }
cat gpurun_out/r6zb/probe_dscan_reduce.jsonl
