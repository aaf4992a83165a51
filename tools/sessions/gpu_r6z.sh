#!/bin/bash
# round 6: Fletcher32 one-launch verify over its grid x slice schedule (lab)
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6z
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/probe_f32_verify_sched.py > gpurun_out/r6z/probe_f32_verify_sched.jsonl 2> gpurun_out/r6z/f32.err || { tail gpurun_out/r6z/f32.err; exit 1; }
cat gpurun_out/r6z/probe_f32_verify_sched.jsonl
