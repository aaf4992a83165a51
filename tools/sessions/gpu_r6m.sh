#!/bin/bash
# round 6: one-launch CRC encode store policy A/B (lab), and the schedule checks
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6m
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/probe_ck_encode.py > gpurun_out/r6m/probe_ck_encode.jsonl 2> gpurun_out/r6m/enc.err || { tail gpurun_out/r6m/enc.err; exit 1; }
cat gpurun_out/r6m/probe_ck_encode.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_sched.py tests/test_gpu_next.py -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r6m/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6m/tests.log; exit $rc
