#!/bin/bash
# round 6: the CRC one-launch finish: tests, tail-cost probe, finish probe
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6l
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_next.py tests/test_gpu_codecs.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6l/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6l/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/probe_ck_tail.py > gpurun_out/r6l/probe_ck_tail.jsonl 2> gpurun_out/r6l/tail.err || { tail gpurun_out/r6l/tail.err; exit 1; }
cat gpurun_out/r6l/probe_ck_tail.jsonl
timeout -k 10 300 python3 tools/probe_ck_stamp.py > gpurun_out/r6l/probe_ck_stamp.jsonl 2> gpurun_out/r6l/stamp.err || { tail gpurun_out/r6l/stamp.err; exit 1; }
grep -v lab_stamped gpurun_out/r6l/probe_ck_stamp.jsonl
