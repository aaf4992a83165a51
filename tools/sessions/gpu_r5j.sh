#!/bin/bash
# round 5: pipelined bitshuffle -- parity, then A/B against the one-tile kernel (variant .so)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_next.py -k "blosc or bitshuffle" > gpurun_out/r5j_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5j_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/probe_r5.py > gpurun_out/probe_r5j_pipe_$r.jsonl 2>&1
  rc=$?; grep bitshuffle gpurun_out/probe_r5j_pipe_$r.jsonl | cut -c1-160; [ $rc -eq 0 ] || exit $rc
  NUMCODECS_AMD_LIB=tools/_build/libmcodec.so timeout -k 10 200 python -u tools/probe_r5.py > gpurun_out/probe_r5j_old_$r.jsonl 2>&1
  rc=$?; grep bitshuffle gpurun_out/probe_r5j_old_$r.jsonl | cut -c1-160; [ $rc -eq 0 ] || exit $rc
done
