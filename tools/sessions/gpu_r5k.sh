#!/bin/bash
# round 5: pipelined bitshuffle in the product -- parity (next rows, chunks), timings
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_next.py tests/test_gpu_chunks.py tests/test_gpu_delta_walk.py > gpurun_out/r5k_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5k_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe_r5.py > gpurun_out/probe_r5k.jsonl 2>&1
rc=$?; grep bitshuffle gpurun_out/probe_r5k.jsonl | cut -c1-170; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f4 256 quick > gpurun_out/walk_f4_randn_r5k.json 2>&1
rc=$?; tail -1 gpurun_out/walk_f4_randn_r5k.json; exit $rc
