#!/bin/bash
# round 5: CRC tile kernel back to the round-4 fused tail -- checksum tests, CRC configs re-profiled
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_next.py tests/test_gpu_codecs.py tests/test_gpu_chunks.py tests/test_gpu_fuzz.py tests/test_gpu_graphs.py > gpurun_out/r5l_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5l_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_all.sh CRC32 CRC32C 2>&1 | cut -c1-150
