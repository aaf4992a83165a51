#!/bin/bash
# round 6: the fuzz suite with the one-launch checksum fuzz
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6s
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider --durations=5 > gpurun_out/r6s/fuzz.log 2>&1; rc=$?
tail -12 gpurun_out/r6s/fuzz.log; exit $rc
