#!/bin/bash
# round 6: longdouble / clongdouble, datetime unit-change Delta, calendar casts (tests/test_gpu_ld.py) then the whole GPU suite
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ld.py tests/test_gpu_ext_dtypes.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r6b_ld.log 2>&1; rc=$?
tail -25 gpurun_out/r6b_ld.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r6b_all.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/r6b_all.log | tail -20; exit $rc
