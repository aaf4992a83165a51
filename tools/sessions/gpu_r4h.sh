#!/usr/bin/env bash
# round 4, session h: same-type Delta encode 4 vs 8 vectors per thread
# (lab A/B + the schedule check of every alternative against the oracle)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/probe_delta_enc_dv.py > gpurun_out/probe_delta_enc_dv.log 2>&1 || exit $?
cat gpurun_out/probe_delta_enc_dv.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_sched.py tests/test_gpu_delta.py tests/test_gpu_nan_bits.py -m gpu -q -x --timeout 500 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_h.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_h.log | tail -20; [ $rc -eq 0 ] || exit $rc
