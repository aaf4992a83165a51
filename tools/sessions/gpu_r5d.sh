#!/bin/bash
# round 5: SGPR-fed chain with global stores -- parity, then noise decode timing
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_delta_walk.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_delta.py tests/test_gpu_nan_bits.py tests/test_gpu_ext_dtypes.py > gpurun_out/r5d_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5d_tests.log; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f4 256 quick > gpurun_out/walk_f4_randn_r5d.json 2>&1
rc=$?; tail -1 gpurun_out/walk_f4_randn_r5d.json; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f8 256 quick > gpurun_out/walk_f8_randn_r5d.json 2>&1
rc=$?; tail -1 gpurun_out/walk_f8_randn_r5d.json; exit $rc
