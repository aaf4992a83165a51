#!/bin/bash
# round 5: loads of the scan passes in flight together -- parity, then the scan configs re-profiled
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_delta.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_delta_walk.py tests/test_gpu_c4.py tests/test_gpu_byteorder.py tests/test_gpu_nan_bits.py tests/test_gpu_chunks.py tests/test_gpu_fullsize.py tests/test_gpu_ext_dtypes.py > gpurun_out/r5t_tests.log 2>&1
rc=$?; tail -1 gpurun_out/r5t_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_all.sh C4 D_i2 DI2_BE DF4_LE DF4_BE 2>&1 | cut -c1-150
