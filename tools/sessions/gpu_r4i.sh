#!/usr/bin/env bash
# round 4, session i: big-endian input swaps after the loads (Delta encode,
# speculative decode): tests, encode A/B, Delta configs on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_delta_walk.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_byteorder.py tests/test_gpu_nan_bits.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_i.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_i.log | tail -20; [ $rc -eq 0 ] || exit $rc
DVS=4,4 timeout -k 10 300 python -u tools/probe_delta_enc_dv.py > gpurun_out/probe_delta_enc_dv.log 2>&1 || exit $?
grep dtype gpurun_out/probe_delta_enc_dv.log
rm -rf gpurun_out/prof
bash tools/prof_all.sh ${PROF_CONFIGS:-D_i2 DI2_BE DF4_LE DF4_BE}
