#!/usr/bin/env bash
# round 4, session e: float same-type Delta encode kernel + ballot-skip in the
# speculative decode: their GPU tests, the chain probe (redundant waves), and
# the little/big-endian Delta configs on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_nan_bits.py tests/test_gpu_byteorder.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_fuzz.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_e.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_e.log | tail -40; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/probe_chain.py > gpurun_out/probe_chain.log 2>&1 || exit $?
grep -E '"round": 2|correctness' gpurun_out/probe_chain.log
rm -rf gpurun_out/prof
bash tools/prof_all.sh ${PROF_CONFIGS:-D_i2 DI2_BE DF4_LE DF4_BE}
