#!/usr/bin/env bash
# CRC v3 (half-pipelined, LDS alignment tables): parity, kernel traces, K/grid A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_next.py tests/test_gpu_sched.py tests/test_gpu_chunks.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/ck_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ck_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v3_kt_32 -o run -- python3 tools/probe_crc_verify.py crc32 > /dev/null 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v3_kt_c -o run -- python3 tools/probe_crc_verify.py crc32c > /dev/null 2>&1 || exit $?
MCODEC_CK_K=8 NUMCODECS_AMD_LIB=tools/_build/libmcodec_lab.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v3_kt_c_k8 -o run -- python3 tools/probe_crc_verify.py crc32c > /dev/null 2>&1 || exit $?
timeout -k 10 600 python3 tools/probe_crc_bs.py bitsliced bs_k8 bs_k8_grid768 bs_grid1024 bs_gridcopy768 > gpurun_out/probe_crc_bs5.jsonl 2> gpurun_out/probe_crc_bs5.err || exit $?
echo done
