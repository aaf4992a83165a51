#!/usr/bin/env bash
# CRC / Adler verify: parity subset, kernel traces (CRC32 start = aligned
# head tiling, CRC32C end, Fletcher32 for reference) and the fold A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_next.py tests/test_gpu_sched.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/ck_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ck_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt_32 -o run -- python3 tools/probe_crc_verify.py crc32 > gpurun_out/kt_32.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt_c -o run -- python3 tools/probe_crc_verify.py crc32c > gpurun_out/kt_c.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f32_kt -o run -- python3 tools/probe_ck_single.py > gpurun_out/kt_f32.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/probe_crc_bs.py bitsliced lds_tables bs_grid1024 bs_grid2048 > gpurun_out/probe_crc_bs3.jsonl 2>&1 || exit $?
timeout -k 10 400 python3 tools/probe_all.py > gpurun_out/probe_all3.jsonl 2>&1 || exit $?

timeout -k 10 400 python3 tools/probe_walk_vs_chain.py 64 > gpurun_out/walk_vs_chain.jsonl 2>&1 || exit $?
echo done
