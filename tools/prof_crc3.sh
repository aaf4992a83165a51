#!/usr/bin/env bash
# CRC fold schedule sweep (aligned verify) + the table fold's aligned kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
MCODEC_CRC_LDS=1 NUMCODECS_AMD_LIB=tools/_build/libmcodec_lab.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt_c_lds -o run -- python3 tools/probe_crc_verify.py crc32c > gpurun_out/kt_c_lds.log 2>&1 || exit $?
timeout -k 10 800 python3 tools/probe_crc_bs.py bitsliced lds_tables bs_grid1024 bs_grid2048 bs_grid4096 bs_k8 bs_k8_grid768 bs_k8_grid1024 bs_k8_grid2048 bs_gridcopy512 bs_gridcopy768 bs_kcopy16_grid512 > gpurun_out/probe_crc_bs4.jsonl 2> gpurun_out/probe_crc_bs4.err || exit $?
echo done
