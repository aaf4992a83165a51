#!/usr/bin/env bash
# rocprofv3 kernel traces and PMC passes of the CRC32 256 MiB verify: the
# product (bit-sliced fold) and, on the lab library, the LDS-table fold.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LAB=tools/_build/libmcodec_lab.so
step() { echo "== $1"; shift; "$@"; local rc=$?; echo "rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
step kt_bs timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt_bs -o run -- python3 tools/probe_crc_verify.py crc32
MCODEC_CRC_LDS=1 NUMCODECS_AMD_LIB=$LAB step kt_lds timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt_lds -o run -- python3 tools/probe_crc_verify.py crc32
step kt_bs_enc timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt_bs_enc -o run -- python3 tools/probe_crc_verify.py crc32 encode
step pmc1_bs timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/crc_pmc1_bs -o run -- python3 tools/probe_crc_verify.py crc32
step pmc2_bs timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/crc_pmc2_bs -o run -- python3 tools/probe_crc_verify.py crc32
MCODEC_CRC_LDS=1 NUMCODECS_AMD_LIB=$LAB step pmc1_lds timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/crc_pmc1_lds -o run -- python3 tools/probe_crc_verify.py crc32
MCODEC_CRC_LDS=1 NUMCODECS_AMD_LIB=$LAB step pmc2_lds timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/crc_pmc2_lds -o run -- python3 tools/probe_crc_verify.py crc32
step ab timeout -k 10 400 python3 tools/probe_crc_bs.py
