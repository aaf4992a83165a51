#!/usr/bin/env bash
# full GPU suite + smoke, then the round-3 checksum / walker measurements
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python3 tools/probe_walk_vs_chain.py 64 > gpurun_out/walk_vs_chain.jsonl 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt_32 -o run -- python3 tools/probe_crc_verify.py crc32 > gpurun_out/kt_32.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt_c -o run -- python3 tools/probe_crc_verify.py crc32c > gpurun_out/kt_c.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f32_kt -o run -- python3 tools/probe_ck_single.py > gpurun_out/kt_f32.log 2>&1 || exit $?

timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/crc_pmc_c -o run -- python3 tools/probe_crc_verify.py crc32c > gpurun_out/pmc_c.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/f32_pmc -o run -- python3 tools/probe_ck_single.py > gpurun_out/pmc_f32.log 2>&1 || exit $?
echo done
