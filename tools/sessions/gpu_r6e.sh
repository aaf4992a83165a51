#!/bin/bash
# round 6 (lab library shipped for this call): every lab schedule vs the oracle (incl. br_planes = 0),
# the C3 plane-masked encode A/B, and its SQ counters / effective clock beside the element-masked kernel
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sched.py tests/test_gpu_lab_kernels.py -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r6e/lab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6e/lab_tests.log; [ $rc -eq 0 ] || exit $rc
NUMCODECS_AMD_LIB=tools/_build/libmcodec_lab.so timeout -k 10 180 python3 tools/probe_c3_planes.py > gpurun_out/r6e/probe_c3_planes.json 2> gpurun_out/r6e/probe.err || { tail gpurun_out/r6e/probe.err; exit 1; }
cat gpurun_out/r6e/probe_c3_planes.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6e/kt_C3 -o run -- python3 tools/prof_configs.py C3 enc > gpurun_out/r6e/kt_C3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r6e/pmc_C3 -o run -- python3 tools/prof_configs.py C3 enc > gpurun_out/r6e/pmc_C3.log 2>&1 || exit $?
python3 tools/pmc_table.py gpurun_out/r6e/kt_C3 gpurun_out/r6e/pmc_C3 k_bitround_shuffle4_planes
