#!/bin/bash
# round 5: bitshuffle kernels -- kernel trace, then SQ and TA/TCP counter passes
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/bsh
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/bsh/trace -o run -- python3 tools/probe_bshuf.py 5 > gpurun_out/bsh/trace.log 2>&1
rc=$?; tail -1 gpurun_out/bsh/trace.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d gpurun_out/bsh/pmc1 -o run -- python3 tools/probe_bshuf.py 2 > gpurun_out/bsh/pmc1.log 2>&1
rc=$?; tail -1 gpurun_out/bsh/pmc1.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE -d gpurun_out/bsh/pmc2 -o run -- python3 tools/probe_bshuf.py 2 > gpurun_out/bsh/pmc2.log 2>&1
rc=$?; tail -1 gpurun_out/bsh/pmc2.log; exit $rc
