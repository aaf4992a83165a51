#!/bin/bash
# round 6: whole GPU suite on the current tree, longdouble throughput, C3 / C2 / DF4 config profiles
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6g
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r6g/pytest_gpu.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed" gpurun_out/r6g/pytest_gpu.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/probe_ld_chain.py > gpurun_out/r6g/probe_ld_chain.json 2> gpurun_out/r6g/ld.err || { tail gpurun_out/r6g/ld.err; exit 1; }
cat gpurun_out/r6g/probe_ld_chain.json
bash tools/prof_all.sh C3 C2_f32 DF4_LE 2>&1 | tail -6
