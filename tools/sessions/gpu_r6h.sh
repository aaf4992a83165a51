#!/bin/bash
# round 6: the longdouble chain on the scalar unit: ld tests + throughput probe
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6h
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ld.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6h/ld_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6h/ld_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/probe_ld_chain.py > gpurun_out/r6h/probe_ld_chain.json 2> gpurun_out/r6h/ld.err || { tail gpurun_out/r6h/ld.err; exit 1; }
cat gpurun_out/r6h/probe_ld_chain.json
