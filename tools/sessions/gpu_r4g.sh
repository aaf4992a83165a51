#!/usr/bin/env bash
# round 4, session g: chain lane stores straight to dst (walker stream and
# k_scan_serial): float Delta GPU tests, then the walk probe (f4 and f8)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_delta_walk.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_chunks.py tests/test_gpu_byteorder.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_g.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_g.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/probe_fspec_walk.py f4 256 > gpurun_out/probe_walk_f4.json 2> gpurun_out/probe_walk_f4.err || exit $?
tail -c 1500 gpurun_out/probe_walk_f4.json
timeout -k 10 300 python3 tools/probe_fspec_walk.py f8 256 quick > gpurun_out/probe_walk_f8.json 2> gpurun_out/probe_walk_f8.err || exit $?
tail -c 800 gpurun_out/probe_walk_f8.json
