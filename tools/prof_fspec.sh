#!/usr/bin/env bash
# float Delta decode after a change to its scans: parity, kernel traces of the
# smooth 256 MiB decode, walker families
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_delta_walk.py tests/test_gpu_delta.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/fspec_tests.log 2>&1; rc=$?; tail -2 gpurun_out/fspec_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fspec_kt -o run -- python3 tools/probe_fspec_walk.py f4 256 quick > gpurun_out/fspec_walk.out 2> gpurun_out/fspec_walk.err || exit $?
tail -1 gpurun_out/fspec_walk.out
timeout -k 10 300 python3 tools/probe_fspec2.py > gpurun_out/fspec2.out 2> gpurun_out/fspec2.err || exit $?
tail -2 gpurun_out/fspec2.out
echo done
