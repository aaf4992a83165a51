#!/usr/bin/env bash
# round 4, session k: f2 chain as half adds (NaN groups redone exactly):
# float Delta tests, then the f2 / f4 walk probes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta.py tests/test_gpu_delta_walk.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_nan_bits.py tests/test_gpu_fuzz.py tests/test_gpu_chunks.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_k.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_k.log | tail -20; [ $rc -eq 0 ] || exit $rc
KINDS=smooth,sin4096,randwalk,randn timeout -k 10 400 python3 tools/probe_fspec_walk.py f2 256 quick > gpurun_out/probe_walk_f2.json 2> gpurun_out/probe_walk_f2.err || exit $?
cat gpurun_out/probe_walk_f2.json
KINDS=randn,smallamp timeout -k 10 300 python3 tools/probe_fspec_walk.py f4 256 quick > gpurun_out/probe_walk_f4b.json 2> gpurun_out/probe_walk_f4b.err || exit $?
cat gpurun_out/probe_walk_f4b.json
