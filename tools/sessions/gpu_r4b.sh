#!/usr/bin/env bash
# round 4, session b: GPU suite (byte order, 8x tiles), chain probe, tile probe, default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_byteorder.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_bo.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_bo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/probe_chain.py > gpurun_out/probe_chain.log 2>&1 || exit $?
tail -5 gpurun_out/probe_chain.log
timeout -k 10 300 python -u tools/probe_shuffle_tiles.py 4 > gpurun_out/probe_shuffle_tiles.log 2>&1 || exit $?
grep -E "v129|v513|mc_copy|copy_u|bad|failures" gpurun_out/probe_shuffle_tiles.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || exit $?
tail -c 3000 gpurun_out/bench_default.log
timeout -k 10 120 python -u tools/probe_verify_overhead.py > gpurun_out/probe_verify_overhead.log 2>&1 || exit $?
cat gpurun_out/probe_verify_overhead.log
