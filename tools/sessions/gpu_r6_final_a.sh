#!/bin/bash
# round 6, final tree part A: the whole GPU suite, smoke(), the driver's default bench line, the headline under rocprofv3
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/final/pytest_gpu.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/final/bench_default.log 2>&1 || { tail -20 gpurun_out/final/bench_default.log; exit 1; }
tail -c 400 gpurun_out/final/bench_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_kt -o bench -- python3 bench.py --no-cpu --quick --steps 50 --warmup 5 > gpurun_out/final/rocprof_headline.log 2>&1 || exit $?
grep -o '"mean_launch_ms": [0-9.]*' gpurun_out/final/rocprof_headline.log
