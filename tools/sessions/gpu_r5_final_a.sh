#!/bin/bash
# round 5, final tree part A: the whole GPU suite, smoke(), the driver's default bench line, the headline under rocprofv3
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu_final.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu_final.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 500 python3 bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -c 600 gpurun_out/bench_final.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o bench -- python3 bench.py --no-cpu --quick --steps 50 --warmup 5 > gpurun_out/rocprof_headline.log 2>&1 || exit $?
grep -o '"mean_launch_ms": [0-9.]*' gpurun_out/rocprof_headline.log
