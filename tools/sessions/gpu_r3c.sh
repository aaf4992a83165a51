#!/usr/bin/env bash
# checkpoint: full GPU suite, smoke, walker vs chain, public-API table, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python3 tools/probe_walk_vs_chain.py 64 > gpurun_out/walk_vs_chain.jsonl 2>&1 || exit $?
timeout -k 10 500 python3 tools/probe_all.py > gpurun_out/probe_all4.jsonl 2> gpurun_out/probe_all4.err || exit $?
timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -c 400 gpurun_out/bench.log
echo done
