#!/usr/bin/env bash
# round-end refresh, part A: full GPU suite, smoke, per-config rocprof + PMC
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
bash tools/prof_all.sh > gpurun_out/prof_all.log 2>&1 || exit $?
tail -2 gpurun_out/prof_all.log
echo done
