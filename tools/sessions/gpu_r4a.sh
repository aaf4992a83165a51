#!/usr/bin/env bash
# round 4, first GPU session: full GPU suite on the current tree, then the
# Shuffle(4) encode schedule probe (tools/probe_enc4_lab.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe_enc4_lab.py 5 > gpurun_out/probe_enc4_lab.log 2>&1 || exit $?
tail -40 gpurun_out/probe_enc4_lab.log
