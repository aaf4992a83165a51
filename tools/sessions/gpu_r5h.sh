#!/bin/bash
# round 5: full GPU suite, smoke, bench, noise decode timings
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5h_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5h_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5h_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r5h_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r5h_bench.json 2> gpurun_out/r5h_bench.err
rc=$?; tail -1 gpurun_out/r5h_bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for t in f4 f8; do
  KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py $t 256 quick > gpurun_out/walk_${t}_randn_r5h.json 2>&1
  rc=$?; tail -1 gpurun_out/walk_${t}_randn_r5h.json; [ $rc -eq 0 ] || exit $rc
done
