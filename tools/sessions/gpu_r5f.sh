#!/bin/bash
# round 5: vector-fed chain (ser_chain_vbc) -- parity, noise decode timing, lab stream sweep
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_delta_walk.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_delta.py tests/test_gpu_nan_bits.py tests/test_gpu_ext_dtypes.py tests/test_gpu_lab_kernels.py > gpurun_out/r5f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5f_tests.log; [ $rc -eq 0 ] || exit $rc
for t in f4 f8; do
  KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py $t 256 quick > gpurun_out/walk_${t}_randn_r5f.json 2>&1
  rc=$?; tail -1 gpurun_out/walk_${t}_randn_r5f.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u tools/probe_stream.py 64 > gpurun_out/probe_stream_r5h.jsonl 2>&1
rc=$?; cut -c1-200 gpurun_out/probe_stream_r5h.jsonl; exit $rc
