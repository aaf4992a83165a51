#!/bin/bash
# round 5: SGPR-fed walker chain -- parity, then noise decode timing; es8 LDS layout; CRC / bitshuffle probe
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_delta_walk.py tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_delta.py tests/test_gpu_nan_bits.py tests/test_gpu_ext_dtypes.py tests/test_gpu_next.py > gpurun_out/r5c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5c_tests.log; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f4 256 quick > gpurun_out/walk_f4_randn_r5c.json 2>&1
rc=$?; tail -1 gpurun_out/walk_f4_randn_r5c.json; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f8 256 quick > gpurun_out/walk_f8_randn_r5c.json 2>&1
rc=$?; tail -1 gpurun_out/walk_f8_randn_r5c.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe_r5.py > gpurun_out/probe_r5c.jsonl 2>&1
rc=$?; grep probe gpurun_out/probe_r5c.jsonl; [ $rc -eq 0 ] || exit $rc
ONLY=shuf_es8 timeout -k 10 300 python -u tools/probe_enc_variants.py 3 > gpurun_out/probe_enc_es8_r5c.log 2>&1
rc=$?; grep -E "bad|variant\": (5|7|23|135|15)," gpurun_out/probe_enc_es8_r5c.log | tail -12; exit $rc
