#!/bin/bash
# round 5: serial-chain floors (f32 + f64 lab kinds) and the product walker on noise
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_chain.py > gpurun_out/probe_chain_r5.jsonl 2>&1
rc=$?; echo "chain rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -m pytest -q --timeout 100 --timeout-method thread tests/test_gpu_lab_kernels.py > gpurun_out/lab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/lab_tests.log; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f4 256 quick > gpurun_out/walk_f4_randn_r5.json 2>&1
rc=$?; tail -2 gpurun_out/walk_f4_randn_r5.json; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f8 256 quick > gpurun_out/walk_f8_randn_r5.json 2>&1
rc=$?; tail -2 gpurun_out/walk_f8_randn_r5.json; exit $rc
