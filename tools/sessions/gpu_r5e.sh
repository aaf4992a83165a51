#!/bin/bash
# round 5: streaming SGPR-chain lab sweep (group size x prefetch windows), then the product's randn decode
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_stream.py 64 > gpurun_out/probe_stream_r5f.jsonl 2>&1
rc=$?; cat gpurun_out/probe_stream_r5f.jsonl | cut -c1-200; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f4 256 quick > gpurun_out/walk_f4_randn_r5f.json 2>&1
rc=$?; tail -1 gpurun_out/walk_f4_randn_r5f.json; [ $rc -eq 0 ] || exit $rc
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f8 256 quick > gpurun_out/walk_f8_randn_r5f.json 2>&1
rc=$?; tail -1 gpurun_out/walk_f8_randn_r5f.json; exit $rc
