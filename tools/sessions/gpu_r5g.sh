#!/bin/bash
# round 5: f8 noise decode, vector-fed chain (product) vs LDS-fed chain (variant .so), alternating
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for r in 1 2; do
  KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f8 256 quick > gpurun_out/walk_f8_vbc_$r.json 2>&1
  rc=$?; echo "vbc $r $(tail -1 gpurun_out/walk_f8_vbc_$r.json)"; [ $rc -eq 0 ] || exit $rc
  NUMCODECS_AMD_LIB=tools/_build/libmcodec.so KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f8 256 quick > gpurun_out/walk_f8_lds_$r.json 2>&1
  rc=$?; echo "lds $r $(tail -1 gpurun_out/walk_f8_lds_$r.json)"; [ $rc -eq 0 ] || exit $rc
done
KINDS=randn timeout -k 10 300 python -u tools/probe_fspec_walk.py f4 256 quick > gpurun_out/walk_f4_vbc.json 2>&1
rc=$?; echo "f4 vbc $(tail -1 gpurun_out/walk_f4_vbc.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_stream.py 64 > gpurun_out/probe_stream_r5i.jsonl 2>&1
rc=$?; cut -c1-200 gpurun_out/probe_stream_r5i.jsonl; exit $rc
