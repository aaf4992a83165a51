#!/bin/bash
# round 5: bitshuffle decode with the plane stride opaque per tile (no hoisted
# SGPR offsets): next-rows tests, then A/B of HEAD / w-image / direct-LDS ES8
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r5u
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_next.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5u/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5u/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base d0 prod; do
  if [ $v = prod ]; then lib=numcodecs_amd/_lib/libmcodec.so; else lib=tools/_build/$v/libmcodec.so; fi
  echo "== $v" >> gpurun_out/r5u/probe.jsonl
  NUMCODECS_AMD_LIB=$lib timeout -k 10 180 python3 -u tools/probe_bshuf_all.py >> gpurun_out/r5u/probe.jsonl 2>&1
  rc=$?; [ $rc -eq 0 ] || { cat gpurun_out/r5u/probe.jsonl; exit $rc; }
done
cat gpurun_out/r5u/probe.jsonl
