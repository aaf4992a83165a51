#!/bin/bash
# round 6: stamped one-launch CRC verify (where the finish goes) + the copy calibration library
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6i
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/probe_ck_stamp.py > gpurun_out/r6i/probe_ck_stamp.jsonl 2> gpurun_out/r6i/stamp.err || { tail gpurun_out/r6i/stamp.err; exit 1; }
cat gpurun_out/r6i/probe_ck_stamp.jsonl
timeout -k 10 300 python3 -c "
import json, torch, bench
print(json.dumps(bench.copy_ceiling(torch.device('cuda:0'))))
" > gpurun_out/r6i/copy_ceiling.json 2> gpurun_out/r6i/copy.err || { tail gpurun_out/r6i/copy.err; exit 1; }
cat gpurun_out/r6i/copy_ceiling.json
