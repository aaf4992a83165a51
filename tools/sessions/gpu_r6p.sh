#!/bin/bash
# round 6: one-launch against two-launch checksum encodes at 256 MiB, 4 rotating sets
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6p
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/probe_adler_encode.py > gpurun_out/r6p/probe_ck_encode_sets.jsonl 2> gpurun_out/r6p/enc.err || { tail gpurun_out/r6p/enc.err; exit 1; }
cat gpurun_out/r6p/probe_ck_encode_sets.jsonl
