#!/usr/bin/env bash
# round 4, session f: chain probe (all-lane lagging stores), elementwise
# configs after the x86 NaN rule (FSO, C4, Quantize/AsType)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/probe_chain.py > gpurun_out/probe_chain.log 2>&1 || exit $?
grep -E '"round": 2|correctness' gpurun_out/probe_chain.log
rm -rf gpurun_out/prof
bash tools/prof_all.sh ${PROF_CONFIGS:-FSO_LE FSO_BE C4 ASTYPE}
