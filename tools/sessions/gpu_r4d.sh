#!/usr/bin/env bash
# round 4, session d: chain schedule probe (SGPR-fed inputs, global stores),
# per-config rocprof passes (second half of the configs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/probe_chain.py > gpurun_out/probe_chain.log 2>&1 || exit $?
grep -E '"round": 2|correctness' gpurun_out/probe_chain.log
bash tools/prof_all.sh ${PROF_CONFIGS:-PACKBITS ASTYPE BLOSC_S BLOSC_B FSO_LE FSO_BE DF4_LE DF4_BE DI2_BE}
