#!/bin/bash
# round 6: per-config rocprofv3 passes, second half
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/prof_all.sh PACKBITS ASTYPE BLOSC_S BLOSC_B FSO_LE FSO_BE DF4_LE DF4_BE DI2_BE 2>&1 | tee gpurun_out/prof_all_b.log | cut -c1-120
