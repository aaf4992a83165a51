#!/bin/bash
# round 5: per-config rocprofv3 passes, second half, then the headline under rocprofv3 and the bench line
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
bash tools/prof_all.sh PACKBITS ASTYPE BLOSC_S BLOSC_B FSO_LE FSO_BE DF4_LE DF4_BE DI2_BE 2>&1 | tee gpurun_out/prof_all_b.log | cut -c1-120
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o bench -- python3 bench.py --no-cpu --quick --steps 50 --warmup 5 > gpurun_out/rocprof_headline.log 2>&1 || exit $?
grep -o '"mean_launch_ms": [0-9.]*' gpurun_out/rocprof_headline.log
