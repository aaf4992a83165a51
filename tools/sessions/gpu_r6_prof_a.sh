#!/bin/bash
# round 6: per-config rocprofv3 passes (kernel trace, FETCH_SIZE, WRITE_SIZE), first half
set -u
cd "${GRAFT_REPO_ROOT}"
bash tools/prof_all.sh C2_f32 C2_f64 C3 C4 C5 D_i2 F32 CRC32 CRC32C ADLER32 2>&1 | tee gpurun_out/prof_all_a.log | cut -c1-120
