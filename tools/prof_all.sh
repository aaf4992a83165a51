#!/usr/bin/env bash
# Per-config rocprofv3 passes on the GPU box (one process per config and
# direction; kernel trace, then FETCH_SIZE and WRITE_SIZE in passes of their
# own).  Usage: tools/prof_all.sh [CONFIG...]   (default: every config)
# Then, in the build container: python tools/prof_summary.py r02
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
CONFIGS=${*:-"C2_f32 C2_f64 C3 C4 C5 D_i2 F32 CRC32 CRC32C ADLER32 PACKBITS ASTYPE BLOSC_S BLOSC_B FSO_LE FSO_BE DF4_LE DF4_BE DI2_BE"}
for cfg in $CONFIGS; do
  for dir in enc dec; do
    key="${cfg}_${dir}"
    timeout -k 10 120 python3 tools/prof_configs.py "$cfg" "$dir" > "gpurun_out/prof/${key}_meta.json" \
      2> "gpurun_out/prof/${key}_meta.err" || { echo "FAIL $key rc=$?"; exit 1; }
    timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/prof/${key}_kt" -o p \
      -- python3 tools/prof_configs.py "$cfg" "$dir" > /dev/null 2>&1 || { echo "FAIL kt $key rc=$?"; exit 1; }
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
      -d "gpurun_out/prof/${key}_fetch" -o p -- python3 tools/prof_configs.py "$cfg" "$dir" > /dev/null 2>&1 \
      || { echo "FAIL fetch $key rc=$?"; exit 1; }
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
      -d "gpurun_out/prof/${key}_write" -o p -- python3 tools/prof_configs.py "$cfg" "$dir" > /dev/null 2>&1 \
      || { echo "FAIL write $key rc=$?"; exit 1; }
    echo "ok $key $(cat gpurun_out/prof/${key}_meta.json)"
  done
done
