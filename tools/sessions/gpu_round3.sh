#!/usr/bin/env bash
# Round-3 measurement pass: checksum parity subset, CRC fold A/B + grid
# sweep, CRC verify kernel trace, float Delta walker families, single-chunk
# verify overhead, every codec through its public API.  Each step under its
# own limit; stops at the first crash / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.out"; grep -v amdgpu.ids "gpurun_out/$name.err" | tail -3
  case $rc in 0|1) ;; *) echo "fatal rc=$rc in $name; stopping"; exit $rc;; esac
}
for step in "$@"; do
  case $step in
    cktests) run crc_tests 600 python -u -m pytest tests/test_gpu_next.py tests/test_gpu_sched.py tests/test_gpu_chunks.py tests/test_gpu_codecs.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf ;;
    crcab) run probe_crc_bs 600 python -u tools/probe_crc_bs.py bitsliced lds_tables bs_grid256 bs_grid768 bs_grid1024 bs_grid2048 bs_k8 bs_kcopy16 ;;
    crckt) run crc_kt 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crc_kt -o run -- python3 tools/probe_crc_verify.py crc32 ;;
    walk) run probe_walk_f4 500 python -u tools/probe_fspec_walk.py f4 256 quick ;;
    walkb) run probe_walk_f4_batch 600 python -u tools/probe_fspec_walk.py f4 16 ;;
    verify) run probe_verify_overhead 200 python -u tools/probe_verify_overhead.py ;;
    all) run probe_all 500 python -u tools/probe_all.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
