#!/usr/bin/env bash
# Run a sequence of GPU steps on the box, each under its own time limit; stop
# at the first step that crashes, aborts or times out (exit 124/134/137/139),
# continue past ordinary test failures.  Usage: tools/gpu_session.sh STEP...
# where STEP is one of: tests, smoke, bench, benchq, benchprof, pmcall, multi, probe, t1p, p1p, prof1p, verify, rocprof, pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "fatal rc=$rc in $name; stopping"; exit $rc;; esac
  return 0
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 1200 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -rf ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchq) run bench_quick 600 python bench.py --no-cpu --quick ;;
    benchprof) run rocprof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_all -o bench -- python3 bench.py --no-cpu --steps 20 --warmup 5 ;;
    pmcall) run pmc_fetch_all 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
               -d gpurun_out/prof_fetch_all -o bench -- python3 bench.py --no-cpu --steps 5 --warmup 1
          run pmc_write_all 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
               -d gpurun_out/prof_write_all -o bench -- python3 bench.py --no-cpu --steps 5 --warmup 1 ;;
    multi) run bench_multi2 600 env MCODEC_BENCH_BACKEND=gloo python bench.py --gpus 2 --no-cpu --quick --steps 50 --warmup 5 ;;
    probe) run probe_enc4 600 python tools/probe_enc.py 4 ;;
    t1p) run pytest_scan1p 600 python -u -m pytest tests/test_gpu_scan1p.py tests/test_gpu_c4.py tests/test_gpu_delta.py tests/test_gpu_fullsize.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -rf ;;
    p1p) run probe_scan1p 300 python tools/probe_scan1p.py ;;
    verify) run probe_verify 300 python tools/probe_verify.py ;;
    prof1p) run rocprof_scan1p 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_scan1p -o scan -- python3 tools/probe_scan1p.py ;;
    rocprof) run rocprof_kt 600 rocprofv3 --kernel-trace --stats --output-format csv \
               -d gpurun_out/prof_kt -o bench -- python3 bench.py --no-cpu --quick --steps 50 --warmup 5 ;;
    pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
               -d gpurun_out/prof_fetch -o bench -- python3 bench.py --no-cpu --quick --steps 20 --warmup 2
         run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
               -d gpurun_out/prof_write -o bench -- python3 bench.py --no-cpu --quick --steps 20 --warmup 2 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
