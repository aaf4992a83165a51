#!/usr/bin/env bash
# Run a sequence of GPU steps on the box, each under its own time limit; stop
# at the first step that crashes, aborts or times out (exit 124/134/137/139),
# continue past ordinary test failures.  Usage: tools/gpu_session.sh STEP...
# where STEP is one of: tests, smoke, bench, benchx, probe, rocprof, pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
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
    tests) run pytest_gpu 1200 python -m pytest tests -m gpu -q --timeout=900 -p no:cacheprovider -rf ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchx) run bench_extra 900 python bench.py --extra --no-cpu ;;
    probe) run probe_enc4 600 python tools/probe_enc.py 4 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
