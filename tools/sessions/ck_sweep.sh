# the MCODEC_* schedule variables act on the lab library only (tools/lab/lab_sched.hip)
export NUMCODECS_AMD_LIB="$(cd "$(dirname "$0")/.." && pwd)/_build/libmcodec_lab.so"
set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 600 python -m pytest tests/test_gpu_next.py -q -m gpu -x -p no:cacheprovider > gpurun_out/next.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/next.log; exit 1; }
tail -2 gpurun_out/next.log
for K in 4 8 16; do for G in 1024 2048 4096 1000000; do
  MCODEC_CK_K=$K MCODEC_CK_GRID=$G timeout -k 10 120 python tools/probe_ck.py >> gpurun_out/probe_ck.jsonl 2>/dev/null || { echo "probe failed rc=$?"; exit 1; }
done; done
cat gpurun_out/probe_ck.jsonl
# the checksum rows of the driver's line: bench.py's cfg_next block (default run, N = 1)
timeout -k 10 400 python bench.py --no-cpu --steps 5 > gpurun_out/bench_next.log 2>&1; tail -1 gpurun_out/bench_next.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['cfg_next'])"
