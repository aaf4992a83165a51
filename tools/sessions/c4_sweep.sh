set -u
cd "${GRAFT_REPO_ROOT}"
for v in 0 2 3; do
  timeout -k 10 120 python tools/probe_c4.py 67108864 $v >> gpurun_out/probe_c4.jsonl 2>&1 || { echo "variant $v failed rc=$?"; exit 1; }
done
timeout -k 10 120 python tools/probe_c4.py 1048576 4 >> gpurun_out/probe_c4.jsonl 2>&1 || { echo "variant 4 failed"; exit 1; }
timeout -k 10 120 python tools/probe_c4.py 1000000 3 >> gpurun_out/probe_c4.jsonl 2>&1 || { echo "variant 3 small failed"; exit 1; }
cat gpurun_out/probe_c4.jsonl
