set -u
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 120 python tools/probe_c4.py 67108864 1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 tools/probe_c4.py > gpurun_out/prof_c4.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_c4/**/c4_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:90], r["Calls"], r["AverageNs"])
PY
