#!/bin/bash
# round 6: the float Delta decode with the tile-prefix scan folded into the reduce pass:
# the speculative / walker / ld suites, then the DF4 / DF8 config profiles
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_delta_walk.py tests/test_gpu_delta.py tests/test_gpu_graphs.py tests/test_gpu_chunks.py tests/test_gpu_ld.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r6c/tests.log 2>&1; rc=$?
tail -5 gpurun_out/r6c/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in DF4_LE DF4_BE; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6c/kt_${cfg} -o run -- python3 tools/prof_configs.py $cfg dec > gpurun_out/r6c/kt_${cfg}.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
for cfg in ("DF4_LE", "DF4_BE"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r6c/kt_{cfg}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(cfg, {k: (round(sum(v) / len(v), 2), len(v)) for k, v in acc.items() if "fspec" in k})
PY
for cfg in "C3 enc" "C2_f32 enc"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6c/kt_$1_$2 -o run -- python3 tools/prof_configs.py $1 $2 > gpurun_out/r6c/kt_$1_$2.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
for cfg in ("C3_enc", "C2_f32_enc"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r6c/kt_{cfg}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(cfg, {k: (round(sum(v) / len(v), 2), len(v)) for k, v in acc.items() if "shuffle" in k})
PY
