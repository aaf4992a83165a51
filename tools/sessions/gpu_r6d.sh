#!/bin/bash
# round 6: float Delta decode schedules A/B (tools/probe_fspec_fold.py), DF4 kernel trace, spec tests
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_delta_spec.py tests/test_gpu_delta_spec2.py tests/test_gpu_delta_walk.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6d/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r6d/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/probe_fspec_fold.py 7 > gpurun_out/r6d/probe_fspec_fold.json 2>gpurun_out/r6d/probe.err || { tail gpurun_out/r6d/probe.err; exit 1; }
cat gpurun_out/r6d/probe_fspec_fold.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6d/kt_DF4_LE -o run -- python3 tools/prof_configs.py DF4_LE dec > gpurun_out/r6d/kt.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r6d/kt_DF4_LE/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print({k: (round(sum(v) / len(v), 2), len(v)) for k, v in acc.items() if "fspec" in k})
PY
