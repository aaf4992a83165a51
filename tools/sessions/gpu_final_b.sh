#!/usr/bin/env bash
# round-end refresh, part B: headline rocprof, public-API table, walker
# families, verify overhead, the driver-contract bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o bench -- python3 bench.py --no-cpu --quick --steps 50 --warmup 5 > gpurun_out/rocprof_headline.log 2>&1 || exit $?
timeout -k 10 400 python3 tools/probe_all.py > gpurun_out/probe_all_final.jsonl 2> gpurun_out/probe_all_final.err || exit $?
timeout -k 10 300 python3 tools/probe_fspec_walk.py f4 256 quick > gpurun_out/probe_walk_final.json 2> gpurun_out/probe_walk_final.err || exit $?
timeout -k 10 200 python3 tools/probe_verify_overhead.py > gpurun_out/probe_verify_overhead_final.json 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/bench_final.log 2>&1 || exit $?
tail -c 300 gpurun_out/bench_final.log
echo done
