#!/usr/bin/env bash
# round 4, session c: chain schedule probe (rotating register sets), headline
# rocprof kernel stats, per-config rocprof passes (first half of the configs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/probe_chain.py > gpurun_out/probe_chain.log 2>&1 || exit $?
grep '"round": 2' gpurun_out/probe_chain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o bench -- python3 bench.py --no-cpu --quick --steps 50 --warmup 5 > gpurun_out/rocprof_headline.log 2>&1 || exit $?
tail -c 600 gpurun_out/rocprof_headline.log
bash tools/prof_all.sh ${PROF_CONFIGS:-C2_f32 C2_f64 C3 C4 C5 D_i2 F32 CRC32 CRC32C ADLER32}
