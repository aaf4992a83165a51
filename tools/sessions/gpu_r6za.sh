#!/bin/bash
# round 6: Fletcher32 one-launch verify on 2048 workgroups: checksum, fuzz and schedule tests, CRC profiles
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r6za
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_next.py tests/test_gpu_codecs.py tests/test_gpu_fuzz.py tests/test_gpu_sched.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r6za/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6za/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_all.sh F32 2>&1 | tee gpurun_out/r6za/prof_crc.log | cut -c1-120
