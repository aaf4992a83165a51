# the MCODEC_* schedule variables act on the lab library only (tools/lab/lab_sched.hip)
export NUMCODECS_AMD_LIB="$(cd "$(dirname "$0")/.." && pwd)/_build/libmcodec_lab.so"
set -e
for env in "MCODEC_COPY_U=4 MCODEC_COPY_GRID=8192" "MCODEC_COPY_U=8 MCODEC_COPY_GRID=8192" "MCODEC_COPY_U=4 MCODEC_COPY_GRID=0" "MCODEC_COPY_U=8 MCODEC_COPY_GRID=0" "MCODEC_COPY_U=4 MCODEC_COPY_GRID=2048" "MCODEC_COPY_U=4 MCODEC_COPY_GRID=4096" "MCODEC_COPY_U=4 MCODEC_COPY_GRID=8192"; do
  env $env timeout -k 10 120 python tools/probe_copy.py 2>/dev/null
done
