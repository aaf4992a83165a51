# A/B of the Fletcher32 kernel knobs on one box (tools/probe_ck_decode.py)
# the MCODEC_* schedule variables act on the lab library only (tools/lab/lab_sched.hip)
export NUMCODECS_AMD_LIB="$(cd "$(dirname "$0")/.." && pwd)/_build/libmcodec_lab.so"
set -e
for env in "MCODEC_F32_SLICE_KB=64" "MCODEC_F32_SLICE_KB=32" "MCODEC_F32_SLICE_KB=16" "MCODEC_F32_SLICE_KB=8" "MCODEC_F32_SLICE_KB=16 MCODEC_F32_UNROLL=1" "MCODEC_F32_SLICE_KB=32 MCODEC_F32_UNROLL=8" "MCODEC_F32_SLICE_KB=64" "MCODEC_F32_SLICE_KB=32" "MCODEC_F32_SLICE_KB=16"; do
  env $env PROBE_ONLY=fletcher32 timeout -k 10 120 python tools/probe_ck_decode.py 2>/dev/null
done
