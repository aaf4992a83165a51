# A/B of the checksum tuning knobs on one box (tools/probe_ck_decode.py)
set -e
for rep in 1 2; do
  for env in "MCODEC_F32_UNROLL=1" "MCODEC_F32_UNROLL=4" "MCODEC_CK_KCOPY=16 MCODEC_CK_GRID_COPY=2048" "MCODEC_CK_KCOPY=8 MCODEC_CK_GRID_COPY=1024" "MCODEC_CK_KCOPY=4 MCODEC_CK_GRID_COPY=100000"; do
    env $env timeout -k 10 120 python tools/probe_ck_decode.py 2>/dev/null
  done
done
