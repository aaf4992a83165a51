#!/usr/bin/env bash
# Compile the reference's own hot-path Cython extensions, from the sources
# where they lie under /root/reference, into oracle/_ref/ (git-ignored, and
# listed in .gpurunignore: it stays in this container and never reaches the GPU
# box).  Test infrastructure only: it pins the oracle restatement
# (tests/test_oracle.py), generates tests/golden/, and times the reference
# beside the restatement (tools/cpu_port_vs_ref.py).  bench.py's cpu_baseline
# times the restatement (oracle/ncoracle.c, kind "port"), not this build.
#
#   src/numcodecs/_shuffle.pyx    -> oracle/_ref/_shuffle.*.so   (_doShuffle/_doUnshuffle)
#   src/numcodecs/fletcher32.pyx  -> oracle/_ref/fletcher32.*.so (+ _utils.pxd)
#   src/numcodecs/jenkins.pyx     -> oracle/_ref/jenkins.*.so    (jenkins_lookup3)
#
# Flags follow the reference's release build (src/numcodecs/meson.build:245-254):
# plain -O3, no -march, -pthread.  Nothing is written outside oracle/_ref/.
set -euo pipefail
REF=${NUMCODECS_REF:-/root/reference}
SRC="$REF/src/numcodecs"
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUT="$HERE/_ref"
if [ ! -f "$SRC/_shuffle.pyx" ]; then
  echo "reference sources not present at $SRC; skipping oracle/_ref build" >&2
  exit 0
fi
mkdir -p "$OUT"
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
PY=${PYTHON:-python3}
EXT=$($PY -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
PYINC=$($PY -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
for mod in _shuffle fletcher32 jenkins; do
  if [ "$OUT/$mod$EXT" -nt "$SRC/$mod.pyx" ] 2>/dev/null; then continue; fi
  # -I $SRC/.. so `from ._utils cimport ...` resolves inside package numcodecs
  $PY -m cython -3 -I "$SRC/.." "$SRC/$mod.pyx" -o "$TMP/$mod.c"
  gcc -O3 -std=gnu11 -pthread -shared -fPIC -I"$PYINC" "$TMP/$mod.c" -o "$OUT/$mod$EXT"
done
echo "built: $(ls "$OUT"/*"$EXT")"
