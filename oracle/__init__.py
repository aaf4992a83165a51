"""Parity oracle for numcodecs_amd -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this package, and only as the checker / the timed CPU baseline.
The product (numcodecs_amd/) never imports it; there is no CPU fallback.

Contents
--------
* ``ncoracle.c`` (built to ``_build/libncoracle.so``): C restatement of the
  reference's Cython loops -- _shuffle.pyx:11-30, fletcher32.pyx:24-57,
  jenkins.pyx:93-325 -- and of CRC-32C (checksum32.py:189-209 delegates it to
  the absent third-party google_crc32c/crc32c package; pinned by the
  reference's fixture/crc32c files).
* CRC32 / Adler32 (checksum32.py:95-130) are zlib.crc32 / zlib.adler32 in
  the reference; the oracle calls the same CPython zlib.
* ``nporacle``: numpy restatement of the numpy-expressed codecs --
  bitround.py:45-80, delta.py:52-83, quantize.py:60-82,
  fixedscaleoffset.py:83-113, astype.py:46-58, packbits.py:33-82.  Their arithmetic lives in numpy (pinned by the
  reference at numpy>=2, pyproject.toml:7,17; 2.2.6 here), so the restatement
  runs the same numpy ufunc loops and promotion rules.
* ``refload``: imports the real reference (sources under /root/reference plus
  the Cython extensions compiled from them into ``_ref/`` by build_ref.sh) to
  pin the restatement and to generate tests/golden/.  Available only where
  /root/reference exists (this container), never on the GPU box.

Pinning: tests/test_oracle.py checks the restatement against the reference's
own fixtures (fixture/{shuffle,delta,quantize,fixedscaleoffset,crc32,crc32c,
adler32,astype,packbits} copied into
tests/golden/reference_fixture/), its known-answer tests (test_shuffle.py:131-159,
test_fletcher32.py:25-48, test_fixedscaleoffset.py:39-55, the docstring
examples) and, here, against the real reference on random and edge inputs.
"""

from . import nporacle  # noqa: F401
from .nporacle import (  # noqa: F401
    adler32,
    astype_decode,
    astype_encode,
    checksum32_decode,
    checksum32_encode,
    crc32,
    crc32c,
    jenkins_encode,
    jenkins_lookup3,
    packbits_decode,
    packbits_encode,
    bitround_decode,
    bitround_encode,
    delta_decode,
    delta_encode,
    fletcher32,
    fletcher32_decode,
    fletcher32_encode,
    fso_decode,
    fso_encode,
    quantize_decode,
    quantize_encode,
    shuffle,
    unshuffle,
)
