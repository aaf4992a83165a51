"""Import the real reference hot path -- TEST INFRASTRUCTURE ONLY.

Builds a ``numcodecs`` package object whose search path is the reference's
own source directory (/root/reference/src/numcodecs) plus oracle/_ref/ (the
reference's Cython extensions compiled from those sources by build_ref.sh),
without executing the reference's ``__init__.py`` (which needs Blosc/Zstd/LZ4,
not buildable here: the c-blosc submodule is empty).  The six hot-path codecs
are then registered into the reference's own registry, as its __init__.py
does at lines 74, 78, 82, 102, 106 and 127.

Used only in this container (where /root/reference exists) to pin the oracle
and to generate tests/golden/.  Never used on the GPU box.
"""

from __future__ import annotations

import importlib
import os
import sys
import types

REF_SRC = os.environ.get("NUMCODECS_REF_SRC", "/root/reference/src/numcodecs")
_HERE = os.path.dirname(os.path.abspath(__file__))
REF_BUILD = os.path.join(_HERE, "_ref")


def available() -> bool:
    return os.path.isfile(os.path.join(REF_SRC, "shuffle.py")) and os.path.isdir(REF_BUILD) and any(
        f.startswith("_shuffle") and f.endswith(".so") for f in os.listdir(REF_BUILD)
    )


def load():
    """Return the reference ``numcodecs`` package namespace (hot path only)."""
    if "numcodecs" in sys.modules and getattr(sys.modules["numcodecs"], "_graft_ref", False):
        return sys.modules["numcodecs"]
    if not available():
        raise ImportError("reference sources or oracle/_ref build not available")
    pkg = types.ModuleType("numcodecs")
    pkg.__path__ = [REF_SRC, REF_BUILD]
    pkg.__file__ = os.path.join(REF_SRC, "__init__.py")
    pkg._graft_ref = True
    sys.modules["numcodecs"] = pkg
    registry = importlib.import_module("numcodecs.registry")
    pkg.get_codec = registry.get_codec
    pkg.register_codec = registry.register_codec
    for modname, clsname in [
        ("delta", "Delta"),
        ("quantize", "Quantize"),
        ("fixedscaleoffset", "FixedScaleOffset"),
        ("shuffle", "Shuffle"),
        ("bitround", "BitRound"),
        ("fletcher32", "Fletcher32"),
        ("astype", "AsType"),
        ("packbits", "PackBits"),
    ]:
        mod = importlib.import_module(f"numcodecs.{modname}")
        cls = getattr(mod, clsname)
        setattr(pkg, clsname, cls)
        registry.register_codec(cls)
    # checksum32.py needs Python >= 3.12 (collections.abc.Buffer, its
    # pyproject.toml:18 pin) and is not importable on this 3.10; its checksums
    # are zlib.crc32 / zlib.adler32 and the compiled jenkins.pyx, which the
    # oracle uses directly, and its framing is pinned by fixture/{crc32,
    # adler32,crc32c}.
    try:
        pkg.jenkins_lookup3 = importlib.import_module("numcodecs.jenkins").jenkins_lookup3
    except ImportError:
        pass
    return pkg
