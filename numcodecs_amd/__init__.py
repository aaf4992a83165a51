"""numcodecs_amd -- numcodecs' per-element filter codecs and Fletcher32 on AMD
Instinct MI355X (gfx950).

A drop-in for the hot path of zarr-developers/numcodecs: the codecs
Shuffle, BitRound, Delta, Quantize, FixedScaleOffset and Fletcher32 (plus the
next-row codecs CRC32, CRC32C, Adler32, JenkinsLookup3, AsType and PackBits)
with the same ids, configs, reprs and error behaviour, executed by hand-written HIP
kernels (libmcodec.so, C ABI in include/mcodec.h) on device-resident chunks.
Device tensors stay on the device; host buffers are staged through it.

Reference registrations: src/numcodecs/__init__.py:74,78,82,102,106,127
(the six hot-path codecs), :68-70 AsType, :84-86 PackBits, :108-112 CRC32 /
Adler32 / JenkinsLookup3, :141-143 CRC32C.
"""

from .abc import Codec
from .errors import UnknownCodecError
from .registry import codec_registry, get_codec, register_codec

from .delta import Delta

register_codec(Delta)

from .quantize import Quantize

register_codec(Quantize)

from .fixedscaleoffset import FixedScaleOffset

register_codec(FixedScaleOffset)

from .shuffle import Shuffle

register_codec(Shuffle)

from .bitround import BitRound

register_codec(BitRound)

from .fletcher32 import Fletcher32

register_codec(Fletcher32)

from .checksum32 import CRC32, CRC32C, Adler32, JenkinsLookup3

register_codec(CRC32)
register_codec(CRC32C)
register_codec(Adler32)
register_codec(JenkinsLookup3)

from .astype import AsType

register_codec(AsType)

from .packbits import PackBits

register_codec(PackBits)

from . import batch  # noqa: E402,F401
from . import blosc_shuffle  # noqa: E402,F401  (Blosc's per-block shuffle filters)
from . import chunks  # noqa: E402,F401  (Zarr-style batched / host-streamed chunk pipelines)
from . import graphs  # noqa: E402,F401  (HIP-graph captured chunk pipelines)

__version__ = "0.1.0"

__all__ = [
    "Adler32",
    "AsType",
    "BitRound",
    "CRC32",
    "CRC32C",
    "JenkinsLookup3",
    "PackBits",
    "Codec",
    "Delta",
    "FixedScaleOffset",
    "Fletcher32",
    "Quantize",
    "Shuffle",
    "UnknownCodecError",
    "batch",
    "blosc_shuffle",
    "chunks",
    "graphs",
    "codec_registry",
    "get_codec",
    "register_codec",
]


def _register_virtual_subclass():
    """Make every numcodecs_amd codec an instance of ``numcodecs.abc.Codec``
    (reference: src/numcodecs/abc.py:33, an ``ABC``) by registering our base
    class as a virtual subclass, so callers that type-check their filters
    (Zarr's numcodecs wrappers, zarr3.py:16-31) accept these codecs.  Returns
    True when numcodecs' ABC was found."""
    try:
        from numcodecs.abc import Codec as _NcCodec
    except Exception:
        return False
    if not issubclass(Codec, _NcCodec):
        _NcCodec.register(Codec)
    return True


_register_virtual_subclass()


def register_with_numcodecs():
    """Register these classes into an installed ``numcodecs`` registry
    (replacing the CPU implementations under the same ids), and make them
    virtual subclasses of ``numcodecs.abc.Codec``.  Returns the list of ids
    registered, or [] when numcodecs is not importable."""
    try:
        import numcodecs  # noqa: F401
        from numcodecs.registry import register_codec as _nc_register
    except Exception:
        return []
    _register_virtual_subclass()
    ids = []
    for cls in (Delta, Quantize, FixedScaleOffset, Shuffle, BitRound, Fletcher32, CRC32, CRC32C,
                Adler32, JenkinsLookup3, AsType, PackBits):
        _nc_register(cls)
        ids.append(cls.codec_id)
    return ids
