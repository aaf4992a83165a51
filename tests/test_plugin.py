"""The plugin side of the drop-in boundary (CPU only, no kernels):

* entry-point discovery in the ``numcodecs.codecs`` group, as the reference's
  own plugin test does with a fake installed package
  (tests/test_entrypoints.py:11-24, tests/package_with_entrypoint/);
* codecs are stateless and picklable (the reference's multiprocessing tests
  ship them to workers, test_shuffle.py:90-109);
* ``register_with_numcodecs()`` replaces the CPU classes inside the real
  numcodecs registry (registry.py:57-74), checked against the reference
  package itself where it is importable (this container).
"""

import pickle
import sys
import textwrap

import pytest

import numcodecs_amd
from numcodecs_amd import registry

CODECS = [
    numcodecs_amd.Shuffle(4),
    numcodecs_amd.BitRound(10),
    numcodecs_amd.Delta("<i2", "<i1"),
    numcodecs_amd.Quantize(3, "<f8", "<f4"),
    numcodecs_amd.FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"),
    numcodecs_amd.Fletcher32(),
    numcodecs_amd.CRC32(location="end"),
    numcodecs_amd.Adler32(),
    numcodecs_amd.JenkinsLookup3(initval=7),  # (with a prefix, == raises in the reference too)
    numcodecs_amd.AsType("<f4", "<f8"),
    numcodecs_amd.PackBits(),
]


@pytest.mark.parametrize("codec", CODECS, ids=lambda c: c.codec_id)
def test_codec_pickles(codec):
    back = pickle.loads(pickle.dumps(codec))
    assert back == codec
    assert back.get_config() == codec.get_config()


def test_entry_point_plugin(tmp_path, monkeypatch):
    pkg = tmp_path / "package_with_entrypoint"
    pkg.mkdir()
    (pkg / "__init__.py").write_text(textwrap.dedent('''
        from numcodecs_amd.abc import Codec

        class TestCodec(Codec):
            codec_id = "test"

            def encode(self, buf):
                return buf

            def decode(self, buf, out=None):
                return buf
    '''))
    dist = tmp_path / "package_with_entrypoint-0.1.dist-info"
    dist.mkdir()
    (dist / "METADATA").write_text("Metadata-Version: 2.1\nName: package_with_entrypoint\nVersion: 0.1\n")
    (dist / "entry_points.txt").write_text("[numcodecs.codecs]\ntest = package_with_entrypoint:TestCodec\n")
    monkeypatch.syspath_prepend(str(tmp_path))
    try:
        registry.run_entrypoints()
        codec = numcodecs_amd.get_codec({"id": "test"})
        assert type(codec).__name__ == "TestCodec"
        assert registry.codec_registry["test"] is type(codec)  # loaded once, then registered
    finally:
        registry.codec_registry.pop("test", None)
        sys.modules.pop("package_with_entrypoint", None)
        monkeypatch.undo()
        registry.run_entrypoints()
    with pytest.raises(numcodecs_amd.UnknownCodecError):
        numcodecs_amd.get_codec({"id": "test"})


def test_register_with_reference_numcodecs():
    try:
        from oracle import refload
    except ImportError:  # the reference loader stays in the build container (.gpurunignore)
        pytest.skip("reference loader not present (GPU box)")
    if not refload.available():
        pytest.skip("reference sources not present (GPU box)")
    ref = refload.load()
    originals = {cid: ref.registry.codec_registry[cid] for cid in ("shuffle", "delta", "fletcher32", "bitround")}
    try:
        ids = numcodecs_amd.register_with_numcodecs()
        assert {"shuffle", "bitround", "delta", "quantize", "fixedscaleoffset", "fletcher32"} <= set(ids)
        codec = ref.get_codec({"id": "shuffle", "elementsize": 4})
        assert isinstance(codec, numcodecs_amd.Shuffle)
        # a config written by the reference codec resolves to the same codec here
        assert ref.get_codec(originals["delta"]("<i4").get_config()) == numcodecs_amd.Delta("<i4")
    finally:
        for cid, cls in originals.items():
            ref.registry.register_codec(cls, codec_id=cid)
        for cid in ("quantize", "fixedscaleoffset", "astype", "packbits"):
            mod = __import__(f"numcodecs.{cid}", fromlist=["x"])
            cls = {c.codec_id: c for c in vars(mod).values() if isinstance(c, type) and hasattr(c, "codec_id")}.get(cid)
            if cls is not None:
                ref.registry.register_codec(cls)
