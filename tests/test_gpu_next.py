"""GPU parity for the §8f next-row codecs: CRC32 / CRC32C / Adler32 /
JenkinsLookup3 (checksum32.py), AsType, PackBits -- through the C ABI on the
device, against the oracle and the reference's fixtures; bit-exact."""

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import CRC32, CRC32C, Adler32, AsType, JenkinsLookup3, PackBits, batch, get_codec
from numcodecs_amd.checksum32 import jenkins_lookup3
from tests.helpers import check_encode_decode, fixture_cases

pytestmark = pytest.mark.gpu
RNG = np.random.default_rng(4242)

SIZES = [0, 1, 2, 3, 4, 5, 15, 16, 17, 255, 4095, 4096, 4097, 65535, 65536, 65537,
         (1 << 20) + 3, (1 << 22) + 16, (1 << 24) + 5]
REF = {"crc32": oracle.crc32, "crc32c": oracle.crc32c, "adler32": oracle.adler32}
CODECS = {"crc32": CRC32, "crc32c": CRC32C, "adler32": Adler32}


@pytest.mark.parametrize("codec_id", ["crc32", "crc32c", "adler32"])
def test_checksum_sizes_device(device, codec_id):
    cls = CODECS[codec_id]
    for n in SIZES:
        x = RNG.integers(0, 256, n, dtype=np.uint8)
        xd = torch.from_numpy(x).to(device)
        assert cls.checksum(xd) == REF[codec_id](x), (codec_id, n)
        enc = cls().encode(xd)
        ref = oracle.checksum32_encode(codec_id, x)
        assert np.array_equal(enc.cpu().numpy(), ref), (codec_id, n)
        assert torch.equal(cls().decode(enc), xd)


@pytest.mark.parametrize("codec_id", ["crc32", "crc32c", "adler32"])
def test_checksum_misaligned_and_values(device, codec_id):
    cls = CODECS[codec_id]
    base = torch.randint(0, 256, (300000,), dtype=torch.uint8, device=device)
    for off in (1, 2, 3, 4, 8, 12):
        for n in (17, 4097, 200001):
            x = base[off: off + n]
            assert cls.checksum(x) == REF[codec_id](x.cpu().numpy()), (off, n)
    x = base[:70001]
    for v in (0, 1, 7, 0xFFFFFFFF, 0x12345678, 65520 | (65520 << 16)):
        assert cls.checksum(x, v) == REF[codec_id](x.cpu().numpy(), v), v


@pytest.mark.parametrize("codec_id", ["crc32", "crc32c", "adler32"])
def test_checksum_edge_values(device, codec_id):
    cls = CODECS[codec_id]
    for fill in (0, 255):
        for n in (1, 5552, 5553, 65537, 1 << 20):  # 5552: zlib's NMAX
            x = torch.full((n,), fill, dtype=torch.uint8, device=device)
            assert cls.checksum(x) == REF[codec_id](x.cpu().numpy()), (fill, n)


def test_checksum_fixtures_device(device):
    for codec_id, cls in CODECS.items():
        n = 0
        for arr, _j, config, enc in fixture_cases(codec_id):
            c = get_codec(dict(config))
            assert isinstance(c, cls)
            got = c.encode(arr)  # host in, host out (staged through the device)
            assert got.tobytes() == enc, (codec_id, _j)
            dec = c.decode(enc)
            assert bytes(dec) == arr.tobytes(order="A")
            check_encode_decode(arr, c)
            n += 1
        assert n == 13


@pytest.mark.parametrize("codec", [CRC32(), CRC32(location="end"), Adler32(), Adler32(location="end"),
                                   CRC32C(), CRC32C(location="start")])
def test_checksum_errors(device, codec):
    arr = np.arange(1000, dtype="i4")
    enc = codec.encode(arr)
    with pytest.raises(RuntimeError):
        codec.decode(enc[:-1])
    with pytest.raises(ValueError):
        codec.decode(b"000")
    with pytest.raises(ValueError):
        codec.encode(np.arange(1000, dtype="i4")[::2])
    encd = codec.encode(torch.from_numpy(arr).to(device))
    bad = encd.clone()
    bad[100] ^= 1
    with pytest.raises(RuntimeError, match="checksum do not match"):
        codec.decode(bad)


@pytest.mark.parametrize("codec_id", ["crc32", "crc32c", "adler32"])
@pytest.mark.parametrize("location", ["start", "end"])
def test_checksum_one_launch_verify_tile_edges(device, codec_id, location):
    """Checksum32.decode of one device buffer: with location="start" on a
    16-B aligned buffer the one-launch verify tiles the stored word together
    with the payload and removes its share at the finish (CrcFin::head,
    adler_arrive_finish).  Sizes around the 16-B vector, the 4 KiB lane step
    and the 64 KiB / 32 KiB tiles, where payload + 4 crosses into one more
    tile; non-default init values; a corrupted stored word and payload;
    the same buffers at misaligned offsets (the dword-aligned path)."""
    cls = CODECS[codec_id]
    sizes = [12, 13, 16, 28, 60, 61, 4092, 4093, 4096, (1 << 15) - 4, (1 << 15) - 3, (1 << 16) - 4, (1 << 16) - 3,
             (1 << 16), (1 << 18) - 4, (1 << 20) - 1, (1 << 20) + 13, (1 << 22) - 4, (1 << 24) + 7]
    for n in sizes:
        x = RNG.integers(0, 256, n, dtype=np.uint8)
        c = cls(location=location)
        ref = oracle.checksum32_encode(codec_id, x, location=location)
        enc = torch.from_numpy(ref).to(device)
        assert enc.data_ptr() % 16 == 0
        assert np.array_equal(c.decode(enc).cpu().numpy(), x), (codec_id, n)
        bad = enc.clone()
        k = 0 if location == "start" else n
        bad[k] ^= 0x40  # stored word
        with pytest.raises(RuntimeError, match="checksum do not match"):
            c.decode(bad)
        bad = enc.clone()
        bad[(4 if location == "start" else 0) + n // 2] ^= 1  # payload
        with pytest.raises(RuntimeError, match="checksum do not match"):
            c.decode(bad)
        big = torch.empty(enc.numel() + 16, dtype=torch.uint8, device=device)
        for off in (1, 4, 8):
            view = big[off: off + enc.numel()]
            view.copy_(enc)
            assert np.array_equal(c.decode(view).cpu().numpy(), x), (codec_id, n, off)
    # zlib's `value` argument: the codecs keep the reference's init, the ABI takes any
    from numcodecs_amd import _native, _ops
    kind = {"crc32": _native.MC_CK_CRC32, "crc32c": _native.MC_CK_CRC32C, "adler32": _native.MC_CK_ADLER32}
    loc = _native.MC_CK_START if location == "start" else _native.MC_CK_END
    x = RNG.integers(0, 256, (1 << 16) + 5, dtype=np.uint8)
    for v in (1, 0xFFFFFFFF, 0x12345678):
        want = REF[codec_id](x, v)
        stored = np.array([want], dtype="<u4").view(np.uint8)
        buf = np.concatenate([stored, x] if location == "start" else [x, stored])
        got = _ops.checksum32_verify(kind[codec_id], torch.from_numpy(buf).to(device), buf.size, v, loc)
        assert got == (want, want), (codec_id, location, v)


def test_jenkins_kats_device(device):
    """test_jenkins.py:8-71 through the device kernel."""
    assert jenkins_lookup3(b"", 0) == 0xDEADBEEF
    assert jenkins_lookup3(b"", 0xDEADBEEF) == 0xBD5B7DDE
    assert jenkins_lookup3(b"Four score and seven years ago", 0) == 0x17770551
    assert jenkins_lookup3(b"Four score and seven years ago", 1) == 0xCD628161
    assert jenkins_lookup3(b"jenkins", 0) == 202276345
    s = b"Four score and seven years ago"
    j = JenkinsLookup3()
    result = j.encode(s)
    assert result[-4:] == b"\x51\x05\x77\x17"
    assert bytes(j.decode(result)) == s
    j = JenkinsLookup3(initval=1230)
    result = j.encode(s)
    assert result[-4:] == b"\xd7Z\xe2\x0e"
    assert bytes(j.decode(result)) == s
    j = JenkinsLookup3(initval=0xDEADBEEF, prefix=b"HDF5 prefix")
    result = j.encode(s)
    assert result[-4:] == np.array([oracle.jenkins_lookup3(b"HDF5 prefix" + s, 0xDEADBEEF)], "<u4").tobytes()
    assert bytes(j.decode(result)) == s
    bad = bytearray(result)
    bad[3] ^= 0x10
    with pytest.raises(RuntimeError, match="lookup3 checksum"):
        j.decode(bytes(bad))


def test_jenkins_sizes_device(device):
    for n in (0, 1, 11, 12, 13, 23, 24, 25, 47, 48, 49, 1000, 65537, (1 << 20) + 7):
        x = RNG.integers(0, 256, n, dtype=np.uint8)
        xd = torch.from_numpy(x).to(device)
        for init in (0, 1230):
            assert jenkins_lookup3(xd, init) == oracle.jenkins_lookup3(x, init), (n, init)
        # unaligned device view
        y = torch.from_numpy(np.concatenate([[7], x]).astype(np.uint8)).to(device)[1:]
        assert jenkins_lookup3(y) == oracle.jenkins_lookup3(x)


def test_jenkins_sizes_and_batches(device):
    """The Jenkins kernel around its 192-B prefetch groups and every tail
    length, single chunks and batches of many small rows."""
    for n in (0, 1, 12, 13, 767, 768, 769, 780, 781, 768 * 8 - 1, 768 * 8 + 11, 768 * 9 + 5, 768 * 17 + 12,
              (1 << 20) + 7):
        x = RNG.integers(0, 256, n, dtype=np.uint8)
        xd = torch.from_numpy(x).to(device)
        assert jenkins_lookup3(xd, 77) == oracle.jenkins_lookup3(x, 77), n
    for b, n in ((2100, 100), (2048, 37), (7, 768 * 3 + 4)):
        rows = torch.randint(0, 256, (b, n), dtype=torch.uint8, device=device)
        host = rows.cpu().numpy()
        sums = batch.checksum32_chunks(rows, "jenkins_lookup3", value=5)
        assert sums.tolist() == [oracle.jenkins_lookup3(host[i], 5) for i in range(b)], (b, n)


@pytest.mark.parametrize("codec_id", ["crc32", "crc32c", "adler32", "jenkins_lookup3"])
def test_checksum_batches(device, codec_id):
    ref = {**REF, "jenkins_lookup3": oracle.jenkins_lookup3}[codec_id]
    for b, n in ((1, 4096), (37, 1000), (64, 65536 + 12), (300, 4096 * 3 + 1), (5, 0)):
        pad = 16 if n % 2 else 0
        rows = torch.randint(0, 256, (b, n + pad), dtype=torch.uint8, device=device)[:, :n]
        sums = batch.checksum32_chunks(rows, codec_id)
        host = rows.cpu().numpy()
        assert sums.tolist() == [ref(host[i]) for i in range(b)], (codec_id, b, n)
        enc = batch.checksum32_encode_chunks(rows, codec_id)
        codec = get_codec({"id": codec_id})
        for i in range(b):
            if codec_id == "jenkins_lookup3":
                exp = oracle.jenkins_encode(host[i])
            else:
                exp = oracle.checksum32_encode(codec_id, host[i]).tobytes()
            assert enc[i].cpu().numpy().tobytes() == exp, (codec_id, i)
            assert torch.equal(torch.as_tensor(codec.decode(enc[i])).to(device), rows[i])


@pytest.mark.parametrize("codec_id", ["crc32", "crc32c", "adler32", "jenkins_lookup3"])
def test_checksum_decode_batches(device, codec_id):
    """mc_checksum32_decode_batch: the payloads compacted, the computed and
    stored checksums, for both locations, row strides of every alignment and
    corrupted rows (checksum32.py:64-88 applied per row)."""
    ref = {**REF, "jenkins_lookup3": oracle.jenkins_lookup3}[codec_id]
    locs = ["end"] if codec_id == "jenkins_lookup3" else ["start", "end"]
    for loc in locs:
        for b, n in ((1, 4096), (37, 1000), (64, 65536 + 12), (9, (1 << 20) + 5), (300, 4096 * 3 + 1), (5, 0)):
            for pad in (0, 3, 16):
                rows = torch.randint(0, 256, (b, n + pad), dtype=torch.uint8, device=device)[:, :n]
                enc = batch.checksum32_encode_chunks(rows, codec_id, location=loc)
                wide = torch.zeros((b, n + 4 + pad), dtype=torch.uint8, device=device)
                wide[:, : n + 4] = enc
                bad = min(b - 1, 3)
                if n:
                    wide[bad, (n + 4) // 2] ^= 0x40
                payload, sums, stored = batch.checksum32_decode_chunks(wide[:, : n + 4], codec_id, location=loc)
                exp = rows.clone()
                if n:
                    exp[bad, (n + 4) // 2 - (4 if loc == "start" else 0)] ^= 0x40
                assert payload.is_contiguous() and torch.equal(payload, exp), (loc, b, n, pad)
                host = exp.cpu().numpy()
                assert (sums.cpu().numpy().view("<u4").tolist() == [ref(host[i]) for i in range(b)]), (loc, b, n, pad)
                want = enc.cpu().numpy()[:, :4] if loc == "start" else enc.cpu().numpy()[:, n:]
                assert stored.cpu().numpy().view("<u4").tolist() == np.ascontiguousarray(want).view("<u4")[:, 0].tolist()
                mismatch = (sums != stored).cpu().numpy()
                assert mismatch[bad] == bool(n)
                assert not mismatch[[i for i in range(b) if i != bad]].any()


def test_packbits_fixtures_and_sizes(device):
    for arr, _j, _config, enc in fixture_cases("packbits"):
        assert PackBits().encode(arr).tobytes() == enc
        assert np.array_equal(PackBits().decode(enc), arr.reshape(-1, order="A"))
        check_encode_decode(arr, PackBits())
    for n in (0, 1, 7, 8, 9, 63, 64, 65, 127, 128, 129, 1023, 1024, 4097, 1 << 20, (1 << 22) + 5):
        raw = RNG.integers(0, 4, n, dtype=np.uint8)  # nonzero bytes other than 1 are True
        x = raw.view(bool)
        xd = torch.from_numpy(raw).to(device).view(torch.bool)
        enc = PackBits().encode(xd)
        assert np.array_equal(enc.cpu().numpy(), oracle.packbits_encode(x)), n
        dec = PackBits().decode(enc)
        assert np.array_equal(dec.cpu().numpy(), raw != 0), n
    # misaligned device input / encoded views
    base = torch.randint(0, 2, (10000,), dtype=torch.uint8, device=device)
    for off in (1, 3, 8):
        x = base[off: off + 9001].view(torch.bool)
        enc = PackBits().encode(x)
        assert np.array_equal(enc.cpu().numpy(), oracle.packbits_encode(x.cpu().numpy()))
        shifted = torch.empty(enc.numel() + off, dtype=torch.uint8, device=device)[off:]
        shifted.copy_(enc)
        assert torch.equal(PackBits().decode(shifted), x)


def test_astype_fixtures_and_casts(device):
    for prefix in ("f", "i"):
        for arr, _j, config, enc in fixture_cases("astype", prefix):
            c = get_codec(dict(config))
            assert c.encode(arr).tobytes(order="A") == enc  # fixtures hold memory order
            dec = c.decode(enc)
            exp = oracle.astype_decode(np.frombuffer(enc, config["encode_dtype"]), config["encode_dtype"],
                                       config["decode_dtype"])
            assert np.array_equal(dec, exp)
    pairs = [("<f4", "<f8"), ("<i2", "<i4"), ("<u1", "<f8"), ("<i4", "<f4"), ("<f2", "<f4"), ("<f8", "<i8"),
             ("|b1", "<i4"), ("<i8", "<u2")]
    for enc_dt, dec_dt in pairs:
        x = (RNG.standard_normal(100003) * 1e5).astype(dec_dt)
        xd = torch.from_numpy(x).to(device)
        got = AsType(enc_dt, dec_dt).encode(xd)
        with np.errstate(all="ignore"):
            ref = oracle.astype_encode(x, enc_dt, dec_dt)
        assert np.array_equal(got.cpu().numpy().view(np.uint8), ref.view(np.uint8)), (enc_dt, dec_dt)
        back = AsType(enc_dt, dec_dt).decode(got)
        with np.errstate(all="ignore"):
            ref_back = oracle.astype_decode(ref, enc_dt, dec_dt)
        assert np.array_equal(back.cpu().numpy().view(np.uint8), ref_back.view(np.uint8)), (enc_dt, dec_dt)


# ---------------------------------------------------------------------------
# Blosc shuffle filters (numcodecs_amd.blosc_shuffle) vs fixture/blosc frames
# ---------------------------------------------------------------------------
def test_blosc_filters_fixture_frames(device):
    from numcodecs_amd import blosc_shuffle as bsh
    from oracle import blosc

    n = 0
    for arr, _j, _config, frame in fixture_cases("blosc"):
        try:
            flags, ts, bs, blocks = blosc.frame_filtered_blocks(frame)
        except NotImplementedError:
            continue
        if blocks is None:
            continue
        mode = 2 if flags & blosc.BLOSC_DOBITSHUFFLE else 1 if flags & blosc.BLOSC_DOSHUFFLE else 0
        raw = arr.tobytes(order="A")
        filtered = b"".join(blocks)
        got = bsh.shuffle(np.frombuffer(raw, "u1"), ts, bs, mode)
        assert got.tobytes() == filtered, (_j, ts, bs, mode)
        back = bsh.unshuffle(np.frombuffer(filtered, "u1"), ts, bs, mode)
        assert back.tobytes() == raw
        n += 1
    assert n == 84


def test_blosc_filters_automatic_blocksize(device):
    """blocksize=AUTOBLOCKS (numcodecs' Blosc default): the blocks c-blosc
    chooses (compute_blocksize, pinned by the frame headers in
    tests/test_oracle_next.py) -- the frames of arrays 05-12 are reproduced
    from the config alone, and large buffers are cut as the rule says."""
    from numcodecs_amd import blosc_shuffle as bsh
    from oracle import blosc

    n = 0
    ncodecs = 13
    for k, (arr, _j, config, frame) in enumerate(fixture_cases("blosc")):
        if k // ncodecs <= 4 and config["blocksize"] == 0:
            continue  # written by an older c-blosc (tests/test_oracle_next.py)
        try:
            flags, ts, bs, blocks = blosc.frame_filtered_blocks(frame)
        except NotImplementedError:  # not an LZ4 frame
            continue
        if blocks is None:
            continue
        mode = 2 if flags & blosc.BLOSC_DOBITSHUFFLE else 1 if flags & blosc.BLOSC_DOSHUFFLE else 0
        raw = arr.tobytes(order="A")
        # a forced blocksize reaches the frame as c-blosc clamps it (256 -> 255 for typesize 3)
        forced = config["blocksize"] and bsh.compute_blocksize(len(raw), ts, config["clevel"], config["cname"],
                                                                config["blocksize"])
        got = bsh.shuffle(np.frombuffer(raw, "u1"), ts, forced or bsh.AUTOBLOCKS, mode, config["clevel"],
                          config["cname"])
        assert got.tobytes() == b"".join(blocks), (k, ts, bs, mode)
        n += 1
    assert n > 40
    for ts, clevel, cname in ((4, 5, "lz4"), (8, 9, "zstd"), (2, 1, "blosclz"), (4, 0, "lz4")):
        raw = RNG.integers(0, 256, (4 << 20) + 3 * ts, dtype=np.uint8)
        xd = torch.from_numpy(raw).to(device)
        bs = bsh.compute_blocksize(raw.size, ts, clevel, cname)
        for mode in (1, 2):
            got = bsh.shuffle(xd, ts, mode=mode, clevel=clevel, cname=cname)
            assert got.cpu().numpy().tobytes() == blosc.blosc_filter(raw, ts, bs, mode), (ts, clevel, cname, mode)
            assert torch.equal(bsh.unshuffle(got, ts, mode=mode, clevel=clevel, cname=cname), xd)


@pytest.mark.parametrize("mode", [1, 2])
def test_blosc_filters_sizes(device, mode):
    from numcodecs_amd import blosc_shuffle as bsh
    from oracle import blosc

    for ts in (1, 2, 3, 4, 8, 16, 24):
        for nel, bs in ((0, 256), (1, 256), (8, 64 * ts), (1000, 8 * ts * 16), (4096 + 5, 65536),
                        (100003, 32768), (262144, 1 << 20)):
            raw = RNG.integers(0, 256, nel * ts + (nel % 5 if ts > 1 else 0), dtype=np.uint8)
            xd = torch.from_numpy(raw).to(device)
            got = bsh.shuffle(xd, ts, bs, mode)
            ref = blosc.blosc_filter(raw, ts, bs, mode)
            assert got.cpu().numpy().tobytes() == ref, (ts, nel, bs, mode)
            assert torch.equal(bsh.unshuffle(got, ts, bs, mode), xd), (ts, nel, bs, mode)


@pytest.mark.parametrize("ts", [1, 2, 4, 8])
def test_bitshuffle_pipelined_grid(device, ts):
    """The persistent bit-shuffle kernel (mc_blosc.hip k_bitshuffle_pipe,
    every fast typesize): more tiles than workgroups (each
    workgroup loops, the next tile's loads in flight), partial last tiles
    (38400-B blocks: 1200 groups of 8 = 1024 + 176 for typesize 4), a shorter
    last block (generic kernel) and a block that is a single partial tile;
    both directions against the oracle."""
    from numcodecs_amd import blosc_shuffle as bsh
    from oracle import blosc

    for nbytes, bs in (((24 << 20) + 12 * ts, 38400), ((6 << 20) + 40 * ts, 32 * ts * 5),
                       (1 << 20, 1 << 20), (3 * 65536 + 64 * ts, 65536)):
        raw = RNG.integers(0, 256, nbytes, dtype=np.uint8)
        xd = torch.from_numpy(raw).to(device)
        ref = blosc.blosc_filter(raw, ts, bs, 2)
        got = bsh.shuffle(xd, ts, bs, 2)
        assert got.cpu().numpy().tobytes() == ref, (ts, nbytes, bs)
        back = bsh.unshuffle(torch.from_numpy(np.frombuffer(ref, np.uint8).copy()).to(device), ts, bs, 2)
        assert torch.equal(back, xd), (ts, nbytes, bs)


@pytest.mark.parametrize("mode", [1, 2])
def test_blosc_filters_blocksize_none_is_one_block(device, mode):
    """blocksize=None filters the whole buffer as ONE block (for every size,
    also >= 32 KiB where AUTOBLOCKS would cut it); AUTOBLOCKS (0) is c-blosc's
    choice."""
    from numcodecs_amd import blosc_shuffle as bsh
    from oracle import blosc

    for ts, nbytes in ((4, 4096), (4, (1 << 20) + 8), (8, 3 << 20), (3, 100 * 1024 + 1)):
        raw = RNG.integers(0, 256, nbytes, dtype=np.uint8)
        xd = torch.from_numpy(raw).to(device)
        got = bsh.shuffle(xd, ts, None, mode)
        assert got.cpu().numpy().tobytes() == blosc.blosc_filter(raw, ts, nbytes, mode), (ts, nbytes, mode)
        assert torch.equal(bsh.unshuffle(got, ts, None, mode), xd)
        auto = bsh.compute_blocksize(nbytes, ts)
        assert bsh.shuffle(xd, ts, bsh.AUTOBLOCKS, mode).cpu().numpy().tobytes() == \
            blosc.blosc_filter(raw, ts, auto, mode)


@pytest.mark.parametrize("kind_name", ["crc32", "crc32c", "adler32", "fletcher32"])
def test_one_launch_encode_abi(device, kind_name):
    """mc_checksum32_encode_fused / mc_fletcher32_encode_fused (the payload
    copy and the checksum footer in ONE launch) against the oracle, at both
    footer locations, with and without a ticket (NULL = the two-launch
    schedule), up to 17 MiB; the arrival ticket is left zero."""
    from numcodecs_amd import _native, _ops
    from numcodecs_amd._native import lib

    st = torch.cuda.current_stream(device).cuda_stream
    ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=device)
    kinds = {"crc32": _native.MC_CK_CRC32, "crc32c": _native.MC_CK_CRC32C, "adler32": _native.MC_CK_ADLER32}
    for n in (1, 17, 4096, 65537, (1 << 20) + 3, (17 << 20) + 5):
        x = RNG.integers(0, 256, n, dtype=np.uint8)
        xd = torch.from_numpy(x).to(device)
        if kind_name == "fletcher32":
            ref = np.frombuffer(oracle.fletcher32_encode(x), dtype=np.uint8)
            for tk in (ticket.data_ptr(), None):
                dst = torch.full((n + 4,), 0xAB, dtype=torch.uint8, device=device)
                ws = torch.empty(max(lib.mc_fletcher32_workspace(n), 16), dtype=torch.uint8, device=device)
                _native.check(lib.mc_fletcher32_encode_fused(xd.data_ptr(), dst.data_ptr(), n, ws.data_ptr(),
                                                             ws.numel(), tk, st))
                assert np.array_equal(dst.cpu().numpy(), ref), (n, tk)
            continue
        kind = kinds[kind_name]
        for loc_name, loc in (("start", _native.MC_CK_START), ("end", _native.MC_CK_END)):
            ref = oracle.checksum32_encode(kind_name, x, location=loc_name)
            for tk in (ticket.data_ptr(), None):
                dst = torch.full((n + 4,), 0xAB, dtype=torch.uint8, device=device)
                out = torch.zeros(1, dtype=torch.int32, device=device)
                ws = torch.empty(max(lib.mc_checksum32_workspace(kind, 1, n), 16), dtype=torch.uint8, device=device)
                _native.check(lib.mc_checksum32_encode_fused(kind, xd.data_ptr(), dst.data_ptr(), n, 1 if
                                                             kind_name == "adler32" else 0, None, 0, loc,
                                                             out.data_ptr(), ws.data_ptr(), ws.numel(), tk, st))
                assert np.array_equal(dst.cpu().numpy(), ref), (n, loc_name, tk)
                assert int(out.cpu().numpy().view(np.uint32)[0]) == REF[kind_name](x), (n, loc_name, tk)
    torch.cuda.synchronize()
    assert not ticket.any()


@pytest.mark.parametrize("codec_id", ["crc32", "crc32c"])
def test_one_launch_crc_arrival_tree(device, codec_id):
    """The bit-sliced CRC kernel's one-launch finish (ck_ride_arrive): the
    workgroups' shifted sums ride a 32-ary tree of returning XOR atomics.
    Tile counts (64 KiB tiles for the verify) around the tree's shapes --
    one level (<= 32 workgroups), two (33..1024), three (1025..2048) and
    grids of 2048 whose workgroups fold 2 or 3 tiles (2049, 4097: the
    stored word alone past the tiles) -- at both locations with several
    init values; last tiles of 1..17 bytes; then the
    copy-fused encode (32 KiB tiles, 1024
    workgroups); the stream's arrival ticket is left zero."""
    from numcodecs_amd import _native, _ops
    from numcodecs_amd._native import lib

    kind = {"crc32": _native.MC_CK_CRC32, "crc32c": _native.MC_CK_CRC32C}[codec_id]
    T = 1 << 16
    for tiles in (2, 31, 32, 33, 64, 65, 1056, 1057, 2048, 2049, 4097):
        for loc_name, loc in (("start", _native.MC_CK_START), ("end", _native.MC_CK_END)):
            n = tiles * T - 4 - (tiles % 7) if tiles != 4097 else (1 << 28)
            x = RNG.integers(0, 256, n, dtype=np.uint8)
            for v in ((0, 0x9E3779B9) if tiles in (33, 2049, 4097) else (0,)):
                want = REF[codec_id](x, v)
                stored = np.array([want], dtype="<u4").view(np.uint8)
                buf = torch.from_numpy(np.concatenate([stored, x] if loc_name == "start" else [x, stored])).to(device)
                assert buf.data_ptr() % 16 == 0
                got = _ops.checksum32_verify(kind, buf, n + 4, v, loc)
                assert got == (want, want), (codec_id, tiles, loc_name, v)
                if v == 0:
                    bad = buf.clone()
                    bad[(4 if loc_name == "start" else 0) + (n * 5) // 7] ^= 0x10
                    got = _ops.checksum32_verify(kind, bad, n + 4, v, loc)
                    assert got[0] != want and got[1] == want, (codec_id, tiles, loc_name)
                del buf
    # last tiles holding 1..17 bytes, a corrupted byte among them
    for extra in (1, 4, 12, 16, 17):
        for loc_name, loc in (("start", _native.MC_CK_START), ("end", _native.MC_CK_END)):
            n = 40 * T + extra - (4 if loc_name == "start" else 0)
            x = RNG.integers(0, 256, n, dtype=np.uint8)
            for v in (0, 0x5A5A5A5A):
                want = REF[codec_id](x, v)
                stored = np.array([want], dtype="<u4").view(np.uint8)
                buf = torch.from_numpy(np.concatenate([stored, x] if loc_name == "start" else [x, stored])).to(device)
                assert _ops.checksum32_verify(kind, buf, n + 4, v, loc) == (want, want), (codec_id, extra, loc_name)
                bad = buf.clone()
                bad[-1 if loc_name == "start" else n - 1] ^= 0x80  # the payload's last byte: in the tail
                got = _ops.checksum32_verify(kind, bad, n + 4, v, loc)
                assert got[0] != want and got[1] == want, (codec_id, extra, loc_name, v)
    st = torch.cuda.current_stream(device).cuda_stream
    ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=device)
    for n in (2 * (1 << 15) - 5, 33 * (1 << 15) - 1, 1025 * (1 << 15) + 3, (64 << 20) + 5):
        x = RNG.integers(0, 256, n, dtype=np.uint8)
        xd = torch.from_numpy(x).to(device)
        for loc_name, loc in (("start", _native.MC_CK_START), ("end", _native.MC_CK_END)):
            ref = oracle.checksum32_encode(codec_id, x, location=loc_name)
            dst = torch.full((n + 4,), 0xAB, dtype=torch.uint8, device=device)
            out = torch.zeros(1, dtype=torch.int32, device=device)
            ws = torch.empty(max(lib.mc_checksum32_workspace(kind, 1, n), 16), dtype=torch.uint8, device=device)
            _native.check(lib.mc_checksum32_encode_fused(kind, xd.data_ptr(), dst.data_ptr(), n, 0, None, 0, loc,
                                                         out.data_ptr(), ws.data_ptr(), ws.numel(),
                                                         ticket.data_ptr(), st))
            assert np.array_equal(dst.cpu().numpy(), ref), (n, loc_name)
            assert int(out.cpu().numpy().view(np.uint32)[0]) == REF[codec_id](x), (n, loc_name)
    torch.cuda.synchronize()
    assert not ticket.any()
    for (dev_idx, _), sl in _ops._TLS.slots.items():
        if dev_idx == device.index:
            assert not sl.ticket.any()
