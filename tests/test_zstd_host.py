"""The device zstd decoder (tempo_amd/csrc/zstd_dev.hpp), built for the host by
tools/zstd_host_check.cpp, against an independent zstd (libzstd through pyarrow):

* every page of the reference's own zstd v2 block (cmd/tempo-cli/test-data, 611 pages,
  copied as data to tests/golden/tempo_cli/) decodes byte-identically;
* randomized pages (sizes 0 B .. 2.5 MiB: multi-block frames, 1- and 4-stream Huffman
  literals, FSE / RLE / repeat sequence tables, long matches) at levels 1..19.
The same decoder runs on the GPU in find.hip (tests/test_gpu_lookup.py)."""
import os
import random
import struct
import subprocess

import pytest

pa = pytest.importorskip("pyarrow")
if not pa.Codec.is_available("zstd"):
    pytest.skip("pyarrow without zstd", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "tempo_cli", "data")


@pytest.fixture(scope="module")
def zcheck(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("z") / "zcheck")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "tempo_amd", "csrc"),
                           os.path.join(ROOT, "tools", "zstd_host_check.cpp"), "-o", exe])
    return exe


def pages_of(data):
    off, out = 0, []
    while off < len(data):
        tl, hl = struct.unpack_from("<IH", data, off)
        out.append(data[off + 6 + hl:off + tl])
        off += tl
    return out


def fcs(frame):
    fhd = frame[4]
    single = (fhd >> 5) & 1
    nb = {0: 1 if single else 0, 1: 2, 2: 4, 3: 8}[fhd >> 6]
    o = 5 + (0 if single else 1)
    v = int.from_bytes(frame[o:o + nb], "little")
    return v + 256 if nb == 2 else v


def run(zcheck, path):
    out = subprocess.run([zcheck, path], check=True, capture_output=True).stdout
    res, o = [], 0
    while o < len(out):
        (l,) = struct.unpack_from("<I", out, o)
        o += 4
        if l == 0xFFFFFFFF:
            res.append(struct.unpack_from("<i", out, o)[0])
            o += 4
        else:
            res.append(out[o:o + l])
            o += l
    return res


def test_reference_fixture_pages(zcheck):
    data = open(FIXTURE, "rb").read()
    frames = pages_of(data)
    assert len(frames) == 611
    got = run(zcheck, FIXTURE)
    codec = pa.Codec("zstd")
    for f, g in zip(frames, got):
        assert g == bytes(codec.decompress(f, decompressed_size=fcs(f)))


def synth(rng, n):
    kind = rng.randrange(4)
    if kind == 0:
        return bytes(rng.getrandbits(8) for _ in range(n))
    if kind == 1:
        words = [b"span", b"trace", b"service", b"GET /api/v1/users/", b"\x00\x00\x10", b"db.statement select"]
        out = bytearray()
        while len(out) < n:
            out += rng.choice(words) + str(rng.randrange(1000)).encode()
        return bytes(out[:n])
    if kind == 2:
        return bytes([rng.randrange(3)]) * n
    base = bytes(rng.getrandbits(8) for _ in range(257))
    return (base * (n // 257 + 1))[:n]


def test_randomized_pages(zcheck, tmp_path):
    rng = random.Random(7)
    codec_levels = [1, 3, 9, 19]
    blobs, contents = bytearray(), []
    for i in range(60):
        n = rng.choice([0, 1, 17, 1000, 70_000, 131_072, 300_000, 1_100_000, 2_600_000])
        if n > 300_000 and i % 3:
            n = 5000
        c = synth(rng, n)
        frame = pa.Codec("zstd", compression_level=rng.choice(codec_levels)).compress(c, asbytes=True)
        blobs += struct.pack("<IH", len(frame) + 6, 0) + frame
        contents.append(c)
    p = str(tmp_path / "data")
    open(p, "wb").write(bytes(blobs))
    got = run(zcheck, p)
    assert len(got) == len(contents)
    for c, g in zip(contents, got):
        assert g == c
