"""GPU parity for batched trace-ID lookup (bloom + index) vs the oracle."""
import os
import random

import numpy as np
import pytest

from oracle import oracle as O
import tempo_amd as T

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def oracle_hits(paths, ids, **kw):
    rc, hits = O.lookup([O.V2Block(p) for p in paths], ids, **kw)
    assert rc == 0
    return np.array(hits, dtype=np.int64).reshape(-1, 5)


def test_v2test_fixture(engine, golden):
    ids = np.array([list(bytes.fromhex(t)) for t in golden["v2test"]["ids"]], dtype=np.uint8)
    blk = engine.open_v2block(os.path.join(GOLD, "v2test"))
    got, _ = engine.lookup([blk], ids)
    # every stored id is bloom-positive and maps to its data page's record
    assert got[:, 0].tolist() == list(range(10))
    assert got[:, 2].tolist() == [0] * 6 + [1] * 4
    assert got[:, 3:].tolist() == [[0, 533]] * 6 + [[533, 590]] * 4
    np.testing.assert_array_equal(got, oracle_hits([os.path.join(GOLD, "v2test")], ids))


def test_synthetic_blocks(engine, tmp_path):
    paths, stored = [], []
    for b in range(4):
        p = os.path.join(str(tmp_path), "v%d" % b)
        stored.append(T.synth_v2_block(p, 20_000 + 5000 * b, seed=b))
        paths.append(p)
    rng = np.random.default_rng(0)
    present = np.concatenate([s[rng.integers(0, len(s), 3000)] for s in stored])
    absent = rng.integers(0, 256, size=(12_000, 16), dtype=np.uint8)
    ids = np.concatenate([present, absent])
    rng.shuffle(ids)
    blocks = [engine.open_v2block(p) for p in paths]
    got, _ = engine.lookup(blocks, ids)
    exp = oracle_hits(paths, ids)
    np.testing.assert_array_equal(got, exp)
    # every present id hits its own block
    assert len(np.unique(got[:, 0])) >= 12_000


def test_time_and_block_range(engine, tmp_path):
    paths = []
    for b in range(3):
        p = os.path.join(str(tmp_path), "v%d" % b)
        T.synth_v2_block(p, 5000, seed=10 + b)
        paths.append(p)
    ids = np.random.default_rng(1).integers(0, 256, size=(4000, 16), dtype=np.uint8)
    blocks = [engine.open_v2block(p) for p in paths]
    ts, te = 1_700_000_000 + 11 * 3600, 1_700_000_000 + 11 * 3600 + 10
    got, _ = engine.lookup(blocks, ids, time_start=ts, time_end=te)
    np.testing.assert_array_equal(got, oracle_hits(paths, ids, ts=ts, te=te))
    lo, hi = bytes(16), bytes([0x80] + [0] * 15)
    got, _ = engine.lookup(blocks, ids, block_start=lo, block_end=hi)
    np.testing.assert_array_equal(got, oracle_hits(paths, ids, bstart=lo, bend=hi))


def test_ids_in_many_blocks(engine, tmp_path):
    """The same block set opened 7 times: every present id hits 7 blocks, more than
    the count pass keeps per id (4), so the write pass re-probes those ids; ids with
    <= 4 hits are copied. Both must give the oracle's (id, block) order."""
    paths = []
    for b in range(2):
        p = os.path.join(str(tmp_path), "m%d" % b)
        T.synth_v2_block(p, 8000, seed=40 + b)
        paths.append(p)
    stored = [T.synth_v2_block(os.path.join(str(tmp_path), "s"), 8000, seed=40)]
    rng = np.random.default_rng(3)
    ids = np.concatenate([stored[0][rng.integers(0, len(stored[0]), 2000)],
                          rng.integers(0, 256, size=(3000, 16), dtype=np.uint8)])
    order = [paths[0]] * 5 + [paths[1]] * 2  # id of block m0: 5 hits; duplicates of m1 ids: 2
    blocks = [engine.open_v2block(p) for p in order]
    got, _ = engine.lookup(blocks, ids)
    np.testing.assert_array_equal(got, oracle_hits(order, ids))
    assert np.bincount(got[:, 0]).max() >= 5


# ---- findOne on the device (tempodb/encoding/v2/finder_paged.go:79-110)
def oracle_find(paths, ids):
    """(id_idx, block_idx) -> the oracle's findOne object (None: not found) for every block."""
    obl = [O.V2Block(p) for p in paths]
    return {(i, b): obl[b].find(bytes(ids[i])) for i in range(len(ids)) for b in range(len(paths))}


def check_find(engine, paths, ids):
    blocks = [engine.open_v2block(p) for p in paths]
    try:
        got, _ = engine.find(blocks, ids)
        lk, _ = engine.lookup(blocks, ids)
    finally:
        for b in blocks:
            b.close()
    # one entry per lookup hit, in the lookup's (id, block) order
    assert [(g[0], g[1]) for g in got] == [(int(r[0]), int(r[1])) for r in lk]
    exp = oracle_find(paths, ids)
    for i, b, st, obj in got:
        want = exp[(i, b)]
        assert (st == T.TSG_OK) == (want is not None), (i, b, st)
        assert obj == want
    # ids the lookup rejected: the oracle finds nothing there either
    hit = {(g[0], g[1]) for g in got}
    assert all(v is None for k, v in exp.items() if k not in hit)
    return got


def test_find_v2test_objects(engine, golden):
    """All 10 objects of the reference's v2test block come back byte-exact through the
    device's snappy page decode (backend_block_test.go:14-85)."""
    ids = np.array([list(bytes.fromhex(t)) for t in golden["v2test"]["ids"]], dtype=np.uint8)
    got = check_find(engine, [os.path.join(GOLD, "v2test")], ids)
    assert [g[2] for g in got] == [T.TSG_OK] * 10
    for (i, _, _, obj) in got:  # the exact object bytes TestV2Block lists
        assert obj.hex() == golden["v2test"]["objs"][i]


def test_find_synthetic_blocks(engine, tmp_path):
    paths, stored = [], []
    for b in range(3):
        p = os.path.join(str(tmp_path), "f%d" % b)
        stored.append(T.synth_v2_block(p, 30_000 + 7000 * b, seed=60 + b))
        paths.append(p)
    rng = np.random.default_rng(8)
    ids = np.concatenate([s[rng.integers(0, len(s), 400)] for s in stored] +
                         [rng.integers(0, 256, size=(300, 16), dtype=np.uint8)])
    rng.shuffle(ids)
    got = check_find(engine, paths, ids)
    assert sum(g[2] == T.TSG_OK for g in got) >= 1200


def _py_find_pages(data_path):
    """Every object of a zstd v2 data file, decoded with libzstd (pyarrow): {id: object}
    (first occurrence per id, as findOne's linear scan returns)."""
    import struct
    pa = pytest.importorskip("pyarrow")
    from tests.test_zstd_host import fcs, pages_of
    codec = pa.Codec("zstd")
    objs = {}
    for f in pages_of(open(data_path, "rb").read()):
        page = bytes(codec.decompress(f, decompressed_size=fcs(f)))
        o = 0
        while o + 8 <= len(page):
            total, il = struct.unpack_from("<II", page, o)
            oid, obj = page[o + 8:o + 8 + il], page[o + 8 + il:o + total]
            objs.setdefault(oid, obj)
            o += total
    return objs


def test_find_zstd_reference_block(engine):
    """The reference's zstd v2 block (cmd/tempo-cli/test-data: 611 pages, 621 objects,
    64-bit ids zero-padded to 16 bytes): every object comes back byte-exact through the
    device zstd decoder; absent ids find nothing."""
    path = os.path.join(GOLD, "tempo_cli")
    objs = _py_find_pages(os.path.join(path, "data"))
    assert len(objs) >= 611
    ids = np.array([list(k) for k in objs if len(k) == 16], dtype=np.uint8)
    rng = np.random.default_rng(4)
    absent = rng.integers(0, 256, size=(500, 16), dtype=np.uint8)
    absent[:, :8] = 0  # same 64-bit-id shape: passes the block's id range more often
    allids = np.concatenate([ids, absent])
    blk = engine.open_v2block(path)
    try:
        got, _ = engine.find([blk], allids)
    finally:
        blk.close()
    found = {i: obj for i, b, st, obj in got if st == T.TSG_OK}
    for i in range(len(ids)):
        assert found.get(i) == objs[bytes(ids[i])], i
    assert all(i < len(ids) for i in found)
    assert all(st in (T.TSG_OK, T.TSG_E_NOT_FOUND) for _, _, st, _ in got)


def test_lookup_and_find_across_devices(tmp_path):
    """Blocks spread over two device contexts (both on ordinal 0 here, so the one-GPU
    box exercises the per-device fan-out, the concurrent probes and the (id, block)
    merge) give the same hits and objects as the single-device call."""
    paths, stored = [], []
    for b in range(5):
        p = os.path.join(str(tmp_path), "d%d" % b)
        stored.append(T.synth_v2_block(p, 6000 + 900 * b, seed=90 + b))
        paths.append(p)
    rng = np.random.default_rng(11)
    ids = np.concatenate([s[rng.integers(0, len(s), 300)] for s in stored] +
                         [rng.integers(0, 256, size=(1000, 16), dtype=np.uint8)])
    rng.shuffle(ids)
    eng = T.Engine(devices=[0, 0])
    assert eng.device_count == 2
    blocks = [eng.open_v2block(p, device=b % 2) for b, p in enumerate(paths)]
    try:
        got, _ = eng.lookup(blocks, ids)
        np.testing.assert_array_equal(got, oracle_hits(paths, ids))
        fgot, _ = eng.find(blocks, ids)
    finally:
        for b in blocks:
            b.close()
        eng.close()
    assert [(g[0], g[1]) for g in fgot] == [(int(r[0]), int(r[1])) for r in got]
    exp = oracle_find(paths, ids)
    for i, b, st, obj in fgot:
        assert obj == exp[(i, b)]
    assert sum(g[2] == T.TSG_OK for g in fgot) >= 1500


_LK_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import tempo_amd as T
ids = np.load(sys.argv[2])
eng = T.Engine(devices=[0])
blocks = [eng.open_v2block(p) for p in sys.argv[4:]]
got, _ = eng.lookup(blocks, ids)
np.save(sys.argv[3], got)
for b in blocks:
    b.close()
eng.close()
"""


@pytest.mark.parametrize("env", [{"TSG_LK_OCAP": "1"}, {"TSG_LK_SLOTMAJOR": "0", "TSG_LK_HOSTSIZE": "1", "TSG_LK_TR": "1"},
                                 {"TSG_LK_OCC": "6"}])
def test_lookup_pass_variants(tmp_path, env):
    """The count / write passes' alternatives, each read once per process (so a child process):
    the write pass's relaunch when the hits outnumber its first columns (TSG_LK_OCAP=1 caps them
    at one hit), the round-5 id-major kept hits with the host reading the total between the
    passes and the bit-at-a-time slab transpose, and the 6-wave count pass — every one returns the oracle's hits."""
    import subprocess
    import sys
    paths, stored = [], []
    for b in range(3):
        p = os.path.join(str(tmp_path), "v%d" % b)
        stored.append(T.synth_v2_block(p, 8000 + 2000 * b, seed=40 + b))
        paths.append(p)
    rng = np.random.default_rng(4)
    ids = np.concatenate([s[rng.integers(0, len(s), 1500)] for s in stored] +
                         [rng.integers(0, 256, size=(3000, 16), dtype=np.uint8)])
    rng.shuffle(ids)
    ip, op = os.path.join(str(tmp_path), "ids.npy"), os.path.join(str(tmp_path), "got.npy")
    np.save(ip, ids)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", _LK_CHILD, root, ip, op, *paths], env=e, timeout=100,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(op)
    exp = oracle_hits(paths, ids)
    assert len(exp) > 1
    np.testing.assert_array_equal(got, exp)
