"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle / reference build.

Bit-exact for every case (integer arithmetic). Mirrors the reference's own tests:
ChecksumTest.java:36-92 (KATs, resume, incremental), CRCTest.java:117-135 (check values),
CompositeByteBufUnwrapBugReproduceTest (DigestManager framing with payload b[i] = (byte) i).
"""
import os
import zlib

import numpy as np
import pytest

import golden_util
import oracle
from bookkeeper_amd import checksum as ck
from bookkeeper_amd import digest as dg
from bookkeeper_amd._native import BkdError

pytestmark = pytest.mark.gpu

LANES = (1, 4, 8, 16, 32, 64)


@pytest.fixture(autouse=True)
def _auto_lanes():
    ck.set_group_lanes(0)
    ck.set_plan_mode(0)
    yield
    ck.set_group_lanes(0)
    ck.set_plan_mode(0)


def _dev_bytes(torch, data: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(data)).to(dev)


def test_known_answers(gpu):
    # CRCTest.java:117-135, ChecksumTest.java:36-42
    assert ck.Crc32cIntChecksum.computeChecksum(b"123456789") == ck.to_java_int(0xE3069283)
    assert ck.Crc32cIntChecksum.computeChecksum(b"Some String") == 608512271
    assert ck.Crc32cIntChecksum.resumeChecksum(0, b"Some String", 0, 11) == 608512271
    assert ck.GpuIntHash(ck.CRC32).calculate(b"123456789") == ck.to_java_int(0xCBF43926)
    assert ck.Crc32cIntChecksum.computeChecksum(b"") == 0
    assert ck.Crc32cIntChecksum.acceptsMemoryAddressBuffer()


def test_incremental_resume(gpu):
    # ChecksumTest.java:52-76
    b = b"Some String"
    c = ck.Crc32cIntChecksum.computeChecksum(b, 0, 1)
    for i in range(1, len(b)):
        c = ck.Crc32cIntChecksum.resumeChecksum(c, b, i, 1)
    assert c == 608512271
    c = ck.Crc32cIntChecksum.computeChecksum(b[:4])
    assert ck.Crc32cIntChecksum.resumeChecksum(c, b, 4, 7) == 608512271


def test_int_hash_errors(gpu):
    # AbstractIncrementalIntHash.java:62-69
    h = ck.GpuIntHash()
    with pytest.raises(ValueError):
        h.resume(0, b"abc", 0, -1)
    with pytest.raises(IndexError):
        h.resume(0, b"abc", 2, 5)


def test_device_pointer_resume(gpu):
    import torch
    data = oracle.fill_splitmix64(70001, 7)
    t = _dev_bytes(torch, data, gpu)
    h = ck.GpuIntHash()
    for off, ln in [(0, 70001), (3, 4093), (100, 16), (5, 15), (9, 0)]:
        want = oracle.resume(0, 0x1234, data[off:off + ln])
        assert (h.resume(0x1234, t, off, ln) & 0xFFFFFFFF) == want


def test_golden_vectors(gpu):
    import torch
    g = golden_util.load()
    for v in g["literal"]:
        data = golden_util.literal_bytes(v)
        if v.get("crc32c") is not None:
            assert (ck.GpuIntHash(ck.CRC32C).calculate(data) & 0xFFFFFFFF) == int(v["crc32c"], 16), v["name"]
        if v.get("crc32") is not None:
            assert (ck.GpuIntHash(ck.CRC32).calculate(data) & 0xFFFFFFFF) == int(v["crc32"], 16), v["name"]
    # seeded batch fixture generated from the reference's compiled crc32c()
    fx = g["batch"]
    data = oracle.fill_splitmix64(fx["bytes"], fx["seed"])
    base = _dev_bytes(torch, data, gpu)
    offs = torch.tensor(fx["offsets"], dtype=torch.int64, device=gpu)
    lens = torch.tensor(fx["lengths"], dtype=torch.int32, device=gpu)
    seeds = torch.tensor(np.array([int(s, 16) for s in fx["seeds"]], dtype=np.uint32).view(np.int32), device=gpu)
    for lanes in LANES:
        ck.set_group_lanes(lanes)
        got = ck.crc_batch(ck.CRC32C, base, offs, lens, seeds=seeds, sync_check=True).cpu().numpy().view(np.uint32)
        want = np.array([int(x, 16) for x in fx["crc32c"]], dtype=np.uint32)
        assert (got == want).all(), lanes
        got = ck.crc_batch(ck.CRC32, base, offs, lens, seeds=seeds, sync_check=True).cpu().numpy().view(np.uint32)
        want = np.array([int(x, 16) for x in fx["crc32"]], dtype=np.uint32)
        assert (got == want).all(), lanes


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_golden_batch_4096(gpu, mode):
    """SURVEY.md §8c's 4096-entry reference-generated set (lengths 0..70000, unaligned offsets into
    a 32 MiB stream, seeded) through the automatic route, the direct kernel and the chunk plan."""
    import torch
    fx = golden_util.load_4096()
    data = oracle.fill_splitmix64(fx["bytes"], fx["seed"])
    base = _dev_bytes(torch, data, gpu)
    offs = torch.from_numpy(fx["offsets"].astype(np.int64)).to(gpu)
    lens = torch.from_numpy(fx["lengths"].view(np.int32)).to(gpu)
    seeds = torch.from_numpy(fx["seeds"].view(np.int32)).to(gpu)
    ck.set_plan_mode(mode)
    try:
        for algo, key in ((ck.CRC32C, "crc32c"), (ck.CRC32, "crc32")):
            got = ck.crc_batch(algo, base, offs, lens, seeds=seeds, sync_check=True).cpu().numpy().view(np.uint32)
            bad = np.nonzero(got != fx[key])[0]
            assert bad.size == 0, (key, bad[:5])
    finally:
        ck.set_plan_mode(0)


def test_fill_splitmix64_matches_oracle(gpu):
    import torch
    for nbytes, first in [(4096, 0), (1000003, 17), (8, 5)]:
        t = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
        ck.fill_splitmix64(t, 42, first_word=first)
        assert (t.cpu().numpy() == oracle.fill_splitmix64(nbytes, 42, first)).all()


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
@pytest.mark.parametrize("lanes", LANES)
def test_uniform_batches(gpu, algo, lanes):
    import torch
    ck.set_group_lanes(lanes)
    for entry_len, stride, n, seed_all in [(4096, 4096, 4096, 0), (4096, 4160, 1000, 0x5A5A5A5A),
                                           (16, 16, 3000, 0), (17, 20, 777, 1), (100, 100, 513, 0),
                                           (4095, 4099, 300, 7), (65536, 65536, 40, 0), (1, 3, 100, 9),
                                           (0, 8, 10, 0xDEADBEEF), (1000, 1001, 2, 0)]:
        nbytes = (n - 1) * stride + entry_len
        data = oracle.fill_splitmix64(nbytes, 1000 + entry_len)
        base = _dev_bytes(torch, data, gpu)
        got = ck.crc_batch_uniform(algo, base, entry_len, n, stride=stride, seed_all=seed_all)
        want = oracle.uniform(algo, data, stride, entry_len, n, seed_all)
        assert (got.cpu().numpy().view(np.uint32) == want).all(), (entry_len, stride, n)


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_uniform_long_held_stores_round_boundaries(gpu, algo):
    """Long uniform entries (8-lane groups, >= 32 steps) keep each group's results in its lanes and
    store them every 8 x 8 rounds and at the end (held_store_loop): batch sizes around the grid
    (one group, a partial first round, exactly one round, one past it, several rounds with a partial
    last one), per-entry seeds and a common seed, unaligned strides; every digest equals the oracle's."""
    import torch
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    ngroups = cus * (1024 // 8)
    ck.set_group_lanes(8)
    try:
        for entry_len, stride, n in [(4096, 4096, 1), (4096, 4096, ngroups - 1), (4096, 4096, ngroups),
                                     (4096, 4096, ngroups + 1), (5000, 5004, 3 * ngroups + 77),
                                     (4096, 4096, 9 * ngroups + 5)]:
            nbytes = (n - 1) * stride + entry_len
            data = oracle.fill_splitmix64(nbytes, 7 + n)
            base = _dev_bytes(torch, data, gpu)
            got = ck.crc_batch_uniform(algo, base, entry_len, n, stride=stride, seed_all=0x5EED)
            want = oracle.uniform(algo, data, stride, entry_len, n, 0x5EED)
            assert (got.cpu().numpy().view(np.uint32) == want).all(), (entry_len, stride, n)
            if n <= ngroups + 1:
                seeds = np.random.default_rng(n).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
                got = ck.crc_batch_uniform(algo, base, entry_len, n, stride=stride,
                                           seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu))
                offs = np.arange(n, dtype=np.uint64) * stride
                want = oracle.batch(algo, data, offs, np.full(n, entry_len, dtype=np.uint32), seeds)
                assert (got.cpu().numpy().view(np.uint32) == want).all(), ("seeds", n)
            del base
    finally:
        ck.set_group_lanes(0)


@pytest.mark.parametrize("lanes", LANES)
def test_uniform_short_entries_seeded(gpu, lanes):
    """Short uniform entries take the pipelined short-entry loop (every load of an entry in one
    register set, the next entry loaded during the fold); per-entry seeds, unaligned strides, and
    batches smaller and larger than the grid."""
    import torch
    ck.set_group_lanes(lanes)
    rng = np.random.default_rng(lanes)
    for entry_len, stride, n in [(16, 16, 5), (20, 23, 70001), (64, 64, 300000), (127, 131, 4097),
                                 (16 * lanes * 3, 16 * lanes * 3 + 5, 20000), (16 * lanes * 3 + 1, 16 * lanes * 3 + 1, 999)]:
        nbytes = (n - 1) * stride + entry_len
        data = oracle.fill_splitmix64(nbytes, entry_len + lanes)
        base = _dev_bytes(torch, data, gpu)
        seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        got = ck.crc_batch_uniform(ck.CRC32C, base, entry_len, n, stride=stride,
                                   seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu))
        offs = np.arange(n, dtype=np.uint64) * stride
        want = oracle.batch(ck.CRC32C, data, offs, np.full(n, entry_len, dtype=np.uint32), seeds=seeds)
        assert (got.cpu().numpy().view(np.uint32) == want).all(), (entry_len, stride, n)


def test_uniform_auto_lanes_short_entries(gpu):
    """Automatic lane choice across the short-entry sizes (1 lane to 48 B, 4 lanes to 255 B, 8 lanes
    from 256 B), seeded and unseeded, batches smaller and larger than the grid."""
    import torch
    ck.set_group_lanes(0)
    rng = np.random.default_rng(7)
    for entry_len, stride, n in [(200, 200, 5000), (255, 257, 3001), (256, 256, 300000), (300, 301, 70001),
                                 (384, 384, 40000), (385, 390, 9999), (511, 512, 20000)]:
        nbytes = (n - 1) * stride + entry_len
        data = oracle.fill_splitmix64(nbytes, entry_len)
        base = _dev_bytes(torch, data, gpu)
        offs = np.arange(n, dtype=np.uint64) * stride
        lens = np.full(n, entry_len, dtype=np.uint32)
        seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        got = ck.crc_batch_uniform(ck.CRC32C, base, entry_len, n, stride=stride,
                                   seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu))
        assert (got.cpu().numpy().view(np.uint32) == oracle.batch(ck.CRC32C, data, offs, lens, seeds=seeds)).all()
        got = ck.crc_batch_uniform(ck.CRC32, base, entry_len, n, stride=stride, seed_all=0x1234)
        assert (got.cpu().numpy().view(np.uint32) == oracle.uniform(ck.CRC32, data, stride, entry_len, n, 0x1234)).all()


@pytest.mark.parametrize("schedule", [1, 2])
def test_fold_schedules_bit_exact(gpu, schedule):
    """Both fold schedules of the one-entry-per-group kernels (the compiler's and the low-clock one
    that keeps a step's 16 lookups in flight; the default picks one from the measured clock):
    uniform entries across lane widths with per-entry seeds, the direct indexed kernel on unaligned
    ragged entries (CRC32C and CRC32), DigestManager package payloads and the fused verify route,
    against the oracle."""
    import torch
    ck.set_fold_schedule(schedule)
    try:
        rng = np.random.default_rng(schedule)
        for lanes, entry_len, stride, n in [(8, 4096, 4096, 5000), (16, 16384, 16400, 300), (32, 70000, 70003, 40),
                                            (4, 1000, 1003, 3000), (8, 700, 700, 9000)]:
            ck.set_group_lanes(lanes)
            nbytes = (n - 1) * stride + entry_len
            data = oracle.fill_splitmix64(nbytes, entry_len + schedule)
            base = _dev_bytes(torch, data, gpu)
            seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            got = ck.crc_batch_uniform(ck.CRC32C, base, entry_len, n, stride=stride,
                                       seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu))
            offs = np.arange(n, dtype=np.uint64) * stride
            want = oracle.batch(ck.CRC32C, data, offs, np.full(n, entry_len, dtype=np.uint32), seeds=seeds)
            assert (got.cpu().numpy().view(np.uint32) == want).all(), (lanes, entry_len)
        ck.set_group_lanes(0)
        ck.set_plan_mode(1)  # the direct indexed kernel: one entry per group
        n = 4000
        data = oracle.fill_splitmix64(8 << 20, 99 + schedule)
        base = _dev_bytes(torch, data, gpu)
        lens = rng.integers(0, 9000, n).astype(np.uint32)
        offs = rng.integers(0, (8 << 20) - 9000, n).astype(np.uint64)
        for algo in (ck.CRC32C, ck.CRC32):
            got = ck.crc_batch(algo, base, torch.from_numpy(offs.astype(np.int64)).to(gpu),
                               torch.from_numpy(lens.astype(np.int32)).to(gpu))
            assert (got.cpu().numpy().view(np.uint32) == oracle.batch(algo, data, offs, lens)).all(), algo
        ck.set_plan_mode(0)
        # package payloads (one entry per group) and the fused verify route under the same schedule
        test_digest_batch_package_and_verify(gpu, dg.DigestType.CRC32C, ck.CRC32C)
        test_verify_batch_near_uniform_frames(gpu, dg.DigestType.CRC32, ck.CRC32, False)
    finally:
        ck.set_fold_schedule(0)
        ck.set_plan_mode(0)
        ck.set_group_lanes(0)


def test_uniform_tiny_entries_auto_one_lane(gpu):
    """16..48-byte uniform entries in large batches pick one lane per entry automatically."""
    import torch
    for entry_len, stride in [(16, 16), (32, 32), (48, 50), (33, 40)]:
        n = 300_000
        nbytes = (n - 1) * stride + entry_len
        data = oracle.fill_splitmix64(nbytes, entry_len)
        base = _dev_bytes(torch, data, gpu)
        for algo in (ck.CRC32C, ck.CRC32):
            got = ck.crc_batch_uniform(algo, base, entry_len, n, stride=stride, seed_all=0x1234567)
            want = oracle.uniform(algo, data, stride, entry_len, n, 0x1234567)
            assert (got.cpu().numpy().view(np.uint32) == want).all(), (entry_len, stride, algo)


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
@pytest.mark.parametrize("lanes,mode", [(l, 1) for l in LANES] + [(0, 2), (0, 0)])
def test_indexed_ragged_unaligned(gpu, algo, lanes, mode):
    """Random lengths 0..70000, random (unaligned, overlapping) offsets, random per-entry seeds;
    mode 1 = one entry per lane group, mode 2 = chunked plan, mode 0 = automatic (the direct kernel
    here: a 3 MB base buffer)."""
    import torch
    ck.set_group_lanes(lanes)
    ck.set_plan_mode(mode)
    rng = np.random.default_rng(lanes * 7 + algo)
    size = 3_000_000
    data = oracle.fill_splitmix64(size, 99)
    n = 1500
    lens = rng.integers(0, 70000, n)
    lens[:100] = rng.integers(0, 40, 100)  # tiny and near-threshold entries
    lens[100:110] = [0, 1, 3, 4, 5, 15, 16, 17, 63, 64]
    offs = np.array([rng.integers(0, size - l + 1) for l in lens], dtype=np.int64)
    offs[110] = 0
    lens[110] = 20
    offs[111] = size - 20
    lens[111] = 20  # entries touching both ends of the buffer
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    base = _dev_bytes(torch, data, gpu)
    got = ck.crc_batch(algo, base, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                       seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu), sync_check=True)
    want = oracle.batch(algo, data, offs, lens, seeds=seeds)
    assert (got.cpu().numpy().view(np.uint32) == want).all()


def test_zipf_config3_sample(gpu):
    """BASELINE config 3 shape (Zipf 64 B-64 KiB, packed back to back), 65536 entries, CRC32C and CRC32."""
    import torch
    from bench import zipf_index
    offs, lens = zipf_index(65536)
    total = int(offs[-1] + lens[-1])
    base = torch.empty(total, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 42)
    host = base.cpu().numpy()
    d_off = torch.from_numpy(offs).to(gpu)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    for algo in (ck.CRC32C, ck.CRC32):
        got = ck.crc_batch(algo, base, d_off, d_len, sync_check=True).cpu().numpy().view(np.uint32)
        assert (got == oracle.batch(algo, host, offs, lens)).all()


def test_bounds_violation_reported(gpu):
    import torch
    base = torch.zeros(1000, dtype=torch.uint8, device=gpu)
    offs = torch.tensor([0, 990, 500], dtype=torch.int64, device=gpu)
    lens = torch.tensor([10, 20, 500], dtype=torch.int32, device=gpu)
    with pytest.raises(BkdError) as e:
        ck.crc_batch(ck.CRC32C, base, offs, lens, sync_check=True)
    assert e.value.code == -4
    out = ck.crc_batch(ck.CRC32C, base, offs, lens)
    with pytest.raises(BkdError):
        ck._native.check(ck.lib().bkd_stream_sync(ck._stream_ptr(None, base)))
    got = out.cpu().numpy().view(np.uint32)
    want = oracle.batch(0, np.zeros(1000, np.uint8), np.array([0, 0, 500]), np.array([10, 0, 500]))
    assert got[0] == want[0] and got[1] == 0 and got[2] == want[2]


def test_host_batch(gpu):
    rng = np.random.default_rng(5)
    data = oracle.fill_splitmix64(1 << 20, 3)
    n = 500
    lens = rng.integers(0, 5000, n)
    offs = np.array([rng.integers(0, data.size - l + 1) for l in lens], dtype=np.uint64)
    for algo in (ck.CRC32C, ck.CRC32):
        got = ck.crc_batch_host(algo, data, offs, lens, seed_all=0x77)
        assert (got == oracle.batch(algo, data, offs, lens, seed_all=0x77)).all()
    with pytest.raises(BkdError):
        ck.crc_batch_host(ck.CRC32C, data, np.array([data.size - 1]), np.array([2]))


def test_zlib_agreement(gpu):
    data = oracle.fill_splitmix64(123457, 11)
    assert (ck.GpuIntHash(ck.CRC32).calculate(data.tobytes()) & 0xFFFFFFFF) == zlib.crc32(data.tobytes())


def test_lane_choice_invariance_full_size(gpu):
    """BASELINE configs[1] at full size (1M x 4 KiB): every lane geometry yields the same digests, and
    a sample agrees with the reference's compiled crc32c()."""
    import torch
    n, L = 1 << 20, 4096
    base = torch.empty(n * L, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 42)
    outs = []
    for lanes in (4, 8, 16):
        ck.set_group_lanes(lanes)
        outs.append(ck.crc_batch_uniform(ck.CRC32C, base, L, n).clone())
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    idx = np.random.default_rng(0).integers(0, n, 2000)
    host = base.view(n, L)[torch.from_numpy(idx).to(gpu)].cpu().numpy()
    got = outs[0].cpu().numpy().view(np.uint32)[idx]
    want = oracle.uniform(ck.CRC32C, host.reshape(-1), L, L, idx.size)
    assert (got == want).all()
    # checksum of checksums over the whole batch vs the same computation on the device output
    assert oracle.calculate(0, outs[0].cpu().numpy().tobytes()) == \
        oracle.calculate(0, outs[1].cpu().numpy().tobytes())


@pytest.mark.parametrize("dtype,algo", [(dg.DigestType.CRC32C, ck.CRC32C), (dg.DigestType.CRC32, ck.CRC32)])
@pytest.mark.parametrize("v2", [True, False])
@pytest.mark.parametrize("size", [16383, 16384])
def test_digest_manager_package(gpu, dtype, algo, v2, size):
    """CompositeByteBufUnwrapBugReproduceTest: ledger 1, entry 1, LAC 0, payload b[i] = (byte) i."""
    payload = (np.arange(size) & 0xFF).astype(np.uint8).tobytes()
    dm = dg.DigestManager.instantiate(1, b"", dtype, v2)
    framed = dm.computeDigestAndPackageForSending(1, 0, size, payload, b"\0" * 20, 0)
    d, hdr = oracle.digest_entry(algo, 1, 1, 0, size, payload)
    body = hdr + oracle.digest_bytes(algo, d) + payload
    assert framed[-len(body):] == body
    # and the reader side accepts it (V3 layout = the body)
    assert dm.verifyDigestAndReturnData(1, body) == payload
    bad = bytearray(body)
    bad[40] ^= 1
    with pytest.raises(dg.BKDigestMatchException):
        dm.verifyDigestAndReturnData(1, bytes(bad))
    with pytest.raises(dg.BKDigestMatchException):
        dm.verifyDigestAndReturnData(2, body)


@pytest.mark.parametrize("dtype,algo", [(dg.DigestType.CRC32C, ck.CRC32C), (dg.DigestType.CRC32, ck.CRC32)])
def test_digest_batch_package_and_verify(gpu, dtype, algo):
    import torch
    rng = np.random.default_rng(algo)
    n = 3000
    lens = rng.integers(0, 20000, n)
    lens[:5] = [0, 1, 16, 31, 4096]
    offs = np.zeros(n, dtype=np.int64)
    np.cumsum(lens[:-1], out=offs[1:])
    payload = oracle.fill_splitmix64(int(lens.sum()), 17)
    dm = dg.DigestManager.instantiate(77, b"", dtype, False)
    entry_ids = np.arange(100, 100 + n, dtype=np.int64)
    lacs = entry_ids - 1
    frames, digests = dm.package_batch(torch.from_numpy(entry_ids).to(gpu), torch.from_numpy(lacs).to(gpu),
                                       torch.from_numpy(lens.astype(np.int64)).to(gpu), _dev_bytes(torch, payload, gpu),
                                       torch.from_numpy(offs).to(gpu),
                                       torch.from_numpy(lens.astype(np.int32)).to(gpu))
    frames = frames.cpu().numpy()
    digests = digests.cpu().numpy().view(np.uint32)
    mac = dm.macCodeLength
    framed_all = []
    for i in range(n):
        p = payload[offs[i]:offs[i] + lens[i]]
        d, hdr = oracle.digest_entry(algo, 77, int(entry_ids[i]), int(lacs[i]), int(lens[i]), p)
        assert digests[i] == d
        assert frames[i].tobytes() == hdr + oracle.digest_bytes(algo, d)
        framed_all.append(frames[i].tobytes() + p.tobytes())
    # verify the framed entries on the device, with one corruption at index 1234
    blob = bytearray(b"".join(framed_all))
    flens = np.array([len(f) for f in framed_all])
    foffs = np.zeros(n, dtype=np.int64)
    np.cumsum(flens[:-1], out=foffs[1:])
    blob[foffs[1234] + 32 + mac + 1 if flens[1234] > 32 + mac + 1 else foffs[1234] + 3] ^= 0x40
    d_framed = _dev_bytes(torch, np.frombuffer(bytes(blob), dtype=np.uint8), gpu)
    status, first_bad = dm.verify_batch(d_framed, torch.from_numpy(foffs).to(gpu),
                                        torch.from_numpy(flens.astype(np.int32)).to(gpu), first_entry_id=100)
    status = status.cpu().numpy()
    want = np.array([oracle.verify_entry(algo, bytes(blob[foffs[i]:foffs[i] + flens[i]]), 77, 100 + i)
                     for i in range(n)])
    assert (status == want).all()
    assert status[1234] != 0 and int(first_bad.item()) == 1234


@pytest.mark.parametrize("dtype,algo,stride", [(dg.DigestType.CRC32C, ck.CRC32C, 37), (dg.DigestType.CRC32, ck.CRC32, 43),
                                               (dg.DigestType.CRC32C, ck.CRC32C, 128)])
def test_package_batch_frame_strides(gpu, dtype, algo, stride):
    """Frames at odd strides (byte stores) and a wide stride, every length class incl. payloads under
    16 bytes: header and digest bytes equal the oracle's."""
    import torch
    rng = np.random.default_rng(stride)
    n = 5000
    lens = rng.integers(0, 9000, n)
    lens[:6] = [0, 1, 15, 16, 17, 4096]
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    payload = oracle.fill_splitmix64(int(lens.sum()) + 64, 29)
    dm = dg.DigestManager.instantiate(5, b"", dtype, False)
    ids = np.arange(n, dtype=np.int64) + 40
    frames, digests = dm.package_batch(torch.from_numpy(ids).to(gpu), torch.from_numpy(ids - 1).to(gpu),
                                       torch.from_numpy(lens.astype(np.int64)).to(gpu), _dev_bytes(torch, payload, gpu),
                                       torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                                       frame_stride=stride, sync_check=True)
    frames = frames.cpu().numpy()
    digests = digests.cpu().numpy().view(np.uint32)
    hl = 32 + dm.macCodeLength
    for i in range(n):
        d, hdr = oracle.digest_entry(algo, 5, int(ids[i]), int(ids[i]) - 1, int(lens[i]), payload[offs[i]:offs[i] + lens[i]])
        assert digests[i] == d, i
        assert frames[i, :hl].tobytes() == hdr + oracle.digest_bytes(algo, d), i


@pytest.mark.parametrize("dtype,algo", [(dg.DigestType.CRC32C, ck.CRC32C), (dg.DigestType.CRC32, ck.CRC32)])
def test_package_in_place_and_apart_routes_agree(gpu, dtype, algo):
    """bkd_digest_package_batch with the frames written in front of their own payloads (one buffer:
    the header-first route) and into a buffer of their own (the fused route): the same digests, and
    frame bytes equal to the oracle's in both, the in-place payloads untouched."""
    import ctypes
    import torch
    n, L = 4096, 4096
    mac = 4 if algo == ck.CRC32C else 8
    hl = 32 + mac
    plen = L - hl
    raw = oracle.fill_splitmix64(n * L, 61)
    ids = np.arange(n, dtype=np.int64) + 9
    buf = _dev_bytes(torch, raw, gpu)
    d_ids, d_lacs = torch.from_numpy(ids).to(gpu), torch.from_numpy(ids - 1).to(gpu)
    d_lenf = torch.full((n,), plen, dtype=torch.int64, device=gpu)
    d_off = torch.from_numpy(np.arange(n, dtype=np.int64) * L + hl).to(gpu)
    d_len = torch.full((n,), plen, dtype=torch.int32, device=gpu)
    apart = torch.empty(n * hl, dtype=torch.uint8, device=gpu)
    dig_a = torch.empty(n, dtype=torch.int32, device=gpu)
    dig_b = torch.empty(n, dtype=torch.int32, device=gpu)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    for frames, stride, dig in ((apart, hl, dig_a), (buf, L, dig_b)):
        ck._native.check(ck.lib().bkd_digest_package_batch(algo, 3, p(d_ids), p(d_lacs), p(d_lenf), p(buf), buf.numel(),
                                                           p(d_off), p(d_len), n, p(frames), stride, p(dig), None))
    torch.cuda.synchronize()
    assert torch.equal(dig_a, dig_b)
    digs = dig_a.cpu().numpy().view(np.uint32)
    got_apart = apart.cpu().numpy().reshape(n, hl)
    got_buf = buf.cpu().numpy().reshape(n, L)
    for i in range(n):
        pay = raw[i * L + hl:(i + 1) * L]
        d, hdr = oracle.digest_entry(algo, 3, int(ids[i]), int(ids[i]) - 1, plen, pay)
        assert digs[i] == d, i
        want = hdr + oracle.digest_bytes(algo, d)
        assert got_apart[i].tobytes() == want, i
        assert got_buf[i, :hl].tobytes() == want, i
        assert got_buf[i, hl:].tobytes() == pay.tobytes(), i


@pytest.mark.parametrize("dtype,algo", [(dg.DigestType.CRC32C, ck.CRC32C), (dg.DigestType.CRC32, ck.CRC32)])
@pytest.mark.parametrize("skip", [False, True])
def test_verify_batch_near_uniform_frames(gpu, dtype, algo, skip):
    """Frames whose lengths all lie in the near-uniform band take the fused verify (gate -> one kernel
    per frame: header CRC, payload, compare); one frame out of band sends the same batch through the
    header / plan / finish sequence. Both give oracle.verify_entry's status for every frame and the
    verified prefix, with every failure kind: payload and digest bytes, CRC32's high digest word,
    ledger id, entry id, a frame past the buffer's end; unaligned frame offsets."""
    import torch
    rng = np.random.default_rng(40 + algo + 2 * skip)
    n, ledger, first = 33000, 31, 9000  # n x 8 lanes >= the chip's lane slots: the fused route
    dm = dg.DigestManager.instantiate(ledger, b"", dtype, False)
    mac = dm.macCodeLength
    plen = rng.integers(3950, 4150, n)  # within 1/16 of each other: the fused route
    payload = oracle.fill_splitmix64(int(plen.sum()), 23)
    poffs = np.concatenate([[0], np.cumsum(plen[:-1])])
    frames = []
    for i in range(n):
        p = payload[poffs[i]:poffs[i] + plen[i]]
        d, hdr = oracle.digest_entry(algo, ledger, first + i, first + i - 1, int(plen[i]), p)
        frames.append(bytearray(hdr + oracle.digest_bytes(algo, d) + p.tobytes()))
    frames[4000][40 + mac] ^= 0x01  # payload
    frames[4500][32 + mac - 1] ^= 0x80  # digest
    frames[5000][7] ^= 0x02  # ledger id
    frames[5500][15] ^= 0x04  # entry id (passes when skip)
    if algo == ck.CRC32:
        frames[5900][33] ^= 0x10  # the zero high word of the 8-byte digest
    gaps = rng.integers(0, 13, n)  # unaligned frame offsets
    flens = np.array([len(f) for f in frames], dtype=np.int64)
    foffs = np.concatenate([[0], np.cumsum(flens[:-1] + gaps[:-1])]) + 5
    blob = np.zeros(int(foffs[-1] + flens[-1]) + 64, dtype=np.uint8)
    for i in range(n):
        blob[foffs[i]:foffs[i] + flens[i]] = np.frombuffer(bytes(frames[i]), dtype=np.uint8)
    want = np.array([oracle.verify_entry(algo, bytes(frames[i]), ledger, first + i, skip) for i in range(n)])
    foffs_oob = foffs.copy()
    foffs_oob[5800] = blob.size - 100  # the frame would run past the buffer: VERIFY_TOO_SHORT
    want_oob = want.copy()
    want_oob[5800] = 1
    d_blob = _dev_bytes(torch, blob, gpu)
    d_len = torch.from_numpy(flens.astype(np.int32)).to(gpu)
    cases = [(foffs_oob, d_len, want_oob)]
    flens_mixed = flens.copy()  # one frame far out of band: the header / plan / finish route
    flens_mixed[10] = 100
    want_mixed = want_oob.copy()
    want_mixed[10] = oracle.verify_entry(algo, bytes(frames[10][:100]), ledger, first + 10, skip)
    cases.append((foffs_oob, torch.from_numpy(flens_mixed.astype(np.int32)).to(gpu), want_mixed))
    for offs, d_l, w in cases:
        status, first_bad = dm.verify_batch(d_blob, torch.from_numpy(offs).to(gpu), d_l, first_entry_id=first,
                                            skip_entry_check=skip)
        status = status.cpu().numpy()
        bad = np.nonzero(status != w)[0]
        assert bad.size == 0, (bad[:5], status[bad[:5]], w[bad[:5]])
        nz = np.nonzero(w)[0]
        assert int(first_bad.item()) == (int(nz[0]) if nz.size else n)


@pytest.mark.parametrize("lanes,n,plen_mid", [(4, 70000, 300), (16, 20000, 4000), (32, 10000, 4000),
                                               (64, 5000, 4000)])
def test_verify_fused_route_every_lane_width(gpu, lanes, n, plen_mid):
    """crc_verify_fused_kernel is instantiated for G = 4/8/16/32/64; each width is reached
    with the plan geometry at that lane count and frames sized so that the automatic lane choice for
    one frame per group equals it (the fused route's condition). Statuses and the verified prefix
    equal oracle.verify_entry's, with payload, digest and id corruptions."""
    import torch
    rng = np.random.default_rng(lanes)
    ledger, first = 44, 100
    algo = ck.CRC32C
    dm = dg.DigestManager.instantiate(ledger, b"", dg.DigestType.CRC32C, False)
    plen = rng.integers(plen_mid - plen_mid // 40, plen_mid + plen_mid // 40, n)
    payload = oracle.fill_splitmix64(int(plen.sum()), 29)
    poffs = np.concatenate([[0], np.cumsum(plen[:-1])])
    frames = []
    for i in range(n):
        p = payload[poffs[i]:poffs[i] + plen[i]]
        d, hdr = oracle.digest_entry(algo, ledger, first + i, first + i - 1, int(plen[i]), p)
        frames.append(bytearray(hdr + oracle.digest_bytes(algo, d) + p.tobytes()))
    for k, (pos, bit) in enumerate(((50, 0x01), (34, 0x80), (7, 0x02), (15, 0x04))):
        frames[(k + 1) * n // 5][pos] ^= bit  # payload, digest, ledger id, entry id
    gaps = rng.integers(0, 9, n)
    flens = np.array([len(f) for f in frames], dtype=np.int64)
    foffs = np.concatenate([[0], np.cumsum(flens[:-1] + gaps[:-1])]) + 3
    blob = np.zeros(int(foffs[-1] + flens[-1]) + 64, dtype=np.uint8)
    for i in range(n):
        blob[foffs[i]:foffs[i] + flens[i]] = np.frombuffer(bytes(frames[i]), dtype=np.uint8)
    # the library's automatic lane choice for one frame per group (bkdigest.hip auto_lanes)
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    mean = blob.size // n
    g = 4 if mean < 512 else (8 if mean < 32768 else 32)
    while g < 64 and n * g < cus * 1024:
        g *= 2
    assert g == lanes, (g, lanes)
    want = np.array([oracle.verify_entry(algo, bytes(frames[i]), ledger, first + i) for i in range(n)])
    steps = min(32, 32768 // (16 * lanes))
    ck.set_plan_geometry(lanes, steps, 16)
    try:
        status, first_bad = dm.verify_batch(_dev_bytes(torch, blob, gpu), torch.from_numpy(foffs).to(gpu),
                                            torch.from_numpy(flens.astype(np.int32)).to(gpu), first_entry_id=first)
        status = status.cpu().numpy()
    finally:
        ck.set_plan_geometry()
    bad = np.nonzero(status != want)[0]
    assert bad.size == 0, (bad[:5], status[bad[:5]], want[bad[:5]])
    assert int(first_bad.item()) == int(np.nonzero(want)[0][0])


def test_plan_overflow_falls_back_to_direct(gpu):
    """Heavily overlapping entries exceed the plan's capacity (n + size/CH + 16 chunks); the
    overflowing entries are computed one entry per group in the chunk kernel's tail, bit-exact."""
    import torch
    ck.set_plan_mode(2)
    size = 1 << 20
    data = oracle.fill_splitmix64(size, 8)
    n = 24
    offs = np.zeros(n, dtype=np.int64)
    offs[1::2] = 3
    lens = np.full(n, size, dtype=np.int64)
    lens[1::2] = size - 3
    lens[5] = 100
    base = _dev_bytes(torch, data, gpu)
    got = ck.crc_batch(ck.CRC32C, base, torch.from_numpy(offs).to(gpu),
                       torch.from_numpy(lens.astype(np.int32)).to(gpu), seed_all=0x1234, sync_check=True)
    assert (got.cpu().numpy().view(np.uint32) == oracle.batch(0, data, offs, lens, seed_all=0x1234)).all()


def test_plan_mid_size_entries_wave_combine(gpu):
    """Entries of 65..4096 chunks (256 KiB .. 16 MiB at 4 KiB chunks) are combined one wave per
    entry, larger ones by the whole block: lengths around both thresholds, several such entries in
    one combine block and across the 1024-entry block boundary, packed at odd offsets, seeded."""
    import torch
    ck.set_plan_mode(2)
    rng = np.random.default_rng(65)
    n = 1100
    lens = rng.integers(0, 5000, n).astype(np.int64)
    big = np.arange(3, n, 37)
    lens[big] = rng.integers(64 * 4096 - 300, 1 << 20, big.size)
    edges = [64 * 4096 - 128, 64 * 4096, 64 * 4096 + 1, 64 * 4096 + 200, 4096 * 4096 - 130, 4096 * 4096,
             4096 * 4096 + 1, 4096 * 4096 + 4096 * 3]
    for k, L in enumerate(edges):
        lens[1010 + 2 * k] = L  # straddles the combine kernel's block boundary at entry 1024
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 200, n - 1))
    size = int(offs[-1] + lens[-1] + 77)
    base = torch.empty(size, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 66)
    host = base.cpu().numpy()
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    d_off, d_len = torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu)
    d_seed = torch.from_numpy(seeds.view(np.int32)).to(gpu)
    for algo in (ck.CRC32C, ck.CRC32):
        got = ck.crc_batch(algo, base, d_off, d_len, seeds=d_seed, sync_check=True).cpu().numpy().view(np.uint32)
        want = oracle.batch(algo, host, offs, lens, seeds=seeds)
        assert (got == want).all(), np.flatnonzero(got != want)[:10]


def test_plan_huge_single_entry_and_small_neighbours(gpu):
    """A 96 MiB entry next to tiny ones: the plan spreads the big entry over the whole chip."""
    import torch
    size = 96 << 20
    base = torch.empty(size + 1000, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 77)
    host = base.cpu().numpy()
    offs = np.array([0, size, size + 10, size + 500, 7], dtype=np.int64)
    lens = np.array([size, 10, 490, 500, size - 7], dtype=np.int64)
    for algo in (ck.CRC32C, ck.CRC32):
        got = ck.crc_batch(algo, base, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                           sync_check=True).cpu().numpy().view(np.uint32)
        assert (got == oracle.batch(algo, host, offs, lens)).all()
    h = ck.GpuIntHash()
    assert (h.resume(5, base, 3, size - 3) & 0xFFFFFFFF) == oracle.resume(0, 5, host[3:size])


@pytest.mark.parametrize("mis", [1, 5, 15])
def test_plan_misaligned_base_pointer(gpu, mis):
    """The plan aligns chunk ends to absolute device addresses; a base pointer that is not
    16-byte aligned shifts that grid (PlanGeo.mis) and must not change any digest."""
    import torch
    ck.set_plan_mode(2)
    rng = np.random.default_rng(mis)
    size = 600_000
    data = oracle.fill_splitmix64(size + 16, 31)
    big = _dev_bytes(torch, data, gpu)
    base = big[mis:mis + size]
    host = data[mis:mis + size]
    n = 700
    lens = rng.integers(0, 20000, n)
    lens[:40] = np.arange(40)
    offs = np.array([rng.integers(0, size - l + 1) for l in lens], dtype=np.int64)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for algo in (ck.CRC32C, ck.CRC32):
        got = ck.crc_batch(algo, base, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                           seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu), sync_check=True)
        assert (got.cpu().numpy().view(np.uint32) == oracle.batch(algo, host, offs, lens, seeds=seeds)).all()


@pytest.mark.parametrize("geom", [(4, 64, 16), (4, 16, 512), (16, 8, 16), (8, 32, 4096), (16, 32, 100), (8, 1, 16),
                                  (32, 8, 16), (64, 4, 300)])
def test_plan_geometries(gpu, geom):
    """Every plan geometry (lanes, steps per chunk, head-merge threshold) gives the oracle's digests."""
    import torch
    ck.set_plan_mode(2)
    ck.set_plan_geometry(*geom)
    try:
        rng = np.random.default_rng(sum(geom))
        size = 2_000_000
        data = oracle.fill_splitmix64(size + 16, 41)
        big = _dev_bytes(torch, data, gpu)
        base = big[3:3 + size]
        host = data[3:3 + size]
        n = 900
        lens = rng.integers(0, 40000, n)
        lens[:64] = np.arange(64) * 7
        offs = np.array([rng.integers(0, size - l + 1) for l in lens], dtype=np.int64)
        seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        got = ck.crc_batch(ck.CRC32C, base, torch.from_numpy(offs).to(gpu),
                           torch.from_numpy(lens.astype(np.int32)).to(gpu),
                           seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu), sync_check=True)
        assert (got.cpu().numpy().view(np.uint32) == oracle.batch(0, host, offs, lens, seeds=seeds)).all()
    finally:
        ck.set_plan_geometry()


@pytest.mark.parametrize("geom", [(8, 1, 16), (16, 8, 16), (4, 16, 16)])
def test_plan_combine_paths_other_chunk_sizes(gpu, geom):
    """The wave and block combines at chunk sizes other than 4 KiB (their X, X^64, X^1024 and power
    tables are built per chunk size): entries of 65..4096 chunks and of more than 4096 chunks beside
    short ones, seeded, both polynomials."""
    import torch
    lanes, steps, _ = geom
    ch = 16 * lanes * steps
    ck.set_plan_mode(2)
    ck.set_plan_geometry(*geom)
    try:
        rng = np.random.default_rng(ch)
        lens = rng.integers(0, 3000, 300).astype(np.int64)
        lens[5::40] = rng.integers(65 * ch, 4096 * ch, lens[5::40].size)
        lens[7] = 4096 * ch + 1
        lens[150] = 4100 * ch + 333
        lens[151] = 3 * 4096 * ch - 5
        offs = np.concatenate([[0], np.cumsum(lens[:-1] + 13)]).astype(np.int64) + 1
        size = int(offs[-1] + lens[-1] + 100)
        base = torch.empty(size, dtype=torch.uint8, device=gpu)
        ck.fill_splitmix64(base, ch)
        host = base.cpu().numpy()
        seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
        for algo in (ck.CRC32C, ck.CRC32):
            got = ck.crc_batch(algo, base, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                               seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu), sync_check=True)
            want = oracle.batch(algo, host, offs, lens, seeds=seeds)
            bad = np.nonzero(got.cpu().numpy().view(np.uint32) != want)[0]
            assert len(bad) == 0, (algo, lens[bad[:10]].tolist())
    finally:
        ck.set_plan_geometry()


@pytest.mark.parametrize("pinned", [False, True])
def test_host_batch_pipelined_segments(gpu, pinned):
    """Host-memory batches spanning several 64 MiB staging segments (sorted, packed), one entry
    larger than a segment, and an unsorted index; pinned and pageable sources."""
    import torch
    size = 150 << 20
    t = torch.empty(size, dtype=torch.uint8, pin_memory=pinned)
    host = t.numpy()
    host[:] = oracle.fill_splitmix64(size, 5)
    rng = np.random.default_rng(int(pinned))
    lens = rng.integers(0, 300000, 900)
    lens[450] = 70 << 20  # > one segment
    offs = np.zeros(lens.size, dtype=np.uint64)
    np.cumsum(lens[:-1], out=offs[1:])
    keep = offs + lens <= size
    offs, lens = offs[keep], lens[keep]
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    got = ck.crc_batch_host(ck.CRC32C, host, offs, lens, seeds=seeds)
    assert (got == oracle.batch(0, host, offs, lens, seeds=seeds)).all()
    perm = rng.permutation(lens.size)[:200]
    got = ck.crc_batch_host(ck.CRC32, host, offs[perm], lens[perm])
    assert (got == oracle.batch(1, host, offs[perm], lens[perm])).all()


@pytest.mark.parametrize("geom", [(4, 16, 16), (8, 32, 16), (16, 8, 16), (32, 4, 300)])
@pytest.mark.parametrize("shift", [0, 5, 100])
def test_plan_length_sweep_packed(gpu, geom, shift):
    """Every entry length 0..2599 (plus multi-chunk lengths), packed with gaps and never overlapping,
    so no entry falls back to the serial path: each goes through chunking, padding to the next
    line and the x^(-8*pad) combine. Base misaligned by `shift` bytes."""
    import torch
    ck.set_plan_mode(2)
    ck.set_plan_geometry(*geom)
    try:
        lens = np.concatenate([np.arange(0, 2600), np.arange(2600, 70000, 997)]).astype(np.int64)
        gaps = (np.arange(len(lens)) * 37) % 91
        offs = np.concatenate([[0], np.cumsum(lens + gaps)[:-1]]).astype(np.int64) + 3
        size = int(offs[-1] + lens[-1] + 64)
        data = oracle.fill_splitmix64(size + shift, 11)
        big = _dev_bytes(torch, data, gpu)
        base, host = big[shift:], data[shift:]
        seeds = (np.arange(len(lens), dtype=np.uint64) * 2654435761 % 2**32).astype(np.uint32)
        for algo in (ck.CRC32C, ck.CRC32):
            got = ck.crc_batch(algo, base, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                               seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu), sync_check=True)
            want = oracle.batch(algo, host, offs, lens, seeds=seeds)
            bad = np.nonzero(got.cpu().numpy().view(np.uint32) != want)[0]
            assert len(bad) == 0, (algo, lens[bad[:10]].tolist())
    finally:
        ck.set_plan_geometry()


def _threaded_reference(algo: int, host: np.ndarray, offs: np.ndarray, lens: np.ndarray) -> tuple[np.ndarray, str]:
    """Every entry's digest from the reference side, threaded: CRC32C through the reference's own
    circe crc32c() (oracle/_ref, crc32c_sse42.cpp:184-217), else the C oracle; CRC32 through zlib's
    crc32() (= java.util.zip.CRC32, CRC32DigestManager.java:28-87)."""
    n = offs.size
    want = np.zeros(n, dtype=np.uint32)
    o64 = np.ascontiguousarray(offs, dtype=np.uint64)
    l32 = np.ascontiguousarray(lens, dtype=np.uint32)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    args = (host.ctypes.data_as(oracle._u8p), o64.ctypes.data_as(oracle._u64p), l32.ctypes.data_as(oracle._u32p), n)
    if algo == ck.CRC32C and oracle.ref() is not None:
        oracle.ref().ref_crc32c_batch_timed(*args, threads, 1, want.ctypes.data_as(oracle._u32p))
        return want, "reference circe crc32c()"
    if algo == ck.CRC32:
        oracle.lib().oracle_zlib_crc32_batch_timed(*args, threads, 1, want.ctypes.data_as(oracle._u32p))
        return want, "zlib crc32()"
    return oracle.batch(algo, host, offs, lens), "C oracle"


def test_zipf_full_size_every_entry_vs_reference(gpu):
    """BASELINE config 3 at full size (1M Zipf entries 64 B-64 KiB, 6.8 GB, packed, unaligned):
    every digest through the automatic route (what bench.py --config zipf times), the chunked plan
    and the one-entry-per-group kernel equals the reference's on the host copy of the same bytes —
    CRC32C against circe crc32c() compiled from the reference, CRC32 against zlib."""
    import torch
    from bench import zipf_index
    offs, lens = zipf_index(1 << 20)
    total = int(offs[-1] + lens[-1])
    base = torch.empty(total, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 42)
    d_off = torch.from_numpy(offs).to(gpu)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    host = base.cpu().numpy()
    try:
        for algo in (ck.CRC32C, ck.CRC32):
            want, _ = _threaded_reference(algo, host, offs, lens)
            for mode in (0, 2, 1):  # auto (the bench's route: the chunked plan), chunked plan forced, direct
                ck.set_plan_mode(mode)
                got = ck.crc_batch(algo, base, d_off, d_len, sync_check=True).cpu().numpy().view(np.uint32)
                bad = np.nonzero(got != want)[0]
                assert bad.size == 0, (algo, mode, bad.size, bad[:5].tolist(), lens[bad[:5]].tolist())
    finally:
        ck.set_plan_mode(0)


def test_concurrent_callers(gpu):
    """§8b threading: one shared library instance called from several host threads at once, each
    with its own HIP stream (device batches through the plan, the direct kernel and the uniform
    path) plus host-memory batches that share the staging slots; every result is exact."""
    import threading
    import torch
    rng = np.random.default_rng(21)
    size = 8_000_000
    data = oracle.fill_splitmix64(size, 77)
    base = _dev_bytes(torch, data, gpu)
    n = 3000
    lens = rng.integers(0, 20000, n)
    offs = np.array([rng.integers(0, size - l + 1) for l in lens], dtype=np.int64)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(ck.CRC32C, data, offs, lens, seeds=seeds)
    want_u = oracle.uniform(ck.CRC32C, data, 4096, 4096, size // 4096)
    d_off = torch.from_numpy(offs).to(gpu)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    d_seed = torch.from_numpy(seeds.view(np.int32)).to(gpu)
    torch.cuda.synchronize()
    errors = []

    def worker(k):
        try:
            st = torch.cuda.Stream(device=gpu)
            for r in range(6):
                kind = (k + r) % 3
                if kind == 0:
                    with torch.cuda.stream(st):
                        got = ck.crc_batch(ck.CRC32C, base, d_off, d_len, seeds=d_seed, stream=st)
                    st.synchronize()
                    assert (got.cpu().numpy().view(np.uint32) == want).all(), ("device", k, r)
                elif kind == 1:
                    with torch.cuda.stream(st):
                        got = ck.crc_batch_uniform(ck.CRC32C, base, 4096, size // 4096, stream=st)
                    st.synchronize()
                    assert (got.cpu().numpy().view(np.uint32) == want_u).all(), ("uniform", k, r)
                else:
                    got = ck.crc_batch_host(ck.CRC32C, data, offs, lens, seeds=seeds)
                    assert (got == want).all(), ("host", k, r)
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors


def test_eight_threads_eight_streams_no_global_lock(gpu):
    """VERDICT r02 item 6 (SURVEY §8b "no global lock on the hot path"): 8 host threads, each with
    its own stream, enqueue device batches back to back — plan, direct and uniform kinds, several
    calls in flight per stream before one sync — while the per-stream scratch maps are read under a
    shared lock only. Every digest is exact; each stream's bounds flag stays its own."""
    import threading
    import torch
    rng = np.random.default_rng(88)
    size = 6_000_000
    data = oracle.fill_splitmix64(size, 5)
    base = _dev_bytes(torch, data, gpu)
    n = 4000
    lens = rng.integers(0, 30000, n)
    offs = np.array([rng.integers(0, size - l + 1) for l in lens], dtype=np.int64)
    small_n = 60  # a 256 KiB window: the direct kernel
    s_lens = rng.integers(0, 4000, small_n)
    s_offs = rng.integers(0, (256 << 10) - 4000, small_n).astype(np.int64)
    d_off, d_len = torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu)
    ds_off, ds_len = torch.from_numpy(s_offs).to(gpu), torch.from_numpy(s_lens.astype(np.int32)).to(gpu)
    small_base = base[: 256 << 10]
    want_p = oracle.batch(ck.CRC32C, data, offs, lens, seeds=np.full(n, 0, np.uint32))
    want_s = oracle.batch(ck.CRC32, data[: 256 << 10], s_offs, s_lens, seeds=np.full(small_n, 0, np.uint32))
    want_u = oracle.uniform(ck.CRC32C, data, 4096, 4096, size // 4096)
    torch.cuda.synchronize()
    errors = []
    barrier = threading.Barrier(8)

    def worker(k):
        try:
            st = torch.cuda.Stream(device=gpu)
            outs = []
            barrier.wait()
            with torch.cuda.stream(st):
                for r in range(12):
                    outs.append(("plan", ck.crc_batch(ck.CRC32C, base, d_off, d_len, stream=st)))
                    outs.append(("direct", ck.crc_batch(ck.CRC32, small_base, ds_off, ds_len, stream=st)))
                    outs.append(("uniform", ck.crc_batch_uniform(ck.CRC32C, base, 4096, size // 4096, stream=st)))
            ck.stream_sync(st)
            for kind, got in outs:
                w = {"plan": want_p, "direct": want_s, "uniform": want_u}[kind]
                assert (got.cpu().numpy().view(np.uint32) == w).all(), (kind, k)
            ck.release_stream(st)
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not errors, errors


@pytest.mark.parametrize("size", [16383, 16384])
@pytest.mark.parametrize("v2", [False, True])
def test_composite_payload_digest_equals_contiguous(gpu, size, v2):
    """CompositeByteBufUnwrapBugReproduceTest (:142-201): every composite wrapping of the payload
    packages to the same bytes as the contiguous payload, and to the oracle's digest."""
    from test_bytebuf import scenarios
    payload = bytes(i & 0xFF for i in range(size))
    for dtype, algo in ((dg.DigestType.CRC32C, ck.CRC32C), (dg.DigestType.CRC32, ck.CRC32)):
        dm = dg.DigestManager.instantiate(1, b"", dtype, v2)
        want = dm.computeDigestAndPackageForSending(1, 0, size, payload, b"\0" * 20, 0)
        d, hdr = oracle.digest_entry(algo, 1, 1, 0, size, payload)
        assert want.endswith(hdr + oracle.digest_bytes(algo, d) + payload)
        for name, buf in scenarios(payload).items():
            assert dm.computeDigestAndPackageForSending(1, 0, size, buf, b"\0" * 20, 0) == want, (name, algo)


def test_crc_batch_segments(gpu):
    """Composite entries on the device: each entry's digest equals the oracle's over the concatenation
    of its segments (empty segments, single segments, many small and a few large pieces, seeds)."""
    import torch
    rng = np.random.default_rng(21)
    size = 3 << 20
    data = oracle.fill_splitmix64(size, 31)
    base = _dev_bytes(torch, data, gpu)
    n = 1500
    counts = rng.integers(0, 9, n)
    counts[:4] = [0, 1, 2, 40]
    seg_first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=seg_first[1:])
    nseg = int(seg_first[-1])
    lens = rng.integers(0, 3000, nseg)
    lens[rng.random(nseg) < 0.15] = 0
    lens[rng.random(nseg) < 0.02] = 200_000
    offs = np.array([int(rng.integers(0, size - l + 1)) for l in lens], dtype=np.int64)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for algo in (ck.CRC32C, ck.CRC32):
        got = ck.crc_batch_segments(algo, base, torch.from_numpy(offs).to(gpu),
                                    torch.from_numpy(lens.astype(np.int32)).to(gpu), torch.from_numpy(seg_first).to(gpu),
                                    seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu), sync_check=True)
        got = got.cpu().numpy().view(np.uint32)
        for i in range(n):
            cat = b"".join(data[offs[k]:offs[k] + lens[k]].tobytes() for k in range(seg_first[i], seg_first[i + 1]))
            assert got[i] == oracle.resume(algo, int(seeds[i]), cat), (algo, i)


@pytest.mark.parametrize("trial", range(6))
def test_plan_random_ragged_batches(gpu, trial):
    """Randomised ragged batches through the automatic route: per trial a fresh mix of length
    distributions (tiny, Zipf-like, near-uniform, huge), packed or scattered or overlapping
    offsets, a base pointer misaligned by 0..127 bytes, per-entry or shared seeds, CRC32C and CRC32
    — every digest against the oracle. Covers the plan's descriptor windows, position-indexed
    partials, separate heads, the uniformity gate and the short-entry launch together."""
    import torch
    rng = np.random.default_rng(9000 + trial)
    n = int(rng.integers(2000, 12000))
    kind = trial % 3
    if kind == 0:
        lens = np.minimum(64 * rng.zipf(1.1, n), 65536) - rng.integers(0, 64, n)
    elif kind == 1:
        lens = rng.integers(0, 300, n)
        lens[rng.integers(0, n, 50)] = rng.integers(4096, 200000, 50)
    else:
        lens = rng.integers(3900, 4300, n)
        lens[rng.integers(0, n, 5)] = rng.integers(0, 100, 5)
    lens = np.maximum(lens, 0).astype(np.int64)
    layout = int(rng.integers(0, 3))
    if layout == 0:  # packed
        offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    elif layout == 1:  # gaps
        offs = np.concatenate([[0], np.cumsum(lens[:-1] + rng.integers(0, 300, n - 1))])
    else:  # shuffled, some overlapping
        offs = np.concatenate([[0], np.cumsum(lens[:-1])])
        rng.shuffle(offs)
        offs = np.maximum(offs - rng.integers(0, 64, n), 0)
    size = int((offs + lens).max()) + int(rng.integers(1, 4096))
    mis = int(rng.integers(0, 128))
    data = oracle.fill_splitmix64(size + 128, 700 + trial)
    big = _dev_bytes(torch, data, gpu)
    base = big[mis:mis + size]
    host = data[mis:mis + size]
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if trial % 2 else None
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    d_seeds = torch.from_numpy(seeds.view(np.int32)).to(gpu) if seeds is not None else None
    for algo in (ck.CRC32C, ck.CRC32):
        want = oracle.batch(algo, host, offs.astype(np.uint64), lens.astype(np.uint32), seeds=seeds)
        got = ck.crc_batch(algo, base, d_offs, d_lens, seeds=d_seeds, sync_check=True).cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (trial, algo, bad.size, lens[bad[:5]], offs[bad[:5]])


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_offsets_beyond_4gib(gpu, mode):
    """64-bit addressing: indexed entries just below, across and above the 4 GiB mark of one base
    buffer (automatic route, one entry per group, chunked plan), and a uniform batch whose stride
    carries entries past 4 GiB — each digest against the oracle over a host copy of its window."""
    import torch
    ck.set_plan_mode(mode)
    four = 1 << 32
    size = four + (3 << 20)
    base = torch.empty(size, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 4242)
    w0 = four - (1 << 20)
    win = base[w0:].cpu().numpy()  # every indexed entry lies in [4 GiB - 1 MiB, size)
    rng = np.random.default_rng(4 + mode)
    n = 3000
    lens = rng.integers(0, 70000, n)
    lens[:300] = rng.integers(0, 300, 300)
    offs = rng.integers(w0, size - 70000, n).astype(np.int64)
    offs[300:340] = four - rng.integers(1, 60000, 40)  # entries straddling 2^32
    lens[300:340] = four - offs[300:340] + rng.integers(1, 5000, 40)
    offs[340] = size - 17
    lens[340] = 17  # the buffer's last bytes
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    d_offs = torch.from_numpy(offs).to(gpu)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    d_seeds = torch.from_numpy(seeds.view(np.int32)).to(gpu)
    for algo in (ck.CRC32C, ck.CRC32):
        got = ck.crc_batch(algo, base, d_offs, d_lens, seeds=d_seeds, sync_check=True).cpu().numpy().view(np.uint32)
        want = oracle.batch(algo, win, (offs - w0).astype(np.uint64), lens.astype(np.uint32), seeds=seeds)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mode, algo, bad.size, offs[bad[:5]], lens[bad[:5]])
    # uniform: entry i at i * stride; the last entries start past 4 GiB
    stride, elen = (1 << 20) + 4160, 4096 + 37
    nu = (size - elen) // stride + 1
    got = ck.crc_batch_uniform(ck.CRC32C, base, elen, nu, stride=stride).cpu().numpy().view(np.uint32)
    hi = [i for i in range(nu) if i * stride + elen > four - (1 << 20)]
    assert hi and hi[-1] * stride > four
    for i in hi + [0, 1]:
        o = i * stride
        blob = base[o:o + elen].cpu().numpy()
        assert got[i] == oracle.resume(ck.CRC32C, 0, blob.tobytes()), i


def test_resume_longer_than_4gib(gpu):
    """IntHash.resume(int, long address, long length) (Sse42Crc32C.java:105-107) on one buffer past
    4 GiB: the per-call device and host routes resume piece by piece; both equal one pass of the
    reference's own crc32c() (CRC32C; the table oracle when that build is absent) and of zlib.crc32
    (CRC32, = java.util.zip.CRC32) over the whole buffer."""
    import zlib

    import torch
    size = (1 << 32) + (3 << 20) + 5
    base = torch.empty(size, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 777)
    host = base.cpu().numpy()
    ref = oracle.ref()
    for algo, seed in ((ck.CRC32C, 0x1234567), (ck.CRC32, 0x89abcdef)):
        if algo == ck.CRC32:
            want = zlib.crc32(host, seed)
        elif ref is not None:
            want = int(ref.ref_crc32c(seed, host.ctypes.data, host.size))
        else:
            want = oracle.resume(algo, seed, host)
        want = ck.to_java_int(want)
        h = ck.GpuIntHash(algo)
        assert h.resume(seed, base) == want, algo
        assert h.resume(seed, host) == want, algo  # host buffer > the CPU-route bound: GPU via staging


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_plan_held_partials_past_one_flush(gpu, algo):
    """The chunk kernel holds each group's partials for 64 rounds of its long loop (HeldResults):
    1100 entries of 8 MiB + 3 bytes are ~2.25 M full chunks, ~69 rounds per group at 256 CUs, so every
    group stores one full set of held partials mid-loop and the rest at its end. The plan's digests
    equal the direct kernel's (one entry per lane group) for every entry and the oracle's on a sample."""
    import torch
    n, L = 1100, (8 << 20) + 3
    total = n * L + 64
    base = torch.empty(total, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 91)
    offs = torch.arange(n, dtype=torch.int64, device=gpu) * L + 5
    lens = torch.full((n,), L, dtype=torch.int32, device=gpu)
    lens[7] = L - 4096 - 77  # a different head geometry
    try:
        ck.set_plan_mode(2)
        planned = ck.crc_batch(algo, base, offs, lens).cpu().numpy().view(np.uint32)
        ck.set_plan_mode(1)
        direct = ck.crc_batch(algo, base, offs, lens).cpu().numpy().view(np.uint32)
    finally:
        ck.set_plan_mode(0)
    assert (planned == direct).all(), np.nonzero(planned != direct)[0][:5]
    o_np, l_np = offs.cpu().numpy(), lens.cpu().numpy()
    for i in (0, 7, 549, n - 1):
        data = base[o_np[i]:o_np[i] + l_np[i]].cpu().numpy()
        assert planned[i] == oracle.resume(algo, 0, data), i
    del base
