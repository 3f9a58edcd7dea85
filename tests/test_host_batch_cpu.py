"""CPU: the CPU route of the host-resident batches (host_batch.cpp over the library's host pool) —
bkd_crc_batch_host, bkd_digest_verify_batch_host, bkd_digest_package_batch_host — bit-exact against
the oracle (pinned to the reference build and the SURVEY §8c vectors), at 1 and several host
threads. Needs no GPU: the route is forced to the CPU (and is the automatic one without a device).
The GPU route of the same entry points is tested in test_gpu_streams_host.py / test_gpu_parity.py."""
import numpy as np
import pytest

import golden_util
import oracle
from bookkeeper_amd import checksum as ck
from bookkeeper_amd import digest as dg


@pytest.fixture(autouse=True, params=[1, 0], ids=["1-thread", "all-threads"])
def cpu_route(request):
    ck.set_host_threads(request.param)
    with ck.host_batch_route(ck.HOST_ROUTE_CPU):
        assert ck.get_host_batch_route() == ck.HOST_ROUTE_CPU
        yield request.param
    ck.set_host_threads(0)


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_crc_batch_host_cpu_golden_batch(algo):
    """The reference-generated fixtures: the 400-entry seeded batch (unaligned offsets, lengths
    0..70 000, random seeds) and the 4096-entry set of tests/golden/."""
    key = "crc32c" if algo == ck.CRC32C else "crc32"
    fx = golden_util.load()["batch"]
    data = oracle.fill_splitmix64(fx["bytes"], fx["seed"])
    got = ck.crc_batch_host(algo, data, np.array(fx["offsets"], np.uint64), np.array(fx["lengths"], np.uint32),
                            seeds=np.array([int(x, 16) for x in fx["seeds"]], np.uint32))
    assert (got == np.array([int(x, 16) for x in fx[key]], np.uint32)).all()
    g = golden_util.load_4096()
    data = oracle.fill_splitmix64(int(g["bytes"]), int(g["seed"]))
    got = ck.crc_batch_host(algo, data, g["offsets"], g["lengths"], seeds=g["seeds"])
    assert (got == g[key]).all()


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_crc_batch_host_cpu_ragged_vs_oracle(algo):
    rng = np.random.default_rng(7 + algo)
    size = 8 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    n = 20000
    lens = rng.choice([0, 1, 15, 16, 64, 100, 4096, 9000, 70000], n).astype(np.uint32)
    offs = rng.integers(0, size - 70000, n).astype(np.uint64)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = ck.crc_batch_host(algo, host, offs, lens, seeds=seeds)
    want = oracle.batch(algo, host, offs.astype(np.int64), lens, seeds=seeds)
    assert (got == want).all()
    got = ck.crc_batch_host(algo, host, offs, lens, seed_all=0x1234)
    assert (got == oracle.batch(algo, host, offs.astype(np.int64), lens, seeds=np.full(n, 0x1234, np.uint32))).all()
    with pytest.raises(ck._native.BkdError):  # out of range: refused before any work
        ck.crc_batch_host(algo, host, np.array([size - 1], np.uint64), np.array([2], np.uint32))


def _frames(algo, rng, n, ledger, first_id, max_payload):
    frames = []
    for i in range(n):
        size = int(rng.choice([0, 1, 5, 31, 100, 4096 - 36, int(rng.integers(0, max_payload))]))
        payload = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        digest, hdr = oracle.digest_entry(algo, ledger, first_id + i, first_id + i - 1, size, payload)
        frames.append(bytearray(hdr + oracle.digest_bytes(algo, digest) + payload))
    return frames


@pytest.mark.parametrize("algo,dtype", [(ck.CRC32C, dg.DigestType.CRC32C), (ck.CRC32, dg.DigestType.CRC32)])
def test_verify_batch_host_cpu_every_failure_kind(algo, dtype):
    """BatchedReadOp.complete (BatchedReadOp.java:164-190): every status equals oracle.verify_entry's
    (DigestManager.java:226-283) and first_bad is the verified prefix."""
    rng = np.random.default_rng(21 + algo)
    ledger, first = 99, 1000
    dm = dg.DigestManager.instantiate(ledger, b"", dtype)
    frames = _frames(algo, rng, 3000, ledger, first, 9000)
    st, fb = dm.verify_batch_host(frames, first)
    assert (st == 0).all() and fb == len(frames)
    frames[2500][-1 if len(frames[2500]) > 40 + dm.macCodeLength else 33] ^= 0x40
    frames[1700][32] ^= 1  # digest byte
    def refr(i, ledger_id, entry_id):  # a frame whose digest is valid for other ids
        pay = bytes(frames[i][32 + dm.macCodeLength:])
        d, hdr = oracle.digest_entry(algo, ledger_id, entry_id, entry_id - 1, len(pay), pay)
        frames[i] = bytearray(hdr + oracle.digest_bytes(algo, d) + pay)
    refr(2100, ledger + 1, first + 2100)  # ledger id mismatch
    refr(2900, ledger, first + 2905)  # entry id mismatch
    frames[2950] = frames[2950][:20]  # too short
    if algo == ck.CRC32:
        frames[1200][32] ^= 0x80  # CRC32's zero high word of the 8-byte digest
    st, fb = dm.verify_batch_host(frames, first)
    want = np.array([oracle.verify_entry(algo, bytes(f), ledger, first + i) for i, f in enumerate(frames)])
    assert (st == want).all()
    assert set(np.unique(want).tolist()) == {0, 1, 2, 3, 4}
    assert fb == int(np.nonzero(want)[0][0])
    # skip_entry_check: entry-id mismatches pass, the rest still fail
    st, _ = dm.verify_batch_host(frames, first, skip_entry_check=True)
    assert (st == np.where(want == 4, 0, want)).all()
    st, fb = dm.verify_batch_host([], first)
    assert fb == 0 and st.size == 0


@pytest.mark.parametrize("algo,dtype", [(ck.CRC32C, dg.DigestType.CRC32C), (ck.CRC32, dg.DigestType.CRC32)])
@pytest.mark.parametrize("stride", [None, 64])
def test_package_batch_host_cpu_matches_oracle(algo, dtype, stride):
    """PendingAddOp's packaging (DigestManager.java:117-181): header and digest bytes equal
    oracle.digest_entry's for every entry."""
    rng = np.random.default_rng(31 + algo)
    ledger = 12345
    dm = dg.DigestManager.instantiate(ledger, b"", dtype)
    n = 3000
    sizes = rng.choice([0, 1, 17, 1000, 4060, 9000], n)
    sizes[-3:] = 70000
    payloads = [rng.integers(0, 256, int(s), dtype=np.uint8) for s in sizes]
    ids = np.arange(n, dtype=np.int64) + 77
    lacs = ids - 1
    lf = np.cumsum(sizes).astype(np.int64)
    frames, digests = dm.package_batch_host(ids, lacs, lf, payloads, frame_stride=stride)
    mac = dm.macCodeLength
    for i in range(n):
        d, hdr = oracle.digest_entry(algo, ledger, int(ids[i]), int(lacs[i]), int(lf[i]), payloads[i])
        assert digests[i] == d, i
        assert bytes(frames[i, :32]) == hdr
        assert bytes(frames[i, 32:32 + mac]) == oracle.digest_bytes(algo, d)


def test_survey_framing_vectors_through_cpu_package():
    """header BE(ledger=1, entry=1, LAC=0, len) || payload b[i] = (byte) i, 16 383 and
    16 384 bytes -> CRC32C 0x24656066 / 0x6fa1a26b, CRC32 0xdf2ebb5b / 0x4512b34e."""
    want = {(ck.CRC32C, 16383): 0x24656066, (ck.CRC32C, 16384): 0x6fa1a26b,
            (ck.CRC32, 16383): 0xdf2ebb5b, (ck.CRC32, 16384): 0x4512b34e}
    for (algo, size), d in want.items():
        dtype = dg.DigestType.CRC32C if algo == ck.CRC32C else dg.DigestType.CRC32
        dm = dg.DigestManager.instantiate(1, b"", dtype)
        payload = (np.arange(size) & 0xFF).astype(np.uint8)
        _, digests = dm.package_batch_host(np.array([1]), np.array([0]), np.array([size]), [payload])
        assert digests[0] == d, (algo, size)


@pytest.mark.parametrize("algo,dtype", [(ck.CRC32C, dg.DigestType.CRC32C), (ck.CRC32, dg.DigestType.CRC32)])
def test_long_entries_fold_over_the_pool(algo, dtype):
    """Entries of >= 4 MiB are folded in 1 MiB pieces over the pool and joined with x^(8 * piece)
    (host_batch.cpp fold): lengths at and around the split and piece boundaries, seeded, mixed with
    short entries; the per-call CPU resume, a long verified frame (and one corrupted in its last
    piece) and a long packaged payload — all against the oracle."""
    rng = np.random.default_rng(51 + algo)
    size = 24 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    M = 1 << 20
    lens = np.array([4 * M, 4 * M - 1, 4 * M + 1, 9 * M + M // 2 + 3, M + 7, 0, 100, 5 * M], np.uint32)
    offs = rng.integers(0, size - int(lens.max()), lens.size).astype(np.uint64)
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    got = ck.crc_batch_host(algo, host, offs, lens, seeds=seeds)
    assert (got == oracle.batch(algo, host, offs.astype(np.int64), lens, seeds=seeds)).all()
    buf = host[3:3 + 9 * M + 5]
    assert ck.cpu_resume(algo, 0x5EED, buf) & 0xFFFFFFFF == oracle.resume(algo, 0x5EED, buf.tobytes())
    ledger, first = 7, 40
    dm = dg.DigestManager.instantiate(ledger, b"", dtype)
    payload = host[11:11 + 5 * M + 13]
    d, hdr = oracle.digest_entry(algo, ledger, first, first - 1, payload.size, payload.tobytes())
    frame = bytearray(hdr + oracle.digest_bytes(algo, d) + payload.tobytes())
    short = bytearray(frame[:32 + dm.macCodeLength] + b"")  # header + digest, empty payload: bad digest
    st, fb = dm.verify_batch_host([frame, short], first)
    assert st[0] == 0 and fb == 1
    frame[-2] ^= 0x10
    st, fb = dm.verify_batch_host([frame], first)
    assert st[0] == 2 and fb == 0
    frames, digests = dm.package_batch_host(np.array([first]), np.array([first - 1]), np.array([payload.size]),
                                            [payload])
    assert digests[0] == d and bytes(frames[0, :32]) == hdr
