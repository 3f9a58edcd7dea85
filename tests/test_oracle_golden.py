"""CPU: pin the oracle to the reference's own known-answer tests and to fixtures generated
from the reference build (tests/golden/crc_golden.json), and cross-check against zlib and,
where it was built, against the reference's compiled crc32c() (oracle/_ref)."""
import zlib

import numpy as np
import pytest

import golden_util
import oracle


def test_reference_known_answers():
    # CRCTest.java:117-135 and CommonHashesTest.java:30-38
    assert oracle.calculate(oracle.CRC32C, b"123456789") == 0xE3069283
    assert oracle.calculate(oracle.CRC32, b"123456789") == 0xCBF43926
    # ChecksumTest.java:36-50
    assert oracle.calculate(oracle.CRC32C, b"Some String") == 608512271
    assert oracle.resume(oracle.CRC32C, 0, b"Some String") == 608512271


def test_incremental_semantics():
    # ChecksumTest.java:52-116: byte-at-a-time and split resumes equal one shot
    b = b"Some String"
    c = oracle.calculate(oracle.CRC32C, b[:1])
    for i in range(1, len(b)):
        c = oracle.resume(oracle.CRC32C, c, b[i:i + 1])
    assert c == 608512271
    for algo in (oracle.CRC32C, oracle.CRC32):
        assert oracle.resume(algo, oracle.calculate(algo, b"data"), b"data") == oracle.calculate(algo, b"datadata")
    # zero-length resume returns the seed (crc32c_sse42.cpp:211-213)
    assert oracle.resume(oracle.CRC32C, 0x12345678, b"") == 0x12345678


def test_golden_literals():
    g = golden_util.load()
    for v in g["literal"]:
        data = golden_util.literal_bytes(v)
        assert oracle.calculate(oracle.CRC32C, data) == int(v["crc32c"], 16), v["name"]
        assert oracle.calculate(oracle.CRC32, data) == int(v["crc32"], 16), v["name"]
        assert oracle.resume_bitwise(oracle.CRC32C, 0, data[:4096]) == oracle.calculate(oracle.CRC32C, data[:4096])


def test_golden_batch():
    fx = golden_util.load()["batch"]
    data = oracle.fill_splitmix64(fx["bytes"], fx["seed"])
    seeds = np.array([int(s, 16) for s in fx["seeds"]], dtype=np.uint32)
    offs = np.array(fx["offsets"], dtype=np.uint64)
    lens = np.array(fx["lengths"], dtype=np.uint32)
    got = oracle.batch(oracle.CRC32C, data, offs, lens, seeds=seeds)
    assert (got == np.array([int(x, 16) for x in fx["crc32c"]], dtype=np.uint32)).all()
    got = oracle.batch(oracle.CRC32, data, offs, lens, seeds=seeds)
    assert (got == np.array([int(x, 16) for x in fx["crc32"]], dtype=np.uint32)).all()


def test_golden_batch_4096():
    """SURVEY.md §8c's larger fixture: 4096 seeded entries, lengths 0..70000, unaligned offsets."""
    fx = golden_util.load_4096()
    data = oracle.fill_splitmix64(fx["bytes"], fx["seed"])
    assert (oracle.batch(oracle.CRC32C, data, fx["offsets"], fx["lengths"], seeds=fx["seeds"]) == fx["crc32c"]).all()
    assert (oracle.batch(oracle.CRC32, data, fx["offsets"], fx["lengths"], seeds=fx["seeds"]) == fx["crc32"]).all()


def test_survey_digest_frame_vectors():
    # SURVEY.md §8c rows restating DigestManager.java:146-153 with CompositeByteBufUnwrapBugReproduceTest inputs
    for size, c32c, c32 in [(16383, 0x24656066, 0xDF2EBB5B), (16384, 0x6FA1A26B, 0x4512B34E)]:
        payload = bytes(i & 0xFF for i in range(size))
        assert oracle.digest_entry(oracle.CRC32C, 1, 1, 0, size, payload)[0] == c32c
        assert oracle.digest_entry(oracle.CRC32, 1, 1, 0, size, payload)[0] == c32
    assert oracle.digest_bytes(oracle.CRC32C, 0x24656066) == bytes.fromhex("24656066")
    assert oracle.digest_bytes(oracle.CRC32, 0xDF2EBB5B) == bytes.fromhex("00000000df2ebb5b")


def test_oracle_vs_zlib_random():
    rng = np.random.default_rng(3)
    for n in [0, 1, 2, 7, 8, 9, 63, 64, 65, 1000, 4096, 65537]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 2**32))
        assert oracle.resume(oracle.CRC32, s, d) == zlib.crc32(d, s) & 0xFFFFFFFF


def test_oracle_vs_reference_build():
    ref = oracle.ref()
    if ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    assert ref.ref_supported() == 1
    rng = np.random.default_rng(4)
    data = oracle.fill_splitmix64(300_000, 5)
    for _ in range(300):
        o = int(rng.integers(0, 200_000))
        n = int(rng.integers(0, 100_000))
        s = int(rng.integers(0, 2**32))
        chunk = data[o:o + n].tobytes()
        want = oracle.resume(oracle.CRC32C, s, chunk)
        assert ref.ref_crc32c(s, chunk, len(chunk)) == want
        assert ref.ref_crc32c_unchunked(s, chunk, len(chunk)) == want


def test_combine_and_verify():
    a, b = b"ledger-entry-", b"payload" * 100
    for algo in (oracle.CRC32C, oracle.CRC32):
        assert oracle.combine(algo, oracle.calculate(algo, a), oracle.calculate(algo, b), len(b)) == \
            oracle.calculate(algo, a + b)
    payload = bytes(range(200))
    d, hdr = oracle.digest_entry(oracle.CRC32C, 9, 4, 3, 200, payload)
    framed = hdr + oracle.digest_bytes(oracle.CRC32C, d) + payload
    assert oracle.verify_entry(oracle.CRC32C, framed, 9, 4) == 0
    assert oracle.verify_entry(oracle.CRC32C, framed, 8, 4) == 3
    assert oracle.verify_entry(oracle.CRC32C, framed, 9, 5) == 4
    assert oracle.verify_entry(oracle.CRC32C, framed, 9, 5, skip_entry_check=True) == 0
    assert oracle.verify_entry(oracle.CRC32C, framed[:35], 9, 4) == 1
    bad = bytearray(framed)
    bad[100] ^= 1
    assert oracle.verify_entry(oracle.CRC32C, bytes(bad), 9, 4) == 2


def test_splitmix_generator_matches_bench_numpy():
    from bench import _splitmix_words
    assert oracle.fill_splitmix64(8 * 1000, 42).tobytes() == _splitmix_words(1000, 42)
