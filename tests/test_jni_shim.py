"""CPU: the JNI shim (native/jni/bkdigest_jni.c) compiled and executed, not just pattern-matched.

No JDK exists in this image, so the shim is compiled with ``-Wall -Werror`` against a TEST-ONLY
<jni.h> (tests/jni_fake/jni.h: the JNI types and the function-table members the shim calls) and
linked with a fake JNIEnv (tests/jni_fake/fake_env.c) plus the real libbkdigest.so. Every native is
then called through ctypes the way the JVM would call it, and each result is checked against the
oracle. Cases follow the reference's natives ($CN/cpp/crc32c_sse42_jni.cpp:20-78) and their Java
declarations (Sse42Crc32C.java:119-129):
  * nativeArray on both branches: the critical-section scan (:26-33) and the copy-out route past the
    per-call CPU bound (forced with bkd_set_cpu_route_max), an out-of-range region (the JVM's
    ArrayIndexOutOfBoundsException left pending), a failed copy allocation (falls back to the
    critical-section CPU route instead of returning a bare 0) and a failed critical section;
  * nativeDirectBuffer with a null address returns 0 (:39-40); nativeUnsafe with length 0 (and < 0)
    returns `current` (crc32c_sse42.cpp:211-213);
  * allocConfig's validation matrix (:56-62): empty, first < min_words, non-decreasing, below
    min_words; a valid ladder returns a handle that freeConfig releases;
  * the GpuDigest batch class: resumeAddress for both polynomials, resumeBatch, verifyBatch's
    verified prefix and its error return, packageBatch's frames, packageBatchArrays over heap
    payloads (GpuBatchPackager, LedgerFragmentReplicator's batch) with its argument errors, lastError.
"""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
from bookkeeper_amd import _native
from bookkeeper_amd.build import LIB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "native", "jni", "bkdigest_jni.c")
FAKE = os.path.join(ROOT, "tests", "jni_fake")
CRC32C, CRC32 = 0, 1
SSE = "Java_com_scurrilous_circe_crc_Sse42Crc32C_"
GPU = "Java_com_scurrilous_circe_checksum_GpuDigest_"


def _jint(v: int) -> int:
    return ctypes.c_int32(v & 0xFFFFFFFF).value


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    _native.lib()  # builds/loads libbkdigest.so first (the shim links against the same file)
    d = tmp_path_factory.mktemp("jni")
    so = str(d / "libjnishim_test.so")
    common = [cc, "-O2", "-fPIC", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", FAKE, "-I",
              os.path.join(ROOT, "include")]
    subprocess.run(common + ["-Dmalloc=bkd_test_malloc", "-Dfree=bkd_test_free", "-c", SHIM, "-o",
                             str(d / "shim.o")], check=True)
    subprocess.run(common + ["-c", os.path.join(FAKE, "fake_env.c"), "-o", str(d / "fake.o")], check=True)
    libdir = os.path.dirname(LIB)
    subprocess.run([cc, "-shared", str(d / "shim.o"), str(d / "fake.o"), "-L", libdir, "-lbkdigest",
                    "-Wl,-rpath," + libdir, "-o", so], check=True)
    S = ctypes.CDLL(so)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        "fake_env": (vp, []), "fake_byte_array": (vp, [vp, i32]), "fake_int_array": (vp, [vp, i32]),
        "fake_direct_buffer": (vp, [vp]), "fake_string": (ctypes.c_char_p, [vp]), "fake_free": (None, [vp]),
        "fake_pending": (ctypes.c_char_p, []), "fake_clear": (None, []), "fake_critical_depth": (i32, []),
        "fake_critical_total": (i32, []), "fake_fail_critical": (None, [i32]), "fake_fail_malloc": (None, [i32]),
        "fake_malloc_calls": (i32, []), "fake_long_array": (vp, [vp, i32]), "fake_object_array": (vp, [vp, i32]),
        "fake_local_refs_deleted": (i32, []),
        SSE + "nativeSupported": (ctypes.c_uint8, [vp, vp]),
        SSE + "nativeArray": (i32, [vp, vp, i32, vp, i32, i32, i64]),
        SSE + "nativeDirectBuffer": (i32, [vp, vp, i32, vp, i32, i32, i64]),
        SSE + "nativeUnsafe": (i32, [vp, vp, i32, i64, i64, i64]),
        SSE + "allocConfig": (i64, [vp, vp, vp]),
        SSE + "freeConfig": (None, [vp, vp, i64]),
        GPU + "deviceCount": (i32, [vp, vp]),
        GPU + "init": (i32, [vp, vp, i32]),
        GPU + "resumeAddress": (i32, [vp, vp, i32, i32, i64, i64]),
        GPU + "resumeArray": (i32, [vp, vp, i32, i32, vp, i32, i32]),
        GPU + "resumeBatch": (i32, [vp, vp, i32, i64, i64, i64, i64, i64, i64, i32, i64]),
        GPU + "verifyBatch": (i64, [vp, vp, i32, i64, i64, ctypes.c_uint8, i64, i64, i64, i64]),
        GPU + "packageBatch": (i32, [vp, vp, i32, i64, i64, i64, i64, i64, i64, i64, i64, i64, i64]),
        GPU + "packageBatchArrays": (i32, [vp, vp, i32, i64, vp, i64, vp, vp, i64, i64, i64]),
        GPU + "lastError": (vp, [vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(S, name)
        f.restype, f.argtypes = res, args
    yield S
    _native.lib().bkd_set_cpu_route_max(ctypes.c_uint64(0xFFFFFFFFFFFFFFFF))


@pytest.fixture()
def env(shim):
    shim.fake_clear()
    yield shim.fake_env()
    assert shim.fake_critical_depth() == 0  # every critical section released
    shim.fake_clear()


def _barray(S, data: bytes):
    return S.fake_byte_array(data, len(data))


def test_native_supported(shim, env):
    assert shim.__getattr__(SSE + "nativeSupported")(env, None) == 1


def test_native_array_critical_section_route(shim, env):
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    arr = _barray(shim, data)
    f = getattr(shim, SSE + "nativeArray")
    before = shim.fake_critical_total()
    for cur, idx, ln in [(0, 0, 5000), (0x1234, 7, 4093), (-1, 4999, 1), (5, 100, 0), (5, 100, -3)]:
        want = oracle.resume(CRC32C, cur, data[idx:idx + max(ln, 0)]) if ln > 0 else cur & 0xFFFFFFFF
        assert f(env, None, _jint(cur), arr, idx, ln, 0) == _jint(want), (cur, idx, ln)
    assert shim.fake_critical_total() - before == 3  # length <= 0 returns before pinning
    assert shim.fake_pending() == b""
    shim.fake_free(arr)
    # the reference KAT through the array native (CRCTest.java:133-135)
    arr = _barray(shim, b"123456789")
    assert f(env, None, 0, arr, 0, 9, 0) == _jint(0xE3069283)
    shim.fake_free(arr)


def test_native_array_copy_out_route(shim, env):
    """Past bkd_get_cpu_route_max() the region is copied out (GetByteArrayRegion) and the critical
    section is never taken; the CPU route serves it when no device is visible."""
    L = _native.lib()
    rng = np.random.default_rng(12)
    data = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    arr = _barray(shim, data)
    f = getattr(shim, SSE + "nativeArray")
    L.bkd_set_cpu_route_max(ctypes.c_uint64(1))
    try:
        crit, mallocs = shim.fake_critical_total(), shim.fake_malloc_calls()
        assert f(env, None, 0x77, arr, 3, 69000, 0) == _jint(oracle.resume(CRC32C, 0x77, data[3:69003]))
        assert f(env, None, 0, arr, 0, 2, 0) == _jint(oracle.resume(CRC32C, 0, data[:2]))
        assert shim.fake_critical_total() == crit and shim.fake_malloc_calls() == mallocs + 2
        # an index/length outside the array: the JVM's exception stays pending, the result is 0
        assert f(env, None, 0, arr, 69990, 100, 0) == 0
        assert shim.fake_pending().startswith(b"java/lang/ArrayIndexOutOfBoundsException")
        shim.fake_clear()
        # the copy cannot be allocated: the critical-section CPU route still returns the checksum
        shim.fake_fail_malloc(1)
        assert f(env, None, 9, arr, 0, 70000, 0) == _jint(oracle.resume(CRC32C, 9, data))
        assert shim.fake_critical_total() == crit + 1 and shim.fake_pending() == b""
    finally:
        L.bkd_set_cpu_route_max(ctypes.c_uint64(0xFFFFFFFFFFFFFFFF))
    # a critical section the JVM refuses (OutOfMemoryError pending): 0, nothing held
    shim.fake_fail_critical(1)
    assert f(env, None, 0, arr, 0, 16, 0) == 0
    assert shim.fake_pending().startswith(b"java/lang/OutOfMemoryError")
    shim.fake_clear()
    shim.fake_free(arr)


def test_gpu_digest_resume_array(shim, env):
    """GpuDigest.resumeArray (GpuIntHash's heap-buffer path) for both polynomials, on both branches."""
    L = _native.lib()
    data = np.random.default_rng(18).bytes(30000)
    arr = _barray(shim, data)
    f = getattr(shim, GPU + "resumeArray")
    for algo in (CRC32C, CRC32):
        assert f(env, None, algo, 0, arr, 0, 9) == _jint(oracle.calculate(algo, data[:9]))
        assert f(env, None, algo, 0x99, arr, 17, 29000) == _jint(oracle.resume(algo, 0x99, data[17:29017]))
        assert f(env, None, algo, 0x99, arr, 17, 0) == 0x99
        L.bkd_set_cpu_route_max(ctypes.c_uint64(1024))
        try:
            assert f(env, None, algo, 0x99, arr, 17, 29000) == _jint(oracle.resume(algo, 0x99, data[17:29017]))
        finally:
            L.bkd_set_cpu_route_max(ctypes.c_uint64(0xFFFFFFFFFFFFFFFF))
    shim.fake_free(arr)


def test_native_direct_buffer_and_unsafe(shim, env):
    data = np.frombuffer(np.random.default_rng(13).bytes(9000), dtype=np.uint8).copy()
    buf = shim.fake_direct_buffer(data.ctypes.data)
    fd = getattr(shim, SSE + "nativeDirectBuffer")
    fu = getattr(shim, SSE + "nativeUnsafe")
    assert fd(env, None, 3, buf, 10, 8000, 0) == _jint(oracle.resume(CRC32C, 3, data[10:8010]))
    assert fd(env, None, 3, buf, 10, 0, 0) == 3
    null = shim.fake_direct_buffer(None)
    assert fd(env, None, 1234, null, 0, 10, 0) == 0  # crc32c_sse42_jni.cpp:39-40
    assert fu(env, None, 0, data.ctypes.data + 1, 8999, 0) == _jint(oracle.resume(CRC32C, 0, data[1:]))
    assert fu(env, None, -7, data.ctypes.data, 0, 0) == -7  # crc32c_sse42.cpp:211-213
    assert fu(env, None, -7, data.ctypes.data, -1, 0) == -7
    # chained resumes equal one pass (Sse42Crc32C.resume with a previous value)
    a = fu(env, None, 0, data.ctypes.data, 4000, 0)
    assert fu(env, None, a, data.ctypes.data + 4000, 5000, 0) == _jint(oracle.calculate(CRC32C, data))
    for o in (buf, null):
        shim.fake_free(o)


@pytest.mark.parametrize("words,ok", [
    ([], False),                    # len < 1
    ([3], False),                   # arr[0] < min_words (4, crc32c_sse42.hpp:22)
    ([4], True),
    ([4096, 512, 64], True),        # the reference's default ladder (Sse42Crc32C.java:41-45)
    ([512, 512], False),            # not strictly decreasing
    ([512, 1024], False),
    ([4096, 3], False),             # a later entry below min_words
    ([64, 16, 4], True),
])
def test_alloc_config_validation(shim, env, words, ok):
    arr = shim.fake_int_array((ctypes.c_int32 * max(1, len(words)))(*words), len(words))
    h = getattr(shim, SSE + "allocConfig")(env, None, arr)
    assert (h != 0) == ok
    if h:
        # the handle is accepted by the array native and ignored by the arithmetic
        b = _barray(shim, b"Some String")
        assert getattr(shim, SSE + "nativeArray")(env, None, 0, b, 0, 11, h) == 608512271  # ChecksumTest.java:41
        getattr(shim, SSE + "freeConfig")(env, None, h)
        shim.fake_free(b)
    shim.fake_free(arr)


def test_gpu_digest_resume_address_and_batch(shim, env):
    L = _native.lib()
    rng = np.random.default_rng(14)
    base = np.frombuffer(rng.bytes(200000), dtype=np.uint8).copy()
    for algo in (CRC32C, CRC32):
        f = getattr(shim, GPU + "resumeAddress")
        assert f(env, None, algo, 0x55, base.ctypes.data + 5, 100000) == _jint(oracle.resume(algo, 0x55, base[5:100005]))
        assert f(env, None, algo, 0x55, base.ctypes.data, 0) == 0x55
        assert f(env, None, algo, 0x55, 0, 10) == 0
        n = 300
        offs = np.sort(rng.integers(0, 190000, n)).astype(np.uint64)
        lens = rng.integers(0, 9000, n).astype(np.uint32)
        seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        out = np.zeros(n, dtype=np.uint32)
        rc = getattr(shim, GPU + "resumeBatch")(env, None, algo, base.ctypes.data, base.size, offs.ctypes.data,
                                                lens.ctypes.data, n, seeds.ctypes.data, 0, out.ctypes.data)
        assert rc == 0
        assert (out == oracle.batch(algo, base, offs, lens, seeds)).all()
        # an entry past the region: BKD_ERR_BOUNDS, and lastError says why
        lens[-1] = 20000
        offs[-1] = 190000
        rc = getattr(shim, GPU + "resumeBatch")(env, None, algo, base.ctypes.data, base.size, offs.ctypes.data,
                                                lens.ctypes.data, n, 0, 0, out.ctypes.data)
        assert rc == -4
        s = getattr(shim, GPU + "lastError")(env, None)
        assert b"exceeds" in shim.fake_string(s)
        shim.fake_free(s)
    assert getattr(shim, GPU + "deviceCount")(env, None) == L.bkd_device_count()
    if L.bkd_device_count() == 0:
        assert getattr(shim, GPU + "init")(env, None, 0) == -2  # BKD_ERR_NO_DEVICE


def _frame(algo, ledger, entry, payload):
    d, hdr = oracle.digest_entry(algo, ledger, entry, entry - 1, len(payload), payload)
    return hdr + oracle.digest_bytes(algo, d) + payload


@pytest.mark.parametrize("algo", [CRC32C, CRC32])
def test_gpu_digest_verify_batch_prefix_and_errors(shim, env, algo):
    rng = np.random.default_rng(15 + algo)
    ledger, first = 77, 1000
    frames = [_frame(algo, ledger, first + i, rng.bytes(int(rng.integers(0, 5000)))) for i in range(64)]
    bufs = [np.frombuffer(f, dtype=np.uint8).copy() for f in frames]
    f = getattr(shim, GPU + "verifyBatch")

    def run(bs, skip=False):
        addrs = np.array([b.ctypes.data for b in bs], dtype=np.uint64)
        lens = np.array([b.size for b in bs], dtype=np.uint32)
        status = np.full(len(bs), -1, dtype=np.int32)
        r = f(env, None, algo, ledger, first, int(skip), addrs.ctypes.data, lens.ctypes.data, len(bs),
              status.ctypes.data)
        return r, status

    r, st = run(bufs)
    assert r == 64 and (st == 0).all()
    bad = [b.copy() for b in bufs]
    bad[40][-1] ^= 1 if bad[40].size > 40 else 0  # a flipped payload byte (or header if no payload)
    if bad[40].size <= 40:
        bad[40][5] ^= 1
    bad[50][9] ^= 0x10  # ledger id
    r, st = run(bad)
    assert r == 40
    want = [oracle.verify_entry(algo, b, ledger, first + i) for i, b in enumerate(bad)]
    assert list(st) == want
    # entry ids checked unless skipped (DigestManager.verifyDigestAndReturnData)
    r, st = run(bufs[1:])
    assert r == 0 and st[0] == 4
    r, st = run(bufs[1:], skip=True)
    assert r == 63
    # an error code comes back negative: a null frame list with n > 0
    assert f(env, None, algo, ledger, first, 0, 0, 0, 3, 0) < 0


def test_gpu_digest_package_batch(shim, env):
    rng = np.random.default_rng(17)
    n, stride = 50, 64
    for algo in (CRC32C, CRC32):
        mac = 4 if algo == CRC32C else 8
        payloads = [np.frombuffer(rng.bytes(int(rng.integers(0, 3000))), dtype=np.uint8).copy() for _ in range(n)]
        ids = np.arange(10, 10 + n, dtype=np.int64)
        lacs = ids - 1
        lfs = np.array([p.size + 1000 for p in payloads], dtype=np.int64)
        addrs = np.array([p.ctypes.data for p in payloads], dtype=np.uint64)
        lens = np.array([p.size for p in payloads], dtype=np.uint32)
        frames = np.zeros(n * stride, dtype=np.uint8)
        digests = np.zeros(n, dtype=np.uint32)
        rc = getattr(shim, GPU + "packageBatch")(env, None, algo, 9, ids.ctypes.data, lacs.ctypes.data,
                                                 lfs.ctypes.data, addrs.ctypes.data, lens.ctypes.data, n,
                                                 frames.ctypes.data, stride, digests.ctypes.data)
        assert rc == 0
        for i in range(n):
            d, hdr = oracle.digest_entry(algo, 9, int(ids[i]), int(lacs[i]), int(lfs[i]), payloads[i])
            assert digests[i] == d
            assert frames[i * stride:i * stride + 32 + mac].tobytes() == hdr + oracle.digest_bytes(algo, d)


def _long_array(S, values):
    a = np.ascontiguousarray(values, dtype=np.int64)
    return S.fake_long_array(a.ctypes.data, a.size)


@pytest.mark.parametrize("algo", [CRC32C, CRC32])
def test_gpu_digest_package_batch_arrays(shim, env, algo):
    """GpuDigest.packageBatchArrays: LedgerFragmentReplicator's batch of heap byte[] payloads
    (LedgerFragmentReplicator.java:497-511) -> frame i = the 32-byte BE header [ledger, entry, LAC,
    length] + the digest, as computeDigestAndPackageForSending writes them (DigestManager.java:146-153,
    172-177), and digest i; lengths 0, 1, odd, 16 KiB +/- 1 (the V2 small-entry bound), 70 000."""
    rng = np.random.default_rng(31 + algo)
    mac = 4 if algo == CRC32C else 8
    sizes = [0, 1, 7, 4096, 16383, 16384, 16385, 70000] + [int(v) for v in rng.integers(0, 9000, 40)]
    n = len(sizes)
    payloads = [rng.bytes(k) for k in sizes]
    arrays = [_barray(shim, p) for p in payloads]
    objs = (ctypes.c_void_p * n)(*arrays)
    parr = shim.fake_object_array(objs, n)
    ids = np.arange(500, 500 + n, dtype=np.int64)
    lfs = np.array([len(p) + 3 for p in payloads], dtype=np.int64)  # length fields need not equal the payload
    lac = 499
    frames = np.zeros(n * (32 + mac), dtype=np.uint8)
    digests = np.zeros(n, dtype=np.uint32)
    idarr, lfarr = _long_array(shim, ids), _long_array(shim, lfs)
    f = getattr(shim, GPU + "packageBatchArrays")
    deleted = shim.fake_local_refs_deleted()
    rc = f(env, None, algo, 77, idarr, lac, lfarr, parr, frames.ctypes.data, 32 + mac, digests.ctypes.data)
    assert rc == 0 and shim.fake_pending() == b""
    assert shim.fake_local_refs_deleted() - deleted == 2 * n  # every element reference released
    for i, p in enumerate(payloads):
        d, hdr = oracle.digest_entry(algo, 77, int(ids[i]), lac, int(lfs[i]), p)
        assert digests[i] == d, i
        assert frames[i * (32 + mac):(i + 1) * (32 + mac)].tobytes() == hdr + oracle.digest_bytes(algo, d), i
    # SURVEY §8c framing vectors: ledger 1, entry 1, LAC 0, payload b[i] = (byte) i of 16 383 / 16 384 B
    want = {CRC32C: (0x24656066, 0x6fa1a26b), CRC32: (0xdf2ebb5b, 0x4512b34e)}[algo]
    for k, L in enumerate((16383, 16384)):
        one = _barray(shim, bytes(i & 0xFF for i in range(L)))
        oa = shim.fake_object_array((ctypes.c_void_p * 1)(one), 1)
        a1, l1 = _long_array(shim, [1]), _long_array(shim, [L])
        fr = np.zeros(32 + mac, dtype=np.uint8)
        dg = np.zeros(1, dtype=np.uint32)
        assert f(env, None, algo, 1, a1, 0, l1, oa, fr.ctypes.data, 32 + mac, dg.ctypes.data) == 0
        assert dg[0] == want[k]
        for o in (one, oa, a1, l1):
            shim.fake_free(o)
    # argument errors leave the JVM's exception pending and return a negative code
    short = _long_array(shim, ids[:-1])
    assert f(env, None, algo, 77, short, lac, lfarr, parr, frames.ctypes.data, 32 + mac, digests.ctypes.data) < 0
    assert shim.fake_pending().startswith(b"java/lang/IllegalArgumentException")
    shim.fake_clear()
    objs[3] = None
    holey = shim.fake_object_array(objs, n)
    assert f(env, None, algo, 77, idarr, lac, lfarr, holey, frames.ctypes.data, 32 + mac, digests.ctypes.data) < 0
    assert shim.fake_pending().startswith(b"java/lang/NullPointerException")
    shim.fake_clear()
    empty = shim.fake_object_array(objs, 0)
    e0 = _long_array(shim, [])
    assert f(env, None, algo, 77, e0, lac, e0, empty, frames.ctypes.data, 32 + mac, digests.ctypes.data) == 0
    for o in arrays + [parr, idarr, lfarr, short, holey, empty, e0]:
        shim.fake_free(o)
