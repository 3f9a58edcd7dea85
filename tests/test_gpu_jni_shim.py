"""GPU: the JNI shim (native/jni/bkdigest_jni.c) on the GPU routes — the whole native chain a JVM
would drive (JNI native -> C-ABI -> pinned staging -> HIP kernels -> result), through the same fake
JNIEnv the CPU suite uses (tests/test_jni_shim.py; no JDK in this image). The library is forced onto
the GPU for every host-memory call: host-resident batches with bkd_set_host_batch_route(2), per-call
resumes with bkd_set_cpu_route_max(0). Every result against the oracle:
  * Sse42Crc32C.nativeArray / nativeUnsafe (crc32c_sse42_jni.cpp:26-48) over 1 MiB and odd lengths;
  * GpuDigest.resumeAddress / resumeArray / resumeBatch for CRC32C and CRC32;
  * GpuDigest.verifyBatch (BatchedReadOp's verified prefix) with corruptions, and packageBatch /
    packageBatchArrays (LedgerFragmentReplicator's batch) with the SURVEY §8c framing vectors.
"""
import ctypes

import numpy as np
import pytest

import oracle
from bookkeeper_amd import _native
from test_jni_shim import GPU, SSE, _barray, _frame, _jint, _long_array, env, shim  # noqa: F401 (fixtures)

pytestmark = pytest.mark.gpu
CRC32C, CRC32 = 0, 1


@pytest.fixture()
def on_gpu(gpu, shim):
    L = _native.lib()
    assert L.bkd_device_count() > 0
    old_max = L.bkd_get_cpu_route_max()
    assert L.bkd_set_host_batch_route(2) == 0 and L.bkd_set_cpu_route_max(ctypes.c_uint64(0)) == 0
    assert L.bkd_get_host_batch_route() == 2 and L.bkd_get_cpu_route_max() == 0
    yield L
    L.bkd_set_host_batch_route(0)
    L.bkd_set_cpu_route_max(ctypes.c_uint64(old_max))


def test_sse42_natives_on_the_gpu(on_gpu, shim, env):
    rng = np.random.default_rng(41)
    data = rng.bytes((1 << 20) + 77)
    arr = _barray(shim, data)
    f = getattr(shim, SSE + "nativeArray")
    for cur, idx, ln in [(0, 0, 1 << 20), (0x1234, 77, 1 << 20), (-1, 3, 4093), (9, 1000, 1)]:
        assert f(env, None, _jint(cur), arr, idx, ln, 0) == _jint(oracle.resume(CRC32C, cur, data[idx:idx + ln]))
    assert shim.fake_pending() == b""
    shim.fake_free(arr)
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    u = getattr(shim, SSE + "nativeUnsafe")
    assert u(env, None, 5, buf.ctypes.data + 11, 500000, 0) == _jint(oracle.resume(CRC32C, 5, buf[11:500011]))


@pytest.mark.parametrize("algo", [CRC32C, CRC32])
def test_gpu_digest_resumes_on_the_gpu(on_gpu, shim, env, algo):
    rng = np.random.default_rng(42 + algo)
    base = np.frombuffer(rng.bytes(3 << 20), dtype=np.uint8).copy()
    ra = getattr(shim, GPU + "resumeAddress")
    assert ra(env, None, algo, 0x55, base.ctypes.data + 5, 2 << 20) == _jint(oracle.resume(algo, 0x55, base[5:5 + (2 << 20)]))
    arr = _barray(shim, base.tobytes())
    rr = getattr(shim, GPU + "resumeArray")
    assert rr(env, None, algo, 7, arr, 1001, 777777) == _jint(oracle.resume(algo, 7, base[1001:1001 + 777777]))
    shim.fake_free(arr)
    n = 5000
    offs = np.sort(rng.integers(0, (3 << 20) - 70000, n)).astype(np.uint64)
    lens = rng.integers(0, 70000, n).astype(np.uint32)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    rc = getattr(shim, GPU + "resumeBatch")(env, None, algo, base.ctypes.data, base.size, offs.ctypes.data,
                                            lens.ctypes.data, n, seeds.ctypes.data, 0, out.ctypes.data)
    assert rc == 0 and (out == oracle.batch(algo, base, offs, lens, seeds)).all()


@pytest.mark.parametrize("algo", [CRC32C, CRC32])
def test_gpu_digest_verify_and_package_on_the_gpu(on_gpu, shim, env, algo):
    rng = np.random.default_rng(43 + algo)
    mac = 4 if algo == CRC32C else 8
    ledger, first, n = 91, 7000, 3000
    frames = [_frame(algo, ledger, first + i, rng.bytes(int(rng.integers(0, 9000)))) for i in range(n)]
    bufs = [np.frombuffer(f, dtype=np.uint8).copy() for f in frames]
    bufs[2100][-1] ^= 0x20 if bufs[2100].size > 32 + mac else 0
    if bufs[2100].size <= 32 + mac:
        bufs[2100][3] ^= 0x20
    addrs = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
    lens = np.array([b.size for b in bufs], dtype=np.uint32)
    status = np.full(n, -1, dtype=np.int32)
    r = getattr(shim, GPU + "verifyBatch")(env, None, algo, ledger, first, 0, addrs.ctypes.data, lens.ctypes.data, n,
                                          status.ctypes.data)
    want = [oracle.verify_entry(algo, b, ledger, first + i) for i, b in enumerate(bufs)]
    assert r == 2100 and list(status) == want
    # packageBatchArrays: heap payloads, frames [32 B header][digest] and the digests
    sizes = [16383, 16384] + [int(v) for v in rng.integers(0, 20000, 700)]
    payloads = [bytes(i & 0xFF for i in range(k)) if j < 2 else rng.bytes(k) for j, k in enumerate(sizes)]
    arrays = [_barray(shim, p) for p in payloads]
    m = len(payloads)
    parr = shim.fake_object_array((ctypes.c_void_p * m)(*arrays), m)
    ids = np.arange(1, 1 + m, dtype=np.int64)
    lfs = np.array([len(p) for p in payloads], dtype=np.int64)
    idarr, lfarr = _long_array(shim, ids), _long_array(shim, lfs)
    fr = np.zeros(m * (32 + mac), dtype=np.uint8)
    dg = np.zeros(m, dtype=np.uint32)
    rc = getattr(shim, GPU + "packageBatchArrays")(env, None, algo, 1, idarr, 0, lfarr, parr, fr.ctypes.data,
                                                   32 + mac, dg.ctypes.data)
    assert rc == 0 and shim.fake_pending() == b""
    # ledger 1, entry 1, LAC 0, b[i] = (byte) i of 16 383 B; entry 2 has 16 384 B
    assert dg[0] == {CRC32C: 0x24656066, CRC32: 0xdf2ebb5b}[algo]
    for i, p in enumerate(payloads):
        d, hdr = oracle.digest_entry(algo, 1, int(ids[i]), 0, int(lfs[i]), p)
        assert dg[i] == d, i
        assert fr[i * (32 + mac):(i + 1) * (32 + mac)].tobytes() == hdr + oracle.digest_bytes(algo, d), i
    for o in arrays + [parr, idarr, lfarr]:
        shim.fake_free(o)
