"""CPU: the C-ABI library loads and exports every symbol include/bkdigest.h declares (and no other
C symbol); its host-side operator tables are right; its per-call CPU route (host_crc.cpp) matches the
golden fixtures and the oracle; the circe-compat config helpers keep the reference's validation; and
the kernel's decomposition (modelled in Python with the library's own tables) reproduces the oracle
bit-exactly. No GPU compute here."""
import ctypes
import subprocess

import numpy as np
import pytest

import oracle
from bookkeeper_amd import _native
from bookkeeper_amd import checksum as ck
from bookkeeper_amd.build import LIB
from kernel_model import KernelModel, plan_model


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    declared = _native.declared_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(_native.PROTOTYPES)
    dyn = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in dyn.splitlines() if " T " in line}
    assert set(declared) <= exported
    # nothing but the declared entry points leaks as a C symbol (C++ kernel stubs are mangled)
    assert {x for x in exported if not x.startswith("_Z") and not x.startswith("__hip")} == set(declared)
    # 3: bkd_stream_release; 4: host batch routes, bkd_host_release; 5: bkd_set_fold_schedule;
    # 6: the stream route and bkd_set_stream_range_max removed
    assert L.bkd_abi_version() == 6


def test_plan_mode_three_is_gone():
    """The stream route (plan mode 3) was removed from the library: the setter
    rejects it and leaves the mode it had."""
    L = _native.lib()
    assert L.bkd_set_plan_mode(3) == -1  # BKD_ERR_INVALID_ARG
    assert not hasattr(L, "bkd_set_stream_range_max")
    for mode in (0, 1, 2):
        assert L.bkd_set_plan_mode(mode) == 0
    assert L.bkd_set_plan_mode(0) == 0


def test_library_contains_gfx950_code():
    blob = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # offload bundle entry id for the gfx950 code object


def test_no_device_per_call_takes_cpu_route_batches_fail_loudly():
    """Crc32cIntChecksum.java:28-36 never throws: with no device the per-call resume and the
    host-resident batches are served by the library's own CPU route; device-resident batches and a
    host batch forced onto the GPU refuse to run (no silent CPU path behind a device API)."""
    if _native.device_count() > 0:
        pytest.skip("a device is visible")
    L = _native.lib()
    out = ctypes.c_uint32(0)
    for fn in (L.bkd_resume, L.bkd_resume_host):
        assert fn(0, 0, b"123456789", 9, ctypes.byref(out)) == 0
        assert out.value == 0xE3069283  # CRCTest.java:133-135
    assert ck.GpuIntHash().calculate(b"123456789") == ck.to_java_int(0xE3069283)
    assert ck.Crc32cIntChecksum.computeChecksum(b"Some String") == 608512271  # ChecksumTest.java:41
    # above the CPU-route threshold too: no device means the CPU route whatever the size
    big = np.arange(3 << 20, dtype=np.uint32).view(np.uint8)
    assert ck.GpuIntHash().calculate(big) == ck.to_java_int(oracle.calculate(0, big))
    offs = np.zeros(1, dtype=np.uint64)
    lens = np.full(1, 9, dtype=np.uint32)
    res = np.zeros(1, dtype=np.uint32)
    assert L.bkd_get_host_batch_route() == 1  # no device: the CPU route
    rc = L.bkd_crc_batch_host(0, b"123456789", 9, offs.ctypes.data, lens.ctypes.data, 1, None, 0, res.ctypes.data)
    assert rc == 0 and res[0] == 0xE3069283
    with ck.host_batch_route(ck.HOST_ROUTE_GPU):
        rc = L.bkd_crc_batch_host(0, b"123456789", 9, offs.ctypes.data, lens.ctypes.data, 1, None, 0,
                                  res.ctypes.data)
        assert rc == -2  # BKD_ERR_NO_DEVICE: the GPU route was asked for
        with pytest.raises(_native.BkdError):
            ck.crc_batch_host(0, b"123456789", offs, lens)
    # device-resident batches are GPU work only
    rc = L.bkd_crc_batch_uniform(0, 1 << 20, 4096, 4096, 1, None, 0, 1 << 21, None)
    assert rc == -2


@pytest.mark.parametrize("algo", [0, 1])
def test_cpu_route_against_golden_and_oracle(algo):
    """host_crc.cpp (PCLMUL folding / crc32q / slice-by-8) vs the reference-generated fixtures, and
    vs the oracle on every length 0..600, lengths around its fold thresholds, and random seeds and
    alignments."""
    import golden_util
    key = "crc32c" if algo == 0 else "crc32"
    for v in golden_util.load()["literal"]:
        assert ck.cpu_resume(algo, 0, golden_util.literal_bytes(v)) & 0xFFFFFFFF == int(v[key], 16), v["name"]
    fx = golden_util.load()["batch"]
    data = oracle.fill_splitmix64(fx["bytes"], fx["seed"])
    for i, (o, n, sd) in enumerate(zip(fx["offsets"], fx["lengths"], fx["seeds"])):
        got = ck.cpu_resume(algo, int(sd, 16), data[o:o + n]) & 0xFFFFFFFF
        assert got == int(fx[key][i], 16), i
    rng = np.random.default_rng(77 + algo)
    buf = rng.integers(0, 256, 1 << 17, dtype=np.uint8)
    lengths = list(range(0, 601)) + [1023, 1024, 1025, 1279, 1280, 1281, 4095, 4096, 4097, 65535, 65536, 100000]
    for n in lengths:
        off = int(rng.integers(0, 64))
        seed = int(rng.integers(0, 2**32))
        want = oracle.resume(algo, seed, buf[off:off + n])
        assert ck.cpu_resume(algo, seed, buf[off:off + n]) & 0xFFFFFFFF == want, n
    assert ck.cpu_impl() in ("vpclmul512+pclmul+sse4.2", "pclmul+sse4.2", "pclmul", "slice8")


@pytest.mark.parametrize("algo", [0, 1])
def test_cpu_route_golden_4096(algo):
    """The CPU route against the 4096-entry reference-generated set (lengths 0..70000, seeded)."""
    import golden_util
    fx = golden_util.load_4096()
    data = oracle.fill_splitmix64(fx["bytes"], fx["seed"])
    key = "crc32c" if algo == 0 else "crc32"
    for i in range(len(fx["lengths"])):
        o, n = int(fx["offsets"][i]), int(fx["lengths"][i])
        assert ck.cpu_resume(algo, int(fx["seeds"][i]), data[o:o + n]) & 0xFFFFFFFF == int(fx[key][i]), i


def test_cpu_route_threshold_setting():
    old = ck.get_cpu_route_max()
    try:
        ck.set_cpu_route_max(12345)
        assert ck.get_cpu_route_max() == 12345
    finally:
        ck.set_cpu_route_max(old)


def test_circe_config_compat():
    """Sse42Crc32C.allocConfig validation (crc32c_sse42_jni.cpp:50-72): >= 1 word, every word >= 4
    (chunk_config::min_words), strictly decreasing; 0 on failure, an opaque non-zero handle otherwise."""
    L = _native.lib()

    def alloc(words):
        a = np.array(words, dtype=np.int32)
        return L.bkd_circe_alloc_config(ctypes.c_void_p(a.ctypes.data if a.size else 0), a.size)

    assert L.bkd_circe_supported() == 1
    for bad in ([], [3], [4096, 4096], [64, 512], [4096, 512, 3], [-1]):
        assert alloc(bad) == 0, bad
    for good in ([4], [4096, 512, 64], [64, 4]):
        h = alloc(good)
        assert h != 0
        L.bkd_circe_free_config(h)
    L.bkd_circe_free_config(0)  # freeing the null config is a no-op, as delete[] of null


@pytest.mark.parametrize("algo", [0, 1])
def test_host_tables_against_oracle(algo):
    L = _native.lib()
    for lanes in (4, 8, 16, 32, 64):
        t = ck.host_tables(algo, lanes)
        bo = (2 + int(np.log2(lanes))) * 1024
        assert t.size == bo + 256 + 2048 + (128 * lanes if lanes in (4, 8) else 0)
        if lanes in (4, 8):  # lane-position nibble tables: (n << 4k) * x^(128 (lanes - 1 - g))
            lo = bo + 2304
            for g, k, nb in ((0, 0, 1), (lanes - 1, 7, 15), (1, 3, 9), (lanes - 2, 5, 4)):
                want = oracle.gf_mul(algo, nb << (4 * k), oracle.xpow8n(algo, 16 * (lanes - 1 - g)))
                assert t[lo + (16 * k + nb) * lanes + g] == want
        assert (t[bo:bo + 256] == oracle.table(algo)).all()  # ReflectedIntCrc.java:30-35
        for off, k in ((bo + 256, 8), (bo + 1280, 12)):  # x^64, x^96 operators
            assert t[off + 256 * 2 + 7] == oracle.gf_mul(algo, 7 << 16, oracle.xpow8n(algo, k))
        # main operator C = x^(128*lanes): every byte table entry is (b << 8t) * C mod P
        C = oracle.xpow8n(algo, 16 * lanes)
        for tb in range(4):
            for b in (0, 1, 0x80, 0xFF, 0x5A):
                assert t[tb * 256 + b] == oracle.gf_mul(algo, b << (8 * tb), C)
    rng = np.random.default_rng(algo)
    for _ in range(50):
        a, b = (int(x) for x in rng.integers(0, 2**32, 2))
        assert L.bkd_host_gf_mul(algo, a, b) == oracle.gf_mul(algo, a, b)
    for n in (0, 1, 4, 16, 4096, 65536, 10**9):
        assert L.bkd_host_xpow8n(algo, n) == oracle.xpow8n(algo, n)


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("lanes", [4, 8, 16, 64])
def test_kernel_decomposition_model(algo, lanes):
    model = KernelModel(ck.host_tables(algo, lanes), lanes)
    rng = np.random.default_rng(lanes + algo)
    for n in [0, 1, 3, 4, 5, 15, 16, 17, 31, 32, 33, 64, 100, 16 * lanes - 1, 16 * lanes, 16 * lanes + 1, 2500]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, int(rng.integers(0, 2**32))):
            assert model.crc(d, seed) == oracle.resume(algo, seed, d), (n, seed)


def test_group_lane_policy():
    L = _native.lib()
    assert ck.set_group_lanes(8) is None
    assert L.bkd_get_group_lanes(0, 4096) == 8
    ck.set_group_lanes(0)
    assert L.bkd_get_group_lanes(0, 4096) in (4, 8, 16)
    with pytest.raises(_native.BkdError):
        ck.set_group_lanes(3)


@pytest.mark.parametrize("algo", [0, 1])
def test_plan_chunk_combine_model(algo):
    """The plan's end-aligned chunking + X = x^(8*CH) Horner combine reproduces the oracle."""
    tabs = ck.host_tables(algo, 4)
    rng = np.random.default_rng(algo + 10)
    jc = 4  # CH = 256 B so that small inputs span many chunks
    for n in [0, 1, 15, 16, 17, 31, 32, 33, 255, 256, 257, 270, 271, 272, 511, 512, 513, 527, 1000, 1283]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        seed = int(rng.integers(0, 2**32))
        for mis in (0, 1, 7, 15, 100, 127):
            got = plan_model(tabs, lambda nb: oracle.xpow8n(algo, nb), lambda a, b: oracle.gf_mul(algo, a, b), d,
                             seed, lanes=4, jc=jc, mis=mis)
            assert got == oracle.resume(algo, seed, d), (n, mis)


@pytest.mark.parametrize("algo", [0, 1])
def test_segments_join_model(algo):
    """bkd_crc_batch_segments' join (plan_kernels.hpp segments_combine_kernel) on CPU: each segment's
    zero-initialised register is ~resume(~0, segment) (the indexed path with seed ~0); the entry is
    reg = ~seed, then per non-empty segment reg = reg * x^(8 len) ^ raw, the power taken as the
    product of x^(8 * 2^b) over the set bits of len — equal to resume(seed, concatenation)."""
    rng = np.random.default_rng(40 + algo)
    pw = [oracle.xpow8n(algo, 1 << b) for b in range(32)]
    for _ in range(40):
        segs = [rng.integers(0, 256, int(rng.choice([0, 1, 3, 16, 100, 4097])), dtype=np.uint8).tobytes()
                for _ in range(int(rng.integers(0, 6)))]
        seed = int(rng.integers(0, 2**32))
        reg = (~seed) & 0xFFFFFFFF
        for sg in segs:
            if not sg:
                continue
            raw = (~oracle.resume(algo, 0xFFFFFFFF, sg)) & 0xFFFFFFFF
            n = len(sg)
            for b in range(32):
                if (n >> b) & 1:
                    reg = oracle.gf_mul(algo, pw[b], reg)
            reg ^= raw
        assert (~reg) & 0xFFFFFFFF == oracle.resume(algo, seed, b"".join(segs))


def test_host_batch_wrapper_validates_index_sizes():
    """crc_batch_host refuses index arrays shorter than the batch before the library reads them."""
    data = bytes(1000)
    with pytest.raises(ValueError):
        ck.crc_batch_host(ck.CRC32C, data, [0, 10, 20], [5, 5])
    with pytest.raises(ValueError):
        ck.crc_batch_host(ck.CRC32C, data, [0, 10], [5, 5], seeds=[1])


def test_host_release_and_route_knobs_without_device():
    """bkd_host_release with nothing staged, route and thread knobs: validation and round trips."""
    L = _native.lib()
    assert L.bkd_host_release() == 0
    assert L.bkd_set_host_batch_route(3) == -1 and L.bkd_set_host_batch_route(-1) == -1
    assert L.bkd_set_host_threads(-2) == -1
    assert L.bkd_set_host_threads(1) == 0 and L.bkd_get_host_threads() == 1
    assert L.bkd_set_host_threads(0) == 0 and L.bkd_get_host_threads() >= 1
    with ck.host_batch_route(ck.HOST_ROUTE_CPU):
        assert ck.get_host_batch_route() == ck.HOST_ROUTE_CPU
