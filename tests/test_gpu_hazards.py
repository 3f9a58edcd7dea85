"""GPU: digests must not depend on memory the call does not own, nor on the allocation history.

* Bytes outside every entry — the pad up to the 128-byte line the plan's chunks read past an entry's
  end, and the bytes past ``base_size`` — are rewritten by another stream WHILE a full-size config-3
  Zipf batch runs, and re-randomised between calls; every digest must still equal the reference's
  (the C-ABI borrow contract, include/bkdigest.h: only [offsets[i], offsets[i] + lengths[i]) is the
  caller's entry).
* The round-3 wrong-digest shape: repeated one-entry 128 MiB host calls through the GPU route, the
  unsorted one-copy route, and device calls of the same entry through the plan (VERDICT r03 item 1,
  DESIGN.md §5a).
* Overlapping host entries around an entry longer than a staging segment.
Reference arithmetic: circe crc32c() ($CN/cpp/crc32c_sse42.cpp:184-217) through oracle/_ref, zlib
for CRC32.
"""
import ctypes

import numpy as np
import pytest

import oracle
from bookkeeper_amd import _native
from bookkeeper_amd import checksum as ck

pytestmark = pytest.mark.gpu


def _reference(algo, host, offs, lens):
    """Every digest on the host (threaded reference for CRC32C, zlib for CRC32; see test_gpu_parity)."""
    from test_gpu_parity import _threaded_reference
    return _threaded_reference(algo, host, offs, lens)[0]


def test_zipf_outside_bytes_rewritten_during_the_call(gpu):
    import torch
    from bench import zipf_index
    offs0, lens = zipf_index(1 << 20)
    rng = np.random.default_rng(404)
    # every entry is followed by 1..127 bytes that belong to no entry, so entry ends are unaligned
    # and the 128-byte line past each end holds foreign bytes
    gaps = rng.integers(1, 128, lens.size)
    offs = np.zeros(lens.size, dtype=np.int64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.int64) + gaps[:-1])
    size = int(offs[-1] + lens[-1]) + 45  # base_size: not a multiple of 128
    assert size % 128 != 0
    big = torch.empty(size + 4096, dtype=torch.uint8, device=gpu)  # bytes past base_size exist
    ck.fill_splitmix64(big, 4242)
    base = big[:size]
    starts = torch.from_numpy(offs).to(gpu)
    # entry bytes: +1 at each start, -1 at each end (all distinct: lengths >= 64, gaps >= 1), prefix
    # sum 1 inside an entry and 0 elsewhere
    edge = torch.zeros(big.numel(), dtype=torch.int8, device=gpu)
    edge[starts] = 1
    edge[starts + torch.from_numpy(lens.astype(np.int64)).to(gpu)] = -1
    foreign = torch.cumsum(edge, 0, dtype=torch.int8) == 0
    del edge
    assert int(foreign[size:].sum()) == big.numel() - size
    pristine = big.clone()
    noise = [torch.randint(0, 256, big.shape, dtype=torch.uint8, device=gpu) for _ in range(2)]
    host = base.cpu().numpy()
    d_off = starts
    d_len = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    side = torch.cuda.Stream(device=gpu)
    main = torch.cuda.current_stream(gpu)

    def scribble(k):
        # entry bytes are rewritten with their own values (unobservable); foreign bytes change
        with torch.cuda.stream(side):
            torch.where(foreign, noise[k & 1], pristine, out=big)

    try:
        for algo in (ck.CRC32C, ck.CRC32):
            want = _reference(algo, host, offs, lens)
            for mode in (0, 2):  # automatic (the bench's route) and the chunked plan forced
                ck.set_plan_mode(mode)
                for rep in range(3):
                    scribble(rep)  # re-randomised between calls ...
                    main.wait_stream(side)
                    for k in range(6):  # ... and rewritten on another stream during the call
                        scribble(rep + k + 1)
                    got = ck.crc_batch(algo, base, d_off, d_len, sync_check=True)
                    torch.cuda.synchronize(gpu)
                    got = got.cpu().numpy().view(np.uint32)
                    bad = np.nonzero(got != want)[0]
                    assert bad.size == 0, (algo, mode, rep, bad.size, bad[:5].tolist(), lens[bad[:5]].tolist())
    finally:
        ck.set_plan_mode(0)


def test_repeated_128mib_entry_host_and_device(gpu):
    """The round-3 failing shape, repeated: one 128 MiB entry per call through the GPU host route
    (pieces through the staging pipeline), the one-copy route of an unsorted index spanning it, and
    the same bytes as a device entry through the plan. Every call equals the reference."""
    import torch
    L = _native.lib()
    M = 1 << 20
    host = oracle.fill_splitmix64(130 * M, 91)
    ent = host[:128 * M]
    want = {a: oracle.resume(a, 0, ent) for a in (ck.CRC32C, ck.CRC32)}
    half = 64 * M + 12345  # an unsorted pair covering the same bytes: [half, 128 MiB), [0, half)
    off2 = np.array([half, 0], dtype=np.uint64)
    len2 = np.array([128 * M - half, half], dtype=np.uint32)
    out2 = np.zeros(2, dtype=np.uint32)
    dev = torch.from_numpy(host).to(gpu)
    old = L.bkd_get_cpu_route_max()
    L.bkd_set_cpu_route_max(ctypes.c_uint64(0))
    try:
        for k in range(6):
            for algo in (ck.CRC32C, ck.CRC32):
                out = ctypes.c_uint32(0)
                assert L.bkd_resume_host(algo, 0, ctypes.c_void_p(ent.ctypes.data), ctypes.c_uint64(ent.size),
                                         ctypes.byref(out)) == 0
                assert out.value == want[algo], ("host", k, algo, hex(out.value))
                rc = L.bkd_crc_batch_host(algo, ctypes.c_void_p(host.ctypes.data), ctypes.c_uint64(host.size),
                                          off2.ctypes.data, len2.ctypes.data, 2, None, 0, out2.ctypes.data)
                assert rc == 0
                # joining the two halves gives the whole entry
                assert oracle.combine(algo, int(out2[1]), int(out2[0]), int(len2[0])) == want[algo], ("oneshot", k)
                got = ck.GpuIntHash(algo).resume(0, dev[:128 * M]) & 0xFFFFFFFF
                assert got == want[algo], ("device", k, algo, hex(got))
                ck.set_plan_mode(2)
                try:
                    d_off = torch.zeros(1, dtype=torch.int64, device=gpu)
                    d_len = torch.full((1,), 128 * M, dtype=torch.int32, device=gpu)
                    got = ck.crc_batch(algo, dev, d_off, d_len, sync_check=True).cpu().numpy().view(np.uint32)[0]
                finally:
                    ck.set_plan_mode(0)
                assert got == want[algo], ("plan", k, algo, hex(int(got)))
    finally:
        L.bkd_set_cpu_route_max(ctypes.c_uint64(old))


def test_host_entry_inside_a_long_entry_gpu_route(gpu):
    """A = [0, 100 MiB) and B = [50 MiB, +1 MiB) through the GPU host route: B starts
    inside A's later pieces, so the piece list is not in offset order; the call must still be exact."""
    M = 1 << 20
    host = oracle.fill_splitmix64(101 * M, 17)
    offs = np.array([0, 50 * M, 100 * M], dtype=np.uint64)
    lens = np.array([100 * M, M, M - 5], dtype=np.uint32)
    seeds = np.array([1, 2, 3], dtype=np.uint32)
    out = np.zeros(3, dtype=np.uint32)
    L = _native.lib()
    assert L.bkd_get_host_batch_route() == 2  # the gpu fixture forces the GPU route
    for algo in (ck.CRC32C, ck.CRC32):
        rc = L.bkd_crc_batch_host(algo, ctypes.c_void_p(host.ctypes.data), ctypes.c_uint64(host.size),
                                  offs.ctypes.data, lens.ctypes.data, 3, seeds.ctypes.data, 0, out.ctypes.data)
        assert rc == 0, _native.last_error()
        assert (out == oracle.batch(algo, host, offs, lens, seeds)).all()
