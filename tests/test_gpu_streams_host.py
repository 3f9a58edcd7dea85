"""GPU: per-stream bounds reporting, stream-ordered per-call resumes, the CPU/GPU per-call routes,
and the host-resident DigestManager batches (BatchedReadOp / PendingAddOp with entries in host
memory), all bit-exact against the oracle."""
import ctypes
import threading

import numpy as np
import pytest

import oracle
from bookkeeper_amd import checksum as ck
from bookkeeper_amd import digest as dg
from bookkeeper_amd._native import BkdError, lib

pytestmark = pytest.mark.gpu


def _dev(torch, a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def test_bounds_flag_is_per_stream(gpu):
    """include/bkdigest.h: an out-of-range entry is reported by bkd_stream_sync of the stream it was
    enqueued on, and only there (one flag per stream, read and cleared in stream order)."""
    import torch
    rng = np.random.default_rng(5)
    size = 1 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    base = _dev(torch, host, gpu)
    n = 5000
    offs = rng.integers(0, size - 4096, n).astype(np.int64)
    lens = rng.integers(0, 4096, n).astype(np.int32)
    bad_offs = offs.copy()
    bad_offs[1234] = size - 10  # 10 bytes left, entry wants more
    lens_bad = lens.copy()
    lens_bad[1234] = 4000
    want = oracle.batch(0, host, offs.astype(np.uint64), lens.astype(np.uint32))
    results = {}
    barrier = threading.Barrier(2)

    def worker(name, o, l):
        s = torch.cuda.Stream(device=gpu)
        d_off, d_len = _dev(torch, o, gpu), _dev(torch, l, gpu)
        torch.cuda.synchronize()
        barrier.wait()
        try:
            for _ in range(20):
                out = ck.crc_batch(0, base, d_off, d_len, stream=s)
            ck.check(lib().bkd_stream_sync(ck._stream_ptr(s)))
            results[name] = ("ok", out.cpu().numpy().view(np.uint32))
        except BkdError as e:
            results[name] = ("err", e.code)

    for mode in (1, 2):  # direct kernel and chunked plan both raise the flag
        ck.set_plan_mode(mode)
        ts = [threading.Thread(target=worker, args=("bad", bad_offs, lens_bad)),
              threading.Thread(target=worker, args=("good", offs, lens))]
        try:
            for t in ts:
                t.start()
            for t in ts:
                t.join(timeout=120)
        finally:
            ck.set_plan_mode(0)
        assert results["bad"] == ("err", -4), mode
        assert results["good"][0] == "ok", mode
        assert (results["good"][1] == want).all()


def test_stream_release_frees_and_restarts(gpu):
    """bkd_stream_release: waits for the stream, reports its pending bounds flag, frees its scratch;
    streams created afterwards (whatever handle they get) run indexed batches correctly."""
    import torch
    rng = np.random.default_rng(11)
    size = 4 << 20
    host = rng.integers(0, 256, size, dtype=np.uint8)
    base = _dev(torch, host, gpu)
    n = 20000
    offs = rng.integers(0, size - 70000, n).astype(np.int64)
    lens = rng.integers(0, 70000, n).astype(np.int32)
    want = oracle.batch(0, host, offs.astype(np.uint64), lens.astype(np.uint32))
    d_off, d_len = _dev(torch, offs, gpu), _dev(torch, lens, gpu)
    bad_off = d_off.clone()
    bad_off[7] = size - 3
    torch.cuda.synchronize()  # inputs were made on the current stream; the batches run on others
    for rnd in range(4):
        s = torch.cuda.Stream(device=gpu)
        out = ck.crc_batch(0, base, d_off, d_len, stream=s)
        if rnd % 2:
            ck.crc_batch(0, base, bad_off, d_len, stream=s)
            with pytest.raises(BkdError) as ei:
                ck.release_stream(s)
            assert ei.value.code == -4
        else:
            ck.release_stream(s)
        assert (out.cpu().numpy().view(np.uint32) == want).all(), rnd
        del s
    ck.release_stream(torch.cuda.current_stream(gpu))  # the current stream's scratch, if it had any
    out = ck.crc_batch(0, base, d_off, d_len)  # ... is made again by its next call
    assert (out.cpu().numpy().view(np.uint32) == want).all()
    # the flag was cleared by the sync that reported it
    s = torch.cuda.Stream(device=gpu)
    ck.crc_batch(0, base, _dev(torch, offs, gpu), _dev(torch, lens, gpu), stream=s, sync_check=True)


def test_resume_device_is_ordered_after_the_producer(gpu):
    """a per-call resume of a tensor written by a still-queued kernel must see the
    new bytes. The producer is queued behind a long matmul on the current stream; no explicit sync."""
    import torch
    h = ck.GpuIntHash(ck.CRC32C)
    a = torch.randn(4096, 4096, device=gpu)
    for trial in range(3):
        buf = torch.zeros(1 << 20, dtype=torch.uint8, device=gpu)
        torch.cuda.synchronize()
        for _ in range(4):
            a = a @ a  # keep the stream busy
            a = a / a.abs().max()
        buf.fill_(0x5A + trial)  # the producer, queued after the matmuls
        got = h.calculate(buf)
        want = oracle.calculate(0, np.full(1 << 20, 0x5A + trial, dtype=np.uint8))
        assert got & 0xFFFFFFFF == want, trial
    # a side stream producer with the resume on that stream
    s = torch.cuda.Stream(device=gpu)
    with torch.cuda.stream(s):
        buf2 = torch.full((70000,), 7, dtype=torch.uint8, device=gpu)
        for _ in range(2):
            a = a @ a
        buf2.add_(1)
        got = h.calculate(buf2)
    assert got & 0xFFFFFFFF == oracle.calculate(0, np.full(70000, 8, dtype=np.uint8))


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_per_call_routes_agree(gpu, algo):
    """bkd_resume_host: CPU route (<= cpu_route_max) and GPU route (threshold 0) give the oracle's
    value; bkd_resume (pointer lookup) on host and device buffers too."""
    import ctypes
    import torch
    rng = np.random.default_rng(11 + algo)
    h = ck.GpuIntHash(algo)
    old = ck.get_cpu_route_max()
    try:
        for n in (1, 15, 16, 63, 64, 100, 4096, 65537, 1 << 20, (3 << 20) + 5):
            data = rng.integers(0, 256, n, dtype=np.uint8)
            seed = int(rng.integers(0, 2**32))
            want = oracle.resume(algo, seed, data)
            for route_max in (0, 1 << 62):  # 0: GPU via pinned staging; huge: CPU
                ck.set_cpu_route_max(route_max)
                assert h.resume(seed, data) & 0xFFFFFFFF == want, (n, route_max)
                out = ctypes.c_uint32(0)
                ck.check(lib().bkd_resume(algo, seed, ctypes.c_void_p(data.ctypes.data), n, ctypes.byref(out)))
                assert out.value == want
            d = _dev(torch, data, gpu)
            assert h.resume(seed, d) & 0xFFFFFFFF == want
            out = ctypes.c_uint32(0)
            ck.check(lib().bkd_resume(algo, seed, ctypes.c_void_p(d.data_ptr()), n, ctypes.byref(out)))
            assert out.value == want
    finally:
        ck.set_cpu_route_max(old)


def test_package_batch_reports_out_of_range_payload(gpu):
    import torch
    dm = dg.DigestManager.instantiate(3, b"", dg.DigestType.CRC32C)
    n = 64
    payload = torch.zeros(n * 100, dtype=torch.uint8, device=gpu)
    ids = torch.arange(n, dtype=torch.int64, device=gpu)
    offs = ids * 100
    lens = torch.full((n,), 100, dtype=torch.int32, device=gpu)
    dm.package_batch(ids, ids - 1, ids, payload, offs, lens, sync_check=True)
    lens[n - 1] = 101  # one byte past the payload buffer
    with pytest.raises(BkdError) as e:
        dm.package_batch(ids, ids - 1, ids, payload, offs, lens, sync_check=True)
    assert e.value.code == -4


def test_batch_wrappers_validate_out_and_seeds(gpu):
    import torch
    base = torch.zeros(4096, dtype=torch.uint8, device=gpu)
    offs = torch.zeros(8, dtype=torch.int64, device=gpu)
    lens = torch.full((8,), 16, dtype=torch.int32, device=gpu)
    with pytest.raises(ValueError):
        ck.crc_batch(0, base, offs, lens, out=torch.empty(4, dtype=torch.int32, device=gpu))
    with pytest.raises(TypeError):
        ck.crc_batch(0, base, offs, lens, seeds=torch.zeros(8, dtype=torch.int64, device=gpu))
    with pytest.raises(TypeError):
        ck.crc_batch_uniform(0, base, 16, 8, out=torch.empty(8, dtype=torch.int64, device=gpu))
    with pytest.raises(ValueError):
        ck.crc_batch_uniform(0, base, 16, 8, seeds=torch.zeros(4, dtype=torch.int32, device=gpu))


def _frames(algo, rng, n, ledger, first_id, max_payload):
    frames = []
    for i in range(n):
        size = int(rng.choice([0, 1, 5, 31, 100, 4096 - 36, int(rng.integers(0, max_payload))]))
        payload = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        digest, hdr = oracle.digest_entry(algo, ledger, first_id + i, first_id + i - 1, size, payload)
        frames.append(bytearray(hdr + oracle.digest_bytes(algo, digest) + payload))
    return frames


@pytest.mark.parametrize("algo,dtype", [(ck.CRC32C, dg.DigestType.CRC32C), (ck.CRC32, dg.DigestType.CRC32)])
def test_verify_batch_host_matches_oracle(gpu, algo, dtype):
    """BatchedReadOp.complete (BatchedReadOp.java:164-190) over a ByteBufList in host memory: every
    entry's status equals oracle.verify_entry's, first_bad is the verified prefix."""
    rng = np.random.default_rng(21 + algo)
    ledger, first = 99, 1000
    dm = dg.DigestManager.instantiate(ledger, b"", dtype)
    frames = _frames(algo, rng, 3000, ledger, first, 9000)
    st, fb = dm.verify_batch_host(frames, first)
    assert (st == 0).all() and fb == len(frames)
    # corruptions: payload byte, digest byte, ledger id, entry id, truncated frame
    frames[2500][-1 if len(frames[2500]) > 40 + dm.macCodeLength else 33] ^= 0x40
    frames[1700][32] ^= 1
    frames[2100][7] ^= 1  # ledger id (BE, last byte)
    frames[2900][15] ^= 1  # entry id
    frames[2950] = frames[2950][:20]
    st, fb = dm.verify_batch_host(frames, first)
    want = np.array([oracle.verify_entry(algo, bytes(f), ledger, first + i) for i, f in enumerate(frames)])
    assert (st == want).all()
    assert fb == 1700
    st, fb = dm.verify_batch_host(frames[:1700], first)
    assert fb == 1700 and (st == 0).all()


def test_verify_batch_host_concurrent_callers(gpu):
    """§8b threading: read completions verify their ByteBufLists from several threads at once; each
    caller takes a staging set of its own (more callers than sets wait for one); every status and
    verified prefix equals the oracle's."""
    algo = ck.CRC32C
    ledger, first = 17, 500
    dm = dg.DigestManager.instantiate(ledger, b"", dg.DigestType.CRC32C)
    rng = np.random.default_rng(91)
    batches = []
    for k in range(10):
        frames = _frames(algo, rng, 200 + 37 * k, ledger, first, 6000)
        bad = int(rng.integers(0, len(frames)))
        if k % 2:
            frames[bad][-1 if len(frames[bad]) > 40 else 33] ^= 0x10
        want = np.array([oracle.verify_entry(algo, bytes(f), ledger, first + i) for i, f in enumerate(frames)])
        nz = np.nonzero(want)[0]
        batches.append((frames, want, int(nz[0]) if nz.size else len(frames)))
    errors = []
    barrier = threading.Barrier(len(batches))

    def worker(k):
        frames, want, fb_want = batches[k]
        try:
            barrier.wait()
            for _ in range(5):
                st, fb = dm.verify_batch_host(frames, first)
                assert (st == want).all() and fb == fb_want, k
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(len(batches))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors


def test_verify_batch_host_many_segments(gpu):
    """> 64 MiB of frames: several double-buffered segments; the first bad entry in a later segment."""
    algo = ck.CRC32C
    n, L = 40000, 4096  # ~156 MiB
    ledger = 5
    dm = dg.DigestManager.instantiate(ledger, b"", dg.DigestType.CRC32C)
    big = oracle.fill_splitmix64(n * L, 42).reshape(n, L)
    plen = L - 36
    for i in range(n):
        d, hdr = oracle.digest_entry(algo, ledger, i, i - 1, plen, big[i, 36:])
        big[i, :32] = np.frombuffer(hdr, dtype=np.uint8)
        big[i, 32:36] = np.frombuffer(oracle.digest_bytes(algo, d), dtype=np.uint8)
    frames = [big[i] for i in range(n)]
    st, fb = dm.verify_batch_host(frames, 0)
    assert fb == n and (st == 0).all()
    big[31000, 2000] ^= 0xFF
    big[39999, 100] ^= 0xFF
    st, fb = dm.verify_batch_host(frames, 0)
    assert fb == 31000
    assert set(np.nonzero(st)[0].tolist()) == {31000, 39999}


@pytest.mark.parametrize("algo,dtype", [(ck.CRC32C, dg.DigestType.CRC32C), (ck.CRC32, dg.DigestType.CRC32)])
@pytest.mark.parametrize("stride", [None, 64])
def test_package_batch_host_matches_oracle(gpu, algo, dtype, stride):
    """PendingAddOp's packaging (DigestManager.java:117-181) of host payloads in one call: header and
    digest bytes equal oracle.digest_entry's for every entry, across several segments."""
    rng = np.random.default_rng(31 + algo)
    ledger = 12345
    dm = dg.DigestManager.instantiate(ledger, b"", dtype)
    n = 20000
    sizes = rng.choice([0, 1, 17, 1000, 4060, 9000], n)
    sizes[-5:] = 70000
    payloads = [rng.integers(0, 256, int(s), dtype=np.uint8) for s in sizes]
    ids = np.arange(n, dtype=np.int64) + 77
    lacs = ids - 1
    lf = np.cumsum(sizes).astype(np.int64)
    frames, digests = dm.package_batch_host(ids, lacs, lf, payloads, frame_stride=stride)
    mac = dm.macCodeLength
    for i in range(0, n, 7):
        d, hdr = oracle.digest_entry(algo, ledger, int(ids[i]), int(lacs[i]), int(lf[i]), payloads[i])
        assert digests[i] == d, i
        assert bytes(frames[i, :32]) == hdr
        assert bytes(frames[i, 32:32 + mac]) == oracle.digest_bytes(algo, d)


@pytest.mark.parametrize("small", [0, 16, 100, 192, 400, 512])
def test_plan_short_entry_class(gpu, small):
    """Indexed batches through the plan with the short-entry class at several bounds: every length
    0..700 packed at odd offsets, seeded, plus out-of-range entries on both sides of the bound — the
    short launch and the plan together give the oracle's digests and one bounds report."""
    import torch
    rng = np.random.default_rng(50 + small)
    lens = np.concatenate([np.arange(0, 701), rng.integers(0, 1000, 3000)]).astype(np.int64)
    rng.shuffle(lens)
    offs = np.concatenate([[3], 3 + np.cumsum(lens[:-1])]).astype(np.int64)
    size = int(offs[-1] + lens[-1]) + 100_000  # > 256 KiB (the plan path), < 1 KiB per entry (the short class)
    assert size > 256 << 10 and size <= 1024 * lens.size
    host = rng.integers(0, 256, size, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    want = oracle.batch(0, host, offs.astype(np.uint64), lens.astype(np.uint32), seeds=seeds)
    base = _dev(torch, host, gpu)
    d_seeds = _dev(torch, seeds.view(np.int32), gpu)
    ck.set_plan_mode(2)
    ck.set_plan_small(small)
    try:
        out = ck.crc_batch(0, base, _dev(torch, offs, gpu), _dev(torch, lens.astype(np.int32), gpu), seeds=d_seeds,
                           sync_check=True)
        assert (out.cpu().numpy().view(np.uint32) == want).all()
        bad_o = offs.copy()
        bad_l = lens.copy()
        bad_o[10], bad_l[10] = size - 5, 50     # short class, out of range
        bad_o[20], bad_l[20] = size - 5, 900    # plan class, out of range
        with pytest.raises(BkdError) as e:
            ck.crc_batch(0, base, _dev(torch, bad_o, gpu), _dev(torch, bad_l.astype(np.int32), gpu), seeds=d_seeds,
                         sync_check=True)
        assert e.value.code == -4
        # only short entries: the plan kernels find no work of their own
        m = (size - 1) // 37
        sl = np.full(m, 37, dtype=np.int64)
        so = np.arange(m, dtype=np.int64) * 37 + 1
        out = ck.crc_batch(0, base, _dev(torch, so, gpu), _dev(torch, sl.astype(np.int32), gpu), sync_check=True)
        want2 = oracle.batch(0, host, so.astype(np.uint64), sl.astype(np.uint32))
        assert (out.cpu().numpy().view(np.uint32) == want2).all()
    finally:
        ck.set_plan_mode(0)
        ck.set_plan_small(192)


@pytest.mark.parametrize("lo,hi", [(3600, 4096), (4096, 4096), (3000, 4096), (1200, 1300)])
def test_plan_near_uniform_lengths(gpu, lo, hi):
    """Plan-path batches whose lengths all lie within 1/16 (+ 64 B) of the first entry's skip the
    chunks: the chunk kernel computes each entry whole (PlanRun::uniform). Both sides of that band
    give the oracle's digests, seeded, and an out-of-range entry is still reported."""
    import torch
    rng = np.random.default_rng(lo + hi)
    n = 6000
    lens = rng.integers(lo, hi + 1, n).astype(np.int64)
    offs = np.concatenate([[5], 5 + np.cumsum(lens[:-1] + 3)]).astype(np.int64)
    size = int(offs[-1] + lens[-1]) + 777
    host = rng.integers(0, 256, size, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    base = _dev(torch, host, gpu)
    d_seeds = _dev(torch, seeds.view(np.int32), gpu)
    ck.set_plan_mode(2)
    try:
        for algo in (0, 1):
            want = oracle.batch(algo, host, offs.astype(np.uint64), lens.astype(np.uint32), seeds=seeds)
            out = ck.crc_batch(algo, base, _dev(torch, offs, gpu), _dev(torch, lens.astype(np.int32), gpu),
                               seeds=d_seeds, sync_check=True)
            assert (out.cpu().numpy().view(np.uint32) == want).all(), algo
        bad_o = offs.copy()
        bad_o[n // 2] = size - 100
        with pytest.raises(BkdError) as e:
            ck.crc_batch(0, base, _dev(torch, bad_o, gpu), _dev(torch, lens.astype(np.int32), gpu), seeds=d_seeds,
                         sync_check=True)
        assert e.value.code == -4
    finally:
        ck.set_plan_mode(0)


@pytest.mark.parametrize("serial", [16, 40, 64])
def test_plan_serial_entries(gpu, serial):
    """Plan entries shorter than the serial bound are computed by the combine kernel, one thread each
    (slice-by-16 over windows cut from aligned 16-byte blocks): every length 0..300 at every start
    alignment mod 16, seeded, both algorithms, plus an entry ending at the buffer's last byte."""
    import torch
    rng = np.random.default_rng(serial)
    lens = np.tile(np.arange(0, 301), 16).astype(np.int64)
    offs = rng.integers(0, 1 << 20, lens.size).astype(np.int64)
    offs = offs - (offs & 15) + np.repeat(np.arange(16), 301)  # every alignment for every length
    size = (1 << 20) + 512
    lens = np.concatenate([lens, [200, 255]])
    offs = np.concatenate([offs, [size - 200, size - 255]])  # last bytes of the buffer
    host = rng.integers(0, 256, size, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    base = _dev(torch, host, gpu)
    d_seeds = _dev(torch, seeds.view(np.int32), gpu)
    ck.set_plan_mode(2)
    ck.set_plan_small(0)
    ck.set_plan_serial(serial)
    try:
        for algo in (0, 1):
            want = oracle.batch(algo, host, offs.astype(np.uint64), lens.astype(np.uint32), seeds=seeds)
            out = ck.crc_batch(algo, base, _dev(torch, offs, gpu), _dev(torch, lens.astype(np.int32), gpu),
                               seeds=d_seeds, sync_check=True)
            got = out.cpu().numpy().view(np.uint32)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (algo, lens[bad[:5]], offs[bad[:5]] & 15)
    finally:
        ck.set_plan_mode(0)
        ck.set_plan_small(192)
        ck.set_plan_serial(16)


def test_plan_short_entries_among_long(gpu):
    """Short entries among long ones (the base buffer holds > 1 KiB per entry, so no short-entry
    launch): they are one-step chunks of the plan. Mixed lengths (0..192 and 3..9 KiB, shuffled),
    seeded, both algorithms; an out-of-range short entry is reported; a batch of nearly equal short
    entries spread over the large buffer takes the uniform route with the same digests."""
    import torch
    rng = np.random.default_rng(71)
    short = rng.integers(0, 193, 3000)
    long_ = rng.integers(3000, 9000, 1500)
    lens = np.concatenate([short, long_, np.arange(0, 193)]).astype(np.int64)
    rng.shuffle(lens)
    offs = np.concatenate([[11], 11 + np.cumsum(lens[:-1] + rng.integers(0, 40, lens.size - 1))]).astype(np.int64)
    size = int(offs[-1] + lens[-1]) + 513
    assert size > 1024 * lens.size  # no short-entry launch
    host = rng.integers(0, 256, size, dtype=np.uint8)
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    base = _dev(torch, host, gpu)
    d_seeds = _dev(torch, seeds.view(np.int32), gpu)
    ck.set_plan_mode(2)
    try:
        for algo in (0, 1):
            want = oracle.batch(algo, host, offs.astype(np.uint64), lens.astype(np.uint32), seeds=seeds)
            out = ck.crc_batch(algo, base, _dev(torch, offs, gpu), _dev(torch, lens.astype(np.int32), gpu),
                               seeds=d_seeds, sync_check=True)
            got = out.cpu().numpy().view(np.uint32)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (algo, lens[bad[:5]])
        k = int(np.nonzero((lens > 20) & (lens < 150))[0][0])
        bad_o = offs.copy()
        bad_o[k] = size - 5
        with pytest.raises(BkdError) as e:
            ck.crc_batch(0, base, _dev(torch, bad_o, gpu), _dev(torch, lens.astype(np.int32), gpu), seeds=d_seeds,
                         sync_check=True)
        assert e.value.code == -4
        # nearly equal short entries spread over the large buffer: uniform route
        n2 = 5000
        l2 = rng.integers(100, 110, n2).astype(np.int64)
        o2 = np.sort(rng.choice(size - 200, n2, replace=False)).astype(np.int64)
        want = oracle.batch(0, host, o2.astype(np.uint64), l2.astype(np.uint32))
        out = ck.crc_batch(0, base, _dev(torch, o2, gpu), _dev(torch, l2.astype(np.int32), gpu), sync_check=True)
        assert (out.cpu().numpy().view(np.uint32) == want).all()
    finally:
        ck.set_plan_mode(0)


def test_host_release_frees_idle_staging_and_restarts(gpu):
    """the GPU route's pinned staging sets can be released (bkd_host_release) by a
    long-lived process; the next host-resident batch through the GPU creates them again and stays
    exact, for verify (first_bad word only) and package (aux + frame buffers)."""
    algo = ck.CRC32C
    ledger, first = 3, 10
    dm = dg.DigestManager.instantiate(ledger, b"", dg.DigestType.CRC32C)
    rng = np.random.default_rng(123)
    frames = _frames(algo, rng, 500, ledger, first, 5000)
    want = np.array([oracle.verify_entry(algo, bytes(f), ledger, first + i) for i, f in enumerate(frames)])
    with ck.host_batch_route(ck.HOST_ROUTE_GPU):
        for _ in range(2):
            st, fb = dm.verify_batch_host(frames, first)
            assert (st == want).all() and fb == len(frames)
            payloads = [bytes(f[36:]) for f in frames]
            ids = np.arange(len(frames), dtype=np.int64) + first
            hdrs, digests = dm.package_batch_host(ids, ids - 1, np.array([len(p) for p in payloads]), payloads)
            for i in range(0, len(frames), 37):
                assert bytes(hdrs[i]) == bytes(frames[i][:36])
            ck.host_release()


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_long_host_entries_gpu_route_repeated(gpu, algo):
    """Host entries longer than a staging segment (64 MiB) through the GPU route: cut into pieces,
    pipelined and joined on the host; an unsorted index takes the one-copy route. Each call is
    repeated — the one-copy route once reused stream-ordered allocations and went wrong from the
    second call on (profiles/r03l_*). The per-call resume of a 150 MiB buffer on the GPU route too."""
    M = 1 << 20
    rng = np.random.default_rng(60 + algo)
    host = np.frombuffer(rng.bytes(200 * M), dtype=np.uint8)
    offs = np.array([0, 5, 64 * M + 9, 150 * M], np.uint64)
    lens = np.array([3, 64 * M + 1, 85 * M + 3, 50 * M], np.uint32)
    seeds = rng.integers(0, 2**32, offs.size, dtype=np.uint64).astype(np.uint32)
    want = np.array([ck.cpu_resume(algo, int(s), host[int(o):int(o) + int(l)]) & 0xFFFFFFFF
                     for o, l, s in zip(offs, lens, seeds)], np.uint32)
    with ck.host_batch_route(ck.HOST_ROUTE_GPU):
        for _ in range(3):
            assert (ck.crc_batch_host(algo, host, offs, lens, seeds=seeds) == want).all()
            perm = np.array([2, 0, 3, 1])  # unsorted: the one-copy route
            assert (ck.crc_batch_host(algo, host, offs[perm], lens[perm], seeds=seeds[perm]) == want[perm]).all()
        old = ck.get_cpu_route_max()
        ck.set_cpu_route_max(0)
        try:
            buf = host[7:7 + 150 * M]
            w = ck.cpu_resume(algo, 0xABCD, buf) & 0xFFFFFFFF
            for _ in range(2):
                out = ctypes.c_uint32(0)
                assert lib().bkd_resume_host(algo, 0xABCD, ctypes.c_void_p(buf.ctypes.data), ctypes.c_uint64(buf.size),
                                             ctypes.byref(out)) == 0
                assert out.value == w
        finally:
            ck.set_cpu_route_max(old)


def test_oversize_frames_take_the_cpu_route_when_automatic(gpu):
    """A framed host batch holding a frame longer than a staging segment (64 MiB): the automatic route
    verifies / packages it on the CPU even where it would pick the GPU (one host thread); the route
    forced to the GPU refuses it (BKD_ERR_INVALID_ARG), never a wrong status."""
    M = 1 << 20
    rng = np.random.default_rng(77)
    payload = np.frombuffer(rng.bytes(65 * M + 3), dtype=np.uint8)
    dm = dg.DigestManager.instantiate(5, b"", dg.DigestType.CRC32C)
    d, hdr = oracle.digest_entry(ck.CRC32C, 5, 9, 8, payload.size, payload.tobytes())
    frame = bytearray(hdr + oracle.digest_bytes(ck.CRC32C, d) + payload.tobytes())
    small = bytearray(frame[:40])  # header + digest of the long frame, no payload: digest mismatch
    ck.set_host_threads(1)
    try:
        with ck.host_batch_route(ck.HOST_ROUTE_AUTO):
            st, fb = dm.verify_batch_host([frame, small], 9, skip_entry_check=True)
            assert st.tolist() == [0, 2] and fb == 1
            frames, digests = dm.package_batch_host(np.array([9]), np.array([8]), np.array([payload.size]), [payload])
            assert digests[0] == d and bytes(frames[0, :32]) == hdr
        with ck.host_batch_route(ck.HOST_ROUTE_GPU):
            with pytest.raises(BkdError):
                dm.verify_batch_host([frame], 9)
    finally:
        ck.set_host_threads(0)
