"""GPU: the stream route for ragged indexed batches (CPU model of the same
decomposition: tests/stream_model.py RangeModel) against the oracle, forced (plan mode 3) and
automatic, on the layouts the index allows: packed (config 3's shape), packed with small gaps
(framed payloads), unsorted, overlapping, empty and out-of-range entries, every base misalignment,
runs of entries under a line (records outside the eight-entry window), ranges that end mid-entry,
entries spanning more than 64 ranges (the combine's block path) and the whole-entry fallback of the
range kernel. Reference arithmetic: circe crc32c() ($CN/cpp/crc32c_sse42.cpp:184-217) through the
oracle, zlib for CRC32."""
import numpy as np
import pytest

import oracle
from bookkeeper_amd import checksum as ck
from bookkeeper_amd._native import BkdError

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset():
    ck.set_plan_mode(0)
    yield
    ck.set_plan_mode(0)
    ck.set_stream_range_max(1 << 22)


def _run(gpu, data, offs, lens, seeds, algo, mis=0, mode=3):
    import torch
    buf = torch.empty(len(data) + 256, dtype=torch.uint8, device=gpu)
    # base pointer at device address = mis (mod 128): torch allocations are 256-aligned
    base = buf[mis:mis + len(data)]
    base.copy_(torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to(gpu))
    buf[:mis].fill_(0xA5)
    buf[mis + len(data):].fill_(0x5A)
    ck.set_plan_mode(mode)
    got = ck.crc_batch(algo, base, torch.from_numpy(np.asarray(offs, dtype=np.int64)).to(gpu),
                       torch.from_numpy(np.asarray(lens).astype(np.int32)).to(gpu),
                       seeds=torch.from_numpy(np.asarray(seeds, dtype=np.uint32).view(np.int32)).to(gpu))
    try:  # read and clear this stream's bounds flag (out-of-range entries are expected in some cases)
        ck.stream_sync(torch.cuda.current_stream(gpu))
    except BkdError:
        pass
    return got.cpu().numpy().view(np.uint32)


def _want(algo, data, offs, lens, seeds):
    arr = np.frombuffer(data, dtype=np.uint8)
    return oracle.batch(algo, arr, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint32),
                        seeds=np.asarray(seeds, dtype=np.uint32))


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
@pytest.mark.parametrize("mis", [0, 1, 61, 125, 127])
def test_packed_every_misalignment(gpu, algo, mis):
    rng = np.random.default_rng(100 + mis)
    lens = rng.choice([1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 100, 127, 128, 129, 300, 1000, 4095, 4096, 4097, 9000,
                       70000], 6000)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    data = rng.bytes(int(lens.sum()))
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64)
    for mode in (3, 0):
        got = _run(gpu, data, offs, lens, seeds, algo, mis, mode)
        want = _want(algo, data, offs, lens, seeds)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mode, bad[:5].tolist(), lens[bad[:5]].tolist())


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_gaps_unsorted_overlapping_invalid(gpu, algo):
    rng = np.random.default_rng(7)
    size = 3_000_000
    data = rng.bytes(size)
    n = 5000
    lens = rng.choice([0, 1, 2, 3, 7, 16, 33, 127, 128, 200, 900, 3000, 9000, 40000], n)
    offs = rng.integers(0, size, n)
    offs[::7] = size - lens[::7] + rng.integers(0, 3, len(offs[::7]))  # some past the end
    for k in range(1000, 3000):  # runs of packed neighbours with small gaps and overlaps
        offs[k] = max(0, offs[k - 1] + lens[k - 1] + rng.integers(-40, 90))
        if offs[k] + lens[k] > size:
            offs[k] = 0
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64)
    for mis in (0, 3, 126):
        got = _run(gpu, data, offs, lens, seeds, algo, mis, 3)
        bad = [k for k in range(n) if got[k] != (0 if offs[k] > size or lens[k] > size - offs[k] else
                                                 oracle.resume(algo, int(seeds[k]), data[offs[k]:offs[k] + lens[k]]))]
        bad = np.array(bad, dtype=np.int64)
        assert bad.size == 0, (mis, bad[:5].tolist(), lens[bad[:5]].tolist(), offs[bad[:5]].tolist())


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_framed_payload_gaps(gpu, algo):
    """Payload ranges of framed entries (a 36/40-byte header and digest between them): every entry
    continues its predecessor's lines, so the automatic route takes the stream."""
    rng = np.random.default_rng(8)
    n = 20000
    lens = rng.integers(0, 9000, n)
    gap = 36 if algo == ck.CRC32C else 40
    offs = np.cumsum(np.concatenate([[gap], lens[:-1] + gap]))
    size = int(offs[-1] + lens[-1] + 5)
    data = rng.bytes(size)
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64)
    for mode in (0, 3):
        got = _run(gpu, data, offs, lens, seeds, algo, 0, mode)
        assert (got == _want(algo, data, offs, lens, seeds)).all(), mode


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_huge_entries_combine_paths(gpu, algo):
    """Entries spanning many ranges (more than 64: the combine's block path) among small ones."""
    rng = np.random.default_rng(9)
    lens = np.array([100, 64 * 4096 * 2 + 7, 50, 4096 * 4100 + 3, 1, 300, 4096 * 65, 4096 * 64, 4096 * 63 + 1, 77])
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    data = rng.bytes(int(lens.sum()))
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64)
    for mis in (0, 77):
        got = _run(gpu, data, offs, lens, seeds, algo, mis, 3)
        assert (got == _want(algo, data, offs, lens, seeds)).all(), mis


def test_stream_repeated_calls_same_stream(gpu):
    """The look-back words, ticket and range arrays are reused between calls on a stream: alternating
    packed and permuted batches through the automatic route stay exact."""
    rng = np.random.default_rng(10)
    lens = rng.integers(1, 20000, 3000)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    data = rng.bytes(int(lens.sum()))
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64)
    perm = rng.permutation(lens.size)
    for k in range(4):
        o, l, s = (offs, lens, seeds) if k % 2 == 0 else (offs[perm], lens[perm], seeds[perm])
        got = _run(gpu, data, o, l, s, ck.CRC32C, 0, 0)
        assert (got == _want(ck.CRC32C, data, o, l, s)).all(), k


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_whole_entry_fallback(gpu, algo):
    """Ranges longer than the bound (lowered here from 2^22 lines): the range kernel takes every entry
    whole, one per lane group, and the combine only the entries outside the stream."""
    rng = np.random.default_rng(12)
    lens = rng.choice([0, 1, 3, 64, 129, 4096, 100000], 3000)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    offs[::11] += 5  # gaps: some entries past the end below
    data = rng.bytes(int(lens.sum()))
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64)
    ck.set_stream_range_max(4)
    got = _run(gpu, data, offs, lens, seeds, algo, 3, 3)
    size = len(data)
    want = [0 if offs[k] > size or lens[k] > size - offs[k] else
            oracle.resume(algo, int(seeds[k]), data[offs[k]:offs[k] + lens[k]]) for k in range(lens.size)]
    assert (got == np.array(want, dtype=np.uint32)).all()


def test_tiny_entry_runs(gpu):
    """Packed runs of 1..40-byte entries (more than eight entries begin within four lines: records
    loaded outside the window) between long entries, at several misalignments."""
    rng = np.random.default_rng(13)
    parts = []
    for k in range(300):
        parts.append(rng.integers(1, 41, rng.integers(5, 60)))
        parts.append(rng.integers(3000, 20000, 1))
    lens = np.concatenate(parts)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    data = rng.bytes(int(lens.sum()))
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64)
    for mis in (0, 45, 126):
        got = _run(gpu, data, offs, lens, seeds, ck.CRC32C, mis, 3)
        assert (got == _want(ck.CRC32C, data, offs, lens, seeds)).all(), mis


def test_many_entry_blocks_lookback(gpu):
    """4M short entries (4096 entry blocks, many look-back windows of 64 blocks): the stream route
    equals the chunked plan on every digest and the oracle on a sample."""
    import torch
    rng = np.random.default_rng(14)
    n = 4 << 20
    lens = rng.integers(1, 200, n)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    size = int(offs[-1] + lens[-1])
    base = torch.empty(size, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 5)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    got = {}
    for mode in (3, 2):
        ck.set_plan_mode(mode)
        got[mode] = ck.crc_batch(ck.CRC32C, base, d_off, d_len).cpu().numpy().view(np.uint32)
    assert (got[3] == got[2]).all()
    host = base.cpu().numpy()
    for k in rng.integers(0, n, 2000):
        o, l = int(offs[k]), int(lens[k])
        assert got[3][k] == oracle.resume(ck.CRC32C, 0, host[o:o + l].tobytes()), k


def test_lookback_words_after_plan_calls(gpu):
    """The stream route's look-back words live in a region of their own (StreamScratch::lookback_words):
    chunked-plan and stream calls of different sizes alternate on one stream with no sync between
    them (the plan's descriptors fill the shared scratch the words once shared), and every stream
    digest equals the plan's; the plan's equal the oracle on a sample."""
    import torch
    rng = np.random.default_rng(15)
    size = 192 << 20
    base = torch.empty(size, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(base, 6)
    batches = []
    for n, hi in ((200_000, 300), (60_000, 5000), (300_000, 120), (20_000, 2000)):
        lens = rng.integers(1, hi, n)
        offs = np.concatenate([[0], np.cumsum(lens[:-1])])
        assert offs[-1] + lens[-1] <= size
        batches.append((offs, lens, torch.from_numpy(offs.astype(np.int64)).to(gpu),
                        torch.from_numpy(lens.astype(np.int32)).to(gpu)))
    outs = []
    for rep in range(3):
        for offs, lens, d_off, d_len in batches:
            for mode in (2, 3):
                ck.set_plan_mode(mode)
                outs.append((mode, len(outs) // 2 % len(batches), ck.crc_batch(ck.CRC32C, base, d_off, d_len)))
    torch.cuda.synchronize(gpu)
    host = base.cpu().numpy()
    ref = {}
    for mode, b, t in outs:
        if mode == 2 and b not in ref:
            ref[b] = t.cpu().numpy().view(np.uint32)
    for mode, b, t in outs:
        assert (t.cpu().numpy().view(np.uint32) == ref[b]).all(), (mode, b)
    for b, (offs, lens, _, _) in enumerate(batches):
        for k in rng.integers(0, len(offs), 300):
            o, l = int(offs[k]), int(lens[k])
            assert ref[b][k] == oracle.resume(ck.CRC32C, 0, host[o:o + l].tobytes()), (b, k)
