"""CPU: the stream route's decomposition (tests/stream_model.py) reproduces the oracle on every
layout the indexed API allows — packed (the config-3 shape), gaps, unsorted, overlapping, empty and
out-of-range entries, every base misalignment, per-entry seeds — before any GPU run."""
import numpy as np
import pytest

import oracle
from stream_model import StreamModel, stream_layout


def _model(algo):
    return StreamModel(oracle.table(algo), lambda a, b: oracle.gf_mul(algo, a, b),
                       lambda nbytes: oracle.xpow8n(algo, nbytes))


def _check(algo, base, mis, offs, lens, seeds, tl=32):
    size = len(base)
    foreign = np.random.default_rng(99).bytes(509)
    got, info = _model(algo).digests(base, mis, offs, lens, seeds, foreign, tl)
    for i in range(len(offs)):
        o, l = int(offs[i]), int(lens[i])
        if o > size or l > size - o:
            want = 0
        else:
            want = oracle.resume(algo, int(seeds[i]), base[o:o + l])
        assert got[i] == want, (i, o, l, mis, hex(got[i]), hex(want))
    return info


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("mis", [0, 1, 61, 125, 127])
@pytest.mark.parametrize("tl", [2, 32])
def test_packed(algo, mis, tl):
    rng = np.random.default_rng(7 + mis + tl)
    lens = rng.choice([1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 100, 127, 128, 129, 300, 1000, 4096, 5000], 120)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    base = rng.bytes(int(lens.sum()))
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64)
    info = _check(algo, base, mis, offs, lens, seeds, tl)
    # packed: only the first entry starts a run, and an entry after one the stream skips (a padded
    # message under 4 bytes: at most 3 bytes in the last 3 of a line)
    geo = stream_layout(mis, offs, lens, len(base))[0]
    assert info["jumps"] == 1 + sum(1 for k in range(1, len(geo)) if geo[k].stream and not geo[k - 1].stream)


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("tl", [2, 32])
def test_gaps_unsorted_overlaps_invalid(algo, tl):
    rng = np.random.default_rng(11 + tl)
    size = 40000
    base = rng.bytes(size)
    n = 150
    lens = rng.choice([0, 1, 2, 3, 7, 16, 33, 127, 128, 200, 900, 3000, 9000], n)
    offs = rng.integers(0, size, n)
    offs[::7] = size - lens[::7] + rng.integers(0, 3, len(offs[::7]))  # some past the end
    offs[5] = size  # an empty entry at the very end: valid
    lens[5] = 0
    # a few runs of packed neighbours and small gaps / overlaps
    for k in range(20, 60):
        offs[k] = offs[k - 1] + lens[k - 1] + rng.integers(-40, 90)
        if offs[k] < 0:
            offs[k] = 0
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64)
    for mis in (0, 3, 126):
        _check(algo, base, mis, offs, lens, seeds, tl)


def test_layout_positions_packed():
    """Packed entries: the stream is the device lines in order, each line once."""
    lens = np.array([100, 28, 200, 56, 4096])
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    geo, shared, jump, V, end, first, k0 = stream_layout(0, offs, lens, int(lens.sum()))
    assert end == (int(lens.sum()) + 127) // 128 and jump == [True, False, False, False, False]
    assert shared == [False, True, False, True, False]  # 100|28 share line 0, 200|56 share line 2


# ---- the free-jump design (one contiguous range of positions per group) ----
from stream_model import RangeModel  # noqa: E402


def _check_range(algo, base, mis, offs, lens, seeds, groups):
    size = len(base)
    foreign = np.random.default_rng(99).bytes(509)
    m = RangeModel(oracle.table(algo), lambda a, b: oracle.gf_mul(algo, a, b),
                   lambda nbytes: oracle.xpow8n(algo, nbytes))
    got, info = m.digests(base, mis, offs, lens, seeds, foreign, groups)
    for i in range(len(offs)):
        o, l = int(offs[i]), int(lens[i])
        want = 0 if (o > size or l > size - o) else oracle.resume(algo, int(seeds[i]), base[o:o + l])
        assert got[i] == want, (i, o, l, mis, groups)
    return info


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("mis", [0, 1, 125])
@pytest.mark.parametrize("groups", [1, 3, 50])
def test_range_packed(algo, mis, groups):
    rng = np.random.default_rng(17 + mis + groups)
    lens = rng.choice([1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 100, 127, 128, 129, 300, 1000, 4096, 5000], 100)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])])
    base = rng.bytes(int(lens.sum()))
    seeds = rng.integers(0, 2**32, lens.size, dtype=np.uint64)
    info = _check_range(algo, base, mis, offs, lens, seeds, groups)
    # packed: every line once, but for the line after an entry the stream skips (at most 3 bytes in
    # the last 3 of a line), which the next entry does not share
    from stream_model import Geo
    skipped = sum(1 for o, l in zip(offs, lens) if not Geo(mis, int(o), int(l), int(lens.sum())).stream)
    assert info["end"] <= (mis + int(lens.sum()) + 127) // 128 + skipped


@pytest.mark.parametrize("algo", [0, 1])
@pytest.mark.parametrize("groups", [1, 5, 40])
def test_range_gaps_unsorted_overlaps_invalid(algo, groups):
    """Free jumps: any index order, gaps and overlaps take the stream too (lines reloaded as needed)."""
    rng = np.random.default_rng(23 + groups)
    size = 30000
    base = rng.bytes(size)
    n = 120
    lens = rng.choice([0, 1, 2, 3, 7, 16, 33, 127, 128, 200, 900, 3000, 9000], n)
    offs = rng.integers(0, size, n)
    offs[::7] = size - lens[::7] + rng.integers(0, 3, len(offs[::7]))
    offs[5] = size
    lens[5] = 0
    for k in range(20, 60):
        offs[k] = max(0, offs[k - 1] + lens[k - 1] + rng.integers(-40, 90))
    seeds = rng.integers(0, 2**32, n, dtype=np.uint64)
    for mis in (0, 3, 126):
        _check_range(algo, base, mis, offs, lens, seeds, groups)
