"""CPU: the stream route's decomposition (tests/stream_model.py RangeModel) reproduces the oracle on
every layout the indexed API allows — packed (the config-3 shape), gaps, unsorted, overlapping, empty
and out-of-range entries, every base misalignment, per-entry seeds, several range counts — before any
GPU run."""
import numpy as np
import pytest

import oracle
from stream_model import RangeModel




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
