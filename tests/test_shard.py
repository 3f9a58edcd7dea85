"""Byte-balanced contiguous split of a ragged batch across ranks (bookkeeper_amd/shard.py; SURVEY.md
§8e: "Partition contiguous entry ranges per GPU. Balance by bytes (prefix-sum of lengths) for
config 3"). CPU only: the split is host/torch arithmetic on the index, before any GPU work."""
import numpy as np
import pytest
import torch

from bench import zipf_index
from bookkeeper_amd.shard import byte_balanced_bounds, shard_span


def _check(lens, n_shards, b):
    lens = np.asarray(lens, dtype=np.int64)
    assert b.dtype == np.int64 and b.shape == (n_shards + 1,)
    assert b[0] == 0 and b[-1] == lens.size and (np.diff(b) >= 0).all()
    per = np.array([lens[b[r]:b[r + 1]].sum() for r in range(n_shards)])
    total = int(lens.sum())
    assert per.sum() == total
    bound = total / n_shards + (int(lens.max()) if lens.size else 0)
    assert (per <= bound).all(), (per.max(), bound)
    return per


@pytest.mark.parametrize("n_shards", [1, 2, 3, 4, 7, 8])
def test_zipf_index_splits_by_bytes(n_shards):
    _, lens = zipf_index(1 << 16)
    b = byte_balanced_bounds(lens, n_shards)
    per = _check(lens, n_shards, b)
    # the same bounds from a torch tensor (the prefix sum and the search run where the tensor is)
    assert (byte_balanced_bounds(torch.from_numpy(lens), n_shards) == b).all()
    assert (byte_balanced_bounds(torch.from_numpy(lens.astype(np.int32)), n_shards) == b).all()
    # by bytes, not by count: the shards' entry counts differ while their bytes stay within one entry
    if n_shards > 1:
        assert per.max() - per.min() <= 2 * int(lens.max()) + 2


def test_each_entry_goes_to_the_shard_its_midpoint_falls_in():
    lens = np.array([10, 10, 10, 10])  # total 40; midpoints 5, 15, 25, 35
    assert byte_balanced_bounds(lens, 2).tolist() == [0, 2, 4]
    assert byte_balanced_bounds(lens, 4).tolist() == [0, 1, 2, 3, 4]
    assert byte_balanced_bounds([100, 1, 1, 1], 2).tolist() == [0, 1, 4]  # midpoint 50 < 51.5
    assert byte_balanced_bounds([1, 1, 1, 100], 2).tolist() == [0, 3, 4]  # midpoint 53 >= 51.5
    assert byte_balanced_bounds([0, 0, 0], 2).tolist() == [0, 0, 3]


@pytest.mark.parametrize("lens,n_shards", [([], 3), ([0, 0, 0], 2), ([5], 4), ([3, 0, 0, 4], 3),
                                           ([1 << 40, 1, 1 << 40], 2)])
def test_edge_cases(lens, n_shards):
    b = byte_balanced_bounds(np.asarray(lens, dtype=np.int64), n_shards)
    _check(lens, n_shards, b)
    assert (byte_balanced_bounds(torch.tensor(lens, dtype=torch.int64), n_shards) == b).all()


def test_argument_errors():
    with pytest.raises(ValueError):
        byte_balanced_bounds([1, 2], 0)
    with pytest.raises(ValueError):
        byte_balanced_bounds([1, -2], 2)
    with pytest.raises(ValueError):
        byte_balanced_bounds(np.ones((2, 2)), 2)
    with pytest.raises(ValueError):
        byte_balanced_bounds(torch.tensor([1, -1]), 2)


def test_shard_span():
    offs, lens = zipf_index(4096)
    b = byte_balanced_bounds(lens, 3)
    spans = [shard_span(offs, lens, int(b[r]), int(b[r + 1]), align=128) for r in range(3)]
    for r, (s, e) in enumerate(spans):
        lo, hi = int(b[r]), int(b[r + 1])
        assert s % 128 == 0 and s <= offs[lo] and e == offs[hi - 1] + lens[hi - 1]
        assert offs[lo] - s < 128
    assert shard_span(offs, lens, 5, 5) == (0, 0)
    # unordered, overlapping entries: the span still holds every one of them
    o, l = np.array([100, 20, 60]), np.array([10, 90, 5])
    assert shard_span(o, l, 0, 3) == (16, 110)
