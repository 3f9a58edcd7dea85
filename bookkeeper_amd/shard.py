"""Splitting a batch across ranks (one process per GPU, no data-path collective).

SURVEY.md §8e: entries are independent, so each GPU takes a contiguous range of them — by count for
uniform entries (bench.py's `shard_first_word`), and for a ragged batch (config 3) *by bytes*, from
the prefix sum of the lengths, so that every rank folds about the same number of bytes whatever the
size distribution. Each rank then holds only its own byte span of the entries and an index rebased to
that span; the concatenation of the ranks' digests is the unsplit batch's.
"""
from __future__ import annotations

import numpy as np


def byte_balanced_bounds(lengths, nshards: int) -> np.ndarray:
    """Entry bounds b[0..nshards] (b[0] = 0, b[nshards] = n, non-decreasing): shard r is entries
    [b[r], b[r+1]). Laid end to end (T bytes in all), entry i goes to the shard r whose byte range
    [r*T/N, (r+1)*T/N) holds the entry's midpoint, so every shard holds at most T/N + max(lengths)
    bytes. Integer arithmetic: with E[i] = the prefix sum through entry i, the midpoint test
    (E[i-1] + E[i]) * N < 2 * (r+1) * T. `lengths` may be a numpy array, a sequence or a torch tensor
    (on any device: the prefix sum and the search then run there)."""
    if nshards < 1:
        raise ValueError("nshards must be >= 1")
    try:
        import torch
        is_tensor = isinstance(lengths, torch.Tensor)
    except ImportError:  # pragma: no cover - torch is part of the image
        is_tensor = False
    if is_tensor:
        if lengths.dim() != 1:
            raise ValueError("lengths must be one-dimensional")
        if lengths.numel() and bool((lengths < 0).any()):
            raise ValueError("lengths must be non-negative")
        cum = torch.cumsum(lengths.to(torch.int64), 0)
        total = int(cum[-1]) if cum.numel() else 0
        key = (2 * cum - lengths.to(torch.int64)) * nshards  # (start + end) * N, non-decreasing
        thr = torch.tensor([2 * k * total for k in range(1, nshards)], dtype=torch.int64, device=cum.device)
        inner = torch.searchsorted(key, thr).cpu().numpy() if nshards > 1 else np.zeros(0, np.int64)
        n = int(cum.numel())
    else:
        lens = np.asarray(lengths)
        if lens.ndim != 1:
            raise ValueError("lengths must be one-dimensional")
        if lens.size and (lens < 0).any():
            raise ValueError("lengths must be non-negative")
        cum = np.cumsum(lens.astype(np.int64))
        total = int(cum[-1]) if cum.size else 0
        key = (2 * cum - lens.astype(np.int64)) * nshards  # (start + end) * N, non-decreasing
        thr = np.array([2 * k * total for k in range(1, nshards)], dtype=np.int64)
        inner = np.searchsorted(key, thr, side="left")
        n = int(cum.size)
    return np.concatenate([[0], inner.astype(np.int64), [n]]).astype(np.int64)


def shard_span(offsets: np.ndarray, lengths: np.ndarray, lo: int, hi: int, align: int = 8) -> tuple[int, int]:
    """Byte span [start, end) of base holding entries [lo, hi): start rounded down to `align` (the
    rank generates or copies its span from there), end the furthest entry end. (0, 0) when empty."""
    if hi <= lo:
        return 0, 0
    o = np.asarray(offsets[lo:hi], dtype=np.int64)
    e = o + np.asarray(lengths[lo:hi], dtype=np.int64)
    start = int(o.min()) // align * align
    return start, int(e.max())
