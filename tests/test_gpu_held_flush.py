"""GPU: held result stores across their flushes.

The uniform, fused-verify and fused-package kernels keep each group's results in its lanes and store
K words per lane at once (HeldResults, crc_kernels.hpp): every K*G rounds of the group's loop, then the
rest when the loop ends. The other parity tests stay within one flush; these batches cross them:

* mid-size uniform entries (512 B at 8 lanes: past the short loop, below 32 steps; held_store_loop):
  exactly 64 rounds per group (K = 8: the one flush inside put()), 63 rounds plus a partial round
  (the final partial slot), and 261 rounds plus 77 entries (K = 32: a flush at round 256 mid-loop,
  then a partial slot) — every digest against the reference's own crc32c() (oracle/_ref, threaded)
  or the oracle (CRC32);
* fused package and fused verify over 2.29 M near-uniform frames (8-lane groups, K = 8: 70 rounds
  per group = one flush mid-loop plus a partial slot): every digest against the oracle (header CRC,
  then the payload resumed from it: DigestManager.java:146-153), every frame's header + digest bytes,
  and the verify statuses and verified prefix with corruptions (payload, digest, header bytes) placed
  past the first flush.
"""
import ctypes

import numpy as np
import pytest

import oracle
from bookkeeper_amd import checksum as ck
from bookkeeper_amd import digest as dg

pytestmark = pytest.mark.gpu


def _ngroups(torch, gpu, lanes):
    return torch.cuda.get_device_properties(gpu).multi_processor_count * (1024 // lanes)


def _uniform_want(algo, host, stride, length, n):
    ref = oracle.ref()
    if algo == ck.CRC32C and ref is not None:  # the reference's crc32c(), 16 threads
        out = np.zeros(n, dtype=np.uint32)
        ref.ref_crc32c_uniform_timed(host.ctypes.data_as(oracle._u8p), stride, length, n, 16, 1,
                                     out.ctypes.data_as(oracle._u32p))
        return out
    return oracle.uniform(algo, host, stride, length, n)


@pytest.mark.parametrize("algo", [ck.CRC32C, ck.CRC32])
def test_uniform_mid_size_held_stores_cross_flushes(gpu, algo):
    import torch
    L = 512
    ng = _ngroups(torch, gpu, 8)
    cases = [64 * ng, 63 * ng + 5] if algo == ck.CRC32 else [64 * ng, 63 * ng + 5, 261 * ng + 77]
    ck.set_group_lanes(8)
    try:
        for n in cases:
            base = torch.empty(n * L, dtype=torch.uint8, device=gpu)
            ck.fill_splitmix64(base, 300 + n % 1000)
            got = ck.crc_batch_uniform(algo, base, L, n).cpu().numpy().view(np.uint32)
            host = base.cpu().numpy()
            del base
            want = _uniform_want(algo, host, L, L, n)
            bad = np.nonzero(got != want)[0]
            assert bad.size == 0, (n, bad.size, bad[:5].tolist())
    finally:
        ck.set_group_lanes(0)
        torch.cuda.empty_cache()


def _headers(ledger, ids, lacs, lens):
    """The 32-byte BE headers [ledgerId, entryId, lastAddConfirmed, length] (DigestManager.java:146-149)."""
    n = ids.size
    h = np.empty((n, 4), dtype=">i8")
    h[:, 0] = ledger
    h[:, 1] = ids
    h[:, 2] = lacs
    h[:, 3] = lens
    return h.view(np.uint8).reshape(n, 32)


@pytest.mark.parametrize("dtype,algo", [(dg.DigestType.CRC32C, ck.CRC32C), (dg.DigestType.CRC32, ck.CRC32)])
def test_fused_package_and_verify_held_stores_cross_flushes(gpu, dtype, algo):
    import torch
    ng = _ngroups(torch, gpu, 8)
    n = 70 * ng + 123  # 70 rounds per 8-lane group: one flush at round 64 and a partial slot
    slot = 1024
    ledger, first = 12, 5000
    dm = dg.DigestManager.instantiate(ledger, b"", dtype, False)
    mac = dm.macCodeLength
    hl = 32 + mac
    rng = np.random.default_rng(71 + algo)
    plen = rng.integers(600, 660, n).astype(np.int64)  # mean >= 512 B: 8 lanes; within the fused band
    blob = torch.empty(n * slot, dtype=torch.uint8, device=gpu)
    ck.fill_splitmix64(blob, 17 + algo)
    ids = np.arange(first, first + n, dtype=np.int64)
    lacs = ids - 1
    d_ids = torch.from_numpy(ids).to(gpu)
    poff = torch.arange(n, dtype=torch.int64, device=gpu) * slot + hl
    frames, digests = dm.package_batch(d_ids, d_ids - 1, torch.from_numpy(plen).to(gpu), blob, poff,
                                       torch.from_numpy(plen.astype(np.int32)).to(gpu), sync_check=True)
    torch.cuda.synchronize()
    digests = digests.cpu().numpy().view(np.uint32)
    host = blob.cpu().numpy()
    # oracle: update(update(0, header), payload) for every entry, vectorised through oracle.batch
    hdr = _headers(ledger, ids, lacs, plen)
    hcrc = oracle.batch(algo, hdr.reshape(-1), np.arange(n, dtype=np.uint64) * 32, np.full(n, 32, np.uint32))
    want = oracle.batch(algo, host, np.arange(n, dtype=np.uint64) * slot + hl, plen.astype(np.uint32), seeds=hcrc)
    bad = np.nonzero(digests != want)[0]
    assert bad.size == 0, ("package", bad.size, bad[:5].tolist())
    fr = frames.cpu().numpy()
    assert (fr[:, :32] == hdr).all()
    be = want.astype(">u4").view(np.uint8).reshape(n, 4)
    assert (fr[:, hl - 4:hl] == be).all() and (mac == 4 or (fr[:, 32:36] == 0).all())
    # the frames in place, then verify; corruptions past the first flush (rounds > 64)
    blob.view(n, slot)[:, :hl].copy_(frames)
    f_off = torch.arange(n, dtype=torch.int64, device=gpu) * slot
    f_len = torch.from_numpy((plen + hl).astype(np.int32)).to(gpu)
    status, first_bad = dm.verify_batch(blob, f_off, f_len, first_entry_id=first)
    assert int(first_bad.item()) == n and int((status != 0).sum().item()) == 0
    picks = {66 * ng + 9: (hl + 5, 0x01), 67 * ng + 2: (hl - 1, 0x80), 69 * ng + 40: (7, 0x02), n - 1: (15, 0x04)}
    view = blob.view(n, slot)
    for i, (pos, bit) in picks.items():
        view[i, pos] ^= bit
    status, first_bad = dm.verify_batch(blob, f_off, f_len, first_entry_id=first)
    status = status.cpu().numpy()
    exp = np.zeros(n, dtype=np.int32)
    for i in picks:
        exp[i] = oracle.verify_entry(algo, view[i, :hl + int(plen[i])].cpu().numpy().tobytes(), ledger, first + i)
    assert (exp[list(picks)] != 0).all()  # (a header byte flipped fails the digest first: DigestManager.java:241-249)
    bad = np.nonzero(status != exp)[0]
    assert bad.size == 0, ("verify", bad[:5].tolist(), status[bad[:5]].tolist())
    assert int(first_bad.item()) == min(picks)
    del blob
    torch.cuda.empty_cache()
