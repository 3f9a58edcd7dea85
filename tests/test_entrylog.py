"""Entry-log scrub (§8f row 4): the record walk against the oracle's restatement of
DefaultEntryLogger.scanEntryLog (CPU, through the C-ABI's host walk), and GPU digest verification
against oracle.verify_entry, including corrupted entries."""
import numpy as np
import pytest

import oracle
from bookkeeper_amd import entrylog as el
from entrylog_util import make_entry_log

LEDGERS = {3: oracle.CRC32C, 7: oracle.CRC32, 11: oracle.CRC32C}


@pytest.mark.parametrize("pad,with_map,truncate", [(False, True, False), (True, True, False), (False, False, True),
                                                   (True, True, True)])
def test_scan_matches_oracle(pad, with_map, truncate):
    rng = np.random.default_rng(int(pad) * 4 + int(with_map) * 2 + int(truncate))
    log, expect = make_entry_log(rng, 300, LEDGERS, pad_between=pad, with_map=with_map, truncate=truncate)
    got = el.scan_entry_log(log)
    offs, lens, lids, end = oracle.entrylog_scan(log)
    assert (got.offsets == offs).all() and (got.lengths == lens).all() and (got.ledger_ids == lids).all()
    assert got.end == end
    if not pad:  # without mid-log padding the walk finds exactly the written entries
        assert [(int(l), int(o), int(n)) for l, o, n in zip(got.ledger_ids, got.offsets, got.lengths)] == \
            [(l, o, n) for l, _, o, n in expect]


def test_scan_edge_cases():
    assert len(el.scan_entry_log(b"")) == 0
    assert len(el.scan_entry_log(bytes(1024))) == 0
    assert len(el.scan_entry_log(bytes(2000))) == 0  # all padding
    # a record header cut short (fewer than 12 bytes left) ends the walk
    log = bytes(1024) + (20).to_bytes(4, "big") + (5).to_bytes(8, "big")[:6]
    r = el.scan_entry_log(log)
    assert len(r) == 0 and r.end == 1024
    assert oracle.entrylog_scan(log)[3] == 1024


@pytest.mark.gpu
def test_scrub_verifies_digests(gpu):
    import torch
    rng = np.random.default_rng(5)
    log, expect = make_entry_log(rng, 2000, LEDGERS, max_payload=20000, min_payload=0)
    buf = np.frombuffer(log, dtype=np.uint8).copy()
    # corrupt: a payload byte, a digest byte, a header byte (ledger id kept)
    bad = {}
    for k, (what, delta) in zip(rng.choice(len(expect), 30, replace=False), [("p", 40), ("d", 33), ("h", 20)] * 10):
        lid, eid, o, n = expect[k]
        pos = o + (delta if what != "p" else min(n - 1, 40 + int(rng.integers(0, max(1, n - 40)))))
        if pos < o + n:
            buf[pos] ^= 0x5A
            bad[int(k)] = what
    scrub = el.EntryLogScrubber(lambda lid: {oracle.CRC32C: "CRC32C", oracle.CRC32: "CRC32"}[LEDGERS[lid]])
    dev = torch.from_numpy(buf).to(gpu)
    scan, status = scrub.verify(buf, dev)
    assert len(scan) == len(expect)
    for k, (lid, eid, o, n) in enumerate(expect):
        # corruptions never touch the ledger id (bytes 0-7), so the oracle's id check is moot
        want = oracle.verify_entry(LEDGERS[lid], buf[o:o + n], lid, eid, skip_entry_check=True)
        assert status[k] == want, (k, lid, n, bad.get(k))
    assert (status != 0).sum() >= 20


@pytest.mark.gpu
def test_scrub_skips_untyped_ledgers(gpu):
    import torch
    rng = np.random.default_rng(9)
    log, expect = make_entry_log(rng, 200, LEDGERS)
    scrub = el.EntryLogScrubber(lambda lid: "CRC32C" if lid == 3 else None)
    scan, status = scrub.verify(np.frombuffer(log, dtype=np.uint8))
    for k, (lid, *_rest) in enumerate(expect):
        assert status[k] == (0 if lid == 3 else -1)


def test_scan_many_tiny_records():
    """a log of records far smaller than 16 bytes (a corrupt or synthetic log) is walked
    whole — the index grows past the first size//256 guess instead of failing with BKD_ERR_BOUNDS."""
    rng = np.random.default_rng(12)
    parts = [bytes(1024)]
    n = 20000
    for _ in range(n):
        size = int(rng.integers(8, 16))
        parts.append(size.to_bytes(4, "big") + (3).to_bytes(8, "big") + bytes(size - 8))
    log = b"".join(parts)
    got = el.scan_entry_log(log)
    offs, lens, lids, end = oracle.entrylog_scan(log)
    assert len(got) == len(offs) == n
    assert (got.offsets == offs).all() and (got.lengths == lens).all() and (got.ledger_ids == lids).all()
    assert got.end == end
