"""Synthetic BookKeeper entry logs for the scrub tests (format: DefaultEntryLogger.java:240-277,
records as addEntryForCompaction writes them, :626-642: [int32 BE size][entry])."""
from __future__ import annotations

import numpy as np

import oracle

HEADER = 1024


def framed_entry(algo: int, ledger_id: int, entry_id: int, payload: bytes) -> bytes:
    """V2 framing (DigestManager.java:146-153): [32 B header][digest][payload]."""
    d, hdr = oracle.digest_entry(algo, ledger_id, entry_id, entry_id - 1, len(payload), payload)
    return hdr + oracle.digest_bytes(algo, d) + payload


def make_entry_log(rng, n_entries: int, ledgers: dict, max_payload: int = 9000, pad_between: bool = False,
                   with_map: bool = True, truncate: bool = False, min_payload: int = 0):
    """ledgers: ledger id -> oracle algo. Returns (log bytes, list of (ledger, entry id, entry offset,
    entry length)) for the entries the walk must find."""
    out = bytearray(HEADER)
    out[0:4] = b"BKLO"
    out[4:8] = (1).to_bytes(4, "big")
    lids = list(ledgers)
    next_eid = {l: 0 for l in lids}
    expect = []
    for _ in range(n_entries):
        lid = lids[int(rng.integers(len(lids)))]
        eid = next_eid[lid]
        next_eid[lid] += 1
        plen = int(rng.integers(min_payload, max_payload + 1))
        payload = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
        f = framed_entry(ledgers[lid], lid, eid, payload)
        out += len(f).to_bytes(4, "big")
        expect.append((lid, eid, len(out), len(f)))
        out += f
        if pad_between and rng.random() < 0.3:
            out += bytes(int(rng.integers(1, 24)))
    if with_map:  # ledgers map record: [size][ledgerId -1][entryId -2][count][(ledger, size)...]
        body = (-1).to_bytes(8, "big", signed=True) + (-2).to_bytes(8, "big", signed=True)
        body += len(lids).to_bytes(4, "big") + b"".join(l.to_bytes(8, "big") + (100).to_bytes(8, "big")
                                                        for l in lids)
        out += len(body).to_bytes(4, "big") + body
    if truncate:  # a record whose entry runs past the end of the file
        out += (5000).to_bytes(4, "big") + lids[0].to_bytes(8, "big") + bytes(100)
    out += bytes(int(rng.integers(0, 40)))  # preallocated zero tail
    return bytes(out), expect
