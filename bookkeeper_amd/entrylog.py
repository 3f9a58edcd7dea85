"""Bookie-side entry-log scrub.

The reference writes entries into entry-log files as ``[int32 BE size][entry]`` records after a
1024-byte header (``DefaultEntryLogger.java:256``, ``addEntryForCompaction`` :626-642) and reads
them back with ``scanEntryLog`` (:995-1060). It never re-verifies their digests on the bookie
(``BookieProtoEncoding.java:152-175``); this module adds that bulk check as a new feature:

* ``scan_entry_log`` — the record walk (host control logic, ``bkd_entrylog_index``), with the
  reference's padding / ledgers-map / short-read rules;
* ``EntryLogScrubber.verify`` — every entry's digest recomputed on the GPU
  (``bkd_entrylog_verify``) from a device-resident copy of the log, grouped by digest type.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import checksum as _ck
from ._native import CRC32, CRC32C, check, lib

BKD_ERR_BOUNDS = -4

LOGFILE_HEADER_SIZE = 1024  # DefaultEntryLogger.java:256
INVALID_LID = -1            # DefaultEntryLogger.java:277

VERIFY_OK = 0
VERIFY_TOO_SHORT = 1
VERIFY_DIGEST_MISMATCH = 2


class ScanResult:
    """Entries found by the walk: offsets of the entry bytes, lengths, ledger ids; `end` = where
    the walk stopped (== log size unless a short read ended it)."""

    def __init__(self, offsets: np.ndarray, lengths: np.ndarray, ledger_ids: np.ndarray, end: int):
        self.offsets = offsets
        self.lengths = lengths
        self.ledger_ids = ledger_ids
        self.end = end

    def __len__(self) -> int:
        return int(self.offsets.size)


def scan_entry_log(log, start: int = LOGFILE_HEADER_SIZE) -> ScanResult:
    """DefaultEntryLogger.scanEntryLog (:995-1060) over a host buffer, accepting every ledger."""
    buf = _ck._host_view(log)
    size = buf.size
    # a record takes at least 5 bytes (size field + 1 entry byte), so size // 5 + 1 always fits; start
    # smaller (ledger entries are rarely tiny) and grow when the walk finds more records than that
    cap = min(size // 5 + 1, max(64, size // 256))
    count = ctypes.c_uint64(0)
    end = ctypes.c_uint64(0)
    while True:
        offs = np.empty(cap, dtype=np.uint64)
        lens = np.empty(cap, dtype=np.uint32)
        lids = np.empty(cap, dtype=np.int64)
        rc = lib().bkd_entrylog_index(buf.ctypes.data if size else None, size, start, offs.ctypes.data,
                                      lens.ctypes.data, lids.ctypes.data, cap, ctypes.byref(count), ctypes.byref(end))
        if rc == BKD_ERR_BOUNDS and cap < size // 5 + 1:
            cap = min(size // 5 + 1, cap * 4)
            continue
        check(rc)
        break
    k = int(count.value)
    return ScanResult(offs[:k].copy(), lens[:k].copy(), lids[:k].copy(), int(end.value))


class EntryLogScrubber:
    """Verifies the digests of all entries of one entry log on the GPU.

    ``digest_type_of(ledger_id)`` returns "CRC32C", "CRC32" or None (skip: DUMMY / HMAC ledgers,
    whose digests are not CRC arithmetic) — in BookKeeper it comes from the ledger metadata."""

    _ALGOS = {"CRC32C": CRC32C, "CRC32": CRC32}

    def __init__(self, digest_type_of=lambda ledger_id: "CRC32C"):
        self.digest_type_of = digest_type_of

    def verify(self, log_host, log_device=None, start: int = LOGFILE_HEADER_SIZE, stream=None):
        """Returns (scan, status int32[n] on the host; -1 = not checked). `log_device` is the same
        bytes resident in HBM (uploaded here when omitted)."""
        import torch
        scan = scan_entry_log(log_host, start)
        n = len(scan)
        status = np.full(n, -1, dtype=np.int32)
        if n == 0:
            return scan, status
        if log_device is None:
            log_device = torch.from_numpy(np.array(_ck._host_view(log_host), copy=True)).cuda()
        dev = log_device.device
        types = np.array([self._ALGOS.get(self.digest_type_of(int(l)), -1) for l in scan.ledger_ids],
                         dtype=np.int32)
        for algo in (CRC32C, CRC32):
            idx = np.nonzero(types == algo)[0]
            if idx.size == 0:
                continue
            d_off = torch.from_numpy(scan.offsets[idx].astype(np.int64)).to(dev)
            d_len = torch.from_numpy(scan.lengths[idx].astype(np.int32)).to(dev)
            d_status = torch.empty(idx.size, dtype=torch.int32, device=dev)
            d_first = torch.empty(1, dtype=torch.int64, device=dev)
            check(lib().bkd_entrylog_verify(
                algo, _ck._dev_ptr(log_device, "log"), log_device.numel() * log_device.element_size(),
                _ck._dev_ptr(d_off, "offsets", torch.int64), _ck._dev_ptr(d_len, "lengths", torch.int32),
                idx.size, _ck._dev_ptr(d_status, "status"), _ck._dev_ptr(d_first, "first_bad"),
                _ck._stream_ptr(stream, log_device)))
            status[idx] = d_status.cpu().numpy()
        return scan, status
