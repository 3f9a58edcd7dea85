"""TEST INFRASTRUCTURE — the CPU oracle for the ledger-entry digest path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker / baseline — never as the thing
measured or shipped. The product (``bookkeeper_amd``) does not import it.

Two checkers live here:

* ``liboracle.so`` — plain-C restatement of the reference's CRC semantics
  (``crc_oracle.c``; ReflectedIntCrc.java:26-48, AbstractIntCrc.java:50-57,
  crc32c_sse42.cpp:184-217, DigestManager.java:126-283).
* ``_ref/libcirce_ref.so`` — the reference's own native ``crc32c()``
  (circe-checksum/src/main/circe/cpp/crc32c_sse42.cpp) compiled from
  /root/reference by ``Makefile`` (git-ignored build output; it travels to the GPU
  box as a prebuilt file because /root/reference does not exist there).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libcirce_ref.so")
REF_ROOT = "/root/reference"

CRC32C = 0
CRC32 = 1

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build(force: bool = False) -> None:
    """Compile the checkers (liboracle.so always; _ref only where the reference exists)."""
    targets = ["oracle"]
    if os.path.isdir(REF_ROOT):
        targets.append("ref")
    if force or not os.path.exists(ORACLE_SO) or ("ref" in targets and not os.path.exists(REF_SO)):
        subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_resume.restype = ctypes.c_uint32
        L.oracle_resume.argtypes = [ctypes.c_int, ctypes.c_uint32, _u8p, ctypes.c_uint64]
        L.oracle_resume_bitwise.restype = ctypes.c_uint32
        L.oracle_resume_bitwise.argtypes = [ctypes.c_int, ctypes.c_uint32, _u8p, ctypes.c_uint64]
        L.oracle_batch.restype = None
        L.oracle_batch.argtypes = [ctypes.c_int, _u8p, _u64p, _u32p, ctypes.c_uint64, _u32p,
                                   ctypes.c_uint32, _u32p]
        L.oracle_uniform.restype = None
        L.oracle_uniform.argtypes = [ctypes.c_int, _u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                     ctypes.c_uint32, _u32p]
        L.oracle_gf_mul.restype = ctypes.c_uint32
        L.oracle_gf_mul.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_xpow8n.restype = ctypes.c_uint32
        L.oracle_xpow8n.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.oracle_combine.restype = ctypes.c_uint32
        L.oracle_combine.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_digest_entry.restype = ctypes.c_uint32
        L.oracle_digest_entry.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int64, _u8p, ctypes.c_uint64, _u8p]
        L.oracle_digest_bytes.restype = ctypes.c_int
        L.oracle_digest_bytes.argtypes = [ctypes.c_int, ctypes.c_uint32, _u8p]
        L.oracle_verify_entry.restype = ctypes.c_int
        L.oracle_verify_entry.argtypes = [ctypes.c_int, _u8p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int]
        L.oracle_fill_splitmix64.restype = None
        L.oracle_fill_splitmix64.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_entrylog_scan.restype = ctypes.c_uint64
        L.oracle_entrylog_scan.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint64, _u64p, _u32p,
                                           ctypes.POINTER(ctypes.c_int64), ctypes.c_uint64, _u64p]
        L.oracle_zlib_crc32_batch_timed.restype = ctypes.c_double
        L.oracle_zlib_crc32_batch_timed.argtypes = [_u8p, _u64p, _u32p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                                    _u32p]
        L.oracle_pclmul_crc32_batch_timed.restype = ctypes.c_double
        L.oracle_pclmul_crc32_batch_timed.argtypes = [_u8p, _u64p, _u32p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                                      _u32p]
        L.oracle_table.restype = None
        L.oracle_table.argtypes = [ctypes.c_int, _u32p]
        L.oracle_zlib_verify_frames_timed.restype = ctypes.c_double
        L.oracle_zlib_verify_frames_timed.argtypes = [ctypes.c_void_p, _u32p, ctypes.c_uint64, ctypes.c_int64,
                                                      ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                                      ctypes.POINTER(ctypes.c_int32)]
        _lib = L
    return _lib


def ref():
    """The reference's compiled circe crc32c(), or None when it was never built here."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_SO) and os.path.isdir(REF_ROOT):
            build()
        if not os.path.exists(REF_SO):
            return None
        L = ctypes.CDLL(REF_SO)
        L.ref_supported.restype = ctypes.c_int
        L.ref_crc32c.restype = ctypes.c_uint32
        L.ref_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        L.ref_crc32c_unchunked.restype = ctypes.c_uint32
        L.ref_crc32c_unchunked.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
        L.ref_crc32c_batch.restype = None
        L.ref_crc32c_batch.argtypes = [_u8p, _u64p, _u32p, ctypes.c_uint64, _u32p, ctypes.c_uint32, _u32p]
        L.ref_crc32c_uniform_timed.restype = ctypes.c_double
        L.ref_crc32c_uniform_timed.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                               ctypes.c_int, ctypes.c_int, _u32p]
        L.ref_crc32c_batch_timed.restype = ctypes.c_double
        L.ref_crc32c_batch_timed.argtypes = [_u8p, _u64p, _u32p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, _u32p]
        L.ref_verify_frames_timed.restype = ctypes.c_double
        L.ref_verify_frames_timed.argtypes = [ctypes.c_void_p, _u32p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                              ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]
        _ref = L
    return _ref


def _as_u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return np.frombuffer(bytes(data), dtype=np.uint8)


def resume(algo: int, current: int, data) -> int:
    """Crc32cIntChecksum.resumeChecksum semantics (finalized `current`)."""
    a = _as_u8(data)
    return int(lib().oracle_resume(algo, current & 0xFFFFFFFF, _ptr(a, _u8p), a.size))


def calculate(algo: int, data) -> int:
    return resume(algo, 0, data)


def resume_bitwise(algo: int, current: int, data) -> int:
    a = _as_u8(data)
    return int(lib().oracle_resume_bitwise(algo, current & 0xFFFFFFFF, _ptr(a, _u8p), a.size))


def batch(algo: int, base: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, seeds=None,
          seed_all: int = 0) -> np.ndarray:
    base = _as_u8(base)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = offsets.size
    out = np.zeros(n, dtype=np.uint32)
    sp = None
    if seeds is not None:
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        sp = _ptr(seeds, _u32p)
    lib().oracle_batch(algo, _ptr(base, _u8p), _ptr(offsets, _u64p), _ptr(lengths, _u32p), n, sp,
                       seed_all & 0xFFFFFFFF, _ptr(out, _u32p))
    return out


def uniform(algo: int, base: np.ndarray, stride: int, length: int, n: int, seed_all: int = 0) -> np.ndarray:
    base = _as_u8(base)
    assert n == 0 or (n - 1) * stride + length <= base.size
    out = np.zeros(n, dtype=np.uint32)
    lib().oracle_uniform(algo, _ptr(base, _u8p), stride, length, n, seed_all & 0xFFFFFFFF, _ptr(out, _u32p))
    return out


def gf_mul(algo: int, a: int, b: int) -> int:
    return int(lib().oracle_gf_mul(algo, a, b))


def xpow8n(algo: int, nbytes: int) -> int:
    return int(lib().oracle_xpow8n(algo, nbytes))


def combine(algo: int, crc_a: int, crc_b: int, len_b: int) -> int:
    return int(lib().oracle_combine(algo, crc_a, crc_b, len_b))


def table(algo: int) -> np.ndarray:
    out = np.zeros(256, dtype=np.uint32)
    lib().oracle_table(algo, _ptr(out, _u32p))
    return out


def digest_entry(algo: int, ledger_id: int, entry_id: int, lac: int, length: int, payload) -> tuple[int, bytes]:
    p = _as_u8(payload)
    hdr = np.zeros(32, dtype=np.uint8)
    d = lib().oracle_digest_entry(algo, ledger_id, entry_id, lac, length, _ptr(p, _u8p), p.size, _ptr(hdr, _u8p))
    return int(d), hdr.tobytes()


def digest_bytes(algo: int, digest: int) -> bytes:
    out = np.zeros(8, dtype=np.uint8)
    k = lib().oracle_digest_bytes(algo, digest & 0xFFFFFFFF, _ptr(out, _u8p))
    return out[:k].tobytes()


def verify_entry(algo: int, framed, ledger_id: int, entry_id: int, skip_entry_check: bool = False) -> int:
    f = _as_u8(framed)
    return int(lib().oracle_verify_entry(algo, _ptr(f, _u8p), f.size, ledger_id, entry_id, int(skip_entry_check)))


def fill_splitmix64(nbytes: int, seed: int, first_word: int = 0) -> np.ndarray:
    out = np.zeros(nbytes, dtype=np.uint8)
    lib().oracle_fill_splitmix64(_ptr(out, _u8p), nbytes, seed, first_word)
    return out


def entrylog_scan(log, start: int = 1024):
    """DefaultEntryLogger.scanEntryLog restated: (offsets u64, lengths u32, ledger ids i64, end)."""
    a = _as_u8(log)
    cap = max(1, a.size // 16)
    while True:  # the walk counts past `cap`: a log of tinier records is walked again with room for all
        offs = np.zeros(cap, dtype=np.uint64)
        lens = np.zeros(cap, dtype=np.uint32)
        lids = np.zeros(cap, dtype=np.int64)
        end = np.zeros(1, dtype=np.uint64)
        n = int(lib().oracle_entrylog_scan(_ptr(a, _u8p), a.size, start, _ptr(offs, _u64p), _ptr(lens, _u32p),
                                           lids.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap, _ptr(end, _u64p)))
        if n <= cap:
            return offs[:n], lens[:n], lids[:n], int(end[0])
        cap = n
