"""ctypes binding of libbkdigest.so (include/bkdigest.h).

There is deliberately no Python fallback: if the library is missing, every call raises
NativeUnavailable. Inside the library, device-resident batch calls always run on the GPU
(BKD_ERR_NO_DEVICE without one); host-resident batches and the per-call host-buffer resume have the
library's own native CPU route (host_crc.cpp, host_batch.cpp), the role the reference's JNI SSE4.2
provider plays in its selection chain (Crc32cIntChecksum.java:28-36).
"""
from __future__ import annotations

import ctypes
import os
import re

from .build import LIB, ROOT

CRC32C = 0
CRC32 = 1

BKD_OK = 0
ERRORS = {-1: "BKD_ERR_INVALID_ARG", -2: "BKD_ERR_NO_DEVICE", -3: "BKD_ERR_HIP", -4: "BKD_ERR_BOUNDS",
          -5: "BKD_ERR_NOMEM"}

VERIFY_OK = 0
VERIFY_TOO_SHORT = 1
VERIFY_DIGEST_MISMATCH = 2
VERIFY_LEDGER_MISMATCH = 3
VERIFY_ENTRY_MISMATCH = 4

HEADER_PATH = os.path.join(ROOT, "include", "bkdigest.h")


class NativeUnavailable(RuntimeError):
    """libbkdigest.so is missing or could not be loaded."""


class BkdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


_c = ctypes
_vp = _c.c_void_p
_u32 = _c.c_uint32
_u64 = _c.c_uint64
_i64 = _c.c_int64
_int = _c.c_int

# name -> (restype, argtypes); must cover every function declared in include/bkdigest.h
PROTOTYPES = {
    "bkd_abi_version": (_int, []),
    "bkd_device_count": (_int, []),
    "bkd_init": (_int, [_int]),
    "bkd_last_error": (_c.c_char_p, []),
    "bkd_crc_batch_uniform": (_int, [_int, _vp, _u64, _u32, _u64, _vp, _u32, _vp, _vp]),
    "bkd_crc_batch": (_int, [_int, _vp, _u64, _vp, _vp, _u64, _vp, _u32, _vp, _vp]),
    "bkd_crc_batch_segments": (_int, [_int, _vp, _u64, _vp, _vp, _u64, _vp, _u64, _vp, _u32, _vp, _vp]),
    "bkd_stream_sync": (_int, [_vp]),
    "bkd_stream_release": (_int, [_vp]),
    "bkd_crc_batch_host": (_int, [_int, _vp, _u64, _vp, _vp, _u64, _vp, _u32, _vp]),
    "bkd_resume": (_int, [_int, _u32, _vp, _u64, _c.POINTER(_u32)]),
    "bkd_resume_host": (_int, [_int, _u32, _vp, _u64, _c.POINTER(_u32)]),
    "bkd_resume_device": (_int, [_int, _u32, _vp, _u64, _vp, _c.POINTER(_u32)]),
    "bkd_cpu_resume": (_int, [_int, _u32, _vp, _u64, _c.POINTER(_u32)]),
    "bkd_set_cpu_route_max": (_int, [_u64]),
    "bkd_get_cpu_route_max": (_u64, []),
    "bkd_cpu_impl": (_c.c_char_p, []),
    "bkd_circe_supported": (_int, []),
    "bkd_circe_alloc_config": (_i64, [_vp, _c.c_int32]),
    "bkd_circe_free_config": (None, [_i64]),
    "bkd_digest_verify_batch_host": (_int, [_int, _i64, _i64, _int, _vp, _vp, _u64, _vp, _vp]),
    "bkd_digest_package_batch_host": (_int, [_int, _i64, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _u64, _vp]),
    "bkd_digest_package_batch": (_int, [_int, _i64, _vp, _vp, _vp, _vp, _u64, _vp, _vp, _u64, _vp, _u64, _vp, _vp]),
    "bkd_digest_verify_batch": (_int, [_int, _i64, _i64, _int, _vp, _u64, _vp, _vp, _u64, _vp, _vp, _vp]),
    "bkd_entrylog_index": (_int, [_vp, _u64, _u64, _vp, _vp, _vp, _u64, _vp, _vp]),
    "bkd_entrylog_verify": (_int, [_int, _vp, _u64, _vp, _vp, _u64, _vp, _vp, _vp]),
    "bkd_fill_splitmix64": (_int, [_vp, _u64, _u64, _u64, _vp]),
    "bkd_host_tables": (_i64, [_int, _int, _vp, _u64]),
    "bkd_host_gf_mul": (_u32, [_int, _u32, _u32]),
    "bkd_host_xpow8n": (_u32, [_int, _u64]),
    "bkd_set_group_lanes": (_int, [_int]),
    "bkd_set_fold_schedule": (_int, [_int]),
    "bkd_set_short_class_mean": (_int, [_u64]),
    "bkd_set_plan_mode": (_int, [_int]),
    "bkd_set_plan_geometry": (_int, [_int, _int, _int]),
    "bkd_set_plan_prefetch": (_int, [_int]),
    "bkd_set_plan_small": (_int, [_u32]),
    "bkd_set_plan_serial": (_int, [_u32]),
    "bkd_get_group_lanes": (_int, [_int, _u64]),
    "bkd_set_host_batch_route": (_int, [_int]),
    "bkd_get_host_batch_route": (_int, []),
    "bkd_set_host_threads": (_int, [_int]),
    "bkd_get_host_threads": (_int, []),
    "bkd_host_release": (_int, []),
}

_lib = None


def declared_functions() -> list[str]:
    """Function names declared in include/bkdigest.h (the ABI contract)."""
    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bkd_[a-z0-9_]+)\s*\(", text)))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise NativeUnavailable(f"{LIB} not built (run __graft_entry__.build() or python -m bookkeeper_amd.build)")
        try:
            L = ctypes.CDLL(LIB)
        except OSError as e:  # pragma: no cover
            raise NativeUnavailable(f"cannot load {LIB}: {e}") from e
        for name, (res, args) in PROTOTYPES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return (lib().bkd_last_error() or b"").decode(errors="replace")


def check(rc: int) -> int:
    if rc < 0:
        raise BkdError(rc, last_error())
    return rc


def device_count() -> int:
    return int(lib().bkd_device_count())
