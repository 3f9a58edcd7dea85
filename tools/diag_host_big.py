#!/usr/bin/env python3
"""Repeated GPU-route host resumes / host batches of one long entry (r03j: a 256 MiB per-call resume
through the GPU route differed from the CPU fold on some calls). Prints rc and value per call."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    from bookkeeper_amd import _native
    from bookkeeper_amd import checksum as ck
    L = _native.lib()
    if os.environ.get("DIAG_LIB"):  # a variant build, same prototypes
        import ctypes as ct
        V = ct.CDLL(os.environ["DIAG_LIB"])
        for name in ("bkd_set_cpu_route_max", "bkd_set_host_batch_route", "bkd_resume_host"):
            f = getattr(V, name)
            f.restype, f.argtypes = getattr(L, name).restype, getattr(L, name).argtypes
        L = V
    M = 1 << 20
    host = np.frombuffer(np.random.default_rng(3).bytes(512 * M), dtype=np.uint8)
    L.bkd_set_cpu_route_max(0)
    L.bkd_set_host_batch_route(2)
    for size in [int(x) * M for x in os.environ.get("SIZES", "64 128 256 512").split()]:
        want = ck.cpu_resume(ck.CRC32C, 0, host[:size]) & 0xFFFFFFFF
        bad = []
        for k in range(int(os.environ.get("REPS", "8"))):
            out = ctypes.c_uint32(0)
            rc = L.bkd_resume_host(0, 0, ctypes.c_void_p(host.ctypes.data), ctypes.c_uint64(size), ctypes.byref(out))
            if rc != 0 or out.value != want:
                bad.append((k, rc, hex(out.value), _native.last_error() if rc else ""))
        print(size, hex(want), "bad calls:", bad, flush=True)
    L.bkd_set_host_batch_route(0)


if __name__ == "__main__":
    main()
