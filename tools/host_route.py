#!/usr/bin/env python3
"""Crossover of the host-resident batch routes.

1M framed 4 KiB entries in pageable host memory, each its own buffer (BatchedReadOp's ByteBufList):
verify and package through the GPU route (gather -> pinned -> PCIe -> device -> D2H) and through the
CPU route at 1, 2, 4, 8, ... host threads; bkd_crc_batch_host over one contiguous pageable buffer
both ways; and the reference's own loop (circe crc32c() per frame, two calls per frame as
DigestManager.verifyDigest makes them, oracle/_ref) at 1 and all threads. One JSON line per
measurement; every route's statuses / digests are checked equal.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

GIB = float(1 << 30)


def main() -> None:
    import bench
    import oracle
    from bookkeeper_amd import checksum as ck
    from bookkeeper_amd import digest as dg
    from bookkeeper_amd._native import check, lib
    n = int(os.environ.get("HOST_ROUTE_N", 1 << 20))
    L = 4096
    reps = int(os.environ.get("HOST_ROUTE_REPS", 3))
    cores, why = bench.host_cores()
    pool = ck.get_host_threads()
    print(json.dumps({"host_cores": cores, "cores_from": why, "pool_threads": pool, "cpu_impl": ck.cpu_impl(),
                      "cpu_model": bench._cpu_model(), "devices": lib().bkd_device_count()}), flush=True)
    dm = dg.DigestManager.instantiate(7, b"", dg.DigestType.CRC32C)
    plen = L - 36
    host = oracle.fill_splitmix64(n * L, 42)  # pageable, like Netty direct buffers
    base = host.ctypes.data
    ids = np.arange(n, dtype=np.int64)
    lacs = ids - 1
    lf = np.full(n, plen, dtype=np.int64)
    pay_ptrs = (base + ids.astype(np.uint64) * L + 36).astype(np.uint64)
    pay_lens = np.full(n, plen, dtype=np.uint32)
    hdrs = np.zeros((n, 36), dtype=np.uint8)
    digests = np.zeros(n, dtype=np.uint32)
    vp = ctypes.c_void_p

    def package():
        check(lib().bkd_digest_package_batch_host(0, 7, vp(ids.ctypes.data), vp(lacs.ctypes.data), vp(lf.ctypes.data),
                                                  vp(pay_ptrs.ctypes.data), vp(pay_lens.ctypes.data), n,
                                                  vp(hdrs.ctypes.data), 36, vp(digests.ctypes.data)))
    with ck.host_batch_route(ck.HOST_ROUTE_CPU):
        package()
    host.reshape(n, L)[:, :36] = hdrs
    ref_digests = digests.copy()
    frame_ptrs = (base + ids.astype(np.uint64) * L).astype(np.uint64)
    frame_lens = np.full(n, L, dtype=np.uint32)
    status = np.zeros(n, dtype=np.int32)
    fb = ctypes.c_uint64(0)

    def verify():
        check(lib().bkd_digest_verify_batch_host(0, 7, 0, 0, vp(frame_ptrs.ctypes.data), vp(frame_lens.ctypes.data), n,
                                                 vp(status.ctypes.data), ctypes.byref(fb)))
    offs = ids.astype(np.uint64) * L
    lens = np.full(n, L, dtype=np.uint32)
    crc_out = {}

    def crc_host():
        crc_out["v"] = ck.crc_batch_host(0, host, offs, lens)

    def timed(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return (time.perf_counter() - t0) / reps

    def emit(route, threads, what, t):
        print(json.dumps({"route": route, "threads": threads, "op": what, "GiB_s": round(n * L / t / GIB, 2),
                          "ms": round(t * 1e3, 2), "entries": n}), flush=True)

    want_crc = None
    for route, name in ((ck.HOST_ROUTE_GPU, "gpu"), (ck.HOST_ROUTE_CPU, "cpu")):
        if route == ck.HOST_ROUTE_GPU and lib().bkd_device_count() <= 0:
            continue
        thread_set = [0] if route == ck.HOST_ROUTE_GPU else sorted({1, 2, 4, 8, pool} & set(range(1, pool + 1)))
        with ck.host_batch_route(route):
            for thr in thread_set:
                ck.set_host_threads(thr)
                label = "copy pool default" if route == ck.HOST_ROUTE_GPU else thr
                emit(name, label, "verify", timed(verify))
                assert (status == 0).all() and fb.value == n, name
                emit(name, label, "package", timed(package))
                assert (digests == ref_digests).all(), name
                emit(name, label, "crc_batch_host (contiguous pageable)", timed(crc_host))
                if want_crc is None:
                    want_crc = crc_out["v"].copy()
                assert (crc_out["v"] == want_crc).all(), name
        ck.set_host_threads(0)
    ref = oracle.ref()
    if ref is not None:
        st = np.zeros(n, dtype=np.int32)
        for thr in sorted({1, cores}):
            t = ref.ref_verify_frames_timed(frame_ptrs.ctypes.data, frame_lens.ctypes.data_as(oracle._u32p), n, 7, 0,
                                            thr, 1, st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
            assert (st == 0).all()
            emit("reference circe (oracle/_ref)", thr, "verify", t)


if __name__ == "__main__":
    main()
