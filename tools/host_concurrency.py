"""Concurrent host-resident verify callers (BatchedReadOp completions on several threads).

Each of T threads verifies its own ByteBufList of B framed 4 KiB entries (separate host buffers)
R times through bkd_digest_verify_batch_host; prints the aggregate GiB/s of payload and the mean
call latency. Run once per BKD_HOST_STAGES value (the staging-set pool size is read once per
process): python3 tools/host_concurrency.py [B]
"""
import ctypes
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from bookkeeper_amd import digest as dg
    from bookkeeper_amd._native import check, lib

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    R = 20
    L = 4096
    dm = dg.DigestManager.instantiate(7, b"", dg.DigestType.CRC32C)
    # frames are packaged by the library itself (host package batch), then verified
    rng = np.random.default_rng(3)
    pay = rng.integers(0, 256, (B, L - 36), dtype=np.uint8)
    ids = np.arange(B, dtype=np.int64)
    hdrs, _ = dm.package_batch_host(ids, ids - 1, np.full(B, L - 36), [pay[i] for i in range(B)])
    frames = [np.concatenate([hdrs[i], pay[i]]) for i in range(B)]
    ptrs = np.array([f.ctypes.data for f in frames], dtype=np.uint64)
    lens = np.array([f.size for f in frames], dtype=np.uint32)

    def call():
        status = np.zeros(B, dtype=np.int32)
        fb = ctypes.c_uint64(0)
        check(lib().bkd_digest_verify_batch_host(0, 7, 0, 0, ctypes.c_void_p(ptrs.ctypes.data),
                                                 ctypes.c_void_p(lens.ctypes.data), B,
                                                 ctypes.c_void_p(status.ctypes.data), ctypes.byref(fb)))
        assert fb.value == B and not status.any()

    for _ in range(3):
        call()
    stages = os.environ.get("BKD_HOST_STAGES", "4 (default)")
    for T in (1, 2, 4, 8):
        def run(reps):
            lat = []
            barrier = threading.Barrier(T)

            def worker():
                barrier.wait()
                for _ in range(reps):
                    t0 = time.perf_counter()
                    call()
                    lat.append(time.perf_counter() - t0)

            ts = [threading.Thread(target=worker) for _ in range(T)]
            t0 = time.perf_counter()
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            return time.perf_counter() - t0, lat

        run(2)  # untimed: staging sets created on first concurrent use (pinned allocations)
        wall, lat = run(R)
        gib = T * R * B * (L - 36) / 2**30
        print(f"stages {stages}  threads {T}  batch {B} x 4 KiB  {gib / wall:7.2f} GiB/s aggregate  "
              f"mean call {1e6 * sum(lat) / len(lat):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
