"""Per-call latency of the IntHash drop-in (bkd_resume) on device and host buffers (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from bookkeeper_amd import checksum as ck

h = ck.GpuIntHash()
dev = torch.device("cuda", 0)
for n in (64, 4096, 65536, 1 << 20, 64 << 20):
    t = torch.empty(n, dtype=torch.uint8, device=dev)
    ck.fill_splitmix64(t, 1)
    a = t.cpu().numpy()
    torch.cuda.synchronize()
    for name, buf in (("device", t), ("host", a)):
        h.resume(0, buf, 0, n)
        reps = 200 if n <= 65536 else 20
        t0 = time.perf_counter()
        for _ in range(reps):
            r = h.resume(0, buf, 0, n)
        dt = (time.perf_counter() - t0) / reps
        print(f"{n:>10} B {name:6s} {dt * 1e6:9.1f} us/call  {n / dt / 2**30:8.2f} GiB/s  crc={r & 0xFFFFFFFF:08x}", flush=True)
