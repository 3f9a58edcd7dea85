"""Kernel breakdown of large uniform entries through the indexed plan (diagnostic, GPU box):
4096 x 1 MiB and 256 x 16 MiB, forced plan mode. Run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bookkeeper_amd import checksum as ck  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    total = 4 << 30
    base = torch.empty(total, dtype=torch.uint8, device=dev)
    ck.fill_splitmix64(base, 42)
    ck.set_plan_mode(2)
    for L in (1 << 20, 16 << 20):
        n = total // L
        offs = torch.arange(n, dtype=torch.int64, device=dev) * L
        lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        for _ in range(3):
            ck.crc_batch(ck.CRC32C, base, offs, lens, out=out)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            ck.crc_batch(ck.CRC32C, base, offs, lens, out=out)
        b.record()
        torch.cuda.synchronize()
        print(f"{n} x {L} B plan: {a.elapsed_time(b) / 10:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
