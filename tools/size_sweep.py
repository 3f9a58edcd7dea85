"""Entry-size sweep (diagnostic, GPU box): device-resident uniform batches of 16 B .. 1 MiB entries
through bkd_crc_batch_uniform (automatic lane choice, and every lane count), plus the same layout
through the indexed path (chunked plan, and the direct indexed kernel). ~4 GiB per batch. Prints one line per point; each
configuration's output is checked against the first lane choice's."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bookkeeper_amd import checksum as ck  # noqa: E402

GIB = 1 << 30
TOTAL = 4 << 30


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / 1e3


def main():
    dev = torch.device("cuda", 0)
    base = torch.empty(TOTAL, dtype=torch.uint8, device=dev)
    ck.fill_splitmix64(base, 42)
    print(f"{'entry B':>9} {'entries':>9} {'path':>10} {'lanes':>5} {'ms':>8} {'GiB/s':>8} {'Mentries/s':>11}")
    for L in (16, 32, 48, 64, 128, 256, 512, 1024, 4096, 16384, 65536, 1 << 20):
        n = TOTAL // L
        out = torch.empty(n, dtype=torch.int32, device=dev)
        ref = None
        for lanes in ((0, 1, 4, 8) if L <= 64 else (0, 4, 8, 16, 32)):
            ck.set_group_lanes(lanes)
            t = timed(lambda: ck.crc_batch_uniform(ck.CRC32C, base, L, n, out=out))
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), (L, lanes)
            # bkd_get_group_lanes knows only the mean length; the uniform call also takes one lane
            # per entry for 16-48 B batches that fill the chip, so those print plain "auto"
            used = "" if L <= 48 else "=" + str(ck.lib().bkd_get_group_lanes(ck.CRC32C, L))
            print(f"{L:9d} {n:9d} {'uniform':>10} {('auto' + used) if lanes == 0 else lanes:>5} "
                  f"{t * 1e3:8.3f} {n * L / t / GIB:8.1f} {n / t / 1e6:11.1f}", flush=True)
        ck.set_group_lanes(0)
        offs = torch.arange(n, dtype=torch.int64, device=dev) * L
        lens = torch.full((n,), L, dtype=torch.int32, device=dev)
        ck.set_plan_mode(2)
        t = timed(lambda: ck.crc_batch(ck.CRC32C, base, offs, lens, out=out))
        ck.set_plan_mode(0)
        assert torch.equal(out, ref), (L, "plan")
        print(f"{L:9d} {n:9d} {'plan':>10} {8:>5} {t * 1e3:8.3f} {n * L / t / GIB:8.1f} {n / t / 1e6:11.1f}",
              flush=True)
        # the direct indexed kernel (one entry per lane group, automatic lanes) on the same index
        ck.set_plan_mode(1)
        t = timed(lambda: ck.crc_batch(ck.CRC32C, base, offs, lens, out=out))
        ck.set_plan_mode(0)
        assert torch.equal(out, ref), (L, "direct")
        print(f"{L:9d} {n:9d} {'direct':>10} {'auto':>5} {t * 1e3:8.3f} {n * L / t / GIB:8.1f} {n / t / 1e6:11.1f}",
              flush=True)
        del out, offs, lens
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
