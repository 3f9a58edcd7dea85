#!/usr/bin/env python3
"""Cost of a head chunk by its step count J (config 3's heads: J = 1..32 steps of 128 B).

For each J: n entries with lengths uniform in [128 J - 100, 128 J - 20], packed back to back
(unaligned, as Zipf heads are), one far longer entry at the end so the near-uniform gate stays off,
the short-entry class off. Every entry is one chunk of J steps. Timed end to end through the plan
(mode 2) and through the direct kernel (mode 1); reports time per chunk-round per lane group
(n / groups rounds) and GB/s. One JSON line per (J, mode).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import torch
    from bookkeeper_amd import checksum as ck
    from bookkeeper_amd._native import lib
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream(dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    groups = cus * 1024 // 8
    n = int(os.environ.get("HEADS_N", 8 * groups))
    rng = np.random.default_rng(5)
    ck.set_plan_small(0)
    reps = 10
    for J in [int(x) for x in os.environ.get("HEADS_J", "1 2 3 4 6 8 12 16 24 32").split()]:
        if os.environ.get("HEADS_ALIGN"):  # whole 128-byte steps, packed: every head line-aligned, no pad
            lens = np.full(n, 128 * J, dtype=np.int64)
        else:
            lens = rng.integers(128 * J - 100, 128 * J - 20, n).astype(np.int64)
            lens = np.maximum(lens, 17)
        lens[-1] = 60000
        offs = np.zeros(n, dtype=np.int64)
        np.cumsum(lens[:-1], out=offs[1:])
        total = int(offs[-1] + lens[-1])
        base = torch.empty(total, dtype=torch.uint8, device=dev)
        ck.fill_splitmix64(base, 42)
        d_off = torch.from_numpy(offs).to(dev)
        d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        res = {}
        for mode in [int(m) for m in os.environ.get("HEADS_MODES", "2 1").split()]:
            if mode == 3:  # the uniform kernel on the same bytes (aligned runs only: every entry 128 J)
                if not os.environ.get("HEADS_ALIGN"):
                    continue
                ck.set_group_lanes(8)
                call = lambda: ck.crc_batch_uniform(ck.CRC32C, base, 128 * J, n - 1, out=out, stream=st)
            else:
                ck.set_plan_mode(mode)
                call = lambda: ck.crc_batch(ck.CRC32C, base, d_off, d_len, out=out, stream=st)
            for _ in range(3):
                call()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                call()
            b.record(st)
            torch.cuda.synchronize()
            t = a.elapsed_time(b) / 1e3 / reps
            ck.set_group_lanes(0)
            res[mode] = out.clone()
            print(json.dumps({"J": J, "mode": {1: "direct", 2: "plan", 3: "uniform"}[mode], "n": n,
                              "aligned": bool(os.environ.get("HEADS_ALIGN")), "mean_len": float(lens[:-1].mean()),
                              "ms": round(t * 1e3, 4), "GB_s": round(total / t / 1e9, 1),
                              "us_per_round": round(t * 1e6 / (n / groups), 3)}), flush=True)
        if 1 in res and 2 in res:
            assert torch.equal(res[1], res[2]), J
        if 3 in res and 2 in res:
            assert torch.equal(res[3][:n - 1], res[2][:n - 1]), J
        del base, d_off, d_len, out
        torch.cuda.empty_cache()
    ck.set_plan_mode(0)
    ck.set_plan_small(192)


if __name__ == "__main__":
    main()
