#!/usr/bin/env python3
"""Per-launch timing of the headline kernel from the first launch on.

Runs the exact setup of `bench.py` (1M x 4 KiB entries, device-generated splitmix64) and times
every one of the first N launches on its own (a HIP event pair per launch on the launch stream),
so a clock ramp, first-touch translation misses or a first-launch cost show up as a trend over
launch index. Prints one JSON line: per-launch ms, plus means over the windows the driver's
command (--steps 20 --warmup 5: launches 5..24) and the builder's (--steps 100 --warmup 50:
launches 50..149) time.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep before the first launch")
    ap.add_argument("--touch", action="store_true", help="read the whole buffer once (torch sum) before launching")
    ap.add_argument("--rounds", type=int, default=1, help="bursts, each after --idle-ms of host sleep")
    ap.add_argument("--lib", default=None, help="a libbkdigest.so build to time (default: the package's)")
    args = ap.parse_args()
    import torch
    from bookkeeper_amd import checksum as ck
    if args.lib:  # a variant build: the checksum wrappers call it through _native.lib()
        import ctypes
        from bookkeeper_amd import _native
        L = ctypes.CDLL(os.path.abspath(args.lib))
        for fn, (res, argt) in _native.PROTOTYPES.items():
            if hasattr(L, fn):
                getattr(L, fn).restype = res
                getattr(L, fn).argtypes = argt
        _native._lib = L
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, L = 1 << 20, 4096
    base = torch.empty(n * L, dtype=torch.uint8, device=dev)
    ck.fill_splitmix64(base, 42)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()
    if args.touch:
        base.view(torch.int64).sum().item()
    for rnd in range(args.rounds):
        if args.idle_ms:
            time.sleep(args.idle_ms / 1e3)
        burst(args, torch, ck, base, out, stream, L, n, rnd)


def burst(args, torch, ck, base, out, stream, L, n, rnd):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.launches)]
    span0, span1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    span0.record(stream)
    for a, b in evs:
        a.record(stream)
        ck.crc_batch_uniform(ck.CRC32C, base, L, n, out=out, stream=stream)
        b.record(stream)
    span1.record(stream)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in evs]

    def mean(lo, hi):
        w = ms[lo:hi]
        return round(sum(w) / len(w), 4) if w else None
    res = {"lib": args.lib or "bookkeeper_amd/libbkdigest.so", "round": rnd, "launches": args.launches, "idle_ms": args.idle_ms, "touch": args.touch,
           "first10_ms": [round(x, 4) for x in ms[:10]],
           "mean_0_5": mean(0, 5), "mean_5_25_driver_window": mean(5, 25), "mean_25_50": mean(25, 50),
           "mean_50_150_builder_window": mean(50, 150), "mean_150_end": mean(150, args.launches),
           "span_ms_per_launch": round(span0.elapsed_time(span1) / args.launches, 4),
           "per_launch_ms": [round(x, 4) for x in ms]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
