#!/usr/bin/env python3
"""Launch ramp with the shader clock beside it (the driver-window transient).

For each library build given (default: the package's), after --idle-ms of host sleep, runs a burst
of --launches back-to-back headline launches (1M x 4 KiB CRC32C, as bench.py) with a HIP event pair
around each, and — with --probe — tools/libclockprobe.so's 20 us clock probe after each launch, so
every launch time has the shader clock measured right after it. Rounds alternate the builds.
One JSON line per (round, build): per-launch ms, per-launch MHz, the driver-window mean
(launches 5..24) and the steady mean (launches 50..).
"""
import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def load_lib(path):
    from bookkeeper_amd import _native
    L = ctypes.CDLL(os.path.abspath(path))
    for fn, (res, argt) in _native.PROTOTYPES.items():
        if hasattr(L, fn):
            getattr(L, fn).restype = res
            getattr(L, fn).argtypes = argt
    return L


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--launches", type=int, default=80)
    ap.add_argument("--idle-ms", type=float, default=2000.0)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="measurement-only builds whose digests differ")
    args = ap.parse_args()
    import torch
    libs = args.libs or [os.path.join(ROOT, "bookkeeper_amd", "libbkdigest.so")]
    # a library may carry ":LANES" (bkd_set_group_lanes before its launches; the same file loads once)
    loaded = {}
    Ls = []
    for spec in libs:
        path, _, lanes = spec.partition(":")
        if path not in loaded:
            loaded[path] = load_lib(path)
        Ls.append((os.path.basename(path) + (f":{lanes}" if lanes else ""), loaded[path], int(lanes or 0)))
    probe = None
    if args.probe:
        probe = ctypes.CDLL(os.path.join(HERE, "libclockprobe.so"))
        probe.clock_probe_launch.restype = ctypes.c_int
        probe.clock_probe_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, E = 1 << 20, 4096
    base = torch.empty(n * E, dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    clk = torch.zeros((args.launches, 8, 2), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    Ls[0][1].bkd_fill_splitmix64(ctypes.c_void_p(base.data_ptr()), base.numel(), 42, 0, sp)
    torch.cuda.synchronize()
    ref = None
    for rnd in range(args.rounds):
        for name, L, lanes in Ls:
            L.bkd_set_group_lanes(lanes)
            time.sleep(args.idle_ms / 1e3)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.launches)]
            for k, (a, b) in enumerate(evs):
                a.record(st)
                rc = L.bkd_crc_batch_uniform(0, ctypes.c_void_p(base.data_ptr()), E, E, n, None, 0,
                                             ctypes.c_void_p(out.data_ptr()), sp)
                assert rc == 0, rc
                b.record(st)
                if probe is not None:
                    assert probe.clock_probe_launch(sp, ctypes.c_void_p(clk[k].data_ptr()), 2000) == 0
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert args.no_check or torch.equal(out, ref), "builds disagree"
            ms = [a.elapsed_time(b) for a, b in evs]
            res = {"lib": name, "round": rnd, "idle_ms": args.idle_ms, "probe": bool(probe),
                   "mean_5_25": round(sum(ms[5:25]) / 20, 4),
                   "mean_50_end": round(sum(ms[50:]) / max(1, len(ms[50:])), 4),
                   "per_launch_ms": [round(x, 4) for x in ms]}
            if probe is not None:
                c = clk.cpu().numpy()
                mhz = (c[:, :, 0] / c[:, :, 1] * 100.0).mean(axis=1)
                res["mhz"] = [round(float(x)) for x in mhz]
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
