"""Diagnostic: per-kernel cost of the ragged-batch plan on several workloads, in one process.

Run under `rocprofv3 --kernel-trace --output-format csv -d DIR -o diag -- python3 tools/diag_ragged.py`,
then `python3 tools/diag_ragged.py --report DIR/diag_kernel_trace.csv`. Workloads are separated in
the trace by a marker launch (fill_splitmix64 on a 64-byte buffer); their order is WORKLOADS'.
"""
import csv
import re
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REPS = 10
WORKLOADS = (os.environ.get("DIAG_WORKLOADS") or
             "uniform4k_direct indexed4k_plan zipf_plan zipf_plan_8x64 zipf_plan_16x16 zipf_ge4k_plan "
             "zipf_lt1k_plan zipf_lt1k_direct zipf_plan_crc32").split()


def run():
    import numpy as np
    import torch
    from bench import zipf_index
    from bookkeeper_amd import checksum as ck

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream()
    marker = torch.empty(64, dtype=torch.uint8, device=dev)
    n = 1 << 20
    offs, lens = zipf_index(n)
    total = int(offs[-1] + lens[-1])
    base = torch.empty(max(total, n * 4096), dtype=torch.uint8, device=dev)
    ck.fill_splitmix64(base, 42)
    out = torch.empty(max(n, int(os.environ.get("DIAG_PACKED_N", n))), dtype=torch.int32, device=dev)

    def indexed(o, l):
        return torch.from_numpy(np.ascontiguousarray(o)).to(dev), torch.from_numpy(l.astype(np.int32)).to(dev)

    zo, zl = indexed(offs, lens)
    uo, ul = indexed(np.arange(n, dtype=np.int64) * 4096, np.full(n, 4096))
    ge = lens >= 4096
    go, gl = indexed(offs[ge], lens[ge])
    lt = lens < 1024
    lo, ll = indexed(offs[lt], lens[lt])
    # the Zipf entries split into what the plan makes of them: full 4 KiB chunks (lengths rounded down to
    # 4 KiB, 4 KiB-aligned, packed: no heads) and the heads alone (len mod 4 KiB, packed, unaligned)
    full_l = (lens // 4096) * 4096
    fl_keep = full_l > 0
    fo = np.zeros(int(fl_keep.sum()), dtype=np.int64)
    np.cumsum(full_l[fl_keep][:-1], out=fo[1:])
    fuo, ful = indexed(fo, full_l[fl_keep])
    head_l = np.where(lens % 4096 == 0, 4096, lens % 4096)
    ho = np.zeros(n, dtype=np.int64)
    np.cumsum(head_l[:-1], out=ho[1:])
    hdo, hdl = indexed(ho, head_l)
    perm = np.random.default_rng(1).permutation(n)
    sho, shl = indexed(np.arange(n, dtype=np.int64)[perm] * 4096, np.full(n, 4096))
    e8o, e8l = indexed(np.arange(n // 2, dtype=np.int64) * 8192, np.full(n // 2, 8192))

    def plan(geom=(8, 32, 16), pf=2, algo=0, o=zo, l=zl):
        def f():
            ck.set_plan_mode(2)
            ck.set_plan_geometry(*geom)
            ck.set_plan_prefetch(pf)
            ck.set_plan_small(int(os.environ.get("DIAG_SMALL", "0")))
            ck.crc_batch(algo, base, o, l, out=out[: o.numel()], stream=st)
        return f

    def direct_idx(o, l):
        def f():
            ck.set_plan_mode(1)
            ck.crc_batch(0, base, o, l, out=out[: o.numel()], stream=st)
        return f

    jobs = {
        "uniform4k_direct": lambda: ck.crc_batch_uniform(0, base, 4096, n, out=out, stream=st),
        "indexed4k_plan": plan(o=uo, l=ul),
        "zipf_plan": plan(),
        "zipf_plan_pf4": plan(pf=4),
        "zipf_plan_8x64": plan(geom=(8, 64, 16)),
        "zipf_plan_16x16": plan(geom=(16, 16, 16)),
        "zipf_ge4k_plan": plan(o=go, l=gl),
        "zipf_lt1k_plan": plan(o=lo, l=ll),
        "zipf_lt1k_direct": direct_idx(lo, ll),
        "zipf_plan_crc32": plan(algo=1),
        "zipf_plan_4x64": plan(geom=(4, 64, 16)),
        "zipf_plan_4x128": plan(geom=(4, 128, 16)),
        "zipf_plan_8x32_m4096": plan(geom=(8, 32, 4096)),
        "zipf_plan_4x64_m4096": plan(geom=(4, 64, 4096)),
        "zipf_plan_8x32_m1024": plan(geom=(8, 32, 1024)),
        "zipf_plan_8x32_m512": plan(geom=(8, 32, 512)),
        "zipf_plan_8x32_m2048": plan(geom=(8, 32, 2048)),
        "zipf_plan_8x32_m1536": plan(geom=(8, 32, 1536)),
        "zipf_plan_8x24_m1024": plan(geom=(8, 24, 1024)),
        "zipf_plan_8x48_m1024": plan(geom=(8, 48, 1024)),
        "zipf_plan_8x64_m2048": plan(geom=(8, 64, 2048)),
        "zipf_heads_plan_4x64": plan(o=hdo, l=hdl, geom=(4, 64, 16)),
        "zipf_lt1k_plan_4x64": plan(o=lo, l=ll, geom=(4, 64, 16)),
        "indexed4k_shuffled_plan": plan(o=sho, l=shl),
        "indexed4k_shuffled_direct": direct_idx(sho, shl),
        "indexed8k_plan": plan(o=e8o, l=e8l),
        "zipf_fullchunks_plan": plan(o=fuo, l=ful),
        "zipf_fullchunks_direct": direct_idx(fuo, ful),
        "zipf_heads_plan": plan(o=hdo, l=hdl),
        "zipf_heads_direct": direct_idx(hdo, hdl),
    }
    # packed{S}_{plan|direct|plan4}: n entries of S bytes back to back (unaligned starts)
    info_pk = {}
    for name in WORKLOADS:
        m = re.match(r"packed(\d+)_(plan4|plan|direct)$", name)
        if not m:
            continue
        S = int(m.group(1))
        npk = min(int(os.environ.get("DIAG_PACKED_N", n)), base.numel() // S)
        po, pl = indexed(np.arange(npk, dtype=np.int64) * S, np.full(npk, S))
        info_pk[name] = (npk, npk * S)
        kind = m.group(2)
        jobs[name] = (direct_idx(po, pl) if kind == "direct" else
                      plan(o=po, l=pl, geom=(4, 64, 16) if kind == "plan4" else (8, 32, 16)))
    info = {"zipf_ge4k_plan": (int(ge.sum()), int(lens[ge].sum())),
            "zipf_ge4k_plan_o0": (int(ge.sum()), int(lens[ge].sum())), "zipf_lt1k_plan": (int(lt.sum()), int(lens[lt].sum())),
            "zipf_lt1k_direct": (int(lt.sum()), int(lens[lt].sum())),
            "zipf_fullchunks_plan": (int(fl_keep.sum()), int(full_l.sum())),
            "zipf_fullchunks_direct": (int(fl_keep.sum()), int(full_l.sum())),
            "zipf_heads_plan": (n, int(head_l.sum())), "zipf_heads_direct": (n, int(head_l.sum())),
            "indexed8k_plan": (n // 2, n * 4096)}
    info.update(info_pk)
    ref = {}
    for name in WORKLOADS:
        f = jobs[name]
        ck.fill_splitmix64(marker, 1, stream=st)
        f()  # warm-up, inside the segment (each segment holds REPS + 1 calls)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(REPS):
            f()
        e1.record(st)
        torch.cuda.synchronize()
        if name.startswith("zipf_plan") and "crc32" not in name:
            if ref.get("zipf") is None:
                ref["zipf"] = out.clone()
            assert torch.equal(ref["zipf"], out), f"{name}: digests differ from the first zipf run"
        ne, nb = info.get(name, (n, total if "zipf" in name else n * 4096))
        ms = e0.elapsed_time(e1) / REPS
        print(f"{name:20s} {ms:.4f} ms/call  entries {ne}  bytes {nb}  {nb / ms / 1e6:.0f} GB/s", flush=True)
    ck.set_plan_mode(0)
    ck.set_plan_geometry(8, 32, 16)
    ck.set_plan_prefetch(2)


def report(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seg = -1
    acc = defaultdict(lambda: defaultdict(list))
    for r in rows:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "fill_splitmix64" in name and dur < 20 and seg + 1 < len(WORKLOADS):
            seg += 1
            continue
        if seg >= 0:
            short = name.split("(")[0].replace("void ", "").replace("bkd::", "")
            acc[WORKLOADS[seg]][short].append(dur)
    for w in WORKLOADS:
        ks = acc[w]
        tot = sum(sum(v) for v in ks.values()) / (REPS + 1)
        print(f"== {w}: sum of kernel time {tot:.1f} us/call")
        for k, v in sorted(ks.items(), key=lambda kv: -sum(kv[1])):
            print(f"   {k[:60]:60s} x{len(v) // (REPS + 1)} {sum(v) / (REPS + 1):9.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
