#!/usr/bin/env python3
"""Headline benchmark: GiB/s CRC32C over batched 4 KiB ledger entries, device-resident.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 launched by
torch.distributed.run, one rank per GPU (``--gpus N`` without that environment starts the N ranks
itself, through torch.distributed.run, before anything touches a GPU). A step = one launch of the
digest engine over the whole per-GPU batch (BASELINE.json configs[1]: 1,048,576 x 4 KiB entries,
CRC32C, CRC init 0, bytes = little-endian splitmix64 stream seed 42, generated on the device). Entries
shard across ranks with no data-path collective (weak scaling); the only collectives are the
timing barriers, the max-over-ranks reduction and the gather of per-rank timings.

Rank 0 prints ONE JSON line with ``roofline`` (dominant kernel, HIP-event timed on its own
stream) and, at N=1, ``cpu_baseline`` (the reference's own circe crc32c() compiled from
/root/reference into oracle/_ref, timed on the host cores over a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters"
METRIC = "GiB/s CRC32C over batched 4 KiB ledger entries (device-resident); % HBM peak"


def metric_for(config: str, algo: str) -> str:
    """The line's metric string. Only config 2 (uniform 4 KiB, CRC32C) carries BASELINE.json's headline
    metric; every other workload names itself, so that no line can be read as the headline."""
    a = algo.upper()
    if config == "uniform4k" and algo == "crc32c":
        return METRIC
    if config == "uniform4k":
        return f"GiB/s {a} over batched 4 KiB ledger entries (device-resident); % HBM peak (not the headline)"
    if config == "shard8m":
        return (f"GiB/s {a} over 4 KiB ledger entries, config 4 shard: 8M entries (32 GiB) per GPU, "
                f"device-resident, aggregate over the GPUs; % HBM peak")
    if config == "zipf":
        return (f"GiB/s {a} over Zipf(1.1) 64 B-64 KiB ledger entries via offset+length index "
                f"(config 3, device-resident); % HBM peak")
    if config == "zipf_split":
        return (f"GiB/s {a} over config 3's Zipf(1.1) 64 B-64 KiB batch split across the GPUs by bytes "
                f"(strong scaling, device-resident); % HBM peak")
    if config == "indexed4k":
        return f"GiB/s {a} over 4 KiB ledger entries via offset+length index (diagnostic, not the headline)"
    return f"GiB/s {a} ({config})"


def zipf_index(n: int, seed: int = 43, s: float = 1.1, kmax: int = 1024, align: int = 1):
    """k ~ Zipf(s) on {1..kmax} by inverse CDF over a splitmix64 stream,
    len = max(64, 64k - (r & 63)); entries packed back to back (unaligned starts)."""
    words = np.frombuffer(_splitmix_words(2 * n, seed), dtype=np.uint64)
    u = (words[0::2] >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    r = words[1::2]
    k = np.arange(1, kmax + 1, dtype=np.float64)
    cdf = np.cumsum(k ** -s)
    cdf /= cdf[-1]
    kk = np.searchsorted(cdf, u, side="right") + 1
    kk = np.minimum(kk, kmax)
    lengths = np.maximum(64, 64 * kk - (r & np.uint64(63)).astype(np.int64)).astype(np.int64)
    if align > 1:  # diagnostic only: round lengths up so every entry starts on an `align` boundary
        lengths = (lengths + align - 1) // align * align
    offsets = np.zeros(n, dtype=np.int64)
    np.cumsum(lengths[:-1], out=offsets[1:])
    return offsets, lengths


def _splitmix_words(nwords: int, seed: int) -> bytes:
    i = np.arange(1, nwords + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.tobytes()


def shard_first_word(rank: int, entries_per_rank: int, entry_len: int) -> int:
    """The job's input is ONE global splitmix64 stream; rank r owns entries
    [r*entries_per_rank, (r+1)*entries_per_rank), i.e. stream words from this index on."""
    assert (entries_per_rank * entry_len) % 8 == 0
    return rank * entries_per_rank * entry_len // 8


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(nprocs: int, argv: list[str]) -> int:
    """``--gpus N`` outside torch.distributed.run: start the N ranks (one process per GPU) through
    torch.distributed.run on 127.0.0.1 as child processes and return their exit code. Called before
    anything in this process touches a GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nprocs}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    return subprocess.call(cmd)


def gather_over_ranks(values: list[float], device=None) -> list[list[float]]:
    """Every rank's timing values (all_gather of a few floats; timing only, never CRC data)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [list(values)]
    t = torch.tensor(values, dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def gather_identity(dev, world: int) -> list[dict]:
    """Each rank's device identity (name, PCI address, UUID) and the world size it saw after
    init_process_group, gathered to every rank: a multi-GPU line names the GPUs it ran on."""
    import torch
    import torch.distributed as dist
    p = torch.cuda.get_device_properties(dev)
    mine = {"device": p.name, "gcn_arch": getattr(p, "gcnArchName", ""),
            "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "uuid": str(getattr(p, "uuid", "")),
            "world_size_seen": dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1}
    if not (dist.is_available() and dist.is_initialized()):
        return [mine]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, mine)
    return out


def max_over_ranks(value: float, device=None) -> float:
    """Whole-job time = the slowest rank's (all_reduce MAX; the only cross-rank traffic)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_cores() -> tuple[int, str]:
    """Every core this process may run on: the affinity mask, capped by a cgroup CPU quota when one
    is set (a quota of Q cores makes more than Q threads time-slice, not run in parallel)."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    why = f"sched_getaffinity: {cores}"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, int(-(-int(quota) // int(period))))
            if q < cores:
                cores, why = q, f"{why}, cgroup cpu.max quota: {q}"
    except (OSError, ValueError):
        pass
    return max(1, cores), why


def cpu_baseline(host_sample: np.ndarray, entry_len: int, algo: int = 0, budget_s: float = 8.0):
    """Reference circe crc32c() (oracle/_ref) over the sample on one core and on every host core
    (all physical host cores)."""
    import oracle
    ref = oracle.ref()
    n = host_sample.size // entry_len
    out = np.zeros(n, dtype=np.uint32)
    cores, cores_why = host_cores()
    u8p = host_sample.ctypes.data_as(oracle._u8p)
    o32 = out.ctypes.data_as(oracle._u32p)
    if ref is not None and algo == 0:
        kind = "reference"
        run = lambda thr, reps: ref.ref_crc32c_uniform_timed(u8p, entry_len, entry_len, n, thr, reps, o32)
        label = "circe crc32c() (crc32c_sse42.cpp, chunk ladder {4096,512,64}) compiled from /root/reference"
    else:  # CRC-32: the JDK intrinsic's PCLMULQDQ folding, restated (oracle/cpu_baseline.c)
        kind = "port"
        lib = oracle.lib()
        offs = np.arange(n, dtype=np.uint64) * np.uint64(entry_len)
        lens = np.full(n, entry_len, dtype=np.uint32)

        def run(thr, reps):
            return lib.oracle_pclmul_crc32_batch_timed(u8p, offs.ctypes.data_as(oracle._u64p),
                                                       lens.ctypes.data_as(oracle._u32p), n, thr, reps, o32)
        label = ("PCLMULQDQ 4x128-bit folding (the arithmetic of java.util.zip.CRC32's HotSpot intrinsic), "
                 "oracle/cpu_baseline.c")
    t1 = run(1, 1)  # calibrate on one core
    one_core = host_sample.size / t1 / GIB
    reps = max(1, int(budget_s / max(1e-6, t1 / cores)))
    t = run(cores, reps)
    value = host_sample.size * reps / t / GIB
    return {"value": round(value, 3), "unit": "GiB/s", "cores": cores, "kind": kind,
            "single_core_value": round(one_core, 3), "cpu_model": _cpu_model(), "cores_from": cores_why,
            "sample": f"{n} x {entry_len} B entries of the same splitmix64 input ({host_sample.size / GIB:.3f} GiB, "
                      f"the full config-1 batch when n = 1M), one pass on 1 core, then {reps} passes over {cores} "
                      f"std::threads, one call per entry; {label}"}, out


def cpu_baseline_indexed(host: np.ndarray, offs: np.ndarray, lens: np.ndarray, algo: int = 0, budget_s: float = 8.0):
    """Config 3's CPU leg: one CRC per entry of an offset+length sample on the host cores. CRC32C:
    the reference's own circe crc32c() (oracle/_ref); CRC32: the PCLMULQDQ folding java.util.zip.CRC32's
    intrinsic runs (CRC32DigestManager.java:28-87), restated in oracle/cpu_baseline.c."""
    import oracle
    cores, cores_why = host_cores()
    n = offs.size
    out = np.zeros(n, dtype=np.uint32)
    o64 = np.ascontiguousarray(offs, dtype=np.uint64)
    l32 = np.ascontiguousarray(lens, dtype=np.uint32)
    ref = oracle.ref()
    if algo == 0 and ref is not None:
        kind, label = "reference", "circe crc32c() compiled from /root/reference"
        u8p = host.ctypes.data_as(oracle._u8p)

        def run(thr, reps):
            return ref.ref_crc32c_batch_timed(u8p, o64.ctypes.data_as(oracle._u64p), l32.ctypes.data_as(oracle._u32p),
                                              n, thr, reps, out.ctypes.data_as(oracle._u32p))
    else:
        kind = "port"
        label = ("PCLMULQDQ 4x128-bit folding, the arithmetic of java.util.zip.CRC32's HotSpot intrinsic "
                 "(CRC32DigestManager.java:28-87), oracle/cpu_baseline.c")
        lib = oracle.lib()
        u8p = host.ctypes.data_as(oracle._u8p)

        def run(thr, reps):
            return lib.oracle_pclmul_crc32_batch_timed(u8p, o64.ctypes.data_as(oracle._u64p),
                                                       l32.ctypes.data_as(oracle._u32p), n, thr, reps,
                                                       out.ctypes.data_as(oracle._u32p))
    nbytes = int(l32.sum())
    t1 = run(1, 1)
    reps = max(1, int(budget_s / max(1e-6, t1 / cores)))
    t = run(cores, reps)
    return {"value": round(nbytes * reps / t / GIB, 3), "unit": "GiB/s", "cores": cores, "kind": kind,
            "single_core_value": round(nbytes / t1 / GIB, 3), "cpu_model": _cpu_model(), "cores_from": cores_why,
            "sample": f"the first {n} entries of the same Zipf index ({nbytes / GIB:.3f} GiB), {reps} passes over "
                      f"{cores} threads, one call per entry; {label}"}, out


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:  # pragma: no cover
        pass
    return "unknown"


def bucket_rates(ck, torch, algo, base, offs, lens, stream, steps: int) -> dict:
    """Config 3's size buckets measured on their own: the entries < 1 KiB and the
    entries >= 16 KiB of the same packed buffer, each as one indexed batch."""
    res = {}
    dev = base.device
    for name, mask in (("lt_1KiB", lens < 1024), ("ge_16KiB", lens >= 16384)):
        idx = np.nonzero(mask)[0]
        if idx.size == 0:
            continue
        d_off = torch.from_numpy(offs[idx]).to(dev)
        d_len = torch.from_numpy(lens[idx].astype(np.int32)).to(dev)
        out = torch.empty(idx.size, dtype=torch.int32, device=dev)
        ck.crc_batch(algo, base, d_off, d_len, out=out, stream=stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(steps):
            ck.crc_batch(algo, base, d_off, d_len, out=out, stream=stream)
        b.record(stream)
        torch.cuda.synchronize()
        t = a.elapsed_time(b) / 1e3 / steps
        nbytes = int(lens[idx].sum())
        res[name] = {"entries": int(idx.size), "bytes": nbytes, "ms": round(t * 1e3, 4),
                     "GiB_s": round(nbytes / t / GIB, 1), "entries_per_s": round(idx.size / t, 0)}
    return res


def _route_name(ck, route: int) -> str:
    return {ck.HOST_ROUTE_CPU: "cpu", ck.HOST_ROUTE_GPU: "gpu"}[route]


def _host_reference_verify(frame_ptrs: np.ndarray, frame_lens: np.ndarray, n: int, ledger: int, algo: int,
                           budget_s: float = 3.0) -> tuple[dict, np.ndarray]:
    """cpu_baseline of the host-resident verify line: the reference's own loop over the same host
    frames (BatchedReadOp.java:164-190 -> DigestManager.verifyDigest, two digest updates per frame)
    on every host core — CRC32C through circe crc32c() compiled from /root/reference (oracle/_ref),
    CRC32 through zlib's crc32() (= java.util.zip.CRC32)."""
    import ctypes
    import oracle
    cores, why = host_cores()
    st = np.zeros(n, dtype=np.int32)
    stp = st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    lp = np.ascontiguousarray(frame_lens, dtype=np.uint32)
    if algo == 0 and oracle.ref() is not None:
        kind, label = "reference", "circe crc32c() compiled from /root/reference, two calls per frame"
        fn = oracle.ref().ref_verify_frames_timed
    else:
        kind, label = "port", "zlib crc32() (java.util.zip.CRC32's arithmetic), oracle/cpu_baseline.c"
        fn = oracle.lib().oracle_zlib_verify_frames_timed

    def run(thr, reps):
        return fn(frame_ptrs.ctypes.data, lp.ctypes.data_as(oracle._u32p), n, ledger, 0, thr, reps, stp)
    t1 = run(1, 1)
    reps = max(1, int(budget_s / max(1e-6, t1 / cores)))
    t = run(cores, reps)
    nbytes = int(lp.sum())
    return ({"value": round(nbytes * reps / t / GIB, 3), "unit": "GiB/s", "cores": cores, "kind": kind,
             "single_core_value": round(nbytes / t1 / GIB, 3), "cpu_model": _cpu_model(), "cores_from": why,
             "sample": f"the same {n} host frames ({nbytes / GIB:.3f} GiB), {reps} passes over {cores} threads, "
                       f"DigestManager.verifyDigest per frame; {label}"}, st)


def host_bench(args, ck, torch, rank) -> None:
    """Config 5 fallback (no JVM/BookKeeper here): host-resident 4 KiB entries, one contiguous host
    buffer, through bkd_crc_batch_host: the automatic route (`value`) and each route on its own —
    GPU = pinned double-buffered H2D -> kernel -> D2H, CPU = the library's threaded fold. End to end
    from host memory; never the headline."""
    n = args.entries or (1 << 20)
    entry_len = 4096
    t = torch.empty(n * entry_len, dtype=torch.uint8, pin_memory=not args.pageable)
    dev_tmp = torch.empty(n * entry_len, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix64(dev_tmp, 42)
    t.copy_(dev_tmp)
    del dev_tmp
    host = t.numpy()
    offs = np.arange(n, dtype=np.uint64) * entry_len
    lens = np.full(n, entry_len, dtype=np.uint32)

    def timed():
        for _ in range(max(1, args.warmup)):
            ck.crc_batch_host(0, host, offs, lens)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            got = ck.crc_batch_host(0, host, offs, lens)
        return (time.perf_counter() - t0) / args.steps, got
    auto = _route_name(ck, ck.get_host_batch_route())
    el, out = timed()
    routes = {}
    for route in (ck.HOST_ROUTE_CPU, ck.HOST_ROUTE_GPU):
        with ck.host_batch_route(route):
            tr, got = timed()
        assert (got == out).all(), "routes disagree"
        routes[_route_name(ck, route)] = {"GiB_s": round(n * entry_len / tr / GIB, 2), "ms": round(tr * 1e3, 3)}
    res = {"metric": "GiB/s CRC32C, host-resident 4 KiB entries, end to end from host memory (not the headline)",
           "value": round(n * entry_len / el / GIB, 2), "unit": "GiB/s", "n_gpus": 1,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(el * 1e3, 3),
           "higher_is_better": True, "dtype": "u8", "route": auto, "routes": routes,
           "host_threads": ck.get_host_threads(),
           "config": {"workload": f"{n} x {entry_len} B host-resident entries, "
                                  f"{'pageable' if args.pageable else 'pinned'} source; GPU route: 64 MiB "
                                  f"double-buffered segments incl. PCIe H2D/D2H; CPU route: host threads"},
           "digest_of_digests": int(np.bitwise_xor.reduce(out))}
    if rank == 0 and not args.no_cpu_baseline:
        cb, want = cpu_baseline(host, entry_len, 0, budget_s=3.0)
        res["cpu_baseline"] = cb
        res["parity_check"] = {"entries": n, "match": bool((want == out).all())}
    if rank == 0:
        print(json.dumps(res), flush=True)


def digest_host_bench(args, ck, torch, rank, algo) -> None:
    """Config 5's workload without a JVM: framed 4 KiB entries that live in HOST
    memory as separate buffers (BatchedReadOp's ByteBufList, PendingAddOp's payloads), verified and
    packaged through bkd_digest_verify_batch_host / bkd_digest_package_batch_host: the automatic
    route (`value`) and each route on its own (GPU: gather into pinned staging, H2D, the device
    sequence, D2H of statuses/frames; CPU: the library's threaded DigestManager arithmetic), next to
    the reference's own per-frame verify loop on the same host cores (cpu_baseline)."""
    import ctypes
    from bookkeeper_amd import digest as dg
    from bookkeeper_amd._native import check, lib
    n = args.entries or (1 << 20)
    L = 4096
    dm = dg.DigestManager.instantiate(7, b"", dg.DigestType.CRC32C if algo == ck.CRC32C else dg.DigestType.CRC32)
    mac = dm.macCodeLength
    plen = L - 32 - mac
    dev_tmp = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ck.fill_splitmix64(dev_tmp, 42)
    host = np.ascontiguousarray(dev_tmp.cpu().numpy())  # pageable host memory, like Netty direct buffers
    del dev_tmp
    ids = np.arange(n, dtype=np.int64)
    lacs = ids - 1
    lf = np.full(n, plen, dtype=np.int64)
    base = host.ctypes.data
    pay_ptrs = (base + ids.astype(np.uint64) * L + 32 + mac).astype(np.uint64)
    pay_lens = np.full(n, plen, dtype=np.uint32)
    hdrs = np.zeros((n, 32 + mac), dtype=np.uint8)
    digests = np.zeros(n, dtype=np.uint32)
    vp = ctypes.c_void_p

    def package():
        check(lib().bkd_digest_package_batch_host(algo, dm.ledgerId, vp(ids.ctypes.data), vp(lacs.ctypes.data),
                                                  vp(lf.ctypes.data), vp(pay_ptrs.ctypes.data),
                                                  vp(pay_lens.ctypes.data), n, vp(hdrs.ctypes.data), 32 + mac,
                                                  vp(digests.ctypes.data)))
    package()
    host.reshape(n, L)[:, :32 + mac] = hdrs  # frames = [header][digest][payload], each its own 4 KiB buffer
    first_digests = digests.copy()
    frame_ptrs = (base + ids.astype(np.uint64) * L).astype(np.uint64)
    frame_lens = np.full(n, L, dtype=np.uint32)
    status = np.zeros(n, dtype=np.int32)
    first_bad = ctypes.c_uint64(0)

    def verify():
        check(lib().bkd_digest_verify_batch_host(algo, dm.ledgerId, 0, 0, vp(frame_ptrs.ctypes.data),
                                                 vp(frame_lens.ctypes.data), n, vp(status.ctypes.data),
                                                 ctypes.byref(first_bad)))

    def timed(fn):
        for _ in range(max(1, min(args.warmup, 2))):
            fn()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        return (time.perf_counter() - t0) / args.steps
    steps = args.steps
    auto = _route_name(ck, ck.get_host_batch_route())
    t_verify = timed(verify)
    ok = bool((status == 0).all()) and first_bad.value == n
    t_pack = timed(package)
    ok = ok and bool((digests == first_digests).all())
    routes = {}
    for route in (ck.HOST_ROUTE_CPU, ck.HOST_ROUTE_GPU):
        with ck.host_batch_route(route):
            tv = timed(verify)
            rok = bool((status == 0).all()) and first_bad.value == n
            tp = timed(package)
            rok = rok and bool((digests == first_digests).all())
        ok = ok and rok
        routes[_route_name(ck, route)] = {"verify_GiB_s": round(n * L / tv / GIB, 2), "verify_ms": round(tv * 1e3, 3),
                                          "package_GiB_s_payload": round(n * plen / tp / GIB, 2),
                                          "package_ms": round(tp * 1e3, 3), "all_verified": rok}
    res = {"metric": "GiB/s framed 4 KiB ledger entries in host memory, batched DigestManager verify, end to end "
                     "(config 5's workload, not the headline)",
           "value": round(n * L / t_verify / GIB, 2), "unit": "GiB/s", "n_gpus": 1, "steps": steps,
           "warmup": args.warmup, "ms_per_step": round(t_verify * 1e3, 3), "higher_is_better": True, "dtype": "u8",
           "data": "synthetic (splitmix64, seed 42), pageable host memory, one 4 KiB buffer per entry",
           "config": {"workload": f"{n} framed entries x {L} B ({args.algo}) as separate host buffers "
                                  f"(ByteBufList); GPU route: 64 MiB double-buffered segments incl. PCIe"},
           "route": auto, "routes": routes, "host_threads": ck.get_host_threads(),
           "all_verified": ok, "entries_per_s": round(n / t_verify, 0),
           "package": {"GiB_s_payload": round(n * plen / t_pack / GIB, 2), "ms": round(t_pack * 1e3, 3),
                       "entries_per_s": round(n / t_pack, 0)}}
    if rank == 0 and not args.no_cpu_baseline:
        cb, st = _host_reference_verify(frame_ptrs, frame_lens, n, dm.ledgerId, algo)
        res["cpu_baseline"] = cb
        res["parity_check"] = {"entries": n, "match": bool((st == status).all())}
        res["vs_cpu_baseline"] = round(res["value"] / cb["value"], 3)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if not ok:
        raise SystemExit("VERIFY FAILURE: host-resident entries did not verify")


def digest_bench(args, ck, torch, rank, dev, stream, algo) -> None:
    """SURVEY §8f rows 1-2 (not the headline): framed ledger entries [32 B header][digest][payload]
    of 4 KiB each, device-resident. Times DigestManager's batched verify (BatchedReadOp's loop,
    BatchedReadOp.java:164-190 -> bkd_digest_verify_batch) and batched packaging (PendingAddOp /
    LedgerFragmentReplicator -> bkd_digest_package_batch) over the same n entries."""
    from bookkeeper_amd import digest as dg
    n = args.entries or (1 << 20)
    L = 4096
    dm = dg.DigestManager.instantiate(7, b"", dg.DigestType.CRC32C if algo == ck.CRC32C else dg.DigestType.CRC32)
    mac = dm.macCodeLength
    framed = torch.empty(n * L, dtype=torch.uint8, device=dev)
    ck.fill_splitmix64(framed, 42)
    ids = torch.arange(n, dtype=torch.int64, device=dev)
    lacs = ids - 1
    plen = L - 32 - mac
    pay_off = ids * L + 32 + mac
    pay_len = torch.full((n,), plen, dtype=torch.int32, device=dev)
    len_field = torch.full((n,), plen, dtype=torch.int64, device=dev)
    frames, digests = dm.package_batch(ids, lacs, len_field, framed, pay_off, pay_len, stream=stream)
    framed.view(n, L)[:, :32 + mac].copy_(frames)
    f_off = ids * L
    f_len = torch.full((n,), L, dtype=torch.int32, device=dev)

    def timed(fn):
        for _ in range(max(1, args.warmup)):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(args.steps):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / 1e3 / args.steps

    t_verify = t_pack = float("nan")
    if args.digest_op in ("both", "verify"):
        t_verify = timed(lambda: dm.verify_batch(framed, f_off, f_len, 0, stream=stream))
    status, first_bad = dm.verify_batch(framed, f_off, f_len, 0, stream=stream)
    torch.cuda.synchronize()
    ok = bool((status == 0).all().item()) and int(first_bad.item()) == n
    if args.digest_op in ("both", "package"):
        t_pack = timed(lambda: dm.package_batch(ids, lacs, len_field, framed, pay_off, pay_len, stream=stream))
    # algorithmic bytes: verify reads every framed byte + 12 B of index, writes a 4 B status;
    # package reads the payload + 24 B of ids/LAC/length + 12 B of index, writes header+digest + 4 B
    v_bytes = n * (L + 12 + 4)
    p_bytes = n * (plen + 24 + 12 + 32 + mac + 4)
    res = {"metric": "GiB/s framed 4 KiB ledger entries, batched DigestManager verify (BatchedReadOp), "
                     "device-resident (not the headline)",
           "value": round(n * L / t_verify / GIB, 2), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(t_verify * 1e3, 4), "higher_is_better": True,
           "dtype": "u8", "data": "synthetic (device-generated splitmix64, seed 42, framed by package_batch)",
           "config": {"workload": f"{n} framed entries x {L} B ({args.algo}: 32 B header + {mac} B digest + "
                                  f"{plen} B payload), verify = header CRC -> payload CRC -> compare"},
           "all_verified": ok,
           "roofline": {"bound": "hbm", "achieved": round(v_bytes / t_verify / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(v_bytes / t_verify / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": _pmc_traffic("verify4k" if algo == ck.CRC32C else "verify4k_crc32"),
                        "kernel": "verify pipeline (length gate + fused verify kernel for near-uniform frames; header + plan + finish otherwise)",
                        "algorithmic_bytes_per_launch": v_bytes},
           "package": {"GiB_s_payload": round(n * plen / t_pack / GIB, 2), "ms": round(t_pack * 1e3, 4),
                       "achieved_GB_s": round(p_bytes / t_pack / 1e9, 1),
                       "frac": round(p_bytes / t_pack / 1e9 / HBM_PEAK_GBS, 4),
                       "traffic": _pmc_traffic("package4k" if algo == ck.CRC32C else "package4k_crc32"),
                       "algorithmic_bytes_per_launch": p_bytes}}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if not ok:
        raise SystemExit("VERIFY FAILURE: freshly packaged entries did not verify")


def default_config(gpus: int, world: int) -> str:
    """The workload without --config: BASELINE configs[1] (1M x 4 KiB) on one GPU; on several,
    configs[3] — 64M x 4 KiB split evenly over 8 GPUs = 8M entries (32 GiB) per GPU, weak scaling
    (SURVEY §8d row 4), so the driver's N = 2/4/8 runs measure config 4's per-GPU shard."""
    return "shard8m" if max(gpus, world) > 1 else "uniform4k"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default=None,
                    choices=["uniform4k", "shard8m", "zipf", "zipf_split", "indexed4k", "host4k", "verify4k",
                             "verify4k_host"],
                    help="default: uniform4k (config 2) at N = 1, shard8m (config 4's 8M x 4 KiB per GPU) at N > 1")
    ap.add_argument("--algo", default="crc32c", choices=["crc32c", "crc32"])
    ap.add_argument("--entries", type=int, default=0, help="entries per GPU (default by config)")
    ap.add_argument("--lanes", type=int, default=0, help="force lanes per entry group (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--zipf-align", type=int, default=1, help="diagnostic: align Zipf entries")
    ap.add_argument("--plan-mode", type=int, default=0, help="0 auto, 1 direct, 2 chunked plan")
    ap.add_argument("--no-buckets", action="store_true", help="zipf: skip the per-bucket timings")
    ap.add_argument("--pageable", action="store_true", help="host4k: pageable instead of pinned host buffer")
    ap.add_argument("--digest-op", default="both", choices=["both", "verify", "package"],
                    help="verify4k: time verify, package or both (profiling one route's kernels alone)")
    ap.add_argument("--trace-launches", action="store_true",
                    help="diagnostic: HIP events around every launch, reported as per_launch_ms")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) on a real node; gloo only to rehearse several ranks on one GPU")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(self_launch(args.gpus, sys.argv[1:]))
    if args.config is None:
        args.config = default_config(args.gpus, int(os.environ.get("WORLD_SIZE", "1")))

    import torch
    import torch.distributed as dist
    from bookkeeper_amd import checksum as ck

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (no CPU path exists)")
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} visible GPUs")
    dev = torch.device("cuda", local % ndev)  # % only matters for a gloo rehearsal on fewer GPUs
    torch.cuda.set_device(dev)
    # a process group whenever torch.distributed.run started this process, a world of one included
    # (its RCCL communicator then runs the same barriers and collectives as N > 1); a plain
    # `python bench.py` at N = 1 (the driver's headline command) has none
    grouped = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    if grouped:
        if args.dist_backend == "nccl":
            # RCCL; device_id binds this rank's communicator to its GPU up front (no lazy init on the
            # first collective). Only timing crosses ranks: barriers, one MAX, one all_gather.
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    try:
        run_rank(args, ck, torch, dist, world, rank, dev)
    finally:  # every exit path, a parity failure's SystemExit included
        if grouped and dist.is_initialized():
            dist.destroy_process_group()


def run_rank(args, ck, torch, dist, world: int, rank: int, dev) -> None:
    """One rank's benchmark (world == 1: the whole job)."""
    algo = ck.CRC32C if args.algo == "crc32c" else ck.CRC32
    ck.set_group_lanes(args.lanes)
    ck.set_plan_mode(args.plan_mode)
    # a multi-GPU line must come from N distinct GPUs: under RCCL every rank checks the gathered PCI
    # addresses before any work, so a misconfigured job stops at once, on every rank
    idents = gather_identity(dev, world)
    if world > 1 and args.dist_backend == "nccl":
        pcis = [d["pci"] for d in idents]
        if len(set(pcis)) != len(pcis):
            raise SystemExit(f"ranks share a GPU under nccl: {pcis}")

    stream = torch.cuda.current_stream(dev)
    if args.config == "host4k":
        return host_bench(args, ck, torch, rank)
    if args.config == "verify4k":
        return digest_bench(args, ck, torch, rank, dev, stream, algo)
    if args.config == "verify4k_host":
        return digest_host_bench(args, ck, torch, rank, algo)
    split = None  # zipf_split: how config 3's one batch is divided over the ranks
    if args.config in ("uniform4k", "shard8m"):
        entry_len = 4096
        n = args.entries or (1 << 20 if args.config == "uniform4k" else 8 << 20)
        base = torch.empty(n * entry_len, dtype=torch.uint8, device=dev)
        # the job's data is ONE global splitmix64 stream; rank r holds its slice
        ck.fill_splitmix64(base, 42, first_word=shard_first_word(rank, n, entry_len))
        out = torch.empty(n, dtype=torch.int32, device=dev)
        payload_bytes = n * entry_len
        algo_bytes = n * (entry_len + 4)  # read payload + write u32 digest

        def step():
            ck.crc_batch_uniform(algo, base, entry_len, n, out=out, stream=stream)
        kernel_name = "crc_groups_kernel"
        if args.config == "shard8m":
            workload = {"workload": f"config 4: 64M x 4 KiB over 8 GPUs, 8M per GPU (this run: {world} GPU"
                                    f"{'s' if world > 1 else ''} x {n} entries = {n * world} x 4 KiB, weak scaling), "
                                    f"device-resident, {args.algo}, CRC init 0, data seed 42",
                        "entries_per_gpu": n, "entry_bytes": entry_len}
        else:
            workload = {"workload": f"{n} x {entry_len} B ledger entries per GPU, device-resident, {args.algo}, "
                                    f"CRC init 0, data seed 42",
                        "entries_per_gpu": n, "entry_bytes": entry_len}
    else:
        n = args.entries or (1 << 20)
        if args.config == "indexed4k":  # diagnostic: the uniform layout through the indexed (plan) path
            offs = np.arange(n, dtype=np.int64) * 4096
            lens = np.full(n, 4096, dtype=np.int64)
        else:
            offs, lens = zipf_index(n, align=args.zipf_align)
        if args.config == "zipf_split":
            from bookkeeper_amd.shard import byte_balanced_bounds, shard_span
            # config 3's ONE batch split over the ranks by bytes: rank r holds entries
            # [b[r], b[r+1]) — its span of the global stream, generated in place, and its index rebased
            bounds = byte_balanced_bounds(lens, world)
            lo, hi = int(bounds[rank]), int(bounds[rank + 1])
            if (np.diff(bounds) == 0).any():  # the same test on every rank: all of them stop together
                raise SystemExit(f"zipf_split: a rank would have no entries ({n} entries over {world} ranks)")
            start, end = shard_span(offs, lens, lo, hi, align=128)  # the single-GPU run's line layout
            split = {"entries_total": n, "bytes_total": int(lens.sum()),
                     "entries_per_rank": np.diff(bounds).tolist(),
                     "bytes_per_rank": [int(lens[bounds[r]:bounds[r + 1]].sum()) for r in range(world)]}
            offs, lens, n = offs[lo:hi] - start, lens[lo:hi], hi - lo
            base = torch.empty(end - start, dtype=torch.uint8, device=dev)
            ck.fill_splitmix64(base, 42, first_word=start // 8)
            total = int(lens.sum())
        else:
            total = int(offs[-1] + lens[-1])
            base = torch.empty(total, dtype=torch.uint8, device=dev)
            ck.fill_splitmix64(base, 42, first_word=0)
        d_off = torch.from_numpy(np.ascontiguousarray(offs)).to(dev)
        d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        payload_bytes = total
        algo_bytes = total + 16 * n  # payload + 8 B offset + 4 B length + 4 B digest

        def step():
            ck.crc_batch(algo, base, d_off, d_len, out=out, stream=stream)
        # the HIP events bracket the whole indexed call: plan kernels + crc_plan_chunks_kernel + combine
        kernel_name = "plan pipeline (plan_* + crc_plan_chunks_kernel + plan_combine_kernel)"
        workload = {"workload": f"{n} Zipf(1.1) entries 64 B-64 KiB per GPU (mean {total / n:.0f} B), packed, "
                                f"{args.algo}", "entries_per_gpu": n, "bytes_per_gpu": total}
        if split:
            workload = {"workload": f"config 3: {split['entries_total']} Zipf(1.1) entries 64 B-64 KiB "
                                    f"({split['bytes_total']} B), packed, split by bytes over {world} GPU"
                                    f"{'s' if world > 1 else ''} (contiguous entry ranges, strong scaling), "
                                    f"{args.algo}", **split}
    torch.cuda.synchronize()

    # --trace-launches (diagnostic): a HIP event pair on the launch stream around every launch from the
    # first warm-up launch on, reported as per_launch_ms (launch 0 = the first warm-up launch). Without
    # it the timed launches run back to back with no event packets between them.
    trace = [] if args.trace_launches else None

    def traced(fn):
        if trace is None:
            return fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        trace.append((a, b))

    for _ in range(args.warmup):
        traced(step)
    torch.cuda.synchronize()

    solo_kernel_s = None
    if world > 1:  # each rank alone on the node, in turn: the same-run 1-GPU rate per rank
        for r in range(world):
            dist.barrier()
            if r == rank:
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                solo_steps = max(5, min(args.steps, 20))
                s0.record(stream)
                for _ in range(solo_steps):
                    step()
                s1.record(stream)
                torch.cuda.synchronize()
                solo_kernel_s = s0.elapsed_time(s1) / 1e3 / solo_steps
            dist.barrier()

    # HIP events on the launch stream bracket the K back-to-back launches (no event packets between
    # launches); the average launch duration is their span / K
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    grouped = dist.is_available() and dist.is_initialized()
    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        traced(step)
    ev1.record(stream)
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    avg_kernel_s = ev0.elapsed_time(ev1) / 1e3 / args.steps

    coll_dev = dev if args.dist_backend == "nccl" else None
    elapsed_max = max_over_ranks(elapsed, coll_dev)
    # N > 1: every rank checks a sample of its own shard against the C oracle after the timed region
    # (N = 1 checks the whole batch against the reference in the cpu_baseline leg below)
    shard_check = None
    if world > 1 and not args.no_check:
        shard_check = shard_parity(ck, torch, algo, args.config, base, out, n,
                                   entry_len if args.config in ("uniform4k", "shard8m") else 0,
                                   None if args.config in ("uniform4k", "shard8m") else (offs, lens))
    per_rank = gather_over_ranks([elapsed, avg_kernel_s, solo_kernel_s or avg_kernel_s,
                                  shard_check["entries"] if shard_check else 0,
                                  float(shard_check["match"]) if shard_check else 1.0], coll_dev)

    # weak scaling: every rank processes a batch of its own once per step; zipf_split: the ranks
    # together process the one batch once per step
    total_payload = (split["bytes_total"] if split else payload_bytes * world) * args.steps
    value = total_payload / elapsed_max / GIB
    achieved_gbs = algo_bytes / avg_kernel_s / 1e9
    result = {
        "metric": metric_for(args.config, args.algo),
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if split else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated splitmix64, seed 42)",
        "config": dict(workload, parallelism=f"shard{world} (independent entries, no collective)",
                       lanes=ck.lib().bkd_get_group_lanes(algo, payload_bytes // max(1, n))),
        # payload GB/s over the aggregate HBM peak of the GPUs used (the metric's "% HBM peak")
        "hbm_peak_frac": round(value * GIB / 1e9 / (HBM_PEAK_GBS * world), 4),
        "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": _pmc_traffic(args.config),
                     "kernel": kernel_name, "avg_kernel_ms": round(avg_kernel_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": algo_bytes},
        # per GPU: its own wall rate over the timed region, its kernel time, and (N > 1) its rate when
        # it ran alone on the node in this same run; efficiency = (aggregate / N) / mean solo rate
        "per_gpu": [{"rank": r, "GiB_s": round(payload_bytes * args.steps / e / GIB, 2),
                     "kernel_ms": round(k * 1e3, 4), "solo_GiB_s": round(payload_bytes / so / GIB, 2), **idents[r],
                     **({"parity_check": {"entries": int(pe), "match": bool(pm)}} if shard_check else {})}
                    for r, (e, k, so, pe, pm) in enumerate(per_rank)],
        "per_gpu_GiB_s": round(value / world, 2),
    }
    if trace is not None:
        result["per_launch_ms"] = [round(a.elapsed_time(b), 4) for a, b in trace]
        result["trace_note"] = (f"HIP events around every launch: launches 0..{args.warmup - 1} warm-up, "
                                f"{args.warmup}..{args.warmup + args.steps - 1} the timed region")
    if world > 1:
        solo_mean = float(np.mean([payload_bytes / so / GIB for _, _, so, _, _ in per_rank]))
        result["efficiency_vs_solo"] = round(value / world / solo_mean, 4)
    if shard_check:
        ok = all(bool(pm) for *_, pm in per_rank)
        result["parity_check"] = {"entries": int(sum(pe for *_, pe, _ in per_rank)), "match": ok,
                                  "sample": f"{SHARD_SAMPLE} entries of each rank's shard vs the C oracle"}
        if not ok:
            if rank == 0:
                print(json.dumps(result), flush=True)
            raise SystemExit("PARITY FAILURE: a rank's GPU digests differ from the oracle's")
    if args.config in ("zipf", "zipf_split") and world == 1 and not args.no_buckets:
        result["buckets"] = bucket_rates(ck, torch, algo, base, offs, lens, stream, max(3, args.steps))
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config in ("zipf", "zipf_split"):
        m = n  # the whole packed batch (6.3 GiB for config 3): well past any cache
        span = int(offs[m - 1] + lens[m - 1])
        host = np.ascontiguousarray(base[:span].cpu().numpy())
        result["cpu_baseline"], want = cpu_baseline_indexed(host, offs[:m], lens[:m], algo)
        got = out[:m].cpu().numpy().view(np.uint32)
        result["parity_check"] = {"entries": m, "match": bool((got == want).all())}
        if not result["parity_check"]["match"]:
            print(json.dumps(result), flush=True)
            raise SystemExit("PARITY FAILURE: GPU digests differ from the CPU baseline's")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config in ("uniform4k", "shard8m"):
        # cpu_baseline leg: the reference timed on the host cores over a bounded sample; its
        # digests for that sample double as a parity spot check of the GPU output.
        m = min(n, 1 << 20)  # config 1's full 1M x 4 KiB (4 GiB)
        host = np.ascontiguousarray(base[: m * entry_len].cpu().numpy())
        result["cpu_baseline"], want = cpu_baseline(host, entry_len, algo)
        got = out[:m].cpu().numpy().view(np.uint32)
        result["parity_check"] = {"entries": m, "match": bool((got == want).all())}
        if not result["parity_check"]["match"]:
            print(json.dumps(result), flush=True)
            raise SystemExit("PARITY FAILURE: GPU digests differ from the CPU baseline's")
    if rank == 0:
        print(json.dumps(result), flush=True)


SHARD_SAMPLE = 65536


def shard_parity(ck, torch, algo, config, base, out, n, entry_len, index) -> dict:
    """Checker leg for N > 1: SHARD_SAMPLE entries of this rank's shard (evenly spaced for uniform
    entries, the first ones of a Zipf index) against the C oracle (oracle/, test infrastructure; the
    GPU result under test is `out` as the timed steps left it)."""
    import oracle
    m = min(n, SHARD_SAMPLE)
    got_all = out.cpu().numpy().view(np.uint32)
    if entry_len:
        idx = np.linspace(0, n - 1, m).astype(np.int64)
        rows = base.view(n, entry_len)[torch.from_numpy(idx).to(base.device)].cpu().numpy().reshape(-1)
        want = oracle.uniform(algo, rows, entry_len, entry_len, m)
        got = got_all[idx]
    else:
        offs, lens = index
        span = int(offs[m - 1] + lens[m - 1])
        host = np.ascontiguousarray(base[:span].cpu().numpy())
        want = oracle.batch(algo, host, offs[:m], lens[:m])
        got = got_all[:m]
    return {"entries": m, "match": bool((got == want).all())}


def _lib_sha256() -> str:
    import hashlib
    from bookkeeper_amd.build import LIB
    with open(LIB, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _pmc_traffic(config: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_<config>.json), or
    None — also None when the summary was collected on another build of libbkdigest.so than the one
    being timed (its lib_sha256 stamp, written by tools/pmc_summary.py, must match)."""
    path = os.path.join(HERE, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None
    try:
        pmc = json.load(open(path))
        if pmc.get("lib_sha256") != _lib_sha256():
            return None
        return pmc.get("hbm_bytes_per_launch")
    except Exception:
        return None


if __name__ == "__main__":
    main()
