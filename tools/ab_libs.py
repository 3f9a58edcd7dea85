"""A/B several builds of libbkdigest.so in ONE process on the same device buffers, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24: cross-box and first-run noise is larger than the
effects being measured).

Usage (GPU box): python3 tools/ab_libs.py [lib.so ...]
Default libraries: bookkeeper_amd/libbkdigest.so and every tools/variants/lib_*.so.
Workloads: zipf (config 3), zipf crc32, zipf < 1 KiB bucket, zipf's full chunks / heads alone, packed 64 B, indexed 4 KiB, uniform 4 KiB.
Each library's digests must equal the first library's, bit for bit.
Environment: AB_WORK (workload names), AB_ROUNDS, AB_MODE (plan mode), AB_SMALL / AB_SHORT_MEAN
(short-entry class bound and gate), AB_LANES (direct-kernel lanes), AB_PF (chunk-kernel loads in
flight), AB_GEOM (plan geometry lanes,steps,merge), AB_NOCHECK (skip the digest comparison).
"""
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ROUNDS = int(os.environ.get("AB_ROUNDS", "5"))
REPS = 10


def main(paths):
    import numpy as np
    import torch
    from bench import zipf_index
    from bookkeeper_amd import _native

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream()
    libs = {}
    for p in paths:
        L = ctypes.CDLL(os.path.abspath(p))
        for fn, (res, args) in _native.PROTOTYPES.items():
            if hasattr(L, fn):
                getattr(L, fn).restype = res
                getattr(L, fn).argtypes = args
        if os.environ.get("AB_SMALL") and hasattr(L, "bkd_set_plan_small"):
            L.bkd_set_plan_small(int(os.environ["AB_SMALL"]))
        if os.environ.get("AB_SHORT_MEAN") and hasattr(L, "bkd_set_short_class_mean"):
            L.bkd_set_short_class_mean(int(os.environ["AB_SHORT_MEAN"]))
        if os.environ.get("AB_MODE") and hasattr(L, "bkd_set_plan_mode"):  # 0 auto, 1 direct, 2 plan
            L.bkd_set_plan_mode(int(os.environ["AB_MODE"]))
        if os.environ.get("AB_LANES"):  # lanes per group of the one-entry-per-group kernels
            assert L.bkd_set_group_lanes(int(os.environ["AB_LANES"])) == 0
        if os.environ.get("AB_PF"):  # loads in flight per lane in the chunk kernel (bkd_set_plan_prefetch)
            assert L.bkd_set_plan_prefetch(int(os.environ["AB_PF"])) == 0
        if os.environ.get("AB_GEOM"):  # lanes,steps,merge for the plan (bkd_set_plan_geometry)
            assert L.bkd_set_plan_geometry(*(int(v) for v in os.environ["AB_GEOM"].split(","))) == 0
        libs[os.path.basename(p)] = L
    n = 1 << 20
    offs, lens = zipf_index(n)
    total = int(offs[-1] + lens[-1])
    base = torch.empty(max(total, n * 4096), dtype=torch.uint8, device=dev)
    first = next(iter(libs.values()))
    first.bkd_fill_splitmix64(ctypes.c_void_p(base.data_ptr()), base.numel(), 42, 0, None)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())

    def idx(o, l):
        return (torch.from_numpy(np.ascontiguousarray(o, dtype=np.int64)).to(dev),
                torch.from_numpy(np.ascontiguousarray(l).astype(np.int32)).to(dev))

    lt = lens < 1024
    head_l = np.where(lens % 4096 == 0, 4096, lens % 4096)  # what the plan leaves as heads, packed alone
    head_o = np.concatenate([[0], np.cumsum(head_l[:-1])])
    hs_l = np.sort(head_l)[::-1]  # the same heads packed in the plan's processing order (longest first)
    hs_o = np.concatenate([[0], np.cumsum(hs_l[:-1])])
    ha_l = (hs_l + 127) // 128 * 128  # the sorted heads rounded up to whole 128-byte lines: no pad, no straddle
    ha_o = np.concatenate([[0], np.cumsum(ha_l[:-1])])
    # the sorted heads, each in its own 128-byte lines (no line shared with a neighbour): starting on
    # a line (heads_sep_al) or at its original offset within the line (heads_sep)
    slot = (hs_l + 127 + 127) // 128 * 128
    sep_base = np.concatenate([[0], np.cumsum(slot[:-1])])
    hsep_al_o, hsep_o = sep_base, sep_base + (hs_o % 128)
    m1_l = np.where(np.arange(n) % 256 == 0, 2048, 1024)  # 1 KiB chunks through the plan (outside the gate's band)
    m1_o = np.concatenate([[0], np.cumsum(m1_l[:-1])])
    order = np.argsort(-lens, kind="stable")  # the same entries, index sorted by descending length
    # config 3 split as the plan splits it (CH = 4 KiB, chunks ending on ae = the entry's end rounded
    # up to 128 B, a head shorter than 16 B merged): the full chunks alone as aligned 4 KiB entries at
    # their own addresses, in the plan's list order (entry order, chunk 0 = the entry's last) or by
    # address; and the heads alone at their own addresses (an entry's head ends on its first full chunk)
    z_ae = (offs + lens + 127) // 128 * 128
    z_m = (z_ae - offs + 4095) // 4096
    z_hl = z_ae - offs - (z_m - 1) * 4096
    z_mg = (z_hl < 16) & (z_m > 1)
    z_m = np.where(z_mg, z_m - 1, z_m)
    z_hl = np.where(z_mg, z_hl + 4096, z_hl)
    z_fullh = (z_hl + 127) // 128 == 32  # a head of exactly 32 steps sits in the full bin
    z_full = (z_m - 1) + z_fullh
    z_own = np.repeat(np.arange(n), z_full)
    z_c = np.arange(z_own.size) - np.repeat(np.cumsum(z_full) - z_full, z_full)
    zf_o = z_ae[z_own] - (z_c + 1) * 4096
    zf_l = np.full(zf_o.size, 4096)
    zf_l[5] = 2048  # out of the near-uniform gate's band, as plan4k
    zh_sel = ~z_fullh
    zh_o = offs[zh_sel]
    zh_l = np.where(z_m == 1, lens, z_hl)[zh_sel]
    work = {
        "zipf": (0, *idx(offs, lens), total),
        "zipf_sorted": (0, *idx(offs[order], lens[order]), total),
        "zipf_crc32": (1, *idx(offs, lens), total),
        "zipf_lt1k": (0, *idx(offs[lt], lens[lt]), int(lens[lt].sum())),
        "zipf_full": (0, *idx(zf_o, zf_l), int(zf_l.sum())),
        "zipf_full_asc": (0, *idx(np.sort(zf_o), zf_l), int(zf_l.sum())),
        "zipf_heads_at": (0, *idx(zh_o, zh_l), int(zh_l.sum())),
        "zipf_heads": (0, *idx(head_o, head_l), int(head_l.sum())),
        "zipf_heads_sorted": (0, *idx(hs_o, hs_l), int(hs_l.sum())),
        "mixed1k": (0, *idx(m1_o, m1_l), int(m1_l.sum())),
        # 1 M chunks of 1 / 2 / 4 steps through the plan (one 4 KiB entry keeps them out of the gate's band)
        **{f"chunk{k}s": (0, *idx(np.arange(n) * 1024 + 7, np.where(np.arange(n) == 5, 4096, 128 * k - 28)),
                          n * (128 * k - 28)) for k in (1, 2, 4)},
        "heads_aligned": (0, *idx(ha_o, ha_l), int(ha_l.sum())),
        "heads_sep_al": (0, *idx(hsep_al_o, hs_l), int(hs_l.sum())),
        "heads_sep": (0, *idx(hsep_o, hs_l), int(hs_l.sum())),
        "uniform1k_idx": (0, *idx(np.arange(n) * 1024, np.full(n, 1024)), n * 1024),
        "packed64": (0, *idx(np.arange(n) * 64, np.full(n, 64)), n * 64),
        "packed64_64m": (0, *idx(np.arange(64 * n) * 64, np.full(64 * n, 64)), 64 * n * 64),
        "indexed4k": (0, *idx(np.arange(n) * 4096, np.full(n, 4096)), n * 4096),
        # 1M aligned 4 KiB entries through the chunk kernel (one 2 KiB entry keeps them out of the
        # near-uniform gate's band): the chunk loop against the uniform kernel on the same bytes
        "plan4k": (0, *idx(np.arange(n) * 4096, np.where(np.arange(n) == 5, 2048, 4096)), n * 4096 - 2048),
        # 512 K aligned 8 KiB entries through the chunk kernel: two full chunks each, partials only (no
        # chunk is final), against u8192_l8 (the uniform kernel on the same 4 GiB)
        "plan8k": (0, *idx(np.arange(n // 2) * 8192, np.where(np.arange(n // 2) == 5, 4096, 8192)), (n // 2) * 8192 - 4096),
        # 16 entries of 256 MiB: the stream route's inner loop with almost no entry boundary
        "big16": (0, *idx(np.arange(16) * (n * 256), np.full(16, n * 256)), 16 * n * 256),
        # 4096 entries of 1 MiB plus 7 bytes (unaligned ends), packed
        "big1m": (0, *idx(np.arange(4096) * ((1 << 20) + 7), np.full(4096, (1 << 20) + 7)), 4096 * ((1 << 20) + 7)),
    }

    small = {f"u{S}_l{G}": (S, G) for S, G in ((32, 1), (32, 4), (64, 1), (64, 4), (64, 8), (128, 1), (128, 4),
                                               (128, 8), (256, 1), (256, 4), (256, 8), (512, 1), (512, 4), (512, 8),
                                               (1024, 8), (2048, 8), (8192, 8), (16384, 16))}

    # one digest per entry of the largest batch (4 GiB of the smallest uniform size)
    out = torch.empty(max(n, max((4 << 30) // S for S, _ in small.values())), dtype=torch.int32, device=dev)
    assert base.numel() >= 4 << 30

    fr = {}
    big = {}  # uniform4k_8m's 32 GiB shard

    def framed():  # 1M framed 4 KiB entries (CRC32C: 32 B header + 4 B digest + payload), packaged once
        if not fr:
            F = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
            first.bkd_fill_splitmix64(ptr(F), F.numel(), 7, 0, None)
            ids = torch.arange(n, dtype=torch.int64, device=dev)
            fr.update(F=F, ids=ids, lacs=ids - 1, lenf=torch.full((n,), 4096 - 36, dtype=torch.int64, device=dev),
                      poff=ids * 4096 + 36, plen=torch.full((n,), 4096 - 36, dtype=torch.int32, device=dev),
                      foff=ids * 4096, flen=torch.full((n,), 4096, dtype=torch.int32, device=dev),
                      dig=torch.empty(n, dtype=torch.int32, device=dev),
                      status=torch.empty(n, dtype=torch.int32, device=dev),
                      fb=torch.empty(1, dtype=torch.int64, device=dev))
            package(first)
            torch.cuda.synchronize()
        return fr

    def package(L):
        f = fr
        return L.bkd_digest_package_batch(0, 7, ptr(f["ids"]), ptr(f["lacs"]), ptr(f["lenf"]), ptr(f["F"]),
                                          f["F"].numel(), ptr(f["poff"]), ptr(f["plen"]), n, ptr(f["F"]), 4096,
                                          ptr(f["dig"]), ctypes.c_void_p(st.cuda_stream))

    def call(L, name):
        if name == "package4k":
            framed()
            return package(L)
        if name == "package4k_sep":  # frames into their own packed buffer (stride 32 + mac), as bench.py
            framed()
            f = fr
            if "sep" not in f:
                f["sep"] = torch.empty(n * 36, dtype=torch.uint8, device=dev)
            return L.bkd_digest_package_batch(0, 7, ptr(f["ids"]), ptr(f["lacs"]), ptr(f["lenf"]), ptr(f["F"]),
                                              f["F"].numel(), ptr(f["poff"]), ptr(f["plen"]), n, ptr(f["sep"]), 36,
                                              ptr(f["dig"]), ctypes.c_void_p(st.cuda_stream))
        if name == "verify4k":
            f = framed()
            r = L.bkd_digest_verify_batch(0, 7, 0, 0, ptr(f["F"]), f["F"].numel(), ptr(f["foff"]), ptr(f["flen"]), n,
                                          ptr(f["status"]), ptr(f["fb"]), ctypes.c_void_p(st.cuda_stream))
            return r
        if name == "uniform4k_8m":  # config 4's per-GPU shard: 8M x 4 KiB (32 GiB, contents as allocated)
            if "big8m" not in big:
                big["big8m"] = torch.empty(8 * n * 4096, dtype=torch.uint8, device=dev)
                big["out8m"] = torch.empty(8 * n, dtype=torch.int32, device=dev)
            L.bkd_set_group_lanes(0)
            r = L.bkd_crc_batch_uniform(0, ptr(big["big8m"]), 4096, 4096, 8 * n, None, 0, ptr(big["out8m"]),
                                        ctypes.c_void_p(st.cuda_stream))
            return r
        if name == "uniform4k":
            L.bkd_set_group_lanes(0)
            return L.bkd_crc_batch_uniform(0, ptr(base), 4096, 4096, n, None, 0, ptr(out), ctypes.c_void_p(st.cuda_stream))
        if name in small:
            S, G = small[name]
            L.bkd_set_group_lanes(G)
            r = L.bkd_crc_batch_uniform(0, ptr(base), S, S, (4 << 30) // S, None, 0, ptr(out),
                                        ctypes.c_void_p(st.cuda_stream))
            L.bkd_set_group_lanes(0)
            return r
        algo, o, l, _ = work[name]
        return L.bkd_crc_batch(algo, ptr(base), base.numel(), ptr(o), ptr(l), o.numel(), None, 0, ptr(out),
                               ctypes.c_void_p(st.cuda_stream))

    names = [w for w in os.environ.get("AB_WORK", " ".join(list(work) + ["uniform4k"] + list(small))).split()]
    res = {}
    for name in names:
        ref = None
        for L in libs.values():  # warm-up + parity
            L.bkd_set_plan_mode(int(os.environ.get("AB_MODE", "0")))
            assert call(L, name) == 0, name
            torch.cuda.synchronize()
            cnt = work[name][1].numel() if name in work else ((4 << 30) // small[name][0] if name in small else n)
            if name in ("package4k", "package4k_sep", "verify4k"):
                out[:n].copy_(fr["status"] if name == "verify4k" else fr["dig"])
            if name == "uniform4k_8m":  # the shard's last 1M digests (its last flushes)
                out[:n].copy_(big["out8m"][-n:])
            if ref is None:
                ref = out[:cnt].clone()
            if not os.environ.get("AB_NOCHECK"):  # (measurement-only variants compute wrong digests)
                if not torch.equal(out[:cnt], ref):
                    bad = torch.nonzero(out[:cnt] != ref).flatten()
                    raise AssertionError(f"{name}: {L._name} differs from the first library on {bad.numel()} "
                                         f"entries, first {bad[:5].tolist()}")
        for _ in range(ROUNDS):
            for lname, L in libs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(REPS):
                    call(L, name)
                e1.record(st)
                torch.cuda.synchronize()
                res.setdefault((name, lname), []).append(e0.elapsed_time(e1) / REPS)
        nbytes = work[name][3] if name in work else (4 << 30 if name in small else
                                                     8 * n * 4096 if name == "uniform4k_8m" else n * 4096)
        for lname in libs:
            v = sorted(res[(name, lname)])
            print(f"{name:12s} {lname:22s} median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f} ms  "
                  f"{nbytes / v[len(v) // 2] / 1e6:7.0f} GB/s payload", flush=True)


if __name__ == "__main__":
    args = sys.argv[1:] or [os.path.join(ROOT, "bookkeeper_amd", "libbkdigest.so")] + sorted(
        glob.glob(os.path.join(ROOT, "tools", "variants", "lib_*.so")))
    main(args)
