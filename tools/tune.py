"""A/B kernel variants in ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).
Usage: python tools/tune.py build   (here: compiles variants into tools/variants/)
       python tools/tune.py run     (GPU box: times every variant on the same input)"""
import ctypes, itertools, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "tools", "variants")
VARIANTS = {f"pf{pf}_nt{nt}": [f"-DBKD_PF={pf}", f"-DBKD_NT={nt}"] for pf, nt in itertools.product((2, 4, 6, 8), (0, 1))}


def build():
    from bookkeeper_amd.build import build_native
    os.makedirs(VDIR, exist_ok=True)
    for name, flags in VARIANTS.items():
        build_native(force=True, extra_flags=flags + ["-w"], out=os.path.join(VDIR, f"lib_{name}.so"))
        print("built", name)


def run():
    import numpy as np, torch
    from bookkeeper_amd import _native
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    libs = {}
    for name in VARIANTS:
        L = ctypes.CDLL(os.path.join(VDIR, f"lib_{name}.so"))
        for fn, (res, args) in _native.PROTOTYPES.items():
            getattr(L, fn).restype = res; getattr(L, fn).argtypes = args
        libs[name] = L
    cfgs = [("uniform4k", 1 << 20, 4096)]
    for cfg, n, L_ in cfgs:
        base = torch.empty(n * L_, dtype=torch.uint8, device=dev)
        libs["pf4_nt0"].bkd_fill_splitmix64(ctypes.c_void_p(base.data_ptr()), base.numel(), 42, 0, None)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        ref = None
        res = {}
        for lanes in (8, 16):
            for r in range(5):
                for name, L in libs.items():
                    L.bkd_set_group_lanes(lanes)
                    st = torch.cuda.current_stream()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    for _ in range(2):
                        L.bkd_crc_batch_uniform(0, ctypes.c_void_p(base.data_ptr()), L_, L_, n, None, 0, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st.cuda_stream))
                    e0.record(st)
                    for _ in range(10):
                        L.bkd_crc_batch_uniform(0, ctypes.c_void_p(base.data_ptr()), L_, L_, n, None, 0, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(st.cuda_stream))
                    e1.record(st); torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / 10
                    if ref is None: ref = out.clone()
                    assert torch.equal(out, ref), name
                    res.setdefault((lanes, name), []).append(ms)
        for (lanes, name), v in sorted(res.items(), key=lambda kv: np.median(kv[1])):
            print(f"{cfg} lanes={lanes:2d} {name:8s} median {np.median(v):.4f} ms min {min(v):.4f}  -> {n*(L_+4)/min(v)/1e6:.0f} GB/s")


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
