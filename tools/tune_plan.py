"""A/B the ragged-batch plan geometry on the Zipf (config 3) workload, interleaved in one process."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from bench import zipf_index
from bookkeeper_amd import checksum as ck

GEOMS = [tuple(int(x) for x in g.split(",")) for g in os.environ["GEOMS"].split()] if "GEOMS" in os.environ else \
    [(8, 32, 16), (16, 16, 16), (16, 8, 16), (16, 32, 16), (16, 64, 16), (16, 16, 2048), (32, 8, 16), (32, 16, 16),
     (32, 4, 16), (64, 4, 16), (64, 8, 16), (64, 2, 16), (32, 8, 2048)]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
n = 1 << 20
offs, lens = zipf_index(n)
total = int(offs[-1] + lens[-1])
base = torch.empty(total, dtype=torch.uint8, device=dev)
ck.fill_splitmix64(base, 42)
d_off = torch.from_numpy(offs).to(dev)
d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream()
ref = None
res = {}
for rnd in range(4):
    for gm in GEOMS + ["direct"]:
        if gm == "direct":
            ck.set_plan_mode(1)
        else:
            ck.set_plan_mode(2)
            ck.set_plan_geometry(*gm[:3])
            ck.set_plan_prefetch(gm[3] if len(gm) > 3 else 2)
        for _ in range(2):
            ck.crc_batch(0, base, d_off, d_len, out=out, stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(5):
            ck.crc_batch(0, base, d_off, d_len, out=out, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        assert torch.equal(ref, out), gm
        res.setdefault(gm, []).append(e0.elapsed_time(e1) / 5)
for gm, v in sorted(res.items(), key=lambda kv: np.median(kv[1])):
    print(f"{str(gm):18s} median {np.median(v):.4f} ms  min {min(v):.4f}  -> {total / min(v) / 1e6:.0f} GB/s payload")
