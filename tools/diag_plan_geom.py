"""Diagnostic: which entries of the test_plan_geometries case differ from the oracle."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import oracle
from bookkeeper_amd import checksum as ck

geom = tuple(int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (4, 16, 512)
oracle.build()
gpu = torch.device("cuda", 0)
ck.set_plan_mode(2)
ck.set_plan_geometry(*geom)
rng = np.random.default_rng(sum(geom))
size = 2_000_000
data = oracle.fill_splitmix64(size + 16, 41)
big = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to(gpu)
base = big[3:3 + size]
host = data[3:3 + size]
n = 900
lens = rng.integers(0, 40000, n)
lens[:64] = np.arange(64) * 7
offs = np.array([rng.integers(0, size - l + 1) for l in lens], dtype=np.int64)
seeds = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
got = ck.crc_batch(ck.CRC32C, base, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                   seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu), sync_check=True).cpu().numpy().view(np.uint32)
want = oracle.batch(0, host, offs, lens, seeds=seeds)
bad = np.nonzero(got != want)[0]
mis = (base.data_ptr()) & 127
G, jc, merge = geom
ch = 16 * G * jc
print("mis", mis, "bad", len(bad), "of", n)
for i in bad[:40]:
    l = int(lens[i]); e = mis + int(offs[i]) + l
    pad = (128 - (e & 127)) & 127
    la = l + pad
    m = -(-la // ch); hl = la - (m - 1) * ch
    merged = hl < merge and m > 1
    print(i, "len", l, "pad", pad, "m", m - merged, "hl", hl + (ch if merged else 0), "merged", merged,
          "J0", -(-min(la, ch if m > 1 else la) // (16 * G)))

# CPU emulation of the plan's capacity check: which entries fall back to the serial path
nbins = (ch + merge - 1 + 16 * G - 1) // (16 * G) + 1
cap = n + (size + 128 * n) // ch + 16
plans = []
for i in range(n):
    l = int(lens[i])
    if l < 16:
        plans.append(None); continue
    e = mis + int(offs[i]) + l
    pad = (128 - (e & 127)) & 127
    la = l + pad
    m = -(-la // ch); hl = la - (m - 1) * ch
    if hl < merge and m > 1:
        m -= 1; hl += ch
    jh = -(-hl // (16 * G))
    full = (m - 1) + (1 if jh == jc else 0)
    ps = 0 if (m == 1 and pad == 0) else m
    plans.append((m, jh, full, ps))
tot = [0] * nbins
for p in plans:
    if p:
        if p[1] != jc: tot[p[1]] += 1
        tot[jc] += p[2]
basev = [0] * nbins; acc = 0
for j in range(nbins - 1, -1, -1):
    basev[j] = acc; acc += tot[j]
rs = basev[jc]; sb = 0
ovf = set()
for i, p in enumerate(plans):
    if not p: continue
    if rs + p[2] > cap or sb + p[3] > cap: ovf.add(i)
    rs += p[2]; sb += p[3]
print("cap", cap, "total", acc, "overflowed", len(ovf), "bad&ovf", len(set(bad.tolist()) & ovf),
      "bad-not-ovf", sorted(set(bad.tolist()) - ovf)[:20])
