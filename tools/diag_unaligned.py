import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import oracle
from bookkeeper_amd import checksum as ck
dev = torch.device("cuda", 0)
data = oracle.fill_splitmix64(1 << 16, 5)
base = torch.from_numpy(data).to(dev)
# single entries: offsets 0..31, lengths in a set, seed 0
rows = []
for lanes in (4, 8):
    ck.set_group_lanes(lanes)
    offs, lens = [], []
    for o in range(0, 20):
        for l in (16, 17, 20, 31, 32, 33, 64, 100, 1000):
            offs.append(o); lens.append(l)
    offs = np.array(offs, np.int64); lens = np.array(lens, np.int64)
    got = ck.crc_batch(0, base, torch.from_numpy(offs).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev)).cpu().numpy().view(np.uint32)
    want = oracle.batch(0, data, offs, lens)
    bad = [(int(o), int(l)) for o, l, g, w in zip(offs, lens, got, want) if g != w]
    print("lanes", lanes, "bad", len(bad), "of", len(offs), bad[:40])
# raw unaligned load probe via uniform batch with odd stride
ck.set_group_lanes(4)
for stride in (4096, 4097, 4100, 4104, 4112):
    n = 8
    got = ck.crc_batch_uniform(0, base, 4096, n, stride=stride).cpu().numpy().view(np.uint32)
    want = oracle.uniform(0, data, stride, 4096, n)
    print("stride", stride, (got == want).tolist())
