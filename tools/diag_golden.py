import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
import oracle, golden_util
from bookkeeper_amd import checksum as ck
dev = torch.device("cuda", 0)
fx = golden_util.load()["batch"]
data = oracle.fill_splitmix64(fx["bytes"], fx["seed"])
base = torch.from_numpy(data).to(dev)
offs = np.array(fx["offsets"], np.int64); lens = np.array(fx["lengths"], np.int64)
seeds = np.array([int(s, 16) for s in fx["seeds"]], dtype=np.uint32)
want = np.array([int(x, 16) for x in fx["crc32c"]], dtype=np.uint32)
for lanes in (4, 8):
    ck.set_group_lanes(lanes)
    for use_seeds in (False, True):
        got = ck.crc_batch(0, base, torch.from_numpy(offs).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev),
                           seeds=torch.from_numpy(seeds.view(np.int32)).to(dev) if use_seeds else None).cpu().numpy().view(np.uint32)
        w = want if use_seeds else oracle.batch(0, data, offs, lens)
        bad = np.nonzero(got != w)[0]
        print("lanes", lanes, "seeds", use_seeds, "bad", bad.size, [(int(i), int(offs[i]) % 16, int(lens[i]), hex(seeds[i])) for i in bad[:12]])
