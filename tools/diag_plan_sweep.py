"""Diagnostic: sweep entry lengths through the chunked plan for one geometry; report mismatches."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import oracle
from bookkeeper_amd import checksum as ck

oracle.build()
gpu = torch.device("cuda", 0)


def run(G, jc, merge, lo, hi):
    ck.set_plan_mode(2)
    ck.set_plan_geometry(G, jc, merge)
    ch = 16 * G * jc
    lens = np.arange(lo, hi, dtype=np.int64)
    offs = np.zeros_like(lens)
    pos = 5
    for i, l in enumerate(lens):
        offs[i] = pos
        pos += int(l) + 37
    size = pos + 64
    data = oracle.fill_splitmix64(size, 7)
    base = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to(gpu)
    mis = base.data_ptr() & 127
    for seeded in (False, True):
        seeds = (np.arange(len(lens), dtype=np.uint32) * 2654435761).astype(np.uint32) if seeded else None
        got = ck.crc_batch(ck.CRC32C, base, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                           seeds=torch.from_numpy(seeds.view(np.int32)).to(gpu) if seeded else None,
                           sync_check=True).cpu().numpy().view(np.uint32)
        want = oracle.batch(0, data, offs, lens, seeds=seeds)
        bad = np.nonzero(got != want)[0]
        print("seeded", seeded, "mis", mis, "bad", len(bad), "of", len(lens))
        for i in bad[:25]:
            l = int(lens[i]); e = mis + int(offs[i]) + l
            pad = (128 - (e & 127)) & 127
            la = l + pad
            m = -(-la // ch); hl = la - (m - 1) * ch
            if hl < merge and m > 1:
                m -= 1; hl += ch
            print("  len", l, "off", int(offs[i]), "pad", pad, "m", m, "hl", hl, "jh", -(-hl // (16 * G)))


args = [int(x) for x in sys.argv[1:]]
for k in range(0, len(args), 5):
    print("geometry", args[k:k + 3], "lengths", args[k + 3:k + 5])
    run(*args[k:k + 5])
