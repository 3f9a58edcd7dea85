#!/usr/bin/env python3
"""One long entry through every device route (auto / plan / direct indexed batch, uniform batch,
per-call device resume) against the host CPU fold, at sizes around 64-512 MiB."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch
    from bookkeeper_amd import checksum as ck
    dev = torch.device("cuda", 0)
    M = 1 << 20
    buf = torch.empty(512 * M + 4096, dtype=torch.uint8, device=dev)
    ck.fill_splitmix64(buf, 9)
    host = buf.cpu().numpy()
    for size in [16 * M, 64 * M, 64 * M + 5, 128 * M + 3, 256 * M, 256 * M + 77, 512 * M]:
        off = 3
        want = ck.cpu_resume(ck.CRC32C, 0x1234, host[off:off + size]) & 0xFFFFFFFF
        res = {}
        for mode in (0, 2, 1):
            ck.set_plan_mode(mode)
            o = ck.crc_batch(ck.CRC32C, buf, torch.tensor([off], dtype=torch.int64, device=dev),
                             torch.tensor([size], dtype=torch.int32, device=dev), seed_all=0x1234, sync_check=True)
            res[f"mode{mode}"] = int(o.cpu().numpy().view(np.uint32)[0])
        ck.set_plan_mode(0)
        print(size, hex(want), {k: (hex(v), v == want) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
