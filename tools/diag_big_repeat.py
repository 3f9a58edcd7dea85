#!/usr/bin/env python3
"""One long entry through the device indexed batch, repeated on one stream (r03l: the host GPU
route's single-entry path gave wrong digests from its second call on, entries > 64 MiB)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch
    from bookkeeper_amd import checksum as ck
    dev = torch.device("cuda", 0)
    M = 1 << 20
    for size in [64 * M, 64 * M + 4096, 128 * M, 256 * M]:
        buf = torch.empty(size, dtype=torch.uint8, device=dev)
        ck.fill_splitmix64(buf, 9)
        want = ck.cpu_resume(ck.CRC32C, 0, buf.cpu().numpy()) & 0xFFFFFFFF
        for mode in (0, 2, 1):
            ck.set_plan_mode(mode)
            got = []
            for k in range(5):
                o = ck.crc_batch(ck.CRC32C, buf, torch.tensor([0], dtype=torch.int64, device=dev),
                                 torch.tensor([size], dtype=torch.int32, device=dev), sync_check=True)
                got.append(int(o.cpu().numpy().view(np.uint32)[0]) == want)
            print(size, "mode", mode, got, flush=True)
        ck.set_plan_mode(0)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
