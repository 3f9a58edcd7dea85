"""Pure-Python model of the GPU kernel's decomposition (crc_kernels.hpp), driven by the
library's own operator tables (bkd_host_tables). Used on CPU to prove that the
end-aligned window / 4-stream Horner / lane tree / seed-fold scheme reproduces the
oracle bit-exactly before any GPU run. Small inputs only (pure-Python loops)."""
from __future__ import annotations

import numpy as np


class KernelModel:
    def __init__(self, tables: np.ndarray, lanes: int):
        self.G = lanes
        self.levels = int(np.log2(lanes))
        t = tables.astype(np.uint64)
        self.main = t[0:1024]
        self.x32 = t[1024:2048]
        self.lv = [t[2048 + 1024 * s: 3072 + 1024 * s] for s in range(self.levels)]
        self.byte = t[(2 + self.levels) * 1024:]

    @staticmethod
    def _mul(tab, v: int) -> int:
        return int(tab[v & 0xFF] ^ tab[256 + ((v >> 8) & 0xFF)] ^ tab[512 + ((v >> 16) & 0xFF)]
                   ^ tab[768 + (v >> 24)])

    def crc(self, data: bytes, seed: int) -> int:
        n = len(data)
        if n < 16:
            r = (~seed) & 0xFFFFFFFF
            for b in data:
                r = int(self.byte[(r ^ b) & 0xFF]) ^ (r >> 8)
            return (~r) & 0xFFFFFFFF
        G, step = self.G, 16 * self.G
        J = (n + step - 1) // step
        buf = bytes(data)
        s, e = 0, n                      # entry byte range (relative)
        wstart = e - J * step
        r0 = (~seed) & 0xFFFFFFFF

        def place(d):                     # place_seed() in crc_kernels.hpp
            if 0 <= d <= 3:
                return (r0 << (8 * d)) & 0xFFFFFFFF
            if -3 <= d < 0:
                return r0 >> (8 * -d)
            return 0

        def load16(addr):                 # addr >= s and addr + 16 <= e, like the kernel
            return [int.from_bytes(buf[addr + 4 * k: addr + 4 * k + 4], "little") for k in range(4)]

        words = np.zeros((J, G, 4), dtype=np.uint64)
        for g in range(G):
            a = wstart + 16 * g
            if a >= s:
                w = load16(a)
            elif a + 16 > s:              # straddling lane: load at s, shift left by s - a bytes
                v = int.from_bytes(buf[s:s + 16], "little") << (8 * (s - a))
                w = [(v >> (32 * k)) & 0xFFFFFFFF for k in range(4)]
            else:
                w = [0, 0, 0, 0]
            if a < s + 4 and a + 16 > s:
                w = [w[k] ^ place(s - a - 4 * k) for k in range(4)]
            words[0, g] = w
            for j in range(1, J):
                words[j, g] = load16(a + j * step)
        fx = place(s - (wstart + step)) if wstart + step < s + 4 else 0
        if J > 1:
            words[1, 0, 0] ^= fx
        lane_vals = []
        for g in range(G):
            acc = [int(words[0, g, k]) for k in range(4)]
            for j in range(1, J):
                acc = [self._mul(self.main, acc[k]) ^ int(words[j, g, k]) for k in range(4)]
            v = self._mul(self.x32, acc[0]) ^ acc[1]
            v = self._mul(self.x32, v) ^ acc[2]
            v = self._mul(self.x32, v) ^ acc[3]
            lane_vals.append(v)
        for s in range(self.levels):
            span = 1 << s
            lane_vals = [self._mul(self.lv[s], lane_vals[2 * m]) ^ lane_vals[2 * m + 1]
                         for m in range(len(lane_vals) // 2)]
            assert len(lane_vals) == G >> (s + 1) and span
        total = self._mul(self.x32, lane_vals[0])
        return (~total) & 0xFFFFFFFF
