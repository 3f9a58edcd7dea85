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
        W = J * step
        pad = W - n
        # virtual window: zeros in front of the entry, then the entry
        win = bytearray(pad) + bytearray(data)
        r0 = (~seed) & 0xFFFFFFFF
        for k in range(4):  # fold the init register into the entry's first 4 bytes
            win[pad + k] ^= (r0 >> (8 * k)) & 0xFF
        words = np.frombuffer(bytes(win), dtype="<u4").reshape(J, G, 4)
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
