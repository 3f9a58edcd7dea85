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
        self.byte = t[(2 + self.levels) * 1024:(2 + self.levels) * 1024 + 256]
        self.x64 = t[(2 + self.levels) * 1024 + 256:(2 + self.levels) * 1024 + 1280]
        self.x96 = t[(2 + self.levels) * 1024 + 1280:(2 + self.levels) * 1024 + 2304]
        lo = (2 + self.levels) * 1024 + 2304  # lane-position nibble tables (groups of 4 / 8 lanes)
        self.lanetab = t[lo:lo + 128 * lanes] if lanes in (4, 8) else None

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
        fast = G <= 16  # finish_lanes(): x^32 folded into the in-lane products, no final multiply
        lane_vals = []
        for g in range(G):
            acc = [int(words[0, g, k]) for k in range(4)]
            for j in range(1, J):
                acc = [self._mul(self.main, acc[k]) ^ int(words[j, g, k]) for k in range(4)]
            if fast:
                v = (self._mul(self.lv[0], acc[0]) ^ self._mul(self.x96, acc[1]) ^ self._mul(self.x64, acc[2])
                     ^ self._mul(self.x32, acc[3]))
            else:
                v = self._mul(self.x32, acc[0]) ^ acc[1]
                v = self._mul(self.x32, v) ^ acc[2]
                v = self._mul(self.x32, v) ^ acc[3]
            lane_vals.append(v)
        if self.lanetab is not None:  # finish_lanes' lane-position products + XOR over the group
            total = 0
            for g, v in enumerate(lane_vals):
                for k in range(8):
                    total ^= int(self.lanetab[(16 * k + ((v >> (4 * k)) & 15)) * G + g])
            return (~total) & 0xFFFFFFFF
        for s in range(self.levels):
            lane_vals = [self._mul(self.lv[s], lane_vals[2 * m]) ^ lane_vals[2 * m + 1]
                         for m in range(len(lane_vals) // 2)]
        total = lane_vals[0] if fast else self._mul(self.x32, lane_vals[0])
        return (~total) & 0xFFFFFFFF


def plan_model(tables_by_lanes, algo_xpow8n, gf_mul, data: bytes, seed: int, lanes: int = 8, jc: int = 32,
               mis: int = 0) -> int:  # mis: entry start address modulo 128
    """Models the ragged-batch plan (plan_kernels.hpp) for one entry starting at a device address
    congruent to `mis` (mod 128): the entry is padded with zeros to ae = the next 128-byte-aligned
    address (the kernel folds the foreign bytes there and XORs them out again, which equals folding
    zeros), [0, ae) is cut into chunks of CH = 16*lanes*jc bytes ending at aligned addresses (head
    chunk carries the seed; a head < 16 B merges into its neighbour), each chunk folded by the kernel
    decomposition, partial registers combined by Horner with X = x^(8*CH), then multiplied by
    x^(-8*pad). Entries shorter than 16 bytes are folded serially."""
    ch, step = 16 * lanes * jc, 16 * lanes
    km = KernelModel(tables_by_lanes, lanes)
    n = len(data)
    byte = km.byte
    poly = int(byte[0x80])  # T[0x80] = P for a reflected CRC

    if n < 16:
        reg = (~seed) & 0xFFFFFFFF
        for b in data:
            reg = int(byte[(reg ^ b) & 0xFF]) ^ (reg >> 8)
        return (~reg) & 0xFFFFFFFF
    al = min(step, 128)  # the pad must fit the final chunk's last step
    pad = (al - ((mis + n) & (al - 1))) & (al - 1)
    padded = bytes(data) + bytes(pad)
    ae = n + pad
    m = (ae + ch - 1) // ch
    hl = ae - (m - 1) * ch
    if hl < 16 and m > 1:
        m -= 1
    parts = []
    for c in range(m):
        e = ae - c * ch
        cs = 0 if c == m - 1 else e - ch
        r0 = (~seed) & 0xFFFFFFFF if c == m - 1 else 0
        # raw register of padded[cs:e] with r0 folded in == ~KernelModel.crc(chunk, ~r0)
        parts.append((~km.crc(padded[cs:e], (~r0) & 0xFFFFFFFF)) & 0xFFFFFFFF)
        assert (e - cs) <= ch + 15 and (e - cs + step - 1) // step <= jc + 1
    X = algo_xpow8n(ch)
    reg = parts[m - 1]
    for c in range(m - 2, -1, -1):
        reg = gf_mul(reg, X) ^ parts[c]
    inv = 0x80000000  # x^(-8*pad): divide by x, 8*pad times
    for _ in range(8 * pad):
        inv = (((inv ^ poly) << 1) | 1) & 0xFFFFFFFF if inv & 0x80000000 else (inv << 1) & 0xFFFFFFFF
    return (~gf_mul(reg, inv)) & 0xFFFFFFFF
