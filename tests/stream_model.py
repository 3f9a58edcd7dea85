"""Pure-Python model of the stream route for ragged indexed batches (stream_kernels.hpp), used on
CPU to check the index arithmetic against the oracle before any GPU run.

The entries' 128-byte device lines are laid end to end in index order (a line shared by an entry's
end and the next entry's start counted once); group r folds the positions [r TL, (r + 1) TL),
TL = ceil(end / groups) rounded up to 8, with a cursor four positions ahead of the fold that walks
the entries' records to find each position's device line; an entry inside one range gets its digest
there, the pieces of longer entries are joined with x^(1024 TL) per range and x^(1024 L) for the
last L lines, then x^(-8 pad).

Geometry of entry i (a = device address modulo 128 + offset, `mis` = base address mod 128):
  as = mis + o, ae = as + l, first line F = as // 128, last line Lst = (ae - 1) // 128,
  d = as - 128 F (bytes before the entry in its first line), pad = 128 (Lst + 1) - ae.
In the stream: valid, l >= 1 and l + pad >= 4 (the seed image must lie inside the padded message);
others (empty, out of range) are done by the combine.
"""
from __future__ import annotations

import numpy as np



class Geo:
    def __init__(self, mis: int, o: int, l: int, size: int):
        self.valid = not (o > size or l > size - o)
        self.o, self.l = o, l
        a_s = mis + o
        a_e = a_s + l
        self.F = a_s // 128
        self.Lst = (a_e - 1) // 128 if l else self.F
        self.J = self.Lst - self.F + 1
        self.d = a_s - 128 * self.F
        self.pad = 128 * (self.Lst + 1) - a_e
        self.as_, self.ae = a_s, a_e
        self.stream = self.valid and l >= 1 and l + self.pad >= 4


class StreamModel:
    def __init__(self, algo_table: np.ndarray, gf_mul, xpow8n):
        self.T = [int(x) for x in algo_table]
        self.gf_mul = gf_mul
        self.xpow8n = xpow8n
        self.poly = self.T[0x80]

    def raw(self, data: bytes, reg: int = 0) -> int:
        T = self.T
        for b in data:
            reg = T[(reg ^ b) & 0xFF] ^ (reg >> 8)
        return reg

    def xinv8(self, pad: int) -> int:  # x^(-8 pad): divide by x, 8 pad times
        inv = 0x80000000
        for _ in range(8 * pad):
            inv = (((inv ^ self.poly) << 1) | 1) & 0xFFFFFFFF if inv & 0x80000000 else (inv << 1) & 0xFFFFFFFF
        return inv


# ---- positions and ranges ----
# An entry takes the positions after its predecessor's whatever its address (gaps, unsorted,
# overlapping); the group loads its lines from its own address. Positions are a plain prefix sum
# of the entries' new lines.

def range_layout(mis, offsets, lengths, size):
    """Per entry: Geo, shared (first line = the previous entry's last, both in the stream), V (its
    first new line's position) and J' (its new lines); end = the stream's length."""
    n = len(offsets)
    geo = [Geo(mis, int(offsets[i]), int(lengths[i]), size) for i in range(n)]
    shared = [False] * n
    V = [0] * n
    Jn = [0] * n
    end = 0
    for i, g in enumerate(geo):
        if not g.stream:
            continue
        shared[i] = i > 0 and geo[i - 1].stream and g.F == geo[i - 1].Lst
        Jn[i] = g.J - int(shared[i])
        V[i] = end
        end += Jn[i]
    return geo, shared, V, Jn, end


def range_geometry(end, groups, unroll=8):
    tl = -(-max(end, 1) // groups)
    tl = -(-tl // unroll) * unroll
    return tl, -(-end // tl)


class RangeModel(StreamModel):
    """The tile kernel of the free-jump design step by step: per group, a fold at position s and a
    cursor that walks entry records to load position s + 4's line; records come from 8-entry windows
    loaded four steps ahead (`slow` counts the changes that needed a record outside the window; the
    kernel loads one window per round of four steps, a round ahead)."""

    WIN = 8

    def digests(self, base, mis, offsets, lengths, seeds, foreign, groups=7):
        size = len(base)
        geo, shared, V, Jn, end = range_layout(mis, offsets, lengths, size)
        n = len(geo)
        tl, nr = range_geometry(end, groups)
        out = [None] * n
        pfirst, plast = {}, {}
        stats = {"slow": 0, "end": end, "tl": tl, "ranges": nr}

        def line_bytes(L):
            b0 = 128 * L - mis
            return bytes(base[b0 + k] if 0 <= b0 + k < size else foreign[(b0 + k) % len(foreign)]
                         for k in range(128))

        def owner(P):  # the entry whose new lines hold position P (the emit's search)
            for j in range(n):
                if geo[j].stream and V[j] <= P < V[j] + Jn[j]:
                    return j
            raise AssertionError(P)

        for r in range(nr):
            R0 = r * tl
            nla = min(tl, end - R0)
            j0 = owner(R0)
            P0 = V[j0] - int(shared[j0])
            # cursor: (entry, device line, new lines left after this one, previous index in stream)
            cur = {"j": j0, "L": geo[j0].F + (R0 - P0), "rem": geo[j0].Lst - (geo[j0].F + (R0 - P0)), "wb": 0}
            ring = [None] * 4  # (device line, window base) of positions s .. s + 3

            def advance():
                """the cursor's next position: the next new line of its entry, or of the next entry"""
                if cur["rem"] > 0:
                    cur["L"] += 1
                    cur["rem"] -= 1
                    return
                j = cur["j"] + 1
                while j < n:
                    g = geo[j]
                    if not (cur["wb"] <= j < cur["wb"] + self.WIN):
                        stats["slow"] += 1
                    if not g.stream:
                        j += 1
                        continue
                    if shared[j] and g.Lst == g.F:  # inside the current line: no position of its own
                        j += 1
                        continue
                    newF = g.F + int(shared[j])
                    cur["j"], cur["L"], cur["rem"] = j, newF, g.Lst - newF
                    return
                cur["j"], cur["rem"] = n, 0  # past the last entry: a clamped load, never folded

            for s in range(4):  # positions R0 .. R0 + 3 (the prologue may wait for its records)
                if s:
                    cur["wb"] = cur["j"] + 1
                    advance()
                ring[s] = (cur["L"], cur["j"] + 1)
            # fold state
            i = j0
            from_start = P0 >= R0
            piece = bytearray()
            for s in range(nla):
                L, wb = ring[s % 4]
                line = line_bytes(L)
                p = R0 + s
                while True:
                    g = geo[i]
                    lo = max(g.as_, 128 * L) - 128 * L
                    hi = min(g.ae, 128 * L + 128) - 128 * L
                    m = bytearray(128)
                    m[lo:hi] = line[lo:hi]
                    assert lo < hi or (g.l == 0), (r, s, i)
                    if L == g.F:
                        img = seed_image_of(seeds, i).to_bytes(4, "little")
                        for k in range(4):
                            if g.d + k < 128:
                                m[g.d + k] ^= img[k]
                    if L == g.F + 1 and g.d > 124:
                        img = seed_image_of(seeds, i).to_bytes(4, "little")
                        for k in range(4):
                            if g.d + k >= 128:
                                m[g.d + k - 128] ^= img[k]
                    piece += m
                    if L != g.Lst:
                        break
                    reg = self.raw(bytes(piece))
                    if from_start:
                        out[i] = (~self.gf_mul(reg, self.xinv8(g.pad))) & 0xFFFFFFFF
                    else:
                        pfirst[r] = reg
                    piece = bytearray()
                    from_start = True
                    # the next entry in the stream (records from the window of this position)
                    i += 1
                    while i < n and not geo[i].stream:
                        if not (wb <= i < wb + self.WIN):
                            stats["slow"] += 1
                        i += 1
                    if i >= n:
                        break
                    if not (wb <= i < wb + self.WIN):
                        stats["slow"] += 1
                    if shared[i]:
                        continue  # it starts in this same line
                    break
                if i >= n:
                    break
                # the cursor moves to position s + 4 with this slot's window, then refills the slot
                cur["wb"] = wb
                advance()
                ring[s % 4] = (cur["L"], cur["j"] + 1)
                if s + 1 < nla and geo[i].stream:
                    nxt = ring[(s + 1) % 4][0]
                    g = geo[i]
                    if not piece:  # entry i starts at the next position: its first line must be there
                        assert nxt == g.F, (r, s, i, nxt, g.F)
                    else:
                        assert nxt == L + 1, (r, s, i)
            if piece:  # the range ends inside entry i
                if from_start:
                    plast[r] = self.raw(bytes(piece))
                else:
                    pfirst[r] = self.raw(bytes(piece))
        # combine
        X = self.xpow8n(128 * tl)
        for i, g in enumerate(geo):
            if not g.stream:
                if not g.valid:
                    out[i] = 0
                else:
                    out[i] = (~self.raw(bytes(base[g.o:g.o + g.l]), (~int(seeds[i])) & 0xFFFFFFFF)) & 0xFFFFFFFF
                continue
            P0 = V[i] - int(shared[i])
            P1 = P0 + g.J - 1
            t0, t1 = P0 // tl, P1 // tl
            if t0 == t1:
                assert out[i] is not None, i
                continue
            reg = plast[t0]
            for t in range(t0 + 1, t1):
                reg = self.gf_mul(reg, X) ^ pfirst[t]
            reg = self.gf_mul(reg, self.xpow8n(128 * (P1 - tl * t1 + 1))) ^ pfirst[t1]
            out[i] = (~self.gf_mul(reg, self.xinv8(g.pad))) & 0xFFFFFFFF
        return out, stats


def seed_image_of(seeds, i):
    return (~int(seeds[i])) & 0xFFFFFFFF
