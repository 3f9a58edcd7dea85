"""CPU: the chunk kernel's branch-free step-0 block (crc_kernels.hpp first_block_fast / seed_part /
pad_junk_fast, BKD_FIRST_FAST) against the branchy form it replaced (mask_low_bytes, the seed image
`part(k)` and place_seed), restated in Python and compared exhaustively over the offsets a lane can
see: d0 (bytes of the lane's step-0 block in front of the chunk's first byte) and keep (bytes of its
last block that belong to the chunk) from -1100 to 1100, every step width the lane groups use.

Branchy form: w = W0 with bytes < d0 cleared (all cleared from d0 >= 16), XOR the seed
image r0 << 8*d0 when -4 < d0 < 16, spill fx = place_seed(r0, d0 - step) when d0 > step - 4; pad:
junk = last (keep <= 0) or last with bytes < keep cleared.
Branch-free form: per dword k with x8 = 8 * (d0 - 4k):
    keep_from(x, x8) = x & low32(~0 << clamp(x8, 0, 32))
    seed_part(r0, x8) = low32((r0 << 32) >> ((32 - clamp(x8, -32, 32)) mod 64))
"""
import random

import pytest

M32 = 0xFFFFFFFF
M64 = (1 << 64) - 1


def _clamp(x, lo, hi):
    return max(lo, min(x, hi))


# ---- the branch-free form (first_block_fast, seed_part, pad_junk_fast) ----
def keep_from(x, x8):
    return x & ((M64 << _clamp(x8, 0, 32)) & M32)


def seed_part(r0, x8):
    sh = 32 - _clamp(x8, -32, 32)
    return (((r0 << 32) & M64) >> (sh & 63)) & M32


def first_block_fast(w, r0, d0):
    x8 = 8 * d0
    return [keep_from(w[k], x8 - 32 * k) ^ seed_part(r0, x8 - 32 * k) for k in range(4)]


def pad_junk_fast(last, keep):
    return [keep_from(last[k], 8 * keep - 32 * k) for k in range(4)]


# ---- the branchy form it replaced ----
def mask_low_bytes(w, d):
    def m(x, k):
        return 0 if k >= 4 else (x if k <= 0 else x & ((M32 << (8 * k)) & M32))
    return [m(w[k], d - 4 * k) for k in range(4)]


def place_seed(r, d):
    if 0 <= d <= 3:
        return (r << (8 * d)) & M32
    if -3 <= d < 0:
        return r >> (8 * -d)
    return 0


def first_block_branchy(w, r0, d0):
    if d0 <= 0:
        out = list(w)
    elif d0 < 16:
        out = mask_low_bytes(w, d0)
    else:
        out = [0, 0, 0, 0]
    if -4 < d0 < 16:
        R = (r0 << 32) & M64
        for k in range(4):
            t = 32 + 32 * k - 8 * d0
            out[k] ^= ((R >> t) & M32) if 0 < t < 64 else 0
    return out


@pytest.mark.parametrize("step", [64, 128, 256, 512, 1024])
def test_step0_block_and_spill_match_the_branchy_form(step):
    rng = random.Random(step)
    for d0 in range(-1100, 1101):
        for r0 in (0, M32, 0x12345678, 0x80000001, rng.getrandbits(32)):
            w = [rng.getrandbits(32) for _ in range(4)]
            assert first_block_fast(w, r0, d0) == first_block_branchy(w, r0, d0), (d0, hex(r0))
            fx_old = place_seed(r0, d0 - step) if d0 > step - 4 else 0
            assert seed_part(r0, 8 * (d0 - step)) == fx_old, (d0, step)


def test_pad_junk_matches_the_branchy_form():
    rng = random.Random(5)
    for keep in range(-1100, 1101):
        last = [rng.getrandbits(32) for _ in range(4)]
        old = list(last) if keep <= 0 else (mask_low_bytes(last, keep) if keep < 16 else [0, 0, 0, 0])
        assert pad_junk_fast(last, keep) == old, keep


def test_seed_image_lands_where_the_chunk_starts():
    """Semantics, not just equivalence: folding w must equal folding the 16 bytes of W0 with the bytes
    in front of the chunk zeroed and ~seed XORed onto the chunk's first four bytes."""
    rng = random.Random(9)
    for d0 in range(-3, 16):
        w = [rng.getrandbits(32) for _ in range(4)]
        r0 = rng.getrandbits(32)
        block = bytearray(b"".join(x.to_bytes(4, "little") for x in w))
        for i in range(max(0, min(d0, 16))):
            block[i] = 0
        for i in range(4):
            if 0 <= d0 + i < 16:
                block[d0 + i] ^= (r0 >> (8 * i)) & 0xFF
        want = [int.from_bytes(block[4 * k:4 * k + 4], "little") for k in range(4)]
        assert first_block_fast(w, r0, d0) == want, d0
