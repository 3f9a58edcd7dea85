// Host-side GF(2) arithmetic and the fold-table image the CRC kernels stage into LDS.
//
// The reference precomputes "shift the CRC register forward by N bytes" operators as
// 256-entry tables (chunk_config::make_shift_table, circe-checksum/src/main/circe/cpp/
// crc32c_sse42.cpp:82-90, via a 32x32 bit-matrix power in gf2.hpp:120-174) to merge its
// three interleaved crc32q streams. The GPU engine needs the same operators, but for
// every byte position of a 32-bit register (4 tables per operator) and for the operator
// set of its lane/stride geometry. They are computed here directly as
// polynomial products modulo P in the reflected bit order, which needs no matrices:
//   bit 31 of a register = coefficient of x^0, bit 0 = coefficient of x^31,
//   multiply-by-x = (r >> 1) ^ (r & 1 ? Prefl : 0).
#pragma once
#include <stdint.h>

namespace bkd {
namespace gf2 {

// Reflected generator polynomials (CRC-32C: crc32c_sse42.cpp:85; CRC-32: CrcParameters.java:167-180).
inline uint32_t poly(int algo) { return algo == 0 ? 0x82F63B78u : 0xEDB88320u; }

inline uint32_t mulx(int algo, uint32_t r) { return (r >> 1) ^ ((r & 1u) ? poly(algo) : 0u); }

// a * b mod P.
inline uint32_t mul(int algo, uint32_t a, uint32_t b) {
    uint32_t p = 0, cur = b;
    for (int k = 0; k < 32; ++k) {
        if ((a >> (31 - k)) & 1u) p ^= cur;
        cur = mulx(algo, cur);
    }
    return p;
}

// x^nbits mod P.
inline uint32_t xpow(int algo, uint64_t nbits) {
    uint32_t result = 0x80000000u;  // x^0
    uint32_t base = 0x40000000u;    // x^1
    while (nbits) {
        if (nbits & 1) result = mul(algo, result, base);
        base = mul(algo, base, base);
        nbits >>= 1;
    }
    return result;
}

// Inverse of mulx: the register before one zero bit was folded in. Prefl has bit 31 (x^0) set,
// so bit 31 of y says whether the low bit of the pre-image was 1.
inline uint32_t divx(int algo, uint32_t y) {
    return (y & 0x80000000u) ? (((y ^ poly(algo)) << 1) | 1u) : (y << 1);
}

// x^(-8k) mod P: undoes k zero bytes appended to a message (the ragged plan pads each entry to
// the next 128-byte line with zeros, plan_kernels.hpp).
inline uint32_t xpow_neg8(int algo, uint32_t k) {
    uint32_t r = 0x80000000u;
    for (uint32_t i = 0; i < 8u * k; ++i) r = divx(algo, r);
    return r;
}

// Operator "multiply a 32-bit register by C" split by byte position:
// out[t*256 + b] = (b << 8t) * C mod P, so r*C = T0[r&255] ^ T1[r>>8&255] ^ T2[r>>16&255] ^ T3[r>>24].
inline void operator_tables(int algo, uint32_t C, uint32_t* out) {
    for (int t = 0; t < 4; ++t)
        for (uint32_t b = 0; b < 256; ++b) out[t * 256 + b] = mul(algo, b << (8 * t), C);
}

inline int log2_lanes(int lanes) {
    int l = 0;
    while ((1 << l) < lanes) ++l;
    return l;
}

// Compact image (u32 words), for a group of `lanes` lanes that each fold 16 bytes per step:
//   set 0                : C_main = x^(128*lanes)   (one step of every lane stream, stride 16*lanes bytes)
//   set 1                : x^32                     (dword-to-dword inside a lane)
//   set 2+s, s<log2 lanes: x^(128 * 2^s)            (lane-tree level s: a block of 2^s lanes = 16*2^s bytes)
//   256 words            : byte table x^8           (serial paths; equals ReflectedIntCrc's table)
//   2 more sets          : x^64, x^96               (one-level in-lane combine of the 4 dword streams)
//   groups of 4 / 8 lanes: lane-position nibble tables, word (16k + n) * lanes + g =
//                          (n << 4k) * x^(128 (lanes - 1 - g)) — lane g's weight in its group's register,
//                          interleaved by lane so that a half-wave's lookups spread over the 32 banks
inline int64_t byte_table_offset(int lanes) { return (int64_t)(2 + log2_lanes(lanes)) * 1024; }
inline bool has_lane_tables(int lanes) { return lanes == 4 || lanes == 8; }
inline int64_t lane_table_offset(int lanes) { return byte_table_offset(lanes) + 256 + 2048; }
inline int64_t compact_words(int lanes) { return lane_table_offset(lanes) + (has_lane_tables(lanes) ? 128 * lanes : 0); }

inline int64_t build_compact(int algo, int lanes, uint32_t* out) {
    const int levels = log2_lanes(lanes);
    operator_tables(algo, xpow(algo, 128ull * (uint64_t)lanes), out);
    operator_tables(algo, xpow(algo, 32), out + 1024);
    for (int s = 0; s < levels; ++s) operator_tables(algo, xpow(algo, 128ull << s), out + 2048 + 1024 * s);
    uint32_t* bt = out + byte_table_offset(lanes);
    const uint32_t x8 = xpow(algo, 8);
    for (uint32_t b = 0; b < 256; ++b) bt[b] = mul(algo, b, x8);
    operator_tables(algo, xpow(algo, 64), bt + 256);
    operator_tables(algo, xpow(algo, 96), bt + 256 + 1024);
    if (has_lane_tables(lanes)) {
        uint32_t* lt = out + lane_table_offset(lanes);
        for (int g = 0; g < lanes; ++g) {
            const uint32_t w = xpow(algo, 128ull * (uint64_t)(lanes - 1 - g));
            for (int k = 0; k < 8; ++k)
                for (uint32_t n = 0; n < 16; ++n) lt[(16 * k + (int)n) * lanes + g] = mul(algo, n << (4 * k), w);
        }
    }
    return compact_words(lanes);
}

}  // namespace gf2
}  // namespace bkd
