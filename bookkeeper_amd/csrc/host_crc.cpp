// CPU route of libbkdigest.so: CRC-32C / CRC-32 of one host buffer on the calling thread.
//
// Used by bkd_resume / bkd_resume_host for host buffers up to the per-call threshold (a launch,
// two PCIe copies and a stream sync cost ~30 us, which a core covers ~500 KiB in) and for every
// host buffer when no HIP device is visible. Clean-room, built on the same GF(2) module as the
// GPU tables (crc_tables.hpp): no code from oracle/ or from the reference.
//
// Large inputs: carry-less-multiply folding. A 16-byte block loaded little-endian is a 128-bit
// reflected polynomial (register bit k = coefficient of x^(127-k)); its low qword H holds
// x^127..x^64, its high qword L x^63..x^0. Moving a block D bits forward multiplies it by x^D:
//   X * x^D = H * x^(64+D) + L * x^D  ==  clmul(H, x^(63+D) mod P) ^ clmul(L, x^(D-1) mod P)
// because pclmulqdq of two reflected qwords yields x * (their product) in the 128-bit reflected
// layout (hence the -1 in both exponents). Eight accumulators stride 128 bytes (D = 1024) and
// pair up into four (D = 512), which merge with D = 384/256/128; single blocks then fold with
// D = 128. The last 128-bit remainder
// X becomes the CRC register X * x^32 mod P through two crc32q steps (CRC-32C) or the slice-by-8
// table (CRC-32); the < 16-byte tail continues bytewise. From 1 KiB on, CPUs with AVX-512
// VPCLMULQDQ fold four 128-bit blocks per instruction (crc_fold512): ~55-65 GB/s on one core
// against ~20 for the 128-bit path. Small inputs: crc32q/crc32b (CRC-32C) or slice-by-8 (CRC-32).
#include "host_crc.hpp"

#include <immintrin.h>
#include <string.h>

#include "crc_tables.hpp"

namespace bkd {
namespace host {
namespace {

struct Consts {
    uint32_t slice[8][256];  // slice[k][b] = b * x^(8(k+1)) mod P (slice[0] = ReflectedIntCrc's table)
    uint64_t k1024[2], k512[2], k384[2], k256[2], k128[2];  // {x^(63+D), x^(D-1)} mod P, as qword operands
    uint64_t k2048[2], k1536[2];                           // the 512-bit path's strides
};

struct AllConsts {
    Consts c[2];
    bool pclmul = false, sse42 = false, vpclmul512 = false;
    AllConsts() {
        for (int algo = 0; algo < 2; ++algo) {
            Consts& k = c[algo];
            for (int s = 0; s < 8; ++s) {
                const uint32_t xs = gf2::xpow(algo, 8ull * (s + 1));
                for (uint32_t b = 0; b < 256; ++b) k.slice[s][b] = gf2::mul(algo, b, xs);
            }
            // a reflected 32-bit operator r (bit j = x^(31-j)) is the qword r << 32 (bit i = x^(63-i))
            auto q = [&](uint64_t e) { return (uint64_t)gf2::xpow(algo, e) << 32; };
            k.k2048[0] = q(63 + 2048), k.k2048[1] = q(2048 - 1);
            k.k1536[0] = q(63 + 1536), k.k1536[1] = q(1536 - 1);
            k.k1024[0] = q(63 + 1024), k.k1024[1] = q(1024 - 1);
            k.k512[0] = q(63 + 512), k.k512[1] = q(512 - 1);
            k.k384[0] = q(63 + 384), k.k384[1] = q(384 - 1);
            k.k256[0] = q(63 + 256), k.k256[1] = q(256 - 1);
            k.k128[0] = q(63 + 128), k.k128[1] = q(128 - 1);
        }
        __builtin_cpu_init();
        pclmul = __builtin_cpu_supports("pclmul");
        sse42 = __builtin_cpu_supports("sse4.2");
        vpclmul512 = pclmul && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                     __builtin_cpu_supports("vpclmulqdq");
    }
};

const AllConsts& consts() {
    static const AllConsts k;  // thread-safe one-time init
    return k;
}

inline uint64_t load64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

uint32_t slice8(const Consts& k, uint32_t reg, const uint8_t* p, size_t n) {
    while (n >= 8) {
        const uint64_t v = load64(p) ^ reg;
        reg = k.slice[7][v & 0xFF] ^ k.slice[6][(v >> 8) & 0xFF] ^ k.slice[5][(v >> 16) & 0xFF] ^
              k.slice[4][(v >> 24) & 0xFF] ^ k.slice[3][(v >> 32) & 0xFF] ^ k.slice[2][(v >> 40) & 0xFF] ^
              k.slice[1][(v >> 48) & 0xFF] ^ k.slice[0][v >> 56];
        p += 8;
        n -= 8;
    }
    while (n--) reg = (reg >> 8) ^ k.slice[0][(reg ^ *p++) & 0xFF];
    return reg;
}

__attribute__((target("sse4.2"))) uint32_t crc32c_hw(uint32_t reg, const uint8_t* p, size_t n) {
    uint64_t r = reg;
    while (n >= 8) {
        r = _mm_crc32_u64(r, load64(p));
        p += 8;
        n -= 8;
    }
    uint32_t r32 = (uint32_t)r;
    while (n--) r32 = _mm_crc32_u8(r32, *p++);
    return r32;
}

__attribute__((target("pclmul,sse4.2"))) inline __m128i fold(__m128i x, const uint64_t* kk) {
    const __m128i k = _mm_set_epi64x((long long)kk[1], (long long)kk[0]);
    return _mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11));
}

__attribute__((target("pclmul,sse4.2"))) uint32_t crc_fold(int algo, const AllConsts& all, uint32_t reg,
                                                             const uint8_t* p, size_t n) {
    const Consts& k = all.c[algo];
    // n >= 64: the raw register enters as the first 4 message bytes XOR-ed with it
    __m128i x[8];
    for (int i = 0; i < 4; ++i) x[i] = _mm_loadu_si128((const __m128i*)(p + 16 * i));
    x[0] = _mm_xor_si128(x[0], _mm_cvtsi32_si128((int)reg));
    p += 64;
    n -= 64;
    if (n >= 64) {  // eight accumulators 128 bytes apart (D = 1024): more clmuls in flight
        for (int i = 4; i < 8; ++i) x[i] = _mm_loadu_si128((const __m128i*)(p + 16 * (i - 4)));
        p += 64;
        n -= 64;
        while (n >= 128) {
            for (int i = 0; i < 8; ++i)
                x[i] = _mm_xor_si128(fold(x[i], k.k1024), _mm_loadu_si128((const __m128i*)(p + 16 * i)));
            p += 128;
            n -= 128;
        }
        for (int i = 0; i < 4; ++i) x[i] = _mm_xor_si128(fold(x[i], k.k512), x[i + 4]);
    }
    while (n >= 64) {
        for (int i = 0; i < 4; ++i)
            x[i] = _mm_xor_si128(fold(x[i], k.k512), _mm_loadu_si128((const __m128i*)(p + 16 * i)));
        p += 64;
        n -= 64;
    }
    __m128i y = _mm_xor_si128(_mm_xor_si128(fold(x[0], k.k384), fold(x[1], k.k256)),
                              _mm_xor_si128(fold(x[2], k.k128), x[3]));
    while (n >= 16) {
        y = _mm_xor_si128(fold(y, k.k128), _mm_loadu_si128((const __m128i*)p));
        p += 16;
        n -= 16;
    }
    // register = X * x^32 mod P = the CRC of X's 16 bytes from a zero register
    alignas(16) uint8_t xb[16];
    _mm_store_si128((__m128i*)xb, y);
    uint32_t r;
    if (algo == 0 && all.sse42) {
        r = (uint32_t)_mm_crc32_u64(_mm_crc32_u64(0, load64(xb)), load64(xb + 8));
        while (n--) r = _mm_crc32_u8(r, *p++);
    } else {
        r = slice8(k, 0, xb, 16);
        r = slice8(k, r, p, n);
    }
    return r;
}

// 512-bit folding (AVX-512 VPCLMULQDQ: four 128-bit blocks per instruction), for long buffers:
// four zmm accumulators stride 256 bytes (D = 2048), merge into one (D = 1536/1024/512), its four
// 128-bit lanes into one (D = 384/256/128), and the 128-bit path finishes the remainder.
#define BKD_AVX512 "avx512f,avx512vl,vpclmulqdq,pclmul,sse4.2"
__attribute__((target(BKD_AVX512))) inline __m512i fold512(__m512i x, const uint64_t* kk) {
    const __m512i k = _mm512_broadcast_i32x4(_mm_set_epi64x((long long)kk[1], (long long)kk[0]));
    return _mm512_xor_si512(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11));
}

__attribute__((target(BKD_AVX512))) uint32_t crc_fold512(int algo, const AllConsts& all, uint32_t reg,
                                                        const uint8_t* p, size_t n) {
    const Consts& k = all.c[algo];
    // n >= 256: the raw register enters as the first 4 message bytes XOR-ed with it
    __m512i x0 = _mm512_loadu_si512(p), x1 = _mm512_loadu_si512(p + 64), x2 = _mm512_loadu_si512(p + 128),
            x3 = _mm512_loadu_si512(p + 192);
    x0 = _mm512_xor_si512(x0, _mm512_castsi128_si512(_mm_cvtsi32_si128((int)reg)));
    p += 256;
    n -= 256;
    while (n >= 256) {
        x0 = _mm512_xor_si512(fold512(x0, k.k2048), _mm512_loadu_si512(p));
        x1 = _mm512_xor_si512(fold512(x1, k.k2048), _mm512_loadu_si512(p + 64));
        x2 = _mm512_xor_si512(fold512(x2, k.k2048), _mm512_loadu_si512(p + 128));
        x3 = _mm512_xor_si512(fold512(x3, k.k2048), _mm512_loadu_si512(p + 192));
        p += 256;
        n -= 256;
    }
    __m512i x = _mm512_ternarylogic_epi64(fold512(x0, k.k1536), fold512(x1, k.k1024), fold512(x2, k.k512), 0x96);
    x = _mm512_xor_si512(x, x3);
    // lanes 0..3 of x are 128-bit blocks 0..3 of the last 64 bytes
    const __m128i l0 = _mm512_extracti32x4_epi32(x, 0), l1 = _mm512_extracti32x4_epi32(x, 1),
                  l2 = _mm512_extracti32x4_epi32(x, 2), l3 = _mm512_extracti32x4_epi32(x, 3);
    __m128i y = _mm_xor_si128(_mm_xor_si128(fold(l0, k.k384), fold(l1, k.k256)), _mm_xor_si128(fold(l2, k.k128), l3));
    while (n >= 16) {
        y = _mm_xor_si128(fold(y, k.k128), _mm_loadu_si128((const __m128i*)p));
        p += 16;
        n -= 16;
    }
    alignas(16) uint8_t xb[16];
    _mm_store_si128((__m128i*)xb, y);
    uint32_t r;
    if (algo == 0) {
        r = (uint32_t)_mm_crc32_u64(_mm_crc32_u64(0, load64(xb)), load64(xb + 8));
        while (n--) r = _mm_crc32_u8(r, *p++);
    } else {
        r = slice8(k, 0, xb, 16);
        r = slice8(k, r, p, n);
    }
    return r;
}

}  // namespace

uint32_t crc_raw(int algo, uint32_t reg, const uint8_t* p, size_t n) {
    const AllConsts& all = consts();
    if (all.vpclmul512 && all.sse42 && n >= 1024) return crc_fold512(algo, all, reg, p, n);
    if (all.pclmul && n >= (algo == 0 && all.sse42 ? 128u : 64u)) return crc_fold(algo, all, reg, p, n);
    if (algo == 0 && all.sse42) return crc32c_hw(reg, p, n);
    return slice8(all.c[algo], reg, p, n);
}

bool has_wide_fold() {
    const AllConsts& all = consts();
    return all.vpclmul512 && all.sse42;
}

const char* impl_name() {
    const AllConsts& all = consts();
    if (all.vpclmul512 && all.sse42) return "vpclmul512+pclmul+sse4.2";
    if (all.pclmul && all.sse42) return "pclmul+sse4.2";
    if (all.pclmul) return "pclmul";
    return "slice8";
}

}  // namespace host
}  // namespace bkd
