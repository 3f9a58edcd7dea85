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
// table (CRC-32); the < 16-byte tail continues bytewise. Small inputs: crc32q/crc32b (CRC-32C)
// or slice-by-8 (CRC-32).
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
};

struct AllConsts {
    Consts c[2];
    bool pclmul = false, sse42 = false;
    AllConsts() {
        for (int algo = 0; algo < 2; ++algo) {
            Consts& k = c[algo];
            for (int s = 0; s < 8; ++s) {
                const uint32_t xs = gf2::xpow(algo, 8ull * (s + 1));
                for (uint32_t b = 0; b < 256; ++b) k.slice[s][b] = gf2::mul(algo, b, xs);
            }
            // a reflected 32-bit operator r (bit j = x^(31-j)) is the qword r << 32 (bit i = x^(63-i))
            auto q = [&](uint64_t e) { return (uint64_t)gf2::xpow(algo, e) << 32; };
            k.k1024[0] = q(63 + 1024), k.k1024[1] = q(1024 - 1);
            k.k512[0] = q(63 + 512), k.k512[1] = q(512 - 1);
            k.k384[0] = q(63 + 384), k.k384[1] = q(384 - 1);
            k.k256[0] = q(63 + 256), k.k256[1] = q(256 - 1);
            k.k128[0] = q(63 + 128), k.k128[1] = q(128 - 1);
        }
        __builtin_cpu_init();
        pclmul = __builtin_cpu_supports("pclmul");
        sse42 = __builtin_cpu_supports("sse4.2");
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

}  // namespace

uint32_t crc_raw(int algo, uint32_t reg, const uint8_t* p, size_t n) {
    const AllConsts& all = consts();
    if (all.pclmul && n >= (algo == 0 && all.sse42 ? 128u : 64u)) return crc_fold(algo, all, reg, p, n);
    if (algo == 0 && all.sse42) return crc32c_hw(reg, p, n);
    return slice8(all.c[algo], reg, p, n);
}

const char* impl_name() {
    const AllConsts& all = consts();
    if (all.pclmul && all.sse42) return "pclmul+sse4.2";
    if (all.pclmul) return "pclmul";
    return "slice8";
}

}  // namespace host
}  // namespace bkd
