// CDNA4 (gfx950) CRC32C / CRC32 batch kernels — one CRC per ledger entry.
//
// Replaces the per-entry host scan of circe-checksum (crc32c(), circe-checksum/src/main/
// circe/cpp/crc32c_sse42.cpp:184-217, hot loop :100-104) with a batched byte scan over
// HBM-resident entries. Design:
//
//  * A GROUP of G lanes (G | 64) owns one entry at a time. Its window is END-aligned:
//    J = ceil(len / 16G) steps; at step j lane g loads the 16 bytes at
//    end - 16G*(J-j) + 16g with one global_load_dwordx4. Bytes in front of the entry
//    (head of step 0) are zero, which leaves a zero-initialised CRC register unchanged,
//    so no length-dependent shift is ever needed.
//  * Each lane keeps 4 independent dword streams; every stream advances by the same
//    operator C = x^(128G) ("skip 16G bytes"), so ONE operator table set serves all
//    streams: acc = acc*C ^ dword. The 4 byte tables of C are replicated 32x in LDS with
//    entry b of table t for bank k at byte (t>>1)*64Ki + b*256 + (t&1)*128 + 4k; lane k of
//    each 32-lane half reads only bank k, so the random-index lookups are bank-conflict free.
//    One v_perm_b32 builds each lookup address (byte index -> bits 8..15, lane bank -> bits 2..6).
//  * The seed is folded into the data: XOR ~seed into the entry's first 4 bytes
//    (reg(r, D) = reg(0, D ^ r||0...)), valid for len >= 4; entries < 16 B take a serial path.
//  * Finish: in-lane Horner over the 4 streams with x^32, a log2(G) shuffle tree with
//    x^(128*2^s), a final x^32, complement. Those operator tables are compact (unreplicated).
//
// The reference merges streams the same way with its shift tables (crc32c_sse42.cpp:107-126,
// make_shift_table :82-90); here the merge operators are per lane tree level.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

namespace bkd {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 1024;          // 16 waves per CU, one workgroup per CU (LDS-limited)
constexpr uint32_t kMainBytes = 131072u;  // 4 tables x 256 entries x 32 banks x 4 B

#ifndef BKD_LANE_POS
#define BKD_LANE_POS 1  // groups of 4 / 8 lanes finish by lane-position tables + DPP XOR (finish_lanes)
#endif

template <int G>
struct Geo {
    static_assert(G == 1 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "group width");
    static constexpr int kLevels = G == 1 ? 0 : G == 4 ? 2 : G == 8 ? 3 : G == 16 ? 4 : G == 32 ? 5 : 6;
    // Groups of <= 16 lanes sit inside one DPP row and have LDS room for the x^64/x^96 sets.
    static constexpr bool kFast = G <= 16;
    // Groups of 4 / 8 lanes also stage the lane-position nibble tables (crc_tables.hpp).
    static constexpr bool kLaneTab = BKD_LANE_POS && (G == 4 || G == 8);
    static constexpr int kCompactWords = (2 + kLevels) * 1024 + 256 + 2048 + (kLaneTab ? 128 * G : 0);
    static constexpr int kAuxWords = kCompactWords - 1024 - (kFast ? 0 : 2048);  // staged after the main set
    static constexpr uint32_t kX32Off = kMainBytes;  // LDS byte offset of the x^32 set
    static constexpr uint32_t kByteTabOff = kMainBytes + (1 + kLevels) * 4096u;
    static constexpr uint32_t kX64Off = kByteTabOff + 1024u;
    static constexpr uint32_t kX96Off = kX64Off + 4096u;
    static constexpr uint32_t kLaneOff = kX96Off + 4096u;
    static constexpr int kLdsWords = (int)(kMainBytes / 4) + kAuxWords;
    static constexpr int64_t kStep = 16 * G;
};

__device__ __forceinline__ uint32_t lds_word(const uint32_t* lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}

// a ^ b ^ c in one v_bitop3_b32 (gfx950; truth table 0x96), for the compact-table products.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

#ifndef BKD_EARLY_PREFETCH
#define BKD_EARLY_PREFETCH 0
#endif
#ifndef BKD_TAIL_UNCOND
#define BKD_TAIL_UNCOND 0  // build-time variant: unconditional tail loads in the A/B fold loops
#endif
#ifndef BKD_CHUNK_UNROLL
#define BKD_CHUNK_UNROLL 2  // chunk halves per iteration of the chunk kernel's loop (2, 4 or 8)
#endif

#ifndef BKD_MAIN_XOR3
#define BKD_MAIN_XOR3 0  // build-time variant: the main fold's five-way XOR as two v_bitop3 (tools/ab_libs.py)
#endif

// v * C_main via the replicated tables. lanereg = 4*(lane&31) | 1<<16.
// v_perm_b32 result bytes (b3..b0) = (0, hi, v.byte_t, 4*(lane&31)); hi = 1 selects the
// upper 64 KiB half (tables 2, 3); the +128 immediate selects the odd table of a pair.
// mul_main_add(.., d) = v * C_main ^ d.
__device__ __forceinline__ uint32_t mul_main_add(const uint32_t* lds, uint32_t v, uint32_t lanereg, uint32_t d) {
    const uint32_t a0 = __builtin_amdgcn_perm(v, lanereg, 0x0C0C0400u);
    const uint32_t a1 = __builtin_amdgcn_perm(v, lanereg, 0x0C0C0500u);
    const uint32_t a2 = __builtin_amdgcn_perm(v, lanereg, 0x0C020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(v, lanereg, 0x0C020700u);
#if BKD_MAIN_XOR3
    return xor3(xor3(lds_word(lds, a0), lds_word(lds, a1 + 128u), lds_word(lds, a2)), lds_word(lds, a3 + 128u), d);
#else
    // plain XORs: consumed in issue order (a v_bitop3 here measured up to 10 % slower on short entries)
    return lds_word(lds, a0) ^ lds_word(lds, a1 + 128u) ^ lds_word(lds, a2) ^ lds_word(lds, a3 + 128u) ^ d;
#endif
}

#ifndef BKD_W0_CACHED
#define BKD_W0_CACHED 0  // 1: every chunk's first block is a cached load (A/B)
#endif
#ifndef BKD_CLOCK_ADAPT
#define BKD_CLOCK_ADAPT 1  // 0: the one-entry-per-group fold always uses mul_main_add
#endif
#ifndef BKD_LOW_CLOCK_MHZ
#define BKD_LOW_CLOCK_MHZ 2000
#endif
constexpr uint64_t kLowClockMHz = BKD_LOW_CLOCK_MHZ;

// One fold step of the four dword streams, c_k = c_k * C_main ^ d_k, with all 16 table lookups in
// flight at once and the XORs as v_bitop3: the compiler's schedule (mul_main_add) issues them 8 at
// a time and drains (lgkmcnt(0)) between the batches, two LDS round trips per step. Faster when the
// shader clock is power-limited, slower at full clock: groups_loop picks one per
// launch from the clock it measures (crc_groups_kernel). The lookups are inline-asm ds_read_b32 from
// the kernel's LDS image (its only __shared__ array, at LDS address 0: the byte addresses v_perm
// builds are absolute), followed by one s_waitcnt that takes every result as an operand, so no use
// can be scheduled before it.
// fold4_main is valid only while the table image really sits at LDS address 0 (another
// __shared__ variable in a kernel that uses it could move the image): the kernels take it only when
// this holds, otherwise they keep the compiler's schedule (same digests, mul_main_add).
__device__ __forceinline__ bool lds_image_at_zero(const uint32_t* lds) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)lds == 0u;
}

// One fold step of the four streams with all 16 lookups requested before any is used, through the
// compiler's own LDS addressing (so valid wherever the image sits; its waits are counted): the
// scheduling barriers keep the 16 address perms, then the 16 reads, then the XORs together.
__device__ __forceinline__ void fold4_grouped(const uint32_t* lds, uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                              uint32_t& c3, uint32_t lanereg, uint32_t d0, uint32_t d1, uint32_t d2,
                                              uint32_t d3) {
    uint32_t t[16];
    const uint32_t cs[4] = {c0, c1, c2, c3};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        t[4 * k + 0] = lds_word(lds, __builtin_amdgcn_perm(cs[k], lanereg, 0x0C0C0400u));
        t[4 * k + 1] = lds_word(lds, __builtin_amdgcn_perm(cs[k], lanereg, 0x0C0C0500u) + 128u);
        t[4 * k + 2] = lds_word(lds, __builtin_amdgcn_perm(cs[k], lanereg, 0x0C020600u));
        t[4 * k + 3] = lds_word(lds, __builtin_amdgcn_perm(cs[k], lanereg, 0x0C020700u) + 128u);
    }
    __builtin_amdgcn_sched_group_barrier(0x0002, 16, 0);  // the 16 address perms (VALU)
    __builtin_amdgcn_sched_group_barrier(0x0100, 16, 0);  // the 16 reads (DS read)
    c0 = xor3(xor3(t[0], t[1], t[2]), t[3], d0);
    c1 = xor3(xor3(t[4], t[5], t[6]), t[7], d1);
    c2 = xor3(xor3(t[8], t[9], t[10]), t[11], d2);
    c3 = xor3(xor3(t[12], t[13], t[14]), t[15], d3);
}

__device__ __forceinline__ void fold4_main(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t lanereg,
                                           uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3) {
    uint32_t t[16];
    const uint32_t cs[4] = {c0, c1, c2, c3};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t a0 = __builtin_amdgcn_perm(cs[k], lanereg, 0x0C0C0400u);
        const uint32_t a1 = __builtin_amdgcn_perm(cs[k], lanereg, 0x0C0C0500u);
        const uint32_t a2 = __builtin_amdgcn_perm(cs[k], lanereg, 0x0C020600u);
        const uint32_t a3 = __builtin_amdgcn_perm(cs[k], lanereg, 0x0C020700u);
        asm volatile("ds_read_b32 %0, %1" : "=v"(t[4 * k + 0]) : "v"(a0));
        asm volatile("ds_read_b32 %0, %1 offset:128" : "=v"(t[4 * k + 1]) : "v"(a1));
        asm volatile("ds_read_b32 %0, %1" : "=v"(t[4 * k + 2]) : "v"(a2));
        asm volatile("ds_read_b32 %0, %1 offset:128" : "=v"(t[4 * k + 3]) : "v"(a3));
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7]),
                   "+v"(t[8]), "+v"(t[9]), "+v"(t[10]), "+v"(t[11]), "+v"(t[12]), "+v"(t[13]), "+v"(t[14]),
                   "+v"(t[15]));
    c0 = xor3(xor3(t[0], t[1], t[2]), t[3], d0);
    c1 = xor3(xor3(t[4], t[5], t[6]), t[7], d1);
    c2 = xor3(xor3(t[8], t[9], t[10]), t[11], d2);
    c3 = xor3(xor3(t[12], t[13], t[14]), t[15], d3);
}

__device__ __forceinline__ uint32_t mul_main(const uint32_t* lds, uint32_t v, uint32_t lanereg) {
    return mul_main_add(lds, v, lanereg, 0u);
}

// v * C via a compact 4x256 operator set at LDS byte offset `off`.
__device__ __forceinline__ uint32_t mul_aux_add(const uint32_t* lds, uint32_t off, uint32_t v, uint32_t d) {
    return xor3(xor3(lds_word(lds, off + ((v & 0xffu) << 2)), lds_word(lds, off + 1024u + (((v >> 8) & 0xffu) << 2)),
                     lds_word(lds, off + 2048u + (((v >> 16) & 0xffu) << 2))),
                lds_word(lds, off + 3072u + ((v >> 24) << 2)), d);
}

__device__ __forceinline__ uint32_t mul_aux(const uint32_t* lds, uint32_t off, uint32_t v) {
    return mul_aux_add(lds, off, v, 0u);
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
}

// 128-bit left shift by d bytes (1..15): out byte k = in byte k-d, zeros below.
__device__ __forceinline__ u32x4 shl_bytes(u32x4 v, uint32_t d) {
    uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
    uint64_t hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
    const uint32_t sh = d * 8u;
    if (sh >= 64u) {
        hi = lo << (sh - 64u);
        lo = 0;
    } else {
        hi = (hi << sh) | (lo >> (64u - sh));
        lo <<= sh;
    }
    u32x4 r;
    r.x = (uint32_t)lo; r.y = (uint32_t)(lo >> 32); r.z = (uint32_t)hi; r.w = (uint32_t)(hi >> 32);
    return r;
}

// The part of the 4-byte register image r that lands in the dword starting d bytes
// before it (d in [-3, 3], little-endian), else 0.
__device__ __forceinline__ uint32_t place_seed(uint32_t r, int64_t d) {
    if (d >= 0 && d <= 3) return r << (8 * (uint32_t)d);
    if (d < 0 && d >= -3) return r >> (8 * (uint32_t)(-d));
    return 0u;
}

// ---- work sources ---------------------------------------------------------------------
// get(w, it) describes work item w: the byte range [s, s+len) of `base`, the raw register r0
// folded into its first bytes (~seed for a whole entry or a chunk at an entry's head, 0 for an
// inner chunk), and where the result goes: *dst = reg ^ xorout (~0 = finalized CRC, 0 = raw
// partial register). Return: 0 compute, 1 write 0 to *dst, 2 out of bounds (write 0, flag),
// 3 nothing to do.

struct Work {
    int64_t s;
    uint32_t len;
    uint32_t r0;
    uint32_t* dst;
    uint32_t xorout;
};

struct UniformSrc {
    uint64_t n;
    uint64_t stride;
    uint32_t len;
    const uint32_t* seeds;
    uint32_t seed_all;
    uint32_t* out;
    __device__ __forceinline__ uint64_t count() const { return n; }
    __device__ __forceinline__ int get(uint64_t i, Work& w) const {
        w.s = (int64_t)(i * stride);
        w.len = len;
        w.r0 = ~(seeds ? seeds[i] : seed_all);
        w.dst = out + i;
        w.xorout = 0xFFFFFFFFu;
        return 0;
    }
};

// Uniform entries of at least kTailUncondSteps steps in 8-lane groups: the same work items, folded
// with unconditional tail loads (fold_range's TAILU; chosen on the host from the entry length).
constexpr uint32_t kTailUncondSteps = 32;
struct UniformLongSrc : UniformSrc {};

struct IndexedSrc {
    uint64_t n;
    const uint64_t* offsets;
    const uint32_t* lengths;
    const uint32_t* seeds;
    uint32_t seed_all;
    uint64_t size;
    uint32_t* out;
    __device__ __forceinline__ uint64_t count() const { return n; }
    __device__ __forceinline__ int get(uint64_t i, Work& w) const {
        const uint64_t o = offsets[i];
        const uint32_t l = lengths[i];
        w.dst = out + i;
        if (o > size || (uint64_t)l > size - o) return 2;
        w.s = (int64_t)o;
        w.len = l;
        w.r0 = ~(seeds ? seeds[i] : seed_all);
        w.xorout = 0xFFFFFFFFu;
        return 0;
    }
};

// The digest field of a packaged frame (f = frame + 32): the BE digest, after a zero high word for
// CRC32's 8-byte digest (CRC32CDigestManager.java:44-46 writeInt, CRC32DigestManager.java:60-63
// writeLong); dword stores when f is 4-byte aligned, bytes otherwise.
__device__ __forceinline__ void put_frame_digest(uint8_t* f, uint32_t digest, uint32_t mac) {
    const uint32_t be = __builtin_bswap32(digest);
    if ((((uintptr_t)f) & 3u) == 0) {
        uint32_t* d = reinterpret_cast<uint32_t*>(f);
        if (mac == 8) *d++ = 0u;
        *d = be;
    } else {
        if (mac == 8) {
            f[0] = f[1] = f[2] = f[3] = 0;
            f += 4;
        }
        for (int k = 0; k < 4; ++k) f[k] = (uint8_t)(be >> (8 * k));
    }
}

// Package payloads: IndexedSrc whose results (seeded with the header CRCs) are also written into
// each frame's digest field by the group that computed them (the BKD_PACKAGE_DIGEST_PASS=0 build:
// 3 % slower than the separate digest pass).
struct PackageSrc : IndexedSrc {
    uint8_t* frames;
    uint64_t stride;
    uint32_t mac;
};

// Where a work item's result goes: *dst, and for package payloads the frame's digest field too.
template <class Src>
__device__ __forceinline__ void put_result(const Src&, uint64_t, const Work& w, uint32_t v) {
    *w.dst = v;
}
__device__ __forceinline__ void put_result(const PackageSrc& src, uint64_t i, const Work& w, uint32_t v) {
    *w.dst = v;
    put_frame_digest(src.frames + i * src.stride + 32, v, src.mac);
}

// Framed entry [32 B header][mac][payload]: CRC the payload resuming from the header CRC
// already stored in seeds[i] (DigestManager.java:236-239); result over seeds[i] in place.
struct FramedPayloadSrc {
    uint64_t n;
    const uint64_t* offsets;
    const uint32_t* lengths;
    uint32_t* seeds;
    uint64_t size;
    uint32_t mac;
    __device__ __forceinline__ uint64_t count() const { return n; }
    __device__ __forceinline__ int get(uint64_t i, Work& w) const {
        const uint64_t o = offsets[i];
        const uint32_t l = lengths[i];
        w.dst = seeds + i;
        if (o > size || (uint64_t)l > size - o) return 2;
        if (l < 32u + mac) return 1;
        w.s = (int64_t)(o + 32u + mac);
        w.len = l - 32u - mac;
        w.r0 = ~seeds[i];
        w.xorout = 0xFFFFFFFFu;
        return 0;
    }
};

// Indexed entries of at most `small` bytes (small <= 16*G*(PF+1)): the short-entry class of a
// ragged batch, run by its own launch (indexed_small_loop) while the chunked plan takes the rest
// (plan_kernels.hpp, PlanGeo::small). Longer entries are skipped here.
struct SmallIndexedSrc {
    uint64_t n;
    const uint64_t* offsets;
    const uint32_t* lengths;
    const uint32_t* seeds;
    uint32_t seed_all;
    uint64_t size;
    uint32_t* out;
    uint32_t small;
    uint32_t* plan_flag;  // set to plan_epoch when an entry of the plan's is met (PlanRun)
    uint32_t plan_epoch;
    __device__ __forceinline__ uint64_t count() const { return n; }
};

// Which launches of an indexed call through the plan have work (no host sync decides it):
//  * with a short-entry class, its launch (which reads every length first) stores `epoch` into
//    *flag when it meets an entry of the plan's; without one, the plan always has entries;
//  * with a uniformity gate, plan_count ballots each entry block's lengths against the first
//    entry's (in_band) and plan_scan's extra block stores `epoch` into *uni when every block
//    agreed (no reset between calls). Lengths that close are balanced one entry per lane group
//    already: emit and combine return at once and the chunk kernel computes every entry whole,
//    as the direct kernel does (PlanDirectSrc::all) — no extra launch. The choice only picks the
//    schedule; both give the same digests.
struct PlanRun {
    const uint32_t* flag;
    const uint32_t* uni;
    uint32_t epoch;
    __device__ __forceinline__ bool plan_entries() const { return !flag || *flag == epoch; }
    __device__ __forceinline__ bool uniform() const { return uni && *uni == epoch; }
    __device__ __forceinline__ bool on() const { return plan_entries() && !uniform(); }
    // (emit, chunk and combine test on(); plan_count and plan_scan run before it is known)
    // within 1/16 of the reference length + half a 128-byte line either way
    __device__ static __forceinline__ bool in_band(uint32_t l, uint32_t ref) {
        const uint32_t d = l > ref ? l - ref : ref - l;
        return d <= ref / 16u + 64u;
    }
};

// DPP row_shl:SH — lane i receives lane i + SH of its 16-lane row (0 past the row end).
template <int SH>
__device__ __forceinline__ uint32_t dpp_row_shl(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 | SH, 0xF, 0xF, false);
}

// Lane tree for groups inside one DPP row: at level LV lane g folds lane g + 2^LV's block,
// v = v * x^(128*2^LV) ^ v[g + 2^LV]. Lane 0 of the group only ever combines lanes of its own
// group (g + 2^LV < G on every path that reaches it), so the result is valid in lane 0.
template <int LV, int LEVELS>
__device__ __forceinline__ uint32_t lane_tree_dpp(const uint32_t* lds, uint32_t x32_off, uint32_t v) {
    if constexpr (LV == LEVELS) {
        return v;
    } else {
        const uint32_t other = dpp_row_shl<(1 << LV)>(v);
        // (every lane multiplies: masking the lanes whose result is unused measured no different)
        v = mul_aux_add(lds, x32_off + 4096u * (uint32_t)(1 + LV), v, other);
        return lane_tree_dpp<LV + 1, LEVELS>(lds, x32_off, v);
    }
}

// Raw register of a group from each lane's four dword-stream accumulators (valid in lane 0).
// Fast path (G <= 16): the final "dword -> register" x^32 is folded into the in-lane products
// (x^128 = the level-0 tree operator, x^96, x^64, x^32: four independent products, one LDS round
// trip), then the lane tree via DPP row_shl; the operators commute, so scaling every lane by x^32
// before the tree equals scaling the tree's result. Wide groups: serial in-lane Horner, a
// __shfl_xor tree, and the final x^32.
template <int G>
__device__ __forceinline__ uint32_t finish_lanes(const uint32_t* lds, uint32_t c0, uint32_t c1, uint32_t c2,
                                                 uint32_t c3) {
    using Gm = Geo<G>;
    if constexpr (G == 1) {
        // one lane per entry: x^128 is the main operator itself (replicated, conflict-free); no tree
        const uint32_t lanereg = ((uint32_t)(threadIdx.x & 31) << 2) | (1u << 16);
        return mul_main_add(lds, c0, lanereg,
                            mul_aux_add(lds, Gm::kX96Off, c1, mul_aux_add(lds, Gm::kX64Off, c2, mul_aux(lds, Gm::kX32Off, c3))));
    } else if constexpr (Gm::kLaneTab) {
#if BKD_FINISH_PROBE
        return c0 ^ c1 ^ c2 ^ c3;  // measurement-only build: the finish's cost (wrong digests)
#endif
        // one more product per lane, by its weight x^(128 (G-1-g)) in the group's register (eight
        // nibble lookups, independent), then an XOR over the group's lanes by DPP: one dependent
        // LDS round trip instead of log2(G)
        const uint32_t v = xor3(mul_aux(lds, Gm::kX32Off + 4096u, c0), mul_aux(lds, Gm::kX96Off, c1),
                                mul_aux_add(lds, Gm::kX64Off, c2, mul_aux(lds, Gm::kX32Off, c3)));
        const uint32_t lb = Gm::kLaneOff + 4u * (uint32_t)(threadIdx.x & (G - 1));
        auto nib = [&](int k) { return lds_word(lds, lb + 64u * G * (uint32_t)k + ((v >> (4 * k)) & 15u) * (4u * G)); };
        uint32_t r = xor3(xor3(nib(0), nib(1), nib(2)), xor3(nib(3), nib(4), nib(5)), nib(6) ^ nib(7));
        r ^= dpp_row_shl<1>(r);
        r ^= dpp_row_shl<2>(r);
        if constexpr (G == 8) r ^= dpp_row_shl<4>(r);
        return r;
    } else if constexpr (Gm::kFast) {
        const uint32_t v = xor3(mul_aux(lds, Gm::kX32Off + 4096u, c0), mul_aux(lds, Gm::kX96Off, c1),
                                mul_aux_add(lds, Gm::kX64Off, c2, mul_aux(lds, Gm::kX32Off, c3)));
        return lane_tree_dpp<0, Gm::kLevels>(lds, Gm::kX32Off, v);
    } else {
        uint32_t v = mul_aux_add(lds, Gm::kX32Off, c0, c1);
        v = mul_aux_add(lds, Gm::kX32Off, v, c2);
        v = mul_aux_add(lds, Gm::kX32Off, v, c3);
#pragma unroll
        for (int lv = 0; lv < Gm::kLevels; ++lv) {
            const uint32_t other = (uint32_t)__shfl_xor((int)v, 1 << lv);
            v = mul_aux_add(lds, Gm::kX32Off + 4096u * (uint32_t)(1 + lv), v, other);
        }
        return mul_aux(lds, Gm::kX32Off, v);
    }
}

// Zero the low d bytes (1..15) of a 16-byte little-endian vector.
__device__ __forceinline__ u32x4 mask_low_bytes(u32x4 w, uint32_t d) {
    auto m = [](uint32_t x, int32_t k) -> uint32_t {  // k = bytes of this dword to clear
        return k >= 4 ? 0u : (k <= 0 ? x : x & (0xFFFFFFFFu << (8 * k)));
    };
    w.x = m(w.x, (int32_t)d);
    w.y = m(w.y, (int32_t)d - 4);
    w.z = m(w.z, (int32_t)d - 8);
    w.w = m(w.w, (int32_t)d - 12);
    return w;
}

// Stage the operator tables: the main operator replicated per bank, the rest compact.
template <int G>
__device__ __forceinline__ void stage_tables(uint32_t* lds, const uint32_t* __restrict__ tables) {
    for (int idx = threadIdx.x; idx < 4 * 256 * 8; idx += kBlock) {
        const int q = idx & 7, b = (idx >> 3) & 255, t = idx >> 11;
        const uint32_t v = tables[t * 256 + b];
        const uint32_t addr = (uint32_t)(t >> 1) * 65536u + (uint32_t)b * 256u + (uint32_t)(t & 1) * 128u +
                              (uint32_t)q * 16u;
        *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(lds) + addr) = u32x4{v, v, v, v};
    }
    for (int idx = threadIdx.x; idx < Geo<G>::kAuxWords; idx += kBlock) lds[kMainBytes / 4 + idx] = tables[1024 + idx];
    __syncthreads();
}

// Raw CRC register of base[s, e) (e - s >= 16 unless ALIGNED), with the register r0 folded into
// its first 4 bytes, computed by the G lanes of one group; the result is valid in lane g == 0.
// ALIGNED: `e` is 16-byte aligned in device memory, so every lane address is aligned; the lane
// straddling s loads its aligned block and clears the bytes before s (any e - s >= 1 works).
// Otherwise the straddling lane loads 16 bytes at s (needs e - s >= 16) and shifts them up.
// TAILU: unconditional tail loads (see below); taken for uniform batches of >= kTailUncondSteps
// steps, where it measured −0.6 % (1M x 4 KiB, same-process A/B in both library orders,
// profiles/r03f_ab_variants_order*.log); indexed and framed batches did not gain (package +1.5 %),
// and short uniform entries lost (512 B +13 %, 1 KiB +2.7 %: most of their loads are tail loads,
// profiles/r03g_ab_order*.log)
// B16: each fold step through fold4_main (16 lookups in flight) instead of mul_main_add.
// R0: the register folded into the range's first bytes — a plain value, or (LateSeed) a callable
// evaluated only after the range's first PF + 1 loads are issued, so a chain computing it (the fused
// package kernel's header CRC) overlaps those loads instead of delaying them.
template <class F>
struct LateSeed {
    F f;
};
__device__ __forceinline__ uint32_t seed_value(uint32_t r0) { return r0; }
template <class F>
__device__ __forceinline__ uint32_t seed_value(const LateSeed<F>& r0) { return r0.f(); }
template <class R0>
struct IsLateSeed : std::false_type {};
template <class F>
struct IsLateSeed<LateSeed<F>> : std::true_type {};

template <int G, int PF, bool NT, bool ALIGNED, bool TAILU = BKD_TAIL_UNCOND != 0, bool B16 = false, class R0 = uint32_t>
__device__ __forceinline__ uint32_t fold_range(const uint32_t* lds, uint32_t lanereg, int g,
                                               const uint8_t* __restrict__ base, int64_t s, int64_t e, R0 r0src) {
    using Gm = Geo<G>;
    constexpr bool kLate = IsLateSeed<R0>::value;
    const uint32_t J = (uint32_t)((e - s + Gm::kStep - 1) / Gm::kStep);
    const int64_t a = e - (int64_t)J * Gm::kStep + 16 * g;

    // Step 0: masked head + seed fold.
    u32x4 w;
    if (a >= s) {
        w = ld16<NT>(base + a);
    } else if (a + 16 > s) {
        if constexpr (ALIGNED) w = mask_low_bytes(ld16<NT>(base + a), (uint32_t)(s - a));
        else w = shl_bytes(ld16<NT>(base + s), (uint32_t)(s - a));
    } else {
        w = u32x4{0u, 0u, 0u, 0u};
    }
    // When the range starts in the last 3 bytes of step 0's window, the tail of the seed
    // image spills into dword 0 of lane 0 at step 1; fx carries it into that first fold.
    uint32_t fx = 0u;
    auto seed_in = [&](uint32_t r0) {
        if (a < s + 4 && a + 16 > s) {
            const int64_t d = s - a;
            w.x ^= place_seed(r0, d);
            w.y ^= place_seed(r0, d - 4);
            w.z ^= place_seed(r0, d - 8);
            w.w ^= place_seed(r0, d - 12);
        }
        if (a + Gm::kStep < s + 4) fx = place_seed(r0, s - (a + Gm::kStep));
    };
    if constexpr (!kLate) seed_in(seed_value(r0src));
    uint32_t c0 = w.x, c1 = w.y, c2 = w.z, c3 = w.w;

    // Steps 1..J-1 with PF loads in flight per lane. The steady-state loop issues its loads
    // unconditionally (a conditional load would merge registers and force an early vmcnt(0)).
    const uint8_t* p = base + a + Gm::kStep;
    const uint32_t rem = J - 1u;
#define BKD_FOLD0(d)                                                                  \
    do {                                                                              \
        if constexpr (B16) {                                                          \
            fold4_main(c0, c1, c2, c3, lanereg, (d).x ^ fx, (d).y, (d).z, (d).w);     \
        } else {                                                                      \
            c0 = mul_main_add(lds, c0, lanereg, (d).x ^ fx);                          \
            c1 = mul_main_add(lds, c1, lanereg, (d).y);                               \
            c2 = mul_main_add(lds, c2, lanereg, (d).z);                               \
            c3 = mul_main_add(lds, c3, lanereg, (d).w);                               \
        }                                                                             \
        fx = 0u;                                                                      \
    } while (0)
#define BKD_FOLD(d)                                                                   \
    do {                                                                              \
        if constexpr (B16) {                                                          \
            fold4_main(c0, c1, c2, c3, lanereg, (d).x, (d).y, (d).z, (d).w);          \
        } else {                                                                      \
            c0 = mul_main_add(lds, c0, lanereg, (d).x);                               \
            c1 = mul_main_add(lds, c1, lanereg, (d).y);                               \
            c2 = mul_main_add(lds, c2, lanereg, (d).z);                               \
            c3 = mul_main_add(lds, c3, lanereg, (d).w);                               \
        }                                                                             \
    } while (0)
    if (rem >= (uint32_t)PF) {
        // A/B register double buffer: fold one block while the other block's loads fly.
        u32x4 A[PF], B[PF];
#pragma unroll
        for (int k = 0; k < PF; ++k) A[k] = ld16<NT>(p + (int64_t)k * Gm::kStep);
        if constexpr (kLate) {  // the seed's chain runs while these loads are in flight
            seed_in(seed_value(r0src));
            c0 = w.x, c1 = w.y, c2 = w.z, c3 = w.w;
        }
        p += (int64_t)PF * Gm::kStep;  // p = first step not yet loaded
        uint32_t left = rem - (uint32_t)PF;
        while (left >= 2u * PF) {
#pragma unroll
            for (int k = 0; k < PF; ++k) B[k] = ld16<NT>(p + (int64_t)k * Gm::kStep);
            BKD_FOLD0(A[0]);
#pragma unroll
            for (int k = 1; k < PF; ++k) BKD_FOLD(A[k]);
#pragma unroll
            for (int k = 0; k < PF; ++k) A[k] = ld16<NT>(p + (int64_t)(PF + k) * Gm::kStep);
#pragma unroll
            for (int k = 0; k < PF; ++k) BKD_FOLD(B[k]);
            p += (int64_t)(2 * PF) * Gm::kStep;
            left -= 2u * PF;
        }
        // Tail: A holds PF loaded steps; `left` (< 2PF) steps remain unloaded.
        if constexpr (TAILU) {
            // every tail load is issued (a step past the range reloads the range's last loaded step):
            // the load count does not depend on `left`
#pragma unroll
            for (int k = 0; k < PF; ++k)
                B[k] = ld16<NT>(p + (int64_t)std::min<int32_t>(k, (int32_t)left - 1) * Gm::kStep);
            asm volatile("" ::: "memory");  // keeps the loads here: not sunk into the conditional folds
        } else {
#pragma unroll
            for (int k = 0; k < PF; ++k)
                if ((uint32_t)k < left) B[k] = ld16<NT>(p + (int64_t)k * Gm::kStep);
        }
        BKD_FOLD0(A[0]);
#pragma unroll
        for (int k = 1; k < PF; ++k) BKD_FOLD(A[k]);
        if constexpr (TAILU) {
#pragma unroll
            for (int k = 0; k < PF; ++k)
                A[k] = ld16<NT>(p + (int64_t)std::min<int32_t>(PF + k, (int32_t)left - 1) * Gm::kStep);
            asm volatile("" ::: "memory");
        } else {
#pragma unroll
            for (int k = 0; k < PF; ++k)
                if ((uint32_t)(PF + k) < left) A[k] = ld16<NT>(p + (int64_t)(PF + k) * Gm::kStep);
        }
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if ((uint32_t)k < left) BKD_FOLD(B[k]);
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if ((uint32_t)(PF + k) < left) BKD_FOLD(A[k]);
    } else {
        if constexpr (kLate) {
            seed_in(seed_value(r0src));
            c0 = w.x, c1 = w.y, c2 = w.z, c3 = w.w;
        }
        for (uint32_t k = 0; k < rem; ++k) {
            const u32x4 d = ld16<NT>(p + (int64_t)k * Gm::kStep);
            BKD_FOLD0(d);
        }
    }
#undef BKD_FOLD
#undef BKD_FOLD0

    return finish_lanes<G>(lds, c0, c1, c2, c3);
}

// Grid-stride loop of the one-entry-per-group kernels: work items gid, gid + ngroups, ... of `src`.
// low_clock: fold each entry through fold4_main (crc_groups_kernel measured a power-limited clock).
template <int G, int PF, bool NT, class Src>
__device__ __forceinline__ void groups_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                            const uint8_t* __restrict__ base, const Src& src, uint64_t n,
                                            uint64_t gid, uint64_t ngroups, uint32_t* __restrict__ err,
                                            bool low_clock = false) {
    using Gm = Geo<G>;
    for (uint64_t i = gid; i < n; i += ngroups) {
        Work wk;
        const int st = src.get(i, wk);
        if (st != 0) {
            if (g == 0 && st != 3) {
                put_result(src, i, wk, 0u);
                if (st == 2 && err) atomicOr(err, 1u);
            }
            continue;
        }
        if (wk.len < 16u) {  // tiny range: serial byte loop (ReflectedIntCrc.java:44-48 form)
            if (g == 0) {
                uint32_t r = wk.r0;
                const uint8_t* q = base + wk.s;
                for (uint32_t k = 0; k < wk.len; ++k)
                    r = lds_word(lds, Gm::kByteTabOff + (((r ^ q[k]) & 0xffu) << 2)) ^ (r >> 8);
                put_result(src, i, wk, r ^ wk.xorout);
            }
            continue;
        }
        constexpr bool kTailU = BKD_TAIL_UNCOND != 0 || std::is_same<Src, UniformLongSrc>::value;
        const uint32_t v =
            low_clock ? fold_range<G, PF, NT, false, kTailU, true>(lds, lanereg, g, base, wk.s, wk.s + (int64_t)wk.len, wk.r0)
                      : fold_range<G, PF, NT, false, kTailU, false>(lds, lanereg, g, base, wk.s, wk.s + (int64_t)wk.len, wk.r0);
        if (g == 0) put_result(src, i, wk, v ^ wk.xorout);
    }
}

// Held result stores. A result store inside the load stream costs in proportion to the bytes it
// writes, whatever its grouping or place: a uniform-kernel build without result stores ran 2.5–2.9 %
// faster, one storing a round in eight 1.8–2.5 % faster, while coalescing each wave's words into one
// 256-byte store, storing one entry late or nontemporal stores gained nothing (profiles/r06ac_ag_*).
// So a group's result of round r (item gid + r·ngroups) moves to lane r mod G of the group
// (ds_bpermute from the group's lane 0) and stays in a register until K·G rounds are held; then
// every lane stores its K words at once, and the rest when the group's loop ends.
#ifndef BKD_HOLD_STORE
#define BKD_HOLD_STORE 8  // K: words held per lane (0: each round stores its result)
#endif

#ifndef BKD_HOLD_LONGLOOP
#define BKD_HOLD_LONGLOOP 8  // the chunk kernel's long loop: 64 rounds per flush (config 3: ~60), 128 VGPRs
#endif
#ifndef BKD_SHORT_FIRST
#define BKD_SHORT_FIRST 1  // Zipf -0.5 %, its < 1 KiB bucket alone +0.7 to +1.1 % (profiles/r06bm_bn_*)
#endif
#ifndef BKD_HOLD_SHORT
#define BKD_HOLD_SHORT 2  // the chunk kernel's short tail: K·G = 16 rounds per group (config 3: ~15)
#endif
constexpr int kHoldLong = 32;  // words held per lane in the uniform kernel for batches of > 8·G rounds

template <int G, int K>
struct HeldResults {
    uint32_t hold[K];
    uint32_t cur = 0u;   // the slot being filled: lane g takes round r0 + k·G + g
    uint64_t r0 = 0;     // first round held
    int k = 0, sub = 0;  // slot and lane of the next round (the same in every lane of the group)
    __device__ __forceinline__ HeldResults() {
#pragma unroll
        for (int q = 0; q < K; ++q) hold[q] = 0u;
    }
    // slots q < kfull from hold[], then slot kfull from cur when `partial`
    __device__ __forceinline__ void flush(int kfull, bool partial, int g, uint32_t* __restrict__ out, uint64_t gid,
                                          uint64_t ngroups, uint64_t n) const {
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint64_t i = gid + (r0 + (uint64_t)q * G + (uint64_t)g) * ngroups;
            if (q < kfull && i < n) out[i] = hold[q];
        }
        const uint64_t i = gid + (r0 + (uint64_t)kfull * G + (uint64_t)g) * ngroups;
        if (partial && i < n) out[i] = cur;
    }
    // v: this round's result, valid in the group's lane 0 (every lane of the group calls). One select
    // per round; the slot is filed into hold[] (a chain of K selects: the index is not static) once
    // every G rounds.
    __device__ __forceinline__ void put(uint32_t v, int g, uint32_t* __restrict__ out, uint64_t gid, uint64_t ngroups,
                                        uint64_t n) {
        const int from = ((int)(threadIdx.x & 63) & ~(G - 1)) << 2;
        const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)v);
        cur = g == sub ? b : cur;
        if (++sub == G) {
            sub = 0;
#pragma unroll
            for (int q = 0; q < K; ++q) hold[q] = q == k ? cur : hold[q];  // selects: no indexed (scratch) array
            if (++k == K) {
                flush(K, false, g, out, gid, ngroups, n);
                r0 += (uint64_t)K * G;
                k = 0;
            }
        }
    }
    // after the group's last round: slots below k are full, `cur` holds lanes 0 .. sub-1 of slot k
    // (the lanes past them hold rounds at or after the one that ended the loop: items >= n, not stored)
    __device__ __forceinline__ void finish(int g, uint32_t* __restrict__ out, uint64_t gid, uint64_t ngroups,
                                           uint64_t n) const {
        flush(k, sub > 0, g, out, gid, ngroups, n);
    }
};

// Uniform entries (>= 16 B: no serial or out-of-range items) with held stores; TAILU as the kernel
// would fold them (unconditional tail loads for UniformLongSrc's 32 steps or more).
template <int G, int PF, bool NT, int K, bool TAILU = true>
__device__ __forceinline__ void held_store_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                                const uint8_t* __restrict__ base, const UniformSrc& src, uint64_t n,
                                                uint64_t gid, uint64_t ngroups, bool low_clock) {
    HeldResults<G, K> held;
    for (uint64_t i = gid; i < n; i += ngroups) {
        Work wk;
        src.get(i, wk);
        const uint32_t v =
            low_clock ? fold_range<G, PF, NT, false, TAILU, true>(lds, lanereg, g, base, wk.s, wk.s + (int64_t)wk.len, wk.r0)
                      : fold_range<G, PF, NT, false, TAILU, false>(lds, lanereg, g, base, wk.s, wk.s + (int64_t)wk.len, wk.r0);
        held.put(v ^ wk.xorout, g, src.out, gid, ngroups, n);
    }
    held.finish(g, src.out, gid, ngroups, n);
}

// Every work item of `src` written (no item left to another launch: PlanDirectSrc with `all`), results
// held (HeldResults): out-of-range items 0 (and the bounds flag), items under 16 bytes serially.
#ifndef BKD_HOLD_DIRECT
#define BKD_HOLD_DIRECT 4  // the chunk kernel's near-uniform direct loop (32 rounds per flush)
#endif
template <int G, int PF, bool NT, int K, class Src>
__device__ __forceinline__ void held_direct_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                                 const uint8_t* __restrict__ base, const Src& src, uint64_t n,
                                                 uint64_t gid, uint64_t ngroups, uint32_t* __restrict__ err) {
    using Gm = Geo<G>;
    HeldResults<G, K> held;
    for (uint64_t i = gid; i < n; i += ngroups) {
        Work wk;
        const int st = src.get(i, wk);
        uint32_t v = 0u;
        if (st == 2) {
            if (g == 0 && err) atomicOr(err, 1u);
        } else if (wk.len < 16u) {  // tiny range: serial byte loop (ReflectedIntCrc.java:44-48 form)
            uint32_t r = wk.r0;
            const uint8_t* q = base + wk.s;
            for (uint32_t k = 0; k < wk.len; ++k)
                r = lds_word(lds, Gm::kByteTabOff + (((r ^ q[k]) & 0xffu) << 2)) ^ (r >> 8);
            v = r ^ wk.xorout;
        } else {
            v = fold_range<G, PF, NT, false, BKD_TAIL_UNCOND != 0, false>(lds, lanereg, g, base, wk.s,
                                                                         wk.s + (int64_t)wk.len, wk.r0) ^ wk.xorout;
        }
        held.put(v, g, src.out, gid, ngroups, n);
    }
    held.finish(g, src.out, gid, ngroups, n);
}

// Uniform batches of short entries (16 B <= len <= 16*G*(PF+1), every load of an entry fits one
// register set): a group's next entry is loaded while the current one folds (X/Y register sets),
// so a wave no longer waits one HBM round trip per entry — the one-entry-per-group loop is
// latency-bound there (its rate falls in proportion to G at 64 B: profiles/r01_size_sweep.log).
struct SmallGeo {
    int64_t s, a, la0;  // entry start, this lane's step-0 block, its load address (>= s, in bounds)
    uint32_t J;
    uint32_t r0;
    uint32_t len;
    int kind;  // indexed entries: 0 fold, 1 shorter than 16 B (serial), 2 out of bounds, 3 the plan's, 4 none
};

// SEEDS: per-entry seeds (src.seeds != nullptr); without, no load sits under a branch in the loop
template <int G, bool SEEDS = true>
__device__ __forceinline__ SmallGeo small_geo(const UniformSrc& src, uint64_t i, int g) {
    SmallGeo c;
    c.s = (int64_t)(i * src.stride);
    c.J = (src.len + (uint32_t)Geo<G>::kStep - 1u) / (uint32_t)Geo<G>::kStep;
    c.a = c.s + (int64_t)src.len - (int64_t)c.J * Geo<G>::kStep + 16 * g;
    c.la0 = c.a >= c.s ? c.a : c.s;  // the straddling lane loads at s and shifts; lanes before s reload s
    if constexpr (SEEDS) c.r0 = ~src.seeds[i];
    else c.r0 = ~src.seed_all;
    return c;
}

// One entry's index words, loaded three entries before its data (no dependent index -> data
// chain). Every load is unconditional: an index past the batch rereads entry n - 1's words and is
// marked past; SEEDS (per-entry seeds) is a template choice, not a branch around a load.
struct SmallIdx {
    uint64_t o;
    uint32_t l;
    uint32_t seed;
};

template <bool SEEDS>
__device__ __forceinline__ SmallIdx small_idx(const SmallIndexedSrc& src, uint64_t i) {
    const uint64_t j = i < src.n ? i : src.n - 1u;
    SmallIdx x;
    x.o = src.offsets[j];
    x.l = src.lengths[j];
    if constexpr (SEEDS) x.seed = src.seeds[j];
    else x.seed = src.seed_all;
    if (i >= src.n) {
        x.o = ~0ull;  // past the batch
        x.l = 0xFFFFFFFFu;
    }
    return x;
}

template <int G>
__device__ __forceinline__ SmallGeo small_geo(const SmallIndexedSrc& src, const SmallIdx& x, int g) {
    SmallGeo c;
    c.len = x.l;
    c.kind = 3;
    c.s = c.a = c.la0 = 0;  // entries not folded here load base[0, 16) (the plan runs only on >= 256 KiB bases)
    c.J = 1;
    c.r0 = 0u;
    if (x.o == ~0ull) {
        c.kind = 4;  // past the batch
    } else if (c.len <= src.small) {
        const uint64_t o = x.o;
        if (o > src.size || (uint64_t)c.len > src.size - o) {
            c.kind = 2;
        } else {
            c.r0 = ~x.seed;
            if (c.len < 16u) {  // folded serially from its one or two 16-byte blocks (la0, then a)
                c.kind = 1;
                c.s = (int64_t)o;
                c.la0 = c.s & ~(int64_t)15;
                c.a = (c.s & 15) + (int64_t)c.len > 16 ? c.la0 + 16 : 0;
            } else {
                c.kind = 0;
                c.s = (int64_t)o;
                c.J = (c.len + (uint32_t)Geo<G>::kStep - 1u) / (uint32_t)Geo<G>::kStep;
                c.a = c.s + (int64_t)c.len - (int64_t)c.J * Geo<G>::kStep + 16 * g;
                c.la0 = c.a >= c.s ? c.a : c.s;
            }
        }
    }
    return c;
}

template <int G, int PF, bool NT>
__device__ __forceinline__ void small_load(const uint8_t* __restrict__ base, const SmallGeo& c, u32x4& W0,
                                           u32x4 (&A)[PF]) {
    W0 = ld16<NT>(base + c.la0);
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const int64_t addr = (uint32_t)(k + 1) < c.J ? c.a + (int64_t)(k + 1) * Geo<G>::kStep : c.la0;
        A[k] = ld16<NT>(base + addr);
    }
}

// small_load for the indexed class: every load is issued, so the compiler can count them, and a
// block the entry does not need (steps past J, entries of other kinds) reads base[0, 16) — the same
// line for every such lane of a wave, one request.
template <int G, int PF, bool NT>
__device__ __forceinline__ void small_load_idx(const uint8_t* __restrict__ base, const SmallGeo& c, u32x4& W0,
                                               u32x4 (&A)[PF]) {
    W0 = ld16<NT>(base + (c.kind <= 1 ? c.la0 : 0));
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        int64_t addr = 0;
        if (c.kind == 0 && (uint32_t)(k + 1) < c.J) addr = c.a + (int64_t)(k + 1) * Geo<G>::kStep;
        else if (c.kind == 1 && k == 0) addr = c.a;  // the second block of an entry < 16 B, or base[0, 16)
        A[k] = ld16<NT>(base + addr);
    }
}

// Raw register of a short entry from its loaded blocks (fold_range's arithmetic, J <= PF + 1).
template <int G, int PF>
__device__ __forceinline__ uint32_t small_fold(const uint32_t* lds, uint32_t lanereg, const SmallGeo& c, u32x4 W0,
                                               const u32x4 (&A)[PF]) {
    using Gm = Geo<G>;
    const int64_t s = c.s, a = c.a;
    u32x4 w;
    if (a >= s) w = W0;
    else if (a + 16 > s) w = shl_bytes(W0, (uint32_t)(s - a));
    else w = u32x4{0u, 0u, 0u, 0u};
    const uint32_t r0 = c.r0;
    if (a < s + 4 && a + 16 > s) {
        const int64_t d = s - a;
        w.x ^= place_seed(r0, d);
        w.y ^= place_seed(r0, d - 4);
        w.z ^= place_seed(r0, d - 8);
        w.w ^= place_seed(r0, d - 12);
    }
    uint32_t fx = 0u;
    if (a + Gm::kStep < s + 4) fx = place_seed(r0, s - (a + Gm::kStep));
    uint32_t c0 = w.x, c1 = w.y, c2 = w.z, c3 = w.w;
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        if ((uint32_t)(k + 1) < c.J) {
            c0 = mul_main_add(lds, c0, lanereg, A[k].x ^ (k == 0 ? fx : 0u));
            c1 = mul_main_add(lds, c1, lanereg, A[k].y);
            c2 = mul_main_add(lds, c2, lanereg, A[k].z);
            c3 = mul_main_add(lds, c3, lanereg, A[k].w);
        }
    }
    return finish_lanes<G>(lds, c0, c1, c2, c3);
}

template <int G, int PF, bool NT, bool SEEDS>
__device__ __forceinline__ void uniform_small_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                                   const uint8_t* __restrict__ base, const UniformSrc& src, uint64_t n,
                                                   uint64_t gid, uint64_t ngroups) {
    // three register sets rotate: an entry's blocks are requested three entries before its fold.
    // Loads are unconditional (a group past the batch reloads entry n - 1 and stores nothing) and
    // the exit is wave-uniform: loads under a divergent branch leave the compiler's waits
    // uncountable, and it then drains every load in flight (vmcnt(0)) before each fold.
    auto geo = [&](uint64_t j) { return small_geo<G, SEEDS>(src, j < n ? j : n - 1, g); };
    u32x4 W0x, Ax[PF], W0y, Ay[PF], W0z, Az[PF];
    SmallGeo cx = geo(gid), cy = geo(gid + ngroups), cz = geo(gid + 2 * ngroups);
    small_load<G, PF, NT>(base, cx, W0x, Ax);
    small_load<G, PF, NT>(base, cy, W0y, Ay);
    small_load<G, PF, NT>(base, cz, W0z, Az);
    uint64_t i = gid;
#define BKD_USMALL_STEP(C, W0C, AC)                                          \
    {                                                                       \
        const uint32_t v = small_fold<G, PF>(lds, lanereg, C, W0C, AC);     \
        if (g == 0 && i < n) src.out[i] = ~v;                               \
        C = geo(i + 3 * ngroups);                                           \
        small_load<G, PF, NT>(base, C, W0C, AC);                            \
        i += ngroups;                                                       \
        if (!__any(i < n)) break;                                           \
    }
    for (;;) {
        BKD_USMALL_STEP(cx, W0x, Ax)
        BKD_USMALL_STEP(cy, W0y, Ay)
        BKD_USMALL_STEP(cz, W0z, Az)
    }
#undef BKD_USMALL_STEP
}

// Byte p (0..15) of a 16-byte little-endian block.
__device__ __forceinline__ uint32_t block_byte(const u32x4& v, uint32_t p) {
    const uint32_t d = p < 4u ? v.x : p < 8u ? v.y : p < 12u ? v.z : v.w;
    return (d >> (8u * (p & 3u))) & 0xffu;
}

// One short-class entry of a group (kind 0 folds, 1 serial bytes, 2 bounds error, else nothing).
template <int G, int PF>
__device__ __forceinline__ void small_entry_finish(const uint32_t* lds, uint32_t lanereg, int g,
                                                   const SmallIndexedSrc& src, const SmallGeo& c, uint64_t i,
                                                   const u32x4& W0, const u32x4 (&A)[PF], uint32_t* __restrict__ err) {
    using Gm = Geo<G>;
    if (c.kind == 0) {
        const uint32_t v = small_fold<G, PF>(lds, lanereg, c, W0, A);
        if (g == 0) src.out[i] = ~v;
    } else if (c.kind == 1) {  // < 16 B: byte-at-a-time from its loaded blocks (ReflectedIntCrc.java:44-48 form)
        if (g == 0) {
            uint32_t r = c.r0;
            const uint32_t off = (uint32_t)(c.s & 15);
            for (uint32_t k = 0; k < c.len; ++k) {
                const uint32_t p = off + k;
                const uint32_t b = p < 16u ? block_byte(W0, p) : block_byte(A[0], p - 16u);
                r = lds_word(lds, Gm::kByteTabOff + (((r ^ b) & 0xffu) << 2)) ^ (r >> 8);
            }
            src.out[i] = ~r;
        }
    } else if (c.kind == 2) {
        if (g == 0) {
            src.out[i] = 0u;
            if (err) atomicOr(err, 1u);
        }
    }
}

// The short-entry class of an indexed batch (SmallIndexedSrc). Three register sets rotate, as in
// uniform_small_loop: an entry's blocks are requested three entries before it is folded and its
// index words three entries before that. Every load is unconditional and the exit wave-uniform
// (a group past the batch walks "past" entries until its wave is done), so the compiler's waits
// count the loads in flight instead of draining them at every entry.
// Returns whether this lane met an entry of the plan's (kind 3).
template <int G, int PF, bool NT, bool SEEDS>
__device__ __forceinline__ bool indexed_small_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                                   const uint8_t* __restrict__ base, const SmallIndexedSrc& src,
                                                   uint64_t n, uint64_t gid, uint64_t ngroups,
                                                   uint32_t* __restrict__ err) {
    bool saw_plan = false;
    auto geo = [&](const SmallIdx& x) { return small_geo<G>(src, x, g); };
    u32x4 W0x, Ax[PF], W0y, Ay[PF], W0z, Az[PF];
    SmallGeo cx = geo(small_idx<SEEDS>(src, gid)), cy = geo(small_idx<SEEDS>(src, gid + ngroups)),
             cz = geo(small_idx<SEEDS>(src, gid + 2 * ngroups));
    small_load_idx<G, PF, NT>(base, cx, W0x, Ax);
    small_load_idx<G, PF, NT>(base, cy, W0y, Ay);
    small_load_idx<G, PF, NT>(base, cz, W0z, Az);
    SmallIdx ix = small_idx<SEEDS>(src, gid + 3 * ngroups), iy = small_idx<SEEDS>(src, gid + 4 * ngroups),
             iz = small_idx<SEEDS>(src, gid + 5 * ngroups);
    uint64_t i = gid;
#define BKD_ISMALL_STEP(C, W0C, AC, IC)                                                \
    {                                                                                 \
        saw_plan |= C.kind == 3;                                                      \
        small_entry_finish<G, PF>(lds, lanereg, g, src, C, i, W0C, AC, err);          \
        C = geo(IC); /* entry i + 3 ngroups */                                        \
        small_load_idx<G, PF, NT>(base, C, W0C, AC);                                  \
        IC = small_idx<SEEDS>(src, i + 6 * ngroups);                                  \
        i += ngroups;                                                                 \
        if (!__any(i < n)) break;                                                     \
    }
    for (;;) {
        BKD_ISMALL_STEP(cx, W0x, Ax, ix)
        BKD_ISMALL_STEP(cy, W0y, Ay, iy)
        BKD_ISMALL_STEP(cz, W0z, Az, iz)
    }
#undef BKD_ISMALL_STEP
    return saw_plan;
}

// One CRC per work item of `src` (uniform / indexed / framed-payload entries), persistent grid.
template <int G, int PF, bool NT, class Src>
// sched: 0 chosen from the measured clock, 1 mul_main_add, 2 fold4_main (bkd_set_fold_schedule)
__global__ void __launch_bounds__(kBlock) crc_groups_kernel(const uint8_t* __restrict__ base, Src src,
                                                            const uint32_t* __restrict__ tables,
                                                            uint32_t* __restrict__ err, int sched) {
    using Gm = Geo<G>;
    __shared__ __attribute__((aligned(16))) uint32_t lds[Gm::kLdsWords];
    const uint64_t n = src.count();
    if (n == 0) return;
    // the shader clock over the table staging (shader cycles against the 100 MHz real-time counter,
    // both scalar reads): below kLowClockMHz the one-entry-per-group fold takes fold4_main
    const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    stage_tables<G>(lds, tables);
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    const bool low_clock = lds_image_at_zero(lds) &&
                           (sched == 2 || (sched == 0 && BKD_CLOCK_ADAPT &&
                                           (clk1 - clk0) * 100u < (rt1 - rt0) * (uint64_t)kLowClockMHz));

    const int lane = threadIdx.x & 63;
    const int g = lane & (G - 1);
    const uint32_t lanereg = ((uint32_t)(lane & 31) << 2) | (1u << 16);
    const uint64_t ngroups = (uint64_t)gridDim.x * (kBlock / G);
    const uint64_t gid = (uint64_t)blockIdx.x * (kBlock / G) + (uint64_t)(threadIdx.x / G);
    if constexpr (std::is_same<Src, UniformSrc>::value) {
        if (src.len >= 16u && src.len <= (uint32_t)Gm::kStep * (uint32_t)(PF + 1)) {
            if (gid < n) {
                if (src.seeds) uniform_small_loop<G, PF, NT, true>(lds, lanereg, g, base, src, n, gid, ngroups);
                else uniform_small_loop<G, PF, NT, false>(lds, lanereg, g, base, src, n, gid, ngroups);
            }
            return;
        }
        // entries past the short loop and below UniformLongSrc's 32 steps, results held as there:
        // 512 B -11 %, 1 KiB -7 %, 2 KiB -6 % (8-lane groups; profiles/r06aw_ax_*). (Held in the
        // short loop itself they cost 2-5 %: its entries are a few folds each.)
        if (BKD_HOLD_STORE > 0 && src.len >= 16u) {
            if (gid < n) {
                if ((n + ngroups - 1) / ngroups <= (uint64_t)BKD_HOLD_STORE * G)
                    held_store_loop<G, PF, NT, BKD_HOLD_STORE, BKD_TAIL_UNCOND != 0>(lds, lanereg, g, base, src, n, gid, ngroups, low_clock);
                else
                    held_store_loop<G, PF, NT, kHoldLong, BKD_TAIL_UNCOND != 0>(lds, lanereg, g, base, src, n, gid, ngroups, low_clock);
            }
            return;
        }
    }
    if constexpr (std::is_same<Src, SmallIndexedSrc>::value) {
        bool saw = false;
        if (gid < n) {
            if (src.seeds) saw = indexed_small_loop<G, PF, NT, true>(lds, lanereg, g, base, src, n, gid, ngroups, err);
            else saw = indexed_small_loop<G, PF, NT, false>(lds, lanereg, g, base, src, n, gid, ngroups, err);
        }
        if (__any(saw) && (threadIdx.x & 63) == 0 && src.plan_flag) *src.plan_flag = src.plan_epoch;
    } else if constexpr (std::is_same<Src, UniformLongSrc>::value && BKD_HOLD_STORE > 0) {
        // (long uniform entries >= 16 B: no serial or out-of-range items)
        // K = 8 holds a group's 64 rounds (1M entries at 32 768 groups: 32); larger batches hold 32
        // words per lane so that they too store only at the end (8M: 256 rounds, -1.5 %; K = 32 for
        // 1M entries measured +0.3 to +0.8 %, profiles/r06aq_*, r06ar_*)
        if (gid < n) {
            if ((n + ngroups - 1) / ngroups <= (uint64_t)BKD_HOLD_STORE * G)
                held_store_loop<G, PF, NT, BKD_HOLD_STORE>(lds, lanereg, g, base, src, n, gid, ngroups, low_clock);
            else
                held_store_loop<G, PF, NT, kHoldLong>(lds, lanereg, g, base, src, n, gid, ngroups, low_clock);
        }
    } else {
        groups_loop<G, PF, NT>(lds, lanereg, g, base, src, n, gid, ngroups, err, low_clock);
    }
}

// ---- chunk descriptors of the ragged-batch plan (built by plan_kernels.hpp) ----
// 16 bytes: W + kWBias (41 bits; W = the byte offset where the chunk's step-aligned window starts,
// up to one step before the chunk's first byte) | pad (7 bits) | len (16 bits; a chunk is at most
// CH + 15 < 64 KiB bytes), the register folded into its first bytes, and the destination (bit 31:
// finalized CRC into out[dst], else raw partial into partials[dst]). len == 0 marks a hole. The
// chunk is [W + lead, W + J*step) with J = ceil(len / step), lead = J*step - len: the chunk kernel
// derives each lane's masks from those small integers instead of 64-bit address arithmetic.
// pad > 0: the chunk ends on a 128-byte line past its entry's end; its last pad bytes belong to
// other data and are folded as zeros (the combine then multiplies by x^(-8*pad)).
constexpr uint32_t kPlanFinal = 0x80000000u;
constexpr int kPlanOffBits = 41;
constexpr uint64_t kPlanMaxSize = 1ull << (kPlanOffBits - 1);  // W + kWBias fits the 41 bits
constexpr int64_t kWBias = 1024;                                 // > the widest step (64 lanes x 16 B)

struct __attribute__((aligned(16))) PlanDesc {
    uint64_t s_len;
    uint32_t r0;
    uint32_t dst;
};

// The 8-byte descriptor of an unseeded batch (no per-entry seeds; base < kPlanMaxSize8): the same
// window / pad / length word, bit 40 set on a head (its register is the batch's one ~seed, a kernel
// argument), and every chunk's partial at its own list position (no final chunks: the combine
// finishes single-chunk entries too). Half the descriptor bytes the plan writes and reads back.
struct __attribute__((aligned(8))) PlanDesc8 {
    uint64_t s_len;
};
constexpr int kPlanHeadBit = 40;
constexpr uint64_t kPlanMaxSize8 = (1ull << kPlanHeadBit) - 4096u;  // W + kWBias below bit 40

// ---- pipelined chunk processing for the plan -------------------------------------------
// A chunk's first PF+1 steps are loaded while the PREVIOUS chunk of the group is still being
// folded and finalised, so a group never waits a full HBM latency at a chunk boundary. Two
// register sets (X, Y) alternate between consecutive chunks: the loads for chunk k+1 land in the
// set chunk k is not using, and no register copy (which would force a vmcnt wait) is needed.

struct ChunkGeo {
    int64_t a;    // this lane's step-0 block (16-byte aligned)
    int64_t la0;  // step-0 load address: a, or for windows wider than a line the block holding the
                  // first byte (a lane's own block could then lie on the page before it)
    uint32_t J;   // steps
    uint32_t r0;  // register folded into the first bytes
    uint32_t dst;
    uint32_t len;
    uint32_t pad;  // trailing bytes of the window that are not the entry's (folded as zeros)
    int32_t d0;    // bytes of this lane's step-0 block before the chunk's first byte (lead - 16g)
    int32_t keep;  // bytes of this lane's last-step block that belong to the chunk (step - pad - 16g)
};

template <int G>
__device__ __forceinline__ ChunkGeo chunk_geo(const PlanDesc& d, int g, uint32_t /*r0h: PlanDesc8 only*/ = 0u) {
    using Gm = Geo<G>;
    ChunkGeo c;
    const int64_t w = (int64_t)(d.s_len & ((1ull << kPlanOffBits) - 1u)) - kWBias;
    c.pad = (uint32_t)(d.s_len >> kPlanOffBits) & 127u;
    c.len = (uint32_t)(d.s_len >> 48);
    c.J = (c.len + (uint32_t)Gm::kStep - 1u) / (uint32_t)Gm::kStep;  // a power of two: a shift
    c.d0 = (int32_t)(c.J * (uint32_t)Gm::kStep - c.len) - 16 * g;
    c.keep = Gm::kStep - (int32_t)c.pad - 16 * g;
    c.a = w + 16 * g;
    if constexpr (Gm::kStep > 128) c.la0 = c.d0 >= 16 ? c.a + (c.d0 & ~15) : c.a;
    else c.la0 = c.a;  // the window's first step is one line, the line of the chunk's first byte
    c.r0 = d.r0;
    c.dst = d.dst;
    return c;
}

template <int G>
__device__ __forceinline__ ChunkGeo chunk_geo(const PlanDesc8& d, int g, uint32_t r0h) {
    PlanDesc full;
    full.s_len = d.s_len & ~(1ull << kPlanHeadBit);
    full.r0 = ((d.s_len >> kPlanHeadBit) & 1u) ? r0h : 0u;
    full.dst = 0u;
    return chunk_geo<G>(full, g);
}

// Loads of step 0 and steps 1..PF of chunk c (addresses past the chunk clamp to a valid block).
template <int G, int PF, bool NT>
__device__ __forceinline__ void chunk_prefetch(const uint8_t* __restrict__ base, const ChunkGeo& c, u32x4& W0,
                                               u32x4 (&A)[PF]) {
    W0 = ld16<NT && !BKD_W0_CACHED>(base + c.la0);  // a head's first line is its neighbour's last
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        const int64_t addr = (uint32_t)(k + 1) < c.J ? c.a + (int64_t)(k + 1) * Geo<G>::kStep : c.la0;
        A[k] = ld16<NT>(base + addr);
    }
}

#ifndef BKD_SHORT_FOLD4
// The short tail's folds with a step's 16 lookups requested before any is used (fold4_grouped; the
// compiler's own schedule waited stream by stream there): two- and four-step chunks -0.9 / -2.6 %,
// the < 1 KiB bucket -0.8 %, config 3 -0.1 % (round 6, profiles/r08o_ab_short_fold_grouped.log; the
// inline-asm fold4_main, which needs the image at LDS address 0, measured alike: r08n_*)
#define BKD_SHORT_FOLD4 1
#endif
#ifndef BKD_HOLE_GEO
// The chunk kernel requests every geometry's blocks as they are: a hole has a window at base[0]
// (skip_desc) and a chunk past the list the last real chunk's, so no geometry is selected per chunk
// (0: the field-by-field selects of a "last real chunk" geometry). The < 1 KiB bucket -2.1 %,
// 1M one-step chunks -1.6 %, 8 KiB chunk pairs -0.6 %, config 3 +-0, and the short tail's one
// spilled register gone (round 6, profiles/r08h_ab_hole_geometry_full_static.log)
#define BKD_HOLE_GEO 1
#endif
#ifndef BKD_FIRST_FAST
// The chunk kernel's step-0 masks, seed image and pad removal as clamped shifts, no branches: bit 0
// its short tail, bit 1 its long loop (0: the branchy form). 1M one-step chunks -6 %, the < 1 KiB
// bucket -3.7 %, config 3 -0.3 % (round 6, profiles/r08b_ab_first_block_fast.log)
#define BKD_FIRST_FAST 3
#endif
// Dword k of a chunk's step-0 block, branch-free: x8 = 8 * (d0 - 4k) bits of it lie in front of the
// chunk's first byte (cleared: low32(~0 << clamp(x8, 0, 32))), and it takes its part of the seed
// image r0 << 8*d0 (low32((r0 : 0) >> (32 - clamp(x8, -32, 32))); a shift of 64 is 0 mod 64 and the
// low half of (r0 : 0) is zero). The same part with x8 = 8 * (d0 - step) is the spill into step 1.
// (tests/test_first_block_model.py pins both to the branchy form, every d0 and keep in [-1100, 1100].)
__device__ __forceinline__ uint32_t seed_part(uint32_t r0, int32_t x8) {
    const uint32_t sh = (uint32_t)(32 - min(max(x8, -32), 32));
    return (uint32_t)(((uint64_t)r0 << 32) >> (sh & 63u));
}
__device__ __forceinline__ uint32_t keep_from(uint32_t x, int32_t x8) {  // bytes at or past x8 / 8
    return x & (uint32_t)(~0ull << (uint32_t)min(max(x8, 0), 32));
}
__device__ __forceinline__ u32x4 first_block_fast(u32x4 W0, uint32_t r0, int32_t d0) {
    const int32_t x8 = 8 * d0;
    return u32x4{keep_from(W0.x, x8) ^ seed_part(r0, x8), keep_from(W0.y, x8 - 32) ^ seed_part(r0, x8 - 32),
                 keep_from(W0.z, x8 - 64) ^ seed_part(r0, x8 - 64), keep_from(W0.w, x8 - 96) ^ seed_part(r0, x8 - 96)};
}
// The bytes of a chunk's last block at or past `keep` (the pad folded last, XORed out again).
__device__ __forceinline__ u32x4 pad_junk_fast(u32x4 last, int32_t keep) {
    const int32_t x8 = 8 * keep;
    return u32x4{keep_from(last.x, x8), keep_from(last.y, x8 - 32), keep_from(last.z, x8 - 64),
                 keep_from(last.w, x8 - 96)};
}

// The lane's step-0 block of chunk `c` with the bytes in front of the chunk cleared and the seed
// image XORed in; fx = the part of the seed image that spills into step 1's dword 0.
template <int G>
__device__ __forceinline__ u32x4 chunk_first_block(const ChunkGeo& c, u32x4 W0, uint32_t& fx) {
    using Gm = Geo<G>;
#if BKD_FIRST_FAST & 1
    fx = seed_part(c.r0, 8 * (c.d0 - Gm::kStep));
    return first_block_fast(W0, c.r0, c.d0);
#endif
    const int32_t d0 = c.d0;
    u32x4 w;
    if (d0 <= 0) w = W0;
    else if (d0 < 16) w = mask_low_bytes(W0, (uint32_t)d0);
    else w = u32x4{0u, 0u, 0u, 0u};
    const uint32_t r0 = c.r0;
    if (d0 > -4 && d0 < 16) {
        // the seed image is r0 << 8*d0 across the 16-byte block: dword k = (r0:0 >> (32 + 32k - 8*d0))
        const uint64_t R = (uint64_t)r0 << 32;
        auto part = [&](int k) -> uint32_t {
            const int32_t t = 32 + 32 * k - 8 * d0;
            return (t > 0 && t < 64) ? (uint32_t)(R >> t) : 0u;
        };
        w.x ^= part(0);
        w.y ^= part(1);
        w.z ^= part(2);
        w.w ^= part(3);
    }
    fx = 0u;
    if (d0 > Gm::kStep - 4) fx = place_seed(r0, d0 - Gm::kStep);
    return w;
}

// Raw register of a short chunk (J <= PF + 1: every block of it is in W0 and A[0..J-2]) — the
// arithmetic of chunk_fold without any loads (short_chunks_loop issued them chunks ahead).
template <int G, int PF>
__device__ __forceinline__ uint32_t short_chunk_fold(const uint32_t* lds, uint32_t lanereg, const ChunkGeo& c,
                                                     const u32x4& W0, const u32x4 (&A)[PF]) {
    uint32_t fx;
    const u32x4 w = chunk_first_block<G>(c, W0, fx);
    uint32_t c0 = w.x, c1 = w.y, c2 = w.z, c3 = w.w;
    const uint32_t rem = c.J - 1u;
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        if ((uint32_t)k < rem) {
#if BKD_SHORT_FOLD4
            fold4_grouped(lds, c0, c1, c2, c3, lanereg, A[k].x ^ (k == 0 ? fx : 0u), A[k].y, A[k].z, A[k].w);
#else
            c0 = mul_main_add(lds, c0, lanereg, A[k].x ^ (k == 0 ? fx : 0u));
            c1 = mul_main_add(lds, c1, lanereg, A[k].y);
            c2 = mul_main_add(lds, c2, lanereg, A[k].z);
            c3 = mul_main_add(lds, c3, lanereg, A[k].w);
#endif
        }
    }
    if (c.pad && c.keep < 16) {  // the last step's bytes past the entry were folded last: XOR them out
        u32x4 last = W0;
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if ((uint32_t)k + 1u == rem) last = A[k];
#if BKD_FIRST_FAST & 1
        const u32x4 junk = pad_junk_fast(last, c.keep);
#else
        const u32x4 junk = c.keep <= 0 ? last : mask_low_bytes(last, (uint32_t)c.keep);
#endif
        c0 ^= junk.x;
        c1 ^= junk.y;
        c2 ^= junk.z;
        c3 ^= junk.w;
    }
    return finish_lanes<G>(lds, c0, c1, c2, c3);
}

// Folds chunk `c` (its W0/A already loaded) and, once its own loads are all issued, prefetches
// chunk `nx` into NW0/NA. Returns the chunk's raw register (valid in lane g == 0).
template <int G, int PF, bool NT>
__device__ __forceinline__ uint32_t chunk_fold(const uint32_t* lds, uint32_t lanereg, int g,
                                               const uint8_t* __restrict__ base, const ChunkGeo& c, u32x4 W0,
                                               u32x4 (&A)[PF], u32x4 (&B)[PF], const ChunkGeo& nx, u32x4& NW0,
                                               u32x4 (&NA)[PF]) {
    using Gm = Geo<G>;
    const int64_t a = c.a;
    const int32_t d0 = c.d0;
    const uint32_t rem = c.J - 1u;
#if BKD_EARLY_PREFETCH
    // the successor is requested before anything waits for this chunk's own blocks (unconditionally,
    // so that the loads land in NW0/NA without a register copy): the compiler's s_waitcnt for W0 then
    // sits after these loads, and consecutive chunks overlap their memory round trips instead of
    // paying one each
    chunk_prefetch<G, PF, NT>(base, nx, NW0, NA);
#endif
#if BKD_FIRST_FAST & 2
    const u32x4 w = first_block_fast(W0, c.r0, d0);
    uint32_t fx = seed_part(c.r0, 8 * (d0 - Gm::kStep));
#else
    u32x4 w;
    if (d0 <= 0) w = W0;
    else if (d0 < 16) w = mask_low_bytes(W0, (uint32_t)d0);
    else w = u32x4{0u, 0u, 0u, 0u};
    const uint32_t r0 = c.r0;
    if (d0 > -4 && d0 < 16) {
        // the seed image is r0 << 8*d0 across the 16-byte block: dword k = (r0:0 >> (32 + 32k - 8*d0))
        const uint64_t R = (uint64_t)r0 << 32;
        auto part = [&](int k) -> uint32_t {
            const int32_t t = 32 + 32 * k - 8 * d0;
            return (t > 0 && t < 64) ? (uint32_t)(R >> t) : 0u;
        };
        w.x ^= part(0);
        w.y ^= part(1);
        w.z ^= part(2);
        w.w ^= part(3);
    }
    uint32_t fx = 0u;
    if (d0 > Gm::kStep - 4) fx = place_seed(r0, d0 - Gm::kStep);
#endif
    uint32_t c0 = w.x, c1 = w.y, c2 = w.z, c3 = w.w;
    // the lane's last block as it was folded: a pad is XORed out of the very register that folded
    // it, so the bytes past the entry (another entry's, or past the caller's buffer) cancel whatever
    // they hold, even if something rewrites them while the chunk runs (no second load of that block)
    u32x4 last = W0;
#define BKD_FOLD0(d)                                    \
    do {                                                 \
        c0 = mul_main_add(lds, c0, lanereg, (d).x ^ fx);    \
        fx = 0u;                                         \
        c1 = mul_main_add(lds, c1, lanereg, (d).y);         \
        c2 = mul_main_add(lds, c2, lanereg, (d).z);         \
        c3 = mul_main_add(lds, c3, lanereg, (d).w);         \
    } while (0)
#define BKD_FOLD(d)                                  \
    do {                                             \
        c0 = mul_main_add(lds, c0, lanereg, (d).x);     \
        c1 = mul_main_add(lds, c1, lanereg, (d).y);     \
        c2 = mul_main_add(lds, c2, lanereg, (d).z);     \
        c3 = mul_main_add(lds, c3, lanereg, (d).w);     \
    } while (0)
    if (rem <= (uint32_t)PF) {
#if !BKD_EARLY_PREFETCH
        chunk_prefetch<G, PF, NT>(base, nx, NW0, NA);
#endif
        if (rem > 0u) BKD_FOLD0(A[0]);
#pragma unroll
        for (int k = 1; k < PF; ++k)
            if ((uint32_t)k < rem) BKD_FOLD(A[k]);
        if (c.pad && c.keep < 16) {  // (selected only where a pad is removed: no cost per full chunk)
#pragma unroll
            for (int k = 0; k < PF; ++k)
                if ((uint32_t)k + 1u == rem) last = A[k];
        }
    } else {
        const uint8_t* p = base + a + (int64_t)(PF + 1) * Gm::kStep;  // first step not yet loaded
        uint32_t left = rem - (uint32_t)PF;
        bool first = true;
        while (left >= 2u * PF) {
#pragma unroll
            for (int k = 0; k < PF; ++k) B[k] = ld16<NT>(p + (int64_t)k * Gm::kStep);
            if (first) BKD_FOLD0(A[0]);
            else BKD_FOLD(A[0]);
            first = false;
#pragma unroll
            for (int k = 1; k < PF; ++k) BKD_FOLD(A[k]);
#pragma unroll
            for (int k = 0; k < PF; ++k) A[k] = ld16<NT>(p + (int64_t)(PF + k) * Gm::kStep);
#pragma unroll
            for (int k = 0; k < PF; ++k) BKD_FOLD(B[k]);
            p += (int64_t)(2 * PF) * Gm::kStep;
            left -= 2u * PF;
        }
        // (the A/B tail loads stay conditional here: with clamped unconditional loads the last block
        // would be requested twice, and the pad must come out of the register that folded it)
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if ((uint32_t)k < left) B[k] = ld16<NT>(p + (int64_t)k * Gm::kStep);
        if (first) BKD_FOLD0(A[0]);
        else BKD_FOLD(A[0]);
#pragma unroll
        for (int k = 1; k < PF; ++k) BKD_FOLD(A[k]);
        last = A[PF - 1];  // the last block when left == 0 (A is reloaded below only for steps < left)
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if ((uint32_t)(PF + k) < left) A[k] = ld16<NT>(p + (int64_t)(PF + k) * Gm::kStep);
#if !BKD_EARLY_PREFETCH
        chunk_prefetch<G, PF, NT>(base, nx, NW0, NA);  // issued after every load of this chunk
#endif
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if ((uint32_t)k < left) BKD_FOLD(B[k]);
#pragma unroll
        for (int k = 0; k < PF; ++k)
            if ((uint32_t)(PF + k) < left) BKD_FOLD(A[k]);
        if (c.pad && c.keep < 16) {
#pragma unroll
            for (int k = 0; k < PF; ++k) {
                if ((uint32_t)k + 1u == left) last = B[k];
                if ((uint32_t)(PF + k) + 1u == left) last = A[k];
            }
        }
    }
#undef BKD_FOLD
#undef BKD_FOLD0
    if (c.pad && c.keep < 16) {
        // the last step's block of this lane ends past the entry: its bytes >= the entry's end were
        // folded last (XORed in after the final multiply), so XOR them out again
        const int32_t keep = c.keep;
#if BKD_FIRST_FAST & 2
        const u32x4 junk = pad_junk_fast(last, keep);
#else
        const u32x4 junk = keep <= 0 ? last : mask_low_bytes(last, (uint32_t)keep);
#endif
        c0 ^= junk.x;
        c1 ^= junk.y;
        c2 ^= junk.z;
        c3 ^= junk.w;
    }
    return finish_lanes<G>(lds, c0, c1, c2, c3);
}

// The short tail of the chunk list, [i, n) in grid stride: chunks of at most PF + 1 steps (the list
// is sorted by descending step count, so they come last: config 3's 1-, 2- and 3-step heads, 437 K
// of its 1 M). A one-step chunk is folded in ~300 VALU per wave, less than a loaded memory round
// trip, so with one chunk prefetched (chunk_fold's X/Y sets) a group waits for memory at every
// chunk. Here three register sets rotate: a chunk's blocks are requested three chunks before its
// fold and its descriptor three chunks before that. Every load is unconditional (a hole or a chunk
// past the list re-reads a real chunk's blocks), so the compiler's waits can count exactly.
template <int G, int PF, bool NT, class Desc>
__device__ __forceinline__ void short_chunks_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                                  const uint8_t* __restrict__ base, const Desc* __restrict__ descs,
                                                  uint32_t r0h,
                                                  uint64_t i, uint64_t n, uint64_t ngroups, uint32_t* __restrict__ out,
                                                  uint32_t* __restrict__ partials, uint64_t nstart) {
#if BKD_HOLD_SHORT > 0
    // partials by list position, held (HeldResults; a final chunk's or a hole's word lands in its own
    // unused slot): the short tail is a group's last work, so they are stored at its very end
    const uint64_t gid0 = i - nstart;
    HeldResults<G, BKD_HOLD_SHORT> held;
#endif
    auto clampi = [&](uint64_t j) { return j < n ? j : n - 1; };
    auto geo_at = [&](uint64_t j) {
        ChunkGeo c = chunk_geo<G>(descs[clampi(j)], g, r0h);
        if (j >= n) c.len = 0;
        return c;
    };
#if BKD_HOLE_GEO
    // every geometry has loadable blocks: a chunk past the list has the last real chunk's (clampi), a
    // hole the window skip_desc() gives it at base[0]
    auto load = [&](const ChunkGeo& c, u32x4& W0, u32x4 (&A)[PF]) { chunk_prefetch<G, PF, NT>(base, c, W0, A); };
#else
    // blocks a hole (or a chunk past the list) loads instead: the last real chunk's, base[0, 16)
    // before one is seen. Selected field by field: a reference to one of two geometries would put
    // both in scratch memory.
    int64_t fa = 0, fla0 = 0;
    uint32_t fJ = 1u;
    auto load = [&](const ChunkGeo& c, u32x4& W0, u32x4 (&A)[PF]) {
        if (c.len) {
            fa = c.a;
            fla0 = c.la0;
            fJ = c.J;
        }
        ChunkGeo t;
        t.a = fa;
        t.la0 = fla0;
        t.J = fJ;
        chunk_prefetch<G, PF, NT>(base, t, W0, A);
    };
#endif
    u32x4 W0x, Ax[PF], W0y, Ay[PF], W0z, Az[PF];
    ChunkGeo cx = geo_at(i), cy = geo_at(i + ngroups), cz = geo_at(i + 2 * ngroups);
    load(cx, W0x, Ax);
    load(cy, W0y, Ay);
    load(cz, W0z, Az);
    Desc dx = descs[clampi(i + 3 * ngroups)], dy = descs[clampi(i + 4 * ngroups)],
         dz = descs[clampi(i + 5 * ngroups)];
#if BKD_HOLD_SHORT > 0
#define BKD_SHORT_EMIT(C, v)                                                                 \
    held.put(v, g, partials + nstart, gid0, ngroups, n - nstart);                            \
    if (g == 0 && C.len && (C.dst & kPlanFinal)) out[C.dst & ~kPlanFinal] = ~v;
#else
#define BKD_SHORT_EMIT(C, v)                                                                 \
    if (g == 0 && C.len) {                                                                   \
        if (C.dst & kPlanFinal) out[C.dst & ~kPlanFinal] = ~v;                               \
        else partials[C.dst] = v;                                                            \
    }
#endif
#define BKD_SHORT_STEP(C, W0C, AC, DC)                                                       \
    {                                                                                        \
        const uint32_t v = C.len ? short_chunk_fold<G, PF>(lds, lanereg, C, W0C, AC) : 0u;   \
        BKD_SHORT_EMIT(C, v)                                                                 \
        C = chunk_geo<G>(DC, g, r0h); /* chunk i + 3 ngroups */                              \
        if (i + 3 * ngroups >= n) C.len = 0;                                                 \
        load(C, W0C, AC);                                                                    \
        DC = descs[clampi(i + 6 * ngroups)];                                                 \
        i += ngroups;                                                                        \
        /* wave-uniform exit (a group past the list folds holes until its wave is done):    \
           loads under a divergent branch would leave the compiler's waits uncountable */   \
        if (!__any(i < n)) break;                                                            \
    }
    for (;;) {
        BKD_SHORT_STEP(cx, W0x, Ax, dx)
        BKD_SHORT_STEP(cy, W0y, Ay, dy)
        BKD_SHORT_STEP(cz, W0z, Az, dz)
    }
#undef BKD_SHORT_STEP
#undef BKD_SHORT_EMIT
#if BKD_HOLD_SHORT > 0
    held.finish(g, partials + nstart, gid0, ngroups, n - nstart);
#endif
}

// Chunks [0, n) of the list in grid stride, one prefetched chunk per group (X/Y sets).
template <int G, int PF, bool NT, class Desc>
__device__ __forceinline__ void long_chunks_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                                 const uint8_t* __restrict__ base, const Desc* __restrict__ descs,
                                                 uint32_t r0h,
                                                 uint64_t n, uint64_t gid, uint64_t ngroups, uint32_t* __restrict__ out,
                                                 uint32_t* __restrict__ partials) {
    auto clampi = [&](uint64_t j) { return j < n ? j : n - 1; };
    // a hole (len == 0) or a missing next chunk prefetches the current chunk's own blocks
    auto pf_geo = [&](const ChunkGeo& nx, const ChunkGeo& cur) -> const ChunkGeo& { return nx.len ? nx : cur; };
#if BKD_HOLD_LONGLOOP > 0
    // partials by list position, held (a final chunk's or a hole's word lands in its own unused slot)
    HeldResults<G, BKD_HOLD_LONGLOOP> held;
    auto emit = [&](const ChunkGeo& c, uint32_t v) {
        held.put(v, g, partials, gid, ngroups, n);
        if (g == 0 && c.len && (c.dst & kPlanFinal)) out[c.dst & ~kPlanFinal] = ~v;
    };
#else
    auto emit = [&](const ChunkGeo& c, uint32_t v) {
        if (g == 0 && c.len) {
            if (c.dst & kPlanFinal) out[c.dst & ~kPlanFinal] = ~v;
            else partials[c.dst] = v;
        }
    };
#endif

    u32x4 W0x, Ax[PF], Bx[PF], W0y, Ay[PF], By[PF];
    uint64_t i = gid;
    ChunkGeo cur = chunk_geo<G>(descs[i], g, r0h);
    // Descriptors of the next chunk of each half live in their own registers (dA for set-X halves,
    // dB for set-Y halves), each loaded two halves before its use and reloaded (three rounds ahead)
    // right after: no copy of a just-loaded value (a `dn = dnn` copy made the compiler wait for that
    // load), and enough loads issued between a descriptor and its use that the compiler's count of
    // them never reaches back into the current chunk's prefetch.
    Desc dA = descs[clampi(i + ngroups)], dB = descs[clampi(i + 2 * ngroups)];
#if BKD_HOLE_GEO
    // every geometry has loadable blocks (a hole's window is base[0], skip_desc; a missing next chunk
    // is the last real one, clampi): the next chunk's blocks are requested whatever it is
#define BKD_PF_GEO(nx, cur) (nx)
    chunk_prefetch<G, PF, NT>(base, cur, W0x, Ax);
#else
    // a hole's prefetch reads base[0, 16) (only plans that overflowed their capacity have holes)
    ChunkGeo safe;
    safe.la0 = safe.a = 0, safe.J = 1;
#define BKD_PF_GEO(nx, cur) pf_geo(nx, cur.len ? cur : safe)
    chunk_prefetch<G, PF, NT>(base, cur.len ? cur : safe, W0x, Ax);
#endif
#define BKD_CHUNK_HALF(DN, W0C, AC, BC, W0N, AN)                                                            \
    {                                                                                                      \
        const bool more = i + ngroups < n;                                                                 \
        ChunkGeo nx = chunk_geo<G>(DN, g, r0h);                                                            \
        DN = descs[clampi(i + 3 * ngroups)];                                                               \
        if (!more) nx.len = 0;                                                                             \
        const ChunkGeo& pg = BKD_PF_GEO(nx, cur);                                                          \
        const uint32_t v = cur.len ? chunk_fold<G, PF, NT>(lds, lanereg, g, base, cur, W0C, AC, BC, pg, W0N, AN) \
                                   : (chunk_prefetch<G, PF, NT>(base, pg, W0N, AN), 0u);                   \
        emit(cur, v);                                                                                      \
        if (!more) break;                                                                                  \
        i += ngroups;                                                                                      \
        cur = nx;                                                                                          \
    }
    for (;;) {
        BKD_CHUNK_HALF(dA, W0x, Ax, Bx, W0y, Ay)  // chunk i in set X, prefetch into Y
        BKD_CHUNK_HALF(dB, W0y, Ay, By, W0x, Ax)  // chunk i in set Y, prefetch into X
#if BKD_CHUNK_UNROLL >= 4
        // the back edge copies the loop-carried descriptor registers, for which the compiler waits
        // with s_waitcnt vmcnt(0) — a full drain of the loads in flight; more halves per iteration,
        // fewer drains
        BKD_CHUNK_HALF(dA, W0x, Ax, Bx, W0y, Ay)
        BKD_CHUNK_HALF(dB, W0y, Ay, By, W0x, Ax)
#endif
#if BKD_CHUNK_UNROLL >= 8
        BKD_CHUNK_HALF(dA, W0x, Ax, Bx, W0y, Ay)
        BKD_CHUNK_HALF(dB, W0y, Ay, By, W0x, Ax)
        BKD_CHUNK_HALF(dA, W0x, Ax, Bx, W0y, Ay)
        BKD_CHUNK_HALF(dB, W0y, Ay, By, W0x, Ax)
#endif
    }
#if BKD_HOLD_LONGLOOP > 0
    held.finish(g, partials, gid, ngroups, n);
#endif
#undef BKD_CHUNK_HALF
#undef BKD_PF_GEO
}

// Blocks per chunk in the short tail's register sets beside step 0: chunks of <= kShortPF + 1 steps
// (PlanGeo::jshort) take short_chunks_loop.
#ifndef BKD_SHORT_PF
#define BKD_SHORT_PF 3
#endif
constexpr int kShortPF = BKD_SHORT_PF;
#ifndef BKD_SHORT_NT
#define BKD_SHORT_NT 0  // the short tail's loads are cached: heads share lines with their neighbours (1: nontemporal)
#endif

// The chunk list [0, n) (crc_plan_chunks_kernel): [0, nmain) by long_chunks_loop, then the short
// tail [nmain, n) by short_chunks_loop (nmain == n: no short tail).
template <int G, int PF, bool NT, class Desc>
__device__ __forceinline__ void plan_chunks_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                                 const uint8_t* __restrict__ base, const Desc* __restrict__ descs,
                                                 uint32_t r0h,
                                                 uint64_t n, uint64_t nmain, uint64_t gid, uint64_t ngroups,
                                                 uint32_t* __restrict__ out, uint32_t* __restrict__ partials) {
#if BKD_SHORT_FIRST
    // the short tail first: the long loop's held partials (the larger set) are then stored at the
    // group's very end (per-group work, and so the kernel's balance, does not depend on the order)
    if (nmain < n && gid < n - nmain)
        short_chunks_loop<G, kShortPF, NT && BKD_SHORT_NT>(lds, lanereg, g, base, descs, r0h, nmain + gid, n, ngroups, out,
                                                          partials, nmain);
    if (gid < nmain) long_chunks_loop<G, PF, NT>(lds, lanereg, g, base, descs, r0h, nmain, gid, ngroups, out, partials);
#else
    if (gid < nmain) long_chunks_loop<G, PF, NT>(lds, lanereg, g, base, descs, r0h, nmain, gid, ngroups, out, partials);
    if (nmain < n && gid < n - nmain)
        short_chunks_loop<G, kShortPF, NT && BKD_SHORT_NT>(lds, lanereg, g, base, descs, r0h, nmain + gid, n, ngroups, out,
                                                          partials, nmain);
#endif
}


// Chunk kernel of the ragged-batch plan: one chunk per group, grid stride over the descriptor
// list (sorted by step count, plan_kernels.hpp). Descriptors are read two rounds ahead and each
// chunk's first loads are issued during the previous chunk (chunk_fold), X/Y register sets
// alternating.
// After its chunks, the grid computes the entries the plan could not hold (`ov`, normally empty).
template <int G, int PF, bool NT, class OvSrc, class Desc = PlanDesc>
__global__ void __launch_bounds__(kBlock) crc_plan_chunks_kernel(const uint8_t* __restrict__ base,
                                                                 const Desc* __restrict__ descs, uint32_t r0h,
                                                                 const uint32_t* __restrict__ count,
                                                                 const uint32_t* __restrict__ tables,
                                                                 uint32_t* __restrict__ out,
                                                                 uint32_t* __restrict__ partials, OvSrc ov,
                                                                 PlanRun run, uint32_t* __restrict__ err) {
    using Gm = Geo<G>;
    if (!run.plan_entries()) return;  // only short entries
    __shared__ __attribute__((aligned(16))) uint32_t lds[Gm::kLdsWords];
    // near-uniform lengths (PlanRun::uniform): no chunks, every entry whole as in the direct kernel
    ov.all = run.uniform();
    const uint64_t n = ov.all ? 0u : *count;
    const uint64_t nov = ov.count();
    if (n == 0 && nov == 0) return;  // every entry was short or serial: no table staging
    stage_tables<G>(lds, tables);

    const int lane = threadIdx.x & 63;
    const int g = lane & (G - 1);
    const uint32_t lanereg = ((uint32_t)(lane & 31) << 2) | (1u << 16);
    const uint64_t ngroups = (uint64_t)gridDim.x * (kBlock / G);
    const uint64_t gid = (uint64_t)blockIdx.x * (kBlock / G) + (uint64_t)(threadIdx.x / G);
    // count[1]: the list position of the first chunk of at most PF + 1 steps (plan_emit_kernel)
    const uint64_t nmain = n ? std::min<uint64_t>(n, count[1]) : 0u;
    if (gid < n) plan_chunks_loop<G, PF, NT>(lds, lanereg, g, base, descs, r0h, n, nmain, gid, ngroups, out, partials);
#if BKD_HOLD_DIRECT > 0
    // near-uniform batches (every entry here, one per group): results held as the uniform kernel's
    if (nov && ov.all) {
        if (gid < nov) held_direct_loop<G, PF, NT, BKD_HOLD_DIRECT>(lds, lanereg, g, base, ov, nov, gid, ngroups, err);
    } else
#endif
    if (nov) groups_loop<G, PF, NT>(lds, lanereg, g, base, ov, nov, gid, ngroups, err);
}

// ---- synthetic input: little-endian splitmix64 stream ----
__device__ __forceinline__ uint64_t splitmix_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_splitmix64_kernel(uint8_t* __restrict__ dst, uint64_t nbytes, uint64_t seed,
                                       uint64_t first_word) {
    const uint64_t nw = nbytes / 8;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t* d64 = reinterpret_cast<uint64_t*>(dst);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += stride)
        d64[i] = splitmix_mix(seed + (first_word + i + 1) * 0x9E3779B97F4A7C15ull);
    if (blockIdx.x == 0 && threadIdx.x == 0 && (nbytes & 7)) {
        const uint64_t v = splitmix_mix(seed + (first_word + nw + 1) * 0x9E3779B97F4A7C15ull);
        for (uint64_t k = 0; k < (nbytes & 7); ++k) dst[nw * 8 + k] = (uint8_t)(v >> (8 * k));
    }
}

// ---- DigestManager framing helpers (one thread per entry; 32-byte headers) ----

// Package step 1: header [ledgerId, entryId, LAC, length] BE into the frame
// (DigestManager.java:146-149 / :172-175) and its CRC (= the payload's seed) into seeds[i]. The
// header is built as 8 little-endian dwords (byte-swapped BE fields), folded with the x^32 operator
// (4 lookups per dword) and stored as dwords when the frame is 4-byte aligned.
// Header kernels: grid stride (2 blocks of 1024 per CU), the x^32 tables staged once per block —
// one 256-thread block per 256 entries staged them 4096 times per 1M entries (verify header 38 us).
__global__ void __launch_bounds__(1024) package_header_kernel(const uint32_t* __restrict__ x32tab, int64_t ledger_id,
                                                             const int64_t* __restrict__ entry_ids,
                                                             const int64_t* __restrict__ lacs,
                                                             const int64_t* __restrict__ length_fields, uint64_t n,
                                                             uint8_t* __restrict__ frames, uint64_t frame_stride,
                                                             uint32_t* __restrict__ seeds) {
    __shared__ uint32_t W[1024];
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) W[k] = x32tab[k];
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t fld[4] = {(uint64_t)ledger_id, (uint64_t)entry_ids[i], (uint64_t)lacs[i],
                             (uint64_t)length_fields[i]};
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        w[2 * k] = __builtin_bswap32((uint32_t)(fld[k] >> 32));
        w[2 * k + 1] = __builtin_bswap32((uint32_t)fld[k]);
    }
    uint32_t reg = 0xFFFFFFFFu;  // update(0, header)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t r = reg ^ w[k];
        reg = W[r & 0xffu] ^ W[256 + ((r >> 8) & 0xffu)] ^ W[512 + ((r >> 16) & 0xffu)] ^ W[768 + (r >> 24)];
    }
    uint8_t* f = frames + i * frame_stride;
    if ((((uintptr_t)f) & 3u) == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) reinterpret_cast<uint32_t*>(f)[k] = w[k];
    } else {
        for (int k = 0; k < 32; ++k) f[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
    seeds[i] = ~reg;
    }
}

// Package step 3: the digest bytes after the header (CRC32CDigestManager.java:44-46: writeInt;
// CRC32DigestManager.java:60-63: writeLong of the zero-extended value).
__global__ void __launch_bounds__(256) package_digest_kernel(const uint32_t* __restrict__ digests, uint64_t n,
                                                             uint8_t* __restrict__ frames, uint64_t frame_stride,
                                                             uint32_t mac) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    put_frame_digest(frames + i * frame_stride + 32, digests[i], mac);
}

// The frames of the fused package route: each frame's 32-byte BE header (DigestManager.java:146-149)
// and its digest at offset 32 (4-byte BE int, or 8-byte BE zero-extended long for CRC32) in one
// pass after crc_package_fused_kernel, one frame per thread.
__global__ void __launch_bounds__(256) package_frame_kernel(int64_t ledger_id, const int64_t* __restrict__ entry_ids,
                                                            const int64_t* __restrict__ lacs,
                                                            const int64_t* __restrict__ length_fields,
                                                            const uint32_t* __restrict__ digests, uint64_t n,
                                                            uint8_t* __restrict__ frames, uint64_t frame_stride,
                                                            uint32_t mac) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // packed frames (stride 32 + mac, the DigestManager layout package_batch returns) on a 4-byte
    // boundary: the block's frames are built in LDS and written as consecutive dwords, every store
    // instruction one contiguous run (a frame per thread wrote 9-10 dwords 36-40 bytes apart)
    if (frame_stride == 32u + mac && (((uintptr_t)frames) & 3u) == 0) {
        __shared__ uint32_t fr[256 * 10];
        const uint32_t fw = (32u + mac) / 4u;  // dwords per frame
        const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x;
        const uint32_t cnt = (uint32_t)(n - i0 < (uint64_t)blockDim.x ? n - i0 : (uint64_t)blockDim.x);
        if (i < n) {
            const uint64_t fld[4] = {(uint64_t)ledger_id, (uint64_t)entry_ids[i], (uint64_t)lacs[i],
                                     (uint64_t)length_fields[i]};
            uint32_t* w = fr + threadIdx.x * fw;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                w[2 * k] = __builtin_bswap32((uint32_t)(fld[k] >> 32));
                w[2 * k + 1] = __builtin_bswap32((uint32_t)fld[k]);
            }
            if (mac == 8u) w[8] = 0u;
            w[fw - 1u] = __builtin_bswap32(digests[i]);
        }
        __syncthreads();
        uint32_t* dst = reinterpret_cast<uint32_t*>(frames + i0 * frame_stride);
        for (uint32_t k = threadIdx.x; k < cnt * fw; k += blockDim.x) dst[k] = fr[k];
        return;
    }
    if (i >= n) return;
    const uint64_t fld[4] = {(uint64_t)ledger_id, (uint64_t)entry_ids[i], (uint64_t)lacs[i], (uint64_t)length_fields[i]};
    const uint32_t dg = digests[i];
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        w[2 * k] = __builtin_bswap32((uint32_t)(fld[k] >> 32));
        w[2 * k + 1] = __builtin_bswap32((uint32_t)fld[k]);
    }
    uint8_t* f = frames + i * frame_stride;
    if ((((uintptr_t)f) & 3u) == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) reinterpret_cast<uint32_t*>(f)[k] = w[k];
    } else {
        for (int k = 0; k < 32; ++k) f[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
    put_frame_digest(f + 32, dg, mac);
}

// Verify step 1 (one thread per framed entry [32 B header][mac][payload], DigestManager.java:226-283):
// reads the header and the stored digest once — 16-byte loads when the frame is 16-byte aligned,
// dword loads when 4-byte aligned, bytes otherwise — and writes everything step 3 needs, so that
// step 3 touches no frame bytes:
//   seeds[i]   CRC of the 32-byte header = the payload's seed (:236)
//   pay_*[i]   the payload range [o + 32 + mac, o + l) step 2 folds (empty for a short entry)
//   expect[i]  the stored digest (low 32 bits; CRC32DigestManager writes a zero-extended long)
//   pre[i]     1 too short / out of range (:229-235); else bit 1 = high digest word non-zero,
//              bits 2.. = the id check's code (3 ledger mismatch :267-273, 4 entry mismatch :275-281)
// The header CRC folds 8 little-endian dwords with the x^32 operator (4 lookups per dword).
__device__ __forceinline__ uint32_t be32_at(const uint32_t* w, int byte) {  // big-endian u32 at a 4-aligned byte
    return __builtin_bswap32(w[byte >> 2]);
}

__global__ void __launch_bounds__(1024) verify_header_kernel(const uint32_t* __restrict__ x32tab,
                                                            const uint8_t* __restrict__ framed, uint64_t size,
                                                            const uint64_t* __restrict__ offsets,
                                                            const uint32_t* __restrict__ lengths, uint64_t n,
                                                            uint32_t mac, int64_t ledger_id, int64_t first_entry_id,
                                                            int id_checks, uint32_t* __restrict__ seeds,
                                                            uint64_t* __restrict__ pay_offsets,
                                                            uint32_t* __restrict__ pay_lengths,
                                                            uint32_t* __restrict__ expect, uint32_t* __restrict__ pre,
                                                            uint64_t* __restrict__ first_bad,
                                                            const uint32_t* __restrict__ vflag, uint32_t vepoch) {
    if (vflag && *vflag != vepoch) return;  // near-uniform frames: crc_verify_fused_kernel does it all
    __shared__ uint32_t W[1024];
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) W[k] = x32tab[k];
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) *first_bad = n;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t o = offsets[i];
    const uint32_t l = lengths[i];
    if (o > size || (uint64_t)l > size - o || l < 32u + mac) {
        seeds[i] = 0u;
        pay_offsets[i] = 0u;
        pay_lengths[i] = 0u;
        expect[i] = 0u;
        pre[i] = 1u;
        continue;
    }
    const uint8_t* f = framed + o;
    uint32_t w[10];  // bytes [0, 40) of the frame as little-endian dwords (the first 32 + mac are used)
    const int nw = (int)(32u + mac) / 4;
    if ((((uintptr_t)f) & 15u) == 0 && l >= 48u) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(f + 16 * k);
            if (4 * k < 10) w[4 * k] = v.x;
            if (4 * k + 1 < 10) w[4 * k + 1] = v.y;
            if (4 * k + 2 < 10) w[4 * k + 2] = v.z;
            if (4 * k + 3 < 10) w[4 * k + 3] = v.w;
        }
    } else if ((((uintptr_t)f) & 3u) == 0) {
        for (int k = 0; k < 10; ++k) w[k] = k < nw ? reinterpret_cast<const uint32_t*>(f)[k] : 0u;
    } else {
        for (int k = 0; k < 10; ++k) {
            uint32_t v = 0u;
            if (k < nw)
                for (int b = 3; b >= 0; --b) v = (v << 8) | f[4 * k + b];
            w[k] = v;
        }
    }
    uint32_t reg = 0xFFFFFFFFu;  // update(0, header): resume from 0 = register ~0
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t r = reg ^ w[k];
        reg = W[r & 0xffu] ^ W[256 + ((r >> 8) & 0xffu)] ^ W[512 + ((r >> 16) & 0xffu)] ^ W[768 + (r >> 24)];
    }
    seeds[i] = ~reg;
    pay_offsets[i] = o + 32u + mac;
    pay_lengths[i] = l - 32u - mac;
    const uint64_t lid = ((uint64_t)be32_at(w, 0) << 32) | be32_at(w, 4);
    const uint64_t eid = ((uint64_t)be32_at(w, 8) << 32) | be32_at(w, 12);
    uint32_t p = 0u;
    if (mac == 8) {
        if (w[8] != 0u) p |= 2u;
        expect[i] = be32_at(w, 36);
    } else {
        expect[i] = be32_at(w, 32);
    }
    // id_checks: 0 ledger + entry ids, 1 ledger id only, 2 digest only (entry-log scrub)
    if (id_checks < 2 && (int64_t)lid != ledger_id) p |= 3u << 2;
    else if (id_checks == 0 && (int64_t)eid != first_entry_id + (int64_t)i) p |= 4u << 2;
    pre[i] = p;
    }
}

// Verify step 3: per-entry status in DigestManager.verifyDigest's order (too short, digest, ledger id,
// entry id) and the first failing index (BatchedReadOp.java:164-190 verified-prefix rule).
__global__ void __launch_bounds__(256) verify_finish_kernel(const uint32_t* __restrict__ expect,
                                                            const uint32_t* __restrict__ pre, uint64_t n,
                                                            int32_t* __restrict__ status,
                                                            unsigned long long* __restrict__ first_bad,
                                                            const uint32_t* __restrict__ vflag, uint32_t vepoch) {
    if (vflag && *vflag != vepoch) return;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t computed = (uint32_t)status[i];
    const uint32_t p = pre[i];
    int32_t st;
    if (p == 1u) st = 1;
    else if ((p & 2u) || computed != expect[i]) st = 2;
    else st = (int32_t)(p >> 2);
    status[i] = st;
    if (st != 0) atomicMin(first_bad, (unsigned long long)i);
}

// ---- fused verify for near-uniform frames ---------------------------------------------------
// Frames whose lengths all lie within PlanRun::in_band of the first frame's are balanced one frame
// per lane group already, so one kernel does the whole verify: each group reads its frame's 32-byte
// header (the first line of the frame, fetched anyway for the payload) and computes the header CRC,
// folds the payload from it, and compares digest and ids — no header pass over 1M scattered lines,
// no plan, no finish launch. The gate runs first: it stores `vepoch` into *vflag when some frame is
// out of band, and then the header / plan / finish sequence runs instead while this kernel returns.
__global__ void __launch_bounds__(1024) verify_gate_kernel(const uint32_t* __restrict__ lengths, uint64_t n,
                                                          uint64_t* __restrict__ first_bad, uint32_t* __restrict__ vflag,
                                                          uint32_t vepoch) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *first_bad = n;
    const uint32_t ref = lengths[0];
    bool out = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out |= !PlanRun::in_band(lengths[i], ref);
    if (__any(out) && (threadIdx.x & 63) == 0) *vflag = vepoch;  // plain stores of one value: no atomics
}

// Fused package payloads (DigestManager.computeDigestAndPackageForSending, DigestManager.java:
// 117-181): one payload per lane group. Every lane of the group builds the entry's 32-byte BE header
// from the index arrays (ledger id, entry id, LAC, length: :146-149; one request per group per
// field) and folds it with the x^32 operator from ~0 — update(0, header), :152 — the register the
// payload then resumes from (:153), as crc_verify_fused_kernel does for a stored header. Only the
// finalized digest is stored here (digests[i], a wave's groups writing consecutive words); the
// frames' header and digest bytes are written afterwards by package_frame_kernel, so no lone frame
// store lands between this kernel's streaming payload reads. Out-of-range payloads: digest 0 and the
// stream's bounds flag, as the indexed path reports them.
template <int G, int PF, bool NT>
__global__ void __launch_bounds__(kBlock) crc_package_fused_kernel(
    const uint8_t* __restrict__ base, uint64_t size, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint64_t n, int64_t ledger_id, const int64_t* __restrict__ entry_ids,
    const int64_t* __restrict__ lacs, const int64_t* __restrict__ length_fields, const uint32_t* __restrict__ tables,
    uint32_t* __restrict__ digests, uint32_t* __restrict__ err, int sched) {
    using Gm = Geo<G>;
    __shared__ __attribute__((aligned(16))) uint32_t lds[Gm::kLdsWords];
    const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    stage_tables<G>(lds, tables);
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    const bool low_clock = lds_image_at_zero(lds) &&
                           (sched == 2 || (sched == 0 && BKD_CLOCK_ADAPT &&
                                           (clk1 - clk0) * 100u < (rt1 - rt0) * (uint64_t)kLowClockMHz));
    const int lane = threadIdx.x & 63;
    const int g = lane & (G - 1);
    const uint32_t lanereg = ((uint32_t)(lane & 31) << 2) | (1u << 16);
    const uint64_t ngroups = (uint64_t)gridDim.x * (kBlock / G);
    const uint64_t gid = (uint64_t)blockIdx.x * (kBlock / G) + (uint64_t)(threadIdx.x / G);
#if BKD_HOLD_STORE > 0
    HeldResults<G, BKD_HOLD_STORE> held;
#endif
    for (uint64_t i = gid; i < n; i += ngroups) {
        const uint64_t o = offsets[i];
        const uint32_t l = lengths[i];
        const uint64_t f4[4] = {(uint64_t)ledger_id, (uint64_t)entry_ids[i], (uint64_t)lacs[i],
                                (uint64_t)length_fields[i]};
        uint32_t d;
        if (o > size || (uint64_t)l > size - o) {
            d = 0u;
            if (g == 0 && err) atomicOr(err, 1u);
        } else {
            // update(0, header): BE fields, high word first, folded by the x^32 operator from ~0 —
            // evaluated by fold_range after the payload's first loads are issued (LateSeed)
            auto header_reg = [&]() {
                uint32_t reg = 0xFFFFFFFFu;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    reg = mul_aux(lds, Gm::kX32Off, reg ^ __builtin_bswap32((uint32_t)(f4[k] >> 32)));
                    reg = mul_aux(lds, Gm::kX32Off, reg ^ __builtin_bswap32((uint32_t)f4[k]));
                }
                return reg;
            };
            uint32_t v;
            if (l < 16u) {  // short payload: serial bytes (ReflectedIntCrc.java:44-48 form)
                v = header_reg();
                for (const uint8_t* q = base + o; q < base + o + l; ++q)
                    v = lds_word(lds, Gm::kByteTabOff + (((v ^ *q) & 0xffu) << 2)) ^ (v >> 8);
            } else {
                const int64_t s = (int64_t)o, e = s + (int64_t)l;
                const LateSeed<decltype(header_reg)> late{header_reg};
                v = low_clock ? fold_range<G, PF, NT, false, BKD_TAIL_UNCOND != 0, true>(lds, lanereg, g, base, s, e, late)
                              : fold_range<G, PF, NT, false, BKD_TAIL_UNCOND != 0, false>(lds, lanereg, g, base, s, e, late);
            }
            d = ~v;
        }
#if BKD_HOLD_STORE > 0
        held.put(d, g, digests, gid, ngroups, n);
#else
        if (g == 0) digests[i] = d;
#endif
    }
#if BKD_HOLD_STORE > 0
    held.finish(g, digests, gid, ngroups, n);
#endif
}

template <int G, int PF, bool NT>
__global__ void __launch_bounds__(kBlock) crc_verify_fused_kernel(
    const uint8_t* __restrict__ base, uint64_t size, const uint64_t* __restrict__ offsets,
    const uint32_t* __restrict__ lengths, uint64_t n, uint32_t mac, int64_t ledger_id, int64_t first_entry_id,
    int id_checks, const uint32_t* __restrict__ tables, int32_t* __restrict__ status,
    unsigned long long* __restrict__ first_bad, const uint32_t* __restrict__ vflag, uint32_t vepoch, int sched) {
    using Gm = Geo<G>;
    if (*vflag == vepoch) return;  // some frame out of band: the header / plan / finish sequence runs
    __shared__ __attribute__((aligned(16))) uint32_t lds[Gm::kLdsWords];
    // payload fold schedule from the shader clock over the table staging (as crc_groups_kernel)
    const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    stage_tables<G>(lds, tables);
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    const bool low_clock = lds_image_at_zero(lds) &&
                           (sched == 2 || (sched == 0 && BKD_CLOCK_ADAPT &&
                                           (clk1 - clk0) * 100u < (rt1 - rt0) * (uint64_t)kLowClockMHz));
    const int lane = threadIdx.x & 63;
    const int g = lane & (G - 1);
    const uint32_t lanereg = ((uint32_t)(lane & 31) << 2) | (1u << 16);
    const uint64_t ngroups = (uint64_t)gridDim.x * (kBlock / G);
    const uint64_t gid = (uint64_t)blockIdx.x * (kBlock / G) + (uint64_t)(threadIdx.x / G);
#if BKD_HOLD_STORE > 0
    HeldResults<G, BKD_HOLD_STORE> held;
#endif
    for (uint64_t i = gid; i < n; i += ngroups) {
        const uint64_t o = offsets[i];
        const uint32_t l = lengths[i];
        int32_t st;
        if (o > size || (uint64_t)l > size - o || l < 32u + mac) {
            st = 1;  // VERIFY_TOO_SHORT (verify_header_kernel's rule for frames outside the buffer too)
        } else {
            const uint8_t* f = base + o;
            // every lane of the group reads the header (same addresses: one request per group) and
            // folds it with the x^32 operator: update(0, header) = register ~0 through 8 dwords
            const u32x4 h0 = ld16<false>(f), h1 = ld16<false>(f + 16);
            const uint32_t hw[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
            uint32_t reg = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < 8; ++k) reg = mul_aux(lds, Gm::kX32Off, reg ^ hw[k]);
            const int64_t s = (int64_t)(o + 32u + mac), e = (int64_t)(o + l);
            uint32_t v;
            if (e - s < 16) {  // short payload: serial bytes (ReflectedIntCrc.java:44-48 form)
                v = reg;
                for (const uint8_t* q = base + s; q < base + e; ++q)
                    v = lds_word(lds, Gm::kByteTabOff + (((v ^ *q) & 0xffu) << 2)) ^ (v >> 8);
            } else {
                v = low_clock ? fold_range<G, PF, NT, false, BKD_TAIL_UNCOND != 0, true>(lds, lanereg, g, base, s, e, reg)
                              : fold_range<G, PF, NT, false, BKD_TAIL_UNCOND != 0, false>(lds, lanereg, g, base, s, e, reg);
            }
            const uint32_t computed = ~v;
            // digest: 4-byte BE int (CRC32C) or 8-byte BE zero-extended long (CRC32) at offset 32
            uint32_t expect, hi = 0u;
            if (mac == 8u) {
                hi = __builtin_bswap32(*reinterpret_cast<const uint32_t*>(f + 32));
                expect = __builtin_bswap32(*reinterpret_cast<const uint32_t*>(f + 36));
            } else {
                expect = __builtin_bswap32(*reinterpret_cast<const uint32_t*>(f + 32));
            }
            const int64_t lid = (int64_t)(((uint64_t)__builtin_bswap32(hw[0]) << 32) | __builtin_bswap32(hw[1]));
            const int64_t eid = (int64_t)(((uint64_t)__builtin_bswap32(hw[2]) << 32) | __builtin_bswap32(hw[3]));
            // DigestManager.verifyDigest's order (DigestManager.java:226-283): digest, ledger id, entry id
            if (hi != 0u || computed != expect) st = 2;
            else if (id_checks < 2 && lid != ledger_id) st = 3;
            else if (id_checks == 0 && eid != first_entry_id + (int64_t)i) st = 4;
            else st = 0;
        }
#if BKD_HOLD_STORE > 0
        held.put((uint32_t)st, g, reinterpret_cast<uint32_t*>(status), gid, ngroups, n);
        if (g == 0 && st != 0) atomicMin(first_bad, (unsigned long long)i);
#else
        if (g == 0) {
            status[i] = st;
            if (st != 0) atomicMin(first_bad, (unsigned long long)i);
        }
#endif
    }
#if BKD_HOLD_STORE > 0
    held.finish(g, reinterpret_cast<uint32_t*>(status), gid, ngroups, n);
#endif
}

}  // namespace bkd
