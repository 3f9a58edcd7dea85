// The stream route for ragged indexed batches (DESIGN.md §3 "Stream route"; CPU model of the same
// decomposition, step by step: tests/stream_model.py RangeModel, checked against the oracle on
// packed, gappy, unsorted and overlapping indexes).
//
// The entries' 128-byte device lines are laid end to end in index order: entry i takes the next J'
// positions of the stream, J' = its lines minus one when its first line is the previous entry's
// last (that line is folded once, into both). Positions are a plain prefix sum of J'. Group r of the
// tile kernel folds the positions [r TL, (r + 1) TL), TL = ceil(end / groups): each line is loaded
// once and folded into every entry it holds, the bytes outside an entry zeroed in the very register
// that is folded. An entry inside one range gets its raw register there; the pieces of a longer
// entry (one raw register per range) are joined by stream_combine_kernel with x^(1024 TL) per range
// and x^(1024 L) for its last L lines, then x^(-8 pad).
//
// Three launches, no host sync: plan_stream_kernel (positions: per-block sums and a decoupled
// look-back across blocks, then each entry's position and record) -> crc_stream_ranges_kernel ->
// stream_combine_kernel. Chunked-plan equivalent: crc32c_sse42.cpp:92-134 cuts one buffer into
// chunks folded in parallel and merged by shift tables; here a batch's entries are cut into equal
// ranges of lines across the whole chip and merged the same way.
#pragma once
#include "plan_kernels.hpp"

namespace bkd {

#ifndef BKD_STREAM
#define BKD_STREAM 1  // 0: ragged batches keep the chunked plan (A/B builds)
#endif
#ifndef BKD_STREAM_FINISH_PROBE
#define BKD_STREAM_FINISH_PROBE 0  // 1: measurement-only build, an entry's finish is an XOR (wrong digests)
#endif
constexpr uint32_t kLbEpochMask = (1u << 22) - 1u;  // tag bits of a look-back word (StreamScratch::lookback_words)
constexpr uint64_t kStreamMaxTL = 1ull << 22;  // lines per range (above: every entry whole, one per group)

struct StreamArgs {
    uint64_t* sdesc;   // [nb] look-back words of the entry blocks: tag | status | value (a region of their own)
    uint64_t* shdr;    // [0] the stream's end (positions)
    uint64_t* spos;    // [n] V (first new line's position) | shared << 62 | outside the stream << 63
    u32x4* srec;       // [n] the entry for the range kernel: {F, J, d | eL << 8 | in << 16, ~seed}
    uint32_t* pfirst;  // [ngroups] raw register of a range's first piece (its entry began before it)
    uint32_t* plast;   // [ngroups] raw register of a range's last piece (its entry goes on after it)
    uint32_t* ticket;  // entry-block ticket of plan_stream_kernel (0 between calls: its last block resets it)
    uint32_t ngroups;  // ranges = 8-lane groups of the tile kernel
    uint32_t mis;      // device address of base modulo 128
    uint32_t epoch;    // the call's look-back tag (words of earlier calls never carry it)
    uint64_t maxtl;    // lines per range above which every entry is taken whole (kStreamMaxTL; tests lower it)
};

__host__ __device__ __forceinline__ uint64_t stream_range_len(uint64_t end, uint64_t ngroups) {
    uint64_t tl = (end + ngroups - 1u) / ngroups;
    if (tl == 0u) tl = 1u;
    return (tl + 7u) & ~7ull;  // a multiple of the range loop's body (two rounds of four line sets)
}

// Stream geometry of one entry (stream_model.Geo).
struct SEnt {
    uint64_t F, Lst;  // first and last device line
    uint32_t d, pad;  // bytes of its first line before the entry; bytes of its last line after it
    bool in;          // in the stream: valid, non-empty, padded message of >= 4 bytes (the seed image)
};

__device__ __forceinline__ SEnt stream_ent(uint64_t o, uint32_t l, uint64_t size, uint32_t mis) {
    SEnt e;
    const uint64_t as = (uint64_t)mis + o, ae = as + l;
    e.F = as >> 7;
    e.Lst = l ? (ae - 1u) >> 7 : e.F;
    e.d = (uint32_t)(as & 127u);
    e.pad = (128u - (uint32_t)(ae & 127u)) & 127u;
    e.in = !(o > size || (uint64_t)l > size - o) && l != 0u && l + e.pad >= 4u;
    return e;
}

// ---- positions: plan_stream_kernel ----
// look-back word: tag (22 bits, the call's kLbEpochMask bits) | status (2: 1 = block aggregate,
// 2 = inclusive prefix; 0 = not written) | value (40 bits: a prefix of lines, < 2^31 below 2^38 bytes)
__device__ __forceinline__ uint64_t sd_pack(uint32_t epoch, uint32_t st, uint64_t v) {
    return ((uint64_t)(epoch & kLbEpochMask) << 42) | ((uint64_t)st << 40) | (v & ((1ull << 40) - 1u));
}
__device__ __forceinline__ uint32_t sd_tag(uint64_t w) { return (uint32_t)(w >> 42); }
__device__ __forceinline__ uint32_t sd_status(uint64_t w) { return (uint32_t)(w >> 40) & 3u; }
__device__ __forceinline__ uint64_t sd_value(uint64_t w) { return w & ((1ull << 40) - 1u); }

// One 1024-thread block per entry block, taken by ticket in the order the blocks start (so a block
// waiting on its predecessors waits only for blocks already running). Per entry: in the stream?, shared with the
// previous entry?, J'; a block scan; the block's aggregate published at once, then a look-back by
// wave 0 over the preceding blocks' words (64 at a time: aggregates summed until an inclusive prefix)
// and the block's own prefix published. The look-back words are device-scope atomics: the value
// travels in the word that carries its status, so no fence or cache write-back is needed on this
// multi-XCD part. Then each entry's position and record; the last block writes the end.
__global__ void __launch_bounds__(kPlanBlock) plan_stream_kernel(const uint64_t* __restrict__ offsets,
                                                                 const uint32_t* __restrict__ lengths,
                                                                 const uint32_t* __restrict__ seeds, uint32_t seed_all,
                                                                 uint64_t size, uint64_t n, uint32_t nb, StreamArgs sa) {
    __shared__ uint64_t wtot[kPlanBlock / 64];
    __shared__ uint64_t s_prefix;
    __shared__ uint32_t s_eb;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t ep = sa.epoch & kLbEpochMask;
    if (threadIdx.x == 0) {
        // one ticket per block; the block taking the last one resets the counter for the next call
        // (a wrong start value could only misorder the blocks, never index past them)
        const uint32_t t = atomicAdd(sa.ticket, 1u);
        if (t == nb - 1u) __hip_atomic_store(sa.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_eb = t < nb ? t : t % nb;
    }
    __syncthreads();
    {
        const uint32_t eb = s_eb;
        const uint64_t i = (uint64_t)eb * kPlanBlock + threadIdx.x;
        const uint64_t o = i < n ? offsets[i] : 0u;
        const uint32_t l = i < n ? lengths[i] : 0u;
        uint64_t po = (uint64_t)__shfl_up((unsigned long long)o, 1);
        uint32_t pl = (uint32_t)__shfl_up((int)l, 1);
        if (lane == 0 && i > 0u && i - 1u < n) {
            po = offsets[i - 1u];
            pl = lengths[i - 1u];
        }
        SEnt e = stream_ent(o, l, size, sa.mis);
        if (i >= n) e.in = false;
        bool sh = false;
        if (e.in && i > 0u) {
            const SEnt p = stream_ent(po, pl, size, sa.mis);
            sh = p.in && e.F == p.Lst;
        }
        const uint64_t jn = e.in ? e.Lst - e.F + 1u - (sh ? 1u : 0u) : 0u;
        // block inclusive scan of jn
        uint64_t v = jn;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = (uint64_t)__shfl_up((unsigned long long)v, d);
            if (lane >= d) v += y;
        }
        if (lane == 63) wtot[wave] = v;
        __syncthreads();
        uint64_t wpre = 0u, agg = 0u;
        for (int k = 0; k < kPlanBlock / 64; ++k) {
            const uint64_t t = wtot[k];
            wpre += k < wave ? t : 0u;
            agg += t;
        }
        if (wave == 0) {  // publish the aggregate, look back, publish the prefix
            if (lane == 0)
                __hip_atomic_store(&sa.sdesc[eb], sd_pack(ep, eb ? 1u : 2u, agg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            uint64_t prefix = 0u;
            int64_t top = (int64_t)eb - 1;  // the look-back window ends at block `top`
            while (top >= 0) {
                const int64_t p = top - lane;
                uint64_t w = 0u;
                bool ready = true;
                if (p >= 0) {
                    w = __hip_atomic_load(&sa.sdesc[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ready = sd_tag(w) == ep && sd_status(w) != 0u;
                }
                // the nearest inclusive prefix in the window (lanes in order of distance)
                const uint64_t pmask = __ballot(p >= 0 && ready && sd_status(w) == 2u);
                const int stop = pmask ? __builtin_ctzll(pmask) : 64;
                // every word up to it must be there; otherwise wait and read the window again
                const uint64_t rmask = __ballot(ready);
                const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1u);
                if ((rmask & need) != need) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint64_t part = (p >= 0 && lane <= stop) ? sd_value(w) : 0u;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) part += (uint64_t)__shfl_xor((unsigned long long)part, d);
                prefix += part;
                if (stop < 64) break;
                top -= 64;
            }
            if (lane == 0) {
                if (eb)
                    __hip_atomic_store(&sa.sdesc[eb], sd_pack(ep, 2u, prefix + agg), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                s_prefix = prefix;
                if (eb == nb - 1u) sa.shdr[0] = prefix + agg;
            }
        }
        __syncthreads();
        if (i < n) {
            const uint64_t V = s_prefix + wpre + v - jn;
            sa.spos[i] = V | ((uint64_t)sh << 62) | ((uint64_t)!e.in << 63);
            // F: first device line, J: lines after it, d: its first byte in line F, eL: bytes of its last
            // line it covers (1..128), in: in the stream
            const uint32_t J = (uint32_t)(e.Lst - e.F), d = e.d;
            const uint32_t eL = (uint32_t)((uint64_t)d + l - 128ull * J);
            sa.srec[i] = u32x4{(uint32_t)e.F, J, d | ((eL & 0xFFu) << 8) | ((uint32_t)e.in << 16),
                               ~(seeds ? seeds[i] : seed_all)};
        }
    }
}

// ---- the tile kernel ----
// Keeps bytes [a, b) of a 16-byte block (block coordinates, any range), zeroes the rest.
__device__ __forceinline__ u32x4 keep_range(u32x4 w, int32_t a, int32_t b) {
    auto m = [](uint32_t x, int32_t lo, int32_t hi) -> uint32_t {  // (selects, no branches)
        const int32_t a = lo < 0 ? 0 : lo, b = hi > 4 ? 4 : hi, wd = b - a;
        const uint32_t msk = (0xFFFFFFFFu >> ((uint32_t)(32 - 8 * wd) & 31u)) << ((uint32_t)(8 * a) & 31u);
        return wd > 0 ? x & msk : 0u;
    };
    w.x = m(w.x, a, b);
    w.y = m(w.y, a - 4, b - 4);
    w.z = m(w.z, a - 8, b - 8);
    w.w = m(w.w, a - 12, b - 12);
    return w;
}

// An entry as the fold needs it, relative to its range (positions: the range's first line = 0; its
// first line at pF, negative when it began in an earlier range; clamped to +-2^29, far enough): the
// steps of its first and last line, and per lane the byte masks of those lines (the first line's
// mask already ANDed with the last's for an entry of one line), the seed image (~seed XORed into
// its first four bytes) and the seed's spill into the next line (d > 124). Computed once per entry
// from its record (srec: F, J, d | eL << 8 | in << 16, ~seed) with 128-bit shifts.
struct SFold {
    int32_t sF, sL;
    uint32_t lst;      // device line of its last line (the next entry shares it if it starts there)
    u32x4 mA, mB;      // keep-masks of its first / last line
    u32x4 simg;        // seed image in its first line
    uint32_t spill;    // the seed image's bytes in the next line (lane 0, d > 124)
};

__device__ __forceinline__ u32x4 u128_from(uint64_t lo, uint64_t hi) {
    return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}
// bytes [k, 16) of a 16-byte block set (k clamped to 0..16): all-ones << 8k
__device__ __forceinline__ u32x4 mask_from(int32_t k) {
    const uint32_t s = 8u * (uint32_t)(k < 0 ? 0 : (k > 16 ? 16 : k));
    const uint64_t lo = s >= 64u ? 0ull : (~0ull << s);
    const uint64_t hi = s >= 128u ? 0ull : (s >= 64u ? (~0ull << (s - 64u)) : ~0ull);
    return u128_from(lo, hi);
}
// bytes [0, k) set (k clamped to 0..16): 2^(8k) - 1
__device__ __forceinline__ u32x4 mask_below(int32_t k) {
    const uint32_t b = 8u * (uint32_t)(k < 0 ? 0 : (k > 16 ? 16 : k));
    const uint64_t lo = b == 0u ? 0ull : (b >= 64u ? ~0ull : (~0ull >> (64u - b)));
    const uint64_t hi = b <= 64u ? 0ull : (~0ull >> (128u - b));
    return u128_from(lo, hi);
}

__device__ __forceinline__ void sfold_setup(SFold& f, const u32x4& rq, int64_t pF, int g) {
    const uint32_t J = rq.y, d = rq.z & 0xFFu, eL = (rq.z >> 8) & 0xFFu;
    auto cl = [](int64_t v) -> int32_t { return (int32_t)(v < -(1 << 29) ? -(1 << 29) : (v > (1 << 29) ? (1 << 29) : v)); };
    f.sF = cl(pF);
    f.sL = cl(pF + (int64_t)J);
    f.lst = rq.x + J;
    const int32_t b = 16 * g;
    f.mB = mask_below((int32_t)(eL == 0u ? 128u : eL) - b);
    const u32x4 ma = mask_from((int32_t)d - b);
    f.mA = J == 0u ? u32x4{ma.x & f.mB.x, ma.y & f.mB.y, ma.z & f.mB.z, ma.w & f.mB.w} : ma;
    // the seed image: ~seed (rq.w) at byte d of the line, i.e. at byte x = d - 16 g of this lane's
    // 16-byte block (x in -3 .. 15 touches it); bytes past the line go to the next line's lane 0
    const int32_t x = (int32_t)d - b;
    const uint64_t v = rq.w;
    uint64_t lo = 0u, hi = 0u;
    if (x >= 0 && x < 16) {
        const uint32_t t = 8u * (uint32_t)x;
        lo = t < 64u ? v << t : 0ull;
        hi = t == 0u ? 0ull : (t < 64u ? v >> (64u - t) : v << (t - 64u));
    } else if (x < 0 && x > -4) {
        lo = v >> (uint32_t)(-8 * x);
    }
    f.simg = u128_from(lo, hi);
    f.spill = (g == 0 && d > 124u) ? (uint32_t)(v >> (8u * (128u - d))) : 0u;
}

// The record's stream status, first and last device line.
struct SLines {
    uint32_t F, Lst;
    bool in;
};
__device__ __forceinline__ SLines slines(const u32x4& r) { return SLines{r.x, r.x + r.y, ((r.z >> 16) & 1u) != 0u}; }

// One range per 8-lane group. Four register sets hold the lines of the next four positions, loaded
// by a cursor that walks the entries' records four positions ahead of the fold (the device line of
// a position is its entry's first new line plus the steps since). Beside every line the group loads
// a window of the eight records after the cursor's entry, one per lane (`W`, base index `B`), used
// four steps later by the cursor and by the fold (an entry change takes its record with a group
// shuffle). Only when more than eight entries begin within four positions (entries of under half a
// line) is a record loaded on the spot, on a path that waits for itself. Every load of the common
// path is unconditional and at a fixed point of the step, so the compiler's memory waits stay
// counted (no drain of the lines in flight); the loop body is the four steps of one line set.
template <bool NT>
__device__ __forceinline__ void stream_ranges_loop(const uint32_t* lds, uint32_t lanereg, int g,
                                                   const uint8_t* __restrict__ base, uint64_t size,
                                                   const StreamArgs& sa, uint64_t n, uint64_t r, uint64_t TL,
                                                   uint64_t end, uint32_t* __restrict__ out) {
    const uint8_t* lb = base - sa.mis;  // device line 0 (the line holding base)
    const uint32_t lmax = (uint32_t)(((uint64_t)sa.mis + size - 1u) >> 7);
    const uint32_t mis = sa.mis;
    const int lane8 = (int)(threadIdx.x & 56u);  // the group's first lane in its wave
    const uint32_t n32 = (uint32_t)n;
    auto ld_line = [&](uint32_t L) { return ld16<NT>(lb + ((uint64_t)(L < lmax ? L : lmax) << 7) + 16 * g); };
    auto ld_rec = [&](uint32_t i) { return sa.srec[i < n32 ? i : n32 - 1u]; };
    auto vpos = [&](uint64_t j) { return sa.spos[j] & ((1ull << 62) - 1u); };

    const uint64_t R0 = r * TL;
    const bool act = R0 < end;
    const uint32_t nla = act ? (uint32_t)(end - R0 < TL ? end - R0 : TL) : 0u;
    // the range's first entry: the last j with V_j <= R0 (V is non-decreasing), 8-ary by the group
    uint64_t lo = 0u, hi = act ? n : 1u;
    while (__any(hi - lo > 1u)) {
        const uint64_t span = hi - lo, step = span > 1u ? (span + 7u) / 8u : 1u;
        const uint64_t probe = lo + (uint64_t)(g + 1) * step;
        const bool le = span > 1u && probe < hi && vpos(probe) <= R0;
        const uint32_t bits = (uint32_t)(__ballot(le) >> lane8) & 0xFFu;
        const uint32_t c = (uint32_t)__popc(bits);
        if (span > 1u) {
            const uint64_t nhi = lo + (uint64_t)(c + 1u) * step;
            lo += (uint64_t)c * step;
            hi = nhi < hi ? nhi : hi;
        }
    }
    const uint32_t j0 = (uint32_t)lo;
    const uint64_t sp0 = sa.spos[j0];
    const u32x4 rec0 = ld_rec(j0);
    const int64_t P0 = (int64_t)(sp0 & ((1ull << 62) - 1u)) - (int64_t)((sp0 >> 62) & 1u);  // its first line
    // fold state
    uint32_t i = j0;
    SFold f;
    sfold_setup(f, rec0, P0 - (int64_t)R0, g);
    const SLines q0 = slines(rec0);
    bool from_start = P0 >= (int64_t)R0, live = act, pin = true;
    uint32_t c0 = 0u, c1 = 0u, c2 = 0u, c3 = 0u;
    // cursor: entry cj, device line cL of its position, crem new lines of cj after it, cpin: the
    // index before the next one looked at is in the stream
    uint32_t cj = j0, cL = q0.F + (uint32_t)((int64_t)R0 - P0), crem = q0.Lst - cL;
    bool cpin = true;
    // the cursor's next position (records from window (WS, BS), or loaded on the spot)
    auto advance = [&](const u32x4& WS, uint32_t BS) {
        if (crem > 0u) {
            ++cL;
            --crem;
            return;
        }
        for (;;) {  // group-uniform
            const uint32_t j = cj + 1u;
            if (j >= n32) {  // past the last entry: a clamped line, never folded
                cj = n32;
                break;
            }
            const uint32_t k = j - BS;
            u32x4 rq;
            if (k < 8u) {
                const int src = lane8 + (int)k;
                rq.x = (uint32_t)__shfl((int)WS.x, src);
                rq.y = (uint32_t)__shfl((int)WS.y, src);
                rq.z = (uint32_t)__shfl((int)WS.z, src);
                rq.w = (uint32_t)__shfl((int)WS.w, src);
            } else {
                rq = ld_rec(j);
                asm volatile("s_waitcnt vmcnt(0)" : "+v"(rq.x), "+v"(rq.y), "+v"(rq.z), "+v"(rq.w));
            }
            cj = j;
            const SLines q = slines(rq);
            if (!q.in) {
                cpin = false;
                continue;
            }
            const bool sh = cpin && q.F == cL;
            cpin = true;
            if (sh && q.Lst == q.F) continue;  // inside the current line: no position of its own
            cL = q.F + (sh ? 1u : 0u);
            crem = q.Lst - cL;
            break;
        }
    };
    // prologue: the range's first four positions (records loaded on the spot: a window based past
    // the end forces it), and the first round's record window
    const u32x4 none{0u, 0u, 0u, 0u};
    u32x4 WA = ld_rec(cj + 1u + (uint32_t)g), WB;
    uint32_t BA = cj + 1u, BB;
    u32x4 X0 = ld_line(cL);
    advance(none, 0xFFFFFFF0u);
    u32x4 X1 = ld_line(cL);
    advance(none, 0xFFFFFFF0u);
    u32x4 X2 = ld_line(cL);
    advance(none, 0xFFFFFFF0u);
    u32x4 X3 = ld_line(cL);

    const u32x4 ones{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    // The next entry of the stream after i, from the window (WS, BS) or loaded on the spot (group-
    // uniform): its fold setup at the position after `sv`, or at `sv` itself when it starts in the
    // line where i ended (returns true then). live = false past the last entry.
    auto next_entry = [&](const u32x4& WS, uint32_t BS, int32_t sv) -> bool {
        const uint32_t plst = f.lst;
        for (;;) {
            ++i;
            if (i >= n32) {
                live = false;
                return false;
            }
            const uint32_t k = i - BS;
            u32x4 rq;
            if (k < 8u) {
                const int src = lane8 + (int)k;
                rq.x = (uint32_t)__shfl((int)WS.x, src);
                rq.y = (uint32_t)__shfl((int)WS.y, src);
                rq.z = (uint32_t)__shfl((int)WS.z, src);
                rq.w = (uint32_t)__shfl((int)WS.w, src);
            } else {
                rq = ld_rec(i);
                asm volatile("s_waitcnt vmcnt(0)" : "+v"(rq.x), "+v"(rq.y), "+v"(rq.z), "+v"(rq.w));
            }
            const SLines q = slines(rq);
            if (!q.in) {
                pin = false;
                continue;
            }
            const bool sh = pin && q.F == plst;
            pin = true;
            sfold_setup(f, rq, (int64_t)sv + (sh ? 0 : 1), g);
            return sh;
        }
    };

    // One step: position s of the range, line XS. The common path is masks by select and the fold;
    // an entry that ends in this line takes the rare path (its finish, then every entry that starts
    // in this same line: its first fold is the masked line itself, no product).
#define BKD_STREAM_STEP(XS, WS, BS, S)                                                                \
    {                                                                                                 \
        const uint32_t s_ = (S);                                                                      \
        const int32_t sv = (int32_t)s_;                                                               \
        const bool act_ = live && s_ < nla;                                                           \
        const bool first = sv == f.sF, last = sv == f.sL, spst = sv == f.sF + 1;                      \
        if (__all(act_ && s_ + 1u < nla && !first && !last && !spst)) {                              \
            /* wave-uniform fast path: every group inside an entry's inner lines */                  \
            c0 = mul_main_add(lds, c0, lanereg, XS.x);                                                \
            c1 = mul_main_add(lds, c1, lanereg, XS.y);                                                \
            c2 = mul_main_add(lds, c2, lanereg, XS.z);                                                \
            c3 = mul_main_add(lds, c3, lanereg, XS.w);                                                \
        } else {                                                                                      \
            /* the line masked to entry i's bytes, its seed image on its first line; c is 0 before */ \
            /* an entry's first line, so its first fold is the masked line itself (a group past */   \
            /* its last position folds garbage it never uses: the range's end was taken below) */    \
            const u32x4 m = first ? f.mA : (last ? f.mB : ones);                                      \
            c0 = mul_main_add(lds, c0, lanereg, (XS.x & m.x) ^ (first ? f.simg.x : (spst ? f.spill : 0u))); \
            c1 = mul_main_add(lds, c1, lanereg, (XS.y & m.y) ^ (first ? f.simg.y : 0u));             \
            c2 = mul_main_add(lds, c2, lanereg, (XS.z & m.z) ^ (first ? f.simg.z : 0u));             \
            c3 = mul_main_add(lds, c3, lanereg, (XS.w & m.w) ^ (first ? f.simg.w : 0u));             \
            if (act_ && last) { /* rare: entry i ends in this line */                                \
                for (;;) {                                                                            \
                    const uint32_t reg = BKD_STREAM_FINISH_PROBE ? (c0 ^ c1 ^ c2 ^ c3) : finish_lanes<8>(lds, c0, c1, c2, c3);                        \
                    if (g == 0) {                                                                     \
                        if (from_start) out[i] = reg;                                                 \
                        else sa.pfirst[r] = reg;                                                      \
                    }                                                                                 \
                    from_start = true;                                                                \
                    c0 = c1 = c2 = c3 = 0u;                                                           \
                    if (!next_entry(WS, BS, sv)) break; /* it starts in the next line */             \
                    /* it starts in this line: its first fold is the line masked, seed XORed in */   \
                    c0 = (XS.x & f.mA.x) ^ f.simg.x;                                                  \
                    c1 = (XS.y & f.mA.y) ^ f.simg.y;                                                  \
                    c2 = (XS.z & f.mA.z) ^ f.simg.z;                                                  \
                    c3 = (XS.w & f.mA.w) ^ f.simg.w;                                                  \
                    if (f.sL != sv) break; /* and goes on into the next line */                       \
                }                                                                                     \
            }                                                                                         \
            if (live && s_ + 1u == nla && f.sF <= sv) { /* the range ends inside entry i */          \
                const uint32_t reg = BKD_STREAM_FINISH_PROBE ? (c0 ^ c1 ^ c2 ^ c3) : finish_lanes<8>(lds, c0, c1, c2, c3);                            \
                if (g == 0) {                                                                         \
                    if (from_start) sa.plast[r] = reg;                                                \
                    else sa.pfirst[r] = reg;                                                          \
                }                                                                                     \
            }                                                                                         \
        }                                                                                             \
        /* the cursor moves to position s + 4 (with this round's window) and the slot is refilled */ \
        if (crem > 0u) {                                                                              \
            ++cL;                                                                                     \
            --crem;                                                                                   \
        } else {                                                                                      \
            advance(WS, BS);                                                                          \
        }                                                                                             \
        XS = ld_line(cL);                                                                             \
    }

    // Rounds of four steps, two per iteration (the record windows alternate without a copy): each
    // round loads the next round's window (the eight records after the cursor's entry) first.
    const uint32_t tl32 = (uint32_t)TL;
    for (uint32_t s0 = 0u; s0 < tl32; s0 += 8u) {  // TL: kernel-uniform, a multiple of 8
        BB = cj + 1u;
        WB = ld_rec(BB + (uint32_t)g);
        BKD_STREAM_STEP(X0, WA, BA, s0)
        BKD_STREAM_STEP(X1, WA, BA, s0 + 1u)
        BKD_STREAM_STEP(X2, WA, BA, s0 + 2u)
        BKD_STREAM_STEP(X3, WA, BA, s0 + 3u)
        BA = cj + 1u;
        WA = ld_rec(BA + (uint32_t)g);
        BKD_STREAM_STEP(X0, WB, BB, s0 + 4u)
        BKD_STREAM_STEP(X1, WB, BB, s0 + 5u)
        BKD_STREAM_STEP(X2, WB, BB, s0 + 6u)
        BKD_STREAM_STEP(X3, WB, BB, s0 + 7u)
    }
#undef BKD_STREAM_STEP
}

// 8-lane groups, one range each (grid = ngroups / 128 blocks). A stream longer than kStreamMaxTL
// lines per range (only a batch of heavily overlapping huge entries) takes every entry whole, one
// per group, and the combine then does nothing but the entries outside the stream.
template <bool NT>
__global__ void __launch_bounds__(kBlock) crc_stream_ranges_kernel(const uint8_t* __restrict__ base, uint64_t size,
                                                                   const uint64_t* __restrict__ offsets,
                                                                   const uint32_t* __restrict__ lengths,
                                                                   const uint32_t* __restrict__ seeds, uint32_t seed_all,
                                                                   uint64_t n, const uint32_t* __restrict__ tables,
                                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ err,
                                                                   StreamArgs sa) {
    using Gm = Geo<8>;
    const uint64_t end = sa.shdr[0];
    if (end == 0u || size == 0u) return;  // no entry in the stream: the combine does them all
    __shared__ __attribute__((aligned(16))) uint32_t lds[Gm::kLdsWords];
    stage_tables<8>(lds, tables);
    const int lane = threadIdx.x & 63;
    const uint32_t lanereg = ((uint32_t)(lane & 31) << 2) | (1u << 16);
    const uint64_t ngroups = (uint64_t)gridDim.x * (kBlock / 8);
    const uint64_t gid = (uint64_t)blockIdx.x * (kBlock / 8) + (uint64_t)(threadIdx.x / 8);
    const uint64_t TL = stream_range_len(end, ngroups);
    if (TL > sa.maxtl) {  // (kernel-uniform)
        const IndexedSrc src{n, offsets, lengths, seeds, seed_all, size, out};
        groups_loop<8, 2, NT>(lds, lanereg, lane & 7, base, src, n, gid, ngroups, err);
        return;
    }
    stream_ranges_loop<NT>(lds, lanereg, lane & 7, base, size, sa, n, gid, TL, end, out);
}

// ---- the combine ----
// One thread per entry: entries outside the stream (empty, out of range, a padded message under
// 4 bytes) folded serially; an entry inside one range: pad product and inversion of its raw
// register; a longer entry: its pieces joined, plast[t0], pfirst[t0 + 1 .. t1] (Horner with
// X = x^(1024 TL), the last piece's weight x^(1024 L)), then x^(-8 pad). Powers come from two
// 64-entry tables in LDS, x^(1024 * 2^k) (xpw, from the host) and X^(2^k) (built from it for this
// TL), so a power costs one product per set bit of its exponent. Entries of more than
// kStreamSerialPieces pieces are joined afterwards by one wave each (lanes split the pieces).
constexpr uint32_t kStreamSerialPieces = 64;

__global__ void __launch_bounds__(1024, BKD_PLAN_OCC) stream_combine_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets, const uint32_t* __restrict__ lengths,
    const uint32_t* __restrict__ seeds, uint32_t seed_all, uint64_t size, uint64_t n, uint32_t nb,
    const uint32_t* __restrict__ btab, const uint32_t* __restrict__ xinv, uint32_t poly,
    const uint32_t* __restrict__ xpw, StreamArgs sa, uint32_t* __restrict__ out, uint32_t* __restrict__ err) {
    __shared__ uint32_t T[16 * 256];  // slice-by-16 (serial entries)
    __shared__ uint32_t big[1024];
    __shared__ uint32_t pwL[64], pwX[64];
    __shared__ uint32_t nbig;
    const uint64_t end = sa.shdr[0];
    const uint64_t TL = stream_range_len(end, sa.ngroups);
    const bool whole = end != 0u && TL > sa.maxtl;  // the range kernel took every entry whole
    build_slice16(T, btab);
    if (threadIdx.x < 64) pwL[threadIdx.x] = xpw[threadIdx.x];
    __syncthreads();
    if (threadIdx.x < 64) {  // X^(2^k) = x^(1024 TL 2^k): one product per set bit of TL
        const uint32_t k = threadIdx.x;
        uint32_t r = 0x80000000u;  // x^0
        for (uint32_t b = 0; b + k < 64u && b < 64u; ++b)
            if ((TL >> b) & 1u) r = gf_mul_bits(r, pwL[b + k], poly);
        pwX[k] = r;
    }
    __syncthreads();
    auto pow_tab = [&](const uint32_t* pw, uint64_t e) {
        uint32_t r = 0x80000000u;
        for (uint32_t b = 0; e; ++b, e >>= 1)
            if (e & 1u) r = gf_mul_bits(r, pw[b], poly);
        return r;
    };
    const uint32_t X = pwX[0];
    for (uint32_t eb = blockIdx.x; eb < nb; eb += gridDim.x) {
        if (threadIdx.x == 0) nbig = 0u;
        __syncthreads();
        const uint64_t i = (uint64_t)eb * 1024u + threadIdx.x;
        if (i < n && !whole) {
            const uint64_t sp = sa.spos[i];
            const uint64_t o = offsets[i];
            const uint32_t l = lengths[i];
            if (sp >> 63) {
                if (!entry_valid(o, l, size)) {
                    out[i] = 0u;
                    if (err) atomicOr(err, 1u);
                } else {
                    const uint32_t reg = ~(seeds ? seeds[i] : seed_all);
                    out[i] = l ? ~serial_crc(base, o, l, reg, T) : ~reg;
                }
            } else {
                const SEnt e = stream_ent(o, l, size, sa.mis);
                const uint64_t P0 = (sp & ((1ull << 62) - 1u)) - ((sp >> 62) & 1u), P1 = P0 + (e.Lst - e.F);
                const uint64_t t0 = P0 / TL, t1 = P1 / TL, m = t1 - t0;
                if (m == 0u) {
                    const uint32_t raw = out[i];
                    out[i] = ~(e.pad ? gf_mul_bits(xinv[e.pad], raw, poly) : raw);
                } else if (m <= kStreamSerialPieces) {
                    uint32_t reg = sa.plast[t0];
                    for (uint64_t t = t0 + 1u; t < t1; t += 8u) {  // pieces loaded eight at a time
                        uint32_t pv[8];
#pragma unroll
                        for (int q = 0; q < 8; ++q) pv[q] = t + q < t1 ? sa.pfirst[t + q] : 0u;
#pragma unroll
                        for (int q = 0; q < 8; ++q)
                            if (t + q < t1) reg = gf_mul_bits(X, reg, poly) ^ pv[q];
                    }
                    reg = gf_mul_bits(pow_tab(pwL, P1 - t1 * TL + 1u), reg, poly) ^ sa.pfirst[t1];
                    out[i] = ~(e.pad ? gf_mul_bits(xinv[e.pad], reg, poly) : reg);
                } else {
                    big[atomicAdd(&nbig, 1u)] = threadIdx.x;
                }
            }
        }
        __syncthreads();
        // entries of many pieces: one wave each, the lanes' Horner runs placed by X^(run start)
        const uint32_t nbg = nbig, lane = threadIdx.x & 63u, nwaves = blockDim.x >> 6;
        for (uint32_t k = threadIdx.x >> 6; k < nbg; k += nwaves) {  // wave-uniform
            const uint64_t ie = (uint64_t)eb * 1024u + big[k];
            const SEnt e = stream_ent(offsets[ie], lengths[ie], size, sa.mis);
            const uint64_t sp = sa.spos[ie];
            const uint64_t P0 = (sp & ((1ull << 62) - 1u)) - ((sp >> 62) & 1u), P1 = P0 + (e.Lst - e.F);
            const uint64_t t0 = P0 / TL, t1 = P1 / TL;
            const uint32_t m = (uint32_t)(t1 - t0);  // pieces before the last: c = 0 .. m - 1, weight X^c
            auto piece = [&](uint32_t c) { return c + 1u == m ? sa.plast[t0] : sa.pfirst[t1 - 1u - c]; };
            const uint32_t per = (m + 63u) >> 6, lo = lane * per, hi = lo + per < m ? lo + per : m;
            uint32_t rr = 0u;
            // pieces loaded eight at a time ahead of their products (one memory round trip per
            // eight pieces instead of one per piece)
            for (int c0 = (int)hi - 1; c0 >= (int)lo; c0 -= 8) {
                uint32_t pv[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) pv[q] = c0 - q >= (int)lo ? piece((uint32_t)(c0 - q)) : 0u;
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (c0 - q >= (int)lo) rr = gf_mul_bits(X, rr, poly) ^ pv[q];
            }
            if (lo < hi && lo) rr = gf_mul_bits(pow_tab(pwX, lo), rr, poly);
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) rr ^= (uint32_t)__shfl_xor((int)rr, d);
            if (lane == 0u) {
                const uint32_t reg = gf_mul_bits(pow_tab(pwL, P1 - t1 * TL + 1u), rr, poly) ^ sa.pfirst[t1];
                out[ie] = ~(e.pad ? gf_mul_bits(xinv[e.pad], reg, poly) : reg);
            }
        }
        __syncthreads();  // big[] and nbig are rebuilt by the next entry block
    }
}

}  // namespace bkd
