// Work plan for ragged (indexed) batches: aligned chunking, bucketing by step count, combine.
//
// Why: a G-lane group walks its work in lockstep with the other groups of its wavefront, so a
// wave holding Zipf-sized entries runs as long as its longest entry (SURVEY.md §7 "load balance
// for Zipf sizes"), and packed entries start and end at arbitrary bytes. The plan therefore
//  * pads every entry [s, e) to ae = the first 128-byte-aligned device address >= e (64 for
//    4-lane groups, whose 64-byte step must hold the whole pad) (the pad
//    bytes lie in e's own 128-byte line, so reading them never leaves mapped memory; the chunk
//    kernel folds them as zeros) and cuts [s, ae) into chunks of CH = 16*G*JC bytes whose ends
//    are aligned (c = 0 ends at ae, c = m-1 is the head and starts at s, carrying the seed), so
//    every 16-byte load of the main kernel is an aligned global_load_dwordx4 and no 128-byte line
//    is fetched by two chunks;
//  * lists the chunks in descending step count (merged heads JC+1, full chunks JC, heads JC-1..1)
//    so that neighbouring groups, which run in lockstep, have equal work;
//  * writes one self-contained 16-byte descriptor per chunk (PlanDesc: window, pad, length, seed
//    register, destination; 8 bytes, PlanDesc8, for a batch without per-entry seeds), which the chunk
//    kernel reads two rounds ahead (six chunks ahead in its short tail) — no dependent index loads at
//    chunk start;
//  * combines multi-chunk entries as reg = sum_c partial_c * X^c, X = x^(8*CH) (Horner from the
//    head), then removes the zero padding (multiply by x^(-8*pad)): the GPU analogue of
//    crc32c_chunk's stream merge by shift tables (crc32c_sse42.cpp:92-134).
// Entries shorter than 16 bytes and invalid (out-of-bounds) entries are handled by
// plan_combine_kernel; entries that do not fit the plan's capacity (only possible when entries
// overlap heavily) are computed one entry per lane group (PlanDirectSrc) in the tail of the chunk
// kernel, a loop that is skipped when nothing overflowed.
//
// Launch sequence (caller's stream, no host sync): plan_count -> plan_scan -> plan_emit ->
// crc_plan_chunks_kernel (+ overflow tail) -> plan_combine.
#pragma once
#include "crc_kernels.hpp"

namespace bkd {

constexpr int kPlanBlock = 1024;
constexpr int kMaxJC = 256;  // bins 0 .. jc + merge steps

constexpr uint32_t kNoSlot = 0xFFFFFFFFu;  // single aligned chunk, no tail: the chunk writes out[] itself
constexpr uint32_t kSerial = 0xFFFFFFFEu;  // whole entry folded serially by the combine kernel
constexpr uint32_t kDirect = 0xFFFFFFFDu;  // plan capacity exceeded: serial too
constexpr uint32_t kSmall = 0xFFFFFFFCu;   // short-entry class: computed by its own launch (SmallIndexedSrc)

struct PlanGeo {
    uint32_t step;   // 16 * G bytes
    uint32_t jc;     // steps per full chunk
    uint32_t ch;     // step * jc
    uint32_t mis;    // device address of base modulo 128
    uint32_t merge;  // a head chunk shorter than this (>= 16) merges into its neighbour
    uint32_t nbins;  // bins 0 .. nbins-1: ceil((ch + merge - 1) / step) + 1
    uint32_t step_sh;  // log2(step)
    uint32_t ch_sh;    // log2(ch) when ch is a power of two, else 0xFF (64-bit divisions are slow)
    uint32_t small;    // entries of <= small bytes belong to the short-entry launch (0: none do)
    uint32_t serial;   // entries shorter than this (16 .. kSerialMax) are computed by plan_combine
    uint32_t jshort;   // chunks of <= jshort steps form the chunk kernel's short tail (PF + 1; 0: none)
    uint32_t d8;       // 8-byte descriptors (PlanDesc8: unseeded batch, no final chunks)
};

// Longest entry plan_combine computes itself, one thread per entry (serial_crc).
constexpr uint32_t kSerialMax = 64u;

// hdr words
constexpr int kHdrTotal = 0;  // all chunks
constexpr int kHdrWork = 2;   // descriptors to process = min(total, capacity)
constexpr int kHdrShort = 3;  // list position of the first chunk of <= PlanGeo::jshort steps (the chunk
                              // kernel's short tail; = total when jshort == 0)
constexpr int kHdrBase = 4;   // kHdrBase + col: total of column col (plan_scan)
constexpr int kHdrWords = kHdrBase + kMaxJC + 2;

__device__ __forceinline__ bool entry_valid(uint64_t o, uint32_t l, uint64_t size) {
    return !(o > size || (uint64_t)l > size - o);
}

struct EntryPlan {
    int64_t s, e, ae;
    uint32_t pad;   // ae - e (0 .. 127)
    uint32_t m;     // chunks of [s, ae)
    uint32_t jh;    // head chunk steps (1 .. nbins-1)
    uint32_t full;  // chunks in the full bucket (bin JC)
    uint32_t ps;    // partial slots (0: the single chunk writes the final CRC)
    uint32_t kind;  // 0 chunked, 1 serial, 2 invalid, 3 short-entry class (not the plan's)
};

__device__ __forceinline__ bool is_small(uint32_t l, const PlanGeo& pg) { return l <= pg.small && pg.small != 0u; }

__device__ __forceinline__ EntryPlan plan_entry(uint64_t o, uint32_t l, uint64_t size, const PlanGeo& pg) {
    EntryPlan p{};
    if (is_small(l, pg)) {  // bounds included: the short-entry launch reports them
        p.kind = 3;
        return p;
    }
    if (!entry_valid(o, l, size)) {
        p.kind = 2;
        return p;
    }
    p.s = (int64_t)o;
    p.e = (int64_t)(o + l);
    // chunk ends sit on 128-byte lines: a line is then never split between two chunks that run
    // at different times (each would fetch it from HBM)
    if (l < pg.serial) {  // plan_combine, one thread per entry (at least every l < 16)
        p.kind = 1;
        return p;
    }
    // pad to the next multiple of min(step, 128): the pad then lies in the entry's last 128-byte
    // line AND in the last step of its final chunk (the chunk kernel clears it there)
    const uint32_t al = pg.step < 128u ? pg.step : 128u;
    p.pad = (uint32_t)((al - ((pg.mis + (uint64_t)p.e) & (al - 1u))) & (al - 1u));
    p.ae = p.e + (int64_t)p.pad;
    const uint64_t la = (uint64_t)(p.ae - p.s);
    uint32_t m = pg.ch_sh < 32u ? (uint32_t)((la + pg.ch - 1) >> pg.ch_sh) : (uint32_t)((la + pg.ch - 1) / pg.ch);
    uint32_t hl = (uint32_t)(la - (uint64_t)(m - 1u) * pg.ch);
    if (hl < pg.merge && m > 1u) {  // a short head merges into its neighbour (up to ch + merge - 1 bytes)
        --m;
        hl += pg.ch;
    }
    p.m = m;
    p.jh = (hl + pg.step - 1u) >> pg.step_sh;
    p.full = (m - 1u) + (p.jh == pg.jc ? 1u : 0u);
    p.ps = (m == 1u && p.pad == 0u && !pg.d8) ? 0u : m;  // (PlanDesc8 has no final chunks)
    p.kind = 0;
    return p;
}

__device__ __forceinline__ PlanDesc chunk_desc(const EntryPlan& p, uint32_t c, uint32_t seed, uint32_t entry,
                                               uint32_t slot, const PlanGeo& pg) {
    PlanDesc d;
    const int64_t e = p.ae - (int64_t)c * pg.ch;
    const bool head = c + 1u == p.m;
    const int64_t s = head ? p.s : e - (int64_t)pg.ch;
    const uint64_t pad = c == 0u ? (uint64_t)p.pad : 0u;
    const uint32_t len = (uint32_t)(e - s);
    const uint32_t J = (len + pg.step - 1u) >> pg.step_sh;
    const int64_t w = e - (int64_t)J * (int64_t)pg.step;  // the chunk's step-aligned window start
    d.s_len = (uint64_t)(w + kWBias) | (pad << kPlanOffBits) | ((uint64_t)len << 48) |
              ((pg.d8 && head) ? 1ull << kPlanHeadBit : 0ull);
    d.r0 = head ? ~seed : 0u;
    d.dst = p.ps == 0u ? (entry | kPlanFinal) : slot;  // slot: the chunk's own list position
    return d;
}

// A hole (an entry past the plan's capacity, computed by the overflow tail instead): no bytes, and a
// window at base[0] so that the chunk kernel may request its blocks like any chunk's (base[16g],
// within the first 16 * G bytes: a plan only overflows with multi-chunk entries, so base holds more
// than one chunk then).
__device__ __forceinline__ PlanDesc skip_desc() { return PlanDesc{(uint64_t)kWBias, 0u, 0u}; }

// A descriptor into the list: 16 bytes, or its first word (PlanDesc8) when the plan uses those.
__device__ __forceinline__ void put_desc(PlanDesc* descs, uint64_t pos, const PlanDesc& d, const PlanGeo& pg) {
    if (pg.d8) reinterpret_cast<PlanDesc8*>(descs)[pos] = PlanDesc8{d.s_len};
    else descs[pos] = d;
}

// Deterministic block-wide exclusive scan (1024 threads = 16 waves).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int k = 0; k < kPlanBlock / 64; ++k) {
            const uint32_t t = wsum[k];
            wsum[k] = acc;
            acc += t;
        }
        wsum[kPlanBlock / 64] = acc;
    }
    __syncthreads();
    const uint32_t r = wsum[wave] + x - v;
    total = wsum[kPlanBlock / 64];
    __syncthreads();
    return r;
}

// columns: bins 0 .. nbins-1 (chunk counts by step count; bin JC = full bucket). (Partials need no
// column of their own: each chunk's partial sits at its own list position.)
__host__ __device__ __forceinline__ uint32_t plan_ncols(const PlanGeo& pg) { return pg.nbins; }

// Per-block column counts (plan_scan_kernel turns them into per-block offsets and totals).
// blive[b]: entries of block b that the plan itself handles (not the short-entry class); emit and
// combine skip blocks without any (a batch of short entries costs them one word per block).
// Entry blocks per plan_count block: thread t counts entry t of each of kCountBlocks consecutive
// entry blocks, their index words requested together (the kernel is bound by load latency: one
// entry per thread ran config 3's 1 M entries in two rounds of 13 us, four per thread in one of 7).
constexpr uint32_t kCountBlocks = 4;

__global__ void __launch_bounds__(kPlanBlock) plan_count_kernel(const uint64_t* __restrict__ offsets,
                                                                const uint32_t* __restrict__ lengths, uint64_t size,
                                                                uint64_t n, PlanGeo pg, uint32_t* __restrict__ blk,
                                                                uint32_t* __restrict__ blive, uint32_t nb, PlanRun run,
                                                                uint32_t* __restrict__ bok) {
    if (!run.plan_entries()) return;
    __shared__ uint32_t col[kCountBlocks][kMaxJC + 2];
    __shared__ uint32_t live[kCountBlocks], bad[kCountBlocks];
    const uint32_t ncols = plan_ncols(pg);
    const uint32_t ref = bok ? lengths[0] : 0u;  // the uniformity ballot's reference length
    const uint32_t ngb = (nb + kCountBlocks - 1u) / kCountBlocks;
    for (uint32_t gb = blockIdx.x; gb < ngb; gb += gridDim.x) {  // kCountBlocks entry blocks at a time, grid stride
    for (uint32_t k = threadIdx.x; k < kCountBlocks * (kMaxJC + 2); k += kPlanBlock) (&col[0][0])[k] = 0u;
    if (threadIdx.x < kCountBlocks) {
        live[threadIdx.x] = 0u;
        bad[threadIdx.x] = 0u;
    }
    __syncthreads();
    // the lengths (and, without a short class, offsets) of the thread's entries requested at once;
    // with a short class offsets are loaded only for the plan's own entries
    uint32_t l[kCountBlocks];
    uint64_t o[kCountBlocks];
#pragma unroll
    for (uint32_t k = 0; k < kCountBlocks; ++k) {
        const uint64_t i = (uint64_t)(gb * kCountBlocks + k) * kPlanBlock + threadIdx.x;
        const uint64_t ic = i < n ? i : n - 1u;
        l[k] = lengths[ic];
        o[k] = pg.small == 0u ? offsets[ic] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kCountBlocks; ++k) {
        const uint64_t i = (uint64_t)(gb * kCountBlocks + k) * kPlanBlock + threadIdx.x;
        uint32_t full = 0u, mine = 0u;
        bool ok = true;  // length within the band of the reference (PlanRun::in_band)
        if (i < n) {
            ok = PlanRun::in_band(l[k], ref);
            if (!is_small(l[k], pg)) {
                mine = 1u;
                const EntryPlan p = plan_entry(pg.small == 0u ? o[k] : offsets[i], l[k], size, pg);
                if (p.kind == 0) {
                    if (p.jh != pg.jc) atomicAdd(&col[k][p.jh], 1u);
                    full = p.full;
                }
            }
        }
        // every entry adds to these columns: one LDS atomic per wave instead of 64
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            full += (uint32_t)__shfl_xor((int)full, d);
            mine += (uint32_t)__shfl_xor((int)mine, d);
        }
        const bool wave_ok = __all(ok);
        if ((threadIdx.x & 63) == 0) {
            if (full) atomicAdd(&col[k][pg.jc], full);
            if (mine) atomicAdd(&live[k], mine);
            if (!wave_ok) bad[k] = 1u;  // (a per-wave min/max with global atomics cost +330 us per 1 M entries)
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kCountBlocks; ++k) {
        const uint32_t eb = gb * kCountBlocks + k;
        if (eb >= nb) break;  // block-uniform
        for (uint32_t c = threadIdx.x; c < ncols; c += kPlanBlock) blk[(uint64_t)c * nb + eb] = col[k][c];
        if (threadIdx.x == 0) {
            blive[eb] = live[k];
            if (bok) bok[eb] = bad[k] ^ 1u;
        }
    }
    __syncthreads();  // col/live are reset for the next entry blocks
    }
}

// One 1024-thread block per column: exclusive scan of the column's per-block counts across blocks
// (thread t sums its run of ceil(nb / 1024) rows, one block scan of the sums, then writes its run);
// the column total goes to hdr[kHdrBase + col]. plan_emit places the bins (descending step count)
// from those totals. A 64-lane block per column walking the rows in order took 258 us at
// nb = 65 536 (64 M entries) against 6 us at 1 024.
// (Folding this scan into the count kernel's last block needs a device-scope release per block,
// an L2 write-back on this multi-XCD part: measured 52 us instead of 7.5 + 5.8.)
__global__ void __launch_bounds__(kPlanBlock) plan_scan_kernel(const uint32_t* __restrict__ blk, uint32_t nb,
                                                               uint32_t* __restrict__ blkoff, uint32_t* __restrict__ hdr,
                                                               PlanRun run, uint32_t ncols,
                                                               const uint32_t* __restrict__ bok) {
    if (!run.plan_entries()) return;
    __shared__ uint32_t wsum[kPlanBlock / 64 + 1];
    const uint32_t c = blockIdx.x;
    if (c == ncols) {  // the extra block: PlanRun::uniform for the whole batch
        uint32_t ok = 1u;
        for (uint32_t b = threadIdx.x; b < nb; b += kPlanBlock) ok &= bok[b];
        ok = (uint32_t)__syncthreads_and((int)ok);
        if (threadIdx.x == 0) *const_cast<uint32_t*>(run.uni) = ok ? run.epoch : 0u;
        return;
    }
    const uint32_t* col = blk + (uint64_t)c * nb;
    uint32_t* dst = blkoff + (uint64_t)c * nb;
    const uint32_t per = (nb + kPlanBlock - 1u) / kPlanBlock;
    const uint32_t b0 = threadIdx.x * per < nb ? threadIdx.x * per : nb;
    const uint32_t b1 = b0 + per < nb ? b0 + per : nb;
    uint32_t sum = 0u;
    for (uint32_t b = b0; b < b1; ++b) sum += col[b];
    uint32_t total;
    uint32_t acc = block_excl_scan(sum, wsum, total);
    for (uint32_t b = b0; b < b1; ++b) {
        const uint32_t v = col[b];
        dst[b] = acc;
        acc += v;
    }
    if (threadIdx.x == 0) hdr[kHdrBase + c] = total;
}

// Descriptor of chunk c of an entry from its stashed plan (plan_emit's cooperative pass).
__device__ __forceinline__ PlanDesc chunk_desc_of(int64_t ae, int64_t s0, uint32_t m, uint32_t pad, bool final,
                                                  uint32_t c, uint32_t seed, uint32_t entry, uint32_t slot,
                                                  const PlanGeo& pg) {
    EntryPlan p{};
    p.ae = ae;
    p.s = s0;
    p.m = m;
    p.pad = pad;
    p.ps = final ? 0u : m;
    return chunk_desc(p, c, seed, entry, slot, pg);
}

// Writes every chunk descriptor. Heads go to their step bin (LDS atomic cursor per bin); the full
// chunks of the block's entries form one contiguous run in the full bin, written by the whole
// block (one descriptor per thread per pass, coalesced, no per-entry serial loop) — including
// entries with thousands of chunks. Grid stride over the nb * reps virtual blocks.
#ifndef BKD_PLAN_OCC
#define BKD_PLAN_OCC 8
#endif
// emit and combine at 8 waves per SIMD (<= 64 VGPRs): two 1024-thread blocks per CU resident, as
// BKD_PLAN_GRID launches them
__global__ void __launch_bounds__(kPlanBlock, BKD_PLAN_OCC) plan_emit_kernel(const uint64_t* __restrict__ offsets,
                                                               const uint32_t* __restrict__ lengths,
                                                               const uint32_t* __restrict__ seeds, uint32_t seed_all,
                                                               uint64_t size, uint64_t n, PlanGeo pg,
                                                               uint64_t capacity, const uint32_t* __restrict__ blkoff,
                                                               uint32_t* __restrict__ pslot, uint32_t* __restrict__ hslot,
                                                               uint32_t* __restrict__ hdr,
                                                               PlanDesc* __restrict__ descs, uint32_t reps,
                                                               const uint32_t* __restrict__ blive, uint32_t nb,
                                                               PlanRun run) {
    // `reps` virtual blocks per 1024-entry block (few entries, many chunks each: 256 x 16 MiB is one
    // entry block): every replica plans the same entries, replica 0 writes heads, slots and the
    // header, and the replicas split the block's full-chunk descriptors
    if (!run.on()) return;
    __shared__ uint32_t wsum[kPlanBlock / 64 + 1];
    __shared__ uint32_t bin0[kMaxJC + 2];  // first position of each bin (descending step count)
    __shared__ uint32_t cursor[kMaxJC + 2];
    __shared__ uint32_t exf[kPlanBlock + 1];  // block-exclusive scan of full-chunk counts (+ total)
    __shared__ int64_t st_ae[kPlanBlock], st_s[kPlanBlock];
    __shared__ uint32_t st_m[kPlanBlock], st_flags[kPlanBlock], st_seed[kPlanBlock];
    __shared__ uint32_t s_total;
    const uint32_t ncols = plan_ncols(pg);
    for (uint32_t k = threadIdx.x; k < ncols; k += kPlanBlock) bin0[k] = hdr[kHdrBase + k];
    __syncthreads();
    if (threadIdx.x == 0) {  // column totals -> first position of each bin, descending step count
        uint32_t acc = 0;
        for (int j = (int)pg.nbins - 1; j >= 0; --j) {
            const uint32_t t = bin0[j];
            bin0[j] = acc;
            acc += t;
        }
        s_total = acc;
        if (blockIdx.x == 0) {  // the block that plans entry block 0, replica 0
            hdr[kHdrTotal] = acc;
            hdr[kHdrWork] = (uint32_t)((uint64_t)acc < capacity ? acc : capacity);
            // bins of <= jshort steps come last: the short tail starts at bin jshort's first position
            hdr[kHdrShort] = pg.jshort == 0u ? acc : (pg.jshort < pg.nbins ? bin0[pg.jshort] : 0u);
        }
    }
    __syncthreads();
    const uint32_t nvb = nb * reps;
    for (uint32_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
    const uint32_t eb = vb / reps, rep = vb - eb * reps;
    // the entry's index words, the live count and the cursors requested together (one round trip)
    const uint64_t i = (uint64_t)eb * kPlanBlock + threadIdx.x;
    const uint64_t ic = i < n ? i : n - 1u;
    const uint64_t o = offsets[ic];
    const uint32_t l = lengths[ic];
    const uint32_t seed = seeds ? seeds[ic] : seed_all;
    if (blive[eb] == 0u) continue;  // only short entries (block-uniform)
    for (uint32_t k = threadIdx.x; k < ncols; k += kPlanBlock) cursor[k] = bin0[k] + blkoff[(uint64_t)k * nb + eb];
    __syncthreads();
    EntryPlan p{};
    p.kind = 1;
    if (i < n) p = plan_entry(o, l, size, pg);
    const bool chunked = i < n && p.kind == 0;
    uint32_t t_full;
    const uint32_t ex_full = block_excl_scan(chunked ? p.full : 0u, wsum, t_full);
    const uint32_t run0 = cursor[pg.jc];  // the block's first full-bin position (heads never move it)
    exf[threadIdx.x] = ex_full;
    if (threadIdx.x == 0) exf[kPlanBlock] = t_full;
    if (rep == 0u && i < n && !chunked) pslot[i] = p.kind == 3u ? kSmall : kSerial;
    if (chunked) {
        const uint32_t rs = run0 + ex_full;
        const bool has_head = p.jh != pg.jc;
        const uint32_t hpos = has_head ? atomicAdd(&cursor[p.jh], 1u) : 0u;
        const bool overflow = ((uint64_t)rs + p.full > capacity) || (has_head && (uint64_t)hpos >= capacity);
        // a chunk's partial goes to partials[its list position]: a wave's groups hold consecutive
        // positions, so their partials are one coalesced write (entry-ordered slots made every
        // partial a lone 4-byte write). pslot: the full run's first position, or the head's
        // position when the entry has no full chunk; hslot: the head's when it has both
        if (rep == 0u) pslot[i] = overflow ? kDirect : (p.ps ? (p.full ? rs : hpos) : kNoSlot);
        if (rep == 0u && p.ps && p.full && has_head) hslot[i] = hpos;
        if (rep == 0u && has_head && (uint64_t)hpos < capacity)
            put_desc(descs, hpos, overflow ? skip_desc() : chunk_desc(p, p.m - 1u, seed, (uint32_t)i, hpos, pg), pg);
        st_ae[threadIdx.x] = p.ae;
        st_s[threadIdx.x] = p.s;
        st_m[threadIdx.x] = p.m;
        st_flags[threadIdx.x] = p.pad | (p.ps == 0u ? 0x100u : 0u) | (overflow ? 0x200u : 0u);
        st_seed[threadIdx.x] = seed;
    }
    __syncthreads();
    // replicas split the full chunks only when nothing can overflow (total <= capacity): head
    // positions come from LDS atomics whose order differs between replicas, and so could the
    // overflow flags; otherwise replica 0 writes them all
    uint32_t k0 = 0u, k1 = t_full;
    if (reps > 1u) {
        if ((uint64_t)s_total <= capacity) {
            k0 = (uint32_t)((uint64_t)t_full * rep / reps);
            k1 = (uint32_t)((uint64_t)t_full * (rep + 1u) / reps);
        } else if (rep != 0u) {
            k1 = 0u;
        }
    }
    for (uint32_t k = k0 + threadIdx.x; k < k1; k += kPlanBlock) {
        // owner: the last thread t with exf[t] <= k (it has full chunks: exf[t + 1] > k)
        uint32_t lo = 0u, hi = kPlanBlock;
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) >> 1;
            if (exf[mid] <= k) lo = mid;
            else hi = mid;
        }
        const uint32_t t = lo, c = k - exf[t];
        const uint64_t pos = (uint64_t)run0 + k;
        const uint32_t fl = st_flags[t];
        if (fl & 0x200u) {
            if (pos < capacity) put_desc(descs, pos, skip_desc(), pg);
        } else {
            put_desc(descs, pos, chunk_desc_of(st_ae[t], st_s[t], st_m[t], fl & 0xFFu, (fl & 0x100u) != 0u, c,
                                               st_seed[t], (uint32_t)((uint64_t)eb * kPlanBlock + t), (uint32_t)pos, pg),
                     pg);
        }
    }
    __syncthreads();  // LDS stashes and cursors are rewritten by the next virtual block
    }
}

// Entries the plan could not hold (pslot == kDirect): one entry per lane group, like IndexedSrc,
// in the chunk kernel's tail. count() is 0 unless the plan overflowed (total chunks > capacity).
struct PlanDirectSrc {
    uint64_t n;
    const uint64_t* offsets;
    const uint32_t* lengths;
    const uint32_t* seeds;
    uint32_t seed_all;
    uint64_t size;
    uint32_t* out;
    const uint32_t* pslot;
    const uint32_t* hdr;
    uint64_t capacity;
    bool all;  // set by the chunk kernel: PlanRun::uniform, every entry is computed here
    __device__ __forceinline__ uint64_t count() const {
        return all || (uint64_t)hdr[kHdrTotal] > capacity ? n : 0u;
    }
    __device__ __forceinline__ int get(uint64_t i, Work& w) const {
        if (!all && pslot[i] != kDirect) return 3;
        w.dst = out + i;
        w.s = (int64_t)offsets[i];
        w.len = lengths[i];
        if (!entry_valid((uint64_t)w.s, w.len, size)) return 2;
        w.r0 = ~(seeds ? seeds[i] : seed_all);
        w.xorout = 0xFFFFFFFFu;
        return 0;
    }
};

// a * b mod P, bitwise (no tables): 32 shift/xor steps, for the few products per entry that have
// no operator table (x^(-8*pad), powers of X).
__device__ __forceinline__ uint32_t gf_mul_bits(uint32_t a, uint32_t b, uint32_t poly) {
    uint32_t prod = 0u, cur = b;
#pragma unroll
    for (int k = 31; k >= 0; --k) {
        prod ^= ((a >> k) & 1u) ? cur : 0u;
        cur = (cur >> 1) ^ ((cur & 1u) ? poly : 0u);
    }
    return prod;
}

__device__ __forceinline__ uint32_t gf_pow_bits(uint32_t x, uint32_t e, uint32_t poly) {
    uint32_t r = 0x80000000u;  // x^0
    while (e) {
        if (e & 1u) r = gf_mul_bits(r, x, poly);
        x = gf_mul_bits(x, x, poly);
        e >>= 1;
    }
    return r;
}

// Horner over the partial registers of each chunked entry, then x^(-8*pad); serial fold of
// entries the plan did not chunk. Entries with more than kCombineSerial chunks are combined by a
// wave (up to kCombineWave chunks) or by the whole block (e.g. one 64 MiB entry = 16 Ki chunks)
// instead of one serial thread: thread t of T (64 or 1024) folds chunks t, t + T, t + 2T, ... with
// Horner by X^T (a wave's loads are consecutive partials), is placed by X^t (one bitwise product
// per table word of t), and the wave or block XOR-reduces.
constexpr uint32_t kCombineSerial = 64;
constexpr uint32_t kCombineWave = 4096;
// The combine's operator block (xtab_for): 4x256 tables of X = x^(8*CH), X^64 and X^1024, then the
// words X^L (L = 0..63) and X^(64 w) (w = 0..15).
constexpr uint32_t kXtabX = 0, kXtabX64 = 1024, kXtabX1024 = 2048, kXtabLane = 3072, kXtabWave = 3136;
constexpr uint32_t kXtabWords = 3152;

// Slice-by-16 tables in LDS: T[k * 256 + b] = byte b followed by k zero bytes; T[0 .. 255] is the
// byte table. The reference's scalar fallback is the byte-at-a-time form of the same arithmetic
// (circe ReflectedIntCrc / crc32c_sse42.cpp's table path).
__device__ __forceinline__ void build_slice16(uint32_t* T, const uint32_t* __restrict__ btab) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) T[b] = btab[b];
    __syncthreads();
    for (int b = threadIdx.x; b < 256; b += blockDim.x) {
        uint32_t v = T[b];
        for (int k = 1; k < 16; ++k) {
            v = (v >> 8) ^ T[v & 0xffu];
            T[k * 256 + b] = v;
        }
    }
}

__device__ __forceinline__ uint32_t fold4_t(const uint32_t* T, uint32_t reg, uint32_t w) {
    const uint32_t c = reg ^ w;
    return xor3(T[3 * 256 + (c & 0xffu)], T[2 * 256 + ((c >> 8) & 0xffu)], T[256 + ((c >> 16) & 0xffu)] ^ T[c >> 24]);
}

// Raw register of base[o, o + l) (1 <= l < kSerialMax) from `reg`, one thread: every 16-byte block
// holding an entry byte is loaded at once (never a byte past those blocks), 16-byte windows of the
// entry are cut from consecutive blocks (dword select + v_alignbyte) and folded slice-by-16 — only
// the four lookups of the register's own bytes sit on the dependency chain.
__device__ __forceinline__ uint32_t serial_crc(const uint8_t* __restrict__ base, uint64_t o, uint32_t l, uint32_t reg,
                                               const uint32_t* T) {
    constexpr int kMaxBlk = (int)(kSerialMax + 30u) / 16;
    const uintptr_t pa = (uintptr_t)(base + o);
    const u32x4* blk = reinterpret_cast<const u32x4*>(pa & ~(uintptr_t)15);
    const uint32_t d = (uint32_t)(pa & 15u), s = d >> 2, sb = d & 3u;
    const uint32_t nb = (d + l + 15u) >> 4, nw = l >> 4, t = l & 15u;
    u32x4 b[kMaxBlk];
#pragma unroll
    for (int k = 0; k < kMaxBlk; ++k) b[k] = (uint32_t)k < nb ? blk[k] : u32x4{0u, 0u, 0u, 0u};
    auto window = [&](const u32x4& lo, const u32x4& hi, uint32_t (&w)[4]) {
        const uint32_t e[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        uint32_t v[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) v[i] = s == 0u ? e[i] : s == 1u ? e[i + 1] : s == 2u ? e[i + 2] : e[i + 3];
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], sb);
    };
#pragma unroll
    for (int j = 0; j + 1 < kMaxBlk; ++j) {
        uint32_t w[4];
        window(b[j], b[j + 1], w);
        if ((uint32_t)j < nw) {
            const uint32_t c = reg ^ w[0];
            const uint32_t rest = xor3(xor3(T[11 * 256 + (w[1] & 0xffu)], T[10 * 256 + ((w[1] >> 8) & 0xffu)],
                                            T[9 * 256 + ((w[1] >> 16) & 0xffu)] ^ T[8 * 256 + (w[1] >> 24)]),
                                       xor3(T[7 * 256 + (w[2] & 0xffu)], T[6 * 256 + ((w[2] >> 8) & 0xffu)],
                                            T[5 * 256 + ((w[2] >> 16) & 0xffu)] ^ T[4 * 256 + (w[2] >> 24)]),
                                       xor3(T[3 * 256 + (w[3] & 0xffu)], T[2 * 256 + ((w[3] >> 8) & 0xffu)],
                                            T[256 + ((w[3] >> 16) & 0xffu)] ^ T[w[3] >> 24]));
            reg = xor3(xor3(T[15 * 256 + (c & 0xffu)], T[14 * 256 + ((c >> 8) & 0xffu)],
                            T[13 * 256 + ((c >> 16) & 0xffu)] ^ T[12 * 256 + (c >> 24)]), rest, 0u);
        } else if ((uint32_t)j == nw && t) {  // the last t < 16 bytes: whole dwords, then bytes
            const uint32_t q = t >> 2;
            if (q > 0u) reg = fold4_t(T, reg, w[0]);
            if (q > 1u) reg = fold4_t(T, reg, w[1]);
            if (q > 2u) reg = fold4_t(T, reg, w[2]);
            uint32_t x = q == 0u ? w[0] : q == 1u ? w[1] : q == 2u ? w[2] : w[3];
            for (uint32_t k = 0; k < (t & 3u); ++k, x >>= 8) reg = T[(reg ^ x) & 0xffu] ^ (reg >> 8);
        }
    }
    return reg;
}

__device__ __forceinline__ uint32_t mul_x(const uint32_t* X, uint32_t r) {
    return xor3(X[r & 0xffu], X[256 + ((r >> 8) & 0xffu)], X[512 + ((r >> 16) & 0xffu)] ^ X[768 + (r >> 24)]);
}

// sum_j partial(t + T j) * (X^T)^j over the chunks t + T j < m of an entry (chunk m - 1, the head,
// at hs; the rest at sl + c), by Horner from the highest j; the partials are loaded 8 at a time.
template <uint32_t T>
__device__ __forceinline__ uint32_t strided_horner(const uint32_t* XT, const uint32_t* __restrict__ partials,
                                                   uint32_t sl, uint32_t hs, uint32_t m, uint32_t t) {
    const int nj = t < m ? (int)((m - 1u - t) / T) + 1 : 0;
    uint32_t r = 0u;
    for (int j0 = nj - 1; j0 >= 0; j0 -= 8) {
        uint32_t pv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t c = t + T * (uint32_t)(j0 - k);
            pv[k] = j0 - k >= 0 ? partials[c + 1u == m ? hs : sl + c] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (j0 - k >= 0) r = mul_x(XT, r) ^ pv[k];
    }
    return r;
}

__global__ void __launch_bounds__(1024, BKD_PLAN_OCC) plan_combine_kernel(
    const uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets, const uint32_t* __restrict__ lengths,
    const uint32_t* __restrict__ seeds, uint32_t seed_all, uint64_t size, uint64_t n, PlanGeo pg,
    const uint32_t* __restrict__ xtab, const uint32_t* __restrict__ btab, const uint32_t* __restrict__ xinv, uint32_t poly,
    const uint32_t* __restrict__ pslot, const uint32_t* __restrict__ hslot, const uint32_t* __restrict__ partials,
    uint32_t* __restrict__ out, uint32_t* __restrict__ err, uint32_t reps, const uint32_t* __restrict__ blive,
    uint32_t nblk, PlanRun run) {
    // `reps` virtual blocks per 1024-entry block (as plan_emit_kernel): each replica lists the
    // block's entries of > kCombineSerial chunks and combines its share of them; replica 0 does the
    // rest (invalid and serial entries are idempotent writes, cheap, and left to every replica).
    // Grid stride over the virtual blocks; the operator tables are staged once per block.
    if (!run.on()) return;
    __shared__ uint32_t X[kXtabWords];  // xtab_for's operator block
    __shared__ uint32_t T[16 * 256];  // slice-by-16 (serial entries)
    __shared__ uint32_t big[1024];
    __shared__ uint32_t wsum[kPlanBlock / 64 + 1];
    __shared__ uint32_t nbig;
    __shared__ uint32_t red[1024 / 64];
    for (int k = threadIdx.x; k < (int)kXtabWords; k += blockDim.x) X[k] = xtab[k];
    build_slice16(T, btab);
    const uint32_t nvb = nblk * reps;
    for (uint32_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
    const uint32_t eb = vb / reps, rep = vb - eb * reps;
    // every index word of the entry is requested at once, with the block's live count: one round
    // trip before the partials (a word the entry turns out not to need costs nothing further)
    const uint64_t i = (uint64_t)eb * blockDim.x + threadIdx.x;
    const uint64_t ic = i < n ? i : n - 1u;
    const uint32_t live = blive[eb];
    uint32_t slot = pslot[ic];
    const uint32_t hs_i = hslot[ic];
    const uint64_t o = offsets[ic];
    const uint32_t l = lengths[ic];
    const uint32_t seed_i = seeds ? seeds[ic] : seed_all;
    if (i >= n) slot = kNoSlot;
    if (live == 0u) continue;  // only short entries: the short-entry launch wrote them
    if (threadIdx.x == 0) nbig = 0u;
    __syncthreads();
    uint32_t is_big = 0u;
    if (slot != kNoSlot && slot != kDirect && slot != kSmall) {
        if (!entry_valid(o, l, size)) {
            out[i] = 0u;
            if (err) atomicOr(err, 1u);
        } else if (slot == kSerial) {
            const uint32_t reg = ~seed_i;
            out[i] = l ? ~serial_crc(base, o, l, reg, T) : ~reg;
        } else {
            const EntryPlan p = plan_entry(o, l, size, pg);
            if (p.m > kCombineSerial) {
                is_big = 1u;
                if (reps == 1u) big[atomicAdd(&nbig, 1u)] = (uint32_t)threadIdx.x;
            } else if (rep == 0u) {
                // partials in batches of 8 independent loads, then Horner from the head (chunk m - 1:
                // at hslot when it is a separate head beside full chunks, else in the full run)
                const bool sep = p.jh != pg.jc && p.full != 0u;
                uint32_t reg = partials[sep ? hs_i : slot + p.m - 1u];
                for (int c0 = (int)p.m - 2; c0 >= 0; c0 -= 8) {
                    uint32_t pv[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) pv[k] = c0 - k >= 0 ? partials[slot + (uint32_t)(c0 - k)] : 0u;
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (c0 - k >= 0) reg = mul_x(X, reg) ^ pv[k];
                }
                // undo the zero padding: reg * x^(-8*pad), a bitwise product (no table dependency chain)
                if (p.pad) reg = gf_mul_bits(xinv[p.pad], reg, poly);
                out[i] = ~reg;
            }
        }
    }
    // the big-entry list in entry order (a scan, not LDS atomics) when replicas must all see the same
    // list, since they split it by position; a single replica keeps the cheaper LDS-atomic list
    uint32_t nb;
    if (reps > 1u) {  // kernel-uniform
        const uint32_t bpos = block_excl_scan(is_big, wsum, nb);
        if (is_big) big[bpos] = (uint32_t)threadIdx.x;
        __syncthreads();
    } else {
        __syncthreads();
        nb = nbig;
    }
    // 65 .. kCombineWave chunks: one wave per entry, the block's waves in parallel (4096 x 1 MiB
    // entries leave 4 blocks of 1024 such entries each; one entry at a time per block took 8 ms)
    const uint32_t lane = threadIdx.x & 63u, nwaves = blockDim.x >> 6;
    for (uint32_t k = rep * nwaves + (threadIdx.x >> 6); k < nb; k += reps * nwaves) {
        const uint64_t e = (uint64_t)eb * blockDim.x + big[k];
        const EntryPlan p = plan_entry(offsets[e], lengths[e], size, pg);
        if (p.m > kCombineWave) continue;  // wave-uniform
        const uint32_t sl = pslot[e], hs = p.jh != pg.jc ? hslot[e] : sl + p.m - 1u;  // m > 64: full chunks exist
        uint32_t r = strided_horner<64u>(X + kXtabX64, partials, sl, hs, p.m, lane);
        r = gf_mul_bits(X[kXtabLane + lane], r, poly);
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) r ^= (uint32_t)__shfl_xor((int)r, d);
        if (lane == 0u) out[e] = ~(p.pad ? gf_mul_bits(xinv[p.pad], r, poly) : r);
    }
    // more chunks (entries of >= 16 MiB at 4 KiB chunks): the whole block per entry
    for (uint32_t k = rep; k < nb; k += reps) {
        const uint64_t e = (uint64_t)eb * blockDim.x + big[k];
        const EntryPlan p = plan_entry(offsets[e], lengths[e], size, pg);
        if (p.m <= kCombineWave) continue;  // block-uniform
        const uint32_t sl = pslot[e], hs = p.jh != pg.jc ? hslot[e] : sl + p.m - 1u;
        uint32_t r = strided_horner<1024u>(X + kXtabX1024, partials, sl, hs, p.m, threadIdx.x);
        r = gf_mul_bits(X[kXtabLane + lane], r, poly);  // X^t = X^lane * X^(64 wave)
        r = gf_mul_bits(X[kXtabWave + (threadIdx.x >> 6)], r, poly);
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) r ^= (uint32_t)__shfl_xor((int)r, d);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = r;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t reg = 0u;
            for (uint32_t w = 0; w < blockDim.x / 64; ++w) reg ^= red[w];
            if (p.pad) reg = gf_mul_bits(xinv[p.pad], reg, poly);
            out[e] = ~reg;
        }
        __syncthreads();
    }
    __syncthreads();  // big[] and nbig are rebuilt by the next virtual block
    }
}

// ---- composite entries (bkd_crc_batch_segments) ----
// x^(8 * 2^b) mod P for b = 0..31: multiplying by x^(8*len) = one product per set bit of len.
struct XPow8 {
    uint32_t p[32];
};

// Entry i = segments first[i] .. first[i+1]-1 in order (DigestManager.update over ByteBufVisitor's
// leaves, DigestManager.java:62-72,380-392): reg = ~seed; per non-empty segment k,
// reg = reg * x^(8*len_k) ^ raw_k (raw_k = ~segcrc[k] = the segment's zero-initialised register);
// out = ~reg. One thread per entry.
__global__ void __launch_bounds__(256) segments_combine_kernel(const uint32_t* __restrict__ seg_lengths,
                                                               const uint32_t* __restrict__ segcrc,
                                                               const uint64_t* __restrict__ first, uint64_t n,
                                                               uint64_t nseg, const uint32_t* __restrict__ seeds,
                                                               uint32_t seed_all, XPow8 pw, uint32_t poly,
                                                               uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t reg = ~(seeds ? seeds[i] : seed_all);
    // a malformed seg_first (decreasing or past nseg) is clamped: never a read past the segments
    const uint64_t k1 = first[i + 1] < nseg ? first[i + 1] : nseg;
    for (uint64_t k = first[i]; k < k1; ++k) {
        uint32_t len = seg_lengths[k];
        if (!len) continue;  // ByteBufVisitor skips empty buffers (ByteBufVisitor.java:100-103,146-149)
        for (int b = 0; len; ++b, len >>= 1)
            if (len & 1u) reg = gf_mul_bits(pw.p[b], reg, poly);
        reg ^= ~segcrc[k];
    }
    out[i] = ~reg;
}

}  // namespace bkd
