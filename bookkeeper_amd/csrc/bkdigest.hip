// libbkdigest.so — C-ABI over the CDNA4 CRC kernels (include/bkdigest.h).
//
// Runtime glue: per-device operator-table images, launch geometry, per-stream bounds flags,
// the host-memory staging paths and the DigestManager batch framing sequences. The only CPU
// arithmetic is the per-call route for host buffers (host_crc.cpp, bkd_resume*); every batch
// entry point runs on the GPU and returns BKD_ERR_NO_DEVICE without one.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bkdigest.h"
#include "crc_kernels.hpp"
#include "plan_kernels.hpp"
#include "crc_tables.hpp"
#include "host_batch.hpp"
#include "host_crc.hpp"

namespace {

thread_local std::string t_err;

int fail(int code, const std::string& msg) {
    t_err = msg;
    return code;
}

#define BKD_HIP(expr)                                                                               \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) return fail(BKD_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

constexpr int kLaneChoices[6] = {1, 4, 8, 16, 32, 64};
constexpr int kNumLaneChoices = 6;
constexpr int kMaxDevices = 64;

int lane_index(int lanes) {
    for (int k = 0; k < kNumLaneChoices; ++k)
        if (kLaneChoices[k] == lanes) return k;
    return -1;
}

// Scratch kept per (device, stream) between calls. A call's kernels use it in stream order, so
// consecutive calls on one stream can share it; the launch sequence is enqueued under `mu` so that
// host threads sharing a stream do not interleave their sequences. It only grows: the old buffer is
// freed after a sync of its stream (growth is rare; per-call allocation left the GPU idle ~40 us
// between calls, profiles/r01_diag_ragged.log). Plain hipMalloc, not the stream-ordered pool:
// reused hipMallocAsync blocks fed stale data to the kernels on the host one-copy route (round 3,
// DESIGN.md §5a), so the library keeps no device memory of its own in that pool.
struct StreamScratch {
    std::recursive_mutex mu;
    uint8_t* buf[3] = {};  // slot 0: plan scratch (launch_plan), 1: verify pipeline, 2: segment CRCs
    size_t cap[3] = {};
    // Sticky bounds-violation flag of the indexed batches enqueued on this stream (one per
    // stream, so a caller's out-of-range entry is reported to that caller's bkd_stream_sync
    // only); read and cleared in stream order. h_err: pinned landing word for the read.
    uint32_t* err = nullptr;
    uint32_t* h_err = nullptr;
    // PlanRun word of the plans enqueued on this stream and the epoch of the latest one
    uint32_t* run = nullptr;
    uint32_t* uni = nullptr;  // PlanRun uniform-lengths word (the epoch of the call it holds for)
    uint32_t epoch = 0;
    // verify gate word (verify_gate_kernel) and the epoch of the latest verify on this stream
    uint32_t* vflag = nullptr;
    uint32_t vepoch = 0;
    hipError_t vflag_word(hipStream_t st, uint32_t** out) {
        if (!vflag) {
            hipError_t e = hipMalloc((void**)&vflag, sizeof(uint32_t));
            if (e == hipSuccess) e = hipMemsetAsync(vflag, 0, sizeof(uint32_t), st);
            if (e != hipSuccess) {
                vflag = nullptr;
                return e;
            }
        }
        *out = vflag;
        return hipSuccess;
    }
    hipError_t run_word(hipStream_t st, uint32_t** out) {
        if (!run) {
            hipError_t e = hipMalloc((void**)&run, sizeof(uint32_t));
            if (e == hipSuccess) e = hipMemsetAsync(run, 0, sizeof(uint32_t), st);
            if (e != hipSuccess) {
                run = nullptr;
                return e;
            }
        }
        *out = run;
        return hipSuccess;
    }
    hipError_t uni_word(hipStream_t st, uint32_t** out) {
        if (!uni) {
            hipError_t e = hipMalloc((void**)&uni, sizeof(uint32_t));
            if (e == hipSuccess) e = hipMemsetAsync(uni, 0, sizeof(uint32_t), st);
            if (e != hipSuccess) {
                uni = nullptr;
                return e;
            }
        }
        *out = uni;
        return hipSuccess;
    }
    hipError_t flag(hipStream_t st, uint32_t** out) {
        if (!err) {
            hipError_t e = hipMalloc((void**)&err, sizeof(uint32_t));
            if (e == hipSuccess) e = hipMemsetAsync(err, 0, sizeof(uint32_t), st);
            if (e == hipSuccess && !h_err) e = hipHostMalloc((void**)&h_err, sizeof(uint32_t), hipHostMallocDefault);
            if (e != hipSuccess) {
                err = nullptr;
                return e;
            }
        }
        *out = err;
        return hipSuccess;
    }
    // Returns slot `which` with at least `bytes` bytes, stream-ordered on `st`.
    hipError_t get(int which, size_t bytes, hipStream_t st, uint8_t** out) {
        if (cap[which] < bytes) {
            if (buf[which]) {  // work already enqueued on this stream may still use the old buffer
                const hipError_t e = hipStreamSynchronize(st);
                if (e != hipSuccess) return e;
                (void)hipFree(buf[which]);
            }
            buf[which] = nullptr;
            cap[which] = 0;
            const size_t want = bytes + bytes / 4 + 4096;
            hipError_t e = hipMalloc((void**)&buf[which], want);
            if (e != hipSuccess) return e;
            cap[which] = want;
        }
        *out = buf[which];
        return hipSuccess;
    }
};

// Lays out 256-byte-aligned sub-buffers of one scratch allocation: take() returns offsets
// during the sizing pass; at(base, off) turns them into pointers.
struct Carver {
    size_t used = 0;
    size_t take(size_t bytes) {
        const size_t at = used;
        used += (bytes + 255) & ~(size_t)255;
        return at;
    }
    template <class T>
    static T* at(uint8_t* base, size_t off) {
        return reinterpret_cast<T*>(base + off);
    }
};

// Per device: tables uploaded once (under g_mu, published by `ready`), then read-only; the two maps
// below grow on first use of an (algo, chunk size) or a stream and are read under a shared lock, so
// concurrent callers on their own streams never serialise on a process-wide lock.
struct DeviceState {
    std::atomic<bool> ready{false};
    int cus = 0;
    uint32_t* tables[2][kNumLaneChoices] = {};  // [algo][lane choice] compact operator images
    uint32_t* xinv[2] = {};       // [algo] x^(-8k), k = 0..127: removes the plan's zero padding
    std::shared_mutex maps_mu;    // guards xtab and scratch
    std::map<uint64_t, uint32_t*> xtab;  // (algo, CH) -> x^(8*CH) operator for the plan's combine
    std::map<hipStream_t, std::unique_ptr<StreamScratch>> scratch;
};

std::mutex g_mu;  // device initialisation only
DeviceState g_dev[kMaxDevices];
std::atomic<int> g_forced_lanes{0};
std::atomic<int> g_plan_mode{0};  // 0 auto, 1 direct (one entry per group), 2 chunked plan

// Chunked plan geometry (bkd_set_plan_geometry): lanes per group, steps per full chunk
// (CH = 16 * lanes * jc bytes) and the head-merge threshold in bytes.
std::atomic<int> g_plan_lanes{8};
std::atomic<int> g_plan_jc{32};
std::atomic<int> g_plan_merge{16};
std::atomic<int> g_fold_sched{0};  // bkd_set_fold_schedule: 0 by the measured clock, 1 fixed, 2 low-clock
std::atomic<int> g_plan_pf{2};  // loads in flight per lane in the chunk kernel (2, 4 or 8)
// Short-entry class of indexed batches: entries of <= this many bytes skip the plan and run in
// their own launch (4-lane groups, next entry loaded during the current one). 0 = none.
constexpr int kSmallLanes = 4;
constexpr uint32_t kSmallBytes4 = 16u * kSmallLanes * 3u;  // one register set per entry (4 lanes, PF = 2): 192 B
#ifndef BKD_SMALL_WIDE
#define BKD_SMALL_WIDE 8
#endif
constexpr int kSmallLanesWide = BKD_SMALL_WIDE;             // bounds above 192 B: 8 lanes, PF = 3 (16: 1 KiB)
constexpr uint32_t kSmallMaxBytes = 16u * kSmallLanesWide * 4u;
std::atomic<uint32_t> g_plan_small{kSmallBytes4};
// Entries shorter than this skip the chunks: plan_combine computes them, one thread each. Longer
// bounds cost more than they save on config 3's Zipf mix: 128 B took 36 us off the chunk kernel
// and added 54 us to combine (random slice-by-16 lookups from 64 lanes conflict in LDS banks).
#ifndef BKD_PLAN_SERIAL
#define BKD_PLAN_SERIAL 16
#endif
std::atomic<uint32_t> g_plan_serial{BKD_PLAN_SERIAL};
#ifndef BKD_SHORT_MEAN_MAX
#define BKD_SHORT_MEAN_MAX 1024
#endif
std::atomic<uint64_t> g_short_mean_max{BKD_SHORT_MEAN_MAX};  // bytes of base buffer per entry (bkd_set_short_class_mean)
#ifndef BKD_VERIFY_FUSED
#define BKD_VERIFY_FUSED 1
#endif
// Indexed batches whose base buffer is at most this size skip the plan (latency over balance).
constexpr uint64_t kDirectMaxBytes = 256u << 10;

// Visible HIP devices, probed once per process (0 when the runtime finds none).
int visible_devices() {
    static std::once_flag once;
    static int count = 0;
    std::call_once(once, [] {
        if (hipGetDeviceCount(&count) != hipSuccess) {
            (void)hipGetLastError();
            count = 0;
        }
    });
    return count;
}

// The device a call runs on: a created stream's own device (hipStreamGetDevice), else the
// calling thread's current device (null, legacy and per-thread default streams).
int stream_device(hipStream_t st, int* dev) {
    if (visible_devices() <= 0) return fail(BKD_ERR_NO_DEVICE, "no HIP device");
    if (st == nullptr || st == hipStreamLegacy || st == hipStreamPerThread) {
        BKD_HIP(hipGetDevice(dev));
    } else {
        hipDevice_t d = 0;
        BKD_HIP(hipStreamGetDevice(st, &d));
        *dev = (int)d;
    }
    if (*dev < 0 || *dev >= kMaxDevices) return fail(BKD_ERR_NO_DEVICE, "device index out of range");
    return BKD_OK;
}

// Makes the stream's device current for the duration of a call and restores the caller's.
struct DeviceScope {
    int prev = -1;
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int init_device_locked(int dev) {
    DeviceState& ds = g_dev[dev];
    if (ds.ready.load(std::memory_order_acquire)) return BKD_OK;
    int prev = 0;
    BKD_HIP(hipGetDevice(&prev));
    BKD_HIP(hipSetDevice(dev));
    hipDeviceProp_t prop;
    BKD_HIP(hipGetDeviceProperties(&prop, dev));
    ds.cus = prop.multiProcessorCount;
    std::vector<uint32_t> img;
    for (int algo = 0; algo < 2; ++algo) {
        for (int k = 0; k < kNumLaneChoices; ++k) {
            const int lanes = kLaneChoices[k];
            img.assign((size_t)bkd::gf2::compact_words(lanes), 0u);
            bkd::gf2::build_compact(algo, lanes, img.data());
            BKD_HIP(hipMalloc(&ds.tables[algo][k], img.size() * sizeof(uint32_t)));
            BKD_HIP(hipMemcpy(ds.tables[algo][k], img.data(), img.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        }
    }
    for (int algo = 0; algo < 2; ++algo) {
        uint32_t inv[128];
        for (uint32_t k = 0; k < 128; ++k) inv[k] = bkd::gf2::xpow_neg8(algo, k);
        BKD_HIP(hipMalloc(&ds.xinv[algo], sizeof(inv)));
        BKD_HIP(hipMemcpy(ds.xinv[algo], inv, sizeof(inv), hipMemcpyHostToDevice));
    }
    BKD_HIP(hipSetDevice(prev));
    ds.ready.store(true, std::memory_order_release);
    return BKD_OK;
}

// The plan combine's operators, built once per (algo, ch) and device (bkd::kXtab* layout):
// tables of X = x^(8*ch), X^64 and X^1024, then X^L (L = 0..63) and X^(64 w) (w = 0..15).
int xtab_for(DeviceState& ds, int algo, uint32_t ch, const uint32_t** out) {
    const uint64_t key = ((uint64_t)algo << 32) | ch;
    {
        std::shared_lock<std::shared_mutex> rd(ds.maps_mu);
        auto it = ds.xtab.find(key);
        if (it != ds.xtab.end()) {
            *out = it->second;
            return BKD_OK;
        }
    }
    std::unique_lock<std::shared_mutex> wr(ds.maps_mu);
    auto it = ds.xtab.find(key);
    if (it == ds.xtab.end()) {
        std::vector<uint32_t> xt(bkd::kXtabWords);
        bkd::gf2::operator_tables(algo, bkd::gf2::xpow(algo, 8ull * ch), xt.data() + bkd::kXtabX);
        bkd::gf2::operator_tables(algo, bkd::gf2::xpow(algo, 8ull * ch * 64u), xt.data() + bkd::kXtabX64);
        bkd::gf2::operator_tables(algo, bkd::gf2::xpow(algo, 8ull * ch * 1024u), xt.data() + bkd::kXtabX1024);
        for (uint32_t k = 0; k < 64u; ++k) xt[bkd::kXtabLane + k] = bkd::gf2::xpow(algo, 8ull * ch * k);
        for (uint32_t k = 0; k < 16u; ++k) xt[bkd::kXtabWave + k] = bkd::gf2::xpow(algo, 8ull * ch * 64u * k);
        uint32_t* d = nullptr;
        BKD_HIP(hipMalloc(&d, xt.size() * sizeof(uint32_t)));
        BKD_HIP(hipMemcpy(d, xt.data(), xt.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        it = ds.xtab.emplace(key, d).first;
    }
    *out = it->second;
    return BKD_OK;
}

int enter(hipStream_t st, DeviceScope& scope, DeviceState** out) {
    int dev = 0;
    int rc = stream_device(st, &dev);
    if (rc) return rc;
    int cur = 0;
    BKD_HIP(hipGetDevice(&cur));
    if (cur != dev) {
        BKD_HIP(hipSetDevice(dev));
        scope.prev = cur;
    }
    if (!g_dev[dev].ready.load(std::memory_order_acquire)) {  // first call on the device only
        std::lock_guard<std::mutex> lk(g_mu);
        rc = init_device_locked(dev);
    }
    if (rc) return rc;
    *out = &g_dev[dev];
    return BKD_OK;
}

// The stream's scratch, or nullptr when nothing was ever enqueued on it (no entry is created).
StreamScratch* scratch_find(DeviceState& ds, hipStream_t st) {
    std::shared_lock<std::shared_mutex> rd(ds.maps_mu);
    auto it = ds.scratch.find(st);
    return it == ds.scratch.end() ? nullptr : it->second.get();
}

StreamScratch& scratch_for(DeviceState& ds, hipStream_t st) {
    if (StreamScratch* sc = scratch_find(ds, st)) return *sc;  // hits take the shared lock only
    std::unique_lock<std::shared_mutex> wr(ds.maps_mu);
    auto& slot = ds.scratch[st];
    if (!slot) slot.reset(new StreamScratch());
    return *slot;
}

// Lanes per entry group for the direct kernel, from the size sweep (profiles/r01_size_sweep.log):
// 4 lanes below 512 B, 8 up to 32 KiB, 32 above; then more lanes while the batch would not give
// every lane slot of the chip (CUs x 1024) one group lane, so a few huge entries still fill it.
int auto_lanes(uint64_t mean_len, uint64_t n = UINT64_MAX, int cus = 256) {
    const int forced = g_forced_lanes.load();
    if (forced) return forced;
    int g = mean_len < 512 ? 4 : (mean_len < 32768 ? 8 : 32);
    while (g < 64 && n < UINT64_MAX / 64 && n * (uint64_t)g < (uint64_t)cus * 1024u) g *= 2;
    return g;
}

// Loads in flight per lane (register double buffer depth) and load cache policy; build-time
// knobs so variants can be A/B-timed in one process (tools/tune.py).
#ifndef BKD_PF
#define BKD_PF 2
#endif
#ifndef BKD_NT
#define BKD_NT 1
#endif
#ifndef BKD_PACKAGE_DIGEST_PASS
// 1: package digests written into the frames by their own kernel; 0: by the payload groups
// (PackageSrc), which measured 3 % slower on 1M x 4 KiB (profiles/r03m_ab_order*.log)
#define BKD_PACKAGE_DIGEST_PASS 1
#endif
constexpr int kPF = BKD_PF;
constexpr bool kNT = BKD_NT != 0;

template <int G, class Src>
int launch_groups(DeviceState& ds, int algo, const uint8_t* base, const Src& src, uint64_t host_count,
                  hipStream_t stream, uint32_t* err) {
    if (host_count == 0) return BKD_OK;
    const uint64_t groups_per_block = bkd::kBlock / G;
    uint64_t blocks = (host_count + groups_per_block - 1) / groups_per_block;
    blocks = std::min<uint64_t>(blocks, (uint64_t)ds.cus);
    const uint32_t* tab = ds.tables[algo][lane_index(G)];
    hipLaunchKernelGGL((bkd::crc_groups_kernel<G, kPF, kNT, Src>), dim3((unsigned)blocks), dim3(bkd::kBlock), 0,
                       stream, base, src, tab, err, g_fold_sched.load());
    BKD_HIP(hipGetLastError());
    return BKD_OK;
}

// host_count: an upper bound of src.count() used only to size the grid.
template <class Src>
int dispatch_lanes(DeviceState& ds, int lanes, int algo, const uint8_t* base, const Src& src, uint64_t host_count,
                   hipStream_t stream, uint32_t* err = nullptr) {
    switch (lanes) {
        case 1: return launch_groups<1>(ds, algo, base, src, host_count, stream, err);
        case 4: return launch_groups<4>(ds, algo, base, src, host_count, stream, err);
        case 8: return launch_groups<8>(ds, algo, base, src, host_count, stream, err);
        case 16: return launch_groups<16>(ds, algo, base, src, host_count, stream, err);
        case 32: return launch_groups<32>(ds, algo, base, src, host_count, stream, err);
        case 64: return launch_groups<64>(ds, algo, base, src, host_count, stream, err);
        default: return fail(BKD_ERR_INVALID_ARG, "lanes must be 1, 4, 8, 16, 32 or 64");
    }
}

template <int G>
void launch_plan_chunks(const bkd::PlanRun& run, const uint8_t* base, const bkd::PlanDesc* descs, bool d8,
                        uint32_t r0h, const uint32_t* count, const uint32_t* tab,
                        uint32_t* out, uint32_t* partials, const bkd::PlanDirectSrc& ov, int blocks, hipStream_t st,
                        uint32_t* err, int pf) {
    // pf: read once by launch_plan (one value per call); d8 (PlanDesc8) only with the default pf
    if (pf == 8)
        hipLaunchKernelGGL((bkd::crc_plan_chunks_kernel<G, 8, kNT, bkd::PlanDirectSrc>), dim3((unsigned)blocks),
                           dim3(bkd::kBlock), 0, st, base, descs, r0h, count, tab, out, partials, ov, run, err);
    else if (pf == 4)
        hipLaunchKernelGGL((bkd::crc_plan_chunks_kernel<G, 4, kNT, bkd::PlanDirectSrc>), dim3((unsigned)blocks),
                           dim3(bkd::kBlock), 0, st, base, descs, r0h, count, tab, out, partials, ov, run, err);
    else if (d8)
        hipLaunchKernelGGL((bkd::crc_plan_chunks_kernel<G, 2, kNT, bkd::PlanDirectSrc, bkd::PlanDesc8>),
                           dim3((unsigned)blocks), dim3(bkd::kBlock), 0, st, base,
                           reinterpret_cast<const bkd::PlanDesc8*>(descs), r0h, count, tab, out, partials, ov, run,
                           err);
    else
        hipLaunchKernelGGL((bkd::crc_plan_chunks_kernel<G, 2, kNT, bkd::PlanDirectSrc>), dim3((unsigned)blocks),
                           dim3(bkd::kBlock), 0, st, base, descs, r0h, count, tab, out, partials, ov, run, err);
}

// Indexed batch through the chunked plan (plan_kernels.hpp): five stream-ordered kernels, no
// host sync, scratch from the stream's arena.
int launch_plan(DeviceState& ds, int algo, const uint8_t* base, uint64_t size, const uint64_t* offsets,
                const uint32_t* lengths, uint64_t n, const uint32_t* seeds, uint32_t seed_all, uint32_t* out,
                hipStream_t st, bool short_class = true, bool direct_gate = true, const uint32_t* ext_flag = nullptr,
                uint32_t ext_epoch = 0) {
    // ext_flag: the plan runs only if *ext_flag == ext_epoch when its kernels start (a gate decided on
    // the device before this call, verify_framed's); no short class and no uniformity gate then
    if (n == 0) return BKD_OK;
    if (ext_flag) short_class = direct_gate = false;
    if (n >= 0xFFFFFFF0ull) return fail(BKD_ERR_INVALID_ARG, "indexed batches hold fewer than 2^32 - 16 entries");
    const int G = g_plan_lanes.load();
    bkd::PlanGeo pg;
    pg.step = 16u * (uint32_t)G;
    pg.jc = (uint32_t)g_plan_jc.load();
    pg.ch = pg.step * pg.jc;
    pg.mis = (uint32_t)((uintptr_t)base & 127u);
    pg.merge = (uint32_t)g_plan_merge.load();
    pg.serial = g_plan_serial.load();
    // chunks of <= kShortPF + 1 steps: the chunk kernel's short tail, three chunks in flight per
    // group (short_chunks_loop; BKD_SHORT_TAIL=0 builds the single-prefetch schedule for A/B timing)
#ifndef BKD_SHORT_TAIL
#define BKD_SHORT_TAIL 1
#endif
    const int pf = g_plan_pf.load();
    pg.jshort = BKD_SHORT_TAIL ? (uint32_t)bkd::kShortPF + 1u : 0u;
    // 8-byte descriptors when the batch has one seed for every entry (its head register is then a
    // kernel argument) and the default loads in flight (PlanDesc8, crc_kernels.hpp)
#ifndef BKD_PLAN_D8
#define BKD_PLAN_D8 1
#endif
    pg.d8 = (BKD_PLAN_D8 && seeds == nullptr && size < bkd::kPlanMaxSize8 && pf == 2) ? 1u : 0u;
    pg.nbins = (pg.ch + pg.merge - 1u + pg.step - 1u) / pg.step + 1u;
    pg.step_sh = (uint32_t)__builtin_ctz(pg.step);
    pg.ch_sh = (pg.ch & (pg.ch - 1u)) == 0u ? (uint32_t)__builtin_ctz(pg.ch) : 0xFFu;
    // The short-entry launch walks every entry's index in rounds of one entry per 4-lane group, a
    // memory round trip each: it pays where short entries dominate (64 M x 64 B: 7.2 -> 1.9 ms) and
    // costs more than it saves where they are a minority of a large-entry batch (config 3's Zipf:
    // +54 us launch, -43 us chunk kernel). So it runs when the mean entry is at most 1 KiB.
    const uint64_t mean_max = g_short_mean_max.load();
    // size <= mean_max * n, without forming the product (it could overflow for large bounds)
    const bool short_gate = mean_max == UINT64_MAX || size / n < mean_max || (size / n == mean_max && size % n == 0u);
    pg.small = (short_class && short_gate) ? g_plan_small.load() : 0u;
    const uint32_t* xtab = nullptr;
    int rc = xtab_for(ds, algo, pg.ch, &xtab);
    if (rc) return rc;
    // non-overlapping entries need at most sum(ceil((len + 127) / CH)) <= n + (size + 127 n) / CH chunks
    const uint64_t capacity = std::min<uint64_t>(n + (size + 128u * n) / pg.ch + 16, 0xFFFFFFF0ull);
    const uint32_t nb = (uint32_t)((n + bkd::kPlanBlock - 1) / bkd::kPlanBlock);
    const uint32_t ncols = bkd::plan_ncols(pg);
    Carver cv;
    const size_t o_blk = cv.take((size_t)nb * ncols * 4), o_live = cv.take((size_t)nb * 4),
                 o_bok = cv.take((size_t)nb * 4),
                 o_blkoff = cv.take((size_t)nb * ncols * 4), o_hdr = cv.take(bkd::kHdrWords * 4),
                 o_ps = cv.take((size_t)n * 4), o_hs = cv.take((size_t)n * 4), o_part = cv.take((size_t)capacity * 4),
                 o_desc = cv.take((size_t)capacity * sizeof(bkd::PlanDesc));
    StreamScratch& sc = scratch_for(ds, st);
    std::lock_guard<std::recursive_mutex> lk(sc.mu);
    uint8_t* sb = nullptr;
    uint32_t* err = nullptr;
    uint32_t* run_word = nullptr;
    uint32_t* uni = nullptr;
    // without a short class (mean entry > 1 KiB), lengths all within 1/16 + 64 B of the first
    // entry's skip the chunks: the chunk kernel computes them whole, as the direct kernel would (PlanRun::uniform,
    // decided on the device: plan_count's per-block ballots, reduced by plan_scan). Only where the
    // direct kernel would use the plan's lane count.
#ifndef BKD_DIRECT_GATE
#define BKD_DIRECT_GATE 1
#endif
    const bool gate = BKD_DIRECT_GATE && pg.small == 0u && direct_gate && auto_lanes(size / n, n, ds.cus) == G;
    hipError_t e = sc.get(0, cv.used, st, &sb);
    if (e == hipSuccess) e = sc.flag(st, &err);
    if (e == hipSuccess && pg.small) e = sc.run_word(st, &run_word);
    if (e == hipSuccess && gate) e = sc.uni_word(st, &uni);
    if (e != hipSuccess) return fail(BKD_ERR_NOMEM, std::string("plan scratch: ") + hipGetErrorString(e));
    if (++sc.epoch == 0u) ++sc.epoch;  // 0 is the words' initial value
    const bkd::PlanRun run = ext_flag ? bkd::PlanRun{ext_flag, nullptr, ext_epoch} : bkd::PlanRun{run_word, uni, sc.epoch};
    uint32_t *blk = Carver::at<uint32_t>(sb, o_blk), *blive = Carver::at<uint32_t>(sb, o_live),
             *bok = gate ? Carver::at<uint32_t>(sb, o_bok) : nullptr,
             *blkoff = Carver::at<uint32_t>(sb, o_blkoff), *hdr = Carver::at<uint32_t>(sb, o_hdr),
             *pslot = Carver::at<uint32_t>(sb, o_ps), *hslot = Carver::at<uint32_t>(sb, o_hs),
             *partials = Carver::at<uint32_t>(sb, o_part);
    bkd::PlanDesc* descs = Carver::at<bkd::PlanDesc>(sb, o_desc);
    if (pg.small) {  // the short-entry class, in its own launch (any order against the plan kernels)
        const bkd::SmallIndexedSrc ss{n, offsets, lengths, seeds, seed_all, size, out, pg.small, run_word, run.epoch};
        if (pg.small <= kSmallBytes4) {
            const uint64_t per_block = bkd::kBlock / kSmallLanes;
            const unsigned sblocks = (unsigned)std::min<uint64_t>((n + per_block - 1) / per_block, (uint64_t)ds.cus);
            hipLaunchKernelGGL((bkd::crc_groups_kernel<kSmallLanes, 2, kNT, bkd::SmallIndexedSrc>), dim3(sblocks),
                               dim3(bkd::kBlock), 0, st, base, ss, ds.tables[algo][lane_index(kSmallLanes)], err, 1);
        } else {  // bounds above 192 B: kSmallLanesWide-lane groups (8: up to 512 B), an entry's PF + 1 steps in one register set
            const uint64_t per_block = bkd::kBlock / kSmallLanesWide;
            const unsigned sblocks = (unsigned)std::min<uint64_t>((n + per_block - 1) / per_block, (uint64_t)ds.cus);
            hipLaunchKernelGGL((bkd::crc_groups_kernel<kSmallLanesWide, 3, kNT, bkd::SmallIndexedSrc>), dim3(sblocks),
                               dim3(bkd::kBlock), 0, st, base, ss, ds.tables[algo][lane_index(kSmallLanesWide)], err, 1);
        }
    }
    // count / emit / combine walk their 1024-entry blocks in grid stride (BKD_PLAN_GRID blocks per CU;
    // 0: one block per entry block)
#ifndef BKD_PLAN_GRID
#define BKD_PLAN_GRID 2
#endif
    const uint32_t pgrid = BKD_PLAN_GRID ? (uint32_t)BKD_PLAN_GRID * (uint32_t)ds.cus : 0xFFFFFFFFu;
    const uint32_t cgrid = std::min((nb + bkd::kCountBlocks - 1u) / bkd::kCountBlocks, pgrid);
    hipLaunchKernelGGL(bkd::plan_count_kernel, dim3(cgrid), dim3(bkd::kPlanBlock), 0, st, offsets,
                       lengths, size, n, pg, blk, blive, nb, run, bok);
    hipLaunchKernelGGL(bkd::plan_scan_kernel, dim3(ncols + (gate ? 1u : 0u)), dim3(bkd::kPlanBlock), 0, st, blk, nb,
                       blkoff, hdr, run, ncols, bok);
    // few entry blocks (large entries): replicate emit and combine blocks so ~2 blocks per CU work
    const uint32_t reps = nb >= 2u * (uint32_t)ds.cus ? 1u : std::min<uint32_t>(64u, (2u * (uint32_t)ds.cus + nb - 1u) / nb);
    hipLaunchKernelGGL(bkd::plan_emit_kernel, dim3(std::min(nb * reps, pgrid)), dim3(bkd::kPlanBlock), 0, st, offsets,
                       lengths, seeds, seed_all, size, n, pg, capacity, blkoff, pslot, hslot, hdr, descs, reps, blive, nb, run);
    const uint32_t* tab = ds.tables[algo][lane_index(G)];
    const bkd::PlanDirectSrc ov{n, offsets, lengths, seeds, seed_all, size, out, pslot, hdr, capacity, false};
    switch (G) {
        case 4: launch_plan_chunks<4>(run, base, descs, pg.d8 != 0u, ~seed_all, hdr + bkd::kHdrWork, tab, out, partials, ov, ds.cus, st, err, pf); break;
        case 8: launch_plan_chunks<8>(run, base, descs, pg.d8 != 0u, ~seed_all, hdr + bkd::kHdrWork, tab, out, partials, ov, ds.cus, st, err, pf); break;
        case 16: launch_plan_chunks<16>(run, base, descs, pg.d8 != 0u, ~seed_all, hdr + bkd::kHdrWork, tab, out, partials, ov, ds.cus, st, err, pf); break;
        case 32: launch_plan_chunks<32>(run, base, descs, pg.d8 != 0u, ~seed_all, hdr + bkd::kHdrWork, tab, out, partials, ov, ds.cus, st, err, pf); break;
        default: launch_plan_chunks<64>(run, base, descs, pg.d8 != 0u, ~seed_all, hdr + bkd::kHdrWork, tab, out, partials, ov, ds.cus, st, err, pf); break;
    }
    const uint32_t* btab = tab + bkd::gf2::byte_table_offset(G);
    hipLaunchKernelGGL(bkd::plan_combine_kernel, dim3(std::min(nb * reps, pgrid)), dim3(1024), 0, st, base, offsets, lengths, seeds,
                       seed_all, size, n, pg, xtab, btab, ds.xinv[algo],
                       bkd::gf2::poly(algo), pslot, hslot, partials, out, err, reps, blive, nb, run);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(BKD_ERR_HIP, std::string("plan kernels: ") + hipGetErrorString(e));
    return BKD_OK;
}

// The route indexed_batch takes: the direct kernel (one entry per group) or the chunked plan.
bool indexed_direct(uint64_t size) {
    const int mode = g_plan_mode.load();
    // plan descriptors hold a biased 41-bit window start (PlanDesc): buffers >= 1 TiB take the direct kernel
    return mode == 1 || (mode == 0 && size <= kDirectMaxBytes) || size >= bkd::kPlanMaxSize;
}

// route: -1 decided here from the plan mode and the buffer size, else the caller's decision
// (0 direct, 1 plan) so that a route chosen once per call cannot change under bkd_set_plan_mode.
int indexed_batch(DeviceState& ds, int algo, const uint8_t* base, uint64_t size, const uint64_t* offsets,
                  const uint32_t* lengths, uint64_t n, const uint32_t* seeds, uint32_t seed_all, uint32_t* out,
                  hipStream_t st, const uint32_t* ext_flag, uint32_t ext_epoch, int route) {
    if (route < 0) route = indexed_direct(size) ? 0 : 1;
    if (route == 1)
        return launch_plan(ds, algo, base, size, offsets, lengths, n, seeds, seed_all, out, st, true, true, ext_flag,
                           ext_epoch);
    uint32_t* err = nullptr;
    {
        StreamScratch& sc = scratch_for(ds, st);
        std::lock_guard<std::recursive_mutex> lk(sc.mu);
        const hipError_t e = sc.flag(st, &err);
        if (e != hipSuccess) return fail(BKD_ERR_NOMEM, std::string("bounds flag: ") + hipGetErrorString(e));
    }
    bkd::IndexedSrc src{n, offsets, lengths, seeds, seed_all, size, out};
    return dispatch_lanes(ds, auto_lanes(n ? size / n : 0, n, ds.cus), algo, base, src, n, st, err);
}

bool valid_algo(int algo) { return algo == BKD_CRC32C || algo == BKD_CRC32; }

// Whether p is device memory; *dev (if given) = the device it lives on.
bool is_device_pointer(const void* p, int* dev = nullptr) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (dev) *dev = attr.device;
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// ---- host-memory batches: pinned, double-buffered H2D -> kernel -> D2H -------------------
// Entries sorted by offset are cut into segments of at most kSeg payload bytes / kSegEntries
// entries; segment k uses staging slot k % 2 (its own stream), so the H2D copy of one segment
// overlaps the kernel and D2H of the other. A pinned (page-locked / registered) source is DMA'd
// in place; a pageable one is first copied into the slot's pinned buffer by the host.
struct HostStage {
    static constexpr size_t kSeg = 64u << 20;
    static constexpr size_t kSegEntries = 1u << 20;
    bool ready = false;
    uint8_t* h_pin[2] = {};
    uint8_t* d_buf[2] = {};
    uint64_t* h_off[2] = {};
    uint32_t* h_len[2] = {};
    uint32_t* h_seed[2] = {};
    uint32_t* h_res[2] = {};
    uint64_t* d_off[2] = {};
    uint32_t* d_len[2] = {};
    uint32_t* d_seed[2] = {};
    uint32_t* d_res[2] = {};
    hipStream_t st[2] = {};
    hipEvent_t done[2] = {};
    // framed-entry batches (bkd_digest_*_batch_host), allocated on first use and sized per path
    // (ADVICE r2): package needs per-entry ids, LACs and length fields in (24 B per entry) and the
    // frame headers out; verify only its first_bad word
    static constexpr size_t kAux = 64u << 20;
    bool pkg_ready = false, fb_ready = false;
    uint8_t* h_aux[2] = {};
    uint8_t* d_aux[2] = {};
    uint8_t* h_frm[2] = {};
    uint8_t* d_frm[2] = {};
    uint64_t* h_fb[2] = {};
    uint64_t* d_fb[2] = {};
    // (each allocation is made once: a call after a failed init completes the set, nothing leaks)
    int init_package() {
        if (pkg_ready) return BKD_OK;
        for (int s = 0; s < 2; ++s) {
            if (!h_aux[s]) BKD_HIP(hipHostMalloc((void**)&h_aux[s], kAux, hipHostMallocDefault));
            if (!d_aux[s]) BKD_HIP(hipMalloc((void**)&d_aux[s], kAux));
            if (!h_frm[s]) BKD_HIP(hipHostMalloc((void**)&h_frm[s], kAux, hipHostMallocDefault));
            if (!d_frm[s]) BKD_HIP(hipMalloc((void**)&d_frm[s], kAux));
        }
        pkg_ready = true;
        return BKD_OK;
    }
    int init_verify() {
        if (fb_ready) return BKD_OK;
        for (int s = 0; s < 2; ++s) {
            if (!h_fb[s]) BKD_HIP(hipHostMalloc((void**)&h_fb[s], sizeof(uint64_t), hipHostMallocDefault));
            if (!d_fb[s]) BKD_HIP(hipMalloc((void**)&d_fb[s], sizeof(uint64_t)));
        }
        fb_ready = true;
        return BKD_OK;
    }
    ~HostStage() {  // (bkd_host_release: idle sets only, so no work of theirs is queued)
        for (int s = 0; s < 2; ++s) {
            for (void* h : {(void*)h_pin[s], (void*)h_off[s], (void*)h_len[s], (void*)h_seed[s], (void*)h_res[s],
                            (void*)h_aux[s], (void*)h_frm[s], (void*)h_fb[s]})
                if (h) (void)hipHostFree(h);
            for (void* d : {(void*)d_buf[s], (void*)d_off[s], (void*)d_len[s], (void*)d_seed[s], (void*)d_res[s],
                            (void*)d_aux[s], (void*)d_frm[s], (void*)d_fb[s]})
                if (d) (void)hipFree(d);
            if (st[s]) (void)hipStreamDestroy(st[s]);
            if (done[s]) (void)hipEventDestroy(done[s]);
        }
    }
    int init() {
        if (ready) return BKD_OK;
        for (int s = 0; s < 2; ++s) {
            if (!h_pin[s]) BKD_HIP(hipHostMalloc((void**)&h_pin[s], kSeg, hipHostMallocDefault));
            if (!d_buf[s]) BKD_HIP(hipMalloc((void**)&d_buf[s], kSeg));
            if (!h_off[s]) BKD_HIP(hipHostMalloc((void**)&h_off[s], kSegEntries * 8, hipHostMallocDefault));
            if (!h_len[s]) BKD_HIP(hipHostMalloc((void**)&h_len[s], kSegEntries * 4, hipHostMallocDefault));
            if (!h_seed[s]) BKD_HIP(hipHostMalloc((void**)&h_seed[s], kSegEntries * 4, hipHostMallocDefault));
            if (!h_res[s]) BKD_HIP(hipHostMalloc((void**)&h_res[s], kSegEntries * 4, hipHostMallocDefault));
            if (!d_off[s]) BKD_HIP(hipMalloc((void**)&d_off[s], kSegEntries * 8));
            if (!d_len[s]) BKD_HIP(hipMalloc((void**)&d_len[s], kSegEntries * 4));
            if (!d_seed[s]) BKD_HIP(hipMalloc((void**)&d_seed[s], kSegEntries * 4));
            if (!d_res[s]) BKD_HIP(hipMalloc((void**)&d_res[s], kSegEntries * 4));
            if (!st[s]) BKD_HIP(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
            if (!done[s]) BKD_HIP(hipEventCreateWithFlags(&done[s], hipEventDisableTiming));
        }
        ready = true;
        return BKD_OK;
    }
};

// Host-resident batches from concurrent callers each take a staging set of their own (created on
// demand, at most BKD_HOST_STAGES per device, default 4; a caller beyond that waits for one), so
// one caller's gather and PCIe copies do not hold up another's (no global lock on the
// hot path). A set with the framed-entry buffers is ~0.4 GiB of pinned memory.
struct StagePool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::unique_ptr<HostStage>> all;
    std::vector<HostStage*> idle;
};
// Deliberately never destroyed: static destructors run after HIP's own teardown, where
// hipHostFree / hipStreamDestroy can crash or hang at exit; bkd_host_release frees idle sets instead.
StagePool* const g_stages = new StagePool[kMaxDevices];

size_t max_stages() {
    static const size_t m = [] {
        const char* v = getenv("BKD_HOST_STAGES");
        const int k = v ? atoi(v) : 4;
        return (size_t)std::max(1, std::min(64, k));
    }();
    return m;
}

// A staging set for the duration of one host-resident call.
class StageLease {
  public:
    explicit StageLease(int dev) : pool_(g_stages[dev]) {
        std::unique_lock<std::mutex> lk(pool_.mu);
        pool_.cv.wait(lk, [&] { return !pool_.idle.empty() || pool_.all.size() < max_stages(); });
        if (!pool_.idle.empty()) {
            hs_ = pool_.idle.back();
            pool_.idle.pop_back();
        } else {
            pool_.all.emplace_back(new HostStage());
            hs_ = pool_.all.back().get();
        }
    }
    ~StageLease() {
        {
            std::lock_guard<std::mutex> lk(pool_.mu);
            pool_.idle.push_back(hs_);
        }
        pool_.cv.notify_one();
    }
    HostStage& operator*() const { return *hs_; }

  private:
    StagePool& pool_;
    HostStage* hs_ = nullptr;
};

// Host copies into pinned staging (a pageable source, or a list of separate entry buffers such as a
// ByteBufList) run on the library's host pool (host_batch.hpp): one core copies ~10-20 GB/s, below
// PCIe Gen5's ~55. At most BKD_COPY_THREADS parts (default 8: 12 measured no better on the 16-core
// share of the GPU box, host verify of 1M separate 4 KiB frames 42.5 vs 43.4 GiB/s mean).
int copy_threads() {
    static const int t = [] {
        const char* v = getenv("BKD_COPY_THREADS");
        return v ? std::max(1, std::min(64, atoi(v))) : 8;
    }();
    return std::min(t, bkd::host::Pool::get().active());
}

// Bytes per copy-pool part (BKD_COPY_PART_KIB overrides the default).
size_t copy_part_bytes() {
    static const size_t b = [] {
        const char* v = getenv("BKD_COPY_PART_KIB");
        const long k = v ? atol(v) : 4096;
        return (size_t)std::max(64L, std::min(1L << 20, k)) << 10;
    }();
    return b;
}

// memcpy of one range on the copy pool (parts of >= copy_part_bytes()).
void parallel_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    bkd::host::Pool& pool = bkd::host::Pool::get();
    const int parts = (int)std::min<size_t>((size_t)copy_threads(), std::max<size_t>(1, n / copy_part_bytes()));
    const size_t per = (n + parts - 1) / parts;
    pool.run(parts, [&](int p) {
        const size_t a = std::min(n, per * (size_t)p), b = std::min(n, a + per);
        if (b > a) memcpy(dst + a, src + a, b - a);
    });
}

// Packs entries src[i] (len[i] bytes) back to back into dst; off[i] = where entry i landed.
// Split over the copy pool by bytes.
void gather_entries(const void* const* src, const uint32_t* len, uint64_t cnt, uint8_t* dst, uint64_t* off) {
    uint64_t at = 0;
    for (uint64_t i = 0; i < cnt; ++i) {
        off[i] = at;
        at += len[i];
    }
    bkd::host::Pool& pool = bkd::host::Pool::get();
    const int parts = (int)std::min<uint64_t>((uint64_t)copy_threads(), std::max<uint64_t>(1, at / copy_part_bytes()));
    const uint64_t per = (at + parts - 1) / parts;
    pool.run(parts, [&](int p) {
        // entries whose first byte lies in [p*per, (p+1)*per)
        const uint64_t lo = per * (uint64_t)p, hi = lo + per;
        uint64_t i = (uint64_t)(std::lower_bound(off, off + cnt, lo) - off);
        for (; i < cnt && off[i] < hi; ++i)
            if (len[i]) memcpy(dst + off[i], src[i], len[i]);
    });
}

int indexed_batch(DeviceState& ds, int algo, const uint8_t* base, uint64_t size, const uint64_t* offsets,
                  const uint32_t* lengths, uint64_t n, const uint32_t* seeds, uint32_t seed_all, uint32_t* out,
                  hipStream_t st, const uint32_t* ext_flag = nullptr, uint32_t ext_epoch = 0, int route = -1);

bool is_pinned_host(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

// Unsorted index: one device copy of the spanned bytes. The buffers are allocated with hipMalloc
// and released with hipFree: reusing stream-ordered (hipMallocAsync) allocations of this size for
// the copy gave wrong digests from the second call on (128-512 MiB spans, both pinned and pageable
// sources, with or without a sync after the copy; tools/diag_host_big.py, profiles/r03l_*), and
// hipMalloc'd buffers did not.
int host_batch_oneshot(DeviceState& ds, HostStage& hs, int algo, const uint8_t* h_base, uint64_t base_size,
                       const uint64_t* h_offsets, const uint32_t* h_lengths, uint64_t n, const uint32_t* h_seeds,
                       uint32_t seed_all, uint32_t* h_out) {
    hipStream_t st = hs.st[0];
    uint8_t* d_base = nullptr;
    uint64_t* d_off = nullptr;
    uint32_t *d_len = nullptr, *d_seeds = nullptr, *d_out = nullptr;
    hipError_t e = hipSuccess;
    if (base_size) e = hipMalloc((void**)&d_base, base_size);
    if (e == hipSuccess) e = hipMalloc((void**)&d_off, n * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&d_len, n * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&d_out, n * 4);
    if (e == hipSuccess && h_seeds) e = hipMalloc((void**)&d_seeds, n * 4);
    int rc = BKD_OK;
    if (e != hipSuccess) rc = fail(BKD_ERR_NOMEM, std::string("host batch staging: ") + hipGetErrorString(e));
    if (rc == BKD_OK && base_size) e = hipMemcpyAsync(d_base, h_base, base_size, hipMemcpyHostToDevice, st);
    if (rc == BKD_OK && e == hipSuccess) e = hipMemcpyAsync(d_off, h_offsets, n * 8, hipMemcpyHostToDevice, st);
    if (rc == BKD_OK && e == hipSuccess) e = hipMemcpyAsync(d_len, h_lengths, n * 4, hipMemcpyHostToDevice, st);
    if (rc == BKD_OK && e == hipSuccess && h_seeds) e = hipMemcpyAsync(d_seeds, h_seeds, n * 4, hipMemcpyHostToDevice, st);
    if (rc == BKD_OK && e != hipSuccess) rc = fail(BKD_ERR_HIP, std::string("host batch staging: ") + hipGetErrorString(e));
    if (rc == BKD_OK) rc = indexed_batch(ds, algo, d_base, base_size, d_off, d_len, n, d_seeds, seed_all, d_out, st);
    if (rc == BKD_OK) {
        e = hipMemcpyAsync(h_out, d_out, n * 4, hipMemcpyDeviceToHost, st);
        if (e != hipSuccess) rc = fail(BKD_ERR_HIP, std::string("host batch: ") + hipGetErrorString(e));
    }
    e = hipStreamSynchronize(st);
    if (rc == BKD_OK && e != hipSuccess) rc = fail(BKD_ERR_HIP, std::string("host batch: ") + hipGetErrorString(e));
    for (void* p : {(void*)d_base, (void*)d_off, (void*)d_len, (void*)d_seeds, (void*)d_out})
        if (p) (void)hipFree(p);
    return rc;
}

int host_batch_pipelined(DeviceState& ds, HostStage& hs, int algo, const uint8_t* h_base, const uint64_t* h_offsets,
                         const uint32_t* h_lengths, uint64_t n, const uint32_t* h_seeds, uint32_t seed_all,
                         uint32_t* h_out) {
    const bool pinned = is_pinned_host(h_base);
    uint64_t pend_i0[2] = {0, 0}, pend_cnt[2] = {0, 0};
    bool busy[2] = {false, false};
    auto drain = [&](int s) -> int {  // wait for slot s and hand its digests back
        if (!busy[s]) return BKD_OK;
        BKD_HIP(hipEventSynchronize(hs.done[s]));
        memcpy(h_out + pend_i0[s], hs.h_res[s], pend_cnt[s] * 4);
        busy[s] = false;
        return BKD_OK;
    };
    uint64_t i0 = 0;
    int rc = BKD_OK;
    for (int k = 0; i0 < n && rc == BKD_OK; ++k) {
        const int s = k & 1;
        const uint64_t b0 = h_offsets[i0];
        uint64_t i1 = i0, b1 = b0;
        while (i1 < n && i1 - i0 < HostStage::kSegEntries) {
            const uint64_t e1 = std::max<uint64_t>(b1, h_offsets[i1] + h_lengths[i1]);
            if (e1 - b0 > HostStage::kSeg && i1 > i0) break;
            b1 = e1;
            ++i1;
        }
        const uint64_t cnt = i1 - i0, span = b1 - b0;  // span <= kSeg: longer entries arrive in pieces
        if ((rc = drain(s))) break;
        for (uint64_t j = 0; j < cnt; ++j) {
            hs.h_off[s][j] = h_offsets[i0 + j] - b0;
            hs.h_len[s][j] = h_lengths[i0 + j];
        }
        if (h_seeds) memcpy(hs.h_seed[s], h_seeds + i0, cnt * 4);
        const uint8_t* src = h_base + b0;
        if (!pinned) {
            parallel_copy(hs.h_pin[s], src, span);
            src = hs.h_pin[s];
        }
        hipStream_t st = hs.st[s];
        hipError_t e = hipMemcpyAsync(hs.d_buf[s], src, span, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(hs.d_off[s], hs.h_off[s], cnt * 8, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(hs.d_len[s], hs.h_len[s], cnt * 4, hipMemcpyHostToDevice, st);
        if (e == hipSuccess && h_seeds) e = hipMemcpyAsync(hs.d_seed[s], hs.h_seed[s], cnt * 4, hipMemcpyHostToDevice, st);
        if (e != hipSuccess) {
            rc = fail(BKD_ERR_HIP, std::string("host batch H2D: ") + hipGetErrorString(e));
            break;
        }
        rc = indexed_batch(ds, algo, hs.d_buf[s], span, hs.d_off[s], hs.d_len[s], cnt, h_seeds ? hs.d_seed[s] : nullptr,
                           seed_all, hs.d_res[s], st);
        if (rc) break;
        e = hipMemcpyAsync(hs.h_res[s], hs.d_res[s], cnt * 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipEventRecord(hs.done[s], st);
        if (e != hipSuccess) {
            rc = fail(BKD_ERR_HIP, std::string("host batch D2H: ") + hipGetErrorString(e));
            break;
        }
        busy[s] = true;
        pend_i0[s] = i0;
        pend_cnt[s] = cnt;
        i0 = i1;
    }
    const int r0 = drain(0), r1 = drain(1);
    return rc ? rc : (r0 ? r0 : r1);
}

// ---- DigestManager batch framing: the device sequences shared by the device- and host-resident
// entry points -------------------------------------------------------------------------------

// Package, fused route (4..64-lane groups, frames apart from the payload; BKD_PACKAGE_FUSED): each lane group
// builds its entry's header from the index arrays and folds header + payload in one pass, storing the
// digest (crc_package_fused_kernel); package_frame_kernel then writes every frame's header and digest.
template <int G>
void launch_package_fused(DeviceState& ds, hipStream_t st, int algo, int64_t ledger_id, const int64_t* d_entry_ids,
                          const int64_t* d_lacs, const int64_t* d_length_fields, const uint8_t* payload,
                          uint64_t payload_size, const uint64_t* d_offsets, const uint32_t* d_lengths, uint64_t n,
                          uint32_t* d_digests, uint32_t* err) {
    const uint64_t per_block = bkd::kBlock / G;
    const unsigned blocks = (unsigned)std::min<uint64_t>((n + per_block - 1) / per_block, (uint64_t)ds.cus);
    hipLaunchKernelGGL((bkd::crc_package_fused_kernel<G, kPF, kNT>), dim3(blocks), dim3(bkd::kBlock), 0, st, payload,
                       payload_size, d_offsets, d_lengths, n, ledger_id, d_entry_ids, d_lacs, d_length_fields,
                       ds.tables[algo][lane_index(G)], d_digests, err, g_fold_sched.load());
}

// Package: header kernel (32 B BE header, header CRC as the payload's seed) -> payload CRCs through
// the direct kernel -> digest kernel (BE digest after the header; BKD_PACKAGE_DIGEST_PASS=0 has the
// payload groups store it instead) — or the fused route above, which folds the header inside the
// payload kernel. Out-of-range payload entries raise the stream's bounds flag.
int package_framed(DeviceState& ds, hipStream_t st, int algo, int64_t ledger_id, const int64_t* d_entry_ids,
                   const int64_t* d_lacs, const int64_t* d_length_fields, const void* d_payload,
                   uint64_t payload_size, const uint64_t* d_offsets, const uint32_t* d_lengths, uint64_t n,
                   void* d_frames, uint64_t frame_stride, uint32_t* d_digests) {
    const uint32_t mac = algo == BKD_CRC32C ? 4u : 8u;
    const int lanes = auto_lanes(payload_size / n, n, ds.cus);
    const uint32_t* tab = ds.tables[algo][lane_index(lanes)];
    uint32_t* err = nullptr;
    {
        StreamScratch& sc = scratch_for(ds, st);
        std::lock_guard<std::recursive_mutex> lk(sc.mu);
        const hipError_t e = sc.flag(st, &err);
        if (e != hipSuccess) return fail(BKD_ERR_NOMEM, std::string("bounds flag: ") + hipGetErrorString(e));
    }
    const unsigned blocks = (unsigned)((n + 255) / 256);
#ifndef BKD_PACKAGE_FUSED
#define BKD_PACKAGE_FUSED 1
#endif
    // The fused route when the frames are their own buffer (DigestManager's ByteBufList(header, data),
    // bench.py --config verify4k: 0.674 -> 0.659 ms per 1M 4 KiB entries); frames written in place in
    // front of their payloads keep the header-first route (0.821 vs 0.832 ms fused, profiles/r06r_*).
    const uint64_t fr0 = (uint64_t)(uintptr_t)d_frames, fr1 = fr0 + (n - 1u) * frame_stride + 32u + mac;
    const uint64_t pl0 = (uint64_t)(uintptr_t)d_payload, pl1 = pl0 + payload_size;
    const bool frames_apart = fr1 <= pl0 || pl1 <= fr0;
    if (BKD_PACKAGE_FUSED && lanes >= 4 && frames_apart) {
        const uint8_t* pl = (const uint8_t*)d_payload;
        switch (lanes) {
            case 4: launch_package_fused<4>(ds, st, algo, ledger_id, d_entry_ids, d_lacs, d_length_fields, pl, payload_size, d_offsets, d_lengths, n, d_digests, err); break;
            case 8: launch_package_fused<8>(ds, st, algo, ledger_id, d_entry_ids, d_lacs, d_length_fields, pl, payload_size, d_offsets, d_lengths, n, d_digests, err); break;
            case 16: launch_package_fused<16>(ds, st, algo, ledger_id, d_entry_ids, d_lacs, d_length_fields, pl, payload_size, d_offsets, d_lengths, n, d_digests, err); break;
            case 32: launch_package_fused<32>(ds, st, algo, ledger_id, d_entry_ids, d_lacs, d_length_fields, pl, payload_size, d_offsets, d_lengths, n, d_digests, err); break;
            default: launch_package_fused<64>(ds, st, algo, ledger_id, d_entry_ids, d_lacs, d_length_fields, pl, payload_size, d_offsets, d_lengths, n, d_digests, err); break;
        }
        BKD_HIP(hipGetLastError());
        hipLaunchKernelGGL(bkd::package_frame_kernel, dim3(blocks), dim3(256), 0, st, ledger_id, d_entry_ids, d_lacs,
                           d_length_fields, d_digests, n, (uint8_t*)d_frames, frame_stride, mac);
        BKD_HIP(hipGetLastError());
        return BKD_OK;
    }
    const unsigned hblocks = (unsigned)std::min<uint64_t>((n + 1023) / 1024, 2u * (uint64_t)ds.cus);
    hipLaunchKernelGGL(bkd::package_header_kernel, dim3(hblocks), dim3(1024), 0, st, tab + 1024, ledger_id, d_entry_ids,
                       d_lacs, d_length_fields, n, (uint8_t*)d_frames, frame_stride, d_digests);
    BKD_HIP(hipGetLastError());
#if BKD_PACKAGE_DIGEST_PASS
    bkd::IndexedSrc src{n, d_offsets, d_lengths, d_digests, 0u, payload_size, d_digests};
    int rc = dispatch_lanes(ds, lanes, algo, (const uint8_t*)d_payload, src, n, st, err);
    if (rc) return rc;
    hipLaunchKernelGGL(bkd::package_digest_kernel, dim3(blocks), dim3(256), 0, st, d_digests, n,
                       (uint8_t*)d_frames, frame_stride, mac);
    BKD_HIP(hipGetLastError());
    return BKD_OK;
#else
    // the payload groups write each frame's digest field themselves (PackageSrc)
    (void)blocks;
    bkd::PackageSrc src{{n, d_offsets, d_lengths, d_digests, 0u, payload_size, d_digests}, (uint8_t*)d_frames,
                        frame_stride, mac};
    return dispatch_lanes(ds, lanes, algo, (const uint8_t*)d_payload, src, n, st, err);
#endif
}

// Fused verify of near-uniform frames: one kernel per lane count (crc_verify_fused_kernel).
template <int G>
void launch_verify_fused(DeviceState& ds, hipStream_t st, int algo, const uint8_t* framed, uint64_t size,
                         const uint64_t* offsets, const uint32_t* lengths, uint64_t n, uint32_t mac, int64_t ledger_id,
                         int64_t first_entry_id, int id_checks, int32_t* status, uint64_t* first_bad,
                         const uint32_t* vflag, uint32_t vepoch) {
    const uint64_t per_block = bkd::kBlock / G;
    const unsigned blocks = (unsigned)std::min<uint64_t>((n + per_block - 1) / per_block, (uint64_t)ds.cus);
    hipLaunchKernelGGL((bkd::crc_verify_fused_kernel<G, kPF, kNT>), dim3(blocks), dim3(bkd::kBlock), 0, st, framed, size,
                       offsets, lengths, n, mac, ledger_id, first_entry_id, id_checks, ds.tables[algo][lane_index(G)],
                       status, (unsigned long long*)first_bad, vflag, vepoch, g_fold_sched.load());
}

// Verify (bkd_digest_verify_batch and bkd_entrylog_verify): header CRCs -> payload CRCs seeded
// with them through the indexed path (chunked plan for large ragged batches) -> compare. Batches
// that take the plan route first run a gate over the frame lengths: when every frame is within
// PlanRun::in_band of the first, the fused kernel verifies each frame whole (header, payload and
// compare in one pass over it) and the header / plan / finish kernels return at once; otherwise
// the fused kernel returns and they run. Both give the same statuses; the device decides, no sync.
int verify_framed(DeviceState& ds, hipStream_t st, int algo, int64_t ledger_id, int64_t first_entry_id,
                  int id_checks, const void* d_framed, uint64_t framed_size, const uint64_t* d_offsets,
                  const uint32_t* d_lengths, uint64_t n, int32_t* d_status, uint64_t* d_first_bad) {
    const uint32_t mac = algo == BKD_CRC32C ? 4u : 8u;
    if (n == 0) {
        BKD_HIP(hipMemsetAsync(d_first_bad, 0, sizeof(uint64_t), st));
        return BKD_OK;
    }
    const uint32_t* x32tab = ds.tables[algo][lane_index(4)] + 1024;  // x^32 operator, 4 x 256
    const unsigned blocks = (unsigned)((n + 255) / 256);
    Carver cv;
    const size_t o_seeds = cv.take(n * 4), o_plen = cv.take(n * 4), o_poff = cv.take(n * 8), o_exp = cv.take(n * 4),
                 o_pre = cv.take(n * 4);
    StreamScratch& sc = scratch_for(ds, st);
    std::lock_guard<std::recursive_mutex> lk(sc.mu);  // held across the nested plan (slot 0)
    uint8_t* sb = nullptr;
    hipError_t e = sc.get(1, cv.used, st, &sb);
    if (e != hipSuccess) return fail(BKD_ERR_NOMEM, std::string("verify scratch: ") + hipGetErrorString(e));
    uint32_t* seeds = Carver::at<uint32_t>(sb, o_seeds);
    uint32_t* plen = Carver::at<uint32_t>(sb, o_plen);
    uint64_t* poff = Carver::at<uint64_t>(sb, o_poff);
    uint32_t* expect = Carver::at<uint32_t>(sb, o_exp);
    uint32_t* pre = Carver::at<uint32_t>(sb, o_pre);
    // the fused route where the payloads would take the plan (large batches; the direct kernel's small
    // ones keep the three-kernel sequence)
    // — and, as the plan's own near-uniform gate, only where one frame per group uses the plan's lane
    // count: a few huge frames need the plan's chunks to fill the chip
    // the payloads' route, decided once for the whole call (a second read of the plan mode
    // could send them to the direct kernel, which ignores the gate, after the fused kernel ran)
    const int route = indexed_direct(framed_size) ? 0 : 1;
    const int fused_lanes = auto_lanes(framed_size / n, n, ds.cus);
    const bool fused = BKD_VERIFY_FUSED && route == 1 && fused_lanes == g_plan_lanes.load();
    uint32_t* vflag = nullptr;
    uint32_t vepoch = 0;
    if (fused) {
        e = sc.vflag_word(st, &vflag);
        if (e != hipSuccess) return fail(BKD_ERR_NOMEM, std::string("verify gate: ") + hipGetErrorString(e));
        if (++sc.vepoch == 0u) ++sc.vepoch;  // 0 is the word's initial value
        vepoch = sc.vepoch;
        const unsigned gblocks = (unsigned)std::min<uint64_t>((n + 1023) / 1024, (uint64_t)ds.cus);
        hipLaunchKernelGGL(bkd::verify_gate_kernel, dim3(gblocks), dim3(1024), 0, st, d_lengths, n, d_first_bad, vflag,
                           vepoch);
        const uint8_t* fb = (const uint8_t*)d_framed;
        switch (fused_lanes) {
            case 1:  // (a forced one-lane geometry: the fused kernel's narrowest group)
            case 4: launch_verify_fused<4>(ds, st, algo, fb, framed_size, d_offsets, d_lengths, n, mac, ledger_id,
                                           first_entry_id, id_checks, d_status, d_first_bad, vflag, vepoch); break;
            case 8: launch_verify_fused<8>(ds, st, algo, fb, framed_size, d_offsets, d_lengths, n, mac, ledger_id,
                                           first_entry_id, id_checks, d_status, d_first_bad, vflag, vepoch); break;
            case 16: launch_verify_fused<16>(ds, st, algo, fb, framed_size, d_offsets, d_lengths, n, mac, ledger_id,
                                             first_entry_id, id_checks, d_status, d_first_bad, vflag, vepoch); break;
            case 32: launch_verify_fused<32>(ds, st, algo, fb, framed_size, d_offsets, d_lengths, n, mac, ledger_id,
                                             first_entry_id, id_checks, d_status, d_first_bad, vflag, vepoch); break;
            default: launch_verify_fused<64>(ds, st, algo, fb, framed_size, d_offsets, d_lengths, n, mac, ledger_id,
                                             first_entry_id, id_checks, d_status, d_first_bad, vflag, vepoch); break;
        }
        e = hipGetLastError();
        if (e != hipSuccess) return fail(BKD_ERR_HIP, hipGetErrorString(e));
    }
    const unsigned hblocks = (unsigned)std::min<uint64_t>((n + 1023) / 1024, 2u * (uint64_t)ds.cus);
    hipLaunchKernelGGL(bkd::verify_header_kernel, dim3(hblocks), dim3(1024), 0, st, x32tab, (const uint8_t*)d_framed,
                       framed_size, d_offsets, d_lengths, n, mac, ledger_id, first_entry_id, id_checks, seeds, poff,
                       plen, expect, pre, d_first_bad, vflag, vepoch);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(BKD_ERR_HIP, hipGetErrorString(e));
    // payload CRCs land in d_status, then verify_finish turns them into status codes
    int rc = indexed_batch(ds, algo, (const uint8_t*)d_framed, framed_size, poff, plen, n, seeds, 0,
                           reinterpret_cast<uint32_t*>(d_status), st, vflag, vepoch, route);
    if (rc) return rc;
    hipLaunchKernelGGL(bkd::verify_finish_kernel, dim3(blocks), dim3(256), 0, st, expect, pre, n, d_status,
                       (unsigned long long*)d_first_bad, vflag, vepoch);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(BKD_ERR_HIP, hipGetErrorString(e));
    return BKD_OK;
}

// ---- host-resident framed batches (BatchedReadOp's ByteBufList, PendingAddOp's payloads) ----
// Entries are separate host buffers. Segments of <= kSeg bytes / kSegEntries entries are gathered
// back to back into the slot's pinned buffer on the copy pool, copied H2D on the slot's stream,
// run through the device sequence, and the per-entry results copied D2H; slot k % 2 alternates
// so one segment's gather and H2D overlap the other's kernels and D2H.
template <class Seg, class Drain>
int host_segments(HostStage& hs, const uint32_t* h_lengths, uint64_t n, uint64_t max_entries, Seg&& seg,
                  Drain&& drain_slot) {
    uint64_t pend_i0[2] = {0, 0}, pend_cnt[2] = {0, 0};
    bool busy[2] = {false, false};
    auto drain = [&](int s) -> int {
        if (!busy[s]) return BKD_OK;
        BKD_HIP(hipEventSynchronize(hs.done[s]));
        busy[s] = false;
        return drain_slot(s, pend_i0[s], pend_cnt[s]);
    };
    // every entry fits a segment, checked before any work is enqueued
    for (uint64_t i = 0; i < n; ++i)
        if (h_lengths[i] > HostStage::kSeg)
            return fail(BKD_ERR_INVALID_ARG, "host entry " + std::to_string(i) + " is larger than 64 MiB");
    int rc = BKD_OK;
    uint64_t i0 = 0;
    for (int k = 0; i0 < n && rc == BKD_OK; ++k) {
        const int s = k & 1;
        uint64_t i1 = i0, bytes = 0;
        while (i1 < n && i1 - i0 < max_entries && (i1 == i0 || bytes + h_lengths[i1] <= HostStage::kSeg))
            bytes += h_lengths[i1++];
        if ((rc = drain(s))) break;
        if ((rc = seg(s, i0, i1 - i0, bytes))) {
            (void)hipStreamSynchronize(hs.st[s]);  // copies of the failed segment may be queued
            break;
        }
        // every exit below goes through the final drains: no staging set returns to the pool with
        // copies or kernels of this call still queued on its streams
        const hipError_t e = hipEventRecord(hs.done[s], hs.st[s]);
        if (e != hipSuccess) {
            rc = fail(BKD_ERR_HIP, std::string("hipEventRecord: ") + hipGetErrorString(e));
            (void)hipStreamSynchronize(hs.st[s]);
            break;
        }
        busy[s] = true;
        pend_i0[s] = i0;
        pend_cnt[s] = i1 - i0;
        i0 = i1;
    }
    const int r0 = drain(0), r1 = drain(1);
    return rc ? rc : (r0 ? r0 : r1);
}

// ---- per-call resume (IntHash.resume) -------------------------------------------------------
// Host buffers up to this many bytes take the CPU route (host_crc.cpp); larger ones the GPU
// through pinned staging. Default from the per-call sweep (profiles/r02_call_latency.log): 4 MiB
// with the 128-bit fold (one core ~210 us vs ~230 us by gather + PCIe + launch for a pageable
// buffer), 64 MiB with the AVX-512 fold (one core then keeps pace with PCIe). UINT64_MAX = unset.
std::atomic<uint64_t> g_cpu_route_max{UINT64_MAX};

uint64_t cpu_route_max() {
    const uint64_t v = g_cpu_route_max.load(std::memory_order_relaxed);
    if (v != UINT64_MAX) return v;
    return bkd::host::has_wide_fold() ? (64ull << 20) : (4ull << 20);
}

// Per-call resumes longer than this run as consecutive pieces, each resuming from the last
// (entry lengths are 32-bit in the batch kernels).
constexpr uint64_t kResumePiece = 1ull << 31;

// Route of the host-resident batches (bkd_crc_batch_host, bkd_digest_*_batch_host): 0 automatic,
// 1 CPU (host_batch.cpp over the host pool), 2 GPU (pinned staging, PCIe, the device sequence).
std::atomic<int> g_host_route{0};

// The automatic choice, from the measured crossover (profiles/r03_host_route.log): a
// host-resident batch through the GPU is bound by PCIe (~51 GiB/s) and, for separate entry buffers,
// by the host gather into pinned staging; the CPU route scales with the cores until host memory
// bandwidth. EPYC 9575F, 1M framed 4 KiB entries: GPU route 46.6 GiB/s verify / 50.6 contiguous;
// CPU route 19.0 / 36.9 / 68.3 / 130 / 228 GiB/s verify at 1 / 2 / 4 / 8 / 16 threads (contiguous
// 30.9 / 61.6 / 106 / 172 / 244) -> the CPU route from 3 threads with the AVX-512 fold. Without it
// (128-bit fold, unmeasured on the box) from 4. BKD_HOST_ROUTE_MIN_THREADS overrides.
int cpu_route_min_threads() {
    static const int t = [] {
        if (const char* v = getenv("BKD_HOST_ROUTE_MIN_THREADS")) return std::max(1, atoi(v));
        return bkd::host::has_wide_fold() ? 3 : 4;
    }();
    return t;
}

// 1 = CPU, 2 = GPU, < 0 = error (a GPU route forced without a device).
// oversize: the batch holds an entry longer than a staging segment, which the framed GPU route
// refuses; the automatic route then takes the CPU (the provider never fails where it can compute).
int host_route(bool oversize = false) {
    const int r = g_host_route.load(std::memory_order_relaxed);
    if (r == 1 || (r == 0 && oversize)) return 1;
    if (visible_devices() <= 0)  // the provider never fails for lack of a device
        return r == 2 ? fail(BKD_ERR_NO_DEVICE, "no HIP device (host batch route forced to the GPU)") : 1;
    if (r == 2) return 2;
    return bkd::host::Pool::get().active() >= cpu_route_min_threads() ? 1 : 2;
}

bool any_longer(const uint32_t* lengths, uint64_t n, uint64_t limit) {
    for (uint64_t i = 0; i < n; ++i)
        if (lengths[i] > limit) return true;
    return false;
}

int cpu_resume(int algo, uint32_t current, const void* p, uint64_t len, uint32_t* out) {
    *out = ~bkd::host::fold(algo, ~current, (const uint8_t*)p, len);  // >= 4 MiB: over the host pool
    return BKD_OK;
}

// Device scratch of one synchronous per-call resume, pooled per device (no per-thread state
// that outlives its thread, no allocation on the hot path after the first calls).
struct CallScratch {
    uint64_t* d_off = nullptr;
    uint32_t* d_len = nullptr;
    uint32_t* h_out = nullptr;  // pinned: [0] result, [1] length for the plan path
};
struct CallPool {
    std::mutex mu;
    std::vector<CallScratch*> free;
};
CallPool g_call_pool[kMaxDevices];

int call_acquire(int dev, hipStream_t st, CallScratch** out) {
    CallPool& p = g_call_pool[dev];
    {
        std::lock_guard<std::mutex> lk(p.mu);
        if (!p.free.empty()) {
            *out = p.free.back();
            p.free.pop_back();
            return BKD_OK;
        }
    }
    std::unique_ptr<CallScratch> c(new CallScratch());
    BKD_HIP(hipMalloc((void**)&c->d_off, 8));
    BKD_HIP(hipMalloc((void**)&c->d_len, 4));
    BKD_HIP(hipHostMalloc((void**)&c->h_out, 8, hipHostMallocDefault));
    BKD_HIP(hipMemsetAsync(c->d_off, 0, 8, st));
    *out = c.release();
    return BKD_OK;
}

void call_release(int dev, CallScratch* c) {
    std::lock_guard<std::mutex> lk(g_call_pool[dev].mu);
    g_call_pool[dev].free.push_back(c);
}

int resume_device(int algo, uint32_t current, const void* ptr, uint64_t len, hipStream_t st, uint32_t* out) {
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    const int dev = (int)(ds - g_dev);
    CallScratch* c = nullptr;
    if ((rc = call_acquire(dev, st, &c))) return rc;
    const uint32_t l32 = (uint32_t)len;
    // the kernel stores the digest straight into the pinned host word (no D2H copy on the call's
    // critical path; visible to the host once the stream has synchronised)
    uint32_t* res = c->h_out;
    if (len < (1u << 20)) {  // one group: the entry as a uniform batch of one
        bkd::UniformSrc src{1, len, l32, nullptr, current, res};
        rc = dispatch_lanes(*ds, auto_lanes(len, 1, ds->cus), algo, (const uint8_t*)ptr, src, 1, st);
    } else {  // large: the chunked plan spreads it over the chip
        c->h_out[1] = l32;
        const hipError_t e = hipMemcpyAsync(c->d_len, c->h_out + 1, 4, hipMemcpyHostToDevice, st);
        rc = e == hipSuccess ? launch_plan(*ds, algo, (const uint8_t*)ptr, len, c->d_off, c->d_len, 1, nullptr,
                                           current, res, st, false, false)
                             : fail(BKD_ERR_HIP, hipGetErrorString(e));
    }
    if (!rc) {
        const hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = fail(BKD_ERR_HIP, std::string("resume: ") + hipGetErrorString(e));
        else *out = __atomic_load_n(c->h_out, __ATOMIC_ACQUIRE);
    }
    call_release(dev, c);
    return rc;
}

}  // namespace

extern "C" {

int bkd_abi_version(void) { return BKD_ABI_VERSION; }

int bkd_device_count(void) { return std::max(0, visible_devices()); }

int bkd_init(int device) {
    int count = bkd_device_count();
    if (count <= 0) return fail(BKD_ERR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= count || device >= kMaxDevices) return fail(BKD_ERR_INVALID_ARG, "bad device");
    std::lock_guard<std::mutex> lk(g_mu);
    return init_device_locked(device);
}

const char* bkd_last_error(void) { return t_err.c_str(); }

int bkd_set_fold_schedule(int schedule) {
    if (schedule < 0 || schedule > 2) return fail(BKD_ERR_INVALID_ARG, "fold schedule must be 0, 1 or 2");
    g_fold_sched.store(schedule);
    return BKD_OK;
}

int bkd_set_group_lanes(int lanes) {
    if (lanes != 0 && lane_index(lanes) < 0) return fail(BKD_ERR_INVALID_ARG, "lanes must be 0, 1, 4, 8, 16, 32 or 64");
    g_forced_lanes.store(lanes);
    return BKD_OK;
}

int bkd_set_plan_mode(int mode) {
    if (mode < 0 || mode > 2)
        return fail(BKD_ERR_INVALID_ARG, "plan mode must be 0 (auto), 1 (direct) or 2 (plan)");
    g_plan_mode.store(mode);
    return BKD_OK;
}

int bkd_set_plan_prefetch(int loads_in_flight) {
    if (loads_in_flight != 2 && loads_in_flight != 4 && loads_in_flight != 8)
        return fail(BKD_ERR_INVALID_ARG, "prefetch depth must be 2, 4 or 8");
    g_plan_pf.store(loads_in_flight);
    return BKD_OK;
}

int bkd_set_plan_geometry(int lanes, int steps_per_chunk, int merge_bytes) {
    if (lanes < 4 || lane_index(lanes) < 0) return fail(BKD_ERR_INVALID_ARG, "plan lanes must be 4, 8, 16, 32 or 64");
    if (steps_per_chunk < 1) return fail(BKD_ERR_INVALID_ARG, "steps_per_chunk must be >= 1");
    const uint32_t step = 16u * (uint32_t)lanes, ch = step * (uint32_t)steps_per_chunk;
    if (ch > 32768u) return fail(BKD_ERR_INVALID_ARG, "chunk size must be <= 32 KiB");
    if (merge_bytes < 16 || (uint32_t)merge_bytes > ch) return fail(BKD_ERR_INVALID_ARG, "merge must be in [16, chunk]");
    const uint32_t nbins = (ch + (uint32_t)merge_bytes - 1u + step - 1u) / step + 1u;
    if (nbins + 1u > (uint32_t)bkd::kMaxJC + 2u) return fail(BKD_ERR_INVALID_ARG, "too many step bins");
    g_plan_lanes.store(lanes);
    g_plan_jc.store(steps_per_chunk);
    g_plan_merge.store(merge_bytes);
    return BKD_OK;
}

int bkd_set_short_class_mean(uint64_t max_bytes_per_entry) {
    g_short_mean_max.store(max_bytes_per_entry);
    return BKD_OK;
}

int bkd_set_plan_small(uint32_t max_bytes) {
    if (max_bytes > kSmallMaxBytes || (max_bytes && max_bytes < 16u))
        return fail(BKD_ERR_INVALID_ARG, "short-entry class bound must be 0 or 16.." + std::to_string(kSmallMaxBytes));
    g_plan_small.store(max_bytes);
    return BKD_OK;
}

int bkd_set_plan_serial(uint32_t max_bytes) {
    if (max_bytes < 16u || max_bytes > bkd::kSerialMax)
        return fail(BKD_ERR_INVALID_ARG, "serial bound must be 16.." + std::to_string(bkd::kSerialMax));
    g_plan_serial.store(max_bytes);
    return BKD_OK;
}

int bkd_get_group_lanes(int algo, uint64_t mean_len) {
    (void)algo;
    return auto_lanes(mean_len);
}

int bkd_crc_batch_uniform(int algo, const void* d_base, uint64_t stride, uint32_t entry_len, uint64_t n,
                          const uint32_t* d_seeds, uint32_t seed_all, uint32_t* d_out, void* stream) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (n && (!d_base || !d_out)) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    if (n > 1 && stride < entry_len) return fail(BKD_ERR_INVALID_ARG, "stride < entry_len");
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    bkd::UniformSrc src{n, stride, entry_len, d_seeds, seed_all, d_out};
    // entries of 16..48 B: one lane per entry, both loads of an entry in flight with the next
    // entry's (uniform_small_loop): 2.2x the 4-lane rate at 32 B; from 64 B on 4 lanes win
    int lanes = auto_lanes(entry_len, n, ds->cus);
    if (g_forced_lanes.load() == 0 && entry_len >= 16u && entry_len <= 48u && n >= (uint64_t)ds->cus * bkd::kBlock)
        lanes = 1;
    // 256..511 B: 8 lanes (two to four 128-byte steps; the three-set short loop up to 384 B) beat 4
    // lanes since the short loop's waits are countable: 256 B 0.934 vs 1.028 ms, 512 B 0.826 vs
    // 0.915 ms per 4 GiB (profiles/r03v_size_sweep.log); indexed batches keep auto_lanes
    if (g_forced_lanes.load() == 0 && lanes == 4 && entry_len >= 256u && entry_len < 512u) lanes = 8;
    if (lanes == 8 && entry_len >= bkd::kTailUncondSteps * 16u * 8u)  // measured at 8 lanes only
        return dispatch_lanes(*ds, lanes, algo, (const uint8_t*)d_base, bkd::UniformLongSrc{src}, n, st);
    return dispatch_lanes(*ds, lanes, algo, (const uint8_t*)d_base, src, n, st);
}

int bkd_crc_batch(int algo, const void* d_base, uint64_t base_size, const uint64_t* d_offsets,
                  const uint32_t* d_lengths, uint64_t n, const uint32_t* d_seeds, uint32_t seed_all,
                  uint32_t* d_out, void* stream) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (n && (!d_offsets || !d_lengths || !d_out)) return fail(BKD_ERR_INVALID_ARG, "null index/out");
    if (n && !d_base && base_size) return fail(BKD_ERR_INVALID_ARG, "null base");
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    return indexed_batch(*ds, algo, (const uint8_t*)d_base, base_size, d_offsets, d_lengths, n, d_seeds, seed_all,
                         d_out, st);
}

int bkd_stream_sync(void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    StreamScratch* scp = scratch_find(*ds, st);  // (no entry for streams that only sync)
    if (!scp) {
        BKD_HIP(hipStreamSynchronize(st));
        return BKD_OK;
    }
    StreamScratch& sc = *scp;
    std::lock_guard<std::recursive_mutex> lk(sc.mu);
    if (!sc.err) {  // nothing indexed was ever enqueued on this stream
        BKD_HIP(hipStreamSynchronize(st));
        return BKD_OK;
    }
    // read and clear this stream's flag in stream order, after the work it guards
    BKD_HIP(hipMemcpyAsync(sc.h_err, sc.err, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    BKD_HIP(hipMemsetAsync(sc.err, 0, sizeof(uint32_t), st));
    BKD_HIP(hipStreamSynchronize(st));
    if (*sc.h_err) return fail(BKD_ERR_BOUNDS, "an indexed entry exceeded its base buffer (entries skipped, out = 0)");
    return BKD_OK;
}

int bkd_stream_release(void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    std::unique_ptr<StreamScratch> sc;
    {
        std::unique_lock<std::shared_mutex> wr(ds->maps_mu);
        auto it = ds->scratch.find(st);
        if (it == ds->scratch.end()) {
            BKD_HIP(hipStreamSynchronize(st));
            return BKD_OK;
        }
        sc = std::move(it->second);
        ds->scratch.erase(it);
    }
    int status = BKD_OK;
    {
        std::lock_guard<std::recursive_mutex> lk(sc->mu);
        BKD_HIP(hipStreamSynchronize(st));  // the stream's kernels are done with the scratch
        if (sc->err) {
            BKD_HIP(hipMemcpy(sc->h_err, sc->err, sizeof(uint32_t), hipMemcpyDeviceToHost));
            if (*sc->h_err) status = fail(BKD_ERR_BOUNDS, "an indexed entry exceeded its base buffer (entries skipped, out = 0)");
        }
        BKD_HIP(hipStreamSynchronize(st));  // the stream's own work is done with them
        for (int k = 0; k < 3; ++k)
            if (sc->buf[k]) BKD_HIP(hipFree(sc->buf[k]));
        for (uint32_t* w : {sc->err, sc->run, sc->uni, sc->vflag})
            if (w) BKD_HIP(hipFree(w));
        if (sc->h_err) BKD_HIP(hipHostFree(sc->h_err));
    }
    return status;
}

int bkd_crc_batch_host(int algo, const void* h_base, uint64_t base_size, const uint64_t* h_offsets,
                       const uint32_t* h_lengths, uint64_t n, const uint32_t* h_seeds, uint32_t seed_all,
                       uint32_t* h_out) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (n == 0) return BKD_OK;
    if (!h_offsets || !h_lengths || !h_out || (!h_base && base_size)) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    bool sorted = true;
    for (uint64_t i = 0; i < n; ++i) {
        if (h_offsets[i] > base_size || (uint64_t)h_lengths[i] > base_size - h_offsets[i])
            return fail(BKD_ERR_BOUNDS, "entry " + std::to_string(i) + " exceeds base buffer");
        if (i && h_offsets[i] < h_offsets[i - 1]) sorted = false;
    }
    const int route = host_route();
    if (route < 0) return route;
    if (route == 1) {
        bkd::host::crc_indexed(algo, (const uint8_t*)h_base, h_offsets, h_lengths, n, h_seeds, seed_all, h_out);
        return BKD_OK;
    }
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(nullptr, scope, &ds);
    if (rc) return rc;
    StageLease lease((int)(ds - g_dev));
    HostStage& hs = *lease;
    rc = hs.init();
    if (rc) return rc;
    if (!sorted) return host_batch_oneshot(*ds, hs, algo, (const uint8_t*)h_base, base_size, h_offsets, h_lengths, n,
                                           h_seeds, seed_all, h_out);
    uint64_t pieces = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (h_lengths[i] > HostStage::kSeg) pieces += (h_lengths[i] + HostStage::kSeg - 1) / HostStage::kSeg - 1;
    if (pieces == 0)
        return host_batch_pipelined(*ds, hs, algo, (const uint8_t*)h_base, h_offsets, h_lengths, n, h_seeds, seed_all,
                                    h_out);
    // Entries longer than a staging segment go through the pipeline as segment-sized pieces (the
    // first with the entry's seed, the others with seed ~0, i.e. their zero-initialised registers)
    // and are joined here, reg = reg * x^(8 len) ^ raw, as the device plan joins its chunks.
    const uint64_t m = n + pieces;
    std::vector<uint64_t> off2(m);
    std::vector<uint32_t> len2(m), seed2(m), out2(m);
    for (uint64_t i = 0, j = 0; i < n; ++i) {
        uint64_t o = h_offsets[i], left = h_lengths[i];
        seed2[j] = h_seeds ? h_seeds[i] : seed_all;
        do {
            const uint32_t l = (uint32_t)std::min<uint64_t>(left, HostStage::kSeg);
            off2[j] = o;
            len2[j] = l;
            if (o != h_offsets[i]) seed2[j] = 0xFFFFFFFFu;
            o += l;
            left -= l;
            ++j;
        } while (left);
    }
    // the pipeline walks offsets in order: an entry that starts inside a long entry's later pieces
    // (overlapping entries are legal, only bounds are checked) breaks that order, so such a
    // batch takes the one-copy route instead
    for (uint64_t j = 1; j < m; ++j)
        if (off2[j] < off2[j - 1])
            return host_batch_oneshot(*ds, hs, algo, (const uint8_t*)h_base, base_size, h_offsets, h_lengths, n,
                                      h_seeds, seed_all, h_out);
    rc = host_batch_pipelined(*ds, hs, algo, (const uint8_t*)h_base, off2.data(), len2.data(), m, seed2.data(), 0,
                              out2.data());
    if (rc) return rc;
    const uint32_t xseg = bkd::gf2::xpow(algo, 8ull * HostStage::kSeg);
    for (uint64_t i = 0, j = 0; i < n; ++i) {
        uint32_t reg = ~out2[j++];
        for (uint64_t at = HostStage::kSeg; at < h_lengths[i]; at += HostStage::kSeg, ++j)
            reg = bkd::gf2::mul(algo, reg, len2[j] == HostStage::kSeg ? xseg : bkd::gf2::xpow(algo, 8ull * len2[j])) ^
                  ~out2[j];
        h_out[i] = h_lengths[i] > HostStage::kSeg ? ~reg : out2[j - 1];
    }
    return BKD_OK;
}

int bkd_cpu_resume(int algo, uint32_t current, const void* h_ptr, uint64_t len, uint32_t* out) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (!out) return fail(BKD_ERR_INVALID_ARG, "null out");
    if (len && !h_ptr) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    return cpu_resume(algo, current, h_ptr, len, out);
}

int bkd_resume_host(int algo, uint32_t current, const void* h_ptr, uint64_t len, uint32_t* out) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (!out) return fail(BKD_ERR_INVALID_ARG, "null out");
    if (len == 0) {  // crc32c_sse42.cpp:211-213: resume of nothing returns the seed
        *out = current;
        return BKD_OK;
    }
    if (!h_ptr) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    if (len <= cpu_route_max() || visible_devices() <= 0)
        return cpu_resume(algo, current, h_ptr, len, out);
    // entries are indexed with 32-bit lengths: a longer buffer resumes piece by piece
    // (Sse42Crc32C.resume takes a long length, Sse42Crc32C.java:105-107)
    const uint8_t* p = (const uint8_t*)h_ptr;
    uint32_t r = current;
    for (uint64_t at = 0; at < len;) {
        const uint64_t off = 0;
        const uint32_t l32 = (uint32_t)std::min<uint64_t>(len - at, kResumePiece);
        const int rc = bkd_crc_batch_host(algo, p + at, l32, &off, &l32, 1, nullptr, r, &r);
        if (rc == BKD_ERR_HIP || rc == BKD_ERR_NOMEM || rc == BKD_ERR_NO_DEVICE)
            // a device that fails (init, allocation, a copy) degrades to the CPU route, never to an
            // error: the reference's provider chain never throws (Crc32cIntChecksum.java:28-36)
            return cpu_resume(algo, current, h_ptr, len, out);
        if (rc) return rc;
        at += l32;
    }
    *out = r;
    return BKD_OK;
}

int bkd_resume_device(int algo, uint32_t current, const void* d_ptr, uint64_t len, void* stream, uint32_t* out) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (!out) return fail(BKD_ERR_INVALID_ARG, "null out");
    if (len == 0) {
        *out = current;
        return BKD_OK;
    }
    if (!d_ptr) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    const uint8_t* p = (const uint8_t*)d_ptr;
    for (uint64_t at = 0; at < len;) {  // 32-bit entry lengths: longer buffers piece by piece
        const uint64_t l = std::min<uint64_t>(len - at, kResumePiece);
        const int rc = resume_device(algo, current, p + at, l, (hipStream_t)stream, &current);
        if (rc) return rc;
        at += l;
    }
    *out = current;
    return BKD_OK;
}

int bkd_resume(int algo, uint32_t current, const void* ptr, uint64_t len, uint32_t* out) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (!out) return fail(BKD_ERR_INVALID_ARG, "null out");
    if (len == 0) {
        *out = current;
        return BKD_OK;
    }
    if (!ptr) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    // a device buffer runs on the null stream, which orders the call after the work queued on
    // the blocking streams (PyTorch's default stream among them) that may still be writing it
    int pdev = -1;
    if (visible_devices() > 0 && is_device_pointer(ptr, &pdev)) {
        // on the null stream of the device that holds the buffer (not whichever is current)
        int cur = 0;
        BKD_HIP(hipGetDevice(&cur));
        DeviceScope scope;
        if (pdev >= 0 && pdev != cur) {
            BKD_HIP(hipSetDevice(pdev));
            scope.prev = cur;
        }
        return bkd_resume_device(algo, current, ptr, len, nullptr, out);
    }
    return bkd_resume_host(algo, current, ptr, len, out);
}

int bkd_circe_supported(void) { return 1; }

int64_t bkd_circe_alloc_config(const int32_t* chunk_words, int32_t len) {
    constexpr int32_t kMinWords = 4;  // chunk_config::min_words (crc32c_sse42.hpp:22)
    if (!chunk_words || len < 1 || chunk_words[0] < kMinWords) return 0;
    for (int32_t i = 1; i < len; ++i)
        if (chunk_words[i] < kMinWords || chunk_words[i] >= chunk_words[i - 1]) return 0;  // strictly decreasing
    int32_t* cfg = new (std::nothrow) int32_t[(size_t)len + 1];
    if (!cfg) return 0;
    cfg[0] = len;
    memcpy(cfg + 1, chunk_words, (size_t)len * sizeof(int32_t));
    return (int64_t)(intptr_t)cfg;
}

void bkd_circe_free_config(int64_t config) { delete[] (int32_t*)(intptr_t)config; }

int bkd_set_cpu_route_max(uint64_t bytes) {
    g_cpu_route_max.store(bytes);
    return BKD_OK;
}

uint64_t bkd_get_cpu_route_max(void) { return cpu_route_max(); }

const char* bkd_cpu_impl(void) { return bkd::host::impl_name(); }

int bkd_set_host_batch_route(int route) {
    if (route < 0 || route > 2) return fail(BKD_ERR_INVALID_ARG, "host batch route must be 0 (auto), 1 (CPU) or 2 (GPU)");
    g_host_route.store(route);
    return BKD_OK;
}

int bkd_get_host_batch_route(void) {
    const int r = host_route();
    return r < 0 ? 2 : r;
}

int bkd_set_host_threads(int threads) {
    if (threads < 0) return fail(BKD_ERR_INVALID_ARG, "threads must be >= 0");
    bkd::host::Pool::get().set_active(threads);
    return BKD_OK;
}

int bkd_get_host_threads(void) { return bkd::host::Pool::get().active(); }

int bkd_host_release(void) {
    for (int d = 0; d < kMaxDevices; ++d) {
        StagePool& pool = g_stages[d];
        std::vector<std::unique_ptr<HostStage>> gone;
        {
            std::lock_guard<std::mutex> lk(pool.mu);
            for (HostStage* hs : pool.idle) {
                auto it = std::find_if(pool.all.begin(), pool.all.end(),
                                       [&](const std::unique_ptr<HostStage>& p) { return p.get() == hs; });
                if (it != pool.all.end()) {
                    gone.push_back(std::move(*it));
                    pool.all.erase(it);
                }
            }
            pool.idle.clear();
        }
        if (!gone.empty()) {
            int prev = 0;
            if (hipGetDevice(&prev) == hipSuccess && hipSetDevice(d) == hipSuccess) {
                gone.clear();  // frees the pinned and device buffers, streams and events
                (void)hipSetDevice(prev);
            }
        }
        pool.cv.notify_all();  // callers waiting for a set may create one again
    }
    return BKD_OK;
}

int bkd_digest_package_batch(int algo, int64_t ledger_id, const int64_t* d_entry_ids, const int64_t* d_lacs,
                             const int64_t* d_length_fields, const void* d_payload, uint64_t payload_size,
                             const uint64_t* d_offsets, const uint32_t* d_lengths, uint64_t n, void* d_frames,
                             uint64_t frame_stride, uint32_t* d_digests, void* stream) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    const uint32_t mac = algo == BKD_CRC32C ? 4u : 8u;
    if (n == 0) return BKD_OK;
    if (!d_entry_ids || !d_lacs || !d_length_fields || !d_offsets || !d_lengths || !d_frames || !d_digests)
        return fail(BKD_ERR_INVALID_ARG, "null buffer");
    if (frame_stride < 32u + mac) return fail(BKD_ERR_INVALID_ARG, "frame_stride < 32 + digest length");
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    return package_framed(*ds, st, algo, ledger_id, d_entry_ids, d_lacs, d_length_fields, d_payload, payload_size,
                          d_offsets, d_lengths, n, d_frames, frame_stride, d_digests);
}

int bkd_digest_verify_batch(int algo, int64_t ledger_id, int64_t first_entry_id, int skip_entry_check,
                            const void* d_framed, uint64_t framed_size, const uint64_t* d_offsets,
                            const uint32_t* d_lengths, uint64_t n, int32_t* d_status, uint64_t* d_first_bad,
                            void* stream) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (!d_first_bad) return fail(BKD_ERR_INVALID_ARG, "null first_bad");
    if (n && (!d_offsets || !d_lengths || !d_status)) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    if (n && !d_framed) return fail(BKD_ERR_INVALID_ARG, "null framed buffer");
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    return verify_framed(*ds, st, algo, ledger_id, first_entry_id, skip_entry_check ? 1 : 0, d_framed, framed_size,
                         d_offsets, d_lengths, n, d_status, d_first_bad);
}

int bkd_digest_verify_batch_host(int algo, int64_t ledger_id, int64_t first_entry_id, int skip_entry_check,
                                 const void* const* h_frames, const uint32_t* h_lengths, uint64_t n,
                                 int32_t* h_status, uint64_t* h_first_bad) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (!h_first_bad) return fail(BKD_ERR_INVALID_ARG, "null first_bad");
    *h_first_bad = n;
    if (n == 0) return BKD_OK;
    if (!h_frames || !h_lengths || !h_status) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    for (uint64_t i = 0; i < n; ++i)
        if (h_lengths[i] && !h_frames[i]) return fail(BKD_ERR_INVALID_ARG, "null frame " + std::to_string(i));
    const int route = host_route(any_longer(h_lengths, n, HostStage::kSeg));
    if (route < 0) return route;
    if (route == 1) {
        *h_first_bad = bkd::host::verify_frames(algo, ledger_id, first_entry_id, skip_entry_check ? 1 : 0,
                                                (const uint8_t* const*)h_frames, h_lengths, n, h_status);
        return BKD_OK;
    }
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(nullptr, scope, &ds);
    if (rc) return rc;
    StageLease lease((int)(ds - g_dev));
    HostStage& hs = *lease;
    if ((rc = hs.init()) || (rc = hs.init_verify())) return rc;
    const int id_checks = skip_entry_check ? 1 : 0;
    auto seg = [&](int s, uint64_t i0, uint64_t cnt, uint64_t bytes) -> int {
        gather_entries(h_frames + i0, h_lengths + i0, cnt, hs.h_pin[s], hs.h_off[s]);
        const hipStream_t st = hs.st[s];
        BKD_HIP(hipMemcpyAsync(hs.d_buf[s], hs.h_pin[s], bytes, hipMemcpyHostToDevice, st));
        BKD_HIP(hipMemcpyAsync(hs.d_off[s], hs.h_off[s], cnt * 8, hipMemcpyHostToDevice, st));
        BKD_HIP(hipMemcpyAsync(hs.d_len[s], h_lengths + i0, cnt * 4, hipMemcpyHostToDevice, st));
        uint64_t* d_fb = hs.d_fb[s];
        int r = verify_framed(*ds, st, algo, ledger_id, first_entry_id + (int64_t)i0, id_checks, hs.d_buf[s], bytes,
                              hs.d_off[s], hs.d_len[s], cnt, reinterpret_cast<int32_t*>(hs.d_res[s]), d_fb);
        if (r) return r;
        BKD_HIP(hipMemcpyAsync(hs.h_res[s], hs.d_res[s], cnt * 4, hipMemcpyDeviceToHost, st));
        BKD_HIP(hipMemcpyAsync(hs.h_fb[s], d_fb, 8, hipMemcpyDeviceToHost, st));
        return BKD_OK;
    };
    auto drain = [&](int s, uint64_t i0, uint64_t cnt) -> int {
        memcpy(h_status + i0, hs.h_res[s], cnt * 4);
        const uint64_t fb = *hs.h_fb[s];
        if (fb < cnt && i0 + fb < *h_first_bad) *h_first_bad = i0 + fb;
        return BKD_OK;
    };
    return host_segments(hs, h_lengths, n, HostStage::kSegEntries, seg, drain);
}

int bkd_digest_package_batch_host(int algo, int64_t ledger_id, const int64_t* h_entry_ids, const int64_t* h_lacs,
                                  const int64_t* h_length_fields, const void* const* h_payloads,
                                  const uint32_t* h_lengths, uint64_t n, void* h_frames, uint64_t frame_stride,
                                  uint32_t* h_digests) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    const uint32_t mac = algo == BKD_CRC32C ? 4u : 8u;
    if (n == 0) return BKD_OK;
    if (!h_entry_ids || !h_lacs || !h_length_fields || !h_payloads || !h_lengths || !h_frames || !h_digests)
        return fail(BKD_ERR_INVALID_ARG, "null buffer");
    if (frame_stride < 32u + mac || frame_stride > 4096u)
        return fail(BKD_ERR_INVALID_ARG, "frame_stride must be in [32 + digest length, 4096]");
    for (uint64_t i = 0; i < n; ++i)
        if (h_lengths[i] && !h_payloads[i]) return fail(BKD_ERR_INVALID_ARG, "null payload " + std::to_string(i));
    const int route = host_route(any_longer(h_lengths, n, HostStage::kSeg));
    if (route < 0) return route;
    if (route == 1) {
        bkd::host::package_frames(algo, ledger_id, h_entry_ids, h_lacs, h_length_fields,
                                  (const uint8_t* const*)h_payloads, h_lengths, n, (uint8_t*)h_frames, frame_stride,
                                  h_digests);
        return BKD_OK;
    }
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(nullptr, scope, &ds);
    if (rc) return rc;
    StageLease lease((int)(ds - g_dev));
    HostStage& hs = *lease;
    if ((rc = hs.init()) || (rc = hs.init_package())) return rc;
    const uint64_t max_entries = std::min<uint64_t>(HostStage::kSegEntries, HostStage::kAux / frame_stride);
    auto seg = [&](int s, uint64_t i0, uint64_t cnt, uint64_t bytes) -> int {
        gather_entries(h_payloads + i0, h_lengths + i0, cnt, hs.h_pin[s], hs.h_off[s]);
        int64_t* aux = reinterpret_cast<int64_t*>(hs.h_aux[s]);
        memcpy(aux, h_entry_ids + i0, cnt * 8);
        memcpy(aux + cnt, h_lacs + i0, cnt * 8);
        memcpy(aux + 2 * cnt, h_length_fields + i0, cnt * 8);
        const hipStream_t st = hs.st[s];
        BKD_HIP(hipMemcpyAsync(hs.d_buf[s], hs.h_pin[s], bytes, hipMemcpyHostToDevice, st));
        BKD_HIP(hipMemcpyAsync(hs.d_off[s], hs.h_off[s], cnt * 8, hipMemcpyHostToDevice, st));
        BKD_HIP(hipMemcpyAsync(hs.d_len[s], h_lengths + i0, cnt * 4, hipMemcpyHostToDevice, st));
        BKD_HIP(hipMemcpyAsync(hs.d_aux[s], aux, cnt * 24, hipMemcpyHostToDevice, st));
        const int64_t* d_aux = reinterpret_cast<const int64_t*>(hs.d_aux[s]);
        int r = package_framed(*ds, st, algo, ledger_id, d_aux, d_aux + cnt, d_aux + 2 * cnt, hs.d_buf[s], bytes,
                               hs.d_off[s], hs.d_len[s], cnt, hs.d_frm[s], frame_stride, hs.d_res[s]);
        if (r) return r;
        BKD_HIP(hipMemcpyAsync(hs.h_frm[s], hs.d_frm[s], cnt * frame_stride, hipMemcpyDeviceToHost, st));
        BKD_HIP(hipMemcpyAsync(hs.h_res[s], hs.d_res[s], cnt * 4, hipMemcpyDeviceToHost, st));
        return BKD_OK;
    };
    auto drain = [&](int s, uint64_t i0, uint64_t cnt) -> int {
        memcpy((uint8_t*)h_frames + i0 * frame_stride, hs.h_frm[s], cnt * frame_stride);
        memcpy(h_digests + i0, hs.h_res[s], cnt * 4);
        return BKD_OK;
    };
    return host_segments(hs, h_lengths, n, max_entries, seg, drain);
}

int bkd_entrylog_verify(int algo, const void* d_log, uint64_t log_size, const uint64_t* d_offsets,
                        const uint32_t* d_lengths, uint64_t n, int32_t* d_status, uint64_t* d_first_bad,
                        void* stream) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (!d_first_bad) return fail(BKD_ERR_INVALID_ARG, "null first_bad");
    if (n && (!d_offsets || !d_lengths || !d_status)) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    if (n && !d_log) return fail(BKD_ERR_INVALID_ARG, "null log buffer");
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    return verify_framed(*ds, st, algo, 0, 0, 2, d_log, log_size, d_offsets, d_lengths, n, d_status, d_first_bad);
}

int bkd_crc_batch_segments(int algo, const void* d_base, uint64_t base_size, const uint64_t* d_seg_offsets,
                           const uint32_t* d_seg_lengths, uint64_t nseg, const uint64_t* d_seg_first, uint64_t n,
                           const uint32_t* d_seeds, uint32_t seed_all, uint32_t* d_out, void* stream) {
    if (!valid_algo(algo)) return fail(BKD_ERR_INVALID_ARG, "unknown algorithm");
    if (n == 0) return BKD_OK;
    if (!d_seg_first || !d_out || (nseg && (!d_seg_offsets || !d_seg_lengths)))
        return fail(BKD_ERR_INVALID_ARG, "null index/out");
    if (nseg && !d_base && base_size) return fail(BKD_ERR_INVALID_ARG, "null base");
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    StreamScratch& sc = scratch_for(*ds, st);
    std::lock_guard<std::recursive_mutex> lk(sc.mu);  // held across the nested plan (slot 0)
    uint8_t* seg = nullptr;
    hipError_t e = sc.get(2, (size_t)std::max<uint64_t>(nseg, 1) * 4, st, &seg);
    if (e != hipSuccess) return fail(BKD_ERR_NOMEM, std::string("segment scratch: ") + hipGetErrorString(e));
    uint32_t* segcrc = reinterpret_cast<uint32_t*>(seg);
    // every segment's raw register reg(0, segment), as ~resume(~0, segment)
    if (nseg) {
        rc = indexed_batch(*ds, algo, (const uint8_t*)d_base, base_size, d_seg_offsets, d_seg_lengths, nseg, nullptr,
                           0xFFFFFFFFu, segcrc, st);
        if (rc) return rc;
    }
    bkd::XPow8 pw;
    for (int b = 0; b < 32; ++b) pw.p[b] = bkd::gf2::xpow(algo, 8ull << b);
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(bkd::segments_combine_kernel, dim3(blocks), dim3(256), 0, st, d_seg_lengths, segcrc,
                       d_seg_first, n, nseg, d_seeds, seed_all, pw, bkd::gf2::poly(algo), d_out);
    BKD_HIP(hipGetLastError());
    return BKD_OK;
}

int bkd_entrylog_index(const void* h_log, uint64_t log_size, uint64_t start, uint64_t* h_offsets,
                       uint32_t* h_lengths, int64_t* h_ledger_ids, uint64_t capacity, uint64_t* h_count,
                       uint64_t* h_end) {
    if (!h_count || (log_size && !h_log) || (capacity && (!h_offsets || !h_lengths)))
        return fail(BKD_ERR_INVALID_ARG, "null buffer");
    const uint8_t* p = (const uint8_t*)h_log;
    auto be32 = [&](uint64_t at) {
        return (int32_t)(((uint32_t)p[at] << 24) | ((uint32_t)p[at + 1] << 16) | ((uint32_t)p[at + 2] << 8) |
                         (uint32_t)p[at + 3]);
    };
    auto be64 = [&](uint64_t at) {
        uint64_t v = 0;
        for (int k = 0; k < 8; ++k) v = (v << 8) | p[at + k];
        return (int64_t)v;
    };
    uint64_t pos = start, count = 0;
    int rc = BKD_OK;
    while (pos < log_size) {
        if (log_size - pos < 12) break;  // short read of [size, ledgerId]: the scan stops
        const int32_t entry_size = be32(pos);
        if (entry_size <= 0) {  // padding
            ++pos;
            continue;
        }
        const int64_t ledger_id = be64(pos + 4);
        pos += 4;
        if (ledger_id == -1) {  // INVALID_LID: ledgers-map record, not an entry
            pos += (uint64_t)entry_size;
            continue;
        }
        if ((uint64_t)entry_size > log_size - pos) break;  // short read of the entry: the scan stops
        if (count < capacity) {
            h_offsets[count] = pos;
            h_lengths[count] = (uint32_t)entry_size;
            if (h_ledger_ids) h_ledger_ids[count] = ledger_id;
        } else {
            rc = fail(BKD_ERR_BOUNDS, "entry-log index capacity exceeded");
            break;
        }
        ++count;
        pos += (uint64_t)entry_size;
    }
    *h_count = count;
    if (h_end) *h_end = pos;
    return rc;
}

int bkd_fill_splitmix64(void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t first_word, void* stream) {
    if (nbytes == 0) return BKD_OK;
    if (!d_dst) return fail(BKD_ERR_INVALID_ARG, "null buffer");
    const hipStream_t st = (hipStream_t)stream;
    DeviceScope scope;
    DeviceState* ds = nullptr;
    int rc = enter(st, scope, &ds);
    if (rc) return rc;
    const uint64_t nw = std::max<uint64_t>(1, nbytes / 8);
    const unsigned blocks = (unsigned)std::min<uint64_t>((nw + 255) / 256, (uint64_t)ds->cus * 16);
    hipLaunchKernelGGL(bkd::fill_splitmix64_kernel, dim3(blocks), dim3(256), 0, st,
                       (uint8_t*)d_dst, nbytes, seed, first_word);
    BKD_HIP(hipGetLastError());
    return BKD_OK;
}

int64_t bkd_host_tables(int algo, int lanes, uint32_t* out, uint64_t out_words) {
    if (!valid_algo(algo) || lane_index(lanes) < 0) return fail(BKD_ERR_INVALID_ARG, "bad algo/lanes");
    const int64_t need = bkd::gf2::compact_words(lanes);
    if (!out || out_words < (uint64_t)need) return fail(BKD_ERR_INVALID_ARG, "output too small");
    return bkd::gf2::build_compact(algo, lanes, out);
}

uint32_t bkd_host_gf_mul(int algo, uint32_t a, uint32_t b) { return bkd::gf2::mul(algo, a, b); }

uint32_t bkd_host_xpow8n(int algo, uint64_t nbytes) { return bkd::gf2::xpow(algo, nbytes * 8); }

}  // extern "C"
