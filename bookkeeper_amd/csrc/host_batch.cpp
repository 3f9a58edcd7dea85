// Host worker pool and the CPU route of host-resident batches (host_batch.hpp). Clean-room: the
// arithmetic is host_crc.cpp's folding; the framing follows DigestManager (cited per function).
#include "host_batch.hpp"

#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>

#include "crc_tables.hpp"
#include "host_crc.hpp"

namespace bkd {
namespace host {

int usable_cores() {
    static const int n = [] {
        int cores = (int)std::max(1u, std::thread::hardware_concurrency());
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) cores = std::max(1, CPU_COUNT(&set));
        if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[64] = {0};
            long long period = 0;
            if (fscanf(f, "%63s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
                const long long quota = atoll(q);
                const int cap = (int)std::max(1LL, (quota + period - 1) / period);
                cores = std::min(cores, cap);
            }
            fclose(f);
        }
        return cores;
    }();
    return n;
}

Pool& Pool::get() {
    static Pool pool;
    return pool;
}

Pool::Pool() {
    int want = usable_cores();
    if (const char* v = getenv("BKD_HOST_THREADS")) want = std::max(1, std::min(256, atoi(v)));
    active_ = want;
    for (int w = 1; w < want; ++w) workers_.emplace_back([this, w] { loop(w); });
}

Pool::~Pool() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
}

int Pool::threads() const { return (int)workers_.size() + 1; }

int Pool::active() const { return std::max(1, std::min(active_.load(std::memory_order_relaxed), threads())); }

void Pool::set_active(int n) { active_ = n <= 0 ? threads() : std::min(n, threads()); }

void Pool::run(int parts, const std::function<void(int)>& f) {
    parts = std::max(1, std::min(parts, active()));
    std::unique_lock<std::mutex> call(call_mu_, std::try_to_lock);
    if (parts == 1 || !call.owns_lock()) {  // one part, or another caller holds the workers
        for (int p = 0; p < parts; ++p) f(p);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(mu_);
        job_ = &f;
        parts_ = parts;
        pending_ = parts - 1;
        ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
}

void Pool::loop(int part) {
    uint64_t seen = 0;
    for (;;) {
        const std::function<void(int)>* f = nullptr;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            if (part >= parts_) continue;
            f = job_;
        }
        (*f)(part);
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_.notify_all();
    }
}

namespace {

// Batches below this many payload bytes run on the calling thread (waking the pool costs more).
constexpr uint64_t kInlineBytes = 512u << 10;

// Runs body(i0, i1) over [0, n) in chunks taken from a shared counter, so ragged entry sizes
// balance without a serial prefix sum. Batches of fewer than 4096 entries and under kInlineBytes
// run inline.
template <class Body>
void for_chunks(uint64_t n, const uint32_t* lens, Body&& body) {
    if (n == 0) return;
    Pool& pool = Pool::get();
    const int threads = pool.active();
    bool inline_run = threads == 1;
    if (!inline_run && n < 4096) {  // small batches: sum their bytes to decide
        uint64_t bytes = 0;
        for (uint64_t i = 0; i < n; ++i) bytes += lens[i];
        inline_run = bytes < kInlineBytes;
    }
    if (inline_run) return body((uint64_t)0, n);
    const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(4096, n / ((uint64_t)threads * 16)));
    const uint64_t nchunks = (n + chunk - 1) / chunk;
    std::atomic<uint64_t> next{0};
    pool.run((int)std::min<uint64_t>((uint64_t)threads, nchunks), [&](int) {
        for (;;) {
            const uint64_t c = next.fetch_add(1, std::memory_order_relaxed);
            if (c >= nchunks) return;
            const uint64_t i0 = c * chunk;
            body(i0, std::min(n, i0 + chunk));
        }
    });
}

// Entries of at least kSplitBytes are folded in kPieceBytes pieces on the whole pool, each piece's
// register from zero, joined by Horner with x^(8 * piece) (the device plan's join,
// plan_kernels.hpp): a long entry is not left to one core while the others idle.
constexpr uint64_t kPieceBytes = 1u << 20;
constexpr uint64_t kSplitBytes = 4u << 20;

inline bool split_on() { return Pool::get().active() > 1; }

inline bool is_big(uint64_t len) { return len >= kSplitBytes; }

inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

inline void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

inline void put_be64(uint8_t* p, uint64_t v) {
    put_be32(p, (uint32_t)(v >> 32));
    put_be32(p + 4, (uint32_t)v);
}

}  // namespace

uint32_t fold(int algo, uint32_t reg, const uint8_t* p, uint64_t len) {
    Pool& pool = Pool::get();
    const int threads = pool.active();
    if (threads == 1 || !is_big(len)) return crc_raw(algo, reg, p, (size_t)len);
    const uint64_t np = (len + kPieceBytes - 1) / kPieceBytes;
    std::vector<uint32_t> raw(np);
    std::atomic<uint64_t> next{0};
    pool.run((int)std::min<uint64_t>((uint64_t)threads, np), [&](int) {
        for (;;) {
            const uint64_t k = next.fetch_add(1, std::memory_order_relaxed);
            if (k >= np) return;
            const uint64_t at = k * kPieceBytes;
            raw[k] = crc_raw(algo, k == 0 ? reg : 0u, p + at, (size_t)std::min(kPieceBytes, len - at));
        }
    });
    const uint32_t xp = gf2::xpow(algo, 8ull * kPieceBytes);
    uint32_t r = raw[0];
    for (uint64_t k = 1; k < np; ++k) {
        const uint64_t l = std::min(kPieceBytes, len - k * kPieceBytes);
        r = gf2::mul(algo, r, l == kPieceBytes ? xp : gf2::xpow(algo, 8ull * l)) ^ raw[k];
    }
    return r;
}

void crc_list(int algo, const uint8_t* const* ptrs, const uint32_t* lens, uint64_t n, const uint32_t* seeds,
              uint32_t seed_all, uint32_t* out) {
    const bool split = split_on();
    std::atomic<bool> big{false};
    for_chunks(n, lens, [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; ++i) {
            if (split && is_big(lens[i])) {
                big.store(true, std::memory_order_relaxed);
                continue;
            }
            const uint32_t seed = seeds ? seeds[i] : seed_all;
            out[i] = lens[i] ? ~crc_raw(algo, ~seed, ptrs[i], lens[i]) : seed;
        }
    });
    if (big.load())
        for (uint64_t i = 0; i < n; ++i)
            if (is_big(lens[i])) out[i] = ~fold(algo, ~(seeds ? seeds[i] : seed_all), ptrs[i], lens[i]);
}

void crc_indexed(int algo, const uint8_t* base, const uint64_t* offsets, const uint32_t* lens, uint64_t n,
                 const uint32_t* seeds, uint32_t seed_all, uint32_t* out) {
    const bool split = split_on();
    std::atomic<bool> big{false};
    for_chunks(n, lens, [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; ++i) {
            if (split && is_big(lens[i])) {
                big.store(true, std::memory_order_relaxed);
                continue;
            }
            const uint32_t seed = seeds ? seeds[i] : seed_all;
            out[i] = lens[i] ? ~crc_raw(algo, ~seed, base + offsets[i], lens[i]) : seed;
        }
    });
    if (big.load())
        for (uint64_t i = 0; i < n; ++i)
            if (is_big(lens[i])) out[i] = ~fold(algo, ~(seeds ? seeds[i] : seed_all), base + offsets[i], lens[i]);
}

// DigestManager.verifyDigest ($BK/proto/checksum/DigestManager.java:226-283), in its order: too
// short (:229-235), digest = update(update(0, [0, 32)), [32 + mac, len)) against getInt(32) /
// getLong(32) (:236-261), ledger id (:267-273), entry id (:275-281).
uint64_t verify_frames(int algo, int64_t ledger_id, int64_t first_entry_id, int id_checks,
                       const uint8_t* const* frames, const uint32_t* lens, uint64_t n, int32_t* status) {
    const uint32_t mac = algo == 0 ? 4u : 8u;
    const bool split = split_on();
    std::atomic<bool> big{false};
    auto one = [&](uint64_t i, bool whole_pool) -> int32_t {
        const uint32_t l = lens[i];
        if (l < 32u + mac) return 1;
        const uint8_t* f = frames[i];
        uint32_t reg = crc_raw(algo, 0xFFFFFFFFu, f, 32);  // update(0, header)
        reg = whole_pool ? fold(algo, reg, f + 32 + mac, l - 32u - mac) : crc_raw(algo, reg, f + 32 + mac, l - 32u - mac);
        const uint32_t computed = ~reg;
        const uint32_t hi = mac == 8u ? be32(f + 32) : 0u;
        const uint32_t expect = be32(f + 32 + (mac - 4u));
        const int64_t lid = (int64_t)(((uint64_t)be32(f) << 32) | be32(f + 4));
        const int64_t eid = (int64_t)(((uint64_t)be32(f + 8) << 32) | be32(f + 12));
        if (hi != 0u || computed != expect) return 2;
        if (id_checks < 2 && lid != ledger_id) return 3;
        if (id_checks == 0 && eid != first_entry_id + (int64_t)i) return 4;
        return 0;
    };
    std::atomic<uint64_t> first_bad{n};
    auto note_bad = [&](uint64_t bad) {
        uint64_t cur = first_bad.load(std::memory_order_relaxed);
        while (bad < cur && !first_bad.compare_exchange_weak(cur, bad, std::memory_order_relaxed)) {
        }
    };
    for_chunks(n, lens, [&](uint64_t i0, uint64_t i1) {
        uint64_t bad = n;
        for (uint64_t i = i0; i < i1; ++i) {
            if (split && is_big(lens[i])) {
                big.store(true, std::memory_order_relaxed);
                continue;
            }
            const int32_t st = one(i, false);
            status[i] = st;
            if (st != 0 && i < bad) bad = i;
        }
        note_bad(bad);
    });
    if (big.load())
        for (uint64_t i = 0; i < n; ++i)
            if (is_big(lens[i])) {
                status[i] = one(i, true);
                if (status[i] != 0) note_bad(i);
            }
    return first_bad.load();
}

// DigestManager.computeDigestAndPackageForSending (:117-181): header [ledgerId, entryId, LAC, length]
// BE (:146-149), digest = update(update(0, header), payload) (:152-153), written after the header
// (CRC32CDigestManager.java:44-46 writeInt; CRC32DigestManager.java:60-63 writeLong, zero-extended).
void package_frames(int algo, int64_t ledger_id, const int64_t* entry_ids, const int64_t* lacs,
                    const int64_t* length_fields, const uint8_t* const* payloads, const uint32_t* lens, uint64_t n,
                    uint8_t* frames, uint64_t stride, uint32_t* digests) {
    const uint32_t mac = algo == 0 ? 4u : 8u;
    const bool split = split_on();
    std::atomic<bool> big{false};
    auto one = [&](uint64_t i, bool whole_pool) {
        uint8_t* f = frames + i * stride;
        put_be64(f, (uint64_t)ledger_id);
        put_be64(f + 8, (uint64_t)entry_ids[i]);
        put_be64(f + 16, (uint64_t)lacs[i]);
        put_be64(f + 24, (uint64_t)length_fields[i]);
        uint32_t reg = crc_raw(algo, 0xFFFFFFFFu, f, 32);
        if (lens[i]) reg = whole_pool ? fold(algo, reg, payloads[i], lens[i]) : crc_raw(algo, reg, payloads[i], lens[i]);
        const uint32_t d = ~reg;
        if (mac == 8u) put_be32(f + 32, 0u);
        put_be32(f + 32 + (mac - 4u), d);
        digests[i] = d;
    };
    for_chunks(n, lens, [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; ++i) {
            if (split && is_big(lens[i])) {
                big.store(true, std::memory_order_relaxed);
                continue;
            }
            one(i, false);
        }
    });
    if (big.load())
        for (uint64_t i = 0; i < n; ++i)
            if (is_big(lens[i])) one(i, true);
}

}  // namespace host
}  // namespace bkd
