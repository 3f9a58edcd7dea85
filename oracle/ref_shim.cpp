// TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.
//
// C-ABI shim over the reference's own native CRC32C (circe-checksum), compiled by
// oracle/Makefile straight from the sources under /root/reference into oracle/_ref/
// (git-ignored). No reference source is copied into this repository.
//
// What it wraps:
//   uint32_t crc32c(uint32_t init, const void*, size_t, const chunk_config*)
//       circe-checksum/src/main/circe/include/crc32c_sse42.hpp:40, cpp/crc32c_sse42.cpp:184-217
//   chunk_config(words, next)   crc32c_sse42.hpp:20-38 with the default ladder {4096, 512, 64}
//       words used by Crc32cSse42Provider.java:33 (DEFAULT_CHUNK)
//   crc32c_initialize()         crc32c_sse42.cpp:48-70 (the JNI nativeSupported() probe)
//
// Used (a) to pin the oracle restatement and generate tests/golden fixtures, and
// (b) as bench.py's cpu_baseline (kind "reference"): one crc32c() call per entry, the
// way JniIntHash -> Sse42Crc32C.nativeUnsafe drives it (JniIntHash.java:45-47).
#include <stdint.h>
#include <stddef.h>
#include <chrono>
#include <thread>
#include <vector>

#include "crc32c_sse42.hpp"

namespace {
const chunk_config& default_config() {
    static const chunk_config c3(64);
    static const chunk_config c2(512, &c3);
    static const chunk_config c1(4096, &c2);
    return c1;
}
}  // namespace

extern "C" {

int ref_supported(void) { return crc32c_initialize() ? 1 : 0; }

uint32_t ref_crc32c(uint32_t init, const void* buf, uint64_t len) {
    crc32c_initialize();
    return crc32c(init, buf, (size_t)len, &default_config());
}

uint32_t ref_crc32c_unchunked(uint32_t init, const void* buf, uint64_t len) {
    crc32c_initialize();
    return crc32c(init, buf, (size_t)len, nullptr);
}

void ref_crc32c_batch(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths, uint64_t n,
                      const uint32_t* seeds, uint32_t seed_all, uint32_t* out) {
    crc32c_initialize();
    const chunk_config* cfg = &default_config();
    for (uint64_t i = 0; i < n; ++i)
        out[i] = crc32c(seeds ? seeds[i] : seed_all, base + offsets[i], lengths[i], cfg);
}

// Times `reps` passes of one crc32c() call per uniform entry, over `threads` std::threads
// (entries split into contiguous ranges). Returns wall seconds for all passes.
double ref_crc32c_uniform_timed(const uint8_t* base, uint64_t stride, uint32_t len, uint64_t n, int threads,
                                int reps, uint32_t* out) {
    crc32c_initialize();
    const chunk_config* cfg = &default_config();
    if (threads < 1) threads = 1;
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) {
            uint64_t lo = n * t / threads, hi = n * (t + 1) / threads;
            pool.emplace_back([=]() {
                for (uint64_t i = lo; i < hi; ++i) out[i] = crc32c(0, base + i * stride, len, cfg);
            });
        }
        for (auto& th : pool) th.join();
    }
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// Times `reps` passes of one crc32c() call per indexed entry (an offset+length batch, e.g. the
// Zipf config), entries split into contiguous ranges of about equal bytes over `threads`.
double ref_crc32c_batch_timed(const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths, uint64_t n,
                              int threads, int reps, uint32_t* out) {
    crc32c_initialize();
    const chunk_config* cfg = &default_config();
    if (threads < 1) threads = 1;
    std::vector<uint64_t> cut(threads + 1, n);
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += lengths[i];
    cut[0] = 0;
    uint64_t acc = 0;
    int t = 1;
    for (uint64_t i = 0; i < n && t < threads; ++i) {
        acc += lengths[i];
        while (t < threads && acc * threads >= total * t) cut[t++] = i + 1;
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
        std::vector<std::thread> pool;
        for (int k = 0; k < threads; ++k) {
            const uint64_t lo = cut[k], hi = cut[k + 1];
            pool.emplace_back([=]() {
                for (uint64_t i = lo; i < hi; ++i) out[i] = crc32c(0, base + offsets[i], lengths[i], cfg);
            });
        }
        for (auto& th : pool) th.join();
    }
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// BatchedReadOp's verify loop over a ByteBufList in host memory ($BK/client/BatchedReadOp.java:164-190),
// CRC32C: per frame DigestManager.verifyDigest's two updates through circe (update(0, [0, 32)) then
// update(digest, [36, len)), DigestManager.java:236-239) and the compare with getInt(32) (:241-249),
// then the ledger / entry id checks (:264-281). Frames split into ranges of about equal bytes over
// `threads` std::threads; `reps` passes. status[i] as bkd_digest_verify_batch_host (0 ok, 1 too
// short, 2 digest, 3 ledger id, 4 entry id). Returns wall seconds for all passes.
double ref_verify_frames_timed(const uint8_t* const* frames, const uint32_t* lengths, uint64_t n, int64_t ledger_id,
                               int64_t first_entry_id, int threads, int reps, int32_t* status) {
    crc32c_initialize();
    const chunk_config* cfg = &default_config();
    if (threads < 1) threads = 1;
    std::vector<uint64_t> cut(threads + 1, n);
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += lengths[i];
    cut[0] = 0;
    uint64_t acc = 0;
    int t = 1;
    for (uint64_t i = 0; i < n && t < threads; ++i) {
        acc += lengths[i];
        while (t < threads && acc * threads >= total * t) cut[t++] = i + 1;
    }
    auto be = [](const uint8_t* p, int k) {
        uint64_t v = 0;
        for (int b = 0; b < k; ++b) v = (v << 8) | p[b];
        return v;
    };
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
        std::vector<std::thread> pool;
        for (int k = 0; k < threads; ++k) {
            const uint64_t lo = cut[k], hi = cut[k + 1];
            pool.emplace_back([=]() {
                for (uint64_t i = lo; i < hi; ++i) {
                    const uint8_t* f = frames[i];
                    const uint32_t l = lengths[i];
                    if (l < 36u) {
                        status[i] = 1;
                        continue;
                    }
                    uint32_t d = crc32c(0, f, 32, cfg);
                    d = crc32c(d, f + 36, l - 36u, cfg);
                    if (d != (uint32_t)be(f + 32, 4)) status[i] = 2;
                    else if ((int64_t)be(f, 8) != ledger_id) status[i] = 3;
                    else if ((int64_t)be(f + 8, 8) != first_entry_id + (int64_t)i) status[i] = 4;
                    else status[i] = 0;
                }
            });
        }
        for (auto& th : pool) th.join();
    }
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
