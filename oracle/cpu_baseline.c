/*
 * TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT (bench.py's cpu_baseline leg only).
 *
 * CPU baseline for the CRC-32 digest path: BookKeeper computes it with java.util.zip.CRC32
 * (CRC32DigestManager.java:28-87 via DirectMemoryCRC32Digest / StandardCRC32Digest), whose
 * arithmetic is zlib's crc32() (the JDK links zlib). This times zlib's crc32() once per entry over
 * an offset+length batch on `threads` pthreads, entries split into ranges of about equal bytes —
 * the CRC-32 counterpart of oracle/ref_shim.cpp's ref_crc32c_batch_timed.
 */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>
#include <zlib.h>

typedef struct {
    const uint8_t* base;
    const uint64_t* offs;
    const uint32_t* lens;
    uint64_t lo, hi;
    uint32_t* out;
} zjob;

static void* zrun(void* p) {
    zjob* j = (zjob*)p;
    for (uint64_t i = j->lo; i < j->hi; ++i)
        j->out[i] = (uint32_t)crc32(0L, j->base + j->offs[i], (uInt)j->lens[i]);
    return NULL;
}

double oracle_zlib_crc32_batch_timed(const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint64_t n,
                                     int threads, int reps, uint32_t* out) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    uint64_t cut[257];
    uint64_t total = 0, acc = 0;
    for (uint64_t i = 0; i < n; ++i) total += lens[i];
    cut[0] = 0;
    for (int t = 1; t <= threads; ++t) cut[t] = n;
    int t = 1;
    for (uint64_t i = 0; i < n && t < threads; ++i) {
        acc += lens[i];
        while (t < threads && acc * (uint64_t)threads >= total * (uint64_t)t) cut[t++] = i + 1;
    }
    pthread_t th[256];
    zjob jobs[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; ++r) {
        for (int k = 0; k < threads; ++k) {
            jobs[k] = (zjob){base, offs, lens, cut[k], cut[k + 1], out};
            pthread_create(&th[k], NULL, zrun, &jobs[k]);
        }
        for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/*
 * CPU baseline for CRC-32 closer to what the JVM runs: java.util.zip.CRC32's HotSpot intrinsic on
 * x86-64 folds 128-bit blocks with PCLMULQDQ (four accumulators, 64-byte stride) instead of zlib's
 * table loop. Restated here with the same folding arithmetic — four accumulators of 16 bytes move
 * 512 bits forward as clmul(lo, x^(63+512)) ^ clmul(hi, x^(512-1)) mod P (reflected operands), are
 * merged, and the 16-byte remainder and the tail bytes are finished by zlib's crc32(). Used only for
 * the timed baseline; its digests are checked against the GPU's in bench.py.
 */
#include <immintrin.h>
#include <string.h>

static uint32_t xpow_bits(uint64_t e) { /* x^e mod P, CRC-32 reflected (bit 31 = x^0) */
    uint32_t r = 0x80000000u;
    while (e--) r = (r >> 1) ^ ((r & 1u) ? 0xEDB88320u : 0u);
    return r;
}

static uint64_t kq[2][2]; /* {x^(63+D), x^(D-1)} << 32 for D = 512 and D = 128 */
static int kq_ready = 0;

__attribute__((target("pclmul,sse4.2"))) static __m128i fold128(__m128i x, const uint64_t* k) {
    const __m128i kk = _mm_set_epi64x((long long)k[1], (long long)k[0]);
    return _mm_xor_si128(_mm_clmulepi64_si128(x, kk, 0x00), _mm_clmulepi64_si128(x, kk, 0x11));
}

__attribute__((target("pclmul,sse4.2"))) static uint32_t crc32_pclmul(const uint8_t* p, uint64_t n) {
    if (n < 64) return (uint32_t)crc32(0L, p, (uInt)n);
    __m128i x0 = _mm_loadu_si128((const __m128i*)p), x1 = _mm_loadu_si128((const __m128i*)(p + 16)),
            x2 = _mm_loadu_si128((const __m128i*)(p + 32)), x3 = _mm_loadu_si128((const __m128i*)(p + 48));
    x0 = _mm_xor_si128(x0, _mm_cvtsi32_si128((int)0xFFFFFFFF)); /* init ~0 into the first 4 bytes */
    p += 64;
    n -= 64;
    while (n >= 64) {
        x0 = _mm_xor_si128(fold128(x0, kq[0]), _mm_loadu_si128((const __m128i*)p));
        x1 = _mm_xor_si128(fold128(x1, kq[0]), _mm_loadu_si128((const __m128i*)(p + 16)));
        x2 = _mm_xor_si128(fold128(x2, kq[0]), _mm_loadu_si128((const __m128i*)(p + 32)));
        x3 = _mm_xor_si128(fold128(x3, kq[0]), _mm_loadu_si128((const __m128i*)(p + 48)));
        p += 64;
        n -= 64;
    }
    __m128i x = _mm_xor_si128(fold128(x0, kq[1]), x1);
    x = _mm_xor_si128(fold128(x, kq[1]), x2);
    x = _mm_xor_si128(fold128(x, kq[1]), x3);
    while (n >= 16) {
        x = _mm_xor_si128(fold128(x, kq[1]), _mm_loadu_si128((const __m128i*)p));
        p += 16;
        n -= 16;
    }
    uint8_t b[16];
    _mm_storeu_si128((__m128i*)b, x);
    /* raw register of the remainder from zero = ~crc32(~0 ...), then the tail bytes */
    uint32_t raw = ~(uint32_t)crc32(0xFFFFFFFFuL, b, 16);
    return (uint32_t)crc32((uLong)~raw, p, (uInt)n);
}

static void* prun(void* q) {
    zjob* j = (zjob*)q;
    for (uint64_t i = j->lo; i < j->hi; ++i) j->out[i] = crc32_pclmul(j->base + j->offs[i], j->lens[i]);
    return NULL;
}

double oracle_pclmul_crc32_batch_timed(const uint8_t* base, const uint64_t* offs, const uint32_t* lens, uint64_t n,
                                       int threads, int reps, uint32_t* out) {
    if (!kq_ready) {
        kq[0][0] = (uint64_t)xpow_bits(63 + 512) << 32;
        kq[0][1] = (uint64_t)xpow_bits(512 - 1) << 32;
        kq[1][0] = (uint64_t)xpow_bits(63 + 128) << 32;
        kq[1][1] = (uint64_t)xpow_bits(128 - 1) << 32;
        kq_ready = 1;
    }
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    uint64_t cut[257];
    uint64_t total = 0, acc = 0;
    for (uint64_t i = 0; i < n; ++i) total += lens[i];
    cut[0] = 0;
    for (int t = 1; t <= threads; ++t) cut[t] = n;
    int t = 1;
    for (uint64_t i = 0; i < n && t < threads; ++i) {
        acc += lens[i];
        while (t < threads && acc * (uint64_t)threads >= total * (uint64_t)t) cut[t++] = i + 1;
    }
    pthread_t th[256];
    zjob jobs[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; ++r) {
        for (int k = 0; k < threads; ++k) {
            jobs[k] = (zjob){base, offs, lens, cut[k], cut[k + 1], out};
            pthread_create(&th[k], NULL, prun, &jobs[k]);
        }
        for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/*
 * BatchedReadOp's verify loop for a CRC-32 ledger (BatchedReadOp.java:164-190 ->
 * DigestManager.verifyDigest, DigestManager.java:226-283, CRC32DigestManager.java:28-87): per frame
 * zlib crc32() over the 32-byte header, resumed over the payload after the 8-byte digest, compared
 * with the BE long at 32; then the ledger / entry ids. The CRC-32 counterpart of
 * oracle/ref_shim.cpp's ref_verify_frames_timed (same status codes).
 */
typedef struct {
    const uint8_t* const* frames;
    const uint32_t* lens;
    uint64_t lo, hi;
    int64_t ledger, first;
    int32_t* status;
} zvjob;

static uint64_t be_n(const uint8_t* p, int k) {
    uint64_t v = 0;
    for (int b = 0; b < k; ++b) v = (v << 8) | p[b];
    return v;
}

static void* zvrun(void* p) {
    zvjob* j = (zvjob*)p;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const uint8_t* f = j->frames[i];
        const uint32_t l = j->lens[i];
        if (l < 40u) {
            j->status[i] = 1;
            continue;
        }
        uLong d = crc32(0L, f, 32);
        d = crc32(d, f + 40, (uInt)(l - 40u));
        if ((uint64_t)d != be_n(f + 32, 8)) j->status[i] = 2;
        else if ((int64_t)be_n(f, 8) != j->ledger) j->status[i] = 3;
        else if ((int64_t)be_n(f + 8, 8) != j->first + (int64_t)i) j->status[i] = 4;
        else j->status[i] = 0;
    }
    return NULL;
}

double oracle_zlib_verify_frames_timed(const uint8_t* const* frames, const uint32_t* lens, uint64_t n, int64_t ledger,
                                       int64_t first, int threads, int reps, int32_t* status) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    uint64_t cut[257];
    uint64_t total = 0, acc = 0;
    for (uint64_t i = 0; i < n; ++i) total += lens[i];
    cut[0] = 0;
    for (int t = 1; t <= threads; ++t) cut[t] = n;
    int t = 1;
    for (uint64_t i = 0; i < n && t < threads; ++i) {
        acc += lens[i];
        while (t < threads && acc * (uint64_t)threads >= total * (uint64_t)t) cut[t++] = i + 1;
    }
    pthread_t th[256];
    zvjob jobs[256];
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; ++r) {
        for (int k = 0; k < threads; ++k) {
            jobs[k] = (zvjob){frames, lens, cut[k], cut[k + 1], ledger, first, status};
            pthread_create(&th[k], NULL, zvrun, &jobs[k]);
        }
        for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
