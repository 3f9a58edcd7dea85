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
