/*
 * JNI shim over libbkdigest.so (include/bkdigest.h). Two Java classes bind to it:
 *
 * 1. com.scurrilous.circe.crc.Sse42Crc32C — the reference's own natives
 *    (circe-checksum/src/main/circe/cpp/crc32c_sse42_jni.cpp:20-78; Java declarations at
 *    circe-checksum/src/main/java/com/scurrilous/circe/crc/Sse42Crc32C.java:119-129), with the same
 *    semantics, so an unmodified JVM that loads this library as /lib/libcirce-checksum.so picks the
 *    engine up through JniIntHash (Crc32cIntChecksum.java:28-36):
 *      nativeSupported          -> bkd_circe_supported (always 1: GPU or the library's CPU route)
 *      nativeArray/DirectBuffer/Unsafe -> bkd_resume_host (host memory: CPU route up to
 *                                  bkd_get_cpu_route_max() bytes, GPU above); a null direct-buffer
 *                                  address returns 0 (:39-40); the config handle is ignored
 *                                  (results never depend on the chunk ladder)
 *      allocConfig / freeConfig -> bkd_circe_alloc_config / bkd_circe_free_config (same validation)
 * 2. com.scurrilous.circe.checksum.GpuDigest — the batch surface the reference lacks
 *    (INTEGRATION.md §2): device count/init, per-call resume for CRC32C and CRC32, host-memory
 *    batches, and the host-resident DigestManager verify/package batches (direct-buffer addresses, or
 *    the entries' heap arrays for LedgerFragmentReplicator's batch: packageBatchArrays).
 *
 * Built into a loadable library only where a JDK is present (native/jni/Makefile; this image has
 * none). The CPU suite compiles this file with -Wall -Werror against a test-only <jni.h>
 * (tests/jni_fake/) and calls every native through a fake JNIEnv (tests/test_jni_shim.py).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "bkdigest.h"

/* ---- com.scurrilous.circe.crc.Sse42Crc32C ---------------------------------------------------- */

JNIEXPORT jboolean JNICALL Java_com_scurrilous_circe_crc_Sse42Crc32C_nativeSupported(JNIEnv* env, jclass cls) {
    (void)env;
    (void)cls;
    return bkd_circe_supported() ? JNI_TRUE : JNI_FALSE;
}

static jint resume_host_or_zero(jint current, const void* p, jlong length) {
    uint32_t out = 0;
    if (length <= 0) return current; /* crc32c_sse42.cpp:211-213 (the Java side rejects length < 0) */
    return bkd_resume_host(BKD_CRC32C, (uint32_t)current, p, (uint64_t)length, &out) == BKD_OK ? (jint)out : 0;
}

/* A heap array's region [index, index + length) (nativeArray and GpuDigest.resumeArray). */
static jint array_resume(JNIEnv* env, int algo, jint current, jbyteArray input, jint index, jint length) {
    if (length <= 0) return current;
    const int long_route = (uint64_t)length > bkd_get_cpu_route_max();
    uint32_t out = 0;
    if (long_route) {
        /* past the per-call CPU bound (the GPU route, a PCIe round trip, or a multi-MiB scan over
         * the host pool): copy the region out instead of holding the array's critical section, which
         * stalls the JVM's collector, across it (the reference held it only for a short CPU scan,
         * crc32c_sse42_jni.cpp:29-31). An index/length outside the array leaves the JVM's
         * ArrayIndexOutOfBoundsException pending and returns 0. */
        jbyte* copy = (jbyte*)malloc((size_t)length);
        if (copy) {
            (*env)->GetByteArrayRegion(env, input, index, length, copy);
            int rc = BKD_ERR_BOUNDS;
            if (!(*env)->ExceptionCheck(env)) rc = bkd_resume_host(algo, (uint32_t)current, copy, (uint64_t)length, &out);
            free(copy);
            return rc == BKD_OK ? (jint)out : 0;
        }
        /* no memory for the copy: the CPU route inside the critical section instead (never a bare 0
         * that a caller could take for a checksum) */
    }
    /* the CPU route: pinned for the duration of the scan only, as crc32c_sse42_jni.cpp:29-31 */
    jbyte* buf = (jbyte*)(*env)->GetPrimitiveArrayCritical(env, input, 0);
    if (!buf) return 0; /* the JVM's OutOfMemoryError is pending */
    const int rc = long_route ? bkd_cpu_resume(algo, (uint32_t)current, buf + index, (uint64_t)length, &out)
                              : bkd_resume_host(algo, (uint32_t)current, buf + index, (uint64_t)length, &out);
    (*env)->ReleasePrimitiveArrayCritical(env, input, buf, JNI_ABORT);
    return rc == BKD_OK ? (jint)out : 0;
}

JNIEXPORT jint JNICALL Java_com_scurrilous_circe_crc_Sse42Crc32C_nativeArray(JNIEnv* env, jclass cls, jint current,
                                                                             jbyteArray input, jint index,
                                                                             jint length, jlong config) {
    (void)cls;
    (void)config;
    return array_resume(env, BKD_CRC32C, current, input, index, length);
}

JNIEXPORT jint JNICALL Java_com_scurrilous_circe_crc_Sse42Crc32C_nativeDirectBuffer(JNIEnv* env, jclass cls,
                                                                                    jint current, jobject input,
                                                                                    jint offset, jint length,
                                                                                    jlong config) {
    (void)cls;
    (void)config;
    const char* address = (const char*)(*env)->GetDirectBufferAddress(env, input);
    if (!address) return 0; /* crc32c_sse42_jni.cpp:39-40 */
    return resume_host_or_zero(current, address + offset, length);
}

JNIEXPORT jint JNICALL Java_com_scurrilous_circe_crc_Sse42Crc32C_nativeUnsafe(JNIEnv* env, jclass cls, jint current,
                                                                              jlong address, jlong length,
                                                                              jlong config) {
    (void)env;
    (void)cls;
    (void)config;
    return resume_host_or_zero(current, (const void*)(intptr_t)address, length);
}

JNIEXPORT jlong JNICALL Java_com_scurrilous_circe_crc_Sse42Crc32C_allocConfig(JNIEnv* env, jclass cls,
                                                                              jintArray chunkWords) {
    (void)cls;
    const jsize len = (*env)->GetArrayLength(env, chunkWords);
    jint* arr = (jint*)(*env)->GetPrimitiveArrayCritical(env, chunkWords, 0);
    if (!arr) return 0;
    const int64_t h = bkd_circe_alloc_config((const int32_t*)arr, (int32_t)len);
    (*env)->ReleasePrimitiveArrayCritical(env, chunkWords, arr, JNI_ABORT);
    return (jlong)h;
}

JNIEXPORT void JNICALL Java_com_scurrilous_circe_crc_Sse42Crc32C_freeConfig(JNIEnv* env, jclass cls, jlong config) {
    (void)env;
    (void)cls;
    bkd_circe_free_config((int64_t)config);
}

/* ---- com.scurrilous.circe.checksum.GpuDigest (new batch surface) ----------------------------- */

JNIEXPORT jint JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_deviceCount(JNIEnv* env, jclass cls) {
    (void)env;
    (void)cls;
    return bkd_device_count();
}

JNIEXPORT jint JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_init(JNIEnv* env, jclass cls, jint dev) {
    (void)env;
    (void)cls;
    return bkd_init(dev);
}

/* resume(algo, current, address, length): a host address (Netty memoryAddress()); CRC32 included, for
 * CRC32DigestManager's DirectMemoryCRC32Digest (CRC32DigestManager.java:28-87) */
JNIEXPORT jint JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_resumeAddress(JNIEnv* env, jclass cls,
                                                                                       jint algo, jint current,
                                                                                       jlong address, jlong len) {
    (void)env;
    (void)cls;
    uint32_t out = 0;
    if (len <= 0) return current;
    if (!address) return 0;
    return bkd_resume_host(algo, (uint32_t)current, (const void*)(intptr_t)address, (uint64_t)len, &out) == BKD_OK
               ? (jint)out
               : 0;
}

/* resumeArray(algo, current, byte[], offset, len): a heap buffer (ByteBuf.array()); the Java side has
 * checked the bounds (AbstractIncrementalIntHash.java:62-69) */
JNIEXPORT jint JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_resumeArray(JNIEnv* env, jclass cls,
                                                                                     jint algo, jint current,
                                                                                     jbyteArray input, jint offset,
                                                                                     jint len) {
    (void)cls;
    return array_resume(env, algo, current, input, offset, len);
}

/* batch over one host region: offsets/lengths/seeds/out are addresses of direct buffers */
JNIEXPORT jint JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_resumeBatch(
    JNIEnv* env, jclass cls, jint algo, jlong base, jlong size, jlong offs, jlong lens, jlong n, jlong seeds,
    jint seedAll, jlong out) {
    (void)env;
    (void)cls;
    return bkd_crc_batch_host(algo, (const void*)(intptr_t)base, (uint64_t)size, (const uint64_t*)(intptr_t)offs,
                              (const uint32_t*)(intptr_t)lens, (uint64_t)n, (const uint32_t*)(intptr_t)seeds,
                              (uint32_t)seedAll, (uint32_t*)(intptr_t)out);
}

/* BatchedReadOp.complete over a ByteBufList (BatchedReadOp.java:164-190): frame addresses and lengths
 * in direct buffers; returns the verified prefix length (n if all verified) or a negative BKD_ERR_* */
JNIEXPORT jlong JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_verifyBatch(
    JNIEnv* env, jclass cls, jint algo, jlong ledgerId, jlong firstEntryId, jboolean skipEntryIdCheck,
    jlong frameAddrs, jlong frameLens, jlong n, jlong statusOut) {
    (void)env;
    (void)cls;
    uint64_t first_bad = 0;
    const int rc = bkd_digest_verify_batch_host(algo, ledgerId, firstEntryId, skipEntryIdCheck ? 1 : 0,
                                                (const void* const*)(intptr_t)frameAddrs,
                                                (const uint32_t*)(intptr_t)frameLens, (uint64_t)n,
                                                (int32_t*)(intptr_t)statusOut, &first_bad);
    return rc == BKD_OK ? (jlong)first_bad : (jlong)rc;
}

/* PendingAddOp / LedgerFragmentReplicator packaging (DigestManager.java:117-181) of n host payloads */
JNIEXPORT jint JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_packageBatch(
    JNIEnv* env, jclass cls, jint algo, jlong ledgerId, jlong entryIds, jlong lacs, jlong lengthFields,
    jlong payloadAddrs, jlong payloadLens, jlong n, jlong framesOut, jlong frameStride, jlong digestsOut) {
    (void)env;
    (void)cls;
    return bkd_digest_package_batch_host(algo, ledgerId, (const int64_t*)(intptr_t)entryIds,
                                         (const int64_t*)(intptr_t)lacs, (const int64_t*)(intptr_t)lengthFields,
                                         (const void* const*)(intptr_t)payloadAddrs,
                                         (const uint32_t*)(intptr_t)payloadLens, (uint64_t)n,
                                         (void*)(intptr_t)framesOut, (uint64_t)frameStride,
                                         (uint32_t*)(intptr_t)digestsOut);
}

/* LedgerFragmentReplicator's batch of heap payloads (GpuBatchPackager; LedgerFragmentReplicator.java:497-511
 * wraps each entry's byte[] in Unpooled.wrappedBuffer). The payloads are copied out back to back into one
 * host buffer (GetByteArrayRegion: no array is pinned across the library call, whose GPU route is a PCIe
 * round trip) and packaged by bkd_digest_package_batch_host with one lastAddConfirmed for the batch.
 * Mismatched array lengths leave IllegalArgumentException pending, a null payload NullPointerException. */
JNIEXPORT jint JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_packageBatchArrays(
    JNIEnv* env, jclass cls, jint algo, jlong ledgerId, jlongArray entryIds, jlong lastAddConfirmed,
    jlongArray lengthFields, jobjectArray payloads, jlong framesOut, jlong frameStride, jlong digestsOut) {
    (void)cls;
    if (!entryIds || !lengthFields || !payloads) {
        (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/NullPointerException"), "packageBatchArrays");
        return BKD_ERR_INVALID_ARG;
    }
    const jsize n = (*env)->GetArrayLength(env, payloads);
    if ((*env)->GetArrayLength(env, entryIds) != n || (*env)->GetArrayLength(env, lengthFields) != n) {
        (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/IllegalArgumentException"),
                         "entryIds, lengthFields and payloads differ in length");
        return BKD_ERR_INVALID_ARG;
    }
    if (n == 0) return BKD_OK;
    int rc = BKD_ERR_NOMEM;
    uint64_t total = 0;
    int64_t* ids = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int64_t* lacs = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int64_t* lfs = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    const void** ptrs = (const void**)malloc((size_t)n * sizeof(void*));
    uint32_t* lens = (uint32_t*)malloc((size_t)n * sizeof(uint32_t));
    char* staging = NULL;
    if (!ids || !lacs || !lfs || !ptrs || !lens) goto done;
    (*env)->GetLongArrayRegion(env, entryIds, 0, n, (jlong*)ids);
    (*env)->GetLongArrayRegion(env, lengthFields, 0, n, (jlong*)lfs);
    for (jsize i = 0; i < n; ++i) {  /* pass 1: the payload lengths */
        lacs[i] = lastAddConfirmed;
        jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, payloads, i);
        if (!a) {
            (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/NullPointerException"), "null payload");
            rc = BKD_ERR_INVALID_ARG;
            goto done;
        }
        lens[i] = (uint32_t)(*env)->GetArrayLength(env, a);
        total += lens[i];
        (*env)->DeleteLocalRef(env, a);
    }
    staging = (char*)malloc(total ? (size_t)total : 1u);
    if (!staging) goto done;
    total = 0;
    for (jsize i = 0; i < n && !(*env)->ExceptionCheck(env); ++i) {  /* pass 2: the bytes, back to back */
        jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, payloads, i);
        if (!a) {  /* replaced by null since pass 1 (another thread) */
            (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/NullPointerException"), "null payload");
            break;
        }
        (*env)->GetByteArrayRegion(env, a, 0, (jsize)lens[i], (jbyte*)(staging + total));
        (*env)->DeleteLocalRef(env, a);
        ptrs[i] = staging + total;
        total += lens[i];
    }
    rc = (*env)->ExceptionCheck(env)
             ? BKD_ERR_INVALID_ARG
             : bkd_digest_package_batch_host(algo, ledgerId, ids, lacs, lfs, (const void* const*)ptrs, lens,
                                             (uint64_t)n, (void*)(intptr_t)framesOut, (uint64_t)frameStride,
                                             (uint32_t*)(intptr_t)digestsOut);
done:
    free(staging);
    free(lens);
    free((void*)ptrs);
    free(lfs);
    free(lacs);
    free(ids);
    return rc;
}

JNIEXPORT jstring JNICALL Java_com_scurrilous_circe_checksum_GpuDigest_lastError(JNIEnv* env, jclass cls) {
    (void)cls;
    return (*env)->NewStringUTF(env, bkd_last_error());
}
