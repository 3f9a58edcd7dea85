/*
 * Java side of the batch surface of libbkdigest (include/bkdigest.h), bound by the JNI shim
 * native/jni/bkdigest_jni.c. It lives in circe-checksum beside the IntHash providers (that module
 * already depends on native-library-common for Sse42Crc32C's loader; bookkeeper-server depends on
 * circe-checksum, never the other way). Not compiled in this repository's image (no JDK); the native
 * declarations below are the table tests/test_jni_signatures.py checks the shim's exports against,
 * and tests/test_jni_shim.py executes every one of those natives through a fake JNIEnv.
 *
 * The reference has no batch API: BatchedReadOp verifies a ByteBufList entry by entry
 * (bookkeeper-server/.../client/BatchedReadOp.java:164-190) and PendingAddOp packages one entry per
 * add (PendingAddOp.java:261, DigestManager.java:117-181). These entry points take whole batches.
 */
package com.scurrilous.circe.checksum;

import org.apache.bookkeeper.common.util.nativelib.NativeUtils;

public final class GpuDigest {
    /** Algorithm ids of the C-ABI (BKD_CRC32C / BKD_CRC32). */
    public static final int CRC32C = 0;
    public static final int CRC32 = 1;

    /** BKD_VERIFY_* codes written per entry by {@link #verifyBatch}. */
    public static final int VERIFY_OK = 0;
    public static final int VERIFY_TOO_SHORT = 1;
    public static final int VERIFY_DIGEST_MISMATCH = 2;
    public static final int VERIFY_LEDGER_MISMATCH = 3;
    public static final int VERIFY_ENTRY_MISMATCH = 4;

    private static final boolean LOADED;
    private static final boolean DEVICE;

    static {
        boolean loaded = false;
        boolean device = false;
        try {
            // the same jar location and loader as the circe natives (Sse42Crc32C.java:18-19,33-40;
            // native-library-common NativeUtils.java:54-116): the shim is packaged as the circe
            // library, so this is the one library Sse42Crc32C loads too
            NativeUtils.loadLibraryFromJar("/lib/libcirce-checksum." + NativeUtils.libType());
            loaded = true;
            device = deviceCount() > 0 && init(0) == 0;
        } catch (Throwable t) {
            // never fatal: without the library Crc32cIntChecksum keeps its own chain
        }
        LOADED = loaded;
        DEVICE = device;
    }

    private GpuDigest() {
    }

    /** The library loaded (per-call resumes work with or without a GPU: the library's CPU route). */
    public static boolean isLoaded() {
        return LOADED;
    }

    /** The library loaded and a HIP device initialised (batches can take the GPU). */
    public static boolean isSupported() {
        return DEVICE;
    }

    public static native int deviceCount();                                        // bkd_device_count

    public static native int init(int device);                                     // bkd_init

    /** resume(current, memoryAddress, len): finalized CRC in and out; len <= 0 returns current. */
    public static native int resumeAddress(int algo, int current, long address, long len);  // bkd_resume_host

    /** resume over buffer[offset, offset + len) of a heap array (bounds checked by the caller). */
    public static native int resumeArray(int algo, int current, byte[] buffer, int offset, int len);

    /** One host region: offsets (u64), lengths (u32), seeds (u32, or 0 for seedAll) and out (u32) are
     *  addresses of direct buffers. Returns 0 or a negative BKD_ERR_* code. */
    public static native int resumeBatch(int algo, long base, long baseSize, long offsets, long lengths,
                                         long n, long seeds, int seedAll, long out);  // bkd_crc_batch_host

    /** BatchedReadOp over a ByteBufList: frame addresses (u64) and lengths (u32) in direct buffers,
     *  one VERIFY_* code per entry to statusOut (i32). Returns the verified-prefix length (n when
     *  every entry verified) or a negative BKD_ERR_* code. */
    public static native long verifyBatch(int algo, long ledgerId, long firstEntryId, boolean skipEntryIdCheck,
                                          long frameAddrs, long frameLens, long n, long statusOut);

    /** Header + digest of n payloads (PendingAddOp / LedgerFragmentReplicator): frame i's first 32 + 4
     *  (CRC32C) or 32 + 8 (CRC32) bytes at framesOut + i * frameStride, digest i at digestsOut. */
    public static native int packageBatch(int algo, long ledgerId, long entryIds, long lacs, long lengthFields,
                                          long payloadAddrs, long payloadLens, long n, long framesOut,
                                          long frameStride, long digestsOut);

    /** LedgerFragmentReplicator's batch (GpuBatchPackager): the same as packageBatch for n heap payloads
     *  (the entries' byte[], as Unpooled.wrappedBuffer(data) wraps them) with one lastAddConfirmed for the
     *  batch; the payloads are copied out with GetByteArrayRegion, never pinned across the call. Returns 0
     *  or a negative BKD_ERR_* code (a null or short array leaves the JVM's exception pending). */
    public static native int packageBatchArrays(int algo, long ledgerId, long[] entryIds, long lastAddConfirmed,
                                                long[] lengthFields, byte[][] payloads, long framesOut,
                                                long frameStride, long digestsOut);

    public static native String lastError();                                       // bkd_last_error
}
