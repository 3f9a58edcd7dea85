/*
 * IntHash over libbkdigest (GpuDigest's natives), first in Crc32cIntChecksum's provider chain when
 * the library loads and a device initialises (GpuProviderChain, INTEGRATION.md §1). Not compiled in
 * this repository's image (no JDK).
 *
 * Interface: circe-checksum/.../checksum/IntHash.java:23-35. Buffer dispatch follows the other
 * providers (JniIntHash.java:45-53): a native address when the ByteBuf has one, the backing array
 * when it has one, else the readable bytes of an NIO view. Per-call resumes of small buffers stay on
 * the library's CPU route (bkd_resume_host); only long buffers take the GPU.
 */
package com.scurrilous.circe.checksum;

import io.netty.buffer.ByteBuf;

public class GpuIntHash implements IntHash {

    private final int algo;

    public GpuIntHash() {
        this(GpuDigest.CRC32C);
    }

    /** CRC32C (circe) or CRC32 (CRC32DigestManager's java.util.zip.CRC32 arithmetic). */
    public GpuIntHash(int algo) {
        if (algo != GpuDigest.CRC32C && algo != GpuDigest.CRC32) {
            throw new IllegalArgumentException("algorithm " + algo);
        }
        this.algo = algo;
    }

    @Override
    public int calculate(ByteBuf buffer) {
        return resume(0, buffer, buffer.readerIndex(), buffer.readableBytes());
    }

    @Override
    public int calculate(ByteBuf buffer, int offset, int len) {
        return resume(0, buffer, offset, len);
    }

    @Override
    public int resume(int current, ByteBuf buffer) {
        return resume(current, buffer, buffer.readerIndex(), buffer.readableBytes());
    }

    @Override
    public int resume(int current, ByteBuf buffer, int offset, int len) {
        if (buffer.hasMemoryAddress()) {
            return GpuDigest.resumeAddress(algo, current, buffer.memoryAddress() + offset, len);
        }
        if (buffer.hasArray()) {
            return resume(current, buffer.array(), buffer.arrayOffset() + offset, len);
        }
        // a composite or otherwise address-less buffer: its readable bytes, copied out once
        byte[] copy = new byte[len];
        buffer.getBytes(offset, copy);
        return resume(current, copy, 0, len);
    }

    @Override
    public int resume(int current, byte[] buffer, int offset, int len) {
        // the array path's argument checks (AbstractIncrementalIntHash.java:62-69)
        if (offset < 0 || len < 0 || offset > buffer.length - len) {
            throw new IndexOutOfBoundsException("offset " + offset + ", length " + len + ", array " + buffer.length);
        }
        return GpuDigest.resumeArray(algo, current, buffer, offset, len);
    }

    @Override
    public boolean acceptsMemoryAddressBuffer() {
        return true;
    }
}
