/*
 * Crc32cIntChecksum's provider selection with the GPU library first. The reference picks one IntHash
 * at class init by capability only — JNI SSE4.2, then java.util.zip.CRC32C, then the table CRC
 * (circe-checksum/.../checksum/Crc32cIntChecksum.java:28-36) — and never throws. The drop-in is a
 * one-line change of that static block (INTEGRATION.md §1):
 *
 *     CRC32C_HASH = GpuProviderChain.select();
 *
 * The GPU provider is taken only when libbkdigest loaded AND a device initialised; every failure
 * falls through to the reference's own chain, unchanged. Not compiled in this repository's image
 * (no JDK): tests/test_java_sources.py resolves its imports against the reference tree.
 */
package com.scurrilous.circe.checksum;

import com.scurrilous.circe.crc.Sse42Crc32C;

final class GpuProviderChain {

    private GpuProviderChain() {
    }

    static IntHash select() {
        try {
            if (GpuDigest.isSupported()) {
                return new GpuIntHash();
            }
        } catch (Throwable t) {
            // a library that fails to initialise leaves the reference's chain in charge
        }
        if (Sse42Crc32C.isSupported()) {
            return new JniIntHash();
        } else if (Java9IntHash.HAS_JAVA9_CRC32C) {
            return new Java9IntHash();
        }
        return new Java8IntHash();
    }
}
