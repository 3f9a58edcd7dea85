/*
 * GpuIntHash against the reference's own IntHash tests, for a maintainer with a JDK (this image has
 * none): drop it into circe-checksum/src/test/java next to Java9IntHashTest. It runs only where
 * libbkdigest loaded (Assume), and checks
 *  - the known answers of CRCTest.java:133-135 ("123456789" -> 0xe3069283) and ChecksumTest.java:41
 *    ("Some String" -> 608512271), through the address, array and copy paths of resume();
 *  - Java9IntHashTest.java:56-108: a checksum over one buffer equals the checksum of its first three
 *    bytes resumed over the rest held in a CompositeByteBuf, and over a view with neither an array nor
 *    a memory address (NoArrayNoMemoryAddrByteBuff);
 *  - the array path's argument checks (AbstractIncrementalIntHash.java:62-69);
 *  - every result equal to Crc32cIntChecksum's (the reference's selected provider) on the same bytes.
 * tests/test_java_sources.py resolves its imports and members against the reference.
 */
package com.scurrilous.circe.checksum;

import static org.junit.Assert.assertEquals;

import io.netty.buffer.ByteBuf;
import io.netty.buffer.ByteBufAllocator;
import io.netty.buffer.CompositeByteBuf;
import io.netty.buffer.Unpooled;
import java.nio.charset.StandardCharsets;
import java.util.Random;
import org.junit.Assume;
import org.junit.Before;
import org.junit.Test;

public class GpuIntHashTest {

    private final GpuIntHash hash = new GpuIntHash();

    @Before
    public void libraryLoaded() {
        Assume.assumeTrue(GpuDigest.isLoaded());
    }

    private void knownAnswer(String text, int want) {
        final byte[] bytes = text.getBytes(StandardCharsets.US_ASCII);
        final ByteBuf direct = ByteBufAllocator.DEFAULT.directBuffer(bytes.length).writeBytes(bytes);
        final ByteBuf heap = Unpooled.wrappedBuffer(bytes);
        final ByteBuf neither = new Java9IntHashTest.NoArrayNoMemoryAddrByteBuff(heap.duplicate());
        assertEquals(want, hash.calculate(direct));
        assertEquals(want, hash.calculate(heap));
        assertEquals(want, hash.calculate(neither));
        assertEquals(want, hash.resume(0, bytes, 0, bytes.length));
        assertEquals(want, Crc32cIntChecksum.computeChecksum(direct));
        direct.release();
    }

    @Test
    public void knownAnswers() {
        knownAnswer("123456789", 0xe3069283);
        knownAnswer("Some String", 608512271);
    }

    @Test
    public void resumeOverCompositeAndAddresslessBuffers() {
        final Random random = new Random(7);
        final byte[] huge = new byte[4096 * 3];
        random.nextBytes(huge);
        final ByteBuf total = ByteBufAllocator.DEFAULT.heapBuffer(6 + huge.length);
        total.writeBytes(new byte[] {1, 2, 3, 4, 5, 6}).writeBytes(huge);
        final ByteBuf b1 = ByteBufAllocator.DEFAULT.heapBuffer(3).writeBytes(new byte[] {1, 2, 3});
        final ByteBuf b2 = ByteBufAllocator.DEFAULT.heapBuffer(3).writeBytes(new byte[] {4, 5, 6});
        final ByteBuf b3 = ByteBufAllocator.DEFAULT.directBuffer(huge.length).writeBytes(huge);
        final CompositeByteBuf rest = new CompositeByteBuf(ByteBufAllocator.DEFAULT, false, 2, b2, b3);

        final int whole = hash.calculate(total);
        assertEquals(Crc32cIntChecksum.computeChecksum(total), whole);
        assertEquals(whole, hash.resume(hash.calculate(b1), rest));
        assertEquals(whole, hash.resume(hash.calculate(b1), new Java9IntHashTest.NoArrayNoMemoryAddrByteBuff(rest)));
        // an offset into a direct buffer: absolute index, as JniIntHash (memoryAddress() + offset)
        final ByteBuf direct = ByteBufAllocator.DEFAULT.directBuffer(total.readableBytes()).writeBytes(total, 0,
                total.readableBytes());
        assertEquals(hash.resume(hash.calculate(b1), rest), hash.resume(hash.calculate(direct, 0, 3), direct, 3,
                direct.readableBytes() - 3));
        total.release();
        b1.release();
        rest.release();
        direct.release();
    }

    @Test(expected = IndexOutOfBoundsException.class)
    public void arrayOffsetPastTheEnd() {
        hash.resume(0, new byte[8], 6, 3);
    }

    @Test(expected = IndexOutOfBoundsException.class)
    public void negativeLength() {
        hash.resume(0, new byte[8], 0, -1);
    }

    @Test
    public void emptyRangeReturnsTheCurrentValue() {
        assertEquals(0x12345678, hash.resume(0x12345678, new byte[8], 8, 0));
    }
}
