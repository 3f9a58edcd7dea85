/*
 * Behavioural test of the two batch hooks against the reference's own per-entry calls, for a
 * maintainer with a JDK (this image has none): drop it into bookkeeper-server/src/test/java next to
 * CompositeByteBufUnwrapBugReproduceTest, whose parameters (payload sizes around
 * BookieProtoEncoding.SMALL_ENTRY_SIZE_THRESHOLD, V2 and V3) and payload pattern (byte i = (byte) i)
 * it reuses. With the GPU library loaded the hooks take the library; without it they take the
 * reference's loops — both must give the reference's results.
 *
 *  - GpuBatchPackager.packageEntries: every packaged object equals
 *    DigestManager.computeDigestAndPackageForSending's (DigestManager.java:117-181) in type
 *    (ByteBuf below 16 KiB under V2, else ByteBufList), readable bytes, and readerIndex / capacity of
 *    a V2 ByteBuf.
 *  - GpuBatchVerifier.verifiedPrefix: the verified prefix equals BatchedReadOp's loop
 *    (BatchedReadOp.java:175-189) and every verified buffer's readerIndex is METADATA_LENGTH +
 *    macCodeLength, as verifyDigestAndReturnData leaves it (DigestManager.java:336); also with a
 *    corrupted entry and with a buffer already partly read.
 *
 * tests/test_java_sources.py resolves its imports against the reference (JUnit and Netty are Maven
 * dependencies of bookkeeper-server's tests).
 */
package org.apache.bookkeeper.proto.checksum;

import static org.junit.Assert.assertArrayEquals;
import static org.junit.Assert.assertEquals;
import static org.junit.Assert.assertTrue;

import io.netty.buffer.ByteBuf;
import io.netty.buffer.ByteBufAllocator;
import io.netty.buffer.Unpooled;
import io.netty.buffer.UnpooledByteBufAllocator;
import io.netty.util.ReferenceCounted;
import java.util.Arrays;
import java.util.Collection;
import org.apache.bookkeeper.client.BKException;
import org.apache.bookkeeper.proto.BookieProtoEncoding;
import org.apache.bookkeeper.proto.BookieProtocol;
import org.apache.bookkeeper.util.ByteBufList;
import org.junit.Test;
import org.junit.runner.RunWith;
import org.junit.runners.Parameterized;

@RunWith(Parameterized.class)
public class GpuBatchHooksTest {
    private static final long LEDGER = 1;
    private static final int N = 24;
    private final int payloadSize;
    private final boolean useV2Protocol;
    private final boolean crc32c;

    @Parameterized.Parameters
    public static Collection<Object[]> scenarios() {
        final int t = BookieProtoEncoding.SMALL_ENTRY_SIZE_THRESHOLD;
        return Arrays.asList(new Object[][] {
                {t - 1, true, true}, {t - 1, false, true}, {t, true, true}, {t, false, true},
                {t - 1, true, false}, {t, false, false}, {37, true, true}, {70000, false, false},
        });
    }

    public GpuBatchHooksTest(int payloadSize, boolean useV2Protocol, boolean crc32c) {
        this.payloadSize = payloadSize;
        this.useV2Protocol = useV2Protocol;
        this.crc32c = crc32c;
    }

    private DigestManager manager() {
        final ByteBufAllocator allocator = UnpooledByteBufAllocator.DEFAULT;
        return crc32c ? new CRC32CDigestManager(LEDGER, useV2Protocol, allocator)
                : new CRC32DigestManager(LEDGER, useV2Protocol, allocator);
    }

    private byte[][] payloads() {
        final byte[][] p = new byte[N][];
        for (int k = 0; k < N; k++) {
            p[k] = new byte[payloadSize + k];  // one size per entry, the scenario's first
            for (int i = 0; i < p[k].length; i++) {
                p[k][i] = (byte) (i + k);
            }
        }
        return p;
    }

    private static byte[] bytesOf(ReferenceCounted r) {
        if (r instanceof ByteBuf) {
            final ByteBuf b = (ByteBuf) r;
            final byte[] out = new byte[b.readableBytes()];
            b.getBytes(b.readerIndex(), out);
            return out;
        }
        return ((ByteBufList) r).toArray();
    }

    @Test
    public void packagerEqualsComputeDigestAndPackageForSending() {
        final DigestManager dm = manager();
        final byte[][] payloads = payloads();
        final long[] ids = new long[N];
        final long[] lengths = new long[N];
        for (int k = 0; k < N; k++) {
            ids[k] = 1000 + k;
            lengths[k] = 5000L * k + payloads[k].length;
        }
        final byte[] masterKey = new byte[BookieProtocol.MASTER_KEY_LENGTH];
        final ReferenceCounted[] got = GpuBatchPackager.packageEntries(dm, UnpooledByteBufAllocator.DEFAULT, ids, 999,
                lengths, payloads, masterKey, BookieProtocol.FLAG_RECOVERY_ADD);
        for (int k = 0; k < N; k++) {
            final ReferenceCounted want = dm.computeDigestAndPackageForSending(ids[k], 999, lengths[k],
                    Unpooled.wrappedBuffer(payloads[k], 0, payloads[k].length), masterKey,
                    BookieProtocol.FLAG_RECOVERY_ADD);
            assertEquals("object shape of entry " + k, want.getClass(), got[k].getClass());
            assertArrayEquals("bytes of entry " + k, bytesOf(want), bytesOf(got[k]));
            if (want instanceof ByteBuf) {
                assertEquals(((ByteBuf) want).readerIndex(), ((ByteBuf) got[k]).readerIndex());
                assertEquals(((ByteBuf) want).capacity(), ((ByteBuf) got[k]).capacity());
            }
            want.release();
            got[k].release();
        }
    }

    // the framed entries [32 B header][digest][payload] as direct buffers, as a batched read returns them
    private ByteBufList framed(DigestManager dm, byte[][] payloads) {
        final DigestManager v3 = crc32c ? new CRC32CDigestManager(LEDGER, false, UnpooledByteBufAllocator.DEFAULT)
                : new CRC32DigestManager(LEDGER, false, UnpooledByteBufAllocator.DEFAULT);
        final ByteBufList list = ByteBufList.get();
        for (int k = 0; k < N; k++) {
            final ReferenceCounted r = v3.computeDigestAndPackageForSending(100 + k, 99 + k, payloads[k].length,
                    Unpooled.wrappedBuffer(payloads[k]), new byte[0], 0);
            final byte[] bytes = bytesOf(r);
            r.release();
            final ByteBuf b = Unpooled.directBuffer(bytes.length);
            b.writeBytes(bytes);
            list.add(b);
        }
        return list;
    }

    private static ByteBufList copyOf(ByteBufList l) {
        final ByteBufList c = ByteBufList.get();
        for (int k = 0; k < l.size(); k++) {
            final ByteBuf b = l.getBuffer(k);
            final ByteBuf d = Unpooled.directBuffer(b.capacity());
            d.writeBytes(b, 0, b.writerIndex());
            d.readerIndex(b.readerIndex());
            c.add(d);
        }
        return c;
    }

    // BatchedReadOp.java:175-189
    private static int referencePrefix(DigestManager dm, long first, ByteBufList l) {
        int verified = 0;
        for (int i = 0; i < l.size(); i++) {
            try {
                dm.verifyDigestAndReturnData(first + i, l.getBuffer(i));
                verified++;
            } catch (BKException.BKDigestMatchException e) {
                break;
            }
        }
        return verified;
    }

    private void assertSameAsReference(DigestManager dm, ByteBufList frames) {
        final ByteBufList mine = copyOf(frames);
        final ByteBufList ref = copyOf(frames);
        final int want = referencePrefix(dm, 100, ref);
        assertEquals("verified prefix", want, GpuBatchVerifier.verifiedPrefix(dm, 100, mine));
        for (int i = 0; i < want; i++) {
            assertEquals("readerIndex of verified entry " + i, ref.getBuffer(i).readerIndex(),
                    mine.getBuffer(i).readerIndex());
            assertEquals(DigestManager.METADATA_LENGTH + dm.macCodeLength, mine.getBuffer(i).readerIndex());
        }
        mine.release();
        ref.release();
    }

    @Test
    public void verifierEqualsBatchedReadOpLoop() {
        final DigestManager dm = manager();
        final ByteBufList frames = framed(dm, payloads());
        assertSameAsReference(dm, frames);  // all verify
        final ByteBuf bad = frames.getBuffer(N / 2);
        bad.setByte(bad.writerIndex() - 1, bad.getByte(bad.writerIndex() - 1) ^ 1);
        assertSameAsReference(dm, frames);  // the prefix before the corrupted payload
        frames.getBuffer(3).readerIndex(5);  // a buffer already partly read: the reference's addressing
        assertSameAsReference(dm, frames);
        assertTrue(frames.release());
    }
}
