/*
 * The batched package hook for LedgerFragmentReplicator's batch-read callback
 * (bookkeeper-server/.../client/LedgerFragmentReplicator.java:480-511). The reference packages the
 * entries of a batch read one by one inside the loop that sends them:
 *
 *     byte[] data = entry.getEntry();
 *     ReferenceCounted toSend = lh.getDigestManager().computeDigestAndPackageForSending(entry.getEntryId(),
 *             lh.getLastAddConfirmed(), entry.getLength(), Unpooled.wrappedBuffer(data, 0, data.length),
 *             lh.getLedgerKey(), BookieProtocol.FLAG_RECOVERY_ADD);
 *
 * With this class the batch is packaged in one call before the loop,
 *
 *     ReferenceCounted[] packaged = GpuBatchPackager.packageEntries(lh.getDigestManager(),
 *             lh.clientCtx.getByteBufAllocator(), entryIds, lh.getLastAddConfirmed(), lengths, payloads,
 *             lh.getLedgerKey(), BookieProtocol.FLAG_RECOVERY_ADD);
 *
 * and packaged[i] is, byte for byte and in object shape, what computeDigestAndPackageForSending returns
 * for entry i (DigestManager.java:117-181):
 *   V2 — one allocator buffer [frame length][packet header][master key][32 B header][digest], readerIndex 0,
 *        capacity exactly bufferSize, with the payload copied in when it is below
 *        BookieProtoEncoding.SMALL_ENTRY_SIZE_THRESHOLD (16 KiB, BookieProtoEncoding.java:48), else
 *        ByteBufList.get(that buffer, payload);
 *   V3 — ByteBufList.get(Unpooled header buffer [32 B header][digest], payload).
 * The 32-byte BE header [ledgerId, entryId, lastAddConfirmed, length] and its digest (CRC32C: 4 B BE int;
 * CRC32: 8 B BE zero-extended long) come from libbkdigest's bkd_digest_package_batch_host in one call
 * for the whole batch; the payloads are the entries' heap arrays (GpuDigest.packageBatchArrays copies
 * them out with GetByteArrayRegion rather than pinning n arrays across the call). CRC32C and CRC32
 * managers take that path; MAC and dummy digests, no library or a library error package every entry
 * through the reference's own per-entry call. It lives in DigestManager's package for the manager's
 * ledgerId, useV2Protocol and macCodeLength. Not compiled in this repository's image (no JDK):
 * tests/test_java_sources.py resolves its imports and members against the reference.
 */
package org.apache.bookkeeper.proto.checksum;

import com.scurrilous.circe.checksum.GpuDigest;
import io.netty.buffer.ByteBuf;
import io.netty.buffer.ByteBufAllocator;
import io.netty.buffer.PooledByteBufAllocator;
import io.netty.buffer.Unpooled;
import io.netty.util.ReferenceCounted;
import org.apache.bookkeeper.proto.BookieProtoEncoding;
import org.apache.bookkeeper.proto.BookieProtocol;
import org.apache.bookkeeper.util.ByteBufList;

public final class GpuBatchPackager {

    private GpuBatchPackager() {
    }

    /**
     * packaged[i] = dm.computeDigestAndPackageForSending(entryIds[i], lastAddConfirmed, lengths[i],
     * Unpooled.wrappedBuffer(payloads[i], 0, payloads[i].length), masterKey, flags). allocator is the one
     * the manager was created with (the ledger's ClientContext.getByteBufAllocator(), LedgerHandle.java:231-232).
     */
    public static ReferenceCounted[] packageEntries(DigestManager dm, ByteBufAllocator allocator, long[] entryIds,
                                                    long lastAddConfirmed, long[] lengths, byte[][] payloads,
                                                    byte[] masterKey, int flags) {
        final int n = payloads.length;
        if (entryIds.length != n || lengths.length != n) {
            throw new IllegalArgumentException("entryIds, lengths and payloads differ in length");
        }
        final int algo = dm instanceof CRC32CDigestManager ? GpuDigest.CRC32C
                : dm instanceof CRC32DigestManager ? GpuDigest.CRC32 : -1;
        final int frameLen = DigestManager.METADATA_LENGTH + dm.macCodeLength;
        // (the frames buffer below is sized n * frameLen bytes: int arithmetic)
        if (n == 0 || (long) n * frameLen > Integer.MAX_VALUE || algo < 0 || !GpuDigest.isLoaded()) {
            return perEntry(dm, entryIds, lastAddConfirmed, lengths, payloads, masterKey, flags);
        }
        // [32 B header][digest] per entry, back to back, and the u32 digests (direct, little-endian)
        final ByteBuf frames = PooledByteBufAllocator.DEFAULT.directBuffer(n * frameLen);
        final ByteBuf digests = PooledByteBufAllocator.DEFAULT.directBuffer(4 * n);
        try {
            if (!frames.hasMemoryAddress() || !digests.hasMemoryAddress()
                    || GpuDigest.packageBatchArrays(algo, dm.ledgerId, entryIds, lastAddConfirmed, lengths, payloads,
                            frames.memoryAddress(), frameLen, digests.memoryAddress()) != 0) {
                return perEntry(dm, entryIds, lastAddConfirmed, lengths, payloads, masterKey, flags);
            }
            final ReferenceCounted[] out = new ReferenceCounted[n];
            for (int i = 0; i < n; i++) {
                final ByteBuf data = Unpooled.wrappedBuffer(payloads[i], 0, payloads[i].length);
                out[i] = dm.useV2Protocol
                        ? packageV2(allocator, frames, i * frameLen, frameLen, data, masterKey, flags)
                        : ByteBufList.get(Unpooled.buffer(frameLen).writeBytes(frames, i * frameLen, frameLen), data);
            }
            return out;
        } finally {
            frames.release();
            digests.release();
        }
    }

    // computeDigestAndPackageForSendingV2 (DigestManager.java:126-167) with the header and digest computed
    private static ReferenceCounted packageV2(ByteBufAllocator allocator, ByteBuf frames, int at, int frameLen,
                                              ByteBuf data, byte[] masterKey, int flags) {
        final boolean isSmallEntry = data.readableBytes() < BookieProtoEncoding.SMALL_ENTRY_SIZE_THRESHOLD;
        final int headersSize = 4 + BookieProtocol.MASTER_KEY_LENGTH + frameLen;
        final int payloadSize = data.readableBytes();
        final int bufferSize = 4 + headersSize + (isSmallEntry ? payloadSize : 0);
        final ByteBuf buf = allocator.buffer(bufferSize, bufferSize);
        buf.writeInt(headersSize + payloadSize);
        buf.writeInt(BookieProtocol.PacketHeader.toInt(
                BookieProtocol.CURRENT_PROTOCOL_VERSION, BookieProtocol.ADDENTRY, (short) flags));
        buf.writeBytes(masterKey, 0, BookieProtocol.MASTER_KEY_LENGTH);
        buf.writeBytes(frames, at, frameLen);  // [ledgerId, entryId, LAC, length] BE + digest BE
        if (isSmallEntry) {
            buf.writeBytes(data, data.readerIndex(), data.readableBytes());
            data.release();
            return buf;
        }
        return ByteBufList.get(buf, data);
    }

    // the reference's own call, entry by entry (LedgerFragmentReplicator.java:505-511)
    private static ReferenceCounted[] perEntry(DigestManager dm, long[] entryIds, long lastAddConfirmed,
                                               long[] lengths, byte[][] payloads, byte[] masterKey, int flags) {
        final ReferenceCounted[] out = new ReferenceCounted[payloads.length];
        for (int i = 0; i < payloads.length; i++) {
            out[i] = dm.computeDigestAndPackageForSending(entryIds[i], lastAddConfirmed, lengths[i],
                    Unpooled.wrappedBuffer(payloads[i], 0, payloads[i].length), masterKey, flags);
        }
        return out;
    }
}
