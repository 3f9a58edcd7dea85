/*
 * The batched verify hook for BatchedReadOp (bookkeeper-server/.../client/BatchedReadOp.java:164-190).
 * The reference verifies the entries of a batched read one by one and keeps the verified prefix:
 *
 *     for (int i = 0; i < bufList.size(); i++) {
 *         try { lh.macManager.verifyDigestAndReturnData(eId + i, buffer); verifiedEntries++; }
 *         catch (BKException.BKDigestMatchException e) { ...; break; }
 *     }
 *
 * With this class that loop becomes one call,
 *
 *     int verifiedEntries = GpuBatchVerifier.verifiedPrefix(lh.macManager, eId, bufList);
 *
 * followed by the reference's own handling of verifiedEntries (re-read from another replica when it
 * is 0, the read-op digest-mismatch counter when it is below bufList.size()). The whole ByteBufList
 * goes to libbkdigest's bkd_digest_verify_batch_host (header CRC, payload CRC, digest compare, ledger
 * and entry id checks — DigestManager.java:226-283 — per entry, the verified prefix returned). CRC32C
 * and CRC32 digest managers with direct (memory-address) buffers whose readerIndex is 0 take that path;
 * anything else (MAC or dummy digests, heap or composite buffers, a buffer already partly read, no
 * library, a library error) runs the reference's loop unchanged.
 *
 * The buffers are left exactly as the reference's loop leaves them. verifyDigest CRCs the absolute
 * ranges [0, 32) and [32 + macCodeLength, readableBytes()) of memoryAddress() (DigestManager.java:
 * 62-64,236-239) and reads the ledger and entry ids at readerIndex (:264-265); with readerIndex 0 that
 * is exactly the frame [memoryAddress(), memoryAddress() + readableBytes()) the library verifies, so
 * the GPU path is taken only then. verifyDigestAndReturnData then sets readerIndex(METADATA_LENGTH +
 * macCodeLength) on every buffer it verified (:336), which BatchedReadOp hands to
 * LedgerEntryImpl.setEntryBuf (BatchedReadOp.java:193-201) so the application sees only the payload;
 * the GPU path does the same for the verified prefix. (Buffers past the prefix are released by
 * BatchedReadOp, :203-206, so their reader index does not matter.)
 *
 * It lives in DigestManager's package for the manager's ledgerId and macCodeLength. Not compiled in
 * this repository's image (no JDK): tests/test_java_sources.py resolves its imports against the
 * reference and checks the two rules above in its source.
 */
package org.apache.bookkeeper.proto.checksum;

import com.scurrilous.circe.checksum.GpuDigest;
import io.netty.buffer.ByteBuf;
import io.netty.buffer.PooledByteBufAllocator;
import org.apache.bookkeeper.client.BKException;
import org.apache.bookkeeper.util.ByteBufList;

public final class GpuBatchVerifier {

    private GpuBatchVerifier() {
    }

    /** How many leading entries of bufList (entry ids firstEntryId, firstEntryId + 1, ...) verify. */
    public static int verifiedPrefix(DigestManager dm, long firstEntryId, ByteBufList bufList) {
        final int n = bufList.size();
        final int algo = dm instanceof CRC32CDigestManager ? GpuDigest.CRC32C
                : dm instanceof CRC32DigestManager ? GpuDigest.CRC32 : -1;
        // (the per-entry index buffers below are sized 8 * n bytes: int arithmetic)
        boolean direct = n > 0 && n <= Integer.MAX_VALUE / 8 && algo >= 0 && GpuDigest.isLoaded();
        for (int i = 0; direct && i < n; i++) {
            final ByteBuf b = bufList.getBuffer(i);
            // the reference's absolute addressing equals the frame [memoryAddress(), + readableBytes())
            // only when nothing of the buffer has been read yet
            direct = b.hasMemoryAddress() && b.readerIndex() == 0;
        }
        if (!direct) {
            return serialPrefix(dm, firstEntryId, bufList);
        }
        // frame addresses (u64), lengths (u32) and per-entry status (i32), little-endian direct buffers
        final ByteBuf addrs = PooledByteBufAllocator.DEFAULT.directBuffer(8 * n);
        final ByteBuf lens = PooledByteBufAllocator.DEFAULT.directBuffer(4 * n);
        final ByteBuf status = PooledByteBufAllocator.DEFAULT.directBuffer(4 * n);
        try {
            if (!addrs.hasMemoryAddress() || !lens.hasMemoryAddress() || !status.hasMemoryAddress()) {
                return serialPrefix(dm, firstEntryId, bufList);
            }
            for (int i = 0; i < n; i++) {
                final ByteBuf b = bufList.getBuffer(i);
                addrs.writeLongLE(b.memoryAddress());  // readerIndex() == 0 (checked above)
                lens.writeIntLE(b.readableBytes());
            }
            final long rc = GpuDigest.verifyBatch(algo, dm.ledgerId, firstEntryId, false, addrs.memoryAddress(),
                    lens.memoryAddress(), n, status.memoryAddress());
            if (rc < 0) {
                return serialPrefix(dm, firstEntryId, bufList);  // no buffer was touched
            }
            final int verified = (int) rc;
            for (int i = 0; i < verified; i++) {
                // verifyDigestAndReturnData's own side effect (DigestManager.java:336)
                bufList.getBuffer(i).readerIndex(DigestManager.METADATA_LENGTH + dm.macCodeLength);
            }
            return verified;
        } finally {
            addrs.release();
            lens.release();
            status.release();
        }
    }

    // BatchedReadOp.java:175-189 without its logging and retry: the verified prefix
    private static int serialPrefix(DigestManager dm, long firstEntryId, ByteBufList bufList) {
        int verified = 0;
        for (int i = 0; i < bufList.size(); i++) {
            try {
                dm.verifyDigestAndReturnData(firstEntryId + i, bufList.getBuffer(i));
                verified++;
            } catch (BKException.BKDigestMatchException e) {
                break;
            }
        }
        return verified;
    }
}
