/*
 * TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.
 *
 * CPU oracle for the BookKeeper ledger-entry digest path (CRC32C / CRC32).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this; the product (bookkeeper_amd/libbkdigest.so) never links or calls it.
 *
 * It is a plain-C restatement of the reference's CRC semantics:
 *   - table generation          ReflectedIntCrc.java:26-36   (circe-checksum/src/main/java/com/scurrilous/circe/crc/)
 *   - byte loop                 ReflectedIntCrc.java:44-48
 *   - resume/initial semantics  AbstractIntCrc.java:50-57  (init = xorOut = ~0, "current" is a finalized CRC)
 *   - native equivalence        crc32c_sse42.cpp:184-217 (~init on entry, ~crc on exit, len==0 -> init)
 *   - parameters                CrcParameters.java:167-180 (CRC32 0x04c11db7, CRC32C 0x1edc6f41, reflected)
 *   - DigestManager framing     DigestManager.java:146-153 (V2), :169-181 (V3), :226-283 (verify)
 *                               CRC32CDigestManager.java:44-46 (4-byte BE int digest)
 *                               CRC32DigestManager.java:60-63 + DirectMemoryCRC32Digest.java:39-43 (8-byte BE long)
 * Pinned by tests/test_oracle_golden.py against the reference's own known-answer
 * vectors (CRCTest.java:117-135, ChecksumTest.java:36-92) and against outputs of the
 * reference native crc32c() compiled from /root/reference (oracle/_ref, tests/golden/).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define ORACLE_CRC32C 0
#define ORACLE_CRC32 1

/* Reflected polynomials: Integer.reverse(poly) as ReflectedIntCrc.java:29 does. */
static const uint32_t POLY_REFLECTED[2] = {0x82F63B78u, 0xEDB88320u};

static uint32_t TABLES[2][256];
static int TABLES_READY = 0;

/* ReflectedIntCrc.java:30-35 */
static void build_tables(void) {
    if (TABLES_READY) return;
    for (int a = 0; a < 2; ++a) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t crc = i;
            for (int j = 0; j < 8; ++j) crc = (crc & 1u) ? (crc >> 1) ^ POLY_REFLECTED[a] : crc >> 1;
            TABLES[a][i] = crc;
        }
    }
    TABLES_READY = 1;
}

void oracle_table(int algo, uint32_t* out256) {
    build_tables();
    memcpy(out256, TABLES[algo & 1], sizeof(TABLES[0]));
}

/* ReflectedIntCrc.java:44-48 (raw register loop, no pre/post inversion). */
uint32_t oracle_resume_raw(int algo, uint32_t reg, const uint8_t* p, uint64_t len) {
    build_tables();
    const uint32_t* t = TABLES[algo & 1];
    for (uint64_t i = 0; i < len; ++i) reg = t[(reg ^ p[i]) & 0xffu] ^ (reg >> 8);
    return reg;
}

/* AbstractIntCrc.java:55-57 — resumeRaw(current ^ xorOut) ^ xorOut, xorOut = ~0.
 * Identical to crc32c_sse42.cpp:187,213 (~init in, ~crc out); len == 0 returns current. */
uint32_t oracle_resume(int algo, uint32_t current, const uint8_t* p, uint64_t len) {
    return ~oracle_resume_raw(algo, ~current, p, len);
}

/* Independent bit-at-a-time definition (no table) used to cross-check the table. */
uint32_t oracle_resume_bitwise(int algo, uint32_t current, const uint8_t* p, uint64_t len) {
    uint32_t poly = POLY_REFLECTED[algo & 1];
    uint32_t reg = ~current;
    for (uint64_t i = 0; i < len; ++i) {
        reg ^= p[i];
        for (int b = 0; b < 8; ++b) reg = (reg >> 1) ^ ((reg & 1u) ? poly : 0u);
    }
    return ~reg;
}

/* One CRC per entry: out[i] = resume(seed_i, base + off[i], len[i]).
 * seeds == NULL means every entry resumes from `seed_all` (calculate() == resume(0, .)). */
void oracle_batch(int algo, const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                  uint64_t n, const uint32_t* seeds, uint32_t seed_all, uint32_t* out) {
    for (uint64_t i = 0; i < n; ++i)
        out[i] = oracle_resume(algo, seeds ? seeds[i] : seed_all, base + offsets[i], lengths[i]);
}

/* Uniform batch: entry i at base + i*stride, len bytes each. */
void oracle_uniform(int algo, const uint8_t* base, uint64_t stride, uint32_t len, uint64_t n,
                    uint32_t seed_all, uint32_t* out) {
    for (uint64_t i = 0; i < n; ++i) out[i] = oracle_resume(algo, seed_all, base + i * stride, len);
}

/* ---- GF(2) helpers (reflected representation: bit 31 = x^0, bit 0 = x^31). ---- */

static uint32_t mulx(int algo, uint32_t r) { return (r >> 1) ^ ((r & 1u) ? POLY_REFLECTED[algo & 1] : 0u); }

uint32_t oracle_gf_mul(int algo, uint32_t a, uint32_t b) {
    uint32_t p = 0, cur = b;
    for (int k = 0; k < 32; ++k) {
        if (a & (0x80000000u >> k)) p ^= cur;
        cur = mulx(algo, cur);
    }
    return p;
}

/* x^(8*nbytes) mod P by square-and-multiply. */
uint32_t oracle_xpow8n(int algo, uint64_t nbytes) {
    uint32_t result = 0x80000000u; /* x^0 */
    uint32_t sq = 0x80000000u >> 8; /* x^8 */
    while (nbytes) {
        if (nbytes & 1) result = oracle_gf_mul(algo, result, sq);
        sq = oracle_gf_mul(algo, sq, sq);
        nbytes >>= 1;
    }
    return result;
}

/* crc(A || B) from crc(A), crc(B), |B| — the property the shift tables of
 * crc32c_sse42.cpp:74-90 (chunk_config::make_shift_table) exist to exploit. */
uint32_t oracle_combine(int algo, uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    /* reg(r, A||B) = reg(r, A)*x^(8|B|) ^ reg(0, B) and reg(0, B) = ~crc_b ^ (~0)*x^(8|B|):
     * the complements cancel, leaving crc_a*x^(8|B|) ^ crc_b. */
    return oracle_gf_mul(algo, crc_a, oracle_xpow8n(algo, len_b)) ^ crc_b;
}

/* ---- DigestManager framing (DigestManager.java:146-153, :172-178). ---- */

static void put_be64(uint8_t* p, uint64_t v) {
    for (int i = 7; i >= 0; --i) { p[i] = (uint8_t)v; v >>= 8; }
}

/* Writes the 32-byte metadata header [ledgerId, entryId, lastAddConfirmed, length] (big-endian,
 * DigestManager.java:146-149) to hdr and returns the 32-bit digest
 * digest = update(update(0, header32), payload)  (DigestManager.java:152-153 / :177-178). */
uint32_t oracle_digest_entry(int algo, int64_t ledger_id, int64_t entry_id, int64_t lac, int64_t length,
                             const uint8_t* payload, uint64_t plen, uint8_t* hdr32) {
    uint8_t h[32];
    put_be64(h + 0, (uint64_t)ledger_id);
    put_be64(h + 8, (uint64_t)entry_id);
    put_be64(h + 16, (uint64_t)lac);
    put_be64(h + 24, (uint64_t)length);
    if (hdr32) memcpy(hdr32, h, 32);
    uint32_t d = oracle_resume(algo, 0, h, 32);
    return oracle_resume(algo, d, payload, plen);
}

/* Digest bytes as written on the wire: CRC32C -> writeInt (4 B BE, CRC32CDigestManager.java:44-46);
 * CRC32 -> writeLong(value & 0xffffffffL) (8 B BE, CRC32DigestManager.java:60-63,
 * DirectMemoryCRC32Digest.java:39-43). Returns the number of bytes written. */
int oracle_digest_bytes(int algo, uint32_t digest, uint8_t* out) {
    if (algo == ORACLE_CRC32C) {
        out[0] = (uint8_t)(digest >> 24); out[1] = (uint8_t)(digest >> 16);
        out[2] = (uint8_t)(digest >> 8); out[3] = (uint8_t)digest;
        return 4;
    }
    put_be64(out, (uint64_t)digest);
    return 8;
}

/* verifyDigest (DigestManager.java:226-283) on one framed entry
 * [32 B header][mac][payload]: returns 0 when the digest matches and the ledger/entry ids
 * match, 1 = too short, 2 = digest mismatch, 3 = ledger id mismatch, 4 = entry id mismatch. */
int oracle_verify_entry(int algo, const uint8_t* framed, uint64_t flen, int64_t ledger_id,
                        int64_t entry_id, int skip_entry_check) {
    uint64_t mac = algo == ORACLE_CRC32C ? 4 : 8;
    if (32 + mac > flen) return 1;
    uint32_t d = oracle_resume(algo, 0, framed, 32);
    d = oracle_resume(algo, d, framed + 32 + mac, flen - 32 - mac);
    uint8_t expect[8];
    oracle_digest_bytes(algo, d, expect);
    if (memcmp(expect, framed + 32, mac) != 0) return 2;
    uint64_t lid = 0, eid = 0;
    for (int i = 0; i < 8; ++i) { lid = (lid << 8) | framed[i]; eid = (eid << 8) | framed[8 + i]; }
    if ((int64_t)lid != ledger_id) return 3;
    if (!skip_entry_check && (int64_t)eid != entry_id) return 4;
    return 0;
}

/* ---- Synthetic input definition shared with the GPU generator. ----
 * Little-endian splitmix64 stream: word i = mix(seed + (i+1)*0x9E3779B97F4A7C15). */
static uint64_t splitmix_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_fill_splitmix64(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t first_word) {
    uint64_t nw = nbytes / 8;
    for (uint64_t i = 0; i < nw; ++i) {
        uint64_t v = splitmix_mix(seed + (first_word + i + 1) * 0x9E3779B97F4A7C15ull);
        memcpy(dst + 8 * i, &v, 8);
    }
    uint64_t rem = nbytes & 7;
    if (rem) {
        uint64_t v = splitmix_mix(seed + (first_word + nw + 1) * 0x9E3779B97F4A7C15ull);
        memcpy(dst + 8 * nw, &v, rem);
    }
}

/* ---- Entry-log record walk (DefaultEntryLogger.scanEntryLog, DefaultEntryLogger.java:995-1060). ----
 * From `start` (LOGFILE_HEADER_SIZE = 1024, :256): read [int32 BE size][int64 BE ledgerId]
 * (a short read of these 12 bytes ends the scan, :1020-1023); size <= 0 is padding -> pos++
 * (:1027-1031); ledgerId == INVALID_LID (-1) -> skip the record (:1037-1041); a short read of the
 * entry ends the scan (:1046-1054); else the entry is [pos+4, pos+4+size). Returns the count,
 * writes at most `cap` entries and the final position to *end. */
uint64_t oracle_entrylog_scan(const uint8_t* log, uint64_t size, uint64_t start, uint64_t* offs,
                              uint32_t* lens, int64_t* lids, uint64_t cap, uint64_t* end) {
    uint64_t pos = start, n = 0;
    while (pos < size) {
        if (size - pos < 12) break;
        int32_t esz = (int32_t)(((uint32_t)log[pos] << 24) | ((uint32_t)log[pos + 1] << 16) |
                                ((uint32_t)log[pos + 2] << 8) | (uint32_t)log[pos + 3]);
        if (esz <= 0) { pos++; continue; }
        uint64_t lid = 0;
        for (int i = 0; i < 8; ++i) lid = (lid << 8) | log[pos + 4 + i];
        pos += 4;
        if ((int64_t)lid == -1) { pos += (uint64_t)esz; continue; }
        if ((uint64_t)esz > size - pos) break;
        if (n < cap) { offs[n] = pos; lens[n] = (uint32_t)esz; lids[n] = (int64_t)lid; }
        n++;
        pos += (uint64_t)esz;
    }
    if (end) *end = pos;
    return n;
}
