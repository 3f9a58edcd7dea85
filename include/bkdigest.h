/*
 * bkdigest — MI355X-native ledger-entry digest engine (CRC32C / CRC32) for Apache BookKeeper.
 *
 * The drop-in boundary: a C-ABI shared library (bookkeeper_amd/libbkdigest.so) with plain
 * pointers and sizes. Every entry point names the reference interface it replaces
 * (paths relative to /root/reference; $CN = circe-checksum/src/main/circe,
 * $CJ = circe-checksum/src/main/java/com/scurrilous/circe,
 * $BK = bookkeeper-server/src/main/java/org/apache/bookkeeper).
 *
 * Semantics shared by every CRC entry point (identical to the reference):
 *   - `current` / seeds are FINALIZED CRCs: resume(prev, x) = ~raw(~prev, x)
 *     ($CN/cpp/crc32c_sse42.cpp:187,213; $CJ/crc/AbstractIntCrc.java:55-57);
 *   - calculate(x) == resume(0, x) ($CJ/checksum/JniIntHash.java:40-42);
 *   - a zero-length entry returns its seed unchanged ($CN/cpp/crc32c_sse42.cpp:211-213);
 *   - the value is the u32 bit pattern of the Java `int` the reference returns.
 * Algorithms: BKD_CRC32C = CRC-32C (Castagnoli, reflected 0x82F63B78, $CN/cpp/crc32c_sse42.cpp:85),
 *             BKD_CRC32  = CRC-32 (ISO-HDLC, reflected 0xEDB88320, java.util.zip.CRC32 as used by
 *                          $BK/proto/checksum/CRC32DigestManager.java:28-87).
 *
 * Errors are return codes only (the reference native never throws, circe-checksum/pom.xml:87);
 * a human-readable message for the calling thread is available from bkd_last_error().
 * All entry points are thread-safe. Device-resident batch calls are asynchronous on the
 * caller's HIP stream (hipStream_t passed as void*, NULL = the null stream) and run on that
 * stream's device (the calling thread's current device for the null stream); buffers are
 * borrowed only until the stream reaches the end of the call's work.
 * Device-resident batch entry points always run on the GPU (BKD_ERR_NO_DEVICE without one).
 * Host-resident batches (bkd_crc_batch_host, bkd_digest_*_batch_host) take the GPU through pinned
 * staging or the library's own threaded CPU route, by the measured crossover (bkd_set_host_batch_route).
 * The per-call host-buffer resumes (bkd_resume / bkd_resume_host) take the CPU route for
 * buffers up to bkd_get_cpu_route_max() bytes and whenever no device is visible, so the
 * provider never fails for lack of a GPU, as the reference's class-init selection never does
 * ($CJ/checksum/Crc32cIntChecksum.java:28-36).
 */
#ifndef BKDIGEST_H_
#define BKDIGEST_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BKD_ABI_VERSION 6

/* only the entry points below are exported (the library is built with -fvisibility=hidden) */
#ifndef BKD_API
#define BKD_API __attribute__((visibility("default")))
#endif

/* return codes */
#define BKD_OK 0
#define BKD_ERR_INVALID_ARG (-1)
#define BKD_ERR_NO_DEVICE (-2)
#define BKD_ERR_HIP (-3)
#define BKD_ERR_BOUNDS (-4)
#define BKD_ERR_NOMEM (-5)

/* algorithms */
#define BKD_CRC32C 0
#define BKD_CRC32 1

/* verify status codes (one per entry), mirroring DigestManager.verifyDigest's failure modes
 * ($BK/proto/checksum/DigestManager.java:226-283) */
#define BKD_VERIFY_OK 0
#define BKD_VERIFY_TOO_SHORT 1      /* :229-235 (METADATA_LENGTH + macCodeLength) > readableBytes */
#define BKD_VERIFY_DIGEST_MISMATCH 2 /* :241-261 */
#define BKD_VERIFY_LEDGER_MISMATCH 3 /* :267-273 */
#define BKD_VERIFY_ENTRY_MISMATCH 4  /* :275-281 */

BKD_API int bkd_abi_version(void);

/* Number of visible HIP devices (0 when none). Replaces the capability probe
 * Sse42Crc32C.isSupported() -> nativeSupported() ($CJ/crc/Sse42Crc32C.java:31-47,
 * $CN/cpp/crc32c_sse42_jni.cpp:20-24). */
BKD_API int bkd_device_count(void);

/* Uploads the CRC fold tables to `device` (idempotent, thread-safe). Replaces the
 * allocConfig chunk/shift-table construction ($CN/cpp/crc32c_sse42_jni.cpp:50-72,
 * $CN/cpp/crc32c_sse42.cpp:74-90). Optional: every call below initialises lazily. */
BKD_API int bkd_init(int device);

/* Message describing the last failure on the calling thread ("" if none). */
BKD_API const char* bkd_last_error(void);

/* ---- device-resident batches: THE HOT PATH ---------------------------------------------
 * One CRC per entry, all entries in one launch. Entry i is the byte range
 *   uniform:  d_base + i*stride, entry_len bytes
 *   indexed:  d_base + d_offsets[i], d_lengths[i] bytes (any alignment, any order)
 * seeded with d_seeds[i] (finalized CRC) or, when d_seeds is NULL, with seed_all.
 * d_out[i] receives the finalized CRC. All pointers are device pointers of the current
 * HIP device. Replaces N calls of Sse42Crc32C.resume(int,long,long) -> nativeUnsafe
 * ($CJ/crc/Sse42Crc32C.java:105-107, $CN/cpp/crc32c_sse42_jni.cpp:44-48) which the
 * reference makes once per entry from DigestManager.update ($BK/proto/checksum/DigestManager.java:62-72).
 * The indexed form checks offset+length <= base_size for every entry on the device and returns
 * BKD_ERR_BOUNDS from the NEXT synchronous call on this stream if any entry was out of range
 * (those entries get out = 0 and are not read). */
BKD_API int bkd_crc_batch_uniform(int algo, const void* d_base, uint64_t stride, uint32_t entry_len, uint64_t n,
                          const uint32_t* d_seeds, uint32_t seed_all, uint32_t* d_out, void* stream);

BKD_API int bkd_crc_batch(int algo, const void* d_base, uint64_t base_size, const uint64_t* d_offsets,
                  const uint32_t* d_lengths, uint64_t n, const uint32_t* d_seeds, uint32_t seed_all,
                  uint32_t* d_out, void* stream);

/* Composite entries (a Netty CompositeByteBuf / ByteBufList visited leaf by leaf): entry i is the
 * concatenation, in order, of segments d_seg_first[i] .. d_seg_first[i+1]-1, segment k being the
 * byte range d_base + d_seg_offsets[k], d_seg_lengths[k] bytes; empty segments are skipped. out[i] =
 * resume(seed_i, concatenation) — the digest DigestManager.update chains over ByteBufVisitor's
 * leaves ($BK/proto/checksum/DigestManager.java:62-72,380-392, $BK/util/ByteBufVisitor.java:72-191),
 * without copying the pieces together. d_seg_first holds n + 1 non-decreasing indices
 * (d_seg_first[n] = nseg). Segments take the indexed path (bounds reported as for bkd_crc_batch);
 * one GF(2) combine per segment joins them. Device pointers; asynchronous on `stream`. */
BKD_API int bkd_crc_batch_segments(int algo, const void* d_base, uint64_t base_size, const uint64_t* d_seg_offsets,
                           const uint32_t* d_seg_lengths, uint64_t nseg, const uint64_t* d_seg_first, uint64_t n,
                           const uint32_t* d_seeds, uint32_t seed_all, uint32_t* d_out, void* stream);

/* Waits for `stream` and reports (BKD_ERR_BOUNDS) any bounds violation recorded by the indexed
 * batches enqueued on THIS stream since its previous bkd_stream_sync; the flag is per stream, so
 * concurrent callers on other streams neither see nor clear it. */
BKD_API int bkd_stream_sync(void* stream);

/* Waits for `stream`, then frees the scratch the library keeps for it (plan arena, bounds flag,
 * run words) and forgets the stream; returns BKD_ERR_BOUNDS as bkd_stream_sync would. Call it
 * before hipStreamDestroy on a stream that ran indexed batches, with no other call on that stream
 * in progress; a later call on the same handle starts afresh. The reference has no per-stream state
 * (its natives are stateless, $CN/cpp/crc32c_sse42_jni.cpp:26-48): this is the lifetime rule a
 * long-lived caller that creates and drops streams needs so that their scratch does not pile up. */
BKD_API int bkd_stream_release(void* stream);

/* ---- host-resident batches (the end-to-end path: Netty buffers in, digests out) -------
 * Synchronous. Same semantics as bkd_crc_batch (bounds checked on the host: BKD_ERR_BOUNDS before
 * any work). GPU route: the payload goes through pinned staging buffers with hipMemcpyAsync
 * (double-buffered H2D -> kernel -> D2H). CPU route: one fold per entry on the library's host
 * threads (host_batch.cpp). */
BKD_API int bkd_crc_batch_host(int algo, const void* h_base, uint64_t base_size, const uint64_t* h_offsets,
                       const uint32_t* h_lengths, uint64_t n, const uint32_t* h_seeds, uint32_t seed_all,
                       uint32_t* h_out);
/* Route of the host-resident batches: 0 = automatic (the CPU route when at least the measured
 * crossover's number of host threads is available: a batch that starts in host memory is bound by
 * PCIe and the host gather through the GPU; the CPU route also whenever no device is
 * visible), 1 = always the CPU route, 2 = always the GPU (BKD_ERR_NO_DEVICE without one).
 * get: the route the next host-resident batch takes (1 or 2). The reference verifies these entries
 * one crc32c() call at a time on its caller's thread ($BK/client/BatchedReadOp.java:164-190). */
BKD_API int bkd_set_host_batch_route(int route);
BKD_API int bkd_get_host_batch_route(void);
/* Host threads the CPU route and the staging copies may use (0 = all of the pool: BKD_HOST_THREADS,
 * else the cores this process may run on, capped by a cgroup CPU quota). */
BKD_API int bkd_set_host_threads(int threads);
BKD_API int bkd_get_host_threads(void);
/* Frees the idle pinned staging sets of the GPU route (host and device memory, streams); sets in use
 * by a running call are kept. A later host-resident batch through the GPU creates them again. */
BKD_API int bkd_host_release(void);

/* ---- per-call drop-in (IntHash.resume) ---------------------------------------------------
 * resume(current, ptr, len) for ONE buffer, synchronous. Replaces Sse42Crc32C.nativeUnsafe /
 * nativeArray / nativeDirectBuffer ($CN/cpp/crc32c_sse42_jni.cpp:26-48) and IntHash.resume
 * ($CJ/checksum/IntHash.java:28-32). len == 0 returns `current` (crc32c_sse42.cpp:211-213).
 *
 * bkd_resume_host: a host buffer. Up to bkd_get_cpu_route_max() bytes, or with no device, the
 *   CPU route (PCLMUL folding / SSE4.2 crc32, host_crc.cpp); above, the GPU through pinned staging
 *   (the CPU route again if the device fails: init, allocation or copy errors never surface here).
 * bkd_resume_device: a device buffer, on the caller's `stream` (ordered after the work that
 *   produced the bytes), synchronous. One launch per call: batch callers use bkd_crc_batch.
 * bkd_resume: either; the pointer kind is looked up (hipPointerGetAttributes), and a device
 *   buffer runs on the null stream of the device that holds it, which orders it after work on
 *   that device's blocking streams.
 * bkd_cpu_resume: always the CPU route (no device needed). */
BKD_API int bkd_resume(int algo, uint32_t current, const void* ptr, uint64_t len, uint32_t* out);
BKD_API int bkd_resume_host(int algo, uint32_t current, const void* h_ptr, uint64_t len, uint32_t* out);
BKD_API int bkd_resume_device(int algo, uint32_t current, const void* d_ptr, uint64_t len, void* stream,
                              uint32_t* out);
BKD_API int bkd_cpu_resume(int algo, uint32_t current, const void* h_ptr, uint64_t len, uint32_t* out);
/* Host buffers up to this many bytes take the CPU route in bkd_resume / bkd_resume_host
 * (0 = always the GPU when one is visible). Default by CPU, from profiles/r02_call_latency.log:
 * 64 MiB where the AVX-512 VPCLMULQDQ fold runs (a core keeps pace with PCIe), else 4 MiB. */
BKD_API int bkd_set_cpu_route_max(uint64_t bytes);
BKD_API uint64_t bkd_get_cpu_route_max(void);
/* The CPU route's implementation on this host: "vpclmul512+pclmul+sse4.2", "pclmul+sse4.2", "pclmul"
 * or "slice8". */
BKD_API const char* bkd_cpu_impl(void);

/* ---- circe-checksum compatibility (the Sse42Crc32C natives, $CN/cpp/crc32c_sse42_jni.cpp) -----
 * Backing for a drop-in libcirce-checksum.so (native/jni/bkdigest_jni.c). The chunk-word config
 * only tunes the reference's SSE4.2 loop; results never depend on it, so it is validated and
 * kept as an opaque handle. alloc: 0 unless len >= 1, every word >= 4 and the words strictly
 * decrease (:50-72); free: releases a non-zero handle (:74-78). supported: 1 (the library
 * always has a route: GPU or CPU), replacing nativeSupported (:20-24). */
BKD_API int bkd_circe_supported(void);
BKD_API int64_t bkd_circe_alloc_config(const int32_t* chunk_words, int32_t len);
BKD_API void bkd_circe_free_config(int64_t config);

/* ---- DigestManager batch framing (§8f rows 1-2) --------------------------------------
 * Package: for entry i with payload d_payload + d_offsets[i], d_lengths[i] bytes, write the
 * 32-byte big-endian header [ledger_id, entry_ids[i], lacs[i], lengths_field[i]]
 * ($BK/proto/checksum/DigestManager.java:146-149) followed by the digest
 * (CRC32C: 4 B BE int, CRC32CDigestManager.java:44-46; CRC32: 8 B BE long zero-extended,
 * CRC32DigestManager.java:60-63) into d_frames + i*frame_stride (frame_stride >= 32 + mac).
 * digest = update(update(0, header), payload) (DigestManager.java:152-153, :177-178).
 * Device pointers; asynchronous on `stream`. An out-of-range payload entry gets digest 0 and is
 * reported by the next bkd_stream_sync on `stream` (BKD_ERR_BOUNDS). */
BKD_API int bkd_digest_package_batch(int algo, int64_t ledger_id, const int64_t* d_entry_ids, const int64_t* d_lacs,
                             const int64_t* d_length_fields, const void* d_payload, uint64_t payload_size,
                             const uint64_t* d_offsets, const uint32_t* d_lengths, uint64_t n,
                             void* d_frames, uint64_t frame_stride, uint32_t* d_digests, void* stream);

/* Verify: entry i is a framed buffer [32 B header][mac][payload] at d_framed + d_offsets[i],
 * d_lengths[i] bytes. Writes a BKD_VERIFY_* code per entry to d_status and the index of the first
 * failing entry (n if none) to *d_first_bad — the verified-prefix rule of BatchedReadOp
 * ($BK/client/BatchedReadOp.java:164-190). expected entry id for entry i = first_entry_id + i
 * (DigestManager.verifyDigestAndReturnData(entryId, buf), :333-338); skip_entry_check mirrors
 * verifyDigest(buf) with skipEntryIdCheck (:206-208). Device pointers; asynchronous. */
BKD_API int bkd_digest_verify_batch(int algo, int64_t ledger_id, int64_t first_entry_id, int skip_entry_check,
                            const void* d_framed, uint64_t framed_size, const uint64_t* d_offsets,
                            const uint32_t* d_lengths, uint64_t n, int32_t* d_status, uint64_t* d_first_bad,
                            void* stream);

/* Host-resident framed batches (SURVEY §8f rows 1-2 with the entries in host memory, BASELINE
 * config 5): entry i is its own host buffer h_frames[i] / h_payloads[i] of h_lengths[i] bytes,
 * as BatchedReadOp's ByteBufList ($BK/client/BatchedReadOp.java:164-190) and PendingAddOp's
 * payloads ($BK/client/PendingAddOp.java:261) hold them. Route as bkd_crc_batch_host: GPU = the
 * library gathers them into pinned staging (segments of <= 64 MiB, double-buffered, host copies on
 * a thread pool), copies H2D, runs the device sequence of the device-resident call and copies the
 * results back; CPU = DigestManager's per-entry arithmetic on the host threads. Synchronous.
 * verify: h_status[i] and *h_first_bad as bkd_digest_verify_batch (n if all verified).
 * package: writes frame i's [32 B header][digest] to h_frames + i*frame_stride
 * (32 + mac <= frame_stride <= 4096) and the digest value to h_digests[i]. */
BKD_API int bkd_digest_verify_batch_host(int algo, int64_t ledger_id, int64_t first_entry_id, int skip_entry_check,
                                         const void* const* h_frames, const uint32_t* h_lengths, uint64_t n,
                                         int32_t* h_status, uint64_t* h_first_bad);
BKD_API int bkd_digest_package_batch_host(int algo, int64_t ledger_id, const int64_t* h_entry_ids,
                                          const int64_t* h_lacs, const int64_t* h_length_fields,
                                          const void* const* h_payloads, const uint32_t* h_lengths, uint64_t n,
                                          void* h_frames, uint64_t frame_stride, uint32_t* h_digests);

/* ---- bookie-side entry-log scrub (§8f row 4) ------------------------------------------
 * An entry log is a 1024-byte file header (LOGFILE_HEADER_SIZE, DefaultEntryLogger.java:256)
 * followed by records [int32 BE size][entry bytes], an entry starting with its BE ledger id.
 *
 * Index: walks the records of a HOST buffer from byte `start` exactly like
 * DefaultEntryLogger.scanEntryLog ($BK/bookie/DefaultEntryLogger.java:995-1060): size <= 0 is
 * padding (advance one byte), ledger id -1 (INVALID_LID) is a ledgers-map record (skipped), a
 * short read of the 12-byte [size, ledgerId] header or of the entry ends the scan. Writes each
 * entry's offset (first byte after the size field), length and ledger id; *h_end = the position
 * where the walk stopped. BKD_ERR_BOUNDS when more than `capacity` entries are found.
 * Host-only control logic: it reads 12 bytes per record and computes no digest. */
BKD_API int bkd_entrylog_index(const void* h_log, uint64_t log_size, uint64_t start, uint64_t* h_offsets,
                       uint32_t* h_lengths, int64_t* h_ledger_ids, uint64_t capacity, uint64_t* h_count,
                       uint64_t* h_end);

/* Verify: the digest of every indexed entry of a DEVICE-resident log, as
 * DigestManager.verifyDigest would (DigestManager.java:226-283: CRC of [0,32) || [32+mac, len)
 * against the stored digest at 32) without ledger/entry id checks (the ledger id comes from the
 * entry itself). Status codes as bkd_digest_verify_batch (0 ok, 1 too short, 2 digest mismatch);
 * *d_first_bad = first failing index or n. One digest type per call (the ledger's, from its
 * metadata). Asynchronous on `stream`; ragged batches go through the chunked plan. */
BKD_API int bkd_entrylog_verify(int algo, const void* d_log, uint64_t log_size, const uint64_t* d_offsets,
                        const uint32_t* d_lengths, uint64_t n, int32_t* d_status, uint64_t* d_first_bad,
                        void* stream);

/* ---- synthetic input + test helpers --------------------------------------------------- */

/* Fills nbytes of device memory with the little-endian splitmix64 stream
 * word_i = mix(seed + (first_word + i + 1) * 0x9E3779B97F4A7C15) (SURVEY.md §8d input definition). */
BKD_API int bkd_fill_splitmix64(void* d_dst, uint64_t nbytes, uint64_t seed, uint64_t first_word, void* stream);

/* Host-only (no GPU needed): the compact fold-table image the kernels load into LDS for
 * `algo` and a group width of `lanes` (4, 8, 16, 32 or 64); returns words written or <0.
 * Layout documented in DESIGN.md §3. */
BKD_API int64_t bkd_host_tables(int algo, int lanes, uint32_t* out, uint64_t out_words);

/* Host-only: GF(2) product a*b mod P in the reflected representation, and x^(8*nbytes) mod P. */
BKD_API uint32_t bkd_host_gf_mul(int algo, uint32_t a, uint32_t b);
BKD_API uint32_t bkd_host_xpow8n(int algo, uint64_t nbytes);

/* Tuning: lanes per entry group (0 = automatic, else 1/4/8/16/32/64); prefetch is fixed at build. */
BKD_API int bkd_set_group_lanes(int lanes);
/* Indexed-batch strategy: 0 = automatic (one entry per lane group when the base buffer is <= 256 KiB,
 * else the chunked plan with the short-entry class when the buffer holds at most 1 KiB per entry),
 * 1 = one entry per lane group, 2 = always the chunked plan. Any other value (the removed stream
 * route was mode 3) returns BKD_ERR_INVALID_ARG. */
BKD_API int bkd_set_plan_mode(int mode);
/* Chunked-plan geometry: lanes per group (4, 8, 16, 32 or 64), steps per full chunk (chunk = 16 * lanes *
 * steps bytes, <= 32 KiB) and the head-merge threshold in bytes (a head chunk shorter than this
 * joins its neighbour; >= 16). Default 8, 32, 16 (4 KiB chunks; tools/tune_plan.py). */
BKD_API int bkd_set_plan_geometry(int lanes, int steps_per_chunk, int merge_bytes);
/* Short-entry class of indexed batches that take the plan: entries of <= max_bytes (16..512; 0 = no
 * class) run in their own launch, loading the next entries while folding the current one (4-lane
 * groups up to 192 B, 8-lane groups above), and skip the plan's count/emit/chunk/combine work
 * (DESIGN.md §3). Used when the base buffer holds at most bkd_set_short_class_mean() bytes per entry
 * (default 1 KiB: short entries dominate). Default 192. */
BKD_API int bkd_set_plan_small(uint32_t max_bytes);
/* The short-entry class's gate: base-buffer bytes per entry at most this (default 1024; UINT64_MAX:
 * whenever a class bound is set). */
BKD_API int bkd_set_short_class_mean(uint64_t max_bytes_per_entry);
/* Entries of the plan shorter than `bytes` (16..64, default 16) skip the chunk kernel: the
 * combine kernel computes each with one thread (slice-by-16 over its 16-byte windows). */
BKD_API int bkd_set_plan_serial(uint32_t bytes);
/* Register double-buffer depth of the plan's chunk kernel (2, 4 or 8 loads per lane). */
BKD_API int bkd_set_plan_prefetch(int loads_in_flight);
/* Fold schedule of the one-entry-per-group kernels (uniform, direct indexed, package payloads):
 * 0 = chosen per launch from the shader clock the kernel measures (the low-clock schedule below
 * 2 GHz), 1 = always the compiler's schedule, 2 = always the low-clock schedule
 * (16 table lookups in flight per step). Results are identical; only the speed differs. */
BKD_API int bkd_set_fold_schedule(int schedule);
BKD_API int bkd_get_group_lanes(int algo, uint64_t mean_len);

#ifdef __cplusplus
}
#endif

#endif /* BKDIGEST_H_ */
