// Host-side batch machinery of libbkdigest.so (host_batch.cpp, plain C++):
//  * Pool — the library's host worker threads: the copies into pinned staging of the GPU route, and
//    the CPU route of host-resident batches;
//  * the CPU route of host-resident batches: one CRC / DigestManager verify / package per entry over
//    the pool, with host_crc.cpp's folding. BookKeeper holds these entries in host memory
//    (BatchedReadOp's ByteBufList, $BK/client/BatchedReadOp.java:164-190; PendingAddOp's payloads,
//    $BK/client/PendingAddOp.java:261), where the reference verifies them one crc32c() call at a time
//    ($CN/cpp/crc32c_sse42.cpp:184-217); a PCIe round trip through the GPU only pays where a core
//    cannot keep pace with the link (the measured crossover).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace bkd {
namespace host {

// Cores this process may run on: the affinity mask, capped by a cgroup v2 cpu.max quota (a quota
// of Q cores makes more than Q threads time-slice, not run in parallel).
int usable_cores();

class Pool {
  public:
    static Pool& get();
    // Runs f(part) for part = 0..parts-1 on up to threads() threads (part 0 on the calling thread)
    // and waits for all. One job at a time: a caller that finds the pool busy runs its parts itself.
    void run(int parts, const std::function<void(int)>& f);
    int threads() const;         // the pool's width: BKD_HOST_THREADS, else usable_cores()
    int active() const;          // threads a job may use (bkd_set_host_threads; <= threads())
    void set_active(int n);      // 0 = threads()
    ~Pool();

  private:
    Pool();
    void loop(int part);
    std::vector<std::thread> workers_;
    std::mutex mu_, call_mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int parts_ = 0, pending_ = 0;
    std::atomic<int> active_{0};  // set_active() may run while other threads submit work
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// ---- the CPU route of host-resident batches (semantics of include/bkdigest.h) ----
// The register after folding p[0, len) onto reg; from 4 MiB on in 1 MiB pieces over the pool,
// joined with x^(8 * piece) (one long buffer uses every core, not one).
uint32_t fold(int algo, uint32_t reg, const uint8_t* p, uint64_t len);
// out[i] = resume(seed_i, entry i): entry i at ptrs[i] (list) or base + offsets[i] (indexed).
void crc_list(int algo, const uint8_t* const* ptrs, const uint32_t* lens, uint64_t n, const uint32_t* seeds,
              uint32_t seed_all, uint32_t* out);
void crc_indexed(int algo, const uint8_t* base, const uint64_t* offsets, const uint32_t* lens, uint64_t n,
                 const uint32_t* seeds, uint32_t seed_all, uint32_t* out);
// DigestManager.verifyDigest per frame ($BK/proto/checksum/DigestManager.java:226-283); id_checks:
// 0 ledger + entry ids, 1 ledger id only. Returns the first failing index (n when all verified).
uint64_t verify_frames(int algo, int64_t ledger_id, int64_t first_entry_id, int id_checks,
                       const uint8_t* const* frames, const uint32_t* lens, uint64_t n, int32_t* status);
// DigestManager.computeDigestAndPackageForSending per entry (DigestManager.java:117-181): the 32-byte
// BE header and the digest into frames + i*stride, the digest value into digests[i].
void package_frames(int algo, int64_t ledger_id, const int64_t* entry_ids, const int64_t* lacs,
                    const int64_t* length_fields, const uint8_t* const* payloads, const uint32_t* lens, uint64_t n,
                    uint8_t* frames, uint64_t stride, uint32_t* digests);

}  // namespace host
}  // namespace bkd
