// Host-side cost of device-batch calls from several threads, each on its own HIP stream (VERDICT r02
// item 6: no process-wide lock on the per-call path). For each library given (dlopen), T threads
// (1, 2, 4, 8) each enqueue K small indexed batches (64 x 4 KiB entries: the direct kernel, one
// launch per call) and K uniform batches on their own stream, then sync; reports calls per second
// over all threads and the per-call host time, and checks every digest against the first library's.
// Build: hipcc -O2 -std=c++17 -o tools/thread_scaling tools/thread_scaling.cpp -ldl -lpthread
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

typedef int (*crc_batch_fn)(int, const void*, uint64_t, const uint64_t*, const uint32_t*, uint64_t, const uint32_t*,
                            uint32_t, uint32_t*, void*);
typedef int (*crc_uniform_fn)(int, const void*, uint64_t, uint32_t, uint64_t, const uint32_t*, uint32_t, uint32_t*,
                              void*);
typedef int (*sync_fn)(void*);
typedef int (*fill_fn)(void*, uint64_t, uint64_t, uint64_t, void*);

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s lib.so [lib.so ...]\n", argv[0]);
        return 2;
    }
    const int K = 400;              // calls of each kind per thread
    const uint64_t n = 64, L = 4096;  // 256 KiB base: the indexed call takes the direct kernel
    const int kMaxT = 8;
    uint8_t* base = nullptr;
    uint64_t* offs = nullptr;
    uint32_t* lens = nullptr;
    CK(hipMalloc(&base, n * L));
    CK(hipMalloc(&offs, n * 8));
    CK(hipMalloc(&lens, n * 4));
    std::vector<uint64_t> ho(n);
    std::vector<uint32_t> hl(n);
    for (uint64_t i = 0; i < n; ++i) ho[i] = i * L + (i % 7), hl[i] = (uint32_t)(L - 16 - (i % 5));
    CK(hipMemcpy(offs, ho.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(lens, hl.data(), n * 4, hipMemcpyHostToDevice));
    std::vector<hipStream_t> streams(kMaxT);
    std::vector<uint32_t*> outs(kMaxT);
    for (int t = 0; t < kMaxT; ++t) {
        CK(hipStreamCreateWithFlags(&streams[t], hipStreamNonBlocking));
        CK(hipMalloc(&outs[t], 2 * n * 4));
    }
    std::vector<uint32_t> want;
    for (int a = 1; a < argc; ++a) {
        void* h = dlopen(argv[a], RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            fprintf(stderr, "dlopen %s: %s\n", argv[a], dlerror());
            return 1;
        }
        auto batch = (crc_batch_fn)dlsym(h, "bkd_crc_batch");
        auto uni = (crc_uniform_fn)dlsym(h, "bkd_crc_batch_uniform");
        auto ssync = (sync_fn)dlsym(h, "bkd_stream_sync");
        auto fill = (fill_fn)dlsym(h, "bkd_fill_splitmix64");
        if (fill(base, n * L, 42, 0, nullptr) || hipDeviceSynchronize() != hipSuccess) return 1;
        for (int T : {1, 2, 4, 8, 1}) {
            std::atomic<int> bad{0};
            auto work = [&](int t) {
                for (int k = 0; k < K; ++k) {
                    if (batch(0, base, n * L, offs, lens, n, nullptr, (uint32_t)t, outs[t], streams[t])) bad++;
                    if (uni(0, base, L, (uint32_t)L, n, nullptr, (uint32_t)t, outs[t] + n, streams[t])) bad++;
                }
                if (ssync(streams[t])) bad++;
            };
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t) th.emplace_back(work, t);
            for (auto& x : th) x.join();
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            // digests of every thread's last calls (seed t): equal across libraries
            std::vector<uint32_t> got(2 * n * T);
            for (int t = 0; t < T; ++t) CK(hipMemcpy(got.data() + 2 * n * t, outs[t], 2 * n * 4, hipMemcpyDeviceToHost));
            bool same = true;
            if (want.size() < got.size()) {
                if (a == 1) want = got;
            }
            for (size_t i = 0; i < got.size() && i < want.size(); ++i) same &= got[i] == want[i];
            printf("{\"lib\": \"%s\", \"threads\": %d, \"calls\": %d, \"calls_per_s\": %.0f, \"us_per_call_per_thread\": %.2f, "
                   "\"errors\": %d, \"digests_equal\": %s}\n",
                   argv[a], T, 2 * K * T, 2.0 * K * T / s, s * 1e6 / (2.0 * K), bad.load(), same ? "true" : "false");
            fflush(stdout);
        }
    }
    return 0;
}
