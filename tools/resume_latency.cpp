// Per-call resume latency through the C-ABI, no Python in the loop (profiles/r02_call_latency.log).
// Routes: cpu = bkd_cpu_resume; host_auto = bkd_resume_host with the default CPU-route threshold;
// host_gpu = bkd_resume_host with the threshold at 0 and the host batch route forced to the GPU
// (pinned staging + kernel), for pageable and pinned sources; cpu takes the host pool from 4 MiB on; device = bkd_resume_device on a device buffer; auto = bkd_resume (pointer lookup).
// Build: hipcc -O2 -Iinclude tools/resume_latency.cpp -Lbookkeeper_amd -lbkdigest -Wl,-rpath,$PWD/bookkeeper_amd
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <functional>
#include <vector>

#include "bkdigest.h"

static double time_calls(int reps, const std::function<void()>& f) {
    f();
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) f();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
}

int main() {
    const size_t sizes[] = {64, 512, 4096, 32768, 65536, 262144, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20};
    const size_t maxn = 256 << 20;
    std::vector<uint8_t> pageable(maxn);
    for (size_t i = 0; i < maxn; ++i) pageable[i] = (uint8_t)(i * 131 + (i >> 9));
    uint8_t* pinned = nullptr;
    void* dbuf = nullptr;
    if (hipHostMalloc((void**)&pinned, maxn, hipHostMallocDefault) != hipSuccess) return 1;
    memcpy(pinned, pageable.data(), maxn);
    if (hipMalloc(&dbuf, maxn) != hipSuccess) return 1;
    hipMemcpy(dbuf, pageable.data(), maxn, hipMemcpyHostToDevice);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const uint64_t route_default = bkd_get_cpu_route_max();
    printf("cpu route: %s, default threshold %llu B\n", bkd_cpu_impl(), (unsigned long long)route_default);
    printf("%10s %12s %12s %12s %12s %12s %12s   (us per call)\n", "bytes", "cpu", "host_auto", "gpu_pageable",
           "gpu_pinned", "device", "auto_host");
    for (size_t n : sizes) {
        uint32_t a = 0, b = 0, c = 0, d = 0, e = 0, f = 0;
        const int reps = n <= 65536 ? 2000 : (n <= (4u << 20) ? 100 : (n <= (64u << 20) ? 10 : 3));
        const int greps = n <= 65536 ? 300 : (n <= (4u << 20) ? 50 : (n <= (64u << 20) ? 10 : 3));
        double t_cpu = time_calls(reps, [&] { bkd_cpu_resume(BKD_CRC32C, 0, pageable.data(), n, &a); });
        double t_auto = time_calls(reps, [&] { bkd_resume_host(BKD_CRC32C, 0, pageable.data(), n, &b); });
        bkd_set_cpu_route_max(0);
        bkd_set_host_batch_route(2);
        double t_gp = time_calls(greps, [&] { bkd_resume_host(BKD_CRC32C, 0, pageable.data(), n, &c); });
        double t_gn = time_calls(greps, [&] { bkd_resume_host(BKD_CRC32C, 0, pinned, n, &d); });
        bkd_set_host_batch_route(0);
        bkd_set_cpu_route_max(route_default);
        double t_dev = time_calls(greps, [&] { bkd_resume_device(BKD_CRC32C, 0, dbuf, n, st, &e); });
        double t_ah = time_calls(reps, [&] { bkd_resume(BKD_CRC32C, 0, pageable.data(), n, &f); });
        const bool same = a == b && b == c && c == d && d == e && e == f;
        printf("%10zu %12.3f %12.3f %12.3f %12.3f %12.3f %12.3f   %s %08x\n", n, t_cpu * 1e6, t_auto * 1e6,
               t_gp * 1e6, t_gn * 1e6, t_dev * 1e6, t_ah * 1e6, same ? "same" : "DIFFER", a);
        if (!same) {
            printf("cpu %08x host_auto %08x gpu_pageable %08x gpu_pinned %08x device %08x auto_host %08x\n", a, b, c,
                   d, e, f);
            bkd_set_cpu_route_max(0);
            bkd_set_host_batch_route(2);
            uint32_t g = 0;
            const int rc = bkd_resume_host(BKD_CRC32C, 0, pinned, n, &g);
            printf("forced GPU route: rc %d (%s) -> %08x\n", rc, bkd_last_error(), g);
            return 2;
        }
    }
    return 0;
}
