// Standalone check of HIP's stream-ordered pool on the round-3 "host one-copy" pattern, without
// libbkdigest: per call hipMallocAsync(span) + small blocks -> H2D of the same pageable bytes ->
// a kernel writes a per-stream scratch block (grown with hipFreeAsync/hipMallocAsync, like the old
// StreamScratch) -> a kernel checksums the span -> D2H -> hipFreeAsync -> sync. Prints per call the
// addresses, whether the checksum matches the host, and whether the device copy equals the source.
// Build: hipcc --offload-arch=gfx950 -O2 tools/pool_reuse_probe.hip -o tools/pool_reuse_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
__global__ void fill(uint32_t* s, size_t n, uint32_t v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s[i] = v ^ (uint32_t)i;
}
__global__ void sum(const uint64_t* p, size_t n, unsigned long long* out) {
    unsigned long long a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a += __builtin_nontemporal_load(p + i) * (2 * i + 1);
    atomicAdd(out, a);
}
int main() {
    hipStream_t st; hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipMemPool_t pool; hipDeviceGetDefaultMemPool(&pool, 0);
    uint64_t thr = UINT64_MAX; hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    const size_t M = 1 << 20; std::vector<uint64_t> h(512 * M / 8), back(512 * M / 8);
    for (size_t i = 0; i < h.size(); ++i) h[i] = i * 0x9E3779B97F4A7C15ull ^ (i >> 7);
    uint32_t* scratch = nullptr; size_t scap = 0; int bad = 0;
    for (size_t mib : {64, 128, 256, 512}) for (int k = 0; k < 6; ++k) {
        const size_t span = mib * M, words = span / 8, need = span / 4096 * 20;
        unsigned long long want = 0, got = 0; for (size_t i = 0; i < words; ++i) want += h[i] * (2 * i + 1);
        uint8_t* d = nullptr; unsigned long long* d_out = nullptr; void *d_off = nullptr, *d_len = nullptr;
        hipMallocAsync((void**)&d, span, st); hipMallocAsync(&d_off, 8, st); hipMallocAsync(&d_len, 4, st);
        hipMallocAsync((void**)&d_out, 8, st);
        hipMemcpyAsync(d, h.data(), span, hipMemcpyHostToDevice, st); hipMemsetAsync(d_out, 0, 8, st);
        if (scap < need) { if (scratch) hipFreeAsync(scratch, st); scap = need + need / 4 + 4096; hipMallocAsync((void**)&scratch, scap, st); }
        fill<<<512, 256, 0, st>>>(scratch, scap / 4, (uint32_t)k);
        sum<<<2048, 256, 0, st>>>((const uint64_t*)d, words, d_out);
        hipMemcpyAsync(&got, d_out, 8, hipMemcpyDeviceToHost, st); hipStreamSynchronize(st);
        hipMemcpy(back.data(), d, span, hipMemcpyDeviceToHost);
        const bool same = memcmp(back.data(), h.data(), span) == 0; bad += (got != want) || !same;
        printf("%4zu MiB call %d: d=%p d_out=%p scratch=%p..%p sum %s copy %s\n", mib, k, (void*)d, (void*)d_out,
               (void*)scratch, (void*)((uint8_t*)scratch + scap), got == want ? "ok" : "BAD", same ? "ok" : "BAD");
        for (void* p : {(void*)d, d_off, d_len, (void*)d_out}) hipFreeAsync(p, st);
        hipStreamSynchronize(st);
    }
    printf("%s: %d bad calls\n", hipGetErrorString(hipGetLastError()), bad);
    return bad ? 1 : 0;
}
