// Standalone check of HIP's stream-ordered pool on the round-3 "host one-copy" pattern, without
// libbkdigest: per call hipMallocAsync(span) + small blocks -> H2D of the same host bytes -> a
// kernel writes a per-stream scratch block (grown with hipFreeAsync/hipMallocAsync, like the old
// StreamScratch) -> a kernel checksums the span -> D2H -> hipFreeAsync -> sync; then a blocking D2H
// of the span checks what the device holds. argv[1]: pool (hipMallocAsync) | malloc (hipMalloc);
// argv[2]: pageable | pinned host source. Build: hipcc --offload-arch=gfx950 -O2 <this> -o <exe>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <string>
__global__ void fill(uint32_t* s, size_t n, uint32_t v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s[i] = v ^ (uint32_t)i;
}
__global__ void sum(const uint64_t* p, size_t n, unsigned long long* out) {
    unsigned long long a = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a += __builtin_nontemporal_load(p + i) * (2 * i + 1);
    atomicAdd(out, a);
}
int main(int argc, char** argv) {
    const bool pool = argc < 2 || std::string(argv[1]) == "pool", pinned = argc > 2 && std::string(argv[2]) == "pinned";
    auto alloc = [&](void** p, size_t b, hipStream_t s) { return pool ? hipMallocAsync(p, b, s) : hipMalloc(p, b); };
    auto release = [&](void* p, hipStream_t s) { return pool ? hipFreeAsync(p, s) : hipFree(p); };
    hipStream_t st; hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    hipMemPool_t mp; hipDeviceGetDefaultMemPool(&mp, 0);
    uint64_t thr = UINT64_MAX; hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &thr);
    const size_t M = 1 << 20; uint64_t *h, *back = new uint64_t[512 * M / 8];
    if (pinned) hipHostMalloc((void**)&h, 512 * M, 0); else h = new uint64_t[512 * M / 8];
    for (size_t i = 0; i < 512 * M / 8; ++i) h[i] = i * 0x9E3779B97F4A7C15ull ^ (i >> 7);
    uint32_t* scratch = nullptr; size_t scap = 0; int bad = 0;
    for (size_t mib : {64, 128, 256, 512}) for (int k = 0; k < 6; ++k) {
        const size_t span = mib * M, words = span / 8, need = span / 4096 * 20;
        unsigned long long want = 0, got = 0; for (size_t i = 0; i < words; ++i) want += h[i] * (2 * i + 1);
        uint8_t* d = nullptr; unsigned long long* d_out = nullptr; void *d_off = nullptr, *d_len = nullptr;
        alloc((void**)&d, span, st); alloc(&d_off, 8, st); alloc(&d_len, 4, st); alloc((void**)&d_out, 8, st);
        hipMemcpyAsync(d, h, span, hipMemcpyHostToDevice, st); hipMemsetAsync(d_out, 0, 8, st);
        if (scap < need) { if (scratch) release(scratch, st); scap = need + need / 4 + 4096; alloc((void**)&scratch, scap, st); }
        fill<<<512, 256, 0, st>>>(scratch, scap / 4, (uint32_t)k);
        sum<<<2048, 256, 0, st>>>((const uint64_t*)d, words, d_out);
        hipMemcpyAsync(&got, d_out, 8, hipMemcpyDeviceToHost, st); hipStreamSynchronize(st);
        hipMemcpy(back, d, span, hipMemcpyDeviceToHost);
        const bool same = memcmp(back, h, span) == 0; bad += (got != want) || !same;
        printf("%s %s %4zu MiB call %d: d=%p scratch=%p..%p sum %s copy %s\n", pool ? "pool" : "malloc", pinned ? "pinned" : "pageable",
               mib, k, (void*)d, (void*)scratch, (void*)((uint8_t*)scratch + scap), got == want ? "ok" : "BAD", same ? "ok" : "BAD");
        for (void* p : {(void*)d, d_off, d_len, (void*)d_out}) release(p, st);
        hipStreamSynchronize(st);
    }
    printf("%s: %d bad calls\n", hipGetErrorString(hipGetLastError()), bad);
    return bad ? 1 : 0;
}
