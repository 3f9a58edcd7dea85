// Shader-clock probe for the launch-ramp study: one small kernel, enqueued between
// CRC launches on the same stream, spins for `ticks` of the constant 100 MHz real-time counter and
// records how many shader cycles (s_memtime) passed meanwhile, so the shader clock in effect right
// after each CRC launch is (cycles / ticks) * 100 MHz. Eight blocks, so several XCDs are sampled.
// Read-only use of the two counters; results go out through ordinary vector stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(64) clock_probe_kernel(uint64_t* __restrict__ out, uint32_t ticks) {
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t r1 = r0, c1 = c0;
    while (r1 - r0 < ticks) {
        __builtin_amdgcn_s_sleep(1);
        r1 = __builtin_amdgcn_s_memrealtime();
    }
    c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = c1 - c0;
        out[2 * blockIdx.x + 1] = r1 - r0;
    }
}

extern "C" int clock_probe_launch(void* stream, uint64_t* out, uint32_t ticks) {
    hipLaunchKernelGGL(clock_probe_kernel, dim3(8), dim3(64), 0, (hipStream_t)stream, out, ticks);
    return (int)hipGetLastError();
}
