// Practical HBM read ceiling on this chip: stream N bytes with 16-B loads, XOR-reduce, write
// one word per block. Variants: plain vs nontemporal loads, grid size, loads in flight.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool NT, int U>
__global__ void __launch_bounds__(1024) rd(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
  u32x4 acc = {0,0,0,0};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = NT ? __builtin_nontemporal_load(p + i + k * stride) : p[i + k * stride];
#pragma unroll
    for (int k = 0; k < U; ++k) acc ^= v[k];
  }
  for (; i < n16; i += stride) acc ^= p[i];
  uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (r == 0x12345678u) out[blockIdx.x] = r;  // keep the loads alive
}
template <bool NT, int U>
float run(const u32x4* d, uint64_t n16, uint32_t* o, int blocks) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) rd<NT, U><<<blocks, 1024>>>(d, n16, o);
  hipEventRecord(a);
  const int R = 20;
  for (int r = 0; r < R; ++r) rd<NT, U><<<blocks, 1024>>>(d, n16, o);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / R;
}
int main() {
  const uint64_t bytes = 4ull << 30;
  u32x4* d; uint32_t* o;
  if (hipMalloc(&d, bytes) != hipSuccess) return 1;
  hipMalloc(&o, 1 << 20);
  hipMemset(d, 1, bytes);
  const uint64_t n16 = bytes / 16;
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int grids[] = {cus, 2 * cus, 4 * cus, 8 * cus};
  for (int g : grids) {
    float t1 = run<false, 4>(d, n16, o, g), t2 = run<true, 4>(d, n16, o, g), t3 = run<false, 8>(d, n16, o, g), t4 = run<true, 8>(d, n16, o, g);
    printf("blocks %5d x1024: plain U4 %.1f GB/s  nt U4 %.1f  plain U8 %.1f  nt U8 %.1f\n", g, bytes / t1 / 1e6, bytes / t2 / 1e6, bytes / t3 / 1e6, bytes / t4 / 1e6);
  }
  return 0;
}
