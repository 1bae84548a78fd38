// Does one ds_add_rtn_u32 instruction serve the lanes that hit the same LDS
// word in increasing lane order?  (The scatter kernel's optimistic stable
// rank relies on it and verifies every chunk; this measures how often a
// chunk would take the verified fallback.)  Random bins per lane, several
// bin-count regimes, packed u16 pairs as the scatter kernel uses them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(uint32_t nb, uint32_t seed, unsigned long long *bad, unsigned long long *pairs) {
  __shared__ uint32_t cur[1024];
  for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) cur[i] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = seed ^ (blockIdx.x * 0x9E3779B9u) ^ (threadIdx.x * 0x85EBCA6Bu);
  uint32_t nbad = 0, npair = 0;
  for (int it = 0; it < 64; ++it) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    const uint32_t b = (x % nb) + wave * (1024 / 8) * 0;   // all waves share the words
    const uint32_t w = b >> 1, sh = 16u * (b & 1u);
    const uint32_t old = (atomicAdd(&cur[w % 1024], 1u << sh) >> sh) & 0xFFFFu;
    // my predecessor in lane order within this instruction and wave, same bin
    for (uint32_t l = 0; l < 64; ++l) {
      const uint32_t bl = __shfl(b, l, 64), ol = __shfl(old, l, 64);
      if (l < lane && bl == b) { ++npair; if (ol >= old) ++nbad; }
    }
  }
  atomicAdd(bad, (unsigned long long)nbad);
  atomicAdd(pairs, (unsigned long long)npair);
}
int main() {
  unsigned long long *d; hipMalloc(&d, 16);
  for (uint32_t nb : {1u, 2u, 3u, 8u, 64u, 1008u, 2048u}) {
    hipMemset(d, 0, 16);
    for (uint32_t s = 0; s < 20; ++s) hipLaunchKernelGGL(k, dim3(4096), dim3(512), 0, 0, nb, s * 7919u + 1, d, d + 1);
    unsigned long long h[2]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("bins %4u: same-word lane pairs %llu, out of lane order %llu\n", nb, h[1], h[0]);
  }
  return 0;
}
