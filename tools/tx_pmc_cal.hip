// tx_pmc_cal: calibrates the tx kernel's HBM-traffic model (VERDICT r04 #3:
// tools/pmc_traffic.py tx_kernel=1+32 had no calibration run).  One kernel
// per request type of tx_kernel, each over a known number of units, so that
// rocprofv3's TCC request counters (TCC_EA0_RDREQ, TCC_EA0_RDREQ_32B,
// TCC_BUBBLE; FETCH_SIZE is derived from them) can be read per unit:
//   cal_hdr    the tx kernel's coalesced header loads: per wave of 64 frames
//              at a 64-byte stride, 3 x 16-byte loads per lane (lane u of load
//              k reads part u % 3 of frame u / 3): 48 of every 64 bytes, every
//              128-byte line touched -> 64 B of lines per frame
//   cal_lens   the 2-byte length per frame (coalesced ushort loads)
//   cal_probe  P scattered 16-byte loads per frame into a table of T bytes
//              (8 MiB: the c4tx rule image's size, Infinity-Cache resident;
//              1 GiB: every probe from HBM)
//   cal_mixed  all three in one kernel, with a 4-byte store per frame (the
//              tx kernel's shape): the counters should add up
// Every kernel stores 4 B per frame.  Frames rotate over 6 buffers (384 MiB,
// past the 256 MiB Infinity Cache).
//
//   hipcc -O3 --offload-arch=gfx950 -o build/tx_pmc_cal tools/tx_pmc_cal.hip
//   build/tx_pmc_cal [frames=1048576] [launches=12]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t P = 3;   // probes per frame

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t hdr_part(const uint8_t *frames, uint32_t n, uint32_t wave0) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x = 0;
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) {
    const uint32_t u = 64u * k + lane, f = (u * 0xAAABu) >> 17, part = u - 3u * f;
    const uint32_t fi = min(wave0 + f, n - 1);
    const v4u q = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(frames + (size_t)fi * 64 + part * 16));
    x ^= q.x ^ q.y ^ q.z ^ q.w;
  }
  return x;
}

__device__ __forceinline__ uint32_t probe_part(const v4u *table, uint32_t mask, uint32_t i) {
  uint32_t x = 0;
#pragma unroll
  for (uint32_t k = 0; k < P; ++k) {
    const v4u q = table[mix(i * P + k + 0x9e3779b9u) & mask];
    x ^= q.x ^ q.y ^ q.z ^ q.w;
  }
  return x;
}

__global__ __launch_bounds__(256) void cal_hdr(const uint8_t *frames, uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t x = hdr_part(frames, n, i & ~63u);
  if (i < n) out[i] = x;
}

__global__ __launch_bounds__(256) void cal_lens(const uint16_t *lens, uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = lens[i] * 3u;
}

template <int TAG>   // (TAG: the table size in the kernel's name, for the counter rows)
__global__ __launch_bounds__(256) void cal_probe(const v4u *table, uint32_t mask, uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = probe_part(table, mask, i);
}

__global__ __launch_bounds__(256) void cal_mixed(const uint8_t *frames, const uint16_t *lens, const v4u *table,
                                                 uint32_t mask, uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  const uint32_t x = hdr_part(frames, n, i & ~63u);
  if (i < n) out[i] = x ^ lens[i] ^ probe_part(table, mask, i);
}

static float median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  const int L = argc > 2 ? atoi(argv[2]) : 12;
  constexpr int R = 6;
  std::vector<uint8_t *> fr(R);
  std::vector<uint16_t *> ln(R);
  for (int k = 0; k < R; ++k) {
    CK(hipMalloc(&fr[k], (size_t)n * 64));
    CK(hipMemset(fr[k], k + 1, (size_t)n * 64));
    CK(hipMalloc(&ln[k], (size_t)n * 2));
    CK(hipMemset(ln[k], 0x40, (size_t)n * 2));
  }
  const size_t small = 8u << 20, big = 1ull << 30;
  v4u *ts, *tb;
  CK(hipMalloc(&ts, small));
  CK(hipMemset(ts, 3, small));
  CK(hipMalloc(&tb, big));
  CK(hipMemset(tb, 5, big));
  uint32_t *out;
  CK(hipMalloc(&out, (size_t)n * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((n + 255) / 256), b(256);
  const uint32_t ms_ = (uint32_t)(small / 16 - 1), mb_ = (uint32_t)(big / 16 - 1);
  auto timed = [&](const char *name, auto launch, double bytes) {
    for (int k = 0; k < 2; ++k) launch(k);   // warm (the 8 MiB table into the Infinity Cache)
    CK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int k = 0; k < L; ++k) {
      CK(hipEventRecord(e0, 0));
      launch(k);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    const float m = median(t);
    printf("{\"kernel\": \"%s\", \"frames\": %u, \"us_median\": %.2f, \"known_bytes\": %.0f, \"GBps\": %.1f}\n",
           name, n, m * 1e3, bytes, bytes / (m * 1e-3) / 1e9);
  };
  timed("cal_hdr", [&](int k) { hipLaunchKernelGGL(cal_hdr, g, b, 0, 0, fr[k % R], n, out); },
        64.0 * n);
  timed("cal_lens", [&](int k) { hipLaunchKernelGGL(cal_lens, g, b, 0, 0, ln[k % R], n, out); }, 2.0 * n);
  timed("cal_probe_8MiB", [&](int) { hipLaunchKernelGGL(cal_probe<8>, g, b, 0, 0, ts, ms_, n, out); },
        16.0 * P * n);
  timed("cal_probe_1GiB", [&](int) { hipLaunchKernelGGL(cal_probe<1024>, g, b, 0, 0, tb, mb_, n, out); },
        16.0 * P * n);
  timed("cal_mixed", [&](int k) {
    hipLaunchKernelGGL(cal_mixed, g, b, 0, 0, fr[k % R], ln[k % R], ts, ms_, n, out);
  }, 66.0 * n);
  CK(hipDeviceSynchronize());
  return 0;
}
