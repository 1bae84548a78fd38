// probe_floor: what the c5 probes cost on their own and beside the header
// stream.  One frame per lane; a frame's "key" hashes to a 16-byte slot of
// table 1 (T1 bytes); 55 % of frames (c5: key1 misses) read a second slot in
// table 2, dependent on the first.  Modes:
//   0  stream only: 64 B per frame read (4 x 16 B, nt), 4 B written
//   1  probes only: slot 1, then slot 2 where needed, 4 B written
//   2  stream + probes: the key is hashed from the frame's bytes
//   3  stream + one probe per frame (no dependent second read)
//   10+c probes only, inline-asm loads with cache policy c (0 none, 1 sc0,
//        2 nt, 3 sc1, 4 sc0 sc1, 5 dword instead of dwordx4)
//   glds stream (the classify kernel's LDS-DMA header stage), alone and with
//        the probes keyed by the staged bytes
// If mode 1 alone takes about as long as the gap between mode 2 and mode 0,
// the probes are bound by their own request rate, not by latency.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/probe_floor tools/probe_floor.hip
//   build/probe_floor [frames=8388608] [table_kib=1700] [launches=40] [policies]
#include <hip/hip_runtime.h>

#include <algorithm>
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

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void probe(const v4u *frames, const v4u *t1, const v4u *t2, uint32_t m1,
                                             uint32_t m2, uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t key = mix(i * 0x9e3779b9u);
  if (MODE != 1) {
    v4u q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = __builtin_nontemporal_load(frames + (size_t)i * 4 + k);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) x ^= q[k].x ^ q[k].y ^ q[k].z ^ q[k].w;
    if (MODE == 0) { out[i] = x; return; }
    key ^= x;
  }
  const v4u s1 = t1[mix(key) % m1];
  uint32_t w = s1.x ^ s1.w;
  if (MODE != 3 && (s1.y % 100u) < 55u) {
    const v4u s2 = t2[mix(key ^ 0x5bd1e995u) % m2];
    w ^= s2.x ^ s2.z;
  }
  out[i] = w;
}

/* The classify kernel's header stream: each wave moves its 64 frames' first
 * 48 bytes into LDS by three 1 KiB LDS-DMA instructions (lane u of
 * instruction k: part (64k+u) % 3 of frame (64k+u) / 3), then each lane reads
 * its frame from LDS.  PROBES: then the two-table probe of mode 2 keyed by
 * the frame's bytes. */
typedef __attribute__((address_space(3))) void lds_void_t;
template <bool PROBES, int PARTS = 3>
__global__ __launch_bounds__(256) void glds_stream(const uint8_t *frames, const v4u *t1, const v4u *t2,
                                                   uint32_t m1, uint32_t m2, uint32_t n, uint32_t *out) {
  // PARTS 3: bytes 0..47 of each frame; PARTS 2: bytes 12..43 (what the rx parse reads)
  constexpr uint32_t OFF = PARTS == 2 ? 12u : 0u;
  __shared__ v4u st[4][192];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t f0 = blockIdx.x * 256 + wave * 64;
  if (f0 >= n) return;
#pragma unroll
  for (uint32_t k = 0; k < PARTS; ++k) {
    const uint32_t u = 64 * k + lane, f = u / PARTS, part = u - PARTS * f;
    __builtin_amdgcn_global_load_lds(frames + (size_t)(f0 + f) * 64 + OFF + part * 16,
                                     (lds_void_t *)(&st[wave][64 * k]), 16, 0, 2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t x;
  if (PARTS == 3) {
    const v4u a = st[wave][3 * lane], b = st[wave][3 * lane + 1], c = st[wave][3 * lane + 2];
    x = a.x ^ a.w ^ b.y ^ b.z ^ c.x ^ c.y;
  } else {
    const v4u a = st[wave][2 * lane], b = st[wave][2 * lane + 1];
    x = a.x ^ a.w ^ b.y ^ b.z;
  }
  if (PROBES) {
    const uint32_t key = mix(x ^ ((f0 + lane) * 0x9e3779b9u));
    const v4u s1 = t1[mix(key) % m1];
    x = s1.x ^ s1.w;
    if ((s1.y % 100u) < 55u) {
      const v4u s2 = t2[mix(key ^ 0x5bd1e995u) % m2];
      x ^= s2.x ^ s2.z;
    }
  }
  out[f0 + lane] = x;
}

template <bool PROBES, int PARTS = 3>
static void run_glds(const uint8_t *f, const v4u *t1, const v4u *t2, uint32_t m, uint32_t n, uint32_t *out,
                     int launches) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((n + 255) / 256), b(256);
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL((glds_stream<PROBES, PARTS>), g, b, 0, 0, f, t1, t2, m, m, n, out);
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int k = 0; k < launches; ++k) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((glds_stream<PROBES, PARTS>), g, b, 0, 0, f, t1, t2, m, m, n, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double us = ms[ms.size() / 2] * 1e3;
  printf("{\"mode\": \"glds stream%s %d parts\", \"frames\": %u, \"table_slots\": %u, \"us_median\": %.2f}\n",
         PROBES ? "+probes" : "", PARTS, n, m, us);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int C>
__device__ __forceinline__ v4u ld_pol(const v4u *p) {
  v4u s;
  if (C == 0) asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(s) : "v"(p) : "memory");
  if (C == 1) asm volatile("global_load_dwordx4 %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(s) : "v"(p) : "memory");
  if (C == 2) asm volatile("global_load_dwordx4 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(s) : "v"(p) : "memory");
  if (C == 3) asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(s) : "v"(p) : "memory");
  if (C == 4) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(s) : "v"(p) : "memory");
  if (C == 5) {
    uint32_t x;
    asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory");
    s = v4u{x, x * 3u, x * 5u, x * 7u};
  }
  return s;
}

template <int C>
__global__ __launch_bounds__(256) void probe_pol(const v4u *t1, const v4u *t2, uint32_t m1, uint32_t m2,
                                                 uint32_t n, uint32_t *out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t key = mix(i * 0x9e3779b9u);
  const v4u s1 = ld_pol<C>(t1 + mix(key) % m1);
  uint32_t w = s1.x ^ s1.w;
  if ((s1.y % 100u) < 55u) {
    const v4u s2 = ld_pol<C>(t2 + mix(key ^ 0x5bd1e995u) % m2);
    w ^= s2.x ^ s2.z;
  }
  out[i] = w;
}

template <int C>
static void run_pol(const v4u *t1, const v4u *t2, uint32_t m, uint32_t n, uint32_t *out, int launches) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((n + 255) / 256), b(256);
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(probe_pol<C>, g, b, 0, 0, t1, t2, m, m, n, out);
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int k = 0; k < launches; ++k) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(probe_pol<C>, g, b, 0, 0, t1, t2, m, m, n, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double us = ms[ms.size() / 2] * 1e3;
  static const char *names[] = {"none", "sc0", "nt", "sc1", "sc0 sc1", "dword"};
  printf("{\"mode\": \"probes asm %s\", \"frames\": %u, \"table_slots\": %u, \"us_median\": %.2f}\n",
         names[C], n, m, us);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

/* F frames per lane, all first probes in flight together, then all second
 * probes (a lane that needs none reads slot 0): the request-rate floor */
template <int F>
__global__ __launch_bounds__(256) void probe_batched(const v4u *t1, const v4u *t2, uint32_t m1, uint32_t m2,
                                                     uint32_t n, uint32_t *out) {
  const uint32_t i0 = (blockIdx.x * 256 + threadIdx.x) * F;
  if (i0 >= n) return;
  uint32_t key[F];
  v4u s1[F], s2[F];
#pragma unroll
  for (int f = 0; f < F; ++f) key[f] = mix((i0 + f) * 0x9e3779b9u);
#pragma unroll
  for (int f = 0; f < F; ++f) s1[f] = t1[mix(key[f]) % m1];
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const bool need = (s1[f].y % 100u) < 55u;
    s2[f] = t2[need ? mix(key[f] ^ 0x5bd1e995u) % m2 : 0u];
  }
  uint32_t w = 0;
#pragma unroll
  for (int f = 0; f < F; ++f) w ^= s1[f].x ^ s2[f].z;
  out[i0 / F] = w;
}

template <int F>
static void run_batched(const v4u *t1, const v4u *t2, uint32_t m, uint32_t n, uint32_t *out, int launches) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((n / F + 255) / 256), b(256);
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(probe_batched<F>, g, b, 0, 0, t1, t2, m, m, n, out);
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int k = 0; k < launches; ++k) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(probe_batched<F>, g, b, 0, 0, t1, t2, m, m, n, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double us = ms[ms.size() / 2] * 1e3;
  printf("{\"mode\": \"probes batched %d\", \"frames\": %u, \"table_slots\": %u, \"us_median\": %.2f}\n",
         F, n, m, us);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int MODE>
static void run(const v4u *f, const v4u *t1, const v4u *t2, uint32_t m, uint32_t n, uint32_t *out,
                int launches, const char *name) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((n + 255) / 256), b(256);
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(probe<MODE>, g, b, 0, 0, f, t1, t2, m, m, n, out);
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int k = 0; k < launches; ++k) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(probe<MODE>, g, b, 0, 0, f, t1, t2, m, m, n, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double us = ms[ms.size() / 2] * 1e3;
  printf("{\"mode\": \"%s\", \"frames\": %u, \"table_slots\": %u, \"us_median\": %.2f, \"mpps\": %.1f}\n", name,
         n, m, us, n / us);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1u << 23;
  const uint32_t kib = argc > 2 ? (uint32_t)atoi(argv[2]) : 1700u;
  const int launches = argc > 3 ? atoi(argv[3]) : 40;
  const uint32_t m = kib * 1024u / 16u;
  v4u *f, *t1, *t2;
  uint32_t *out;
  // frames: 2 GiB rotating would be fairer; 8M x 64 B = 512 MiB is past the
  // 256 MiB Infinity Cache already
  CK(hipMalloc(&f, (size_t)n * 64));
  CK(hipMemset(f, 0x37, (size_t)n * 64));
  std::vector<uint32_t> h((size_t)m * 4);
  uint32_t s = 12345u;
  for (auto &x : h) { s = s * 1664525u + 1013904223u; x = s; }
  CK(hipMalloc(&t1, (size_t)m * 16));
  CK(hipMalloc(&t2, (size_t)m * 16));
  CK(hipMemcpy(t1, h.data(), (size_t)m * 16, hipMemcpyHostToDevice));
  for (auto &x : h) { s = s * 1664525u + 1013904223u; x = s; }
  CK(hipMemcpy(t2, h.data(), (size_t)m * 16, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)n * 4));
  run<0>(f, t1, t2, m, n, out, launches, "stream");
  run<1>(f, t1, t2, m, n, out, launches, "probes");
  run<2>(f, t1, t2, m, n, out, launches, "stream+probes");
  run<3>(f, t1, t2, m, n, out, launches, "stream+probe1");
  if (argc > 4) {
    run_pol<0>(t1, t2, m, n, out, launches);
    run_pol<1>(t1, t2, m, n, out, launches);
    run_pol<2>(t1, t2, m, n, out, launches);
    run_pol<3>(t1, t2, m, n, out, launches);
    run_pol<4>(t1, t2, m, n, out, launches);
    run_pol<5>(t1, t2, m, n, out, launches);
  }
  run_glds<false>(reinterpret_cast<const uint8_t *>(f), t1, t2, m, n, out, launches);
  run_glds<true>(reinterpret_cast<const uint8_t *>(f), t1, t2, m, n, out, launches);
  run_glds<false, 2>(reinterpret_cast<const uint8_t *>(f), t1, t2, m, n, out, launches);
  run_glds<true, 2>(reinterpret_cast<const uint8_t *>(f), t1, t2, m, n, out, launches);
  run_glds<false>(reinterpret_cast<const uint8_t *>(f), t1, t2, m, n, out, launches);
  run_glds<false, 2>(reinterpret_cast<const uint8_t *>(f), t1, t2, m, n, out, launches);
  run_batched<1>(t1, t2, m, n, out, launches);
  run_batched<2>(t1, t2, m, n, out, launches);
  run_batched<4>(t1, t2, m, n, out, launches);
  run_batched<8>(t1, t2, m, n, out, launches);
  run_batched<16>(t1, t2, m, n, out, launches);
  CK(hipFree(f));
  CK(hipFree(t1));
  CK(hipFree(t2));
  CK(hipFree(out));
  return 0;
}
