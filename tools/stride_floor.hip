// stride_floor: the HBM read floor of one header window per frame at a wide
// slot stride (c3: 2048-byte netmap slots), as a function of how many bytes of
// the window are read.  One frame per lane, P 16-byte loads from the slot
// start (nt), a 4-byte result stored per frame.  If the time does not change
// from P = 1 to P = 8, every frame costs one 128-byte L2 line from HBM however
// few of its bytes are read: the line-granular floor of the c3 workload.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/stride_floor tools/stride_floor.hip
//   build/stride_floor [frames=4194304] [stride=2048] [launches=40]
// (4M frames: 512 MiB of touched lines, past the 256 MiB Infinity Cache, so
// every launch reads HBM; the buffer is frames x stride = 8 GiB)
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

template <int P>
__global__ __launch_bounds__(256) void read_windows(const uint8_t *frames, uint32_t stride, uint32_t n,
                                                    uint32_t *out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u *w = reinterpret_cast<const v4u *>(frames + (size_t)i * stride);
  v4u q[P];
#pragma unroll
  for (int k = 0; k < P; ++k) q[k] = __builtin_nontemporal_load(w + k);
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < P; ++k) x ^= q[k].x ^ q[k].y ^ q[k].z ^ q[k].w;
  out[i] = x;
}

template <int P>
static void run(const uint8_t *d, uint32_t stride, uint32_t n, uint32_t *out, int launches) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 g((n + 255) / 256), b(256);
  for (int k = 0; k < 3; ++k) hipLaunchKernelGGL(read_windows<P>, g, b, 0, 0, d, stride, n, out);
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int k = 0; k < launches; ++k) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(read_windows<P>, g, b, 0, 0, d, stride, n, out);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double us = ms[ms.size() / 2] * 1e3;
  const double bytes = (double)n * (16 * P + 4);
  const double lines = (double)n * (128.0 * ((16 * P + 127) / 128) + 4);
  printf("{\"stride\": %u, \"read_bytes_per_frame\": %d, \"us_median\": %.2f, \"gbs_read_bytes\": %.1f, "
         "\"gbs_128B_lines\": %.1f, \"mpps\": %.1f}\n",
         stride, 16 * P, us, bytes / us / 1e3, lines / us / 1e3, n / us);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1u << 22;
  const uint32_t stride = argc > 2 ? (uint32_t)atoi(argv[2]) : 2048u;
  const int launches = argc > 3 ? atoi(argv[3]) : 40;
  uint8_t *d;
  uint32_t *out;
  // + 128 bytes: the 128-byte variant at a 64-byte stride reads past the last slot
  const size_t bytes = (size_t)n * stride + 128;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 0x5a, bytes));
  CK(hipMalloc(&out, (size_t)n * 4));
  run<1>(d, stride, n, out, launches);
  run<2>(d, stride, n, out, launches);
  run<3>(d, stride, n, out, launches);
  run<4>(d, stride, n, out, launches);
  run<8>(d, stride, n, out, launches);
  CK(hipFree(d));
  CK(hipFree(out));
  return 0;
}
