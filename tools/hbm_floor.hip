// hbm_floor: what the HBM read path alone allows for the classify access
// pattern (64-byte header window + 2-byte length read, 4 + 2 bytes written per
// frame), with no parse, probe or ordering.  Prints one line per variant:
// isolated-launch time (one launch at a time, HIP events) and back-to-back
// time, both per launch of `frames` frames, and the GB/s of 72 B per frame.
//
//   hipcc -O3 --offload-arch=gfx950 -o build/hbm_floor tools/hbm_floor.hip
//   build/hbm_floor [frames_per_launch=8388608] [launches=50]
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

struct Args {
  const uint8_t *frames;
  const uint16_t *lens;
  uint32_t *dec;
  uint16_t *order;
  uint32_t n;        // frames
  uint32_t ntiles;   // tiles of 1024
};

__device__ __forceinline__ uint32_t fold(const uint4 *q, uint32_t len) {
  return q[0].w ^ q[1].x ^ q[1].y ^ q[1].z ^ q[1].w ^ q[2].x ^ q[2].y ^ q[3].w ^ len;
}

// one tile of 1024 frames per workgroup pass, 4 rounds per lane, round r+1's
// loads issued before round r is consumed (the production load order)
template <int NT>
__device__ __forceinline__ void tile_lane64(const Args &a, uint32_t tile) {
  constexpr int R = 1024 / NT;
  const uint32_t tid = threadIdx.x;
  const uint64_t base = (uint64_t)tile * 1024;
  uint4 q[R][4];
  uint32_t len[R];
#pragma unroll
  for (int r = 0; r < R; ++r) len[r] = a.lens[base + r * NT + tid];
  {
    const uint4 *w = reinterpret_cast<const uint4 *>(a.frames + (base + tid) * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) q[0][k] = w[k];
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r + 1 < R) {
      __builtin_amdgcn_sched_barrier(0);
      const uint4 *w = reinterpret_cast<const uint4 *>(a.frames + (base + (r + 1) * NT + tid) * 64);
#pragma unroll
      for (int k = 0; k < 4; ++k) q[r + 1][k] = w[k];
      __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t d = fold(q[r], len[r]);
    a.dec[base + r * NT + tid] = d;
    a.order[base + r * NT + tid] = (uint16_t)(d & 1023);
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_lane64(Args a) {
  tile_lane64<NT>(a, blockIdx.x);
}

// persistent: gridDim.x workgroups, each takes tiles w, w + grid, ...
template <int NT>
__global__ __launch_bounds__(NT) void k_lane64_persist(Args a) {
  for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) tile_lane64<NT>(a, t);
}

// persistent with a contiguous chunk of tiles per workgroup
template <int NT>
__global__ __launch_bounds__(NT) void k_lane64_chunk(Args a) {
  const uint32_t per = (a.ntiles + gridDim.x - 1) / gridDim.x;
  const uint32_t t0 = blockIdx.x * per, t1 = min(a.ntiles, t0 + per);
  for (uint32_t t = t0; t < t1; ++t) tile_lane64<NT>(a, t);
}

// dense: every wave instruction reads 1 KiB contiguous (16 frames), no transpose
__global__ __launch_bounds__(256) void k_dense(Args a) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * 1024;
  uint4 q[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint4 *c = reinterpret_cast<const uint4 *>(a.frames + (base + r * 256 + wave * 64) * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) q[r][k] = c[64 * k + lane];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t len = a.lens[base + r * 256 + tid];
    uint32_t d = len;
#pragma unroll
    for (int k = 0; k < 4; ++k) d ^= q[r][k].x ^ q[r][k].y ^ q[r][k].z ^ q[r][k].w;
    a.dec[base + r * 256 + tid] = d;
    a.order[base + r * 256 + tid] = (uint16_t)(d & 1023);
  }
}

// LDS-DMA: global_load_lds_dwordx4, 1 KiB per wave instruction into a
// wave-private 4 KiB stage per round, then each lane reads its own frame
__global__ __launch_bounds__(256) void k_glds(Args a) {
  __shared__ __align__(16) uint8_t stage[4][4][4096];   // [round][wave][...]
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * 1024;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint8_t *c = a.frames + (base + r * 256 + wave * 64) * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(c + k * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void *)(&stage[r][wave][k * 1024]),
                                       16, 0, 0);
  }
  uint32_t len[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) len[r] = a.lens[base + r * 256 + tid];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint4 *f = reinterpret_cast<const uint4 *>(&stage[r][wave][lane * 64]);
    uint4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = f[k];
    const uint32_t d = fold(q, len[r]);
    a.dec[base + r * 256 + tid] = d;
    a.order[base + r * 256 + tid] = (uint16_t)(d & 1023);
  }
}

typedef __attribute__((address_space(3))) void lds_void;
#define VMWAIT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-DMA with DEPTH rounds in flight per wave (DEPTH 4 KiB buffers per
// wave); lengths ride along as a 128-byte glds per round.  AUX = 2: nt.
template <int AUX, int DEPTH>
__global__ __launch_bounds__(256) void k_glds_pipe(Args a) {
  __shared__ __align__(16) uint8_t stage[4][DEPTH][4096];   // [wave][buf][...]
  __shared__ __align__(16) uint16_t slen[4][DEPTH][64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * 1024;
  auto issue = [&](int r) {
    const uint8_t *c = a.frames + (base + r * 256 + wave * 64) * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(c + k * 1024 + lane * 16),
                                       (lds_void *)(&stage[wave][r % DEPTH][k * 1024]), 16, 0, AUX);
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a.lens + base + r * 256 + wave * 64 + lane),
                                     (lds_void *)(&slen[wave][r % DEPTH][0]), 2, 0, AUX);
  };
#pragma unroll
  for (int r = 0; r < DEPTH; ++r) issue(r);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    // round r landed: the rounds issued after it may still fly (5 glds each)
    constexpr int dummy = 0;
    (void)dummy;
    const int after = (DEPTH - 1 < 3 - r) ? DEPTH - 1 : 3 - r;
    if (after == 3) vmwait<15>();
    else if (after == 2) vmwait<10>();
    else if (after == 1) vmwait<5>();
    else vmwait<0>();
    const uint4 *f = reinterpret_cast<const uint4 *>(&stage[wave][r % DEPTH][lane * 64]);
    uint4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = f[k];
    const uint32_t len = slen[wave][r % DEPTH][lane];
    if (r + DEPTH < 4) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the refill
      issue(r + DEPTH);
    }
    const uint32_t d = fold(q, len);
    a.dec[base + r * 256 + tid] = d;
    a.order[base + r * 256 + tid] = (uint16_t)(d & 1023);
  }
}

// register loads with the nt hint
__global__ __launch_bounds__(256) void k_lane64_nt(Args a) {
  const uint32_t tid = threadIdx.x;
  const uint64_t base = (uint64_t)blockIdx.x * 1024;
  uint4 q[4][4];
  uint32_t len[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) len[r] = a.lens[base + r * 256 + tid];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const v4u *w = reinterpret_cast<const v4u *>(a.frames + (base + r * 256 + tid) * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const v4u v = __builtin_nontemporal_load(w + k);
      q[r][k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t d = fold(q[r], len[r]);
    a.dec[base + r * 256 + tid] = d;
    a.order[base + r * 256 + tid] = (uint16_t)(d & 1023);
  }
}

/* placement mode: the same kernel over many separately allocated buffers,
 * each timed on its own (does where hipMalloc put a buffer change its rate?) */
/* mode 0: hipMalloc per array; 1: hipDeviceMallocContiguous; 2: one pool,
 * arrays carved at 2 MiB-aligned offsets; 3: hipMalloc after a 32 GiB
 * allocate-and-free */
static void *dev_alloc(size_t bytes, int mode) {
  static uint8_t *pool = nullptr;
  static size_t used = 0;
  void *p = nullptr;
  bytes = (bytes + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
  if (mode == 1) {
    CK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous));
  } else if (mode == 2) {
    if (!pool) CK(hipMalloc((void **)&pool, (size_t)24 << 30));
    p = pool + used;
    used += bytes;
  } else {
    CK(hipMalloc(&p, bytes));
  }
  return p;
}

static int placement(uint32_t n, int nbuf, int launches, int mode) {
  if (mode == 3) {
    void *big;
    CK(hipMalloc(&big, (size_t)32 << 30));
    CK(hipFree(big));
  }
  std::vector<Args> args(nbuf);
  for (int b = 0; b < nbuf; ++b) {
    uint8_t *f = (uint8_t *)dev_alloc((size_t)n * 64, mode);
    uint16_t *l = (uint16_t *)dev_alloc((size_t)n * 2, mode);
    uint32_t *d = (uint32_t *)dev_alloc((size_t)n * 4, mode);
    uint16_t *o = (uint16_t *)dev_alloc((size_t)n * 2, mode);
    CK(hipMemset(f, 0x45, (size_t)n * 64));
    CK(hipMemset(l, 0, (size_t)n * 2));
    args[b] = Args{f, l, d, o, n, n / 1024};
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("mode %d\n", mode);
  for (int rep = 0; rep < 1; ++rep)
    for (int b = 0; b < nbuf; ++b) {
      std::vector<float> t;
      for (int i = 0; i < launches; ++i) {
        // flush: touch another buffer so this one is not Infinity-Cache resident
        k_lane64<256><<<args[(b + 1) % nbuf].ntiles, 256, 0, s>>>(args[(b + 1) % nbuf]);
        CK(hipEventRecord(e0, s));
        k_lane64<256><<<args[b].ntiles, 256, 0, s>>>(args[b]);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3f);
      }
      std::sort(t.begin(), t.end());
      printf("buffer %2d at %p: median %8.2f us (%6.0f GB/s)\n", b, (void *)args[b].frames,
             t[t.size() / 2], 72.0 * n / t[t.size() / 2] / 1e3);
    }
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && argv[1][0] == 'p')
    return placement(argc > 2 ? (uint32_t)atoi(argv[2]) : (1u << 20), argc > 3 ? atoi(argv[3]) : 16,
                     argc > 4 ? atoi(argv[4]) : 20, argc > 5 ? atoi(argv[5]) : 0);
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (8u << 20);
  const int launches = argc > 2 ? atoi(argv[2]) : 50;
  const int NB = 4;   // rotating buffers: 4 x (64 + 2) B x n > Infinity Cache
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<Args> args(NB);
  for (int b = 0; b < NB; ++b) {
    uint8_t *f;
    uint16_t *l;
    uint32_t *d;
    uint16_t *o;
    CK(hipMalloc(&f, (size_t)n * 64));
    CK(hipMalloc(&l, (size_t)n * 2));
    CK(hipMalloc(&d, (size_t)n * 4));
    CK(hipMalloc(&o, (size_t)n * 2));
    CK(hipMemset(f, 0x45, (size_t)n * 64));
    CK(hipMemset(l, 0, (size_t)n * 2));
    args[b] = Args{f, l, d, o, n, n / 1024};
  }
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    const char *name;
    void (*launch)(const Args &, hipStream_t, int);
    int grid_arg;
  };
  auto L64 = [](const Args &a, hipStream_t st, int) {
    k_lane64<256><<<a.ntiles, 256, 0, st>>>(a);
  };
  auto L64_512 = [](const Args &a, hipStream_t st, int) {
    k_lane64<512><<<a.ntiles, 512, 0, st>>>(a);
  };
  auto LP = [](const Args &a, hipStream_t st, int g) {
    k_lane64_persist<256><<<g, 256, 0, st>>>(a);
  };
  auto LC = [](const Args &a, hipStream_t st, int g) {
    k_lane64_chunk<256><<<g, 256, 0, st>>>(a);
  };
  auto LD = [](const Args &a, hipStream_t st, int) { k_dense<<<a.ntiles, 256, 0, st>>>(a); };
  auto LG = [](const Args &a, hipStream_t st, int) { k_glds<<<a.ntiles, 256, 0, st>>>(a); };
  auto LGP = [](const Args &a, hipStream_t st, int) { k_glds_pipe<0, 2><<<a.ntiles, 256, 0, st>>>(a); };
  auto LGPN = [](const Args &a, hipStream_t st, int) { k_glds_pipe<2, 2><<<a.ntiles, 256, 0, st>>>(a); };
  auto LGP1N = [](const Args &a, hipStream_t st, int) { k_glds_pipe<2, 1><<<a.ntiles, 256, 0, st>>>(a); };
  auto LGP3N = [](const Args &a, hipStream_t st, int) { k_glds_pipe<2, 3><<<a.ntiles, 256, 0, st>>>(a); };
  auto LGP4N = [](const Args &a, hipStream_t st, int) { k_glds_pipe<2, 4><<<a.ntiles, 256, 0, st>>>(a); };
  auto LNT = [](const Args &a, hipStream_t st, int) { k_lane64_nt<<<a.ntiles, 256, 0, st>>>(a); };
  std::vector<V> vs = {
      {"lane64", L64, 0},           {"lane64_t512", L64_512, 0},
      {"chunk_x8", LC, 8 * cus},
      {"dense", LD, 0},             {"glds", LG, 0},
      {"glds_pipe", LGP, 0},        {"glds_pipe_nt", LGPN, 0},
      {"glds_p1_nt", LGP1N, 0},     {"glds_p3_nt", LGP3N, 0},
      {"glds_p4_nt", LGP4N, 0},
  };
  printf("frames/launch %u, %d CUs, %d launches, 72 B/frame\n", n, cus, launches);
  for (int rep = 0; rep < 2; ++rep) {
    for (auto &v : vs) {
      for (int i = 0; i < 5; ++i) v.launch(args[i % NB], s, v.grid_arg);
      CK(hipStreamSynchronize(s));
      std::vector<float> iso;
      for (int i = 0; i < launches; ++i) {
        CK(hipEventRecord(e0, s));
        v.launch(args[i % NB], s, v.grid_arg);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        iso.push_back(ms * 1e3f);
      }
      std::sort(iso.begin(), iso.end());
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < launches; ++i) v.launch(args[i % NB], s, v.grid_arg);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double b2b = ms * 1e3 / launches, med = iso[iso.size() / 2];
      printf("%-12s isolated %8.2f us (%6.0f GB/s)   back-to-back %8.2f us (%6.0f GB/s)\n", v.name,
             med, 72.0 * n / med / 1e3, b2b, 72.0 * n / b2b / 1e3);
      CK(hipGetLastError());
    }
  }
  return 0;
}
