/*
 * usn_device.hip -- gfx950 kernels of the usnetd match path.
 *
 * classify: one workgroup (256 threads, 4 waves) per tile of USN_TILE = 1024
 * frames, one frame per lane per round, four rounds.  Per frame:
 *   1. four 16-byte loads of the 64-byte header window + the 2-byte length
 *      (all 16 loads of a lane issued before any is consumed);
 *   2. extract_pkt_info in registers           /root/reference/src/pkt.rs:158-218
 *   3. get_endpoint: two exact-match probes     /root/reference/src/endpoint.rs:307-338
 *      into the bucketed rule table (LDS copy when it fits, else L2-resident);
 *   4. the per-frame decision of find_forward   /root/reference/src/endpoint.rs:172-296
 *      for a NIC source (incoming): FLOOD / loopback DROP / lookup / DHCP flag;
 *   5. stable per-endpoint order of the tile: wave ballots give each frame its
 *      rank inside its 64-frame segment and per-segment bin counts; a column
 *      scan over the 16 segments and a block scan over bins turn them into
 *      slots; the sorted tile-local indices and the bin runs are written with
 *      coalesced stores.
 * No MFMA: this is byte parsing and hash probing, bounded by HBM reads.
 *
 * Order-dependent state (fragment map, DHCP next endpoint, a stale carried
 * cache entry) never changes a decision silently: frames that need it carry
 * USN_F_HOST and are listed per tile for the ordered host stage (usn_finalize).
 */
#include <hip/hip_runtime.h>

#include "usn_internal.h"
#include "usn_kernels.h"

namespace usn {

#define TILE USN_TILE
#define NTHREADS 256
#define ROUNDS (TILE / NTHREADS)
#define NSEG (TILE / 64)

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

#ifndef USN_LOAD_NT
#define USN_LOAD_NT 0
#endif

/* 16-byte header load (`nt` streaming hint only when USN_LOAD_NT) */
__device__ __forceinline__ uint4 ld_stream(const uint4 *p) {
#if USN_LOAD_NT
  const v4u32 v = __builtin_nontemporal_load(reinterpret_cast<const v4u32 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}

__device__ __forceinline__ uint32_t be16lo(uint32_t v) {  // bytes [0,1] of v as big-endian u16
  return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu);
}

struct Parsed {
  uint32_t status;   // 0 parse fail, 1 IPv4, 2 ARP, 3 EAPOL, 4 later fragment
  uint32_t i0, src, dst, ports;   // PacketInfo words (usn_internal.h)
  uint32_t sport, dport, proto, has_ports, frag_first;
};

/* extract_pkt_info (pkt.rs:158-218) with smoltcp 0.7.0's EthernetFrame /
 * Ipv4Packet::new_checked length rules.  q = 64-byte window, little-endian
 * words; every field offset is a compile-time constant except the L4 ports. */
__device__ __forceinline__ void parse(const uint4 q[4], uint32_t len, const uint8_t *frame,
                                      Parsed &p) {
  p.status = 0; p.i0 = 0; p.src = 0; p.dst = 0; p.ports = 0;
  p.sport = 0; p.dport = 0; p.proto = 0; p.has_ports = 0; p.frag_first = 0;
  if (len < 14) return;                                    // EthernetFrame::new_checked
  const uint32_t w3 = q[0].w;
  const uint32_t et = be16lo(w3);                          // bytes 12..13
  if (et == 0x0806u) { p.status = 2; p.i0 = USN_INFO_ARP; return; }     // pkt.rs:167
  if (et == 0x888Eu) { p.status = 3; p.i0 = USN_INFO_EAPOL; return; }   // pkt.rs:206-213
  if (et != 0x0800u) return;                               // IPv6, 802.1Q, ...: None
  const uint32_t n = len - 14;
  if (n < 20) return;                                      // Ipv4Packet::check_len
  const uint32_t ihl = (w3 >> 16) & 0xFu;                  // byte 14
  const uint32_t hl = ihl * 4;
  const uint32_t w4 = q[1].x, w5 = q[1].y, w6 = q[1].z, w7 = q[1].w;
  const uint32_t w8 = q[2].x, w9 = q[2].y;
  const uint32_t tl = be16lo(w4);                          // bytes 16..17
  if (n < hl || hl > tl || n < tl) return;
  const uint32_t ff = be16lo(w5);                          // bytes 20..21
  p.proto = w5 >> 24;                                      // byte 23
  p.src = __builtin_bswap32(__builtin_amdgcn_alignbyte(w7, w6, 2));   // bytes 26..29
  p.dst = __builtin_bswap32(__builtin_amdgcn_alignbyte(w8, w7, 2));   // bytes 30..33
  if (ff & 0x1FFFu) { p.status = 4; return; }              // frag_offset() > 0: pkt.rs:172
  const uint32_t pr = p.proto;
  const bool port_proto = pr == 6u || pr == 17u || pr == 0x21u || pr == 0x84u || pr == 0x88u;
  p.has_ports = (port_proto && (tl - hl) > 4u) ? 1u : 0u;  // pkt.rs:128-133, 179
  if (p.has_ports) {
    uint32_t a, b;
    if (ihl == 5u) {
      a = w8; b = w9;                                      // ports at bytes 34..37
    } else {                                               // ports at 14+hl: reload (rare)
      a = *reinterpret_cast<const uint32_t *>(frame + 12 + hl);
      b = *reinterpret_cast<const uint32_t *>(frame + 16 + hl);
    }
    p.sport = be16lo(a >> 16);
    p.dport = be16lo(b);
    p.ports = p.sport | (p.dport << 16);
  }
  p.i0 = USN_INFO_IPV4 | (pr << 8) | (p.has_ports << 16);
  p.frag_first = (!(ff & 0x4000u) && (ff & 0x2000u)) ? 1u : 0u;   // pkt.rs:198
  p.status = 1;
}

/* One exact-match probe.  Returns the slot's meta word (0 = miss). */
template <bool LDS>
__device__ __forceinline__ uint32_t probe(const uint4 *T, uint32_t bmask, uint32_t x, uint32_t y,
                                          uint32_t z, uint32_t meta) {
  uint32_t b = usn_key_hash(x, y, z, meta) & bmask;
  for (uint32_t it = 0; it <= bmask; ++it) {
    const uint4 *s = T + b * 4;
    const uint4 s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
    if (s0.x == x && s0.y == y && s0.z == z && (s0.w & USN_KEY_META_MASK) == meta) return s0.w;
    if (s1.x == x && s1.y == y && s1.z == z && (s1.w & USN_KEY_META_MASK) == meta) return s1.w;
    if (s2.x == x && s2.y == y && s2.z == z && (s2.w & USN_KEY_META_MASK) == meta) return s2.w;
    if (s3.x == x && s3.y == y && s3.z == z && (s3.w & USN_KEY_META_MASK) == meta) return s3.w;
    if (!(s3.w & USN_SLOT_VALID)) return 0;                // bucket not full: chain ends
    b = (b + 1) & bmask;
  }
  return 0;
}

/* get_endpoint (endpoint.rs:307-338): key1 = to_match_want_with_src(true),
 * key2 = ..(false) only on a key1 miss; a hit on a NIC-owned rule or on the
 * source itself yields None with no retry.  Returns owner, or -1 with *excl. */
template <bool LDS>
__device__ __forceinline__ int get_endpoint(const uint4 *T, uint32_t bmask, const Parsed &p,
                                            uint32_t src, bool &excl) {
  const uint32_t pres1 = p.has_ports ? (USN_WANT_DPORT | USN_WANT_SRC | USN_WANT_SPORT) : USN_WANT_SRC;
  const uint32_t z1 = p.has_ports ? (p.dport | (p.sport << 16)) : 0u;
  uint32_t w = probe<LDS>(T, bmask, p.dst, p.src, z1, usn_key_meta(p.proto, pres1));
  if (!w) {
    const uint32_t pres2 = p.has_ports ? USN_WANT_DPORT : 0u;
    const uint32_t z2 = p.has_ports ? p.dport : 0u;
    w = probe<LDS>(T, bmask, p.dst, 0u, z2, usn_key_meta(p.proto, pres2));
  }
  excl = false;
  if (!w) return -1;
  const uint32_t owner = w >> 16;
  if ((w & USN_SLOT_NICOWNER) || owner == src) { excl = true; return -1; }
  return (int)owner;
}

/* find_forward for a NIC source (incoming == true), cache handled outside. */
template <bool LDS>
__device__ __forceinline__ uint32_t decide_rx(const uint4 *T, uint32_t bmask, const Parsed &p,
                                              uint32_t src) {
  switch (p.status) {
    case 0: return usn_mkdec(USN_CLS_DROP, USN_R_PARSE, 0xFFFFu);
    case 4: return usn_mkdec(USN_CLS_DROP, USN_R_FRAGMISS, 0xFFFFu) | USN_F_FRAGN | USN_F_HOST;
    case 2:
    case 3: return usn_mkdec(USN_CLS_FLOOD, USN_R_NONE, 0xFFFFu);    // endpoint.rs:199-204
    default: break;
  }
  if ((p.dst >> 24) == 127u) return usn_mkdec(USN_CLS_DROP, USN_R_LOOPBACK, 0xFFFFu);
  bool excl;
  const int e = get_endpoint<LDS>(T, bmask, p, src, excl);
  uint32_t d;
  if (e >= 0) {
    d = usn_mkdec(USN_CLS_EP, USN_R_NONE, (uint32_t)e);
  } else if (p.proto == 17u && p.has_ports && p.sport == 67u && p.dport == 68u) {
    // is_dhcp_answer with no rule: next_dhcp_endpoint.take() is ordered state
    d = usn_mkdec(USN_CLS_DROP, USN_R_DHCP_NONE, 0xFFFFu) | USN_F_DHCP | USN_F_HOST;
  } else {
    d = usn_mkdec(USN_CLS_DROP, excl ? USN_R_EXCLUDED : USN_R_NOMATCH, 0xFFFFu);
  }
  if (p.frag_first) d |= USN_F_FRAG1 | USN_F_HOST;
  return d;
}

__device__ __forceinline__ uint32_t dec_bin(uint32_t d, uint32_t n_ep) {
  const uint32_t c = USN_DEC_CLASS(d);
  if (c == USN_CLS_EP) return USN_DEC_EP(d);
  if (c == USN_CLS_NIC) return USN_BIN_NIC(n_ep);
  if (c == USN_CLS_FLOOD) return USN_BIN_FLOOD(n_ep);
  return USN_BIN_DROP(n_ep);
}

/* --------------------------------------------------------------------------- */
/* LDS layout of a block                                                        */
struct Lds {
  uint16_t *cnt;      // [NSEG][nbins]: per-segment counts, then segment prefixes
  uint16_t *bstart;   // [nbins]: tile totals, then bin start slots
  uint16_t *order;    // [TILE]
  uint16_t *fbin;     // [TILE]: bin of each tile-local frame
  uint32_t *scratch;  // [16]
  uint4 *table;       // staged rule table (optional)
  uint4 *stage;       // dense layout: 4 KiB per wave for the header transpose
};

__host__ __device__ inline size_t lds_core_bytes(uint32_t nbins) {
  size_t cnt = (size_t)NSEG * nbins * 2;
  size_t bst = (size_t)nbins * 2;
  size_t b = cnt + bst;
  b = (b + 15) & ~(size_t)15;
  b += TILE * 2 + TILE * 2 + 16 * 4;
  return (b + 15) & ~(size_t)15;
}

#define STAGE_BYTES ((NTHREADS / 64) * 4096)

__device__ __forceinline__ Lds carve(uint8_t *smem, uint32_t nbins, bool dense = false) {
  Lds L;
  L.cnt = reinterpret_cast<uint16_t *>(smem);
  L.bstart = L.cnt + (size_t)NSEG * nbins;
  size_t off = ((size_t)NSEG * nbins * 2 + (size_t)nbins * 2 + 15) & ~(size_t)15;
  L.order = reinterpret_cast<uint16_t *>(smem + off);
  L.fbin = L.order + TILE;
  L.scratch = reinterpret_cast<uint32_t *>(L.fbin + TILE);
  L.stage = reinterpret_cast<uint4 *>(smem + lds_core_bytes(nbins));
  L.table = L.stage + (dense ? (NTHREADS / 64) * 256 : 0);
  return L;
}

__device__ __forceinline__ uint64_t lanemask_lt(uint32_t lane) {
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

/* Inclusive scan of v across the 64 lanes of a wave. */
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

/* Exclusive scan of one value per thread over the block; returns the
 * exclusive prefix, *total = block sum.  Uses scratch[0..4]. */
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *scratch,
                                                    uint32_t *total) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t inc = wave_incl_scan(v, lane);
  if (lane == 63) scratch[wave] = inc;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < NTHREADS / 64; ++w) {
    const uint32_t s = scratch[w];
    if (w < wave) base += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + inc - v;
}

/* Stable counting sort of the tile by bin.  bins[r] is the bin of tile-local
 * frame r*256 + tid (valid when < nt).  Leaves L.order sorted, L.fbin filled. */
__device__ void tile_sort(const uint32_t bins[ROUNDS], uint32_t nt, uint32_t nbins, const Lds &L) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (uint32_t i = tid; i < NSEG * nbins; i += NTHREADS) L.cnt[i] = 0;
  __syncthreads();
  uint32_t rank[ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    const bool valid = local < nt;
    const uint32_t s = r * (NTHREADS / 64) + wave;        // 64-frame segment, index order
    const uint32_t b = bins[r];
    uint64_t remaining = __ballot(valid);
    rank[r] = 0;
    while (remaining) {                                    // one pass per distinct bin
      const uint32_t leader = (uint32_t)__builtin_ctzll(remaining);
      const uint32_t lb = __builtin_amdgcn_readlane(b, leader);
      const bool mine = valid && b == lb;
      const uint64_t m = __ballot(mine);
      if (mine) rank[r] = (uint32_t)__popcll(m & lanemask_lt(lane));
      if (lane == leader) L.cnt[s * nbins + lb] = (uint16_t)__popcll(m);
      remaining &= ~m;
    }
    if (valid) L.fbin[local] = (uint16_t)b;
  }
  __syncthreads();
  // column scan over segments: cnt[s][b] := frames of bin b in segments < s
  for (uint32_t b = tid; b < nbins; b += NTHREADS) {
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t s = 0; s < NSEG; ++s) {
      const uint32_t c = L.cnt[s * nbins + b];
      L.cnt[s * nbins + b] = (uint16_t)acc;
      acc += c;
    }
    L.bstart[b] = (uint16_t)acc;
  }
  __syncthreads();
  // exclusive scan of bin totals: each thread owns a contiguous chunk of bins
  const uint32_t per = (nbins + NTHREADS - 1) / NTHREADS;
  const uint32_t b0 = tid * per;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; ++k)
    if (b0 + k < nbins) sum += L.bstart[b0 + k];
  uint32_t total;
  uint32_t run = block_excl_scan(sum, L.scratch, &total);
  for (uint32_t k = 0; k < per; ++k)
    if (b0 + k < nbins) {
      const uint32_t c = L.bstart[b0 + k];
      L.bstart[b0 + k] = (uint16_t)run;
      run += c;
    }
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    if (local < nt) {
      const uint32_t s = r * (NTHREADS / 64) + wave;
      const uint32_t b = bins[r];
      const uint32_t dest = L.bstart[b] + L.cnt[s * nbins + b] + rank[r];
      L.order[dest] = (uint16_t)local;
    }
  }
  __syncthreads();
}

/* Write the sorted tile (coalesced) and its bin runs; returns n_runs. */
__device__ uint32_t tile_emit(uint32_t tile, uint32_t nt, const Lds &L, uint16_t *order_out,
                              uint32_t *runs_out) {
  const uint32_t tid = threadIdx.x;
  const uint32_t p0 = tid * ROUNDS;
  uint16_t *dst = order_out + (size_t)tile * TILE;
  if (p0 + ROUNDS <= nt) {
    const uint2 v = *reinterpret_cast<const uint2 *>(L.order + p0);
    *reinterpret_cast<uint2 *>(dst + p0) = v;
  } else {
    for (uint32_t k = 0; k < ROUNDS; ++k)
      if (p0 + k < nt) dst[p0 + k] = L.order[p0 + k];
  }
  uint32_t heads = 0;
  uint32_t hb[ROUNDS];
#pragma unroll
  for (uint32_t k = 0; k < ROUNDS; ++k) {
    const uint32_t p = p0 + k;
    hb[k] = 0xFFFFFFFFu;
    if (p < nt) {
      const uint32_t b = L.fbin[L.order[p]];
      const bool head = p == 0 || L.fbin[L.order[p - 1]] != b;
      if (head) { hb[k] = b; ++heads; }
    }
  }
  uint32_t n_runs;
  uint32_t pos = block_excl_scan(heads, L.scratch, &n_runs);
  uint32_t *rdst = runs_out + (size_t)tile * TILE;
#pragma unroll
  for (uint32_t k = 0; k < ROUNDS; ++k)
    if (hb[k] != 0xFFFFFFFFu) rdst[pos++] = (hb[k] << 16) | (p0 + k);
  return n_runs;
}

/* --------------------------------------------------------------------------- */
/* Carried-in decision cache for this batch, resolved by all threads of
 * workgroup 0: the state after the last cache-touching frame of the previous
 * batch (its tiles are scanned in parallel), or that batch's own carried-in
 * state when none of its frames touched the cache.  out[0..5] in LDS. */
__device__ void resolve_carry(const ClassifyArgs &a, uint32_t *out, uint32_t *scratch) {
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const bool chain = a.carry_mode == CARRY_CHAIN && !(a.prev_summary->flags & USN_S_COUT);
  uint32_t best = 0;   // 1 + index of the last previous tile with a touching frame
  if (chain) {
    for (uint32_t t = tid; t < a.prev_ntiles; t += NTHREADS)
      if (a.prev_tiles[t].last_state & USN_TS_HAS) best = t + 1;
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) best = max(best, (uint32_t)__shfl_xor(best, d, 64));
    if (tid == 0) scratch[8] = 0;
    __syncthreads();
    if (lane == 0 && best) atomicMax(&scratch[8], best);
    __syncthreads();
    best = scratch[8];
  }
  if (tid != 0) return;
  uint32_t st = 0, dst = 0, info[4] = {0, 0, 0, 0};
  if (a.carry_mode == CARRY_EXPLICIT) {
    st = a.cin_state; dst = a.cin_dst;
    for (int k = 0; k < 4; ++k) info[k] = a.cin_info[k];
  } else if (a.carry_mode == CARRY_CHAIN) {
    const usn_summary *ps = a.prev_summary;
    if (!chain) {                                   // finalize wrote the authoritative state
      st = ps->cout_state; dst = ps->cout_dst;
      for (int k = 0; k < 4; ++k) info[k] = ps->cout_info[k];
    } else if (best) {
      const usn_tile_hdr &h = a.prev_tiles[best - 1];
      if ((h.last_state & USN_TS_RETAINED) && !(h.last_state & USN_TS_UNKNOWN)) {
        st = USN_CS_VALID; dst = h.last_dst;
        for (int k = 0; k < 4; ++k) info[k] = h.last_info[k];
      }
    } else {
      st = ps->cin_state; dst = ps->cin_dst;
      for (int k = 0; k < 4; ++k) info[k] = ps->cin_info[k];
    }
  }
  out[0] = st; out[1] = dst;
  for (int k = 0; k < 4; ++k) out[2 + k] = info[k];
}

/* Decision for a carried PacketInfo X under the current table (rx). */
template <bool LDS>
__device__ uint32_t decide_info_rx(const uint4 *T, uint32_t bmask, const uint32_t *info,
                                   uint32_t src) {
  Parsed p;
  p.status = 1; p.i0 = info[0]; p.src = info[1]; p.dst = info[2]; p.ports = info[3];
  p.proto = (info[0] >> 8) & 0xFFu; p.has_ports = (info[0] >> 16) & 1u;
  p.sport = info[3] & 0xFFFFu; p.dport = info[3] >> 16; p.frag_first = 0;
  return decide_rx<LDS>(T, bmask, p, src);
}

/* --------------------------------------------------------------------------- */
/* Swizzled 16-byte slot of part j of frame f in a wave's 4 KiB stage: the
 * XOR with (f >> 2) & 3 makes both the linear writes and the per-frame reads
 * of ds_*_b128 bank-conflict free. */
__device__ __forceinline__ uint32_t stage_slot(uint32_t f, uint32_t j) {
  return 4 * f + (j ^ ((f >> 2) & 3u));
}

template <bool LDS, bool DENSE>
__global__ __launch_bounds__(NTHREADS) void classify_rx_kernel(ClassifyArgs a) {
  extern __shared__ __align__(16) uint8_t smem[];
  const Lds L = carve(smem, a.nbins, DENSE);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t tile = blockIdx.x;
  const uint64_t base = (uint64_t)tile * TILE;
  const uint32_t nt = (uint32_t)min((uint64_t)TILE, a.n - base);

  // ---- issue every header load of this thread first (16 x 16 B + 4 lengths)
  uint4 q[ROUNDS][4];
  uint32_t len[ROUNDS];
  const uint8_t *fp[ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    const uint64_t i = base + (local < nt ? local : 0);
    fp[r] = a.offsets ? a.frames + a.offsets[i] : a.frames + i * a.stride;
    if (DENSE) {
      // 64 contiguous 64-byte frames per wave and round: 4 fully coalesced
      // 1 KiB wave loads; frame lane/4 + 16k arrives in lane (4 lanes each)
      const uint64_t f0 = base + r * NTHREADS + wave * 64;
      const uint4 *chunk = reinterpret_cast<const uint4 *>(a.frames + f0 * 64);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t f = f0 + 16 * k + (lane >> 2);
        q[r][k] = f < a.n ? ld_stream(chunk + 64 * k + lane) : make_uint4(0, 0, 0, 0);
      }
    } else {
      const uint4 *w = reinterpret_cast<const uint4 *>(fp[r]);
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) q[r][k] = ld_stream(w + k);
    }
    len[r] = local < nt ? (uint32_t)a.lens[i] : 0u;
  }

  // ---- stage the rule table into LDS
  const uint4 *T = a.table;
  if (LDS) {
    for (uint32_t k = tid; k < a.table_slots; k += NTHREADS) L.table[k] = a.table[k];
    T = L.table;
  }
  __syncthreads();

  // ---- carried-in cache (block 0): stale check against the current table
  __shared__ uint32_t s_carry[8];
  if (tile == 0) {
    resolve_carry(a, s_carry, L.scratch);
    if (tid == 0) {
      const uint32_t st = s_carry[0], dst = s_carry[1];
      uint32_t flags = 0;
      if (st & USN_CS_VALID) {
        const uint32_t now = decide_info_rx<LDS>(T, a.bucket_mask, s_carry + 2, a.src);
        if ((now & USN_PARITY_MASK) != (dst & USN_PARITY_MASK)) flags |= USN_S_STALE;
      }
      s_carry[6] = flags;
      s_carry[7] = TILE;   // first break in tile 0 (min over frames), TILE = none
      usn_summary *S = a.summary;
      S->cin_state = st; S->cin_dst = dst;
      for (int k = 0; k < 4; ++k) S->cin_info[k] = s_carry[2 + k];
      S->n_frames = (uint32_t)a.n; S->n_tiles = a.ntiles;
    }
    __syncthreads();
  }

  // ---- parse + decide
  uint32_t dec[ROUNDS], bins[ROUNDS], touch[ROUNDS], inf[ROUNDS][4];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    if (DENSE) {   // wave-private transpose through LDS: lane <- its own frame
      uint4 *st = L.stage + wave * 256;
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) st[stage_slot(16 * k + (lane >> 2), lane & 3)] = q[r][k];
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) q[r][k] = st[stage_slot(lane, k)];
    }
#if USN_ABL_LOADONLY
    const uint32_t x = q[r][0].x ^ q[r][1].y ^ q[r][2].z ^ q[r][3].w ^ len[r];
    dec[r] = usn_mkdec(USN_CLS_DROP, USN_R_PARSE, x & 0xFFFF);
    touch[r] = 0;
    inf[r][0] = inf[r][1] = inf[r][2] = inf[r][3] = 0;
    continue;
#endif
    Parsed p;
    parse(q[r], len[r], fp[r], p);
    dec[r] = decide_rx<LDS>(T, a.bucket_mask, p, a.src);
    // cache touch: 0 none (parse failure), 1 retains Some(info), 2 leaves None, 3 unknown
    touch[r] = p.status == 0 ? 0u
             : p.status == 4 ? 3u
             : (p.status == 1 && (p.dst >> 24) != 127u) ? 1u : 2u;
    inf[r][0] = p.i0; inf[r][1] = p.src; inf[r][2] = p.dst; inf[r][3] = p.ports;
    if (r * NTHREADS + tid >= nt) touch[r] = 0;
  }

  // ---- stale carried cache: frames before the first break take the cached
  //      decision (endpoint.rs:186-191); only tile 0 is resolved here.
  if (tile == 0 && (s_carry[6] & USN_S_STALE)) {
    uint32_t fb = TILE;
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) {
      const uint32_t local = r * NTHREADS + tid;
      if (touch[r] == 0) continue;
      const bool same = touch[r] == 1 && inf[r][0] == s_carry[2] && inf[r][1] == s_carry[3] &&
                        inf[r][2] == s_carry[4] && inf[r][3] == s_carry[5];
      if (!same) fb = min(fb, local);   // later fragments also stop the device prefix
    }
    atomicMin(&s_carry[7], fb);
    __syncthreads();
    const uint32_t first = s_carry[7];
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) {
      const uint32_t local = r * NTHREADS + tid;
      if (local < first && touch[r] == 1)
        dec[r] = (s_carry[1] & USN_PARITY_MASK) | USN_F_CACHE | (dec[r] & USN_F_HOST) |
                 (dec[r] & (USN_F_FRAG1 | USN_F_DHCP));
    }
    if (tid == 0) {
      uint32_t f = s_carry[6];
      if (first >= nt && a.n > TILE) f |= USN_S_STALE_EXTENDS;
      // a later fragment at the break: the host decides whether the prefix goes on
      a.summary->first_break = first;
      s_carry[6] = f;
    }
  }
  if (tile == 0 && tid == 0) {
    a.summary->flags = s_carry[6];
    if (!(s_carry[6] & USN_S_STALE)) a.summary->first_break = 0xFFFFFFFFu;
  }

  // ---- decisions out (coalesced) + host list
  uint32_t nhost = 0;
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    if (local < nt) {
      a.decisions[base + local] = dec[r];
      nhost += (dec[r] & USN_F_HOST) ? 1u : 0u;
    }
    bins[r] = dec_bin(dec[r], a.n_ep);
  }

  // ---- per-tile class counts and host list
  __shared__ uint32_t s_cls[4];
  __shared__ uint32_t s_last;
  if (tid < 4) s_cls[tid] = 0;
  if (tid == 0) s_last = 0;
  __syncthreads();
  uint32_t cc[4] = {0, 0, 0, 0};
  uint32_t last = 0;   // 1 + tile-local index of the last cache-touching frame
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    if (local < nt) cc[USN_DEC_CLASS(dec[r])]++;
    if (touch[r]) last = local + 1;
  }
#pragma unroll
  for (uint32_t c = 0; c < 4; ++c) {
    uint32_t v = cc[c];
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == 0 && v) atomicAdd(&s_cls[c], v);
  }
  uint32_t lm = last;
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) lm = max(lm, (uint32_t)__shfl_xor(lm, d, 64));
  if (lane == 0 && lm) atomicMax(&s_last, lm);
  uint32_t total_host;
  uint32_t hpos = block_excl_scan(nhost, L.scratch, &total_host);
  if (nhost) {
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) {
      const uint32_t local = r * NTHREADS + tid;
      if (local < nt && (dec[r] & USN_F_HOST)) a.host_list[(size_t)tile * TILE + hpos++] = (uint32_t)(base + local);
    }
  }

  // ---- stable per-endpoint order of the tile
#if USN_ABL_NOSORT || USN_ABL_LOADONLY
  const uint32_t n_runs = 0;
#else
  tile_sort(bins, nt, a.nbins, L);
  const uint32_t n_runs = tile_emit(tile, nt, L, a.order, a.runs);
#endif

  // ---- tile header
  const uint32_t lastp = s_last;
  if (lastp) {
    const uint32_t li = lastp - 1;
    if ((li & (NTHREADS - 1)) == tid) {
      const uint32_t r = li / NTHREADS;
      usn_tile_hdr *H = a.tiles + tile;
      uint32_t st = USN_TS_HAS;
#pragma unroll
      for (uint32_t rr = 0; rr < ROUNDS; ++rr) {
        if (rr != r) continue;
        if (touch[rr] == 1) st |= USN_TS_RETAINED;
        if (touch[rr] == 3) st |= USN_TS_UNKNOWN;
        H->last_dst = dec[rr] & USN_PARITY_MASK;
        for (int k = 0; k < 4; ++k) H->last_info[k] = inf[rr][k];
      }
      H->last_state = st;
      H->last_idx = (uint32_t)(base + li);
    }
  }
  if (tid == 0) {
    usn_tile_hdr *H = a.tiles + tile;
    H->n_frames = (uint16_t)nt;
    H->n_runs = (uint16_t)n_runs;
    H->n_host = (uint16_t)total_host;
    H->_reserved = 0;
    for (int c = 0; c < 4; ++c) H->class_count[c] = (uint16_t)s_cls[c];
    if (!lastp) { H->last_state = 0; H->last_dst = 0; H->last_idx = 0xFFFFFFFFu; }
  }
}

/* Rebuild order / runs / class counts of tiles from patched decisions. */
__global__ __launch_bounds__(NTHREADS) void resort_kernel(ClassifyArgs a, uint32_t t0) {
  extern __shared__ __align__(16) uint8_t smem[];
  const Lds L = carve(smem, a.nbins);
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t tile = t0 + blockIdx.x;
  const uint64_t base = (uint64_t)tile * TILE;
  const uint32_t nt = (uint32_t)min((uint64_t)TILE, a.n - base);
  __shared__ uint32_t s_cls[4];
  if (tid < 4) s_cls[tid] = 0;
  uint32_t bins[ROUNDS];
  uint32_t cc[4] = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    const uint32_t d = local < nt ? a.decisions[base + local] : 0u;
    bins[r] = dec_bin(d, a.n_ep);
    if (local < nt) cc[USN_DEC_CLASS(d)]++;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t c = 0; c < 4; ++c) {
    uint32_t v = cc[c];
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == 0 && v) atomicAdd(&s_cls[c], v);
  }
  tile_sort(bins, nt, a.nbins, L);
  const uint32_t n_runs = tile_emit(tile, nt, L, a.order, a.runs);
  if (tid == 0) {
    a.tiles[tile].n_runs = (uint16_t)n_runs;
    for (int c = 0; c < 4; ++c) a.tiles[tile].class_count[c] = (uint16_t)s_cls[c];
  }
}

/* --------------------------------------------------------------------------- */
#define LDS_TABLE_MAX_BYTES (32u * 1024u)

bool table_fits_lds(uint32_t nbins, uint32_t table_slots) {
  return (size_t)table_slots * 16 <= LDS_TABLE_MAX_BYTES &&
         lds_core_bytes(nbins) + STAGE_BYTES + (size_t)table_slots * 16 <= 64u * 1024u;
}

size_t classify_lds_bytes(uint32_t nbins, uint32_t table_slots, bool table_in_lds, bool dense) {
  return lds_core_bytes(nbins) + (dense ? STAGE_BYTES : 0) +
         (table_in_lds ? (size_t)table_slots * 16 : 0);
}

#ifndef USN_DENSE
#define USN_DENSE 1
#endif

hipError_t launch_classify(const ClassifyArgs &a, hipStream_t stream) {
  if (a.ntiles == 0) return hipSuccess;
  const bool in_lds = table_fits_lds(a.nbins, a.table_slots);
  const bool dense = USN_DENSE && a.stride == 64 && a.offsets == nullptr;
  const size_t lds = classify_lds_bytes(a.nbins, a.table_slots, in_lds, dense);
  const dim3 g(a.ntiles), b(NTHREADS);
  if (in_lds && dense) hipLaunchKernelGGL((classify_rx_kernel<true, true>), g, b, lds, stream, a);
  else if (in_lds) hipLaunchKernelGGL((classify_rx_kernel<true, false>), g, b, lds, stream, a);
  else if (dense) hipLaunchKernelGGL((classify_rx_kernel<false, true>), g, b, lds, stream, a);
  else hipLaunchKernelGGL((classify_rx_kernel<false, false>), g, b, lds, stream, a);
  return hipGetLastError();
}

hipError_t launch_resort(const ClassifyArgs &a, uint32_t t0, uint32_t t1, hipStream_t stream) {
  if (t1 <= t0) return hipSuccess;
  const size_t lds = lds_core_bytes(a.nbins);
  hipLaunchKernelGGL(resort_kernel, dim3(t1 - t0), dim3(NTHREADS), lds, stream, a, t0);
  return hipGetLastError();
}

}  // namespace usn
