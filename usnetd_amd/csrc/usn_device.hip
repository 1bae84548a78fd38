/*
 * usn_device.hip -- gfx950 kernels of the usnetd match path.
 *
 * classify_rx_kernel: one workgroup per tile of USN_TILE = 1024 frames, 512
 * threads (two rounds per lane; the 256-thread build, four rounds, only where
 * its smaller header stage is what lets the rule image fit LDS).  Per frame:
 *   1. the header window + the 2-byte length: fixed-stride layouts stream
 *      bytes 12..43 into a wave-private LDS stage by LDS-DMA (glds, `nt`),
 *      round 1 in flight while round 0 is parsed; offsets layouts and wide
 *      strides use per-lane 16-byte register loads;
 *   2. extract_pkt_info in registers, branch-free    /root/reference/src/pkt.rs:158-218
 *   3. get_endpoint: perfect-hash probes of the rule image (whole image in
 *      LDS when it fits; else displacements in LDS and slots from L2: one U
 *      slot answers key1 and key2, X only for shared projections)
 *                                                      /root/reference/src/endpoint.rs:307-338
 *   4. the decision of find_forward for a NIC source    /root/reference/src/endpoint.rs:172-296
 *   5. the tile's frames per bin (LDS histogram) -> its count row; frames
 *      that need ordered state are listed for usn_finalize.
 * tx_kernel: the sending-endpoint direction in one launch (learning, the
 * inner L2 bridge, epoch-tagged cross-tile hand-offs; §3.4).
 * scan_kernel + scatter_kernel: the device-wide per-endpoint lists (index,
 * bin_off) from the decisions and the count rows (§3.2): stable, frame order
 * inside each bin; a count row that disagrees with the decisions is reported
 * (diag USN_DIAG_LISTS -> usn_finalize USN_ELIST), never hidden.  About one
 * chunk per CU; a launch whose chunks are all resident and whose rows are
 * few skips the scan (each chunk sums its batch's rows: scatter_kernel<TC,
 * true>; the plan is usn_host.cpp scatter_plan).
 * No MFMA: byte parsing and hash probing, bounded by HBM reads.
 *
 * Order-dependent state (fragment map, DHCP next endpoint, a stale carried
 * cache entry) never changes a decision silently: frames that need it carry
 * USN_F_HOST and are listed per tile for the ordered host stage (usn_finalize).
 */
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "usn_internal.h"
#include "usn_kernels.h"

/* The file is compiled twice into libusn.so: namespace usn (256 threads per
 * tile) and, for rule tables in global memory, usn_t512 (-DUSN_NTHREADS=512
 * -DUSN_NS=usn_t512: twice the waves per tile, half the probe chains per
 * lane). */
#ifndef USN_NS
#define USN_NS usn
#endif

namespace USN_NS {
using namespace ::usn;

#define TILE USN_TILE
#ifndef USN_NTHREADS
#define USN_NTHREADS 256
#endif
#define NTHREADS USN_NTHREADS   /* 256, 512 or 1024 threads per 1024-frame tile */
#define ROUNDS (TILE / NTHREADS)
#define NSEG (TILE / 64)
#ifndef USN_STAGE32   /* header stage: bytes 12..43 of a frame (2 parts), else 0..47 (3) */
#define USN_STAGE32 1
#endif
#define GLDS_PARTS (USN_STAGE32 ? 2u : 3u)       /* 16-byte LDS-DMA parts per frame and round */
#define GLDS_OFF (USN_STAGE32 ? 12u : 0u)        /* first byte of a frame in the stage */
#ifndef USN_STAGE_SLOTS   /* A/B: 16-byte slots per wave and round (round 4: 192, a sort's counts
                             shared the stage; nothing else uses it since the device-wide lists) */
#define USN_STAGE_SLOTS (64u * GLDS_PARTS)
#endif
#define STAGE_ROUND_SLOTS (USN_STAGE_SLOTS)      /* 16 KiB at 512 threads and 2 parts: with c5's 16 KiB
                                                    of displacements, 4 workgroups per CU instead of 3 */
#define MAX_NBITS 13   /* nbins <= USN_MAX_ENDPOINTS + 3 <= 8192 */
#define LDS_TABLE_MAX_BYTES (32u * 1024u)   /* rule images up to 32 KiB live in LDS */
/* the LDS copy of the image, rounded up to whole 64-unit glds chunks */
__host__ __device__ inline uint32_t table_lds_units(uint32_t units) { return (units + 63) & ~63u; }

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

/* Diagnostic build only (-DUSN_STAMPS=1, tools/stamps.py): wave 0 of every
 * workgroup records the global 100 MHz clock at phase boundaries.  The stamps
 * go to their own buffer; no output depends on them. */
#ifndef USN_STAMPS
#define USN_STAMPS 0
#endif
#if USN_STAMPS
#define USN_NSTAMP 16
/* slots 0..16383: the classify / tx kernels' workgroups; 16384..32767: the
 * scatter kernel's (a classify call runs both) */
__device__ unsigned long long usn_stamp_buf[2 * 16384 * USN_NSTAMP];
/* stamps live in registers until the end: a global store per stamp would
 * queue behind the header loads and time the memory queue instead */
#ifndef USN_STAMP_MIN   /* 1: only the first and last stamp (registers as in the product) */
#define USN_STAMP_MIN 0
#endif
#define STAMP(k)                                                                 \
  do {                                                                           \
    if (!USN_STAMP_MIN || (k) == 0 || (k) == 11) {                               \
      __builtin_amdgcn_sched_barrier(0);                                         \
      stamp_t[(k)] = wall_clock64();                                             \
      __builtin_amdgcn_sched_barrier(0);                                         \
    }                                                                            \
  } while (0)
#define STAMP_DECL unsigned long long stamp_t[12] = {0};
#define STAMP_FLUSH_AT(slot)                                                     \
  do {                                                                           \
    if (threadIdx.x == 0)                                                        \
      for (int k_ = 0; k_ < 12; ++k_)                                            \
        usn_stamp_buf[((slot) & 32767) * USN_NSTAMP + k_] = stamp_t[k_];         \
  } while (0)
#define STAMP_FLUSH() STAMP_FLUSH_AT(blockIdx.x)
#define STAMP_FLUSH_SCATTER(slot) STAMP_FLUSH_AT(16384 + ((slot) & 16383))
#else
#define STAMP(k) do { } while (0)
#define STAMP_DECL
#define STAMP_FLUSH() do { } while (0)
#define STAMP_FLUSH_AT(slot) do { } while (0)
#define STAMP_FLUSH_SCATTER(slot) do { } while (0)
#endif

/* The wrong-result ablations of rounds 2-5 (no probes, load floor, no X,
 * one U line, scatter without ranks / write-out) were removed from this
 * source in round 6; git history keeps them (tools/abl.py builds knobs that
 * keep results exact).  The one knob left that breaks the kernel on purpose
 * is the ISA test's: those builds define USN_AB_BUILD=1 (tests/isa_check.py);
 * a product build that sets it fails here. */
#ifndef USN_AB_BUILD
#define USN_AB_BUILD 0
#endif
#ifndef USN_ISA_PERTURB   /* tests/test_isa_waits.py only: 1 an extra load, 2 a stale wait count */
#define USN_ISA_PERTURB 0
#endif
static_assert(USN_AB_BUILD || !USN_ISA_PERTURB,
              "the ISA test's perturbation in a build without USN_AB_BUILD=1");
/* tx wave priority (s_setprio; results unchanged): a tile's waves at the
 * highest priority while they issue its header loads, then 0, and 1 from its
 * phase 2 on.  8-ring grid 0.3177 -> 0.3115 ms (three runs each, one process
 * per run, profiles/r06/r06m, r06n).  Measured and dropped:
 * wave 0 alone raised, priority rising with every phase, phase 2 at 2, and
 * the same ideas in the rx classify and the scatter (no change).
 * USN_AB_TXPRIO=0 (tools/abl_flags.sh) builds the kernel without it. */
#ifndef USN_AB_TXPRIO
#define USN_AB_TXPRIO 1
#endif
#define USN_PRIO(cond, p) do { if (cond) __builtin_amdgcn_s_setprio(p); } while (0)

/* 16-byte header load, default cache policy (the `nt` hint was slower on
 * these per-lane loads: c3 and the tx kernel, profiles/r02cp, r04/r04at) */
__device__ __forceinline__ uint4 ld_stream(const uint4 *p) { return *p; }

__device__ __forceinline__ uint32_t be16lo(uint32_t v) {  // bytes [0,1] of v as big-endian u16
  return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu);
}

struct Parsed {
  uint32_t status;   // 0 parse fail, 1 IPv4, 2 ARP, 3 EAPOL, 4 later fragment,
                     // 5 IPv4 whose L4 ports lie past the batch window (the host parses it)
  uint32_t i0, src, dst, ports;   // PacketInfo words (usn_internal.h)
  uint32_t sport, dport, proto, has_ports, frag_first;
};

/* extract_pkt_info (pkt.rs:158-218) with smoltcp 0.7.0's EthernetFrame /
 * Ipv4Packet::new_checked length rules, computed for every lane with selects
 * (no divergent early exits).  q = 64-byte window as little-endian words;
 * `window` = readable bytes at `frame` (never read past: a frame whose ports
 * end beyond it gets status 5). */
__device__ __forceinline__ void parse(const uint4 q[4], uint32_t len, const uint8_t *frame,
                                      uint32_t window, Parsed &p) {
  const uint32_t w3 = q[0].w, w4 = q[1].x, w5 = q[1].y, w6 = q[1].z, w7 = q[1].w;
  const uint32_t w8 = q[2].x, w9 = q[2].y;
  const uint32_t et = be16lo(w3);                                    // bytes 12..13
  const uint32_t ihl = (w3 >> 16) & 0xFu, hl = ihl * 4;              // byte 14
  const uint32_t tl = be16lo(w4);                                    // bytes 16..17
  const uint32_t ff = be16lo(w5);                                    // bytes 20..21
  const uint32_t pr = w5 >> 24;                                      // byte 23
  const uint32_t n = len - 14;                                       // valid when len >= 14
  const bool eth = len >= 14;                                        // EthernetFrame::new_checked
  const bool ip = eth && et == 0x0800u && len >= 34 &&               // Ipv4Packet::check_len
                  n >= hl && hl <= tl && n >= tl;
  const bool later = ip && (ff & 0x1FFFu) != 0;                      // frag_offset() > 0
  // protocol_has_ports: pr in {6, 17, 33, 132, 136} as two bit-set tests
  // (an || chain of compares became a branch tree)
  const uint32_t ph = pr ^ 0x80u;
  const uint32_t pp_lo = (uint32_t)(0x200020040ull >> (pr & 63u)) & (uint32_t)(pr < 64u);
  const uint32_t pp_hi = (0x110u >> (ph & 31u)) & (uint32_t)(ph < 32u);
  const bool pp = ((pp_lo | pp_hi) & 1u) != 0u;
  const bool has = ip && !later && pp && (tl - hl) > 4u;             // pkt.rs:128-133, 179
  // ports at bytes 34..37, or at 14+hl when IHL != 5 (rare: reloaded).  The
  // reload goes to its own registers (defaults are constants, so nothing
  // waits on this round's headers before the branch) and is waited for in
  // the branch: a wait after the join would be vmcnt(0) on every path and
  // drain the next round's prefetch.  The reload reads bytes 12+hl .. 17+hl
  // (a dword, then the dport halfword), never past the ports' last byte, so
  // `18 + hl <= window` is exactly what it needs for any window (a second
  // dword would end at 19+hl: 1-2 bytes past a window of 66 or 67).
  uint32_t ra = 0, rb = 0;
  const bool beyond = has && 18u + hl > window;                      // ports at 14+hl..17+hl
  const bool reload = has && ihl != 5u && !beyond;
  if (reload) {
    ra = *reinterpret_cast<const uint32_t *>(frame + 12 + hl);
    rb = *reinterpret_cast<const uint16_t *>(frame + 16 + hl);
    __builtin_amdgcn_s_waitcnt(0);
  }
  const uint32_t a = reload ? ra : w8, b = reload ? rb : w9;
  p.sport = has ? be16lo(a >> 16) : 0u;
  p.dport = has ? be16lo(b) : 0u;
  p.ports = p.sport | (p.dport << 16);
  p.has_ports = has ? 1u : 0u;
  p.proto = pr;
  p.src = __builtin_bswap32(__builtin_amdgcn_alignbyte(w7, w6, 2));  // bytes 26..29
  p.dst = __builtin_bswap32(__builtin_amdgcn_alignbyte(w8, w7, 2));  // bytes 30..33
  p.frag_first = (!(ff & 0x4000u) && (ff & 0x2000u)) ? 1u : 0u;      // pkt.rs:198
  const bool arp = eth && et == 0x0806u, eapol = eth && et == 0x888Eu;
  p.status = arp ? 2u : eapol ? 3u : !ip ? 0u : later ? 4u : beyond ? 5u : 1u;
  p.i0 = arp ? USN_INFO_ARP : eapol ? USN_INFO_EAPOL
       : (p.status == 1u ? (USN_INFO_IPV4 | (pr << 8) | (p.has_ports << 16)) : 0u);
}

__device__ __forceinline__ bool slot_is(const uint4 &t, uint32_t x, uint32_t y, uint32_t z,
                                        uint32_t meta) {
  return ((t.x ^ x) | (t.y ^ y) | (t.z ^ z) | ((t.w ^ meta) & USN_KEY_META_MASK)) == 0u;
}

/* ---- rule lookups: the perfect-hash image (usn_internal.h) ----------------
 * A key's probe reads one 16-bit displacement and exactly ONE 16-byte slot,
 * hit or miss: no chains, no tag line.  In LDS (small images) both reads are
 * inline asm: the classify kernel has LDS-DMA header writes in flight, and
 * hipcc cannot tell that the image does not alias the DMA's stage, so plain
 * LDS reads got an s_waitcnt vmcnt(0) that drained the next round's headers;
 * the asm waits for its own reads (lgkmcnt) and nothing else. */
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void *)p;
}

struct PhKeyH {        // a key's hashes for one table
  uint32_t grp, h2, sbase;   // displacement index, slot hash, first slot of its shard
};

__device__ __forceinline__ PhKeyH ph_hash(const usn_ph_table &t, uint32_t x, uint32_t y,
                                          uint32_t z, uint32_t meta) {
  PhKeyH k;
  const uint32_t h1 = usn_ph_h1(x, y, z, meta, t.seed);
  k.grp = usn_ph_group(h1, t.shift, t.g);
  k.sbase = usn_ph_sbase(h1, t.shift, t.m);
  k.h2 = usn_key_hash2(x, y, z, meta, t.seed);
  return k;
}

__device__ __forceinline__ uint32_t ph_hit(const uint4 &sl, uint32_t x, uint32_t y, uint32_t z,
                                           uint32_t meta) {
  return slot_is(sl, x, y, z, meta) ? sl.w : 0u;
}

/* Where a probe reads the image from (template TM of the classify kernel):
 * TM_GLOBAL  displacements and slots from global memory (L1/L2);
 * TM_LDS     the whole image staged in LDS (small tables);
 * TM_DISPLDS the displacement arrays staged in LDS, slots from global
 *            memory: one L2 request per key. */
#ifndef USN_LATE_DMA
#define USN_LATE_DMA 1
#endif
/* tests/test_isa_waits.py builds perturbed variants to show its check fails:
 * 1 = an extra load between a slot read and its wait, 2 = a stale count */
#ifndef USN_ISA_PERTURB
#define USN_ISA_PERTURB 0
#endif
#if USN_ISA_PERTURB == 2
#define USN_U_WAIT0 "2"
#else
#define USN_U_WAIT0 "1"   /* round 0's U slot read: round 1's is the one younger load */
#endif
/* cache policy of the image's slot reads (one scattered 16-byte read per
 * frame and key): A/B knob, "" = default policy.  L1 bypass (" sc1",
 * " sc0 sc1") changed nothing and " nt" made c5's classify 157 -> 264 us per
 * 8M (the U table then leaves L2), profiles/r06/r06t: the probes cost L2
 * requests, one per frame, not L1 line fills. */
#ifndef USN_SLOT_POL
#define USN_SLOT_POL ""
#endif
#ifndef USN_SEQ_K2    /* key2's slot read only where key1 missed (get_endpoint's order) */
#define USN_SEQ_K2 1
#endif
#define TM_GLOBAL 0
#define TM_LDS 1
#define TM_DISPLDS 2

/* Both keys of a frame, issued together: two displacement reads, then two
 * slot reads (one round trip each for a global image).  use1/use2 are
 * wave-uniform (the image's probe_mask).  ph_issue returns with the slot
 * loads ISSUED (s1, s2 not yet waited for), so the caller can put the next
 * round's header DMA behind them: the compiler's wait before the compare is
 * then vmcnt(GLDS_PARTS), not a wait for the DMA.  Dl: the LDS copy of the
 * displacements, indexed like the image (TM_DISPLDS). */
template <int TM, bool ASM_SLOTS = false>
__device__ __forceinline__ void ph_issue(const uint4 *T, const uint16_t *Dl, const ClassifyArgs &a,
                                         bool use1, bool use2, uint32_t x1, uint32_t y1,
                                         uint32_t z1, uint32_t m1, uint32_t x2, uint32_t y2,
                                         uint32_t z2, uint32_t m2, v4u32 &s1, v4u32 &s2) {
  const PhKeyH k1 = ph_hash(a.ph[0], x1, y1, z1, m1);
  const PhKeyH k2 = ph_hash(a.ph[1], x2, y2, z2, m2);
  const uint16_t *D = TM == TM_DISPLDS ? Dl : reinterpret_cast<const uint16_t *>(T);
  uint32_t d1 = 0, d2 = 0;
  if (TM != TM_GLOBAL) {
    // an unused table's read goes to the first displacement (always present)
    const uint32_t di1 = a.ph[0].disp_off + (use1 ? k1.grp : 0u);
    const uint32_t di2 = a.ph[1].disp_off + (use2 ? k2.grp : 0u);
    asm volatile("ds_read_u16 %0, %2\n\tds_read_u16 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(d1), "=&v"(d2)
                 : "v"(lds_addr(D + di1)), "v"(lds_addr(D + di2)));
  } else {
    // branch-free: an unused table reads a valid address (the image always
    // has a unit past its end), so the waits stay straight-line counts
    d1 = D[a.ph[0].disp_off + (use1 ? k1.grp : 0u)];
    d2 = D[a.ph[1].disp_off + (use2 ? k2.grp : 0u)];
  }
  const uint32_t si1 = a.ph[0].slot_off + (use1 ? k1.sbase + usn_ph_slot(k1.h2, d1, a.ph[0].m) : 0u);
  const uint32_t si2 = a.ph[1].slot_off + (use2 ? k2.sbase + usn_ph_slot(k2.h2, d2, a.ph[1].m) : 0u);
  if (TM == TM_LDS) {
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(s1), "=&v"(s2)
                 : "v"(lds_addr(T + si1)), "v"(lds_addr(T + si2)));
  } else if (ASM_SLOTS) {
    // issued here, waited for by ph_slots_wait: hipcc's own wait before the
    // compare would be vmcnt(0), draining the header DMA issued after them
    asm volatile("global_load_dwordx4 %0, %2, off" USN_SLOT_POL "\n\tglobal_load_dwordx4 %1, %3, off" USN_SLOT_POL
                 : "=&v"(s1), "=&v"(s2)
                 : "v"(T + si1), "v"(T + si2)
                 : "memory");
  } else {
    const uint4 a1 = T[si1], a2 = T[si2];
    s1 = v4u32{a1.x, a1.y, a1.z, a1.w};
    s2 = v4u32{a2.x, a2.y, a2.z, a2.w};
  }
}

/* the two ASM_SLOTS loads of ph_issue have landed; `younger` = vector memory
 * instructions issued after them (the next round's 4 header DMAs, or 0) */
template <int YOUNGER>
__device__ __forceinline__ void ph_slots_wait(v4u32 &s1, v4u32 &s2) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(s1), "+v"(s2) : "n"(YOUNGER) : "memory");
}

__device__ __forceinline__ uint32_t ph_hitv(const v4u32 &sl, uint32_t x, uint32_t y, uint32_t z,
                                            uint32_t meta) {
  return ph_hit(make_uint4(sl.x, sl.y, sl.z, sl.w), x, y, z, meta);
}

/* Two-round batched probes (the 512-thread build, global image): both
 * rounds' keys are formed first, then their four displacement reads fly
 * together, then their four slot reads -- two round trips per wave for both
 * rounds instead of two per round.  The loads are inline asm and every wait
 * is an explicit count (hipcc's own waits would be vmcnt(0) and drain the
 * next round's header DMA). */
__device__ __forceinline__ void rx_keys(const Parsed &p, uint32_t &x1, uint32_t &y1, uint32_t &z1,
                                        uint32_t &m1, uint32_t &x2, uint32_t &y2, uint32_t &z2,
                                        uint32_t &m2);

struct RoundKeys {
  uint32_t x1, y1, z1, m1, x2, y2, z2, m2;
  PhKeyH k1, k2;
};

__device__ __forceinline__ void round_keys(const ClassifyArgs &a, const Parsed &p, RoundKeys &k) {
  rx_keys(p, k.x1, k.y1, k.z1, k.m1, k.x2, k.y2, k.z2, k.m2);
  k.k1 = ph_hash(a.ph[0], k.x1, k.y1, k.z1, k.m1);
  k.k2 = ph_hash(a.ph[1], k.x2, k.y2, k.z2, k.m2);
}

__device__ __forceinline__ void asm_disp2(const uint16_t *D, const ClassifyArgs &a, bool use1,
                                          bool use2, const RoundKeys &k, uint32_t &d1,
                                          uint32_t &d2) {
  const uint16_t *p1 = D + a.ph[0].disp_off + (use1 ? k.k1.grp : 0u);
  const uint16_t *p2 = D + a.ph[1].disp_off + (use2 ? k.k2.grp : 0u);
  asm volatile("global_load_ushort %0, %2, off\n\tglobal_load_ushort %1, %3, off"
               : "=&v"(d1), "=&v"(d2) : "v"(p1), "v"(p2) : "memory");
}

__device__ __forceinline__ void asm_slot2(const uint4 *T, const ClassifyArgs &a, bool use1,
                                          bool use2, const RoundKeys &k, uint32_t d1, uint32_t d2,
                                          v4u32 &s1, v4u32 &s2) {
  const uint4 *p1 = T + a.ph[0].slot_off + (use1 ? k.k1.sbase + usn_ph_slot(k.k1.h2, d1, a.ph[0].m) : 0u);
  const uint4 *p2 = T + a.ph[1].slot_off + (use2 ? k.k2.sbase + usn_ph_slot(k.k2.h2, d2, a.ph[1].m) : 0u);
  asm volatile("global_load_dwordx4 %0, %2, off" USN_SLOT_POL "\n\tglobal_load_dwordx4 %1, %3, off" USN_SLOT_POL
               : "=&v"(s1), "=&v"(s2) : "v"(p1), "v"(p2) : "memory");
}

/* one slot read of table t; a lane that does not need it reads the table's
 * first slot, which every such lane of the wave shares: one L2 request */
__device__ __forceinline__ void asm_slot1(const uint4 *T, const usn_ph_table &t, bool need,
                                          const PhKeyH &k, uint32_t d, v4u32 &s) {
  const uint4 *p = T + t.slot_off + (need ? k.sbase + usn_ph_slot(k.h2, d, t.m) : 0u);
  asm volatile("global_load_dwordx4 %0, %1, off" USN_SLOT_POL : "=&v"(s) : "v"(p) : "memory");
}

/* TM_DISPLDS: both displacements from the LDS copy (indexed like the image) */
__device__ __forceinline__ void lds_disp2(const uint16_t *Dl, const ClassifyArgs &a, bool use1,
                                          bool use2, const RoundKeys &k, uint32_t &d1,
                                          uint32_t &d2) {
  const uint16_t *p1 = Dl + a.ph[0].disp_off + (use1 ? k.k1.grp : 0u);
  const uint16_t *p2 = Dl + a.ph[1].disp_off + (use2 ? k.k2.grp : 0u);
  asm volatile("ds_read_u16 %0, %2\n\tds_read_u16 %1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(d1), "=&v"(d2) : "v"(lds_addr(p1)), "v"(lds_addr(p2)) : "memory");
}

template <int YOUNGER>
__device__ __forceinline__ void vm_wait2(uint32_t &d1, uint32_t &d2) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(d1), "+v"(d2) : "n"(YOUNGER) : "memory");
}

template <int TM>
__device__ __forceinline__ void ph_probe2(const uint4 *T, const uint16_t *Dl, const ClassifyArgs &a,
                                          bool use1, bool use2, uint32_t x1, uint32_t y1,
                                          uint32_t z1, uint32_t m1, uint32_t x2, uint32_t y2,
                                          uint32_t z2, uint32_t m2, uint32_t &w1, uint32_t &w2) {
  v4u32 s1, s2;
  ph_issue<TM>(T, Dl, a, use1, use2, x1, y1, z1, m1, x2, y2, z2, m2, s1, s2);
  w1 = use1 ? ph_hitv(s1, x1, y1, z1, m1) : 0u;
  w2 = use2 ? ph_hitv(s2, x2, y2, z2, m2) : 0u;
}

/* One key in table `tb` (0 = K1, 1 = K2); 0 when the table is empty. */
template <bool IN_LDS>
__device__ __forceinline__ uint32_t ph_probe1(const uint4 *T, const ClassifyArgs &a, uint32_t tb,
                                              uint32_t x, uint32_t y, uint32_t z, uint32_t meta) {
  const usn_ph_table &t = a.ph[tb];
  if (!(a.probe_mask & (1u << tb))) return 0u;
  const PhKeyH k = ph_hash(t, x, y, z, meta);
  const uint16_t *D = reinterpret_cast<const uint16_t *>(T);
  if (IN_LDS) {
    uint32_t d;
    asm volatile("ds_read_u16 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(d)
                 : "v"(lds_addr(D + t.disp_off + k.grp)));
    v4u32 sv;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(sv)
                 : "v"(lds_addr(T + t.slot_off + k.sbase + usn_ph_slot(k.h2, d, t.m))));
    return ph_hit(make_uint4(sv.x, sv.y, sv.z, sv.w), x, y, z, meta);
  }
  const uint32_t d = D[t.disp_off + k.grp];
  return ph_hit(T[t.slot_off + k.sbase + usn_ph_slot(k.h2, d, t.m)], x, y, z, meta);
}

/* One key's displacement read of table `tb` (0 = K1, 1 = K2): its hash,
 * whether it is probed at all (use, and the table non-empty), and the read
 * (a key not probed reads the table's first displacement). */
template <bool IN_LDS>
__device__ __forceinline__ void ph_disp_issue(const uint4 *T, const ClassifyArgs &a, int tb, uint32_t x,
                                              uint32_t y, uint32_t z, uint32_t m, bool use, PhKeyH &k,
                                              uint32_t &d, bool &on) {
  typedef __attribute__((address_space(3))) const uint16_t lds_u16;
  const uint16_t *D = reinterpret_cast<const uint16_t *>(T);
  const usn_ph_table &t = a.ph[tb];
  on = use && ((a.probe_mask >> tb) & 1u);
  k = ph_hash(t, x, y, z, m);
  const uint32_t di = t.disp_off + (on ? k.grp : 0u);
  d = IN_LDS ? (uint32_t)((lds_u16 *)D)[di] : (uint32_t)D[di];
}

/* The slot reads of N keys whose displacements were read (ph_disp_issue;
 * keys [0, N1) in K1, the rest in K2), then the hits. */
template <bool IN_LDS, int N, int N1>
__device__ __forceinline__ void ph_slots_hit(const uint4 *T, const ClassifyArgs &a,
                                             const uint32_t (&x)[N], const uint32_t (&y)[N],
                                             const uint32_t (&z)[N], const uint32_t (&m)[N],
                                             const PhKeyH (&k)[N], const uint32_t (&d)[N],
                                             const bool (&on)[N], uint32_t (&w)[N]) {
  typedef __attribute__((address_space(3))) const v4u32 lds_v4;
  uint4 sl[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const usn_ph_table &t = a.ph[i < N1 ? 0 : 1];
    const uint32_t si = t.slot_off + (on[i] ? k[i].sbase + usn_ph_slot(k[i].h2, d[i], t.m) : 0u);
    if (IN_LDS) {
      const v4u32 v = ((lds_v4 *)T)[si];
      sl[i] = make_uint4(v.x, v.y, v.z, v.w);
    } else {
      sl[i] = T[si];
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) w[i] = on[i] ? ph_hit(sl[i], x[i], y[i], z[i], m[i]) : 0u;
}

/* N probes issued together: all N displacement reads, then all N slot
 * reads -- two round trips for the lot instead of two per key.  Keys
 * [0, N1) go to table K1, the rest to K2; use[i] false (or an empty table)
 * gives w[i] = 0 with a harmless read of the table's first entries.  IN_LDS:
 * the image is the LDS copy. */
template <bool IN_LDS, int N, int N1>
__device__ __forceinline__ void ph_probe_many(const uint4 *T, const ClassifyArgs &a,
                                              const uint32_t (&x)[N], const uint32_t (&y)[N],
                                              const uint32_t (&z)[N], const uint32_t (&m)[N],
                                              const bool (&use)[N], uint32_t (&w)[N]) {
  PhKeyH k[N];
  uint32_t d[N];
  bool on[N];
#pragma unroll
  for (int i = 0; i < N; ++i)
    ph_disp_issue<IN_LDS>(T, a, i < N1 ? 0 : 1, x[i], y[i], z[i], m[i], use[i], k[i], d[i], on[i]);
  ph_slots_hit<IN_LDS, N, N1>(T, a, x, y, z, m, k, d, on, w);
}

/* ---- get_endpoint through the projection table U (usn_internal.h) ---------
 * Both lookups of a frame from ONE U slot: U's displacement from the LDS
 * copy (Dl), its slot from L2.  X (the projection's further K1 rules) only
 * when the slot says MORE and its inline K1 rule is not the frame's key1. */
/* E of a parsed frame.  A frame has ports only for the five protocols of
 * protocol_has_ports, so pidx is usn_u_pidx_ports's branch-free form (hipcc
 * turned usn_u_pidx's compare chain into divergent branches) */
__device__ __forceinline__ uint32_t u_key_e(const Parsed &p) {
  return p.has_ports ? (usn_u_pidx_ports(p.proto) << 16 | p.dport) : (5u << 16 | p.proto);
}

/* w1/w2 as a K1/K2 probe would return them, and whether key1 needs X */
__device__ __forceinline__ void u_decode(const v4u32 &s, const Parsed &p, uint32_t E, uint32_t &w1,
                                         uint32_t &w2, bool &need_x) {
  const bool hit = s.x == p.dst && (s.w & USN_U_EMASK) == E;
  const uint32_t o1 = (s.z >> 16) & 0x1FFFu;
  const bool in1 = hit && o1 != USN_U_NONE && s.y == p.src && (s.z & 0xFFFFu) == p.sport;
  w1 = in1 ? usn_u_meta(o1) : 0u;
  w2 = hit ? usn_u_meta(s.w >> 19) : 0u;
  need_x = hit && !in1 && (s.z & USN_U_MORE) != 0u;
}

/* one displacement read from the LDS copy (a lane that skips reads the table's first) */
__device__ __forceinline__ uint32_t lds_disp1(const uint16_t *Dl, const usn_ph_table &t, bool need,
                                              const PhKeyH &k) {
  uint32_t d;
  asm volatile("ds_read_u16 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(d)
               : "v"(lds_addr(Dl + t.disp_off + (need ? k.grp : 0u))) : "memory");
  return d;
}

/* key1 in X for the lanes with `need` (all of this wave's loads are done) */
__device__ __forceinline__ uint32_t x_probe(const uint4 *T, const uint16_t *Dl, const ClassifyArgs &a,
                                            const Parsed &p, bool need) {
  uint32_t x1, y1, z1, m1, x2, y2, z2, m2;
  rx_keys(p, x1, y1, z1, m1, x2, y2, z2, m2);
  const usn_ph_table &t = a.ph[3];
  const PhKeyH k = ph_hash(t, x1, y1, z1, m1);
  const uint32_t d = lds_disp1(Dl, t, need, k);
  v4u32 s;
  asm_slot1(T, t, need, k, d, s);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(s) :: "memory");
  return need ? ph_hitv(s, x1, y1, z1, m1) : 0u;
}

/* key1 of both rounds' frames in X, the two slot reads in flight together */
__device__ __forceinline__ void x_probe2(const uint4 *T, const uint16_t *Dl, const ClassifyArgs &a,
                                         const Parsed &p0, bool need0, const Parsed &p1, bool need1,
                                         uint32_t &w0, uint32_t &w1) {
  const usn_ph_table &t = a.ph[3];
  uint32_t x0, y0, z0, m0, x1, y1, z1, m1, xx, yy, zz, mm;
  rx_keys(p0, x0, y0, z0, m0, xx, yy, zz, mm);
  rx_keys(p1, x1, y1, z1, m1, xx, yy, zz, mm);
  const PhKeyH k0 = ph_hash(t, x0, y0, z0, m0), k1 = ph_hash(t, x1, y1, z1, m1);
  const uint32_t d0 = lds_disp1(Dl, t, need0, k0), d1 = lds_disp1(Dl, t, need1, k1);
  v4u32 s0, s1;
  asm_slot1(T, t, need0, k0, d0, s0);
  asm_slot1(T, t, need1, k1, d1, s1);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(s0), "+v"(s1) :: "memory");
  w0 = need0 ? ph_hitv(s0, x0, y0, z0, m0) : 0u;
  w1 = need1 ? ph_hitv(s1, x1, y1, z1, m1) : 0u;
}

/* both lookups, synchronous (tile 0's carried-cache check, the generic rounds) */
__device__ __forceinline__ void u_probe_sync(const uint4 *T, const uint16_t *Dl, const ClassifyArgs &a,
                                             const Parsed &p, uint32_t &w1, uint32_t &w2) {
  const uint32_t E = u_key_e(p);
  const PhKeyH k = ph_hash(a.ph[2], p.dst, 0u, E, 0u);
  const uint32_t d = lds_disp1(Dl, a.ph[2], true, k);
  v4u32 s;
  asm_slot1(T, a.ph[2], true, k, d, s);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(s) :: "memory");
  bool nx;
  u_decode(s, p, E, w1, w2, nx);
  if (nx) w1 = x_probe(T, Dl, a, p, true);
}

/* find_forward for a NIC source (incoming == true), cache handled outside:
 * ARP/EAPOL -> FLOOD, loopback -> DROP, else get_endpoint (endpoint.rs:307-338:
 * key1 = with src, key2 = without, only on a key1 miss; a hit on a NIC-owned
 * rule or on the source itself is None with no retry), else DHCP / DROP. */
/* key1 = to_match_want_with_src(true), key2 = (false) of a parsed frame (pkt.rs:96-113) */
__device__ __forceinline__ void rx_keys(const Parsed &p, uint32_t &x1, uint32_t &y1, uint32_t &z1,
                                        uint32_t &m1, uint32_t &x2, uint32_t &y2, uint32_t &z2,
                                        uint32_t &m2) {
  const bool has = p.has_ports != 0;
  x1 = p.dst; y1 = p.src; z1 = has ? (p.dport | (p.sport << 16)) : 0u;
  m1 = usn_key_meta(p.proto, has ? (USN_WANT_DPORT | USN_WANT_SRC | USN_WANT_SPORT) : USN_WANT_SRC);
  x2 = p.dst; y2 = 0u; z2 = has ? p.dport : 0u;
  m2 = usn_key_meta(p.proto, has ? USN_WANT_DPORT : 0u);
}

/* the decision from the two probe results (w1 = key1's slot meta, w2 = key2's) */
__device__ __forceinline__ uint32_t decide_rx_w(const ClassifyArgs &a, const Parsed &p, uint32_t w1,
                                                uint32_t w2);

template <int TM>
__device__ __forceinline__ uint32_t decide_rx(const uint4 *T, const uint16_t *Dl,
                                              const ClassifyArgs &a, const Parsed &p) {
  uint32_t w1 = 0, w2 = 0;
  if (TM == TM_DISPLDS && (a.probe_mask & 4u)) {   // Dl holds U's and X's displacements
    u_probe_sync(T, Dl, a, p, w1, w2);
  } else {
    uint32_t x1, y1, z1, m1, x2, y2, z2, m2;
    rx_keys(p, x1, y1, z1, m1, x2, y2, z2, m2);
    ph_probe2<TM>(T, Dl, a, (a.probe_mask & 1u) != 0, (a.probe_mask & 2u) != 0, x1, y1, z1, m1, x2,
                  y2, z2, m2, w1, w2);
  }
  return decide_rx_w(a, p, w1, w2);
}

__device__ __forceinline__ uint32_t decide_rx_w(const ClassifyArgs &a, const Parsed &p, uint32_t w1,
                                                uint32_t w2) {
  const bool has = p.has_ports != 0;
  const uint32_t w = w1 ? w1 : w2;
  const uint32_t owner = w >> 16;
  const bool excl = w && ((w & USN_SLOT_NICOWNER) || owner == a.src);
  const bool dhcp = p.proto == 17u && has && p.sport == 67u && p.dport == 68u;
  const uint32_t d_look =
      (w && !excl) ? usn_mkdec(USN_CLS_EP, USN_R_NONE, owner)
      // is_dhcp_answer: next_dhcp_endpoint.take() (endpoint.rs:262-273) is ordered
      // state, so the host decides -- unless it is None, when it is a plain drop
      : dhcp ? (usn_mkdec(USN_CLS_DROP, USN_R_DHCP_NONE, 0xFFFFu) |
                (a.next_dhcp_set ? (USN_F_DHCP | USN_F_HOST) : 0u))
             : usn_mkdec(USN_CLS_DROP, excl ? USN_R_EXCLUDED : USN_R_NOMATCH, 0xFFFFu);
  uint32_t d =
      p.status == 0u ? usn_mkdec(USN_CLS_DROP, USN_R_PARSE, 0xFFFFu)
      : p.status == 4u ? (usn_mkdec(USN_CLS_DROP, USN_R_FRAGMISS, 0xFFFFu) | USN_F_FRAGN | USN_F_HOST)
      : p.status == 5u ? (usn_mkdec(USN_CLS_DROP, USN_R_WINDOW, 0xFFFFu) | USN_F_HOST)
      : p.status != 1u ? usn_mkdec(USN_CLS_FLOOD, USN_R_NONE, 0xFFFFu)            // ARP/EAPOL
      : (p.dst >> 24) == 127u ? usn_mkdec(USN_CLS_DROP, USN_R_LOOPBACK, 0xFFFFu)   // :205-208
                              : d_look;
  // a first fragment is remembered by extract_pkt_info before any decision
  // (status 5: the host parses the frame and remembers it itself)
  if (p.status == 1u && p.frag_first) d |= USN_F_FRAG1 | USN_F_HOST;
  return d;
}

/* bin of a decision: its endpoint, else NIC / FLOOD / DROP after the
 * endpoints.  Classes 2, 3, 0 map to offsets 0, 1, 2 as (c + 2) & 3: one
 * select, no divergent branch (a branch here kept the compiler from
 * overlapping the loads ahead of it). */
static_assert(USN_CLS_DROP == 0 && USN_CLS_EP == 1 && USN_CLS_NIC == 2 && USN_CLS_FLOOD == 3,
              "dec_bin's class arithmetic");
static_assert(USN_BIN_NIC(0) == 0 && USN_BIN_FLOOD(0) == 1 && USN_BIN_DROP(0) == 2, "bin order");
__device__ __forceinline__ uint32_t dec_bin(uint32_t d, uint32_t n_ep) {
  const uint32_t c = USN_DEC_CLASS(d);
  const uint32_t other = n_ep + ((c + 2u) & 3u);
  const uint32_t m = 0u - (uint32_t)(c == USN_CLS_EP);   // mask form: stays a select
  return other ^ ((other ^ USN_DEC_EP(d)) & m);
}

/* --------------------------------------------------------------------------- */
/* LDS layout of a block                                                        */
struct Lds {
  uint32_t *hist;     // [nbw / 2]: the tile's frames per bin, u16 pairs (tile_hist)
  uint32_t *scratch;  // [16]
  uint16_t *order;    // [TILE] u16 scratch row (the tx kernel's prefix max)
  uint4 *table;       // staged rule table (optional)
};

/* bins of a per-tile count row, rounded up to 8 (16-byte rows) */
__host__ __device__ inline uint32_t bin_words(uint32_t nbins) { return (nbins + 7u) & ~7u; }
__host__ __device__ inline size_t hist_bytes(uint32_t nbins) { return (size_t)bin_words(nbins) * 2; }

/* hist | scratch[16] | order[TILE] | table.  A kernel with a header stage
 * (the GLDS classify) passes it as `stage`: its (unused) order row is then
 * the stage's, which leaves the dynamic LDS to the histogram and the image. */
__host__ __device__ inline size_t lds_head_bytes(uint32_t nbins) { return hist_bytes(nbins) + 16 * 4; }
__host__ __device__ inline size_t lds_core_bytes(uint32_t nbins, bool own_stage = true) {
  return own_stage ? lds_head_bytes(nbins) + TILE * 2 : lds_head_bytes(nbins);
}
__device__ __forceinline__ Lds carve(uint8_t *smem, uint32_t nbins, uint4 *stage = nullptr) {
  Lds L;
  L.hist = reinterpret_cast<uint32_t *>(smem);
  L.scratch = reinterpret_cast<uint32_t *>(smem + hist_bytes(nbins));
  L.order = stage ? reinterpret_cast<uint16_t *>(stage)
                  : reinterpret_cast<uint16_t *>(smem + lds_head_bytes(nbins));
  L.table = reinterpret_cast<uint4 *>(smem + lds_core_bytes(nbins, stage == nullptr));
  return L;
}

__device__ __forceinline__ uint64_t lanemask_lt(uint32_t lane) {
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

/* Inclusive scan of v across the 64 lanes of a wave with DPP row shifts and
 * row broadcasts (VALU only; no LDS permute traffic). */
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
  (void)lane;
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1,3
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2,3
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

/* Largest r (0..ROUNDS-1) among the lanes with `valid`, via one ballot per round. */
__device__ __forceinline__ uint32_t __reduce_max_rounds(uint32_t r, bool valid) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t k = 1; k < ROUNDS; ++k)
    if (__ballot(valid && r >= k)) m = k;
  return m;
}

/* Mask of the lanes of this wave whose bin equals this lane's bin: one
 * ballot per bin bit (bit-sliced match), restricted to `valid`. */
__device__ __forceinline__ uint64_t match_bin(uint32_t b, uint64_t valid, uint32_t nbits) {
  uint64_t same = valid;
#pragma unroll
  for (uint32_t k = 0; k < MAX_NBITS; ++k) {
    if (k < nbits) {
      const bool bit = (b >> k) & 1u;
      const uint64_t bal = __ballot(bit);
      same &= bit ? bal : ~bal;
    }
  }
  return same;
}

/* The tile's frames per bin (the scatter's input, scan_agg / scan_off /
 * scatter below) into the LDS histogram: u16 counts in pairs per u32 word,
 * zeroed by the caller before a barrier.  With few bins (nbits <= 6) one LDS
 * add per distinct bin of a wave (bit-sliced match: c2's 19 bins would put
 * ~50 lanes of a wave on a handful of words), else one per frame (c5: ~1000
 * bins, lanes rarely collide).  Replaces round 2's per-tile stable sort: the
 * ranks are computed by the scatter kernel, outside this latency-bound
 * kernel. */
__device__ __forceinline__ void tile_hist(const uint32_t bins[ROUNDS], uint32_t nt, uint32_t nbits,
                                          uint32_t *hist) {
  const uint32_t tid = threadIdx.x, lane = tid & 63;
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    const bool v = local < nt;
    const uint32_t b = bins[r];
    if (nbits <= 6) {
      const uint64_t same = match_bin(b, __ballot(v), nbits);
      if (v && (same & lanemask_lt(lane)) == 0)
        atomicAdd(&hist[b >> 1], (uint32_t)__popcll(same) << (16u * (b & 1u)));
    } else if (v) {
      atomicAdd(&hist[b >> 1], 1u << (16u * (b & 1u)));
    }
  }
}
__device__ __forceinline__ uint32_t byte_sum(uint32_t v) { return __builtin_amdgcn_sad_u8(v, 0u, 0u); }
__device__ __forceinline__ uint32_t hist_get(const uint32_t *hist, uint32_t b) {
  return (hist[b >> 1] >> (16u * (b & 1u))) & 0xFFFFu;
}
/* after a barrier: the histogram as the tile's count row (16-byte stores) */
__device__ __forceinline__ void hist_out(const uint32_t *hist, uint32_t nbw, uint16_t *row) {
  const uint4 *h = reinterpret_cast<const uint4 *>(hist);
  uint4 *w = reinterpret_cast<uint4 *>(row);
  for (uint32_t i = threadIdx.x; i < nbw / 8; i += NTHREADS) w[i] = h[i];
}
__device__ __forceinline__ void hist_zero(uint32_t *hist, uint32_t nbw) {
  for (uint32_t i = threadIdx.x; i < nbw / 2; i += NTHREADS) hist[i] = 0;
}

/* --------------------------------------------------------------------------- */
/* Carried-in decision cache for this batch, resolved by all threads of
 * workgroup 0: the state after the last cache-touching frame of the previous
 * batch (its tiles are scanned in parallel), or that batch's own carried-in
 * state when none of its frames touched the cache.  out[0..5] in LDS. */
__device__ __forceinline__ void resolve_carry(const ClassifyArgs &a, uint32_t *out, uint32_t *scratch) {
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
template <int TM>
__device__ __forceinline__ uint32_t decide_info_rx(const uint4 *T, const uint16_t *Dl, const ClassifyArgs &a,
                                   const uint32_t *info) {
  Parsed p;
  p.status = 1; p.i0 = info[0]; p.src = info[1]; p.dst = info[2]; p.ports = info[3];
  p.proto = (info[0] >> 8) & 0xFFu; p.has_ports = (info[0] >> 16) & 1u;
  p.sport = info[3] & 0xFFFFu; p.dport = info[3] >> 16; p.frag_first = 0;
  return decide_rx<TM>(T, Dl, a, p);
}

/* The stage holds bytes 12..43 of each frame (USN_STAGE32; else 0..47): the
 * parse reads 12..39, and the port words of longer IPv4 headers come from
 * the frame itself.  16-byte part j of frame f at slot GLDS_PARTS f + j of a
 * wave's round stage.  glds writes it linearly, and the per-frame
 * ds_read_b128s (an 8- or 12-dword stride) cover distinct 4-bank groups per
 * 16 lanes: no bank conflicts either way.  Two parts instead of three: one
 * DMA instruction less per wave and round, the same HBM lines
 * (tools/probe_floor: stream + probes 134.7 vs 141.3 us per 8M frames). */
__device__ __forceinline__ uint32_t stage_slot(uint32_t f, uint32_t j) {
  return GLDS_PARTS * f + j;
}

/* ---- header loads -----------------------------------------------------------
 * GLDS (fixed-stride layouts, the default): LDS-DMA (`global_load_lds_dwordx4`)
 * with the non-temporal hint straight into a wave-private stage of
 * USN_GLDS_DEPTH rounds x 64 frames x 48 B.  No VGPRs are held for data in
 * flight, and it is the fastest way found to stream the windows
 * (tools/hbm_floor.hip, 8M frames per launch: 100-103 us vs 113 us for
 * per-lane 16-byte register loads; register loads with nt: 199 us).
 * glds writes LDS lane-linearly (base + 16 x lane), so each lane's SOURCE is
 * the chunk that belongs at its slot: lane L of instruction k fills slot
 * u = 64k + L = stage_slot(f, p) with f = u / 3, p = u % 3, and every lane
 * then reads its own frame's parts.
 * LANE (offsets layout, strides that are not 16-byte multiples): one 64-byte
 * window per lane with 16-byte register loads, one round in flight ahead. */
#ifndef USN_GLDS_DEPTH
#define USN_GLDS_DEPTH 1
#endif
#define GD USN_GLDS_DEPTH
#define NWAVES (NTHREADS / 64)
#ifndef GLDS_NT                  /* aux bits of the header glds: non-temporal */
#define GLDS_NT 2
#endif
#ifndef USN_GLDS_ENABLE          /* A/B only: 0 = register loads for every layout */
#define USN_GLDS_ENABLE 1
#endif

typedef __attribute__((address_space(3))) void lds_void_t;

template <int N>
__device__ __forceinline__ void vm_wait() {   /* hipcc does not count LDS-DMA for LDS reads */
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

/* glds of round r of this wave's 64 frames into stage `st` (wave-uniform) */
__device__ __forceinline__ void glds_round(const ClassifyArgs &a, uint64_t base, uint32_t nt,
                                           uint32_t r, uint32_t wave, uint32_t lane, uint4 *st) {
#pragma unroll
  for (uint32_t k = 0; k < GLDS_PARTS; ++k) {
    const uint32_t u = 64 * k + lane;
    const uint32_t f = u / GLDS_PARTS, p = u - GLDS_PARTS * f;
    uint32_t local = r * NTHREADS + wave * 64 + f;
    local = local < nt ? local : nt - 1;          // tail tile: re-read the last frame
    // the tile's first frame (scalar) + a 32-bit lane offset: local < 1024 and
    // a GLDS stride <= 128, so one full-rate 24-bit multiply (a 64-bit index
    // times the stride was three quarter-rate multiplies per instruction)
    const uint8_t *tf = a.frames + base * a.stride;
    const uint8_t *src = tf + (__umul24(local, a.stride) + GLDS_OFF + p * 16);
    __builtin_amdgcn_global_load_lds(src, (lds_void_t *)(st + 64 * k), 16, 0, GLDS_NT);
  }
}

/* the staged bytes 12..43 as the 64-byte window words parse() reads
 * (bytes 0..11 and 44.. read as zero; nothing on the rx path uses them) */
__device__ __forceinline__ void stage32_words(const v4u32 &a0, const v4u32 &a1, uint4 (&q)[4]) {
  q[0] = make_uint4(0, 0, 0, a0.x);
  q[1] = make_uint4(a0.y, a0.z, a0.w, a1.x);
  q[2] = make_uint4(a1.y, a1.z, a1.w, 0);
  q[3] = make_uint4(0, 0, 0, 0);
}

/* this lane's frame (parse reads bytes 12..39) */
__device__ __forceinline__ void stage_read(const uint4 *st, uint32_t lane, uint4 (&q)[4]) {
  if (USN_STAGE32) {
    const uint4 b0 = st[stage_slot(lane, 0)], b1 = st[stage_slot(lane, 1)];
    stage32_words(v4u32{b0.x, b0.y, b0.z, b0.w}, v4u32{b1.x, b1.y, b1.z, b1.w}, q);
    return;
  }
#pragma unroll
  for (uint32_t j = 0; j < 3; ++j) q[j] = st[stage_slot(lane, j)];
  q[3] = make_uint4(0, 0, 0, 0);
}

/* the same by inline asm: no vmcnt wait of hipcc's (which would also wait
 * for asm probe loads in flight); the caller has waited for the DMA */
__device__ __forceinline__ void stage_read_asm(const uint4 *st, uint32_t lane, uint4 (&q)[4]) {
  if (USN_STAGE32) {
    v4u32 a0, a1;
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(a0), "=&v"(a1)
                 : "v"(lds_addr(st + stage_slot(lane, 0))), "v"(lds_addr(st + stage_slot(lane, 1))));
    stage32_words(a0, a1, q);
    return;
  }
  v4u32 a0, a1, a2;
  asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b128 %2, %5\n\t"
               "s_waitcnt lgkmcnt(0)"
               : "=&v"(a0), "=&v"(a1), "=&v"(a2)
               : "v"(lds_addr(st + stage_slot(lane, 0))), "v"(lds_addr(st + stage_slot(lane, 1))),
                 "v"(lds_addr(st + stage_slot(lane, 2))));
  q[0] = make_uint4(a0.x, a0.y, a0.z, a0.w);
  q[1] = make_uint4(a1.x, a1.y, a1.z, a1.w);
  q[2] = make_uint4(a2.x, a2.y, a2.z, a2.w);
  q[3] = make_uint4(0, 0, 0, 0);
}

/* LANE: bytes 0..47 of this lane's window of round r into registers (parse
 * reads 12..39; longer IPv4 headers' ports come from the frame).  At the
 * 2048-byte stride a frame's read is one scattered HBM access whose cost
 * grows with its bytes: 4M frames in 89 / 108 / 140 us at 32 / 48 / 64 bytes
 * (tools/stride_floor.hip, profiles/r02f). */
/* (Bytes 12..43 in two dword-aligned 16-byte loads instead, as the 32-byte
 * stage's DMA does: slower here, c3 1M frames 34.7 vs 33.4 us, profiles/r02bh;
 * again in round 4, calls of 4 x 256K frames: 11.74 vs 11.56 us per ring,
 * profiles/r04/r04m.) */
__device__ __forceinline__ void lane_round(const uint8_t *fp, uint4 (&q)[4]) {
  const uint4 *w = reinterpret_cast<const uint4 *>(fp);
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k) q[k] = ld_stream(w + k);
  q[3] = make_uint4(0, 0, 0, 0);
}

/* Which batch of a launch tile w belongs to: tile_base[] is increasing, so
 * bi = #{k in [1, count): w >= tile_base[k]}.  Unrolled over USN_MAX_MULTI
 * so the bases arrive in one scalar load, not a dependent load per step. */
__device__ __forceinline__ uint32_t batch_of(const MultiArgs &m, uint32_t w) {
  uint32_t bi = 0;
#pragma unroll
  for (uint32_t k = 1; k < USN_MAX_MULTI; ++k)
    bi += (k < m.count && w >= m.tile_base[k]) ? 1u : 0u;
  return bi;
}

/* The 1024-frame tiles of a launch (several batches = drained rx rings may
 * share one launch), one workgroup each.  (A persistent grid looping over
 * tiles, copying the displacements once per workgroup, was slower in rounds
 * 2 and 4: c5 8M 185.5 vs 170.5 us, profiles/r02ah; with the next tile's
 * headers prefetched 175.4 vs 159.1, profiles/r04/r04ao.  Both rounds' header
 * DMA at the workgroup's start was a wash, r04l.) */
template <int TM, bool GLDS>
__global__ __launch_bounds__(NTHREADS) void classify_rx_kernel(MultiArgs m) {
  // global-image probes: the next round's header DMA goes out after this
  // round's slot loads (USN_LATE_DMA=0: right after this round's stage reads)
  constexpr bool LATE_DMA = GLDS && TM != TM_LDS && USN_LATE_DMA;
  // both rounds' probes batched (two rounds per lane, global image)
  constexpr bool BATCH2 = GLDS && TM != TM_LDS && ROUNDS == 2 && GD == 1;
  constexpr uint32_t WSTAGE = GD * STAGE_ROUND_SLOTS;   // per wave
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint4 s_stage[GLDS ? NWAVES * WSTAGE : 1];
  __shared__ uint32_t s_carry[8];
  __shared__ uint32_t s_misc[8];   // [0] last touching frame + 1, [1] host-list fill, [3..5] NIC/FLOOD/DROP
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // bins and table are shared by the batches.  GLDS: the order row and the
  // radix keys live in the header stage (carve)
  const Lds L = carve(smem, m.b[0].nbins, GLDS ? s_stage : nullptr);
  uint4 *st = s_stage + (GLDS ? wave * WSTAGE : 0);   // this wave's stage
  const uint4 *T = m.b[0].table;
  const uint16_t *Dl = nullptr;
  if (TM != TM_GLOBAL) {   // image (or its displacements) -> LDS by glds, 64 units per instruction
    // TM_DISPLDS with U built: U's and X's displacements, else K1's and K2's
    const bool um = TM == TM_DISPLDS && (m.b[0].probe_mask & 4u);
    const uint32_t u0 = TM == TM_LDS ? 0u : um ? m.b[0].u_disp_unit : m.b[0].disp_unit;
    const uint32_t uend = um ? m.b[0].u_end_unit : m.b[0].table_units;
    const uint32_t units = uend - u0;
    for (uint32_t c = wave; c * 64 < units; c += NWAVES) {
      const uint32_t sl = u0 + min(c * 64 + lane, units - 1);
      __builtin_amdgcn_global_load_lds(m.b[0].table + sl, (lds_void_t *)(L.table + c * 64), 16, 0, 0);
    }
    if (TM == TM_LDS) T = L.table;
    else Dl = reinterpret_cast<const uint16_t *>(L.table) - (size_t)u0 * 8;
  }
  // (the tile's first barrier also waits for the image copy)
  {
    const uint32_t w = blockIdx.x;
    uint4 *const st1 = st;   // round 1's stage: round 0's, once its reads are done
    const uint32_t bi = batch_of(m, w);
    const ClassifyArgs &a = m.b[bi];
    const uint32_t tile = w - m.tile_base[bi];
    const uint64_t base = (uint64_t)tile * TILE;
    const uint32_t nt = (uint32_t)min((uint64_t)TILE, a.n - base);
    STAMP_DECL
    STAMP(0);

    // ---- loads, oldest first: lengths, headers.
    //      Unpredicated at a clamped index: a load under `local < nt` made the
    //      compiler wait for each before issuing the next; lanes past nt are
    //      masked at use.
    uint32_t len[ROUNDS];
    const uint8_t *fp[ROUNDS];
    if (!GLDS && a.offsets) {   // uniform; GLDS launches have no offsets array
#pragma unroll
      for (uint32_t r = 0; r < ROUNDS; ++r)
        fp[r] = a.frames + a.offsets[base + min(r * NTHREADS + tid, nt - 1)];
    } else {
      const uint8_t *tf = a.frames + base * a.stride;   // the tile's first frame (scalar)
#pragma unroll
      for (uint32_t r = 0; r < ROUNDS; ++r) {
        const uint32_t i = min(r * NTHREADS + tid, nt - 1);
        fp[r] = tf + (GLDS ? (size_t)__umul24(i, a.stride) : (size_t)i * a.stride);
      }
    }
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) len[r] = a.lens[base + min(r * NTHREADS + tid, nt - 1)];
    uint4 q[ROUNDS][4];
    if (GLDS) {
#pragma unroll
      for (uint32_t r = 0; r < GD && r < ROUNDS; ++r)
        glds_round(a, base, nt, r, wave, lane, st + r * STAGE_ROUND_SLOTS);
    } else {
      lane_round(fp[0], q[0]);
    }
    STAMP(1);
    // ---- while they fly: zero the bin histogram (the barrier also waits
    //      for every load: table and round 0 are in LDS / registers after it)
    hist_zero(L.hist, a.nbw);
    if (tid < 8) s_misc[tid] = 0;
    __syncthreads();
    STAMP(2);

    // ---- carried-in cache (block 0): stale check against the current table
    if (tile == 0) {
      resolve_carry(a, s_carry, L.scratch);
      if (tid == 0) {
        const uint32_t cst = s_carry[0], dst = s_carry[1];
        uint32_t flags = 0;
        if ((cst & USN_CS_VALID) &&
            ((decide_info_rx<TM>(T, Dl, a, s_carry + 2) ^ dst) & USN_PARITY_MASK))
          flags |= USN_S_STALE;
        s_carry[6] = flags;
        s_carry[7] = TILE;   // first break in tile 0 (min over frames), TILE = none
        usn_summary *S = a.summary;
        S->cin_state = cst; S->cin_dst = dst;
        for (int k = 0; k < 4; ++k) S->cin_info[k] = s_carry[2 + k];
        S->n_frames = (uint32_t)a.n; S->n_tiles = a.ntiles;
        S->n_ep = a.n_ep; S->n_bins = a.nbins;
      }
      __syncthreads();
    }
    const bool stale = tile == 0 && (s_carry[6] & USN_S_STALE);
    STAMP(3);

    // ---- parse + decide, the next round's headers in flight meanwhile
    uint32_t dec[ROUNDS], bins[ROUNDS];
    uint32_t differs = 0;          // stale mode: bit r = touching frame whose info != carried
    uint32_t my_last = 0;          // 1 + tile-local index of this lane's last touching frame
    uint32_t my_touch = 0, my_dec = 0, my_info[4] = {0, 0, 0, 0};
    Parsed pr[ROUNDS];
    if (BATCH2 && TM == TM_DISPLDS && (a.probe_mask & 4u)) {
      // U: one slot read per frame answers key1 AND key2 (they share the
      // projection); both rounds' reads fly together, round 1's header DMA
      // under round 0's parse.  X only where a projection holds several K1
      // rules and the inline one is not the frame's key1 (rare: one wave-
      // uniform branch, after every load of the wave has landed).
      uint4 *sb = st;
      uint32_t du0, du1;
      v4u32 su0, su1;
      stage_read_asm(sb, lane, q[0]);
      glds_round(a, base, nt, 1, wave, lane, sb);                 // round 1's headers
      __builtin_amdgcn_sched_barrier(0);
      parse(q[0], tid < nt ? len[0] : 0u, fp[0], a.window, pr[0]);
      const uint32_t e0 = u_key_e(pr[0]);
      const PhKeyH ku0 = ph_hash(a.ph[2], pr[0].dst, 0u, e0, 0u);
      const bool n0 = pr[0].status == 1u;
      du0 = lds_disp1(Dl, a.ph[2], n0, ku0);
      asm_slot1(T, a.ph[2], n0, ku0, du0, su0);
      __builtin_amdgcn_sched_barrier(0);
      vm_wait<1>();                                               // round 1 landed (1 younger load)
      stage_read_asm(st1, lane, q[1]);
      parse(q[1], NTHREADS + tid < nt ? len[1] : 0u, fp[1], a.window, pr[1]);
      const uint32_t e1 = u_key_e(pr[1]);
      const PhKeyH ku1 = ph_hash(a.ph[2], pr[1].dst, 0u, e1, 0u);
      const bool n1 = pr[1].status == 1u;
      du1 = lds_disp1(Dl, a.ph[2], n1, ku1);
      asm_slot1(T, a.ph[2], n1, ku1, du1, su1);
#if USN_ISA_PERTURB == 1   /* tests/test_isa_waits.py only: a load between issue and wait */
      uint32_t perturb;
      asm volatile("global_load_dword %0, %1, off" : "=v"(perturb) : "v"(a.lens + tid) : "memory");
#endif
      uint32_t w01, w02, w11, w12;
      bool x0, x1;
      asm volatile("s_waitcnt vmcnt(" USN_U_WAIT0 ")" : "+v"(su0) :: "memory");
      u_decode(su0, pr[0], e0, w01, w02, x0);
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(su1) :: "memory");
      u_decode(su1, pr[1], e1, w11, w12, x1);
#if USN_ISA_PERTURB == 1
      if (perturb == 0xFFFFFFFFu) w01 = 0;
#endif
      x0 = x0 && n0;
      x1 = x1 && n1;
      STAMP(4);
      if (__ballot(x0 || x1)) {
        uint32_t wx0, wx1;   // both rounds' X reads in flight together
        x_probe2(T, Dl, a, pr[0], x0, pr[1], x1, wx0, wx1);
        if (x0) w01 = wx0;
        if (x1) w11 = wx1;
      }
      dec[0] = decide_rx_w(a, pr[0], w01, w02);
      dec[1] = decide_rx_w(a, pr[1], w11, w12);
    } else if (BATCH2 && TM == TM_DISPLDS && USN_SEQ_K2) {
      // displacements from LDS; key1's slot reads of both rounds first, then
      // key2's only where key1 missed (get_endpoint reads key2 only then,
      // endpoint.rs:317-327): a lane that needs no read shares the table's
      // first line, so c5's half of frames that hit key1 cost no second L2
      // request.  Round 1's header DMA flies under round 0's parse.
      uint4 *sb = st;
      const bool use1 = (a.probe_mask & 1u) != 0, use2 = (a.probe_mask & 2u) != 0;
      RoundKeys k0, k1;
      uint32_t d01, d02, d11, d12;
      v4u32 s01, s02, s11, s12;
      stage_read_asm(sb, lane, q[0]);
      glds_round(a, base, nt, 1, wave, lane, sb);                 // round 1's headers
      __builtin_amdgcn_sched_barrier(0);
      parse(q[0], tid < nt ? len[0] : 0u, fp[0], a.window, pr[0]);
      round_keys(a, pr[0], k0);
      lds_disp2(Dl, a, use1, use2, k0, d01, d02);
      const bool n01 = use1 && pr[0].status == 1u;
      asm_slot1(T, a.ph[0], n01, k0.k1, d01, s01);
      __builtin_amdgcn_sched_barrier(0);
      vm_wait<1>();                                               // round 1 landed (1 younger load)
      stage_read_asm(st1, lane, q[1]);
      parse(q[1], NTHREADS + tid < nt ? len[1] : 0u, fp[1], a.window, pr[1]);
      round_keys(a, pr[1], k1);
      lds_disp2(Dl, a, use1, use2, k1, d11, d12);
      const bool n11 = use1 && pr[1].status == 1u;
      asm_slot1(T, a.ph[0], n11, k1.k1, d11, s11);
      asm volatile("s_waitcnt vmcnt(1)" : "+v"(s01) :: "memory");
      const uint32_t w01 = n01 ? ph_hitv(s01, k0.x1, k0.y1, k0.z1, k0.m1) : 0u;
      const bool n02 = use2 && pr[0].status == 1u && !w01;
      asm_slot1(T, a.ph[1], n02, k0.k2, d02, s02);
      asm volatile("s_waitcnt vmcnt(1)" : "+v"(s11) :: "memory");
      const uint32_t w11 = n11 ? ph_hitv(s11, k1.x1, k1.y1, k1.z1, k1.m1) : 0u;
      const bool n12 = use2 && pr[1].status == 1u && !w11;
      asm_slot1(T, a.ph[1], n12, k1.k2, d12, s12);
      STAMP(4);
      asm volatile("s_waitcnt vmcnt(1)" : "+v"(s02) :: "memory");
      dec[0] = decide_rx_w(a, pr[0], w01, n02 ? ph_hitv(s02, k0.x2, k0.y2, k0.z2, k0.m2) : 0u);
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(s12) :: "memory");
      dec[1] = decide_rx_w(a, pr[1], w11, n12 ? ph_hitv(s12, k1.x2, k1.y2, k1.z2, k1.m2) : 0u);
    } else if (BATCH2 && TM == TM_DISPLDS) {
      // displacements from LDS: one global round trip (the slots) per round,
      // round 1's header DMA in flight under round 0's parse and slot loads
      uint4 *sb = st;
      const bool use1 = (a.probe_mask & 1u) != 0, use2 = (a.probe_mask & 2u) != 0;
      RoundKeys k0, k1;
      uint32_t d01, d02, d11, d12;
      v4u32 s01, s02, s11, s12;
      stage_read_asm(sb, lane, q[0]);
      glds_round(a, base, nt, 1, wave, lane, sb);                 // round 1's headers
      __builtin_amdgcn_sched_barrier(0);
      parse(q[0], tid < nt ? len[0] : 0u, fp[0], a.window, pr[0]);
      round_keys(a, pr[0], k0);
      lds_disp2(Dl, a, use1, use2, k0, d01, d02);
      asm_slot2(T, a, use1, use2, k0, d01, d02, s01, s02);
      __builtin_amdgcn_sched_barrier(0);
      vm_wait<2>();                                               // round 1 landed (2 younger loads)
      stage_read_asm(st1, lane, q[1]);
      parse(q[1], NTHREADS + tid < nt ? len[1] : 0u, fp[1], a.window, pr[1]);
      round_keys(a, pr[1], k1);
      lds_disp2(Dl, a, use1, use2, k1, d11, d12);
      asm_slot2(T, a, use1, use2, k1, d11, d12, s11, s12);
      asm volatile("s_waitcnt vmcnt(2)" : "+v"(s01), "+v"(s02) :: "memory");
      dec[0] = decide_rx_w(a, pr[0], use1 ? ph_hitv(s01, k0.x1, k0.y1, k0.z1, k0.m1) : 0u,
                           use2 ? ph_hitv(s02, k0.x2, k0.y2, k0.z2, k0.m2) : 0u);
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(s11), "+v"(s12) :: "memory");
      dec[1] = decide_rx_w(a, pr[1], use1 ? ph_hitv(s11, k1.x1, k1.y1, k1.z1, k1.m1) : 0u,
                           use2 ? ph_hitv(s12, k1.x2, k1.y2, k1.z2, k1.m2) : 0u);
    } else if (BATCH2) {
      // round 0's headers are in the stage (the barrier above waited for them)
      uint4 *sb = st;
      const bool use1 = (a.probe_mask & 1u) != 0, use2 = (a.probe_mask & 2u) != 0;
      const uint16_t *D = reinterpret_cast<const uint16_t *>(T);
      RoundKeys k0, k1;
      uint32_t d01, d02, d11, d12;
      v4u32 s01, s02, s11, s12;
      stage_read_asm(sb, lane, q[0]);
      glds_round(a, base, nt, 1, wave, lane, sb);                 // round 1's headers
      __builtin_amdgcn_sched_barrier(0);
      parse(q[0], tid < nt ? len[0] : 0u, fp[0], a.window, pr[0]);
      round_keys(a, pr[0], k0);
      asm_disp2(D, a, use1, use2, k0, d01, d02);
      __builtin_amdgcn_sched_barrier(0);
      vm_wait<2>();                                               // round 1 landed (2 younger loads)
      stage_read_asm(st1, lane, q[1]);
      parse(q[1], NTHREADS + tid < nt ? len[1] : 0u, fp[1], a.window, pr[1]);
      round_keys(a, pr[1], k1);
      asm_disp2(D, a, use1, use2, k1, d11, d12);
      vm_wait2<2>(d01, d02);
      asm_slot2(T, a, use1, use2, k0, d01, d02, s01, s02);
      vm_wait2<2>(d11, d12);
      asm_slot2(T, a, use1, use2, k1, d11, d12, s11, s12);
      asm volatile("s_waitcnt vmcnt(2)" : "+v"(s01), "+v"(s02) :: "memory");
      dec[0] = decide_rx_w(a, pr[0], use1 ? ph_hitv(s01, k0.x1, k0.y1, k0.z1, k0.m1) : 0u,
                           use2 ? ph_hitv(s02, k0.x2, k0.y2, k0.z2, k0.m2) : 0u);
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(s11), "+v"(s12) :: "memory");
      dec[1] = decide_rx_w(a, pr[1], use1 ? ph_hitv(s11, k1.x1, k1.y1, k1.z1, k1.m1) : 0u,
                           use2 ? ph_hitv(s12, k1.x2, k1.y2, k1.z2, k1.m2) : 0u);
    }
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS && !BATCH2; ++r) {
      const uint32_t local = r * NTHREADS + tid;
      uint4 *sb = st + (r % GD) * STAGE_ROUND_SLOTS;
      if (GLDS) {
        // round r landed: only the rounds issued after it may still fly (GLDS_PARTS glds each)
        constexpr uint32_t kAfterMax = GD - 1;
        const uint32_t after = min(kAfterMax, ROUNDS - 1 - r);
        if (r > 0) {
          if (after >= 3) vm_wait<3 * GLDS_PARTS>();
          else if (after == 2) vm_wait<2 * GLDS_PARTS>();
          else if (after == 1) vm_wait<GLDS_PARTS>();
          else vm_wait<0>();
        }
        stage_read(sb, lane, q[r]);
        if (!LATE_DMA && r + GD < ROUNDS) {
          lgkm_wait0();          // this round's reads are done before its buffer is refilled
          glds_round(a, base, nt, r + GD, wave, lane, sb);
        }
      } else if (r + 1 < ROUNDS) {   // one round of headers in flight ahead of the one decided
        __builtin_amdgcn_sched_barrier(0);
        lane_round(fp[r + 1], q[r + 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
      Parsed &p = pr[r];
      parse(q[r], local < nt ? len[r] : 0u, fp[r], a.window, p);
      if (LATE_DMA && TM == TM_DISPLDS && (a.probe_mask & 4u)) {
        // U (rare here: the 512-thread build batches both rounds above);
        // synchronous, then the next round's header DMA
        uint32_t w1 = 0, w2 = 0;
        u_probe_sync(T, Dl, a, p, w1, w2);
        if (r + GD < ROUNDS) {
          __builtin_amdgcn_sched_barrier(0);
          lgkm_wait0();
          glds_round(a, base, nt, r + GD, wave, lane, sb);
          __builtin_amdgcn_sched_barrier(0);
        }
        dec[r] = decide_rx_w(a, p, w1, w2);
      } else if (LATE_DMA) {
        // global probes: the slot loads first, then the next round's header DMA,
        // so the wait for the slots does not also wait for the DMA
        uint32_t x1, y1, z1, m1, x2, y2, z2, m2;
        rx_keys(p, x1, y1, z1, m1, x2, y2, z2, m2);
        const bool use1 = (a.probe_mask & 1u) != 0, use2 = (a.probe_mask & 2u) != 0;
        v4u32 s1, s2;
        ph_issue<TM, true>(T, Dl, a, use1, use2, x1, y1, z1, m1, x2, y2, z2, m2, s1, s2);
        if (r + GD < ROUNDS) {
          __builtin_amdgcn_sched_barrier(0);
          lgkm_wait0();
          glds_round(a, base, nt, r + GD, wave, lane, sb);
          __builtin_amdgcn_sched_barrier(0);
          ph_slots_wait<GLDS_PARTS>(s1, s2);   // the next round's header DMAs may still fly
        } else {
          ph_slots_wait<0>(s1, s2);
        }
        const uint32_t w1 = use1 ? ph_hitv(s1, x1, y1, z1, m1) : 0u;
        const uint32_t w2 = use2 ? ph_hitv(s2, x2, y2, z2, m2) : 0u;
        dec[r] = decide_rx_w(a, p, w1, w2);
      } else {
        dec[r] = decide_rx<TM>(T, Dl, a, p);
      }
      if (r == 0) STAMP(4);
    }
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) {
      const uint32_t local = r * NTHREADS + tid;
      const Parsed &p = pr[r];
      // cache touch: 0 none (parse failure), 1 retains Some(info), 2 leaves None, 3 unknown
      uint32_t touch = p.status == 0u ? 0u : p.status >= 4u ? 3u
                     : (p.status == 1u && (p.dst >> 24) != 127u) ? 1u : 2u;
      if (local >= nt) touch = 0;
      if (touch) {
        my_last = local + 1; my_touch = touch; my_dec = dec[r];
        my_info[0] = p.i0; my_info[1] = p.src; my_info[2] = p.dst; my_info[3] = p.ports;
      }
      if (stale && touch && !(touch == 1 && p.i0 == s_carry[2] && p.src == s_carry[3] &&
                              p.dst == s_carry[4] && p.ports == s_carry[5]))
        differs |= 1u << r;        // later fragments also stop the device prefix
    }
    STAMP(5);

    // ---- stale carried cache: frames before the first break take the cached
    //      decision (endpoint.rs:186-191); only tile 0 is resolved here.
    if (stale) {
      uint32_t fb = TILE;
#pragma unroll
      for (uint32_t r = 0; r < ROUNDS; ++r)
        if (differs & (1u << r)) fb = min(fb, r * NTHREADS + tid);
      atomicMin(&s_carry[7], fb);
      __syncthreads();
      const uint32_t first = s_carry[7];
#pragma unroll
      for (uint32_t r = 0; r < ROUNDS; ++r) {
        const uint32_t local = r * NTHREADS + tid;
        const bool touching_same = local < nt && local < first &&
                                   USN_DEC_REASON(dec[r]) != USN_R_PARSE;
        if (touching_same)
          dec[r] = (s_carry[1] & USN_PARITY_MASK) | USN_F_CACHE |
                   (dec[r] & (USN_F_HOST | USN_F_FRAG1 | USN_F_DHCP));
        if (local + 1 == my_last && touching_same) my_dec = dec[r];
      }
      if (tid == 0) {
        uint32_t f = s_carry[6];
        if (first >= nt && a.n > TILE) f |= USN_S_STALE_EXTENDS;
        a.summary->first_break = first;
        s_carry[6] = f;
      }
    }
    if (tile == 0 && tid == 0) {
      a.summary->flags = s_carry[6];
      if (!(s_carry[6] & USN_S_STALE)) a.summary->first_break = 0xFFFFFFFFu;
    }

    // ---- decisions out (coalesced), host list, last touching frame
    uint32_t *hl = a.host_list + (size_t)tile * TILE;
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) {
      const uint32_t local = r * NTHREADS + tid;
      const bool v = local < nt;
      if (v) a.decisions[base + local] = dec[r];
      bins[r] = dec_bin(dec[r], a.n_ep);
      const bool host = v && (dec[r] & USN_F_HOST);
      if (__ballot(host)) {                                // rare: unordered append (host sorts)
        if (host) hl[atomicAdd(&s_misc[1], 1u)] = (uint32_t)(base + local);
      }
    }
    {
      // the wave's last touching frame: highest lane of the latest round with one
      const uint64_t rounds_with = __ballot(my_last != 0);
      if (rounds_with) {
        const uint32_t r_last = (my_last - 1) / NTHREADS;
        const uint32_t rmax = __builtin_amdgcn_readfirstlane(
            __reduce_max_rounds(r_last, my_last != 0));
        const uint64_t in_r = __ballot(my_last != 0 && r_last == rmax);
        const uint32_t hi = 63 - (uint32_t)__builtin_clzll(in_r);
        if (lane == 0) atomicMax(&s_misc[0], rmax * NTHREADS + wave * 64 + hi + 1);
      }
    }

    STAMP(6);
    // ---- the tile's frames per bin: LDS histogram, then its count row
    tile_hist(bins, nt, a.nbits, L.hist);
    __syncthreads();
    STAMP(10);
    hist_out(L.hist, a.nbw, a.cnt + (size_t)tile * a.nbw);

    // ---- tile header
    usn_tile_hdr *H = a.tiles + tile;
    const uint32_t lastp = s_misc[0];
    if (lastp && my_last == lastp) {
      H->last_state = USN_TS_HAS | (my_touch == 1u ? USN_TS_RETAINED : 0u) |
                      (my_touch == 3u ? USN_TS_UNKNOWN : 0u);
      H->last_dst = my_dec & USN_PARITY_MASK;
      for (int k = 0; k < 4; ++k) H->last_info[k] = my_info[k];
      H->last_idx = (uint32_t)(base + lastp - 1);
    }
    if (tid == 0) {
      const uint32_t nic = hist_get(L.hist, a.n_ep), fl = hist_get(L.hist, a.n_ep + 1),
                     dr = hist_get(L.hist, a.n_ep + 2);
      if (s_misc[1]) a.summary->host_epoch = a.epoch;   // (usn_finalize's rx state)
      H->n_frames = (uint16_t)nt;
      H->_r0 = 0;
      H->n_host = (uint16_t)s_misc[1];
      H->bin_nic = (uint16_t)a.n_ep;
      H->class_count[0] = (uint16_t)dr;                              // DROP bin
      H->class_count[2] = (uint16_t)nic;                             // NIC bin
      H->class_count[3] = (uint16_t)fl;                              // FLOOD bin
      H->class_count[1] = (uint16_t)(nt - nic - fl - dr);
      if (!lastp) { H->last_state = 0; H->last_dst = 0; H->last_idx = 0xFFFFFFFFu; }
    }
    STAMP(11);
    STAMP_FLUSH_AT(w);
  }
}


/* Recount the bin rows and class counts of tiles from patched decisions
 * (usn_finalize; the scatter then runs again over the whole batch). */
__global__ __launch_bounds__(NTHREADS) void recount_kernel(ClassifyArgs a, uint32_t t0) {
  extern __shared__ __align__(16) uint8_t smem[];
  const Lds L = carve(smem, a.nbins);
  const uint32_t tid = threadIdx.x;
  const uint32_t tile = t0 + blockIdx.x;
  const uint64_t base = (uint64_t)tile * TILE;
  const uint32_t nt = (uint32_t)min((uint64_t)TILE, a.n - base);
  hist_zero(L.hist, a.nbw);
  uint32_t bins[ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    const uint32_t d = a.decisions[base + (local < nt ? local : 0)];   // unpredicated load
    bins[r] = dec_bin(local < nt ? d : 0u, a.n_ep);
  }
  __syncthreads();
  tile_hist(bins, nt, a.nbits, L.hist);
  __syncthreads();
  hist_out(L.hist, a.nbw, a.cnt + (size_t)tile * a.nbw);
  if (tid == 0) {
    usn_tile_hdr *H = a.tiles + tile;
    const uint32_t nic = hist_get(L.hist, a.n_ep), fl = hist_get(L.hist, a.n_ep + 1),
                   dr = hist_get(L.hist, a.n_ep + 2);
    H->class_count[0] = (uint16_t)dr;
    H->class_count[2] = (uint16_t)nic;
    H->class_count[3] = (uint16_t)fl;
    H->class_count[1] = (uint16_t)(nt - nic - fl - dr);
  }
}

/* ===========================================================================
 * tx direction: frames sent by a non-NIC endpoint S (incoming == false).
 * find_forward then also learns: unicast source MACs join the inner L2
 * bridge (endpoint.rs:195-197) and answer keys become rules owned by S
 * (:210-253), while the 1-entry cache ignores MACs (:186-191).  Every
 * decision depends on what earlier frames of the batch learned, so the batch
 * is classified exactly, in four launches:
 *   tx_scan   parse, snapshot membership (bridge, table, S.listening) -> records
 *   tx_hits   each frame's previous cache-touching frame -> cache hits; the
 *             frames that really learn insert (key, first index) into
 *             epoch-tagged hash sets (first occurrence = atomic max of ~index)
 *   tx_decide decisions of non-hit frames against snapshot + "learned by a
 *             frame <= me"; the first learner of each item is listed
 *   tx_fill   a hit copies its run head's decision; tile order + headers
 * Frames whose decision needs ordered host state (later fragments, a DHCP
 * request's cross-endpoint side effect, steered DHCP answers) are flagged;
 * usn_finalize resolves them sequentially from the first one.
 * =========================================================================== */

__device__ __forceinline__ uint32_t tx_touch(const uint4 &r0) { return (r0.x >> TXR_TOUCH_SHIFT) & 3u; }
/* r1 = the frame's first 16 bytes (dmac, smac, ethertype), re-read from the
 * batch where a later pass needs the MACs: rarer than writing a MAC record
 * for every frame in tx_scan */
__device__ __forceinline__ uint4 frame_head(const ClassifyArgs &a, uint64_t i) {
  const uint8_t *fp = a.offsets ? a.frames + a.offsets[i] : a.frames + i * a.stride;
  return *reinterpret_cast<const uint4 *>(fp);
}
__device__ __forceinline__ uint64_t rec_smac(const uint4 &r1) {
  return (uint64_t)(r1.y >> 16) | ((uint64_t)r1.z << 16);
}
__device__ __forceinline__ uint64_t rec_dmac(const uint4 &r1) {
  return (uint64_t)r1.x | ((uint64_t)(r1.y & 0xFFFFu) << 32);
}

__device__ __forceinline__ bool bridge_has(const unsigned long long *set, uint32_t mask, uint64_t mac) {
  uint32_t h = usn_mac_hash(mac) & mask;
  for (uint32_t it = 0; it <= mask; ++it) {
    const unsigned long long v = set[h];
    if (!(v >> 63)) return false;
    if ((v & 0xFFFFFFFFFFFFull) == mac) return true;
    h = (h + 1) & mask;
  }
  return false;
}

/* the same on the LDS copy, read as LDS (a generic pointer's flat loads
 * would also wait for every global load in flight) */
__device__ __forceinline__ bool bridge_has_lds(const unsigned long long *set, uint32_t mask, uint64_t mac) {
  typedef __attribute__((address_space(3))) const unsigned long long lds_u64;
  const lds_u64 *S = (const lds_u64 *)set;
  uint32_t h = usn_mac_hash(mac) & mask;
  for (uint32_t it = 0; it <= mask; ++it) {
    const unsigned long long v = S[h];
    if (!(v >> 63)) return false;
    if ((v & 0xFFFFFFFFFFFFull) == mac) return true;
    h = (h + 1) & mask;
  }
  return false;
}

/* atomic max of (epoch << 32 | ~idx): the newest epoch wins, then the smallest index */
__device__ __forceinline__ void first_index_update(unsigned long long *w, uint32_t epoch, uint32_t idx) {
  atomicMax(w, ((unsigned long long)epoch << 32) | (unsigned long long)(~idx));
}

/* The sets are written and read by tiles of the same launch: every access
 * is an agent-scope atomic or an sc1 (write-through / L1- and stale-L2-free)
 * load or store (MI355X guide, Guideline 16). */
__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long *p) {
  return __hip_atomic_load((__attribute__((address_space(1))) unsigned long long *)p, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned long long *p, unsigned long long v) {
  __hip_atomic_store((__attribute__((address_space(1))) unsigned long long *)p, v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

/* Insert a 48-bit key into an epoch-tagged set (slot stride in u64 words). */
__device__ __forceinline__ unsigned long long *set_claim(unsigned long long *set, uint32_t mask,
                                                         uint32_t stride, uint32_t epoch,
                                                         uint64_t key48, uint32_t home,
                                                         uint32_t *overflow) {
  const unsigned long long key = ((unsigned long long)epoch << 48) | key48;
  uint32_t h = home & mask;
  for (uint32_t it = 0; it <= mask; ++it) {
    unsigned long long *slot = set + (size_t)h * stride;
    unsigned long long cur = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((cur >> 48) != epoch) {                      // free in this epoch: try to claim
      const unsigned long long prev = atomicCAS(slot, cur, key);
      if (prev == cur) return slot;
      cur = prev;
    }
    if (cur == key) return slot;
    h = (h + 1) & mask;
  }
  atomicOr(overflow, 1u);
  return nullptr;
}

/* Look up a 48-bit key; returns the slot or nullptr. */
__device__ __forceinline__ const unsigned long long *set_find(const unsigned long long *set,
                                                              uint32_t mask, uint32_t stride,
                                                              uint32_t epoch, uint64_t key48,
                                                              uint32_t home) {
  const unsigned long long key = ((unsigned long long)epoch << 48) | key48;
  uint32_t h = home & mask;
  for (uint32_t it = 0; it <= mask; ++it) {
    const unsigned long long *slot = set + (size_t)h * stride;
    const unsigned long long cur = ld_sc1(slot);
    if ((cur >> 48) != epoch) return nullptr;
    if (cur == key) return slot;
    h = (h + 1) & mask;
  }
  return nullptr;
}

/* first index recorded in a set slot, or ~0 */
__device__ __forceinline__ uint32_t slot_first(const unsigned long long *slot, uint32_t epoch) {
  if (!slot) return 0xFFFFFFFFu;
  const unsigned long long v = ld_sc1(slot + 1);
  return (uint32_t)(v >> 32) == epoch ? ~(uint32_t)v : 0xFFFFFFFFu;
}

/* answer key to_want (pkt.rs:78-95) of an IPv4 PacketInfo, packed as a table key */
__device__ __forceinline__ void want_key(const uint4 &r0, uint32_t &x, uint32_t &y, uint32_t &z,
                                         uint32_t &meta) {
  const uint32_t proto = (r0.x >> 8) & 0xFFu, has = (r0.x >> 16) & 1u;
  x = r0.y;                       // dst_addr := src
  y = r0.z;                       // src_addr := Some(dst)
  z = has ? ((r0.w & 0xFFFFu) | ((r0.w >> 16) << 16)) : 0u;   // dport := sport, sport := dport
  meta = usn_key_meta(proto, USN_WANT_SRC | (has ? (USN_WANT_DPORT | USN_WANT_SPORT) : 0u));
}

/* key1 = to_match_want_with_src(true) */
__device__ __forceinline__ void key1_of(const uint4 &r0, uint32_t &x, uint32_t &y, uint32_t &z,
                                        uint32_t &meta) {
  const uint32_t proto = (r0.x >> 8) & 0xFFu, has = (r0.x >> 16) & 1u;
  x = r0.z;
  y = r0.y;
  z = has ? ((r0.w >> 16) | ((r0.w & 0xFFFFu) << 16)) : 0u;
  meta = usn_key_meta(proto, USN_WANT_SRC | (has ? (USN_WANT_DPORT | USN_WANT_SPORT) : 0u));
}

/* Exclusive prefix max, in tile-local frame order, of v[r] (frame
 * r * NTHREADS + tid).  Each round's wave-inclusive max by DPP, the 16 wave
 * totals through L.scratch, ONE barrier (which also publishes whatever the
 * block wrote to LDS before the call), then each lane folds the totals of the
 * waves before it.  (Round 5's version staged the values through L.order and
 * took four barriers; two calls per tx tile.) */
__device__ void tile_prefix_max(const uint32_t v[ROUNDS], const Lds &L, uint32_t out[ROUNDS]) {
  static_assert(ROUNDS * NWAVES <= 16, "L.scratch holds 16 wave totals");
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint32_t inc[ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    uint32_t x = v[r];   // wave inclusive max scan (DPP row shifts, then row broadcasts)
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false));
    inc[r] = x;
    if (lane == 63) L.scratch[r * NWAVES + wave] = x;
  }
  __syncthreads();
  uint32_t before = 0;   // every wave of the earlier rounds, then the earlier waves of round r
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    uint32_t b = before;
    for (uint32_t w = 0; w < wave; ++w) b = max(b, L.scratch[r * NWAVES + w]);
    uint32_t exc = __shfl_up(inc[r], 1, 64);
    if (lane == 0) exc = 0;
    out[r] = max(b, exc);
    for (uint32_t w = 0; w < NWAVES; ++w) before = max(before, L.scratch[r * NWAVES + w]);
  }
}

#define TX_BRIDGE_LDS_SLOTS 2048u   /* bridge sets up to 16 KiB are staged in LDS */
#define TX_LISTEN_LDS 64u           /* listening triples of the source staged in LDS */

/* (W.dst, proto, W.dport) in S.listening?  W.dst = src, W.dport = sport; L:
 * the source's {ip, proto | has_ports << 8 | port << 16} pairs (global or LDS) */
template <typename P>
__device__ __forceinline__ bool tx_listening(P L, uint32_t n, const Parsed &p) {
  bool listening = false;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t ld = L[2 * k], lw = L[2 * k + 1];
    const uint32_t lhas = (lw >> 8) & 1u;
    listening |= ld == p.src && (lw & 0xFFu) == p.proto && lhas == p.has_ports &&
                 (!lhas || (lw >> 16) == p.sport);
  }
  return listening;
}

/* Decision of a non-hit, non-host, cache-retaining tx frame i (IPv4, not
 * loopback): endpoint.rs:254-295 against the snapshot plus everything learned
 * by a frame <= i. */
/* dmac in the inner bridge: in the snapshot, or learned by a frame <= i
 * (endpoint.rs:254); r1 is read only when this batch learned a MAC */
__device__ __forceinline__ bool tx_dmac_in(const TxArgs &t, uint32_t fl, const uint4 &r1, uint32_t i,
                                           uint32_t ins) {
  bool d_in = (fl & TXR_DMAC_IN) != 0;
  if (!d_in && (ins & 1u)) {
    const uint64_t dmac = rec_dmac(r1);
    d_in = slot_first(set_find(t.macset, t.macset_mask, 2, t.epoch, dmac, usn_mac_hash(dmac)),
                      t.epoch) <= i;
  }
  return d_in;
}

/* key1 = a rule learned by a frame <= i: it is owned by S (so excluded) */
__device__ __forceinline__ uint32_t tx_learned_key1(const TxArgs &t, uint32_t x, uint32_t y, uint32_t z,
                                                    uint32_t meta, uint32_t i) {
  const unsigned long long *slot = set_find(t.ruleset, t.ruleset_mask, 4, t.epoch,
                                            usn_key_fp48(x, y, z, meta), usn_key_hash(x, y, z, meta));
  if (slot_first(slot, t.epoch) > i) return 0u;
  if (ld_sc1(slot + 2) != (((unsigned long long)y << 32) | x) ||
      ld_sc1(slot + 3) != (((unsigned long long)meta << 32) | z))
    atomicOr(t.counters + 1, 2u);                      // fingerprint collision: host redoes
  return USN_SLOT_VALID | (t.a[0].src << 16);
}

/* key2 = to_match_want_with_src(false) */
__device__ __forceinline__ void key2_of(const uint4 &r0, uint32_t &x, uint32_t &y, uint32_t &z,
                                        uint32_t &meta) {
  const uint32_t has = (r0.x >> 16) & 1u;
  x = r0.z;
  y = 0u;
  z = has ? (r0.w >> 16) : 0u;
  meta = usn_key_meta((r0.x >> 8) & 0xFFu, has ? USN_WANT_DPORT : 0u);
}

/* the decision from get_endpoint's result w (endpoint.rs:256-284) */
__device__ __forceinline__ uint32_t tx_lookup_dec(const ClassifyArgs &a, uint32_t fl, uint32_t w) {
  const uint32_t owner = w >> 16;
  const bool excl = w && ((w & USN_SLOT_NICOWNER) || owner == a.src);
  if (w && !excl) return usn_mkdec(USN_CLS_EP, USN_R_NONE, owner);
  if (fl & TXR_DHCPANS)
    return usn_mkdec(USN_CLS_DROP, USN_R_DHCP_NONE, 0xFFFFu) |
           (a.next_dhcp_set ? (USN_F_DHCP | USN_F_HOST) : 0u);
  return usn_mkdec(USN_CLS_DROP, excl ? USN_R_EXCLUDED : USN_R_NOMATCH, 0xFFFFu);
}

template <bool IN_LDS>
__device__ uint32_t decide_tx_ipv4(const TxArgs &t, const uint4 *T, const uint4 &r0,
                                   const uint4 &r1, uint32_t i, uint32_t ins) {
  const ClassifyArgs &a = t.a[0];
  const uint32_t fl = r0.x;
  if (!tx_dmac_in(t, fl, r1, i, ins)) return usn_mkdec(USN_CLS_NIC, USN_R_NONE, a.for_nic);   // :254-255
  uint32_t x, y, z, meta;
  key1_of(r0, x, y, z, meta);
  uint32_t w = ph_probe1<IN_LDS>(T, a, 0, x, y, z, meta);
  if (!w && (ins & 2u)) w = tx_learned_key1(t, x, y, z, meta, i);
  if (!w && (a.probe_mask & 2u)) {
    key2_of(r0, x, y, z, meta);
    w = ph_probe1<IN_LDS>(T, a, 1, x, y, z, meta);
  }
  return tx_lookup_dec(a, fl, w);
}

/* ---- the tx batch in one launch ------------------------------------------
 * A tile waits only on tiles with smaller indices, which are dispatched
 * before it (blocks go out in index order, dealt round-robin over the XCDs;
 * HIP does not promise it, so every wait is bounded: see below).  An
 * ordered-ticket counter instead (one atomic per block on one word) spread
 * the block starts over 12 us at 1024 blocks.  What crosses a tile boundary
 * goes through per-tile aux granules: 8 bytes {epoch, value}, each written
 * by ONE agent-scope (sc1, write-through) store and read by sc1 loads until
 * its tag is the batch epoch, so a granule is its own flag (MI355X guide,
 * Guideline 16 R2; no fences, no stale L1/L2 copies):
 *   phase 1  parse, flags and the answer-key probes of the tile; publish its
 *            last touching frame (LAST, LREC); take the last touching frame
 *            before the tile from the tiles before; cache hits; the
 *            first-occurrence claims of what the tile learns (atomics and
 *            sc1 stores, drained by every wave); then publish the last
 *            non-hit touching frame (HEAD, HREC) and INS, whose arrival also
 *            says that the tile's claims are in the sets (R1)
 *   phase 2  one wave waits for INS of every earlier tile; the run head
 *            before the tile, decisions (get_endpoint probes batched; set
 *            slots read sc1), run-head fill, learned list, order, header.
 * A wait that outlasts TX_SPIN_TICKS marks the batch (counters[3] = epoch;
 * later waits then give up at once): usn_finalize redoes it on the host. */
#define TXG_LAST 0u    /* 1 + tile-local index of the last touching frame, 0 none */
#define TXG_LREC 1u    /* 4 granules: its record (flags of the scan; zeros if none) */
#define TXG_INS 5u     /* bit 0/1: the tile inserted MACs / rules, bit 2: a set overflowed */
#define TXG_HEAD 6u    /* 1 + tile-local index of the last non-hit touching frame, 0 none */
#define TXG_HDEC 7u    /* the decision of TXG_HEAD's frame (out with the tile's decisions) */
#define TXG_PINS 11u   /* INS of every tile up to and including this one */
#define TXG_PHEAD 12u  /* 1 + batch index of the last non-hit touching frame up to this tile, 0 none */
#define TXG_CIN 13u    /* tile 0: 6 granules, the carried-in cache {state, dst, info[4]} */
#define TXG_EARLY 19u  /* (unused since round 6: EARLY is packed, TxArgs::early) bit 0/1: the tile has frames flagged to learn a MAC / rule (before
                          the hit pass: a superset of what it inserts), out with LAST */
#define TXG_PEARLY 20u /* EARLY of every tile up to and including this one */
static_assert(TXG_CIN + 6 <= TXA_GRANULES, "aux granules");
#define TX_SPIN_TICKS (200u * 100000u)   /* 200 ms of the 100 MHz real-time clock */

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;

__device__ __forceinline__ void g_put(unsigned long long *g, uint32_t epoch, uint32_t v) {
  __hip_atomic_store((gu64 *)g, ((unsigned long long)epoch << 32) | v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_put4(unsigned long long *g, uint32_t epoch, const uint4 &v) {
  g_put(g, epoch, v.x); g_put(g + 1, epoch, v.y); g_put(g + 2, epoch, v.z); g_put(g + 3, epoch, v.w);
}
__device__ __forceinline__ bool tx_timed_out(const TxArgs &t) {
  return __hip_atomic_load((gu32 *)(t.counters + 3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
         t.epoch;
}
/* the values of granules g[0..N) once all carry the batch epoch (the N
 * loads of a poll fly together); false after TX_SPIN_TICKS or once any wait
 * of the batch has timed out */
template <int N>
__device__ bool g_getn(const unsigned long long *g, const TxArgs &t, uint32_t (&v)[N]) {
  uint64_t t0 = 0;
  for (uint32_t it = 0;; ++it) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const unsigned long long x =
          __hip_atomic_load((gu64 *)(g + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v[k] = (uint32_t)x;
      ok &= (uint32_t)(x >> 32) == t.epoch;
    }
    if (ok) return true;
    if (tx_timed_out(t)) return false;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (it == 0) {
      t0 = now;
    } else if (now - t0 > TX_SPIN_TICKS) {
      atomicMax(t.counters + 3, t.epoch);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

/* one read of granule g: true (and v) when it carries the batch epoch */
__device__ __forceinline__ bool g_try(const unsigned long long *g, const TxArgs &t, uint32_t &v) {
  const unsigned long long x = __hip_atomic_load((gu64 *)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v = (uint32_t)x;
  return (uint32_t)(x >> 32) == t.epoch;
}

/* Tiles [0, tile): the OR of their INS and the last non-hit touching frame
 * among them (1 + batch index, 0 none), once every one of them has published
 * (INS comes after its claims landed).  All threads of the block: thread k
 * reads the INS/HEAD granules of tiles tile-1-k, tile-1-k-NTHREADS, ... down
 * to tile-TX_LOOKBACK, all loads of a poll together; the tiles below that are
 * covered by the prefix (PINS/PHEAD) that tile tile-TX_LOOKBACK-1 published
 * after its own look-back.  Results into *ins_out / *head_out (LDS, zeroed by
 * the caller); false after a timeout. */
#define TX_LB_PER_THREAD 4
#define TX_LOOKBACK (NTHREADS * TX_LB_PER_THREAD)
__device__ bool tx_lookback(const TxArgs &t, uint32_t tile, uint32_t *ins_out, uint32_t *head_out) {
  const uint32_t tid = threadIdx.x;
  uint32_t ins = 0, head = 0;
  bool ok = true;
#pragma unroll
  for (int k = 0; k < TX_LB_PER_THREAD; ++k) {
    const int u = (int)tile - 1 - (int)tid - k * (int)NTHREADS;
    if (u < 0 || !ok) continue;
    uint32_t v[2];
    ok = g_getn<2>(t.aux + (size_t)u * TXA_GRANULES + TXG_INS, t, v);   // INS, HEAD
    if (!ok) break;
    ins |= v[0] & 3u;
    const uint32_t h = min(v[1], (uint32_t)TILE);
    if (h) head = max(head, (uint32_t)u * TILE + h);
  }
  const int below = (int)tile - 1 - (int)TX_LOOKBACK;   // the prefix of [0, below]
  if (ok && tid == 0 && below >= 0) {
    uint32_t v[2];
    ok = g_getn<2>(t.aux + (size_t)below * TXA_GRANULES + TXG_PINS, t, v);   // PINS, PHEAD
    if (ok) { ins |= v[0] & 3u; head = max(head, v[1]); }
  }
  if (ins) atomicOr(ins_out, ins);
  if (head) atomicMax(head_out, head);
  return ok;
}

/* The OR of EARLY over tiles [0, tile) (EARLY goes out long before INS: a
 * tile whose predecessors flag nothing to learn need not wait for their
 * claims).  The last TX_LOOKBACK tiles' EARLY words are packed (TxArgs::
 * early), four per 16-byte agent-scope load, so the look-back of a tile deep
 * in an 8-ring grid is one load per thread instead of four loads of one line
 * each (round 5: 2048 lines per tile); the tiles below are covered by the
 * PEARLY prefix granule of tile tile - TX_LOOKBACK - 1. */
__device__ bool tx_lookback_early(const TxArgs &t, uint32_t tile, uint32_t *early_out) {
  const uint32_t tid = threadIdx.x;
  const int below = (int)tile - 1 - (int)TX_LOOKBACK;   // the prefix of [0, below]
  const uint32_t lo = below >= 0 ? (uint32_t)below + 1u : 0u;   // words of [lo, tile)
  uint32_t e = 0;
  bool ok = true;
  for (uint32_t g = (lo >> 2) + tid; (g << 2) < tile && ok; g += NTHREADS) {
    uint64_t t0 = 0;
    for (uint32_t it = 0;; ++it) {
      v4u32 v;
      asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)"
                   : "=v"(v) : "v"(t.early + 4u * g) : "memory");
      bool all = true;
      uint32_t acc = 0;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t u = 4u * g + j, w = v[j];
        if (u < lo || u >= tile) continue;
        all &= (w >> 16) == t.epoch;
        acc |= w & 3u;
      }
      if (all) { e |= acc; break; }
      if (tx_timed_out(t)) { ok = false; break; }
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (it == 0) {
        t0 = now;
      } else if (now - t0 > TX_SPIN_TICKS) {
        atomicMax(t.counters + 3, t.epoch);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  if (ok && tid == 0 && below >= 0) {
    uint32_t v[1];
    ok = g_getn<1>(t.aux + (size_t)below * TXA_GRANULES + TXG_PEARLY, t, v);
    if (ok) e |= v[0];
  }
  if (e) atomicOr(early_out, e);
  return ok;
}

__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

/* tile 0's carried-in cache {state, dst, info[4]} (zeros after a timeout) */
__device__ __forceinline__ void tx_load_cin(const TxArgs &t, uint32_t *cin) {
  uint32_t v[6];
  const bool ok = g_getn<6>(t.aux + TXG_CIN, t, v);
  for (int k = 0; k < 6; ++k) cin[k] = ok ? v[k] : 0u;
}

/* LDS of the tx kernel: core | records | decisions | table (LDS) | bridge.
 * The header loads' per-wave redistribution scratch (3 KiB per wave: 64
 * frames x 48 bytes) aliases the records and decisions, which are written
 * only after every wave has parsed (a barrier in between). */
#define TX_SCRATCH_BYTES ((size_t)NWAVES * 64 * 48)
__host__ __device__ inline size_t tx_lds_head(uint32_t nbins) {
  const size_t recs = (size_t)TILE * 16 + (size_t)TILE * 4;
  return lds_core_bytes(nbins) + (recs > TX_SCRATCH_BYTES ? recs : TX_SCRATCH_BYTES);
}

#ifndef USN_TX_COAL   /* coalesced header loads at a fixed stride (0: each lane its own frame) */
#define USN_TX_COAL 1
#endif
#ifndef USN_TX_PIPE   /* phase 1: probes of a round issued as it is parsed; LDS-only barrier */
#define USN_TX_PIPE 1
#endif
template <bool LDS>
__global__ __launch_bounds__(NTHREADS) __attribute__((amdgpu_waves_per_eu(NTHREADS / 64)))
void tx_kernel(TxArgs t) {   // (4 workgroups per CU: 1024 tiles of 1M frames all resident)
  extern __shared__ __align__(16) uint8_t smem[];
  /* tile: this workgroup's tile in the launch (the protocol's); rt: in its
     ring (rings > 1: ring k's tiles follow ring k - 1's, TxArgs) */
  const uint32_t tile = blockIdx.x;
  uint32_t ring = 0;
#pragma unroll
  for (uint32_t k = 1; k < USN_TX_RINGS; ++k) ring += (k < t.rings && tile >= t.tile_base[k]) ? 1u : 0u;
  const ClassifyArgs &a = t.a[ring];
  const uint32_t rt = tile - t.tile_base[ring];
  const Lds L = carve(smem, t.a[0].nbins);
  uint4 *srec = reinterpret_cast<uint4 *>(smem + lds_core_bytes(a.nbins));   // the tile's records
  uint32_t *sdec = reinterpret_cast<uint32_t *>(srec + TILE);               // its decisions
  uint4 *stab = reinterpret_cast<uint4 *>(smem + tx_lds_head(a.nbins));
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  __shared__ uint32_t s_last, s_lastnh, s_ins, s_ovf, s_insall, s_hidx, s_before, s_head;
  __shared__ uint32_t s_early, s_early_all, s_slow, s_dlearn;
  __shared__ uint32_t s_cin[6];   // the carried-in cache {state, dst, info[4]} (tile 0's)
  __shared__ uint4 s_brec;
  __shared__ uint32_t s_carry[8];
  __shared__ uint32_t s_misc[8];   // [0] 1+last touching, [1] host-list fill, [3..5] NIC/FLOOD/DROP
  __shared__ uint32_t s_listen[2 * TX_LISTEN_LDS];
  STAMP_DECL
  STAMP(0);   // tickets out of step with the host: the waits time out
  USN_PRIO(USN_AB_TXPRIO, 3);   // while the tile's header loads issue
  const uint64_t base = (uint64_t)rt * TILE;      // the tile's first frame in its ring
  const uint32_t vbase = tile * TILE;             // ... in the launch
  const uint32_t nt = (uint32_t)min((uint64_t)TILE, a.n - base);
  unsigned long long *aux = t.aux + (size_t)tile * TXA_GRANULES;
  const uint4 *T = a.table;
  if (LDS) {
    for (uint32_t k = tid; k < a.table_units; k += NTHREADS) stab[k] = a.table[k];
    T = stab;
  }
  /* the bridge snapshot set goes to LDS when small; its loads go out first
     (USN_TX_PIPE), so that its LDS copy and the barrier after it wait for
     them and not for the header loads */
  const unsigned long long *BS = t.bridge_set;
  const bool bridge_lds = t.bridge_mask < TX_BRIDGE_LDS_SLOTS;
  unsigned long long *bs = reinterpret_cast<unsigned long long *>(stab + (LDS ? table_lds_units(a.table_units) : 0));
  constexpr uint32_t BRIDGE_PER_THREAD = TX_BRIDGE_LDS_SLOTS / NTHREADS;
  unsigned long long bv[USN_TX_PIPE ? BRIDGE_PER_THREAD : 1];
  if (USN_TX_PIPE && bridge_lds) {
#pragma unroll
    for (uint32_t j = 0; j < BRIDGE_PER_THREAD; ++j) {
      const uint32_t k = tid + j * NTHREADS;
      bv[j] = k <= t.bridge_mask ? t.bridge_set[k] : 0ull;
    }
  }
  // the source's listening triples (read by every frame): to LDS with the bridge
  const bool listen_lds = t.n_listen <= TX_LISTEN_LDS;
  const uint32_t lv = listen_lds && tid < 2 * t.n_listen ? t.listen[tid] : 0u;
  /* all header loads of the tile first (48 B x 4 frames per lane in flight:
     the MACs and up to byte 39 for parse; tools/stride_floor.hip, 4M frames
     at a 64-byte stride: 61.6 us reading 48 B per frame, 73.3 us reading 64).
     Every round's frame address first: an offsets[] read feeding a round's
     loads made hipcc wait for all earlier loads before each round's. */
  uint4 qq[ROUNDS][4];
  uint4 cc[ROUNDS][3];
  uint32_t ll[ROUNDS];
  const uint8_t *fps[ROUNDS];
#pragma unroll   // lengths before the headers: round 0's parse then waits for round 0 only
  for (uint32_t r = 0; r < ROUNDS; ++r) ll[r] = a.lens[base + min(r * NTHREADS + tid, nt - 1)];
  if (a.offsets) {
    uint64_t off[ROUNDS];
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) off[r] = a.offsets[base + min(r * NTHREADS + tid, nt - 1)];
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) fps[r] = a.frames + off[r];
  } else {
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) fps[r] = a.frames + (base + min(r * NTHREADS + tid, nt - 1)) * a.stride;
  }
  /* fixed stride (16-byte aligned): coalesced loads.  Lane u of instruction k
     reads part u % 3 of frame u / 3 (u = 64k + lane) of its wave's 64 frames
     of the round, so an instruction reads 1 KiB runs instead of 16 bytes at
     every frame start (tools/probe_floor, 8M x 64 B: 86 vs 145 us); the parse
     loop moves each part to its frame's lane through the wave's LDS scratch.
     Otherwise lane L reads its own frame.  One load instruction either way. */
  const bool coal = USN_TX_COAL && !a.offsets && (a.stride & 15u) == 0 &&
                    (reinterpret_cast<uintptr_t>(a.frames) & 15u) == 0;
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
      const uint32_t u = 64u * k + lane, f = (u * 0xAAABu) >> 17, part = u - 3u * f;
      const uint64_t fi = base + min(r * NTHREADS + wave * 64u + f, nt - 1);
      const uint8_t *pc = a.frames + fi * a.stride + part * 16u;
      const uint8_t *pl = fps[r] + 16u * k;
      cc[r][k] = ld_stream(reinterpret_cast<const uint4 *>(coal ? pc : pl));
    }
    qq[r][3] = make_uint4(0, 0, 0, 0);
  }
  USN_PRIO(USN_AB_TXPRIO, 0);
  /* the LDS state's zeroing after the loads went out: the LDS barrier below
     publishes it (a barrier before the loads held them for every wave) */
  if (tid == 0) {
    s_last = 0; s_lastnh = 0; s_ins = 0; s_ovf = 0; s_insall = 0; s_hidx = 0; s_before = 0;
    s_early = 0; s_early_all = 0; s_slow = 0; s_dlearn = 0;
  }
  if (tid < 8) s_misc[tid] = 0;
  hist_zero(L.hist, a.nbw);
  // tile 0: the carried-in cache of this source; counters for phase 2 (all
  // wait for tile 0; resolve_carry's barriers wait for its header loads)
  if (tile == 0) {
    if (tid < USN_TXC_WORDS && tid != 3)   // learned, flags, sets, host frames (3: the timeout epoch stays)
      __hip_atomic_store((gu32 *)(t.counters + tid), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    resolve_carry(a, s_carry, L.scratch);
    if (tid == 0) {
      for (int k = 0; k < 6; ++k) {
        s_cin[k] = s_carry[k];
        g_put(aux + TXG_CIN + k, t.epoch, s_carry[k]);
      }
      usn_summary *S = a.summary;
      S->cin_state = s_carry[0]; S->cin_dst = s_carry[1];
      for (int k = 0; k < 4; ++k) S->cin_info[k] = s_carry[2 + k];
      S->n_frames = (uint32_t)a.n; S->n_tiles = a.ntiles;
      S->n_ep = a.n_ep; S->n_bins = a.nbins;
      S->flags = 0; S->first_break = 0xFFFFFFFFu;
    }
  }
  if (listen_lds && tid < 2 * TX_LISTEN_LDS) s_listen[tid] = lv;
  if (bridge_lds) {
    if (USN_TX_PIPE) {
#pragma unroll
      for (uint32_t j = 0; j < BRIDGE_PER_THREAD; ++j) {
        const uint32_t k = tid + j * NTHREADS;
        if (k <= t.bridge_mask) bs[k] = bv[j];
      }
    } else {
      for (uint32_t k = tid; k <= t.bridge_mask; k += NTHREADS) bs[k] = t.bridge_set[k];
    }
    BS = bs;
  }
  if (USN_TX_PIPE) {
    // LDS only: the header loads stay in flight; each round below waits for its own
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  } else {
    __syncthreads();
  }
  STAMP(1);
  // parse and flag every round; the answer-key probes of all rounds are then
  // issued together (two round trips for the tile's four rounds)
  uint32_t last = 0;
  uint4 rec[ROUNDS];
  // keys probed in phase 1: [0, R) answer keys (table K1), [R, 2R) key1 (K1)
  // and [2R, 3R) key2 (K2) of the frames that will likely need get_endpoint
  // (dmac in the bridge snapshot; phase 2 probes any other that turns out to)
  constexpr int R3 = 3 * ROUNDS;
  bool need[R3];
  uint32_t ax[R3], ay[R3], az[R3], am[R3];
  PhKeyH pk[R3];      // USN_TX_PIPE: each round's displacement reads go out when it is parsed
  uint32_t pd[R3];
  bool pon[R3];
#pragma unroll
  for (int k = 0; k < R3; ++k) { need[k] = false; ax[k] = 0; ay[k] = 0; az[k] = 0; am[k] = 0; }
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    if (coal) {   // the wave's parts to their frames' lanes (in order per wave: no barrier)
      typedef __attribute__((address_space(3))) v4u32 lds_v4;
      lds_v4 *ws = (lds_v4 *)srec + wave * 192u;
#pragma unroll
      for (uint32_t k = 0; k < 3; ++k) ws[64u * k + lane] = v4u32{cc[r][k].x, cc[r][k].y, cc[r][k].z, cc[r][k].w};
#pragma unroll
      for (uint32_t k = 0; k < 3; ++k) {
        const v4u32 v = ws[3u * lane + k];
        qq[r][k] = make_uint4(v.x, v.y, v.z, v.w);
      }
    } else {
#pragma unroll
      for (uint32_t k = 0; k < 3; ++k) qq[r][k] = cc[r][k];
    }
    const uint4 *q = qq[r];
    Parsed p;
    parse(q, local < nt ? ll[r] : 0u, fps[r], a.window, p);
    const uint64_t dmac = (uint64_t)q[0].x | ((uint64_t)(q[0].y & 0xFFFFu) << 32);
    const uint64_t smac = (uint64_t)(q[0].y >> 16) | ((uint64_t)q[0].z << 16);
    const bool loop = p.status == 1u && (p.dst >> 24) == 127u;
    const uint32_t touch = p.status == 0u ? 0u : p.status >= 4u ? 3u
                         : (p.status == 1u && !loop) ? 1u : 2u;
    uint32_t f = (touch << TXR_TOUCH_SHIFT);
    uint4 r0 = make_uint4(p.status == 4u ? 0u : p.i0, p.src, p.dst, p.ports);
    if (p.status != 1u) { r0.y = 0; r0.z = 0; r0.w = 0; }
    // the frame before it in the tile (lane - 1) retains the same info: this
    // one is a cache hit (or the host's, as that one is) and learns nothing,
    // so its answer key need not be probed
    const uint32_t i0 = r0.x & TXR_I0_MASK;
    const uint32_t pi0 = __shfl_up(touch == 1u ? i0 : 0xFFFFFFFFu, 1, 64);
    const uint32_t py = __shfl_up(r0.y, 1, 64), pz = __shfl_up(r0.z, 1, 64), pw = __shfl_up(r0.w, 1, 64);
    const bool repeat = lane > 0 && touch == 1u && pi0 == i0 && py == r0.y && pz == r0.z && pw == r0.w;
    if (touch == 1u || touch == 2u) {
      const bool s_in = bridge_lds ? bridge_has_lds(BS, t.bridge_mask, smac)
                                   : bridge_has(BS, t.bridge_mask, smac);
      const bool d_in = bridge_lds ? bridge_has_lds(BS, t.bridge_mask, dmac)
                                   : bridge_has(BS, t.bridge_mask, dmac);
      if (s_in) f |= TXR_SMAC_IN;
      if (d_in) f |= TXR_DMAC_IN;
      if (!(smac & 1u) && !s_in) f |= TXR_LEARNMAC;           // is_unicast && not contained
    }
    if (touch == 3u) f |= TXR_HOST;                           // later fragment: map lookup
    if (p.status == 5u) f |= TXR_WINDOW;                      // ports past the window
    if (touch == 1u) {
      // (W.dst, proto, W.dport) in S.listening?  W.dst = src, W.dport = sport
      typedef __attribute__((address_space(3))) const uint32_t lds_u32;
      const bool listening = listen_lds ? tx_listening((const lds_u32 *)s_listen, t.n_listen, p)
                                        : tx_listening(t.listen, t.n_listen, p);
      // is_unspecified() is smoltcp 0.7.0's 0.0.0.0/8 range test (src[0] == 0), pkt.rs:46
      const bool dhcp_req = p.proto == 17u && (p.src >> 24) == 0u && p.has_ports && p.sport == 68u &&
                            p.dport == 67u && (p.dst & 0xFFu) == 255u;
      if (!listening && dhcp_req) f |= TXR_HOST;              // NIC.next_dhcp := S (cross-endpoint)
      if (!listening && !dhcp_req && !repeat) {   // learned unless the table has the answer key
        want_key(make_uint4(p.i0, p.src, p.dst, p.ports), ax[r], ay[r], az[r], am[r]);
        need[r] = true;
      }
      if (p.proto == 17u && p.has_ports && p.sport == 67u && p.dport == 68u) f |= TXR_DHCPANS;
    }
    if (p.status == 1u && p.frag_first) f |= TXR_FRAG1;
    r0.x = i0 | f;
    rec[r] = r0;
    if (local < nt && touch) last = local + 1;
    const uint32_t kind = i0 & 0xFFu;
    if (touch == 1u && !(f & TXR_HOST) && (f & TXR_DMAC_IN) && !repeat && kind != USN_INFO_ARP &&
        kind != USN_INFO_EAPOL) {
      need[ROUNDS + r] = need[2 * ROUNDS + r] = true;
      key1_of(r0, ax[ROUNDS + r], ay[ROUNDS + r], az[ROUNDS + r], am[ROUNDS + r]);
      key2_of(r0, ax[2 * ROUNDS + r], ay[2 * ROUNDS + r], az[2 * ROUNDS + r], am[2 * ROUNDS + r]);
    }
    if (USN_TX_PIPE) {   // under the later rounds' header loads
#pragma unroll
      for (uint32_t j = 0; j < 3; ++j) {
        const uint32_t i = j * ROUNDS + r;
        ph_disp_issue<LDS>(T, a, j < 2 ? 0 : 1, ax[i], ay[i], az[i], am[i], need[i], pk[i], pd[i], pon[i]);
      }
    }
  }
  uint32_t w1e[ROUNDS], w2e[ROUNDS];   // key1 / key2 results, valid where need[R + r]
  bool pre[ROUNDS];
  {
    uint32_t w[R3];
    if (USN_TX_PIPE) ph_slots_hit<LDS, R3, 2 * ROUNDS>(T, a, ax, ay, az, am, pk, pd, pon, w);
    else ph_probe_many<LDS, R3, 2 * ROUNDS>(T, a, ax, ay, az, am, need, w);
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) {
      if (need[r] && !w[r]) rec[r].x |= TXR_LEARNRULE;
      pre[r] = need[ROUNDS + r];
      w1e[r] = w[ROUNDS + r];
      w2e[r] = w[2 * ROUNDS + r];
    }
  }

  STAMP(2);
  // every wave is done with its header scratch before the records overwrite it
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  // ---- the tile's records in LDS; each frame's previous touching frame
  uint32_t vt[ROUNDS], prev[ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    if (local >= nt) rec[r] = make_uint4(0, 0, 0, 0);
    srec[local] = rec[r];
    vt[r] = (local < nt && tx_touch(rec[r])) ? local + 1 : 0u;
    if (local < nt && (rec[r].x & (TXR_LEARNMAC | TXR_LEARNRULE)))
      atomicOr(&s_early, ((rec[r].x & TXR_LEARNMAC) ? 1u : 0u) | ((rec[r].x & TXR_LEARNRULE) ? 2u : 0u));
  }
  // (publishing LAST before the probes instead: 52.9 -> 61 us per 1M frames,
  // the probes' compiler-placed vmcnt(0) then also waits for the sc1 stores)
  if (last) atomicMax(&s_last, last);
  tile_prefix_max(vt, L, prev);   // its barriers also publish srec, s_last and s_early
  if (tid == 0) {
    const uint32_t lt = s_last;
    g_put4(aux + TXG_LREC, t.epoch, lt ? srec[lt - 1] : make_uint4(0, 0, 0, 0));
    g_put(aux + TXG_LAST, t.epoch, lt);
    __hip_atomic_store((gu32 *)(t.early + tile), (t.epoch << 16) | s_early, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);   // EARLY, packed (tx_lookback_early)
  }
  // tid 0: tile - 1's LAST and LREC granules read now, under the hit pass
  // (the walk back below takes them when they carry the epoch, else polls)
  unsigned long long pl[5] = {0, 0, 0, 0, 0};
  if (tid == 0 && tile > 0) {
#pragma unroll
    for (int k = 0; k < 5; ++k)
      pl[k] = __hip_atomic_load((gu64 *)(t.aux + (size_t)(tile - 1) * TXA_GRANULES + TXG_LAST + k),
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  STAMP(3);
  // ---- cache hits (endpoint.rs:186-191); what a frame really learns is
  //      claimed in the epoch-tagged sets with its index (first occurrence wins).
  //      Only the tile's first touching frame compares with a frame before the
  //      tile: it is done after the others, once the tiles before have
  //      published (the walk back), and HEAD / INS go out before that walk
  //      whenever that frame cannot change them (a later frame is a non-hit,
  //      and it has nothing to claim): the tiles after then do not wait on the
  //      tiles before this one through it.
  uint32_t last_nh = 0, ins = 0;
  int deferred = -1;   // the round of this lane's first touching frame (touch 1, prev 0)
  auto hit_claim = [&](uint32_t r, bool hit) {
    const uint32_t local = r * NTHREADS + tid;
    const uint32_t i = vbase + local;
    uint32_t fl = rec[r].x;
    if (hit) fl |= TXR_HIT;
    rec[r].x = fl;
    if (!hit) last_nh = local + 1;
    if (hit || (fl & TXR_HOST)) return;
    if (fl & (TXR_LEARNMAC | TXR_LEARNRULE)) {
      if (fl & TXR_LEARNMAC) {
        const uint64_t m = rec_smac(frame_head(a, base + local));
        unsigned long long *slot = set_claim(t.macset, t.macset_mask, 2, t.epoch, m,
                                             usn_mac_hash(m), &s_ovf);
        if (slot) first_index_update(slot + 1, t.epoch, i);
        ins |= 1u;
      }
      if (fl & TXR_LEARNRULE) {
        uint32_t x, y, z, meta;
        want_key(rec[r], x, y, z, meta);
        const uint64_t fp = usn_key_fp48(x, y, z, meta);
        unsigned long long *slot = set_claim(t.ruleset, t.ruleset_mask, 4, t.epoch, fp,
                                             usn_key_hash(x, y, z, meta), &s_ovf);
        if (slot) {
          st_sc1(slot + 2, ((unsigned long long)y << 32) | x);   // full key: collision check below
          st_sc1(slot + 3, ((unsigned long long)meta << 32) | z);
          first_index_update(slot + 1, t.epoch, i);
        }
        ins |= 2u;
      }
    }
  };
  // (a frame equal to a host-decided one takes the host's cache effect)
  auto same_as = [&](uint32_t r, const uint4 &pr, bool &hit) {
    const uint32_t info0 = rec[r].x & TXR_I0_MASK;
    const bool same = tx_touch(pr) == 1u && (pr.x & TXR_I0_MASK) == info0 && pr.y == rec[r].y &&
                      pr.z == rec[r].z && pr.w == rec[r].w;
    if (same && (pr.x & TXR_HOST)) rec[r].x |= TXR_HOST;
    else hit = same;
  };
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    if (local >= nt) continue;
    const uint32_t touch = tx_touch(rec[r]);
    if (!touch) continue;
    bool hit = false;
    if (touch == 1u) {
      if (!prev[r]) { deferred = (int)r; continue; }
      same_as(r, srec[prev[r] - 1], hit);
    }
    hit_claim(r, hit);
  }
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r)
    if ((int)r == deferred && (rec[r].x & (TXR_LEARNMAC | TXR_LEARNRULE))) atomicOr(&s_dlearn, 1u);
  if (last_nh) atomicMax(&s_lastnh, last_nh);
  if (ins) atomicOr(&s_ins, ins);
  vm_drain();                  // this wave's claims (atomics, sc1 stores) have landed
  __syncthreads();             // (and every frame has read srec)
  // HEAD and INS now unless the first touching frame can change them
  const bool early_pub = s_lastnh != 0 && s_dlearn == 0;
  if (tid == 0) {
    if (early_pub) {   // INS last: its arrival also says the claims above have landed (R1)
      g_put(aux + TXG_HEAD, t.epoch, s_lastnh);
      g_put(aux + TXG_INS, t.epoch, s_ins | (s_ovf ? 4u : 0u));
    }
    // the last touching frame before the tile (a tile without one is skipped)
    uint32_t before = 0;
    uint4 brec = make_uint4(0, 0, 0, 0);
    for (int u = (int)tile - 1; u >= 0; --u) {
      uint32_t v[5];   // LAST, LREC
      bool pre = u == (int)tile - 1;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        v[k] = (uint32_t)pl[k];
        pre &= (uint32_t)(pl[k] >> 32) == t.epoch;
      }
      if (!pre && !g_getn<5>(t.aux + (size_t)u * TXA_GRANULES + TXG_LAST, t, v)) break;
      const uint32_t lu = min(v[0], (uint32_t)TILE);
      if (lu) {
        before = (uint32_t)u * TILE + lu;
        brec = make_uint4(v[1], v[2], v[3], v[4]);
        break;
      }
    }
    s_before = before;
    s_brec = brec;
    if (tile > 0 && before == 0) tx_load_cin(t, s_cin);   // the first touching frame's cache
  }
  __syncthreads();
  if (deferred >= 0) {   // the tile's first touching frame
    last_nh = 0;
    ins = 0;
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) {
      if ((int)r != deferred) continue;
      bool hit = false;
      if (s_before) {
        same_as(r, s_brec, hit);
      } else {
        const uint32_t info0 = rec[r].x & TXR_I0_MASK;
        hit = (s_cin[0] & USN_CS_VALID) && s_cin[2] == info0 && s_cin[3] == rec[r].y &&
              s_cin[4] == rec[r].z && s_cin[5] == rec[r].w;
      }
      hit_claim(r, hit);
    }
    if (last_nh) atomicMax(&s_lastnh, last_nh);
    if (ins) atomicOr(&s_ins, ins);
    vm_drain();
  }
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) srec[r * NTHREADS + tid] = rec[r];   // flags after the hit pass
  __syncthreads();
  if (tid == 0 && !early_pub) {   // INS last: its arrival also says the claims above have landed (R1)
    g_put(aux + TXG_HEAD, t.epoch, s_lastnh);
    g_put(aux + TXG_INS, t.epoch, s_ins | (s_ovf ? 4u : 0u));
  }
  STAMP(4);
  USN_PRIO(USN_AB_TXPRIO, 1);   // phase 2: ahead of the younger tiles' parse
  // ---- phase 2: the sets as every earlier frame left them, and the last
  //      non-hit touching frame before the tile.  When no earlier tile
  //      flagged anything to learn (EARLY, out with LAST), no earlier tile
  //      claims: only the nearest tiles' HEAD is waited for.  Otherwise, or
  //      when the head is further back, every earlier tile's INS (tx_lookback).
  // tid 0: tile - 1's HEAD read now, under the EARLY look-back
  unsigned long long ph = 0;
  if (tid == 0 && tile > 0)
    ph = __hip_atomic_load((gu64 *)(t.aux + (size_t)(tile - 1) * TXA_GRANULES + TXG_HEAD),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  tx_lookback_early(t, tile, &s_early_all);
  __syncthreads();
  if (tid == 0) {
    bool slow = s_early_all != 0;
    if (!slow) {
      uint32_t hx = 0;
      int u = (int)tile - 1;
      for (int steps = 0; u >= 0 && steps < 8; --u, ++steps) {
        uint32_t v[1] = {(uint32_t)ph};
        const bool pre = steps == 0 && (uint32_t)(ph >> 32) == t.epoch;
        if (!pre && !g_getn<1>(t.aux + (size_t)u * TXA_GRANULES + TXG_HEAD, t, v)) break;
        const uint32_t h = min(v[0], (uint32_t)TILE);
        if (h) { hx = (uint32_t)u * TILE + h; break; }
      }
      if (hx || u < 0) s_hidx = hx;   // found, or none in the batch
      else slow = true;               // further back than 8 tiles
    }
    s_slow = slow;
  }
  __syncthreads();
  if (s_slow) {
    tx_lookback(t, tile, &s_insall, &s_hidx);
    __syncthreads();
  }
  if (tid == 0) {   // this tile's prefixes, for the tiles TX_LOOKBACK + 1 and more after it
    const uint32_t own = s_lastnh;
    g_put(aux + TXG_PINS, t.epoch, s_insall | s_ins);
    g_put(aux + TXG_PHEAD, t.epoch, own ? vbase + own : s_hidx);
    g_put(aux + TXG_PEARLY, t.epoch, s_early_all | s_early);
  }
  const uint32_t insall = __builtin_amdgcn_readfirstlane(s_insall | s_ins);
  if (tid == 0) {
    if (s_ovf) atomicOr(t.counters + 1, 1u);
    if (s_ins) atomicOr(t.counters + 2, s_ins);
  }
  STAMP(5);
  // MACs (dmac test, the first learner's smac) only when some frame <= this tile learned one
  uint4 r1[ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    r1[r] = make_uint4(0, 0, 0, 0);
    if ((insall & 1u) && local < nt) r1[r] = frame_head(a, base + local);
  }
  const uint32_t ins_d = insall;
  const uint32_t my_nh = s_lastnh;   // 1 + this tile's last non-hit touching frame
  uint32_t dec[ROUNDS], v[ROUNDS], head[ROUNDS];
  // every decision but get_endpoint's first; then key1 and key2 of all the
  // rounds that need get_endpoint are probed together (two round trips for
  // the tile instead of up to four per round), then those decisions
  bool use[2 * ROUNDS];
  uint32_t kx[2 * ROUNDS], ky[2 * ROUNDS], kz[2 * ROUNDS], km[2 * ROUNDS], w[2 * ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    const uint32_t fl = rec[r].x, touch = local < nt ? tx_touch(rec[r]) : 0u, kind = fl & 0xFFu;
    use[r] = false; use[ROUNDS + r] = false;
    kx[r] = ky[r] = kz[r] = km[r] = 0;
    kx[ROUNDS + r] = ky[ROUNDS + r] = kz[ROUNDS + r] = km[ROUNDS + r] = 0;
    uint32_t d;
    if (touch == 0u) {
      d = usn_mkdec(USN_CLS_DROP, USN_R_PARSE, 0xFFFFu);
    } else if (fl & TXR_HOST) {
      d = usn_mkdec(USN_CLS_DROP, (fl & TXR_WINDOW) ? USN_R_WINDOW : touch == 3u ? USN_R_FRAGMISS
                                                                          : USN_R_NOMATCH, 0xFFFFu) |
          USN_F_HOST;
    } else if (fl & TXR_HIT) {
      d = USN_F_CACHE;                                     // the run head's, below
    } else if (kind == USN_INFO_ARP || kind == USN_INFO_EAPOL) {
      d = usn_mkdec(USN_CLS_FLOOD, USN_R_NONE, 0xFFFFu);
    } else if (touch == 2u) {
      d = usn_mkdec(USN_CLS_DROP, USN_R_LOOPBACK, 0xFFFFu);
    } else if (!tx_dmac_in(t, fl, r1[r], vbase + local, ins_d)) {
      d = usn_mkdec(USN_CLS_NIC, USN_R_NONE, a.for_nic);   // endpoint.rs:254-255
    } else {
      d = usn_mkdec(USN_CLS_DROP, USN_R_NOMATCH, 0xFFFFu);
      use[r] = true;
      use[ROUNDS + r] = use[r] && !pre[r];                   // not probed in phase 1
      key1_of(rec[r], kx[r], ky[r], kz[r], km[r]);
      key2_of(rec[r], kx[ROUNDS + r], ky[ROUNDS + r], kz[ROUNDS + r], km[ROUNDS + r]);
    }
    dec[r] = d;
  }
  {
    bool late = false;
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r) late |= use[ROUNDS + r];
    if (__any(late)) {   // frames whose dmac a MAC learned earlier in the batch put on this path
      bool u2[2 * ROUNDS];
#pragma unroll
      for (uint32_t r = 0; r < ROUNDS; ++r) { u2[r] = use[ROUNDS + r]; u2[ROUNDS + r] = use[ROUNDS + r]; }
      ph_probe_many<LDS, 2 * ROUNDS, ROUNDS>(T, a, kx, ky, kz, km, u2, w);
    }
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; ++r)
      if (pre[r]) { w[r] = w1e[r]; w[ROUNDS + r] = w2e[r]; }
  }
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    v[r] = 0;
    if (local >= nt) { dec[r] = 0; continue; }
    const uint32_t i = vbase + local;
    const uint32_t fl = rec[r].x, touch = tx_touch(rec[r]);
    uint32_t d = dec[r];
    if (use[r]) {   // key1, then a key1 learned by a frame <= i, then key2 (endpoint.rs:317-327)
      uint32_t wr = w[r];
      if (!wr && (ins_d & 2u)) wr = tx_learned_key1(t, kx[r], ky[r], kz[r], km[r], i);
      if (!wr) wr = w[ROUNDS + r];
      d = tx_lookup_dec(a, fl, wr);
    }
    if (fl & TXR_FRAG1) d |= USN_F_FRAG1;                  // first fragment: remembered (host map)
    // the first frame that learns an item lists it for the host registry / bridge
    if (touch && !(fl & (TXR_HIT | TXR_HOST)) && (fl & (TXR_LEARNMAC | TXR_LEARNRULE))) {
      bool learned = false;
      if (fl & TXR_LEARNMAC) {
        const uint64_t m = rec_smac(r1[r]);
        if (slot_first(set_find(t.macset, t.macset_mask, 2, t.epoch, m, usn_mac_hash(m)), t.epoch) == i) {
          const uint32_t pos = atomicAdd(t.counters, 1u);
          if (ring) atomicAdd(t.counters + USN_TXC_LEARNED + ring, 1u);
          if (pos < t.learned_cap) {
            t.learned[2 * pos] = make_uint4(i, 0u, 0u, 0u);
            t.learned[2 * pos + 1] = make_uint4((uint32_t)m, (uint32_t)(m >> 32), 0u, 0u);
          } else {
            atomicOr(t.counters + 1, 4u);
          }
          learned = true;
        }
      }
      if (fl & TXR_LEARNRULE) {
        uint32_t x, y, z, meta;
        want_key(rec[r], x, y, z, meta);
        const unsigned long long *slot = set_find(t.ruleset, t.ruleset_mask, 4, t.epoch,
                                                  usn_key_fp48(x, y, z, meta),
                                                  usn_key_hash(x, y, z, meta));
        if (slot_first(slot, t.epoch) == i) {
          if (ld_sc1(slot + 2) != (((unsigned long long)y << 32) | x) ||
              ld_sc1(slot + 3) != (((unsigned long long)meta << 32) | z))
            atomicOr(t.counters + 1, 2u);
          const uint32_t pos = atomicAdd(t.counters, 1u);
          if (ring) atomicAdd(t.counters + USN_TXC_LEARNED + ring, 1u);
          if (pos < t.learned_cap) {
            t.learned[2 * pos] = make_uint4(i, 1u, 0u, 0u);
            t.learned[2 * pos + 1] = make_uint4(x, y, z, meta);
          } else {
            atomicOr(t.counters + 1, 4u);
          }
          learned = true;
        }
      }
      if (learned) d |= USN_F_LEARN;
    }
    dec[r] = d;
    sdec[local] = d;
    v[r] = (touch && !(fl & TXR_HIT)) ? local + 1 : 0u;
    if (local + 1 == my_nh) g_put(aux + TXG_HDEC, t.epoch, d);   // for the tiles after
  }
  if (tid == 0) {
    // the decision of the run head before the tile: that tile's own, published
    // with its decisions (round 1 recomputed it here from the head's record:
    // up to four dependent probes in one lane)
    const uint32_t hx = s_hidx;
    uint32_t hd = 0;
    if (!hx) {   // no non-hit touching frame before the tile: the carried-in cache's
      if (tile > 0) tx_load_cin(t, s_cin);
      hd = s_cin[1];
    } else {
      uint32_t hv[1];
      if (g_getn<1>(t.aux + (size_t)((hx - 1) / TILE) * TXA_GRANULES + TXG_HDEC, t, hv)) hd = hv[0];
    }
    s_head = hd;
    if (ring && rt == 0) {   // ring k's summary: the cache ring k - 1 hands on (state after its last frame)
      usn_summary *S = a.summary;
      const uint32_t st = s_before ? (tx_touch(s_brec) == 1u && !(s_brec.x & TXR_HOST) ? USN_CS_VALID : 0u)
                                   : s_cin[0];
      S->cin_state = st;
      S->cin_dst = (hx ? hd : s_cin[1]) & USN_PARITY_MASK;
      if (s_before) {
        S->cin_info[0] = s_brec.x & TXR_I0_MASK; S->cin_info[1] = s_brec.y;
        S->cin_info[2] = s_brec.z; S->cin_info[3] = s_brec.w;
      } else {
        for (int k = 0; k < 4; ++k) S->cin_info[k] = s_cin[2 + k];
      }
      S->n_frames = (uint32_t)a.n; S->n_tiles = a.ntiles;
      S->n_ep = a.n_ep; S->n_bins = a.nbins;
      S->flags = 0; S->first_break = 0xFFFFFFFFu;
    }
  }
  STAMP(6);
  tile_prefix_max(v, L, head);   // its barriers also publish sdec and s_head
  uint32_t my_last = 0, my_touch = 0, my_dec = 0, my_host = 0;
  uint4 my_info = make_uint4(0, 0, 0, 0);
  uint32_t *hl = a.host_list + (size_t)rt * TILE;
  uint32_t bins[ROUNDS];
#pragma unroll
  for (uint32_t r = 0; r < ROUNDS; ++r) {
    const uint32_t local = r * NTHREADS + tid;
    const bool valid = local < nt;
    if (valid && (rec[r].x & TXR_HIT)) {
      const uint32_t hd = head[r] ? sdec[head[r] - 1] : s_head;
      dec[r] = (hd & USN_PARITY_MASK) | USN_F_CACHE | (dec[r] & USN_F_FRAG1);
    }
    if (valid) a.decisions[base + local] = dec[r];
    const uint32_t touch = valid ? tx_touch(rec[r]) : 0u;
    if (touch) {
      my_last = local + 1; my_touch = touch; my_dec = dec[r];
      my_host = (rec[r].x & TXR_HOST) != 0;
      my_info = make_uint4(rec[r].x & TXR_I0_MASK, rec[r].y, rec[r].z, rec[r].w);
    }
    bins[r] = dec_bin(dec[r], a.n_ep);
    const bool host = valid && (dec[r] & (USN_F_HOST | USN_F_FRAG1 | USN_F_LEARN));
    if (__ballot(host))
      if (host) hl[atomicAdd(&s_misc[1], 1u)] = (uint32_t)(base + local);
  }
  {
    uint32_t lm = my_last;
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) lm = max(lm, (uint32_t)__shfl_xor(lm, d, 64));
    if (lane == 0 && lm) atomicMax(&s_misc[0], lm);
  }
  tile_hist(bins, nt, a.nbits, L.hist);
  __syncthreads();
  STAMP(7);
  hist_out(L.hist, a.nbw, a.cnt + (size_t)rt * a.nbw);
  STAMP(10);
  usn_tile_hdr *H = a.tiles + rt;
  const uint32_t lastp = s_misc[0];
  if (lastp && my_last == lastp) {
    H->last_state = USN_TS_HAS | (my_touch == 1u && !my_host ? USN_TS_RETAINED : 0u) |
                    ((my_touch == 3u || my_host) ? USN_TS_UNKNOWN : 0u);
    H->last_dst = my_dec & USN_PARITY_MASK;
    H->last_info[0] = my_info.x; H->last_info[1] = my_info.y;
    H->last_info[2] = my_info.z; H->last_info[3] = my_info.w;
    H->last_idx = (uint32_t)(base + lastp - 1);
  }
  if (tid == 0) {
    const uint32_t nic = hist_get(L.hist, a.n_ep), fl = hist_get(L.hist, a.n_ep + 1),
                   dr = hist_get(L.hist, a.n_ep + 2);
    H->n_frames = (uint16_t)nt;
    H->_r0 = 0;
    H->n_host = (uint16_t)s_misc[1];
    H->bin_nic = (uint16_t)a.n_ep;
    H->class_count[0] = (uint16_t)dr;
    H->class_count[2] = (uint16_t)nic;
    H->class_count[3] = (uint16_t)fl;
    H->class_count[1] = (uint16_t)(nt - nic - fl - dr);
    if (!lastp) { H->last_state = 0; H->last_dst = 0; H->last_idx = 0xFFFFFFFFu; }
    if (s_misc[1]) atomicAdd(t.counters + USN_TXC_HOST + ring, s_misc[1]);   // after phase 2: tile 0 zeroed it
  }
  STAMP(11);
  STAMP_FLUSH_AT(tile);
}


static inline size_t table_lds_bytes(uint32_t table_units);

hipError_t launch_tx(const TxArgs &t, hipStream_t stream) {
  const ClassifyArgs &a = t.a[0];
  const uint32_t ntiles = t.tile_base[t.rings];
  if (ntiles == 0) return hipSuccess;
  const dim3 g(ntiles), b(NTHREADS);
  const size_t head = tx_lds_head(a.nbins);
  const size_t bridge = t.bridge_mask < TX_BRIDGE_LDS_SLOTS ? (size_t)(t.bridge_mask + 1) * 8 : 0;
  const size_t with_table = head + table_lds_bytes(a.table_units) + bridge;
  const bool in_lds = table_fits_lds(a.nbins, a.table_units) && with_table <= 64u * 1024u;
  if (in_lds) hipLaunchKernelGGL(tx_kernel<true>, g, b, with_table, stream, t);
  else hipLaunchKernelGGL(tx_kernel<false>, g, b, head + bridge, stream, t);
  return hipGetLastError();
}

/* --------------------------------------------------------------------------- */
/* The classify kernel's header stage (static LDS; GLDS only). */
#define STAGE_BYTES_GLDS ((size_t)NWAVES * GD * STAGE_ROUND_SLOTS * 16)

/* LDS copy of the rule table, rounded up to whole 64-slot glds chunks. */
static inline size_t table_lds_bytes(uint32_t table_units) {
  return (size_t)table_lds_units(table_units) * 16;
}

bool table_fits_lds(uint32_t nbins, uint32_t table_units) {
  return (size_t)table_units * 16 <= LDS_TABLE_MAX_BYTES &&
         lds_core_bytes(nbins) + STAGE_BYTES_GLDS + table_lds_bytes(table_units) <= 64u * 1024u;
}

/* where the classify kernel reads the image from (TM_*) */
/* displacement arrays up to this size go to LDS: up to 13 KiB the 512-thread
 * kernel keeps 4 workgroups per CU, up to 26 KiB 3, and at 3 the LDS copy
 * still beats global displacements at 4 (A/B, c5 16 KiB: 161.3 vs 174.2 us
 * per 8M frames, profiles/r02d) */
#ifndef USN_DISP_LDS_MAX
#define USN_DISP_LDS_MAX (26u * 1024u)
#endif
/* units of the displacements TM_DISPLDS copies to LDS: U's and X's when U is
 * built (one slot read per frame), else K1's and K2's */
static uint32_t disp_lds_units(const ClassifyArgs &a) {
  return (a.probe_mask & 4u) ? a.u_end_unit - a.u_disp_unit : a.table_units - a.disp_unit;
}
static int table_mode(const ClassifyArgs &a) {
  if (table_fits_lds(a.nbins, a.table_units)) return TM_LDS;
  const size_t disp = (size_t)disp_lds_units(a) * 16;
  return disp <= USN_DISP_LDS_MAX ? TM_DISPLDS : TM_GLOBAL;
}

/* dynamic LDS of the classify kernels; glds: the order row is in the stage */
size_t classify_lds_bytes(uint32_t nbins, uint32_t table_units, bool table_in_lds, bool glds) {
  return lds_core_bytes(nbins, !glds) + (table_in_lds ? table_lds_bytes(table_units) : 0);
}

/* glds needs 16-byte aligned sources: every window start of every batch.
 * Only dense slots use it: at a 2048-byte stride (c3, netmap-sized slots)
 * per-lane register loads were 8 % faster (A/B 40.9 vs 44.3 us per 1M frames),
 * at 64 bytes glds is (c2). */
#define USN_GLDS_MAX_STRIDE 128u
static bool glds_layout(const MultiArgs &m) {
  for (uint32_t k = 0; k < m.count; ++k) {
    const ClassifyArgs &b = m.b[k];
    if (b.offsets != nullptr || b.stride % 16 != 0 || b.stride > USN_GLDS_MAX_STRIDE ||
        (reinterpret_cast<uintptr_t>(b.frames) & 15))
      return false;
  }
  return true;
}

hipError_t launch_classify(const MultiArgs &m, hipStream_t stream) {
  const uint32_t tiles = m.tile_base[m.count];
  if (tiles == 0) return hipSuccess;
  const ClassifyArgs &a = m.b[0];   // table and bins are shared by every batch
  const int tm = table_mode(a);
  const bool glds = USN_GLDS_ENABLE && glds_layout(m);
  const size_t lds = lds_core_bytes(a.nbins, !glds) +
                     (tm == TM_LDS ? table_lds_bytes(a.table_units)
                      : tm == TM_DISPLDS ? table_lds_bytes(disp_lds_units(a)) : 0);
  const dim3 b(NTHREADS);
#define USN_LAUNCH(T_, G_) \
  hipLaunchKernelGGL((classify_rx_kernel<T_, G_>), dim3(tiles), b, lds, stream, m)
  if (tm == TM_LDS) { if (glds) USN_LAUNCH(TM_LDS, true); else USN_LAUNCH(TM_LDS, false); }
  else if (tm == TM_DISPLDS) { if (glds) USN_LAUNCH(TM_DISPLDS, true); else USN_LAUNCH(TM_DISPLDS, false); }
  else { if (glds) USN_LAUNCH(TM_GLOBAL, true); else USN_LAUNCH(TM_GLOBAL, false); }
#undef USN_LAUNCH
  return hipGetLastError();
}

/* in-place image update (usn_host.cpp upload_table): n patched 16-byte
 * units, buf = {n values (uint4)} {n unit indices (u32)} */
__global__ __launch_bounds__(256) void patch_kernel(uint4 *table, const uint4 *buf, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) table[reinterpret_cast<const uint32_t *>(buf + n)[i]] = buf[i];
}
hipError_t launch_patch(uint4 *table, const void *buf, uint32_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(patch_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, table,
                     static_cast<const uint4 *>(buf), n);
  return hipGetLastError();
}

hipError_t launch_recount(const ClassifyArgs &a, uint32_t t0, uint32_t t1, hipStream_t stream) {
  if (t1 <= t0) return hipSuccess;
  const size_t lds = lds_core_bytes(a.nbins);
  hipLaunchKernelGGL(recount_kernel, dim3(t1 - t0), dim3(NTHREADS), lds, stream, a, t0);
  return hipGetLastError();
}

#if USN_NTHREADS == 512
/* ===========================================================================
 * Per-endpoint lists: the device-wide stable scatter (usn_kernels.h).
 * The classify / tx kernel leaves each tile's decisions and its count row
 * cnt[tile][bin] (u16).  Two launches turn them into `index` (the batch's
 * frame indices grouped by bin, frame order inside a bin) and bin_off:
 *   scan     (range of 64 chunks, block of 64 bins): agg[chunk][bin] = the
 *            bin's frames in the chunks before (exclusive scan over the
 *            batch's chunks), tot = the bin's frames
 *   scatter  (chunk): the chunk's frames sorted by bin in an LDS stage, then
 *            written out in stage order: a bin's frames of the chunk leave as
 *            one contiguous run of index
 * Algorithmic bytes per frame: 4 (index).  The reference writes each frame
 * straight into its target's ring (endpoint.rs:61-74) and copies FLOOD frames
 * to every other endpoint (:340-363): an endpoint's frames are its list merged
 * in frame order with the FLOOD list.
 * =========================================================================== */
__device__ __forceinline__ uint32_t base_of(const uint32_t *base, uint32_t count, uint32_t w) {
  uint32_t bi = 0;
#pragma unroll
  for (uint32_t k = 1; k < USN_MAX_MULTI; ++k) bi += (k < count && w >= base[k]) ? 1u : 0u;
  return bi;
}

#define SCAN_THREADS 256
static_assert(USN_SCAN_BLK == 64, "scan: 16 lanes x 4 bins");
#define SCAN_SPIN_TICKS (200u * 100000u)   /* 200 ms of the 100 MHz real-time clock */

typedef __attribute__((address_space(1))) unsigned long long gu64s;
/* a range total: {epoch, value} in one 8-byte agent-scope (sc1) store */
__device__ __forceinline__ void scan_put(unsigned long long *g, uint32_t epoch, uint32_t v) {
  __hip_atomic_store((gu64s *)g, ((unsigned long long)epoch << 32) | v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

/* (range r of 16 CPT chunks of a batch, bin block bb), range-major so that a
 * workgroup waits only on workgroups dispatched before it:
 *  1. thread (rg, l) sums the count rows of its CPT chunks of the range
 *     for bins 4l..4l+3 of the block (every load in flight together);
 *  2. the block's 16 row groups are scanned in LDS: each chunk's prefix
 *     inside the range, and the range's totals, published as epoch-tagged
 *     granules gran[r][bin];
 *  3. carry = the totals of ranges 0..r-1 (their granules, polled; each
 *     range publishes before it waits, so the wait ends);
 *  4. agg[chunk][bin] = carry + prefix (16-byte stores); the last range
 *     writes tot.  (Bin bases here too, handed on between bin blocks, cost
 *     the scan's last ranges one more round trip: 15.4 against 13.9 us for
 *     c5, more than the scatter's block scan they saved, profiles/r03.) */
template <int CPT>   // chunks per thread: a range is 16 * CPT chunks
__global__ __launch_bounds__(SCAN_THREADS) void scan_kernel(ScatterArgs s) {
  __shared__ uint32_t s_t[16][USN_SCAN_BLK];
  __shared__ uint32_t s_c[4][USN_SCAN_BLK];
  __shared__ uint32_t s_tot[USN_SCAN_BLK];
  const uint32_t tid = threadIdx.x, l = tid & 15, rg = tid >> 4;
  const uint32_t rgl = blockIdx.x / s.nbb, bb = blockIdx.x - rgl * s.nbb;
  const uint32_t bi = base_of(s.range_base, s.count, rgl);
  const ScatterBatch &B = s.b[bi];
  const uint32_t r = rgl - s.range_base[bi];
  const uint32_t b0 = bb * USN_SCAN_BLK + 4 * l;             // this thread's 4 bins
  const bool binok = b0 < s.nbw;                            // nbw is a multiple of 8
  const uint32_t c0 = r * 16 * CPT + rg * CPT;              // this thread's CPT chunks
  // 1.
  uint2 v[CPT][8];
#pragma unroll
  for (uint32_t j = 0; j < CPT; ++j)
#pragma unroll
    for (uint32_t w = 0; w < 8; ++w) {
      const uint32_t t = (c0 + j) * s.tc + w;
      const bool ok = binok && w < s.tc && t < B.ntiles;
      v[j][w] = ok ? *reinterpret_cast<const uint2 *>(B.cnt + (size_t)t * s.nbw + b0) : make_uint2(0, 0);
    }
  uint32_t ex[CPT][4], tot[4] = {0, 0, 0, 0};
#pragma unroll
  for (uint32_t j = 0; j < CPT; ++j) {
    uint32_t a[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t w = 0; w < 8; ++w) {
      a[0] += v[j][w].x & 0xFFFFu; a[1] += v[j][w].x >> 16;
      a[2] += v[j][w].y & 0xFFFFu; a[3] += v[j][w].y >> 16;
    }
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) { ex[j][i] = tot[i]; tot[i] += a[i]; }
  }
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) s_t[rg][4 * l + i] = tot[i];
  __syncthreads();
  // 2.
  unsigned long long *gran = B.gran + (size_t)r * s.nbw;
  if (tid < USN_SCAN_BLK) {
    uint32_t run = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      const uint32_t x = s_t[k][tid];
      s_t[k][tid] = run;
      run += x;
    }
    s_tot[tid] = run;
    if (bb * USN_SCAN_BLK + tid < s.nbw) scan_put(gran + bb * USN_SCAN_BLK + tid, s.epoch, run);
  }
  // 3. thread (part, k) sums ranges part, part + 4, ... < r of bin k: the
  // loads of 16 ranges issued together (what is still pending is fixed
  // before they issue, so none waits for another), then checked
  {
    const uint32_t k = tid & 63, part = tid >> 6, bin = bb * USN_SCAN_BLK + k;
    uint32_t sum = 0;
    if (bin < s.nbw) {
      const unsigned long long *col = B.gran + bin;
      uint64_t t0 = 0;
      for (uint32_t q0 = part; q0 < r; q0 += 64) {
        uint32_t pend = 0;
#pragma unroll
        for (uint32_t u = 0; u < 16; ++u) pend |= (q0 + 4 * u < r ? 1u : 0u) << u;
        for (uint32_t it = 0;; ++it) {
          unsigned long long x[16];
#pragma unroll
          for (uint32_t u = 0; u < 16; ++u)
            x[u] = ((pend >> u) & 1u) ? __hip_atomic_load((const gu64s *)(col + (size_t)(q0 + 4 * u) * s.nbw),
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : 0ull;
#pragma unroll
          for (uint32_t u = 0; u < 16; ++u)
            if (((pend >> u) & 1u) && (uint32_t)(x[u] >> 32) == s.epoch) {
              sum += (uint32_t)x[u];
              pend &= ~(1u << u);
            }
          if (!pend) break;
          const uint64_t now = __builtin_amdgcn_s_memrealtime();
          if (it == 0) t0 = now;
          else if (now - t0 > SCAN_SPIN_TICKS) { atomicOr(B.diag, USN_DIAG_TIMEOUT); break; }   // never seen; lists wrong
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    s_c[part][k] = sum;
  }
  __syncthreads();
  // 4.
  uint32_t carry[4];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    const uint32_t k = 4 * l + i;
    carry[i] = s_c[0][k] + s_c[1][k] + s_c[2][k] + s_c[3][k] + s_t[rg][k];
  }
  if (binok) {
#pragma unroll
    for (uint32_t j = 0; j < CPT; ++j)
      if (c0 + j < B.nchunks)
        *reinterpret_cast<uint4 *>(B.agg + (size_t)(c0 + j) * s.nbw + b0) =
            make_uint4(carry[0] + ex[j][0], carry[1] + ex[j][1], carry[2] + ex[j][2], carry[3] + ex[j][3]);
  }
  if (r + 1 == B.nranges && tid < USN_SCAN_BLK && bb * USN_SCAN_BLK + tid < s.nbw)
    B.tot[bb * USN_SCAN_BLK + tid] = s_c[0][tid] + s_c[1][tid] + s_c[2][tid] + s_c[3][tid] + s_tot[tid];
}

/* (chunk of TC <= 8 tiles): one workgroup of 512 threads; wave w owns tile w
 * of the chunk.
 *  1. each wave loads its tile's decisions at once (16 per lane: segment k
 *     of 64 frames is lane + 64k), every wave in flight together;
 *  2. per bin: off[b] = bin base (block scan of the totals) + the chunks
 *     before (agg) - b's start in the chunk (block scan of the chunk's
 *     counts), and each
 *     wave's cursor cur[w][b] = b's start in the chunk + b's frames in the
 *     chunk's tiles before w (the classify kernel's count rows) -- one
 *     barrier;
 *  3. each wave ranks its tile's frames with one LDS atomic each on its own
 *     cursors (below): the chunk sorted by (bin, frame) in LDS -- one
 *     barrier;
 *  4. the stage is written out in order: index[off[bin] + q], contiguous
 *     runs per bin (one L2 request per run instead of one per frame; c5,
 *     1005 bins: about 8 frames per run), and checked to be stably sorted.
 * Blocks are dealt round-robin over the 8 XCDs; USN_SCATTER_XCD remaps them
 * so that an XCD takes a contiguous run of chunks (cdna_hip_programming.md T1
 * swizzle, bijective). */
#ifndef USN_SCATTER_XCD
#define USN_SCATTER_XCD 1
#endif
/* chunks that took step 5 (usn_debug_scatter_fallbacks) */
__device__ uint32_t usn_scatter_fallbacks = 0;
#ifndef USN_SC_CHECKS   /* A/B only: 0 = no empty-slot sentinel and no inconsistency report
                           (the bounds clamps stay) */
#define USN_SC_CHECKS 1
#endif
#ifndef USN_SCATTER_WPE   /* waves per SIMD the scatter is compiled for: 8 = 64 VGPRs, no spills
                             (since the fallback's lane is opaque, step 5): 4 workgroups per CU
                             where the LDS allows (c2's few bins: scan + scatter 27.5-27.6 vs
                             28.4 us at 6), c5 (3 per CU by LDS) and c4 equal (profiles/r05/r05ax);
                             round 4: 6 against 4, c5 57.5 vs 61.7 us (profiles/r04/r04b) */
#define USN_SCATTER_WPE 8
#endif
template <int TC, bool SELF>   // SELF: USN_SCF_SELFSCAN launches (one workgroup per CU at most:
                               // registers for the row sums instead of occupancy)
__global__ __launch_bounds__(NTHREADS) __attribute__((amdgpu_waves_per_eu(SELF ? 2 : USN_SCATTER_WPE)))
void scatter_kernel(ScatterArgs s) {
  static_assert(TC >= 1 && TC <= NTHREADS / 64, "a wave per tile");
  constexpr uint32_t SEGS = TILE / 64;                               // 16 segments per tile
  extern __shared__ __align__(16) uint8_t smem[];
  __shared__ uint32_t s_scan[16];
  uint32_t *stage = reinterpret_cast<uint32_t *>(smem);              // [TC * TILE]: bin << 16 | frame
  uint32_t *off = stage + TC * TILE;                                 // [nbw]
  uint16_t *cur = reinterpret_cast<uint16_t *>(off + s.nbw);         // [TC][nbw]: < TC * TILE
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t nwg = s.chunk_base[s.count];
  uint32_t g = blockIdx.x;
  if (USN_SCATTER_XCD) {
    const uint32_t q = nwg / 8, r = nwg % 8, x = g % 8;
    g = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + g / 8;
  }
  const uint32_t bi = base_of(s.chunk_base, s.count, g);
  const ScatterBatch &B = s.b[bi];
  const uint32_t c = g - s.chunk_base[bi];
  const uint32_t t0 = c * TC, ntc = min((uint32_t)TC, B.ntiles - t0);
  const uint64_t first = (uint64_t)t0 * TILE;                        // the chunk's first frame
  STAMP_DECL
  STAMP(0);
  const uint32_t *ex = B.agg + (size_t)c * s.nbw;             // frames of b in the chunks before
  // up to 1024 bins (a pair per thread): totals, chunk offsets and the
  // chunk's count rows are loaded first, then the decisions: waiting for the
  // former leaves the decisions in flight
  const bool pair = s.nbw <= 2 * NTHREADS;
  const bool mine = pair && 2 * tid < s.nbw;
  const bool noscan = (s.flags & USN_SCF_NOSCAN) != 0;   // one chunk per batch: its counts are the batch's
  const bool selfscan = SELF && pair;   // the scan's sums done here (USN_SCF_SELFSCAN)
  if (selfscan) {   // the sums zeroed before any load is in flight (the barrier waits for none)
    uint32_t *sa = reinterpret_cast<uint32_t *>(cur + (size_t)TC * s.nbw);
    for (uint32_t i = tid; i < 2 * s.nbw; i += NTHREADS) sa[i] = 0;
    __syncthreads();
  }
  uint2 vt = make_uint2(0, 0), ve = make_uint2(0, 0);
  uint32_t rc[TC];
  if (mine && !noscan && !selfscan) {
    vt = *reinterpret_cast<const uint2 *>(B.tot + 2 * tid);
    ve = *reinterpret_cast<const uint2 *>(ex + 2 * tid);
  }
#pragma unroll
  for (uint32_t w = 0; w < TC; ++w) {   // count rows of the chunk's tiles (bins 2 tid, 2 tid + 1)
    const uint32_t t = t0 + min(w, ntc - 1);
    rc[w] = mine ? reinterpret_cast<const uint32_t *>(B.cnt + (size_t)t * s.nbw)[tid] : 0u;
    if (w >= ntc) rc[w] = 0;
  }
  // 1. this wave's tile (waves past the chunk's end re-read its last tile, unused)
  const uint32_t wt = min(wave, ntc - 1);
  const uint64_t tbase = first + (uint64_t)wt * TILE;
  const uint32_t tn = (uint32_t)min((uint64_t)TILE, (uint64_t)B.n - tbase);
  uint32_t d[SEGS];
#pragma unroll
  for (uint32_t k = 0; k < SEGS; ++k) d[k] = B.decisions[tbase + min(k * 64 + lane, tn - 1)];
  // 1b. (small launches) the scan's two sums for this chunk from the batch's
  // count rows: thread (g, q) adds bins 8q..8q+7 (one 16-byte load) of tiles
  // g, g + G, ... into the totals and, for the tiles before the chunk, into
  // its offsets; up to 8 loads per thread in flight together
  if (selfscan) {
    uint32_t *sa = reinterpret_cast<uint32_t *>(cur + (size_t)TC * s.nbw);   // [nbw] totals (zeroed above)
    uint32_t *sb = sa + s.nbw;                                                // [nbw] before the chunk
    const uint32_t nq = s.nbw / 8, G = NTHREADS / nq, qq = tid % nq, g = tid / nq;
    if (g < G) {
      const uint4 *rows = reinterpret_cast<const uint4 *>(B.cnt) + qq;   // row t: rows[t * nq]
      uint32_t at[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ab[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t t = g; t < B.ntiles; t += 8 * G) {
        uint4 v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
          const uint32_t tt = t + k * G;
          v[k] = tt < B.ntiles ? rows[(size_t)tt * nq] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
          const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
          const bool before = t + k * G < t0;
#pragma unroll
          for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t lo = w[j] & 0xFFFFu, hi = w[j] >> 16;
            at[2 * j] += lo; at[2 * j + 1] += hi;
            if (before) { ab[2 * j] += lo; ab[2 * j + 1] += hi; }
          }
        }
      }
#pragma unroll
      for (uint32_t j = 0; j < 8; ++j) {
        if (at[j]) atomicAdd(&sa[8 * qq + j], at[j]);
        if (ab[j]) atomicAdd(&sb[8 * qq + j], ab[j]);
      }
    }
    __syncthreads();
    if (mine) {
      vt = make_uint2(sa[2 * tid], sa[2 * tid + 1]);
      ve = make_uint2(sb[2 * tid], sb[2 * tid + 1]);
    }
  }
  // 2. bases, the chunk's bin starts, the waves' cursors
  if (pair) {
    uint32_t c0 = 0, c1 = 0;
#pragma unroll
    for (uint32_t w = 0; w < TC; ++w) { c0 += rc[w] & 0xFFFFu; c1 += rc[w] >> 16; }
    if (noscan) vt = make_uint2(c0, c1);
    uint32_t total;
    const uint32_t pt = block_excl_scan(vt.x + vt.y, s_scan, &total);
    const uint32_t pc = block_excl_scan(c0 + c1, s_scan, &total);
    if (mine) {
      const uint32_t b = 2 * tid;
      *reinterpret_cast<uint2 *>(off + b) = make_uint2(pt + ve.x - pc, pt + vt.x + ve.y - (pc + c0));
      uint32_t s0 = pc, s1 = pc + c0;
#pragma unroll
      for (uint32_t w = 0; w < TC; ++w) {
        reinterpret_cast<uint32_t *>(cur + (size_t)w * s.nbw)[tid] = (s0 & 0xFFFFu) | (s1 << 16);
        s0 += rc[w] & 0xFFFFu;
        s1 += rc[w] >> 16;
      }
      if (c == 0) {
        if (b <= s.nbins) B.bin_off[b] = pt;                   // pad bins past nbins are empty
        if (b + 1 <= s.nbins) B.bin_off[b + 1] = pt + vt.x;
        if (s.txs_out) {   // tx: the ring's class totals for usn_finalize (host memory)
          uint32_t *to = s.txs_out + USN_TXS_WORDS * bi;
          if (b >= s.n_ep && b < s.n_ep + 3) to[6 + b - s.n_ep] = pt;
          if (b + 1 >= s.n_ep && b + 1 < s.n_ep + 3) to[7 + b - s.n_ep] = pt + vt.x;
        }
        if (B.rx_state) {             // rx: the same into the batch's state
          if (b >= s.n_ep && b < s.n_ep + 3) B.rx_state[4 + b - s.n_ep] = pt;
          if (b + 1 >= s.n_ep && b + 1 < s.n_ep + 3) B.rx_state[5 + b - s.n_ep] = pt + vt.x;
        }
      }
    }
  } else {   // more bins: per-thread contiguous runs of bins, the same sums
    const uint32_t per = (s.nbw + NTHREADS - 1) / NTHREADS;
    const uint32_t b0 = tid * per;
    uint32_t st = 0, sc = 0;
    for (uint32_t k = 0; k < per; ++k) {
      const uint32_t b = b0 + k;
      if (b >= s.nbw) break;
      uint32_t cb = 0;
      for (uint32_t w = 0; w < ntc; ++w) cb += B.cnt[(size_t)(t0 + w) * s.nbw + b];
      sc += cb;
      st += noscan ? cb : B.tot[b];
    }
    uint32_t total;
    uint32_t pt = block_excl_scan(st, s_scan, &total);
    uint32_t pc = block_excl_scan(sc, s_scan, &total);
    for (uint32_t k = 0; k < per; ++k) {
      const uint32_t b = b0 + k;
      if (b >= s.nbw) break;
      off[b] = pt + (noscan ? 0u : ex[b]) - pc;
      if (c == 0 && b <= s.nbins) B.bin_off[b] = pt;
      if (c == 0 && s.txs_out && b >= s.n_ep && b < s.n_ep + 3) s.txs_out[USN_TXS_WORDS * bi + 6 + b - s.n_ep] = pt;
      if (c == 0 && B.rx_state && b >= s.n_ep && b < s.n_ep + 3) B.rx_state[4 + b - s.n_ep] = pt;
      if (noscan) {
        for (uint32_t w = 0; w < ntc; ++w) pt += B.cnt[(size_t)(t0 + w) * s.nbw + b];
      } else {
        pt += B.tot[b];
      }
      for (uint32_t w = 0; w < TC; ++w) {
        cur[(size_t)w * s.nbw + b] = (uint16_t)pc;
        if (w < ntc) pc += B.cnt[(size_t)(t0 + w) * s.nbw + b];
      }
    }
  }
  // every stage slot starts empty: a slot still empty at the write-out means
  // the count rows disagree with the decisions (reported, never hidden)
  if (USN_SC_CHECKS) {
    uint4 *st4 = reinterpret_cast<uint4 *>(stage);
#pragma unroll
    for (uint32_t q4 = tid; q4 < TC * TILE / 4; q4 += NTHREADS) st4[q4] = make_uint4(~0u, ~0u, ~0u, ~0u);
  }
  if (c == 0 && tid == 0) B.bin_off[s.nbins] = B.n;
  if (c == 0 && B.rx_state && tid == 0) {   // rx: what usn_finalize reads first (host memory)
    B.rx_state[1] = B.summary->flags;
    B.rx_state[3] = B.summary->host_epoch == s.epoch ? 1u : 0u;
    B.rx_state[7] = *B.diag;
    B.rx_state[0] = s.epoch;
  }
  if (c == 0 && s.txs_out && tid < 6) {   // tx, per ring: summary flags, counters, n, diag
    auto ctr = [&](uint32_t k) {
      return __hip_atomic_load(s.txs_counters + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    uint32_t v;
    if (tid == 0) v = B.summary->flags;
    else if (tid == 1) {                                          // the ring's learned items
      v = bi ? ctr(USN_TXC_LEARNED + bi) : ctr(0);
      if (bi == 0)
        for (uint32_t k = 1; k < s.count; ++k) v -= ctr(USN_TXC_LEARNED + k);
    } else if (tid == 5) v = ctr(USN_TXC_HOST + bi);              // ... frames for the host stage
    else v = ctr(tid - 1);                                        // flags, sets, timeout epoch
    uint32_t *to = s.txs_out + USN_TXS_WORDS * bi;
    to[tid] = v;
    if (tid == 0) { to[9] = B.n; to[10] = *B.diag; }
  }
  __syncthreads();
  STAMP(1);
  // 3. each wave ranks its tile into the stage: one LDS atomic add per frame
  // on the wave's own cursor of its bin (u16 pairs) returns the frame's stage
  // slot.  The 16 segments' atomics are issued back to back (a wave's LDS
  // operations execute in order, so segment k's frames precede segment
  // k+1's); within one instruction the LDS serves the lanes that hit one word
  // in lane order (tools/lds_order_check: 0 of 2.5e11 same-word lane pairs
  // out of order).  That is not an ISA guarantee, so step 4 verifies the
  // stage and a chunk that is not stably sorted is ranked again the
  // ballot way (5).
  const uint32_t nf = (uint32_t)min((uint64_t)TC * TILE, (uint64_t)B.n - first);
  // bad: a decision naming a bin past the batch's bins, a rank past the
  // chunk, an empty stage slot or a list position past n -- the count rows
  // and the decisions disagree.  Every access stays in bounds regardless, and
  // the batch's diag word gets USN_DIAG_LISTS (usn_finalize: USN_ELIST).
  bool bad = false;
  if (wave < ntc) {
    uint32_t *cw = reinterpret_cast<uint32_t *>(cur + (size_t)wave * s.nbw);
    uint32_t at[SEGS];   // (the bins are recomputed below: 16 VGPRs fewer while the atomics fly)
#pragma unroll
    for (uint32_t k = 0; k < SEGS; ++k) {
      const uint32_t raw = dec_bin(d[k], s.n_ep);
      const uint32_t b = min(raw, s.nbins - 1u);
      const uint32_t sh = 16u * (b & 1u);
      const bool v = k * 64 + lane < tn;
      at[k] = v ? atomicAdd(&cw[b >> 1], 1u << sh) >> sh : 0u;
      bad |= v && raw >= s.nbins;
    }
#pragma unroll
    for (uint32_t k = 0; k < SEGS; ++k)
      if (k * 64 + lane < tn) {
        const uint32_t b = min(dec_bin(d[k], s.n_ep), s.nbins - 1u), q = at[k] & 0xFFFFu;
        bad |= q >= nf;
        stage[min(q, TC * TILE - 1u)] = (b << 16) | (wave * TILE + k * 64 + lane);
      }
  }
  __syncthreads();
  STAMP(10);
  // 4. the stage out, in order (every address bounds-checked: counts that
  // disagree with the decisions, or an A/B build that skips a phase, cannot
  // write past index), checking that each bin's run is in frame order
  bool unsorted = false;
  uint32_t q0 = 0;
  {
    // groups of 8 entries per thread: every stage read of the group, then
    // every offset read, then the stores (the LDS round trips overlap)
    constexpr uint32_t G = 8;
    for (; q0 + G * NTHREADS <= nf; q0 += G * NTHREADS) {
      uint32_t e[G], p[G], o[G];
#pragma unroll
      for (uint32_t j = 0; j < G; ++j) {
        const uint32_t q = q0 + j * NTHREADS + tid;
        e[j] = stage[q];
        p[j] = q ? stage[q - 1] : 0u;
      }
#pragma unroll
      for (uint32_t j = 0; j < G; ++j) o[j] = off[min(e[j] >> 16, s.nbw - 1u)];
#pragma unroll
      for (uint32_t j = 0; j < G; ++j) {
        const uint32_t q = q0 + j * NTHREADS + tid;
        const uint32_t pos = o[j] + q;
        if (pos < B.n) B.index[pos] = (uint32_t)first + (e[j] & 0xFFFFu);
        bad |= pos >= B.n || e[j] == ~0u;
        unsorted |= q && (p[j] >> 16) == (e[j] >> 16) && (p[j] & 0xFFFFu) >= (e[j] & 0xFFFFu);
      }
    }
  }
  for (uint32_t q = q0 + tid; q < nf; q += NTHREADS) {
    const uint32_t e = stage[q];
    const uint32_t b = min(e >> 16, s.nbw - 1u);
    const uint32_t pos = off[b] + q;
    if (pos < B.n) B.index[pos] = (uint32_t)first + (e & 0xFFFFu);
    bad |= pos >= B.n || e == ~0u;
    const uint32_t p = q ? stage[q - 1] : 0u;
    unsorted |= q && (p >> 16) == (e >> 16) && (p & 0xFFFFu) >= (e & 0xFFFFu);
  }
  STAMP(11);
  if (USN_SC_CHECKS && __ballot(bad) && lane == 0) {   // rare: one report per wave
    atomicOr(B.diag, USN_DIAG_LISTS);
    if (s.txs_out) s.txs_out[11] = USN_DIAG_LISTS;   // tx: beside chunk 0's copy of the scan's word
    if (B.rx_state) B.rx_state[2] = USN_DIAG_LISTS;
  }
  if (__syncthreads_or(unsorted || (s.flags & USN_SCF_SLOW_RANK))) {
    // 5. (not taken on gfx950 so far) the wave's cursors back to their
    // seeds (final value - the tile's count), the ranks from bit-sliced
    // ballots segment by segment, the stage out again
    if (wave < ntc) {
      uint16_t *cw = cur + (size_t)wave * s.nbw;
      const uint16_t *row = B.cnt + (size_t)(t0 + wave) * s.nbw;
      for (uint32_t bb = lane; bb < s.nbw; bb += 64) cw[bb] = (uint16_t)(cw[bb] - row[bb]);
      // the lane made opaque to the compiler: otherwise it keeps step 1's
      // per-segment indices and addresses live for this rare path (spilled:
      // 6-7 scratch stores per lane and chunk, ~25 MB per c5 call)
      uint32_t lf = lane;
      asm volatile("" : "+v"(lf));
#pragma unroll
      for (uint32_t k = 0; k < SEGS; ++k) {
        const uint32_t local = k * 64 + lf;
        const bool v = local < tn;
        // the decision again from memory: keeping d[] live to here costs the
        // common path VGPRs
        const uint32_t dk = B.decisions[tbase + min(local, tn - 1)];
        const uint32_t b = min(dec_bin(dk, s.n_ep), s.nbins - 1u);
        const uint64_t same = match_bin(b, __ballot(v), s.nbits);
        const uint32_t rank = (uint32_t)__popcll(same & lanemask_lt(lane));
        const uint32_t at = cw[b];
        if (v) {
          stage[min(at + rank, TC * TILE - 1u)] = (b << 16) | (wave * TILE + local);
          if (rank == 0) cw[b] = (uint16_t)(at + __popcll(same));
        }
      }
    }
    __syncthreads();
    for (uint32_t q = tid; q < nf; q += NTHREADS) {
      const uint32_t e = stage[q];
      const uint32_t b = min(e >> 16, s.nbw - 1u);
      const uint32_t pos = off[b] + q;
      if (pos < B.n) B.index[pos] = (uint32_t)first + (e & 0xFFFFu);
    }
    if (tid == 0) atomicAdd(&usn_scatter_fallbacks, 1u);
  }
  STAMP_FLUSH_SCATTER(blockIdx.x);
}
static_assert(NTHREADS == 512, "scatter: 8 waves, a tile each");
static_assert(8 * TILE <= 0x10000, "scatter: a stage entry holds a 16-bit frame offset");

uint32_t scatter_fallbacks() {
  uint32_t v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(usn_scatter_fallbacks), sizeof v, 0, hipMemcpyDeviceToHost) !=
      hipSuccess)
    return 0xFFFFFFFFu;
  return v;
}

hipError_t launch_scatter(const ScatterArgs &s, hipStream_t stream, hipEvent_t done) {
  const uint32_t chunks = s.chunk_base[s.count];
  if (chunks == 0) return hipSuccess;
  const dim3 sg(s.range_base[s.count] * s.nbb), sb(SCAN_THREADS);
  if (!(s.flags & (USN_SCF_NOSCAN | USN_SCF_SELFSCAN))) switch (s.cpt) {
    case 4: hipLaunchKernelGGL(scan_kernel<4>, sg, sb, 0, stream, s); break;
    case 2: hipLaunchKernelGGL(scan_kernel<2>, sg, sb, 0, stream, s); break;
    case 1: hipLaunchKernelGGL(scan_kernel<1>, sg, sb, 0, stream, s); break;
    default: return hipErrorInvalidValue;
  }
  const size_t lds = scatter_lds(s.nbins, s.tc, (s.flags & USN_SCF_SELFSCAN) != 0);
  const dim3 g(chunks), b(NTHREADS);
  const bool self = (s.flags & USN_SCF_SELFSCAN) != 0;
  // `done`: bound to the scatter's own dispatch (no marker packet between
  // this launch and the next, as hipEventRecord would add)
#define USN_SC_LAUNCH(TC_)                                                                       \
  do {                                                                                           \
    if (done && self)                                                                            \
      hipExtLaunchKernelGGL((scatter_kernel<TC_, true>), g, b, lds, stream, nullptr, done, 0, s); \
    else if (done)                                                                               \
      hipExtLaunchKernelGGL((scatter_kernel<TC_, false>), g, b, lds, stream, nullptr, done, 0, s); \
    else if (self) hipLaunchKernelGGL((scatter_kernel<TC_, true>), g, b, lds, stream, s);        \
    else hipLaunchKernelGGL((scatter_kernel<TC_, false>), g, b, lds, stream, s);                 \
  } while (0)
  switch (s.tc) {
    case 8: USN_SC_LAUNCH(8); break;
    case 4: USN_SC_LAUNCH(4); break;
    case 2: USN_SC_LAUNCH(2); break;
    case 1: USN_SC_LAUNCH(1); break;
    default: return hipErrorInvalidValue;
  }
#undef USN_SC_LAUNCH
  return hipGetLastError();
}
#endif  // USN_NTHREADS == 512

}  // namespace USN_NS

#if USN_STAMPS
#if USN_NTHREADS == 512
#define USN_STAMPS_FN usn_debug_stamps512
#else
#define USN_STAMPS_FN usn_debug_stamps
#endif
extern "C" int USN_STAMPS_FN(void *host, size_t bytes) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(USN_NS::usn_stamp_buf), bytes, 0,
                                  hipMemcpyDeviceToHost);
}
#endif
