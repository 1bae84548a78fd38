/*
 * usn_kernels.h -- launch interface between the C++ host (usn_host.cpp) and
 * the HIP kernels (usn_device.hip).  Internal; not part of the C ABI.
 */
#ifndef USN_KERNELS_H
#define USN_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/usn_classify.h"
#include "usn_internal.h"

namespace usn {

enum CarryMode : uint32_t { CARRY_NONE = 0, CARRY_EXPLICIT = 1, CARRY_CHAIN = 2 };

struct ClassifyArgs {
  /* batch */
  const uint8_t *frames;
  uint64_t stride;
  const uint64_t *offsets;
  const uint16_t *lens;
  uint64_t n;
  uint32_t ntiles;
  uint32_t window;          /* readable bytes at every frame start (usn_batch.window) */
  uint32_t epoch;           /* the launch tag (ScatterArgs::epoch): a tile that lists frames for
                               the host stage stores it in summary->host_epoch */
  /* outputs */
  uint32_t *decisions;
  uint16_t *cnt;            /* [ntiles][nbw] frames per bin of each tile (the scatter's input) */
  uint32_t nbw;             /* row length of cnt: nbins rounded up to 8 */
  usn_tile_hdr *tiles;
  usn_summary *summary;
  uint32_t *host_list;      /* per tile USN_TILE slots */
  /* rule image (usn_internal.h): K1 / K2 perfect-hash tables in one buffer */
  const uint4 *table;
  uint32_t table_units;     /* 16-byte units of the K1/K2 image (U and X follow it) */
  uint32_t disp_unit;       /* first unit of the K1/K2 displacement arrays (up to table_units) */
  usn_ph_table ph[4];       /* K1 (key1 shapes), K2 (key2 shapes), U (projections), X (U overflow) */
  uint32_t u_disp_unit;     /* first unit of U's then X's displacements (probe_mask bit 2) */
  uint32_t u_end_unit;      /* end of the image */
  /* inner L2 bridge (tx): MACs in the low 48 bits */
  const uint64_t *bridge;
  uint32_t n_bridge;
  /* source endpoint */
  uint32_t src;
  uint32_t src_is_nic;
  uint32_t for_nic;
  uint32_t nbins;           /* endpoints + 3 */
  uint32_t nbits;           /* bits to tell bins apart (ceil log2 nbins) */
  uint32_t n_ep;            /* endpoints (bin of NIC) */
  uint32_t probe_mask;      /* bit0: K1 holds rules; bit1: K2 holds rules; bit2: U and X built */
  uint32_t next_dhcp_set;   /* the source's next_dhcp_endpoint is Some: DHCP answers need the host */
  /* carried 1-entry decision cache */
  uint32_t carry_mode;
  uint32_t cin_state, cin_dst;
  uint32_t cin_info[4];
  const usn_tile_hdr *prev_tiles;
  uint32_t prev_ntiles;
  const usn_summary *prev_summary;
};

/* Several batches (distinct sources) classified by one launch: workgroup w
 * takes tile w - tile_base[i] of batch i, tile_base[i] <= w < tile_base[i+1]. */
#define USN_MAX_MULTI 8
struct MultiArgs {
  ClassifyArgs b[USN_MAX_MULTI];
  uint32_t tile_base[USN_MAX_MULTI + 1];
  uint32_t count;
};
static_assert(sizeof(MultiArgs) <= 4096, "kernel argument block");

/* ---- tx direction (a non-NIC source sends): four launches ---------------- */
/* per-frame record, two planes of n uint4 written by tx_scan:
 *   rec[i]     r0 = {i0 | TXR_* flags, src, dst, ports}
 *   rec[n + i] r1 = {smac[0..3], smac[4..5] | dmac[0..1] << 16, dmac[2..5], 0}
 * r0 is all a frame's decision needs unless this batch learns a MAC (the
 * dmac test) or the frame is the first to learn one (its smac); in steady
 * state tx_hits and tx_decide read 16 B per frame, not 32.                   */
#define TXR_TOUCH_SHIFT 20u    /* 2 bits: 0 none, 1 retains, 2 leaves None, 3 unknown */
#define TXR_LEARNMAC (1u << 22)  /* unicast smac not in the bridge snapshot */
#define TXR_LEARNRULE (1u << 23) /* answer key not listened, not in the table snapshot */
#define TXR_HOST (1u << 24)      /* ordered host stage decides this frame */
#define TXR_SMAC_IN (1u << 25)
#define TXR_DMAC_IN (1u << 26)
#define TXR_HIT (1u << 27)       /* 1-entry cache hit (set by tx_hits) */
#define TXR_DHCPANS (1u << 28)
#define TXR_FRAG1 (1u << 29)     /* first fragment: extract_pkt_info remembers it (host map) */
#define TXR_WINDOW (1u << 30)    /* L4 ports lie past the batch window: the host reads the frame */
#define TXR_I0_MASK 0x1FFFFu

/* A tx launch takes one ring of the source, or up to USN_TX_RINGS consecutive
 * rings (rings > 1): workgroups [tile_base[k], tile_base[k + 1]) take ring k's
 * tiles.  The cross-tile protocol (aux granules, the learning sets' first
 * learners, learned items) runs over the launch's frame index: ring k's frame
 * j is tile_base[k] * USN_TILE + j; decisions, host lists, count rows and tile
 * headers are each ring's own. */
#define USN_TX_RINGS 8u
#define USN_TXC_HOST 4u         /* counters: frames ring k listed for the host stage, [4 + k] */
#define USN_TXC_LEARNED (USN_TXC_HOST + USN_TX_RINGS)   /* ... ring k's learned items (k >= 1) */
#define USN_TXC_WORDS (USN_TXC_LEARNED + USN_TX_RINGS)
struct TxArgs {
  ClassifyArgs a[USN_TX_RINGS];  /* ring k's batch and outputs; ring 0's also the shared
                                    fields: table, source, carried cache */
  uint32_t tile_base[USN_TX_RINGS + 1];
  uint32_t rings;
  unsigned long long *aux;    /* per tile x TXA_GRANULES {epoch, value}: what crosses a tile boundary */
  uint32_t *early;            /* per tile: epoch << 16 | EARLY, packed (the EARLY look-back reads
                                 four tiles per 16-byte load; granules would take one line each) */
  unsigned long long *macset; /* slots x 2: {epoch<<48 | mac, epoch<<32 | ~first} */
  unsigned long long *ruleset;/* slots x 4: {epoch<<48 | fp48, epoch<<32 | ~first, key xy, key zw} */
  uint32_t macset_mask, ruleset_mask;
  uint32_t epoch;             /* 1..65535 */
  uint4 *learned;             /* items appended by tx_decide: {frame, kind 0 mac | 1 rule},
                                 {mac lo, mac hi} or the packed rule key {x, y, z, meta} */
  uint32_t *counters;         /* USN_TXC_WORDS: [0] learned items, [1] overflow/collision flags,
                                 [2] sets with items, [3] epoch of a batch whose tile waits timed
                                 out, [USN_TXC_HOST + k] frames of ring k listed for the host
                                 stage, [USN_TXC_LEARNED + k] learned items of ring k >= 1's
                                 frames (ring 0's: [0] minus the others) */
  uint32_t learned_cap;
  const unsigned long long *bridge_set; /* open addressing, bit 63 = used */
  uint32_t bridge_mask;
  const uint32_t *listen;     /* n_listen x {dst, proto | has_port << 8 | port << 16} */
  uint32_t n_listen;
  uint32_t next_dhcp_set;     /* the source's next_dhcp_endpoint is Some */
};

#define TXA_GRANULES 24u       /* aux granules (8 bytes) per tile */
constexpr size_t TXA_WORDS_BYTES = TXA_GRANULES * 8;
constexpr size_t TXA_TILE_BYTES = TXA_WORDS_BYTES + 4;   /* + the tile's packed EARLY word */
static_assert(sizeof(TxArgs) <= 4096, "kernel argument block");
static_assert(USN_TXC_WORDS <= 64, "tile 0's first wave zeroes the counters");
hipError_t launch_tx(const TxArgs &t, hipStream_t stream);

/* LDS bytes a classify block needs (table staged in LDS when table_in_lds). */
size_t classify_lds_bytes(uint32_t nbins, uint32_t table_units, bool table_in_lds, bool glds);
bool table_fits_lds(uint32_t nbins, uint32_t table_units);

hipError_t launch_classify(const MultiArgs &m, hipStream_t stream);
/* Recount the bin rows and class counts of tiles [t0, t1) from the (patched)
 * decisions (the scatter then runs again). */
hipError_t launch_recount(const ClassifyArgs &a, uint32_t t0, uint32_t t1, hipStream_t stream);
/* table[idx[k]] = val[k] for the n units of buf = {val[n] (uint4)} {idx[n] (u32)} */
hipError_t launch_patch(uint4 *table, const void *buf, uint32_t n, hipStream_t stream);

/* ---- per-endpoint lists: the device-wide stable scatter ------------------
 * After the classify (or tx) kernel has written each tile's decisions and its
 * row of per-bin frame counts (cnt[tile][bin], u16), two launches:
 *   scan     (range of 16 x cpt chunks, block of USN_SCAN_BLK bins):
 *            agg[chunk][bin] = frames of the bin in the batch's chunks before
 *            (ranges hand their totals on through epoch-tagged granules),
 *            tot[bin] = the bin's frames
 *   scatter  (chunk of tc tiles): one LDS atomic per frame ranks it in the
 *            chunk's bin-sorted LDS stage (verified; ballot ranks as the
 *            fallback); the stage is written out in order, so each bin's
 *            frames of the chunk leave as one contiguous run
 * Stable: bins in order, frames in frame order inside a bin. */
#define USN_SCAN_RANGE_MIN 16u   /* chunks per scan workgroup: 16 x cpt (1, 2, 4) */
#define USN_SCAN_BLK 64u     /* bins per scan workgroup */
struct ScatterBatch {
  const uint32_t *decisions;
  const uint16_t *cnt;      /* [ntiles][nbw] */
  uint32_t *agg;            /* [nchunks][nbw]: frames per bin in the chunks before */
  uint32_t *tot;            /* [nbw]: frames per bin */
  unsigned long long *gran; /* [nranges][nbw]: {epoch, range total} */
  uint32_t *diag;           /* USN_DIAG_*: the lists are wrong (usn_finalize reports it) */
  uint32_t *index;          /* [n] */
  uint32_t *bin_off;        /* [nbins + 1] */
  uint32_t n, ntiles, tc, nchunks, nranges;
  /* an rx batch's state for usn_finalize, in host-mapped memory (or null):
   * [0] the launch tag, [1] summary flags, [2] USN_DIAG_LISTS when a chunk
   * found inconsistent lists, [3] 1 when a tile listed frames for the host
   * stage, [4..6] bin_off at the NIC, FLOOD and DROP bins, [7] the scan's
   * diag word.  Written by the scatter (chunk 0; [2] by any chunk). */
  uint32_t *rx_state;
  const usn_summary *summary;
};
struct ScatterArgs {
  ScatterBatch b[USN_MAX_MULTI];
  uint32_t chunk_base[USN_MAX_MULTI + 1];   /* scatter grid: chunks of batch i */
  uint32_t range_base[USN_MAX_MULTI + 1];   /* scan grid (x nbb): ranges of batch i */
  uint32_t count;
  uint32_t nbins, nbw, nbb, n_ep, nbits;
  uint32_t tc;                              /* the scatter kernel's chunk length for this launch */
  uint32_t flags;                           /* USN_SCF_* */
  uint32_t epoch;                           /* this launch's granule tag (never 0) */
  uint32_t cpt;                             /* scan: chunks per thread (1, 2, 4) */
  /* tx: chunk 0 of each batch (ring) also writes its state into host-mapped
   * memory for usn_finalize, USN_TXS_WORDS per ring: [0] summary flags,
   * [1] the ring's learned items, [2] counters[1] (flags), [3] counters[2],
   * [4] counters[3] (timeout epoch), [5] the ring's host-stage frames,
   * [6..8] bin_off[n_ep .. n_ep + 2], [9] n, [10] the scan's diag; word 11 of
   * ring 0's set by any chunk that finds inconsistent lists */
  uint32_t *txs_out;
  const uint32_t *txs_counters;
};
#define USN_TXS_WORDS 16u
#define USN_DIAG_TIMEOUT 1u     /* a scan wait timed out (200 ms; never observed) */
#define USN_DIAG_LISTS 2u       /* the scatter found count rows that disagree with the decisions */
#define USN_SCF_NOSCAN 2u      /* every batch is one chunk: no scan launch; the chunk's own counts
                                  are the batch's (agg = 0, tot = the chunk's sums) */
#define USN_SCF_SELFSCAN 4u    /* a small launch (every chunk resident at once, few count-row
                                  bytes per batch): no scan launch; each chunk sums its batch's
                                  count rows itself (the totals, and the tiles before it) */
#define USN_SCF_SLOW_RANK 1u   /* test hook (USN_SCATTER_SLOW_RANK=1): every chunk also ranks the
                                  ballot way and writes its stage out again */
/* The scatter kernel's chunk length (tc tiles, one wave each) for nbins
 * bins: the longest chunk (contiguous runs per bin) whose LDS -- stage
 * tc x 4 KiB | offsets nbw x 4 | cursors tc x nbw x 2 (| self-scan sums
 * nbw x 8) -- fits 64 KiB. */
struct ScatterShape { uint32_t tc; size_t lds; };
inline size_t scatter_lds(uint32_t nbins, uint32_t tc, bool selfscan = false) {
  const size_t nbw = (nbins + 7u) & ~7u;
  return (size_t)tc * USN_TILE * 4 + nbw * 4 + (size_t)tc * nbw * 2 + (selfscan ? nbw * 8 : 0);
}
inline ScatterShape scatter_shape(uint32_t nbins) {
  for (uint32_t tc : {8u, 4u, 2u})
    if (scatter_lds(nbins, tc) <= 64u * 1024u) return ScatterShape{tc, scatter_lds(nbins, tc)};
  return ScatterShape{1, scatter_lds(nbins, 1)};
}
inline uint32_t scatter_occupancy(size_t lds) {
  const uint32_t occ = (uint32_t)((160u * 1024u) / (lds ? lds : 1));
  return occ > 4 ? 4 : occ;
}
/* how a launch's lists are built (usn_host.cpp scatter_plan) */
struct ScatterPlan { uint32_t tc, cpt; bool noscan, selfscan; };
ScatterPlan scatter_plan(const uint32_t *ntiles, uint32_t count, uint32_t nbins, uint32_t cus,
                         uint32_t tc_knob, uint32_t cpt_knob, uint32_t selfscan_kb);
/* scratch bytes of one batch (cnt | agg | tot | gran | diag; agg and gran
 * sized for one-tile chunks) and its carve for chunks of tc tiles */
size_t scatter_scratch_bytes(uint64_t n, uint32_t nbins);
void scatter_carve(void *scratch, uint64_t cap, uint64_t n, uint32_t nbins, uint32_t tc, uint32_t cpt,
                   ScatterBatch &sb, uint16_t **cnt);
void scatter_tail(void *scratch, uint64_t cap, uint32_t nbins, void **p, size_t *bytes);
uint32_t *scatter_diag(void *scratch, uint64_t cap, uint32_t nbins);

}  // namespace usn

/* the same kernels at 512 threads per tile (a second compilation of
 * usn_device.hip); usn_host.cpp use_t512() picks the build per launch */
namespace usn_t512 {
hipError_t launch_classify(const usn::MultiArgs &m, hipStream_t stream);
/* done (optional): an event bound to the scatter kernel's dispatch, complete
 * when the lists are (hipExtLaunchKernel's stop event) */
hipError_t launch_scatter(const usn::ScatterArgs &s, hipStream_t stream, hipEvent_t done = nullptr);
uint32_t scatter_fallbacks();   /* chunks the scatter ranked again (current device) */
hipError_t launch_tx(const usn::TxArgs &t, hipStream_t stream);
bool table_fits_lds(uint32_t nbins, uint32_t table_units);
}

#endif
