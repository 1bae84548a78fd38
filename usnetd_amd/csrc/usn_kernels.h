/*
 * usn_kernels.h -- launch interface between the C++ host (usn_host.cpp) and
 * the HIP kernels (usn_device.hip).  Internal; not part of the C ABI.
 */
#ifndef USN_KERNELS_H
#define USN_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/usn_classify.h"

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
  /* outputs */
  uint32_t *decisions;
  uint16_t *order;
  uint32_t *runs;
  usn_tile_hdr *tiles;
  usn_summary *summary;
  uint32_t *host_list;      /* per tile USN_TILE slots */
  /* rule table: nbuckets * 4 slots of uint4 */
  const uint4 *table;
  uint32_t bucket_mask;
  uint32_t table_slots;
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
  uint32_t probe_mask;      /* bit0: rules key1 can hit exist; bit1: rules key2 can hit */
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

/* LDS bytes a classify block needs (table staged in LDS when table_in_lds). */
size_t classify_lds_bytes(uint32_t nbins, uint32_t table_slots, bool table_in_lds, bool dense);
bool table_fits_lds(uint32_t nbins, uint32_t table_slots);

hipError_t launch_classify(const MultiArgs &m, hipStream_t stream);
/* Rebuild order/runs/counts of tiles [t0, t1) from the (patched) decisions. */
hipError_t launch_resort(const ClassifyArgs &a, uint32_t t0, uint32_t t1, hipStream_t stream);

}  // namespace usn

#endif
