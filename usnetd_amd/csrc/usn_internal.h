/*
 * usn_internal.h -- layouts shared by the HIP kernels and the C++ host.
 *
 * Rule table in HBM/LDS: open addressing over 64-byte buckets of four 16-byte
 * slots (one cache line per probe).  A slot is the exact Want key of
 * /root/reference/src/pkt.rs:220-227 packed into three words plus a meta word:
 *   x = dst_addr
 *   y = src_addr          (0 when absent)
 *   z = dst_port | src_port << 16   (absent ports are 0)
 *   w = protocol | present << 8 | VALID | owner_is_nic << 12 | owner << 16
 * The key compare is (x, y, z, w & KEY_META_MASK); `present` makes
 * Option::None differ from Some(0) exactly as derive(Eq) on Want does.
 * The table is rebuilt from the host registry on every change (no
 * tombstones), so a probe ends at the first bucket that has a free slot.
 * Tables too large for LDS also get a tag array: one 16-byte line per
 * bucket holding the four slots' 32-bit key tags (usn_key_tag of the bucket
 * hash), so a global-memory probe is one 16-byte load plus one 16-byte slot
 * load on a tag match, instead of four slot loads.
 *
 * PacketInfo (pkt.rs:11-22) as 4 words, compared whole for the 1-entry
 * decision cache (endpoint.rs:186-191, derive(PartialEq)):
 *   i0 = kind | proto << 8 | has_ports << 16     kind: 1 Ipv4, 2 Arp, 3 Eapol
 *   i1 = src_addr, i2 = dst_addr                 (0 for Arp/Eapol)
 *   i3 = has_ports ? src_port | dst_port << 16 : 0
 */
#ifndef USN_INTERNAL_H
#define USN_INTERNAL_H

#include <stdint.h>

#ifndef USN_AB_OLDKEYHASH
#define USN_AB_OLDKEYHASH 0
#endif

#define USN_SLOT_VALID (1u << 11)
#define USN_SLOT_NICOWNER (1u << 12)
#define USN_KEY_META_MASK 0x0FFFu

#define USN_INFO_IPV4 1u
#define USN_INFO_ARP 2u
#define USN_INFO_EAPOL 3u

/* tile header last_state bits */
#define USN_TS_HAS 1u       /* a frame in the tile touched the cache */
#define USN_TS_RETAINED 2u  /* ...and left last_pkt = Some(info) */
#define USN_TS_UNKNOWN 4u   /* ...but it is a later fragment (host resolves) */

/* summary cin/cout state bits */
#define USN_CS_VALID 1u     /* last_pkt is Some(info) */

/* bins of the per-tile order: endpoints 0..E-1, then NIC, FLOOD, DROP */
#define USN_BIN_NIC(E) (E)
#define USN_BIN_FLOOD(E) ((E) + 1)
#define USN_BIN_DROP(E) ((E) + 2)

#if defined(__HIPCC__) || defined(__HIP__)
#define USN_HD __host__ __device__ __forceinline__
#else
#define USN_HD static inline
#endif

USN_HD uint32_t usn_rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

/* Bucket hash of a packed key.  Shared bit-for-bit by host build and device probe. */
USN_HD uint32_t usn_key_hash(uint32_t x, uint32_t y, uint32_t z, uint32_t meta) {
  uint32_t h = x * 0x9E3779B1u;
  h ^= usn_rotl32(y * 0x85EBCA77u, 13);
  h ^= usn_rotl32(z * 0xC2B2AE3Du, 7);
  h ^= meta * 0x27D4EB2Fu;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

/* ---- perfect-hash rule image (hash-and-displace) ------------------------
 * The device image holds two tables: K1 = the rules key1 can hit (present
 * SRC or SRC|DPORT|SPORT), K2 = the rules key2 can hit (present 0 or DPORT);
 * rules of any other shape never match a frame and are not in the image.
 * Each table: 2^shift shards of m slots (16 B, the packed key above) and g
 * 16-bit displacements each (one shard up to 64K keys).  A key's shard is the
 * top `shift` bits of h1, its group within the shard mulhi(h1 << shift, g),
 * its slot shard * m + usn_ph_slot(h2, disp[shard * g + group], m): a probe
 * is one displacement read and ONE slot read, hit or miss.  Shards are
 * placed independently (in parallel on the host). */
USN_HD uint32_t usn_mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}
/* the low 32 bits of a 24 x 24-bit product: one full-rate v_mul_u32_u24 /
 * v_mad_u32_u24 on CDNA (a 32-bit v_mul_lo_u32 is quarter rate).  Callers
 * keep both operands below 2^24 (shard ids < 2^16, m and g < 2^24: ph_build) */
USN_HD uint32_t usn_mul24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul24(a, b);
#else
  return (a & 0xFFFFFFu) * (b & 0xFFFFFFu);
#endif
}
USN_HD uint32_t usn_fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
/* second key hash, independent of usn_key_hash (other multipliers).  Not
 * finalised: usn_ph_slot mixes h2 + d * phi through usn_fmix32 anyway, so
 * the probe spends two quarter-rate multiplies fewer (round 6); keys of one
 * group only need distinct h2 values */
USN_HD uint32_t usn_key_hash2(uint32_t x, uint32_t y, uint32_t z, uint32_t meta, uint32_t seed) {
  uint32_t h = (x ^ seed) * 0xCC9E2D51u;
  h = usn_rotl32(h, 15) ^ (y * 0x1B873593u);
  h = usn_rotl32(h, 13);
  h = (h ^ (h << 5)) + 0xE6546B64u;   // (murmur's h * 5 + c became a quarter-rate 64-bit mad)
  h ^= usn_rotl32(z * 0x85EBCA77u, 17);
  h ^= (meta + seed) * 0x165667B1u;
#if USN_AB_OLDKEYHASH   /* A/B (tools/abl_flags.sh): round 5's finalised h2 */
  return usn_fmix32(h);
#else
  return h ^ (h >> 16);
#endif
}
USN_HD uint32_t usn_ph_h1(uint32_t x, uint32_t y, uint32_t z, uint32_t meta, uint32_t seed) {
  return usn_key_hash(x, y ^ seed, z, meta);
}
/* d is a 16-bit displacement: d * phi with a 24-bit odd phi is one
 * full-rate 24-bit multiply */
USN_HD uint32_t usn_ph_slot(uint32_t h2, uint32_t d, uint32_t m) {
  return usn_mulhi32(usn_fmix32(h2 + usn_mul24(d, 0x9E3779u)), m);
}
USN_HD uint32_t usn_ph_shard(uint32_t h1, uint32_t shift) {
  return shift ? h1 >> (32u - shift) : 0u;
}
/* index of the key's displacement within its table's displacements */
USN_HD uint32_t usn_ph_group(uint32_t h1, uint32_t shift, uint32_t g) {
  return usn_mul24(usn_ph_shard(h1, shift), g) + usn_mulhi32(h1 << shift, g);
}
/* the first slot of the key's shard */
USN_HD uint32_t usn_ph_sbase(uint32_t h1, uint32_t shift, uint32_t m) {
  return usn_mul24(usn_ph_shard(h1, shift), m);
}

/* one table of the image, in 16-byte units / u16 units from the image base */
typedef struct {
  uint32_t slot_off;   /* first slot (16-B units) */
  uint32_t m;          /* slots per shard */
  uint32_t disp_off;   /* first displacement (u16 units) */
  uint32_t g;          /* groups per shard */
  uint32_t seed;
  uint32_t shift;      /* log2 of the shards */
  uint32_t _pad[2];
} usn_ph_table;

/* ---- projection table U and its overflow table X (rx, displacements in LDS)
 * key1 and key2 of a frame (pkt.rs:96-113) share their projection (dst,
 * proto, has_ports, dport): key2 IS the projection, key1 adds (src, sport).
 * U holds one slot per projection that some matchable K1 or K2 rule has:
 *   x = dst
 *   y = src of one K1 rule of the projection (inline)
 *   z = that rule's sport | o1 << 16 | USN_U_MORE
 *   w = E | o2 << 19                       (o2: the K2 rule of the projection)
 * E = has_ports ? pidx(proto) << 16 | dport : 5 << 16 | proto (19 bits; a
 * frame has ports only for the five protocols of protocol_has_ports).
 * o1 / o2: the owner id, USN_U_NIC (owned by a NIC: get_endpoint returns
 * None) or USN_U_NONE.  USN_U_MORE: further K1 rules share the projection;
 * they are in table X (K1's slot format).  A frame reads ONE U slot for both
 * of get_endpoint's lookups (endpoint.rs:317-327), and X only when MORE is
 * set and the inline rule is not its key1.  Empty U slots are USN_U_EMPTY_W
 * in w (E = 0x7FFFF never occurs).  Hashed as the key (dst, 0, E, 0). */
#define USN_U_NONE 0x1FFFu
#define USN_U_NIC 0x1FFEu
#define USN_U_MORE (1u << 29)
#define USN_U_EMASK 0x7FFFFu
#define USN_U_EMPTY_W 0xFFFFFFFFu
/* 0..4 for TCP, UDP, DCCP, SCTP, UDPLite (pkt.rs protocol_has_ports), 7 else */
USN_HD uint32_t usn_u_pidx(uint32_t proto) {
  return proto == 6u ? 0u : proto == 17u ? 1u : proto == 33u ? 2u : proto == 132u ? 3u
         : proto == 136u ? 4u : 7u;
}
/* usn_u_pidx of a protocol that has ports (6, 17, 33 -> p >> 4; 132, 136 ->
 * 3 + bit 3), without compares (the rx kernel's form) */
USN_HD constexpr uint32_t usn_u_pidx_ports(uint32_t proto) {
  return (proto & 0x80u) ? 3u + ((proto >> 3) & 1u) : (proto >> 4);
}
static_assert(usn_u_pidx_ports(6) == 0 && usn_u_pidx_ports(17) == 1 && usn_u_pidx_ports(33) == 2 &&
                  usn_u_pidx_ports(132) == 3 && usn_u_pidx_ports(136) == 4,
              "usn_u_pidx_ports differs from usn_u_pidx on a protocol with ports");
USN_HD uint32_t usn_u_e(uint32_t proto, uint32_t has_ports, uint32_t dport) {
  return has_ports ? (usn_u_pidx(proto) << 16 | (dport & 0xFFFFu)) : (5u << 16 | (proto & 0xFFu));
}
/* an owner code as the slot meta word a K1/K2 probe returns (0 = no rule) */
USN_HD uint32_t usn_u_meta(uint32_t o) {
  return o == USN_U_NONE ? 0u
         : o == USN_U_NIC ? (USN_SLOT_VALID | USN_SLOT_NICOWNER)
                          : (USN_SLOT_VALID | (o << 16));
}

/* 32-bit tag of a key in the tag array of a global-memory table (0 = empty) */
USN_HD uint32_t usn_key_tag(uint32_t h) { return h | 1u; }

/* MAC (48 bits) set hash, shared by the host bridge-set build and the device
 * probe.  (Round 6 tried 24-bit multiplies here: the tx grid ran 9 % slower,
 * longer probe runs on c4tx's MAC pattern, profiles/r06/r06d.) */
USN_HD uint32_t usn_mac_hash(uint64_t m) {
  m ^= m >> 29;
  m *= 0xBF58476D1CE4E5B9ull;
  m ^= m >> 32;
  return (uint32_t)m;
}

/* 48-bit fingerprint of a packed Want key (tx learned-rule set) */
USN_HD uint64_t usn_key_fp48(uint32_t x, uint32_t y, uint32_t z, uint32_t meta) {
  uint64_t h = ((uint64_t)x << 32 | y) * 0x9E3779B97F4A7C15ull;
  h ^= (((uint64_t)z << 32) | meta) + 0x632BE59BD9B4E019ull + (h << 6) + (h >> 2);
  h *= 0xC2B2AE3D27D4EB4Full;
  h ^= h >> 31;
  return h & 0xFFFFFFFFFFFFull;
}

USN_HD uint32_t usn_key_meta(uint32_t proto, uint32_t present) {
  return (proto & 0xFFu) | ((present & 7u) << 8) | USN_SLOT_VALID;
}

USN_HD uint32_t usn_mkdec(uint32_t cls, uint32_t reason, uint32_t ep) {
  return (ep & 0xFFFFu) | (cls << 16) | (reason << 20);
}

#endif
