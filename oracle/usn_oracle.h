/*
 * usn_oracle.h -- CPU restatement of usnetd's per-frame match path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (usnetd_amd/, include/)
 * includes, links or loads this file.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it, and only as the checker.
 *
 * This is a sequential, single-threaded restatement of
 *   extract_pkt_info   /root/reference/src/pkt.rs:158-218
 *   PacketInfo preds   /root/reference/src/pkt.rs:23-126
 *   find_forward       /root/reference/src/endpoint.rs:172-296
 *   get_endpoint       /root/reference/src/endpoint.rs:307-338
 *   mirror_to_all      /root/reference/src/endpoint.rs:340-363 (as a FLOOD decision)
 *   add_listening_match /root/reference/src/main.rs:266-298
 *   RemoveMatch        /root/reference/src/main.rs:608-625 (act_on)
 *   endpoint removal   /root/reference/src/main.rs:1063-1069 (match_register.retain)
 * plus the smoltcp 0.7.0 wire semantics the reference calls
 * (EthernetFrame::new_checked, Ipv4Packet::new_checked/check_len, frag_offset,
 * dont_frag, more_frags; restated in SURVEY.md Appendix A.1).
 *
 * PARITY UNPINNED: the reference ships no tests, no golden vectors and cannot
 * be built here (Rust toolchain absent, smoltcp 0.7.0 / usnet_devices not
 * vendored).  The restatement is cross-checked against an independent Python
 * restatement (oracle/pyoracle.py) and against hand-derived known-answer
 * frames (tests/golden/), each citing the reference line it follows.
 *
 * Decision word (u32), shared by the oracle and the product by SPEC:
 *   [15:0]  endpoint id (0xFFFF = none)
 *   [19:16] class   0 DROP, 1 EP, 2 NIC, 3 FLOOD
 *   [23:20] reason  0 none, 1 PARSE, 2 LOOPBACK, 3 NOMATCH, 4 EXCLUDED,
 *                   5 FRAGMISS, 6 DHCP_NONE
 *   [31:24] flags   informational only; parity compares bits [23:0]
 */
#ifndef USN_ORACLE_H
#define USN_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { USO_KIND_NIC = 0, USO_KIND_HOST = 1, USO_KIND_PIPE = 2, USO_KIND_UDS = 3 };

typedef struct {
  uint32_t dst_addr;   /* IPv4, a.b.c.d == (a<<24)|(b<<16)|(c<<8)|d */
  uint32_t src_addr;   /* valid iff mask bit1 */
  uint16_t dst_port;   /* valid iff mask bit0 */
  uint16_t src_port;   /* valid iff mask bit2 */
  uint8_t protocol;
  uint8_t mask;        /* bit0 dst_port, bit1 src_addr, bit2 src_port */
  uint16_t _pad;
} uso_want;            /* Want, pkt.rs:220-227 */

typedef struct uso_ctx uso_ctx;

uso_ctx *uso_create(void);
void uso_destroy(uso_ctx *c);
/* Endpoint with a caller-chosen stable id (all_devices entry).  for_nic = -1
 * for NICs (main.rs Endpoints::add asserts NIC <=> for_nic is None). */
int uso_add_endpoint(uso_ctx *c, int id, int kind, int for_nic);
/* EntryChange::Remove: drops the endpoint and every rule it owns. */
int uso_remove_endpoint(uso_ctx *c, int id);
/* add_listening_match: 1 = inserted ("OK"), 0 = key existed ("ER"), <0 error
 * (owner is a NIC: the reference panics). */
int uso_add_match(uso_ctx *c, const uso_want *w, int owner, int sticky);
/* act_on RemoveMatch: 1 removed, 0 absent, -1 owner mismatch (not removed). */
int uso_remove_match(uso_ctx *c, const uso_want *w, int requester);
/* Lookup helper for tests: owner id or -1. */
int uso_lookup(const uso_ctx *c, const uso_want *w);
int uso_rule_count(const uso_ctx *c);
/* Copy out all rules (order unspecified). Returns count written (<= cap). */
int uso_rules(const uso_ctx *c, uso_want *w, int32_t *owner, uint8_t *sticky, int cap);
void uso_bridge_add(uso_ctx *c, const uint8_t mac[6]);
int uso_bridge_count(const uso_ctx *c);
void uso_frag_clear(uso_ctx *c);
/* Per-endpoint state inspection (for carried-state tests). */
int uso_get_cache(const uso_ctx *c, int id, uint32_t *last_dst, uint8_t info16[16]);
int uso_get_next_dhcp(const uso_ctx *c, int id);

/* find_forward for one frame from source endpoint src. */
uint32_t uso_forward(uso_ctx *c, int src, const uint8_t *frame, uint32_t len);
/* Endpoint::forward over a drained batch: frames at base + i*stride (stride>0)
 * or base + offsets[i] (offsets != NULL). */
void uso_forward_batch(uso_ctx *c, int src, const uint8_t *base, uint64_t stride,
                       const uint64_t *offsets, const uint16_t *lens, uint64_t n,
                       uint32_t *out);

#ifdef __cplusplus
}
#endif
#endif
