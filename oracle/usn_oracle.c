/*
 * usn_oracle.c -- sequential CPU restatement of usnetd's match path.
 * TEST INFRASTRUCTURE ONLY (see usn_oracle.h).  PARITY UNPINNED: no
 * reference tests or fixtures exist; see DESIGN.md "Oracle".
 */
#include "usn_oracle.h"

#include <stdlib.h>
#include <string.h>

#define USO_MAX_EP 8192

/* ------------------------------------------------------------------ */
/* decision word (see header)                                          */
enum { C_DROP = 0, C_EP = 1, C_NIC = 2, C_FLOOD = 3 };
enum { R_NONE = 0, R_PARSE = 1, R_LOOPBACK = 2, R_NOMATCH = 3, R_EXCLUDED = 4,
       R_FRAGMISS = 5, R_DHCP_NONE = 6 };
#define F_CACHE_HIT (1u << 24)
#define F_DHCP_STEER (1u << 27)

static uint32_t mkdec(uint32_t cls, uint32_t reason, uint32_t ep) {
  return (ep & 0xFFFFu) | (cls << 16) | (reason << 20);
}
static uint32_t drop(uint32_t reason) { return mkdec(C_DROP, reason, 0xFFFF); }

/* ------------------------------------------------------------------ */
/* PacketInfo, pkt.rs:11-22.  kind: 1 Ipv4, 2 Arp, 3 Eapol.            */
typedef struct {
  uint8_t kind, proto, has_ports, _p;
  uint32_t src, dst;
  uint16_t sport, dport;
} info_t;

/* derive(PartialEq) on PacketInfo: variant + every Ipv4 field; Option<u16>
 * ports compare presence and value.  MACs are not part of PacketInfo. */
static int info_eq(const info_t *a, const info_t *b) {
  if (a->kind != b->kind) return 0;
  if (a->kind != 1) return 1;
  if (a->src != b->src || a->dst != b->dst || a->proto != b->proto) return 0;
  if (a->has_ports != b->has_ports) return 0;
  if (a->has_ports && (a->sport != b->sport || a->dport != b->dport)) return 0;
  return 1;
}

static uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
static uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* ------------------------------------------------------------------ */
/* generic open-addressing map with backward-shift deletion            */
typedef struct {
  uint8_t *slots;     /* cap * stride bytes; byte 0 of a slot = used flag */
  uint64_t cap, n, stride, keylen;  /* key lives at slot+8, value after key */
} omap;

static uint64_t hash_bytes(const uint8_t *k, uint64_t len) {
  uint64_t h = 1469598103934665603ull;
  for (uint64_t i = 0; i < len; i++) { h ^= k[i]; h *= 1099511628211ull; }
  h ^= h >> 31; h *= 0x9E3779B97F4A7C15ull; h ^= h >> 29;
  return h;
}

static void omap_init(omap *m, uint64_t keylen, uint64_t vallen) {
  m->keylen = keylen;
  m->stride = (8 + keylen + vallen + 7) & ~7ull;
  m->cap = 16; m->n = 0;
  m->slots = (uint8_t *)calloc(m->cap, m->stride);
}
static void omap_free(omap *m) { free(m->slots); m->slots = NULL; m->cap = m->n = 0; }
static uint8_t *slot_at(const omap *m, uint64_t i) { return m->slots + i * m->stride; }

static uint8_t *omap_find(const omap *m, const uint8_t *key) {
  uint64_t mask = m->cap - 1, i = hash_bytes(key, m->keylen) & mask;
  for (;;) {
    uint8_t *s = slot_at(m, i);
    if (!s[0]) return NULL;
    if (memcmp(s + 8, key, m->keylen) == 0) return s + 8 + m->keylen;
    i = (i + 1) & mask;
  }
}
static void omap_grow(omap *m);
/* returns value pointer; *existed set */
static uint8_t *omap_insert(omap *m, const uint8_t *key, int *existed) {
  if ((m->n + 1) * 2 > m->cap) omap_grow(m);
  uint64_t mask = m->cap - 1, i = hash_bytes(key, m->keylen) & mask;
  for (;;) {
    uint8_t *s = slot_at(m, i);
    if (!s[0]) {
      s[0] = 1; memcpy(s + 8, key, m->keylen); m->n++;
      *existed = 0; return s + 8 + m->keylen;
    }
    if (memcmp(s + 8, key, m->keylen) == 0) { *existed = 1; return s + 8 + m->keylen; }
    i = (i + 1) & mask;
  }
}
static void omap_grow(omap *m) {
  omap old = *m;
  m->cap = old.cap * 2; m->n = 0;
  m->slots = (uint8_t *)calloc(m->cap, m->stride);
  for (uint64_t i = 0; i < old.cap; i++) {
    uint8_t *s = slot_at(&old, i);
    if (s[0]) { int ex; uint8_t *v = omap_insert(m, s + 8, &ex);
      memcpy(v, s + 8 + old.keylen, old.stride - 8 - old.keylen); }
  }
  free(old.slots);
}
static void omap_erase_slot(omap *m, uint64_t i) {
  uint64_t mask = m->cap - 1;
  slot_at(m, i)[0] = 0; m->n--;
  uint64_t j = i;
  for (;;) {
    j = (j + 1) & mask;
    uint8_t *s = slot_at(m, j);
    if (!s[0]) break;
    uint64_t home = hash_bytes(s + 8, m->keylen) & mask;
    /* can s move to the hole at i? yes if home is not cyclically in (i, j] */
    int between = (i <= j) ? (home > i && home <= j) : (home > i || home <= j);
    if (!between) {
      memcpy(slot_at(m, i), s, m->stride);
      s[0] = 0;
      i = j;
    }
  }
}
static int omap_erase(omap *m, const uint8_t *key) {
  uint64_t mask = m->cap - 1, i = hash_bytes(key, m->keylen) & mask;
  for (;;) {
    uint8_t *s = slot_at(m, i);
    if (!s[0]) return 0;
    if (memcmp(s + 8, key, m->keylen) == 0) { omap_erase_slot(m, i); return 1; }
    i = (i + 1) & mask;
  }
}
static void omap_clear(omap *m) {
  memset(m->slots, 0, m->cap * m->stride); m->n = 0;
}

/* ------------------------------------------------------------------ */
/* canonical Want key: Option fields zeroed when absent so that the   */
/* byte image is a faithful derive(Hash, Eq) key (pkt.rs:220-227).    */
typedef struct { uint32_t dst, src; uint16_t dport, sport; uint8_t proto, mask, p0, p1; } wkey;
static wkey want_key(const uso_want *w) {
  wkey k; memset(&k, 0, sizeof k);
  k.dst = w->dst_addr; k.proto = w->protocol; k.mask = w->mask & 7;
  if (k.mask & 1) k.dport = w->dst_port;
  if (k.mask & 2) k.src = w->src_addr;
  if (k.mask & 4) k.sport = w->src_port;
  return k;
}
typedef struct { int32_t owner; uint8_t sticky, p[3]; } rval;

/* FragmentationKey, pkt.rs:135-156 */
typedef struct { uint32_t src, dst; uint16_t id; uint8_t proto, p0; uint8_t smac[6], dmac[6]; } fkey;
typedef struct { info_t info; uint8_t smac[6], dmac[6]; } fval;

typedef struct { uint32_t dst; uint8_t proto, has_port; uint16_t port; } listen_t;

typedef struct {
  int used, kind, for_nic;
  listen_t *listening; int n_listen, cap_listen;
  int next_dhcp;                 /* -1 = None */
  int has_last; info_t last_pkt; /* last_pkt: Option<PacketInfo> */
  uint32_t last_dst;             /* last_pkt_dst as a decision word (DROP = None) */
} ep_t;

struct uso_ctx {
  ep_t ep[USO_MAX_EP];
  omap rules;     /* Want -> (owner, sticky): match_register, main.rs:448 */
  omap frags;     /* fragmentation_map, main.rs:447 */
  uint8_t (*bridge)[6]; int n_bridge, cap_bridge;   /* innerl2bridge, main.rs:449 */
};

uso_ctx *uso_create(void) {
  uso_ctx *c = (uso_ctx *)calloc(1, sizeof(uso_ctx));
  omap_init(&c->rules, sizeof(wkey), sizeof(rval));
  omap_init(&c->frags, sizeof(fkey), sizeof(fval));
  return c;
}
void uso_destroy(uso_ctx *c) {
  if (!c) return;
  for (int i = 0; i < USO_MAX_EP; i++) free(c->ep[i].listening);
  omap_free(&c->rules); omap_free(&c->frags); free(c->bridge); free(c);
}

int uso_add_endpoint(uso_ctx *c, int id, int kind, int for_nic) {
  if (id < 0 || id >= USO_MAX_EP || c->ep[id].used) return -1;
  if ((kind == USO_KIND_NIC) != (for_nic < 0)) return -1;
  ep_t *e = &c->ep[id];
  memset(e, 0, sizeof *e);
  e->used = 1; e->kind = kind; e->for_nic = for_nic; e->next_dhcp = -1;
  return 0;
}

int uso_remove_endpoint(uso_ctx *c, int id) {
  if (id < 0 || id >= USO_MAX_EP || !c->ep[id].used) return -1;
  /* match_register.retain(|_, (_, rc)| !ptr_eq(rc, e)) */
  for (uint64_t i = 0; i < c->rules.cap;) {
    uint8_t *s = slot_at(&c->rules, i);
    if (s[0] && ((rval *)(s + 8 + sizeof(wkey)))->owner == id) {
      omap_erase_slot(&c->rules, i);   /* slot i refilled: re-check it */
    } else i++;
  }
  free(c->ep[id].listening);
  memset(&c->ep[id], 0, sizeof(ep_t));
  return 0;
}

static void push_listen(ep_t *e, uint32_t dst, uint8_t proto, int has_port, uint16_t port) {
  if (e->n_listen == e->cap_listen) {
    e->cap_listen = e->cap_listen ? 2 * e->cap_listen : 4;
    e->listening = (listen_t *)realloc(e->listening, e->cap_listen * sizeof(listen_t));
  }
  listen_t *l = &e->listening[e->n_listen++];
  l->dst = dst; l->proto = proto; l->has_port = (uint8_t)has_port; l->port = has_port ? port : 0;
}

int uso_add_match(uso_ctx *c, const uso_want *w, int owner, int sticky) {
  if (owner < 0 || owner >= USO_MAX_EP || !c->ep[owner].used) return -2;
  wkey k = want_key(w);
  if (omap_find(&c->rules, (const uint8_t *)&k)) return 0;          /* main.rs:272-274 */
  ep_t *e = &c->ep[owner];
  push_listen(e, k.dst, k.proto, k.mask & 1, k.dport);              /* main.rs:276-279 */
  if (e->for_nic < 0) return -1;                                    /* main.rs:287-289 panics */
  c->ep[e->for_nic].has_last = 0;                                   /* main.rs:281-286 */
  int ex; rval *v = (rval *)omap_insert(&c->rules, (const uint8_t *)&k, &ex);
  v->owner = owner; v->sticky = (uint8_t)(sticky != 0);
  return 1;
}

int uso_remove_match(uso_ctx *c, const uso_want *w, int requester) {
  wkey k = want_key(w);
  rval *v = (rval *)omap_find(&c->rules, (const uint8_t *)&k);
  if (v && v->owner != requester) return -1;                        /* main.rs:612-616 */
  return omap_erase(&c->rules, (const uint8_t *)&k);                /* no cache clear */
}

int uso_lookup(const uso_ctx *c, const uso_want *w) {
  wkey k = want_key(w);
  rval *v = (rval *)omap_find(&c->rules, (const uint8_t *)&k);
  return v ? v->owner : -1;
}
int uso_rule_count(const uso_ctx *c) { return (int)c->rules.n; }
int uso_rules(const uso_ctx *c, uso_want *w, int32_t *owner, uint8_t *sticky, int cap) {
  int n = 0;
  for (uint64_t i = 0; i < c->rules.cap && n < cap; i++) {
    uint8_t *s = slot_at(&c->rules, i);
    if (!s[0]) continue;
    const wkey *k = (const wkey *)(s + 8);
    const rval *v = (const rval *)(s + 8 + sizeof(wkey));
    memset(&w[n], 0, sizeof(uso_want));
    w[n].dst_addr = k->dst; w[n].src_addr = k->src; w[n].dst_port = k->dport;
    w[n].src_port = k->sport; w[n].protocol = k->proto; w[n].mask = k->mask;
    owner[n] = v->owner; sticky[n] = v->sticky; n++;
  }
  return n;
}

static int bridge_contains(const uso_ctx *c, const uint8_t *mac) {
  for (int i = 0; i < c->n_bridge; i++) if (memcmp(c->bridge[i], mac, 6) == 0) return 1;
  return 0;
}
void uso_bridge_add(uso_ctx *c, const uint8_t mac[6]) {
  /* ADD_MACS prefill pushes unconditionally (main.rs:450-462) */
  if (c->n_bridge == c->cap_bridge) {
    c->cap_bridge = c->cap_bridge ? 2 * c->cap_bridge : 16;
    c->bridge = (uint8_t(*)[6])realloc(c->bridge, (size_t)c->cap_bridge * 6);
  }
  memcpy(c->bridge[c->n_bridge++], mac, 6);
}
int uso_bridge_count(const uso_ctx *c) { return c->n_bridge; }
void uso_frag_clear(uso_ctx *c) { omap_clear(&c->frags); }

int uso_get_cache(const uso_ctx *c, int id, uint32_t *last_dst, uint8_t info16[16]) {
  const ep_t *e = &c->ep[id];
  if (!e->has_last) return 0;
  *last_dst = e->last_dst;
  memset(info16, 0, 16);
  info16[0] = e->last_pkt.kind; info16[1] = e->last_pkt.proto; info16[2] = e->last_pkt.has_ports;
  memcpy(info16 + 4, &e->last_pkt.src, 4); memcpy(info16 + 8, &e->last_pkt.dst, 4);
  if (e->last_pkt.has_ports) { memcpy(info16 + 12, &e->last_pkt.sport, 2); memcpy(info16 + 14, &e->last_pkt.dport, 2); }
  return 1;
}
int uso_get_next_dhcp(const uso_ctx *c, int id) { return c->ep[id].next_dhcp; }

/* ------------------------------------------------------------------ */
/* extract_pkt_info, pkt.rs:158-218 (+ smoltcp 0.7.0 checks).          */
/* returns 0 ok, else drop reason                                       */
static int extract(uso_ctx *c, const uint8_t *b, uint32_t len, info_t *info,
                   uint8_t smac[6], uint8_t dmac[6]) {
  memset(info, 0, sizeof *info);
  if (len < 14) return R_PARSE;                         /* EthernetFrame::new_checked */
  memcpy(dmac, b, 6); memcpy(smac, b + 6, 6);
  uint16_t et = be16(b + 12);
  if (et == 0x0806) { info->kind = 2; return 0; }       /* pkt.rs:167-169 */
  if (et == 0x0800) {                                   /* pkt.rs:170-204 */
    const uint8_t *p = b + 14;
    uint32_t n = len - 14;
    if (n < 20) return R_PARSE;                         /* check_len: len < DST_ADDR.end */
    uint32_t hl = (uint32_t)(p[0] & 0x0F) * 4;
    uint32_t tl = be16(p + 2);
    if (n < hl) return R_PARSE;
    if (hl > tl) return R_PARSE;
    if (n < tl) return R_PARSE;
    uint16_t ff = be16(p + 6);
    fkey fk; memset(&fk, 0, sizeof fk);
    fk.id = be16(p + 4); fk.src = be32(p + 12); fk.dst = be32(p + 16); fk.proto = p[9];
    memcpy(fk.smac, smac, 6); memcpy(fk.dmac, dmac, 6);
    if ((uint16_t)(ff << 3) != 0) {                     /* frag_offset() > 0, pkt.rs:172-176 */
      fval *v = (fval *)omap_find(&c->frags, (const uint8_t *)&fk);
      if (!v) return R_FRAGMISS;
      *info = v->info; memcpy(smac, v->smac, 6); memcpy(dmac, v->dmac, 6);
      return 0;
    }
    uint8_t proto = p[9];
    int ports = (proto == 6 || proto == 17 || proto == 0x21 || proto == 0x84 || proto == 0x88) &&
                (tl - hl) > 4;                         /* pkt.rs:128-133, 179 */
    info->kind = 1; info->proto = proto;
    info->src = be32(p + 12); info->dst = be32(p + 16);
    if (ports) { info->has_ports = 1; info->sport = be16(p + hl); info->dport = be16(p + hl + 2); }
    if (!(ff & 0x4000) && (ff & 0x2000)) {              /* pkt.rs:198-202 */
      int ex; fval *v = (fval *)omap_insert(&c->frags, (const uint8_t *)&fk, &ex);
      v->info = *info; memcpy(v->smac, smac, 6); memcpy(v->dmac, dmac, 6);
    }
    return 0;
  }
  if (et == 0x888E) { info->kind = 3; return 0; }       /* pkt.rs:206-213 */
  return R_PARSE;                                       /* Ipv6 (pkt.rs:205) and Unknown */
}

/* pkt.rs:36-58.  src_addr.is_unspecified() (pkt.rs:46) is smoltcp 0.7.0's
 * "falls into the unspecified range" test, self.0[0] == 0 (0.0.0.0/8), written
 * like is_loopback's self.0[0] == 127 (recalled; tag smoltcp-recall). */
static int is_dhcp_request(const info_t *i) {
  return i->kind == 1 && i->proto == 17 && (i->src >> 24) == 0 && i->has_ports &&
         i->sport == 68 && i->dport == 67 && (i->dst & 0xFF) == 255;
}
static int is_dhcp_answer(const info_t *i) {            /* pkt.rs:59-76 */
  return i->kind == 1 && i->proto == 17 && i->has_ports && i->sport == 67 && i->dport == 68;
}

/* get_endpoint, endpoint.rs:307-338.  Returns owner or -1; *excluded set when
 * the hit was discarded (NIC owner or the source itself). */
static int get_endpoint(const uso_ctx *c, int src, const info_t *i, int *excluded) {
  uso_want w; memset(&w, 0, sizeof w);
  w.dst_addr = i->dst; w.protocol = i->proto;
  w.mask = (uint8_t)(i->has_ports ? 1 : 0);
  w.dst_port = i->dport;
  /* to_match_want_with_src(true), pkt.rs:96-113 */
  uso_want w1 = w; w1.mask |= 2; w1.src_addr = i->src;
  if (i->has_ports) { w1.mask |= 4; w1.src_port = i->sport; }
  int e = uso_lookup(c, &w1);
  if (e < 0) e = uso_lookup(c, &w);                     /* with_src(false) */
  *excluded = 0;
  if (e >= 0 && (c->ep[e].kind == USO_KIND_NIC || e == src)) { *excluded = 1; return -1; }
  return e;
}

static int listening_contains(const ep_t *e, uint32_t dst, uint8_t proto, int has_port, uint16_t port) {
  for (int k = 0; k < e->n_listen; k++) {
    const listen_t *l = &e->listening[k];
    if (l->dst == dst && l->proto == proto && l->has_port == has_port && (!has_port || l->port == port))
      return 1;
  }
  return 0;
}

uint32_t uso_forward(uso_ctx *c, int src, const uint8_t *frame, uint32_t len) {
  ep_t *S = &c->ep[src];
  int incoming = S->kind == USO_KIND_NIC;               /* endpoint.rs:184 */
  info_t info; uint8_t smac[6], dmac[6];
  int r = extract(c, frame, len, &info, smac, dmac);
  if (r) return drop((uint32_t)r);                      /* endpoint.rs:292-295 */
  if (S->has_last && info_eq(&S->last_pkt, &info))      /* endpoint.rs:186-191 */
    return S->last_dst | F_CACHE_HIT;
  S->has_last = 0;                                      /* endpoint.rs:193 */
  if (!incoming && !(smac[0] & 1) && !bridge_contains(c, smac))
    uso_bridge_add(c, smac);                            /* endpoint.rs:195-197 */
  if (info.kind == 2 || info.kind == 3)                 /* endpoint.rs:199-204 */
    return mkdec(C_FLOOD, R_NONE, 0xFFFF);
  if ((info.dst >> 24) == 127) return drop(R_LOOPBACK); /* endpoint.rs:205-208 */
  S->has_last = 1; S->last_pkt = info;                  /* endpoint.rs:209 */
  if (!incoming) {                                      /* endpoint.rs:210-253 */
    /* to_want, pkt.rs:78-95: reversed tuple, src_addr = Some(dst) */
    uso_want w; memset(&w, 0, sizeof w);
    w.dst_addr = info.src; w.src_addr = info.dst; w.protocol = info.proto; w.mask = 2;
    if (info.has_ports) { w.mask |= 1 | 4; w.dst_port = info.sport; w.src_port = info.dport; }
    if (!listening_contains(S, w.dst_addr, w.protocol, w.mask & 1, w.dst_port)) {
      if (is_dhcp_request(&info)) {
        if (S->for_nic >= 0) {
          ep_t *N = &c->ep[S->for_nic];
          N->next_dhcp = src; N->has_last = 0; S->has_last = 0;
        }
      } else {
        wkey k = want_key(&w);
        if (!omap_find(&c->rules, (const uint8_t *)&k)) {
          if (S->for_nic >= 0) c->ep[S->for_nic].has_last = 0;  /* else: reference panics */
          int ex; rval *v = (rval *)omap_insert(&c->rules, (const uint8_t *)&k, &ex);
          v->owner = src; v->sticky = 0;
        }
      }
    }
  }
  uint32_t d;
  if (!incoming && !bridge_contains(c, dmac)) {         /* endpoint.rs:254-255 */
    d = mkdec(C_NIC, R_NONE, (uint32_t)S->for_nic);
  } else {
    int excluded;
    int e = get_endpoint(c, src, &info, &excluded);
    if (e < 0) {
      if (is_dhcp_answer(&info)) {                      /* endpoint.rs:262-273 */
        if (S->next_dhcp >= 0) {
          d = mkdec(C_EP, R_NONE, (uint32_t)S->next_dhcp) | F_DHCP_STEER;
          S->next_dhcp = -1; S->has_last = 0;
        } else d = drop(R_DHCP_NONE);
      } else d = drop(excluded ? R_EXCLUDED : R_NOMATCH);
    } else d = mkdec(C_EP, R_NONE, (uint32_t)e);
  }
  S->last_dst = d & 0x00FFFFFFu;                        /* endpoint.rs:285-290 */
  return d;
}

void uso_forward_batch(uso_ctx *c, int src, const uint8_t *base, uint64_t stride,
                       const uint64_t *offsets, const uint16_t *lens, uint64_t n,
                       uint32_t *out) {
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t *f = offsets ? base + offsets[i] : base + i * stride;
    out[i] = uso_forward(c, src, f, lens[i]);
  }
}
