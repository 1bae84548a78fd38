/*
 * usn_classify.h -- C ABI of the MI355X-native usnetd match path.
 *
 * This is the drop-in boundary for usnetd's per-frame decision path.  The
 * reference has no FFI; the path is internal Rust and is called once per
 * received frame:
 *
 *   Endpoint::forward (drain loop)       /root/reference/src/endpoint.rs:114-171
 *     -> Endpoint::find_forward          /root/reference/src/endpoint.rs:172-296
 *        -> extract_pkt_info             /root/reference/src/pkt.rs:158-218
 *        -> get_endpoint                 /root/reference/src/endpoint.rs:307-338
 *        -> mirror_to_all (FLOOD)        /root/reference/src/endpoint.rs:340-363
 *
 * Here a drained rx ring is one batch resident in HBM and one call classifies
 * all of it.  The state the reference keeps in `main` and in each `Endpoint`
 * (match_register, innerl2bridge, fragmentation_map, listening, last_pkt,
 * last_pkt_dst, next_dhcp_endpoint) lives in a usn_ctx; the rule-registry
 * operations keep the reference's semantics so a host (Rust over this ABI,
 * see INTEGRATION.md, or the C++ control plane) can drive it directly.
 *
 * Conventions: every function returns int status (0 = ok, negative = error,
 * see USN_E*), never throws, never aborts.  Pointers named dev_* or documented
 * "device" are HIP device pointers on the ctx's device.  Nothing here takes
 * or returns a torch type.
 */
#ifndef USN_CLASSIFY_H
#define USN_CLASSIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 4: usn_result_release; two consecutive tx rings per usn_classify_multi;
 *    usn_finalize waits for the batch's own launch, not the stream
 * 5: up to eight consecutive tx rings per usn_classify_multi */
#define USN_ABI_VERSION 5
#define USN_WINDOW 64     /* default readable header bytes at every frame start (usn_batch.window) */
#define USN_WINDOW_MAX 80 /* the most extract_pkt_info ever reads: L4 ports of IHL 15 end at byte 78 */
#define USN_TILE 1024     /* frames per tile (one classify workgroup; tile headers) */
#define USN_MAX_ENDPOINTS 4095 /* endpoint ids 0..4094 (0xFFFF = none); netmap pipe ids are 12 bits
                                  (/root/reference/src/devices.rs:36-37) */

/* status codes */
#define USN_OK 0
#define USN_EINVAL (-22)
#define USN_ENOMEM (-12)
#define USN_EEXIST (-17)
#define USN_ENOENT (-2)
#define USN_EPERM (-1)
#define USN_EHIP (-5)        /* HIP runtime error; usn_last_hip_error() */
#define USN_ENODEV (-19)     /* no gfx950 device */
#define USN_ERANGE (-34)
#define USN_EBUSY (-16)      /* a tx batch awaits usn_finalize (shared state not final yet) */
#define USN_ELIST (-74)      /* EBADMSG: the device found the batch's per-bin counts disagreeing with
                                its decisions; index / bin_off of that batch are not valid */

/* ---- decision word (u32), one per frame --------------------------------
 *   [15:0]  endpoint id (0xFFFF = none)            Target::Endpoint/EndpointRef
 *   [19:16] class                                  Option<Target>
 *   [23:20] drop reason (informational, exact)
 *   [31:24] flags (informational)
 * Parity with the reference is defined on bits [23:0]. */
#define USN_CLS_DROP 0u    /* None: endpoint.rs:207, 275, 293 */
#define USN_CLS_EP 1u      /* Target::Endpoint / EndpointRef / Last->endpoint */
#define USN_CLS_NIC 2u     /* Target::Nic (endpoint id = the source's NIC) */
#define USN_CLS_FLOOD 3u   /* mirror_to_all: every endpoint except the source */
#define USN_R_NONE 0u
#define USN_R_PARSE 1u     /* extract_pkt_info -> None */
#define USN_R_LOOPBACK 2u  /* endpoint.rs:205-208 */
#define USN_R_NOMATCH 3u   /* endpoint.rs:274-277 */
#define USN_R_EXCLUDED 4u  /* get_endpoint hit a NIC or the source (endpoint.rs:328-336) */
#define USN_R_FRAGMISS 5u  /* later fragment without a remembered first (pkt.rs:172-176) */
#define USN_R_DHCP_NONE 6u /* DHCP answer, no rule, no next_dhcp (endpoint.rs:269-272) */
#define USN_R_WINDOW 7u    /* device: L4 ports lie beyond usn_batch.window; usn_finalize resolves
                              the frame from the host frame reader (usn_set_frame_reader) */
#define USN_F_CACHE (1u << 24)   /* decision taken from the 1-entry cache (endpoint.rs:186-191) */
#define USN_F_FRAG1 (1u << 25)   /* first fragment: remembered in the fragment map */
#define USN_F_FRAGN (1u << 26)   /* later fragment: resolved through the fragment map */
#define USN_F_DHCP (1u << 27)    /* DHCP steering involved */
#define USN_F_HOST (1u << 28)    /* resolved by the ordered host stage (usn_finalize) */
#define USN_F_LEARN (1u << 29)   /* tx: this frame learned a MAC or an answer rule */
#define USN_DEC_CLASS(d) (((d) >> 16) & 0xFu)
#define USN_DEC_EP(d) ((d) & 0xFFFFu)
#define USN_DEC_REASON(d) (((d) >> 20) & 0xFu)
#define USN_PARITY_MASK 0x00FFFFFFu

/* ---- endpoints (all_devices entries; devices.rs:14-25) ------------------ */
#define USN_EP_NIC 0   /* NicNetmap / NicMacVtap: get_nic().is_some() */
#define USN_EP_HOST 1  /* HostRing / HostTap */
#define USN_EP_PIPE 2  /* UserNetmap */
#define USN_EP_UDS 3   /* UserUnixDomainSocket */

/* ---- rule key: Want (pkt.rs:220-227) ------------------------------------ */
#define USN_WANT_DPORT 1u  /* dst_port is Some */
#define USN_WANT_SRC 2u    /* src_addr is Some */
#define USN_WANT_SPORT 4u  /* src_port is Some */
typedef struct {
  uint32_t dst_addr;   /* IPv4 a.b.c.d as (a<<24)|(b<<16)|(c<<8)|d */
  uint32_t src_addr;
  uint16_t dst_port;
  uint16_t src_port;
  uint8_t protocol;
  uint8_t present;     /* USN_WANT_* bits; absent fields are ignored */
  uint16_t _reserved;
} usn_want;

/* ---- batch of frames (one drained rx ring of one source endpoint) -------- */
typedef struct {
  const uint8_t *frames;   /* device: frame i starts at frames + i*stride or frames + offsets[i];
                              16-byte aligned, `window` readable bytes of frame i at every start */
  uint64_t stride;         /* > 0 selects the fixed-stride layout (netmap-slot like) */
  const uint64_t *offsets; /* device, or NULL when stride > 0 */
  const uint16_t *lens;    /* device: frame lengths (netmap_slot.len) */
  uint64_t n;              /* frames in the batch */
  uint16_t src_endpoint;   /* the endpoint whose ring was drained */
  uint16_t window;         /* bytes of frame i readable at its start, >= USN_WINDOW (0 means
                              USN_WINDOW); with a stride, window <= stride.  A frame whose ports
                              lie past the window (IPv4 with IHL >= 12 at window 64: pkt.rs:177-186
                              reads 14+hl .. 18+hl) is never read past it: the kernel flags it
                              USN_R_WINDOW | USN_F_HOST and usn_finalize resolves it from the host
                              frame reader.  window >= USN_WINDOW_MAX never needs the reader. */
  uint16_t _reserved[2];
} usn_batch;

/* Tile header: one per USN_TILE frames (written by the tile's workgroup only,
 * so no device-wide atomics and no per-batch memset are needed). */
typedef struct {
  uint16_t n_frames;       /* frames in this tile */
  uint16_t _r0;
  uint16_t n_host;         /* frames of this tile listed for the ordered host stage */
  uint16_t bin_nic;        /* = usn_summary.n_ep: the bin of Target::Nic (see usn_result.index) */
  uint16_t class_count[4]; /* frames per decision class (before host fix-ups) */
  uint32_t last_state;     /* internal: 1-entry cache state after this tile */
  uint32_t last_dst;
  uint32_t last_idx;
  uint32_t last_info[4];
  uint32_t _pad;
} usn_tile_hdr;            /* 48 bytes */

/* Batch summary (device), written by workgroup 0 and by usn_finalize. */
typedef struct {
  uint32_t flags;          /* USN_S_* */
  uint32_t first_break;    /* stale mode: first frame that ends the stale prefix */
  uint32_t n_frames;
  uint32_t n_tiles;
  uint32_t cin_state, cin_dst, cin_info[4];   /* carried-in cache as resolved on device */
  uint32_t cout_state, cout_dst, cout_info[4];/* carried-out override (finalize) */
  uint32_t n_ep;           /* endpoint bins of usn_result.index: bins 0..n_ep-1 are endpoint ids,
                              n_ep = NIC, n_ep+1 = FLOOD, n_ep+2 = DROP */
  uint32_t n_bins;         /* n_ep + 3: usn_result.bin_off has n_bins + 1 entries */
  uint32_t host_epoch;     /* internal: the launch tag of the last classify whose tiles listed
                              frames for the ordered host stage */
  uint32_t _pad;
} usn_summary;             /* 80 bytes */
#define USN_S_STALE 1u         /* carried cache entry disagrees with the current table */
#define USN_S_STALE_EXTENDS 2u /* stale prefix may continue past tile 0 */
#define USN_S_COUT 8u          /* cout_* is authoritative (set by finalize) */

/* Result buffers (device), carved by usn_result_bind from one allocation.
 *
 * The per-endpoint output (SURVEY §2 scatter_by_endpoint; the reference
 * writes each frame straight into its target's ring, endpoint.rs:61-74, and
 * copies FLOOD frames to every other endpoint, :340-363): `index` holds the
 * batch's frame indices grouped by bin and in frame order within each bin,
 * bin b's frames at index[bin_off[b] .. bin_off[b+1]).  Bins are the
 * endpoint ids 0..n_ep-1, then NIC (Target::Nic, the source's NIC), FLOOD
 * (mirror_to_all: every endpoint but the source) and DROP; n_ep and n_bins
 * are in the summary.  An endpoint receives its own list merged in frame
 * order with the FLOOD list.  Both are final after usn_classify (stream
 * order), and again after usn_finalize where the host stage patched
 * decisions. */
typedef struct {
  uint32_t *decisions;     /* n decision words */
  uint32_t *index;         /* n: frame indices grouped by bin, stable */
  uint32_t *bin_off;       /* USN_MAX_BINS + 1: bin b = index[bin_off[b] .. bin_off[b+1]) */
  usn_tile_hdr *tiles;     /* ceil(n / USN_TILE) */
  usn_summary *summary;    /* 1 */
  uint32_t *host_list;     /* per tile USN_TILE slots: frames for the ordered host stage */
  void *scratch;           /* device scratch of the per-endpoint scatter (per-tile bin counts
                              and list offsets) */
  uint64_t n;
  uint32_t max_bins;       /* bins the scratch holds (a batch with more endpoints: USN_ERANGE) */
  uint32_t bind_tag;       /* internal: distinct per usn_result_bind call (the scratch's state
                              is re-initialised on the first classify after a bind) */
} usn_result;
#define USN_MAX_BINS (USN_MAX_ENDPOINTS + 3)

/* Per-batch outcome of the ordered host stage. */
typedef struct {
  uint32_t n_host;         /* frames resolved on the host */
  uint32_t n_patched;      /* decisions changed by the host stage */
  uint32_t n_learned;      /* tx: MACs + answer rules learned */
  uint32_t flags;          /* summary flags seen */
  uint32_t class_count[4]; /* final per-class frame counts */
} usn_finalize_info;

/* ---- context --------------------------------------------------------------- */
typedef struct usn_ctx usn_ctx;

int usn_abi_version(void);
const char *usn_strerror(int status);
int usn_last_hip_error(void);

/* Binds to HIP device `hip_device` (must be gfx950).  Replaces the daemon
 * state set up in main() (main.rs:447-449: fragmentation_map, match_register,
 * innerl2bridge).  USN_HOST_ONLY gives a registry-only context for a control
 * plane without a GPU: every device entry point (classify, finalize,
 * plumbing) then returns USN_ENODEV -- there is no CPU classify path. */
#define USN_HOST_ONLY (-1)
int usn_ctx_create(int hip_device, usn_ctx **out);
void usn_ctx_destroy(usn_ctx *ctx);

/* ---- several GPUs behind one registry (replicas only) -------
 * One context, one match_register / bridge / fragment map / per-endpoint
 * state (the reference's single daemon, main.rs:447-449), and one device
 * replica of the rule image and bridge set per entry of hip_devices (the same
 * device may appear twice).  Every registry or bridge change -- AddMatch,
 * RemoveMatch, endpoint removal, usn_table_build / usn_bridge_set, and what a
 * tx batch learned (applied by its usn_finalize, endpoint.rs:194-253) -- bumps
 * the image version; a replica uploads the current version before its next
 * batch (the table-version fence), and while a tx batch awaits usn_finalize
 * every classify on every replica returns USN_EBUSY.  usn_classify /
 * usn_classify_multi and the device plumbing calls act on the selected
 * replica (0 after creation); usn_finalize finds the batch's replica itself.
 * A source whose batches move to another replica carries its decision cache
 * across through the host. */
#define USN_MAX_REPLICAS 16
int usn_ctx_create_group(const int *hip_devices, uint32_t n, usn_ctx **out);
int usn_ctx_replicas(usn_ctx *ctx);
int usn_replica_select(usn_ctx *ctx, uint32_t replica);
int usn_replica_device(usn_ctx *ctx, uint32_t replica);

/* Endpoints::add / EntryChange::Add (main.rs:151-166).  for_nic = -1 iff NIC. */
int usn_endpoint_add(usn_ctx *ctx, uint16_t id, int kind, int32_t for_nic);
/* EntryChange::Remove (main.rs:1058-1069): drops the endpoint and its rules.
 * Cached decisions that name it stay (as in the reference). */
int usn_endpoint_remove(usn_ctx *ctx, uint16_t id);

/* add_listening_match (main.rs:266-298): 1 inserted, 0 key exists ("ER"),
 * USN_EPERM owner is a NIC (the reference panics). Clears the owner's NIC
 * decision cache and records the listening triple.  The device image takes
 * the key in place before the next classify (a few slots, not a rebuild). */
int usn_add_match(usn_ctx *ctx, const usn_want *w, uint16_t owner, int sticky);
/* act_on RemoveMatch (main.rs:608-625): 1 removed, 0 absent, USN_EPERM if
 * requester is not the owner.  Does NOT clear any cache (as the reference). */
int usn_remove_match(usn_ctx *ctx, const usn_want *w, uint16_t requester);
/* QueryUsedPorts / introspection: number of rules, and a copy of them. */
int usn_rule_count(usn_ctx *ctx);
int usn_rules_get(usn_ctx *ctx, usn_want *w, uint16_t *owner, uint8_t *sticky, uint32_t cap);
/* Owner of an exact key, or USN_ENOENT. */
int usn_lookup(usn_ctx *ctx, const usn_want *w);

/* Bulk registry load (SURVEY §8b usn_table_build): replaces match_register
 * (main.rs:867) with `n` rules in one call -- e.g. a daemon restoring its
 * table.  Later duplicates of a key are ignored (HashMap::entry().or_insert).
 * Listening triples are not touched (only AddMatch records them); every NIC
 * decision cache is cleared.  Returns the number of rules in the registry. */
typedef struct {
  uint32_t dst_addr, src_addr;
  uint16_t dst_port, src_port;
  uint8_t protocol;
  uint8_t present;     /* USN_WANT_* bits | USN_RULE_STICKY */
  uint16_t endpoint;   /* owner */
} usn_rule;
#define USN_RULE_STICKY 0x80u
int usn_table_build(usn_ctx *ctx, const usn_rule *rules, uint32_t n);

/* ADD_MACS prefill (main.rs:450-462): appends to the inner L2 bridge. */
int usn_bridge_add(usn_ctx *ctx, const uint8_t mac[6]);
int usn_bridge_count(usn_ctx *ctx);
/* Replace the whole bridge with `n` MACs (SURVEY §8b usn_bridge_set). */
int usn_bridge_set(usn_ctx *ctx, const uint8_t (*macs)[6], uint32_t n);
/* 90 s cleanup: fragmentation_map.clear() (main.rs Cleanup handler). */
int usn_frag_clear(usn_ctx *ctx);

/* ---- the hot path ------------------------------------------------------------ */
/* Bytes of a result for n frames, sized for any endpoint count (USN_MAX_BINS:
 * about 24 bytes of scatter scratch per frame); usn_result_bytes_ep sizes it
 * for endpoint ids < max_endpoints (max id + 1; c5's 1002 endpoints: 6 bytes
 * per frame).  usn_result_bind carves a buffer of `bytes` and sets max_bins
 * from what the scratch holds. */
size_t usn_result_bytes(uint64_t n);
size_t usn_result_bytes_ep(uint64_t n, uint32_t max_endpoints);
int usn_result_bind(void *dev_mem, size_t bytes, uint64_t n, usn_result *out);
/* Drops what the context keeps per result (keyed by its arrays: the replica
 * and bins its last batch ran with, a side-stream lists event, the scan
 * scratch's zeroing tag) before the caller frees or re-binds its memory.  An
 * rx batch classified into it and not finalized is waited for first (its
 * launch's completion event, or the side-stream lists event), so nothing of
 * it still writes the memory when this returns.  A source whose carried
 * decision cache lives in this result's tile headers takes the cache to the
 * host first (it stays valid).  USN_EBUSY while the
 * result belongs to a tx batch not yet finalized.  Bind a result once per
 * allocation and reuse it: results are meant to be long-lived, and a context
 * whose caller never releases them keeps one small record per result. */
int usn_result_release(usn_ctx *ctx, const usn_result *r);

/* Classify one batch on `hip_stream` (hipStream_t; NULL = default stream).
 * Asynchronous: writes decisions, the per-endpoint lists (index, bin_off),
 * tile headers and the summary.
 * Consecutive batches of one source may be enqueued back to back; the 1-entry
 * decision cache is carried on the device from the previous batch's result,
 * which must stay allocated until this call's work has been enqueued.
 * A batch sent by a non-NIC endpoint (tx: find_forward with incoming ==
 * false) learns bridge MACs and answer rules; until its usn_finalize every
 * other call that reads or changes the registry returns USN_EBUSY, except
 * the source's next tx ring(s) on the same stream: at most two tx launches
 * (each one ring, or up to eight rings through usn_classify_multi) are in flight,
 * and their rings are finalized in order (a later one first: USN_EBUSY).
 * A launch ran against the state the launch before it started from; when a
 * usn_finalize of the earlier launch's rings changed that state (it learned,
 * or ran a host tail that left another carried cache or DHCP steering), the
 * later launch's rings are decided again on the host from their first
 * frame. */
int usn_classify(usn_ctx *ctx, const usn_batch *b, usn_result *r, void *hip_stream);
/* Several drained rings of DISTINCT sources (e.g. the rx queues of the NICs
 * polled in one poll() round, main.rs:1029-1046) in one launch: b[k] -> r[k],
 * count <= 8.  Same semantics as `count` usn_classify calls.
 * A sending endpoint's (tx) rings: one ring, or up to eight CONSECUTIVE rings
 * of the same source (count <= 8, distinct results) in one grid, each ring's
 * frames following the ring before's: the same decisions, learning and
 * carried cache as `count` usn_classify calls finalized in turn (ring k sees
 * what the rings before it learned on the device, and is decided again on the
 * host only when ring k - 1's usn_finalize ran a host tail or redid it).
 * Finalize the rings in order.  tx rings of different sources: USN_EINVAL.
 * The launch's frame index must fit 32 bits: the sum over rings k < count - 1
 * of ceil(n_k / USN_TILE) * USN_TILE, plus n of the last ring, must be below
 * 2^32 - 1, else USN_ERANGE. */
int usn_classify_multi(usn_ctx *ctx, const usn_batch *b, usn_result *r, uint32_t count,
                       void *hip_stream);

/* Per-endpoint lists on a side stream (off by default).  With on != 0,
 * usn_classify / usn_classify_multi of NIC rings enqueue the classify kernel
 * on the caller's stream and the scatter that builds index / bin_off on a
 * stream of the library's (one per replica), ordered after it: the caller's
 * stream does not wait for the lists, so the next batch's classify overlaps
 * this batch's scatter.  Decisions, tile headers and the summary stay in the
 * caller's stream order.  The lists are final when usn_finalize returns (it
 * waits for them), or in the order of `hip_stream` after usn_lists_wait.  A
 * result is not overwritten by a later classify before its lists are done.
 * tx batches (learning) always build their lists on the caller's stream. */
int usn_set_lists_async(usn_ctx *ctx, int on);
int usn_lists_wait(usn_ctx *ctx, const usn_result *r, void *hip_stream);

/* Ordered host stage for one classified batch.  Waits for the batch's own
 * launches, not for work queued behind them on the stream (a NIC batch whose
 * lists are built on the side stream: for the stream and its lists); for a
 * tx batch `hip_stream` must be the stream the batch was classified on (else
 * USN_EINVAL).  When the batch needs the host stage, its copies and patches
 * are ordered on `hip_stream` and the call returns after them.  A NIC batch
 * with nothing for the host stage (no stale carried cache, no frame listed)
 * reads only the few words its scatter left in host-mapped memory: about one
 * microsecond of host time.
 * Resolves fragments, DHCP steering, stale cache prefixes and tx learning in
 * frame order and patches decisions and the per-endpoint lists on the device.  Must be called
 * before the next usn_classify of the same source whenever the summary has
 * n_host > 0 or flags != 0; calling it always is allowed.  The batch's
 * index / bin_off are not valid when it returns USN_ELIST (the scatter found
 * a decision naming a bin past the batch's bins, or per-tile counts that
 * disagree with the decisions) or USN_EHIP with usn_last_hip_error() ==
 * hipErrorLaunchTimeOut (702: the device gave up waiting inside the lists'
 * scan, bounded at 200 ms); neither has been observed outside the test hook
 * that forces them.  The batch keeps the bins it was classified with
 * (summary n_bins) when endpoints were added since; only a host-stage
 * decision naming such an endpoint rebuilds its lists with today's bins
 * (summary n_ep / n_bins updated).  USN_ERANGE, before any side effect: the
 * batch needs the host stage and today's bins exceed the result's max_bins
 * (a result sized by usn_result_bytes_ep for fewer endpoints than the context
 * has by then).  This is decided before the host stage runs, so it holds even
 * when no resolved decision would name a new endpoint; the batch cannot be
 * finalized into that result -- classify the ring again into a result sized
 * by usn_result_bytes (any endpoint count never gets USN_ERANGE). */
int usn_finalize(usn_ctx *ctx, const usn_batch *b, usn_result *r, void *hip_stream,
                 usn_finalize_info *info);

/* Host frame reader for frames whose ports lie past usn_batch.window: copies
 * up to `cap` bytes (cap >= USN_WINDOW_MAX) of frame `index` of the batch of
 * `src_endpoint` being finalized into `out`, returns the bytes copied (the
 * frame length when shorter) or a negative value on failure.  Called only
 * from usn_finalize, on the calling thread.  Without a reader, usn_finalize
 * of a batch holding such frames returns USN_EINVAL before any side effect
 * (their decisions stay USN_R_WINDOW drops).  NULL fn unregisters. */
typedef int (*usn_frame_reader)(void *user, uint16_t src_endpoint, uint64_t index, uint8_t *out,
                                uint32_t cap);
int usn_set_frame_reader(usn_ctx *ctx, usn_frame_reader fn, void *user);

/* Forget the carried decision cache of one endpoint (last_pkt = None). */
int usn_cache_clear(usn_ctx *ctx, uint16_t endpoint);

/* ---- device plumbing for hosts without their own HIP bindings -------------------- */
int usn_dev_alloc(usn_ctx *ctx, size_t bytes, void **dev);
int usn_dev_free(usn_ctx *ctx, void *dev);
int usn_host_alloc_pinned(usn_ctx *ctx, size_t bytes, void **host);
int usn_host_free_pinned(usn_ctx *ctx, void *host);
int usn_memcpy_h2d(usn_ctx *ctx, void *dev, const void *host, size_t bytes, void *hip_stream);
int usn_memcpy_d2h(usn_ctx *ctx, void *host, const void *dev, size_t bytes, void *hip_stream);
int usn_memset_d(usn_ctx *ctx, void *dev, int value, size_t bytes, void *hip_stream);
int usn_stream_create(usn_ctx *ctx, void **stream);
int usn_stream_destroy(usn_ctx *ctx, void *stream);
int usn_stream_sync(usn_ctx *ctx, void *stream);
int usn_device_sync(usn_ctx *ctx);
/* Events: elapsed milliseconds between two recorded events. */
int usn_event_create(usn_ctx *ctx, void **ev);
int usn_event_destroy(usn_ctx *ctx, void *ev);
int usn_event_record(usn_ctx *ctx, void *ev, void *hip_stream);
int usn_event_elapsed_ms(usn_ctx *ctx, void *ev_start, void *ev_end, float *ms);
/* Make `hip_stream` wait (on the device) for an event recorded on another stream. */
int usn_stream_wait_event(usn_ctx *ctx, void *hip_stream, void *ev);

#ifdef __cplusplus
}
#endif
#endif /* USN_CLASSIFY_H */
