/*
 * usn_host.cpp -- C ABI implementation: context, rule registry, device table
 * build, batch launch and the ordered host stage (usn_finalize).
 *
 * State model (all from /root/reference):
 *   match_register  HashMap<Want, (bool sticky, Rc<endpoint>)>   main.rs:448
 *   innerl2bridge   Vec<EthernetAddress>                         main.rs:449
 *   fragmentation_map HashMap<FragmentationKey, (PacketInfo,..)> main.rs:447
 *   Endpoint { listening, next_dhcp_endpoint, last_pkt, last_pkt_dst, for_nic }
 *                                                                endpoint.rs:19-29
 * The device sees an immutable snapshot of match_register (rebuilt when the
 * registry changes) and the bridge; the 1-entry decision cache of each source
 * is carried on the device from batch to batch (see usn_device.hip).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <deque>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <random>
#include <atomic>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "usn_internal.h"
#include "usn_kernels.h"

using usn::ClassifyArgs;

/* perfect-hash image geometry: slot load and keys per displacement group.
 * 10 keys per u16 displacement keep c5's two arrays (65536 keys) at 13 KiB,
 * which the classify kernel stages in LDS at 4 workgroups per CU.
 * A/B, c5, 8M frames per launch: group 8 / load 0.85 with the displacements
 * in global memory 174.2 us, the same in LDS (3 workgroups per CU) 161.3 us,
 * group 10 / load 0.75 in LDS 156.5 us (profiles/r02d).  The slot load then
 * went from 0.75 to 0.65: the kernel does not notice (c5 157.0 vs 158.1 us,
 * c4 160.9 vs 162.5), and placement takes a third of the time (a group of s
 * keys needs ~1/(1-fill)^s trials): 1.19M rules rebuilt in 83 instead of
 * 155 ms (profiles/r02g).  Round 3: 0.5, so that a key inserted in place
 * (AddMatch between full builds, refresh_image) finds a free slot under its
 * group's displacement half the time and its group a new displacement
 * almost always; a table is rebuilt once its keys pass IMG_MAX_LOAD. */
#ifndef USN_PH_LOAD
#define USN_PH_LOAD 0.5
#endif
#ifndef USN_PH_GROUP
#define USN_PH_GROUP 10
#endif

namespace {

thread_local int g_last_hip = 0;

int hip_fail(hipError_t e) {
  g_last_hip = (int)e;
  return USN_EHIP;
}
#define HIPCHK(x)                              \
  do {                                         \
    hipError_t _e = (x);                       \
    if (_e != hipSuccess) return hip_fail(_e); \
  } while (0)

struct WantKey {
  uint32_t dst, src;
  uint16_t dport, sport;
  uint8_t proto, present;
  bool operator==(const WantKey &o) const {
    return dst == o.dst && src == o.src && dport == o.dport && sport == o.sport &&
           proto == o.proto && present == o.present;
  }
};
struct WantHash {
  size_t operator()(const WantKey &k) const {
    return usn_key_hash(k.dst, k.src, (uint32_t)k.dport | ((uint32_t)k.sport << 16),
                        usn_key_meta(k.proto, k.present));
  }
};
/* canonical key: absent Option fields are zero (derive(Hash, Eq) on Want) */
WantKey canon(const usn_want &w) {
  WantKey k;
  k.present = w.present & 7u;
  k.dst = w.dst_addr;
  k.proto = w.protocol;
  k.dport = (k.present & USN_WANT_DPORT) ? w.dst_port : 0;
  k.src = (k.present & USN_WANT_SRC) ? w.src_addr : 0;
  k.sport = (k.present & USN_WANT_SPORT) ? w.src_port : 0;
  return k;
}

struct Rule {
  uint16_t owner;
  uint8_t sticky;
};

/* match_register (main.rs:867, a hashbrown HashMap<Want, (usize, bool)>):
 * open addressing with linear probing over one flat array.  A tx batch can
 * learn ~10^5 answer rules at once; node-per-entry std::unordered_map spent
 * most of usn_finalize on those inserts.  Erase leaves a tombstone, so an
 * iterator stays valid across erase (match_register.retain). */
class RuleMap {
 public:
  struct value_type {   // the slot state shares the key's cache line
    WantKey first;
    Rule second;
    uint8_t state;
  };
  /* the flat slot array, from calloc: all-zero bytes are EMPTY slots, so a
   * new table of 10^7 slots costs no fill pass, and its pages are first
   * touched by the (parallel) inserts of a rehash */
  struct Slots {
    value_type *p = nullptr;
    size_t n = 0;
    Slots() = default;
    Slots(const Slots &) = delete;
    Slots &operator=(const Slots &) = delete;
    ~Slots() { std::free(p); }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    value_type &operator[](size_t i) const { return p[i]; }
    value_type *begin() const { return p; }
    value_type *end() const { return p + n; }
    void swap(Slots &o) { std::swap(p, o.p); std::swap(n, o.n); }
    bool zeroed(size_t cap) {
      value_type *q = static_cast<value_type *>(std::calloc(cap, sizeof(value_type)));
      if (!q) return false;
      std::free(p);
      p = q;
      n = cap;
      return true;
    }
  };
  class iterator {
   public:
    iterator(RuleMap *m, size_t i) : m_(m), i_(i) { skip(); }
    value_type &operator*() const { return m_->slot_[i_]; }
    value_type *operator->() const { return &m_->slot_[i_]; }
    iterator &operator++() { ++i_; skip(); return *this; }
    bool operator==(const iterator &o) const { return i_ == o.i_; }
    bool operator!=(const iterator &o) const { return i_ != o.i_; }

   private:
    friend class RuleMap;
    void skip() { while (i_ < m_->slot_.size() && m_->slot_[i_].state != FULL) ++i_; }
    RuleMap *m_;
    size_t i_;
  };
  using const_iterator = iterator;

  size_t size() const { return n_; }
  /* slot i of the flat array (0 <= i < slots()), or nullptr when it holds no
   * entry: lets a scan of the map be split over threads */
  size_t slots() const { return slot_.size(); }
  const value_type *at_slot(size_t i) const { return slot_[i].state == FULL ? &slot_[i] : nullptr; }
  iterator begin() const { return iterator(self(), 0); }
  iterator end() const { return iterator(self(), slot_.size()); }
  void clear() { for (value_type &v : slot_) v.state = EMPTY; n_ = used_ = 0; }
  void reserve(size_t n) { if (2 * n > slot_.size()) rehash(n); }
  iterator find(const WantKey &k) const {
    const size_t i = locate(k);
    return i == NPOS ? end() : iterator(self(), i);
  }
  size_t count(const WantKey &k) const { return locate(k) != NPOS; }
  void prefetch(const WantKey &k) const {
    if (!slot_.empty()) __builtin_prefetch(&slot_[WantHash()(k) & mask()]);
  }
  Rule &operator[](const WantKey &k) { return slot_[insert_slot(k, Rule{0, 0})].second; }
  bool emplace(const WantKey &k, Rule r) {
    const size_t before = n_;
    const size_t i = insert_slot(k, r);
    (void)i;
    return n_ != before;
  }
  iterator erase(iterator it) {
    slot_[it.i_].state = TOMB;
    --n_;
    return iterator(this, it.i_ + 1);
  }

 private:
  static constexpr uint8_t EMPTY = 0, FULL = 1, TOMB = 2;
  static constexpr size_t NPOS = ~(size_t)0;
  RuleMap *self() const { return const_cast<RuleMap *>(this); }
  size_t mask() const { return slot_.size() - 1; }
  size_t locate(const WantKey &k) const {
    if (slot_.empty()) return NPOS;
    for (size_t i = WantHash()(k) & mask();; i = (i + 1) & mask()) {
      if (slot_[i].state == EMPTY) return NPOS;
      if (slot_[i].state == FULL && slot_[i].first == k) return i;
    }
  }
  /* slot of k, inserting (k, r) when absent; load (entries + tombstones) <= 1/2 */
  size_t insert_slot(const WantKey &k, Rule r) {
    if (2 * (used_ + 1) > slot_.size()) rehash(n_ + 1);
    size_t tomb = NPOS;
    for (size_t i = WantHash()(k) & mask();; i = (i + 1) & mask()) {
      if (slot_[i].state == FULL) {
        if (slot_[i].first == k) return i;
      } else if (slot_[i].state == TOMB) {
        if (tomb == NPOS) tomb = i;
      } else {
        if (tomb != NPOS) i = tomb;
        else ++used_;
        slot_[i] = value_type{k, r, FULL};
        ++n_;
        return i;
      }
    }
  }
  void rehash(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 2) cap <<= 1;
    static_assert(EMPTY == 0, "calloc'd slots are EMPTY");
    Slots fresh;
    if (!fresh.zeroed(cap)) throw std::bad_alloc();   // the map is unchanged then
    Slots old_slot;
    old_slot.swap(slot_);
    slot_.swap(fresh);
    const size_t old_n = n_;
    n_ = used_ = 0;
    if (old_n >= (1u << 18) && rehash_parallel(old_slot)) return;
    for (size_t i = 0; i < old_slot.size(); ++i) {
      if (i + 16 < old_slot.size() && old_slot[i + 16].state == FULL)
        __builtin_prefetch(&slot_[WantHash()(old_slot[i + 16].first) & mask()], 1);
      const value_type &v = old_slot[i];
      if (v.state == FULL) {
        size_t j = WantHash()(v.first) & mask();
        while (slot_[j].state != EMPTY) j = (j + 1) & mask();
        slot_[j] = v;
        ++n_;
        ++used_;
      }
    }
  }
  /* Large tables (a tx batch learning 10^5 answer rules grows the registry
   * past a power of two): the entries are grouped by the region of the new
   * table their home slot lies in, and the regions are filled by parallel
   * threads; a probe never leaves its region there (an entry that would is
   * set aside), so the threads write disjoint slots.  The set-aside entries
   * are inserted afterwards, in order, with wrap-around: every entry then
   * sits at the first empty slot of its probe sequence, as linear probing
   * requires.  1.2 M entries: 41 ms sequential (random DRAM writes).  False
   * when the host has one thread. */
  bool rehash_parallel(const Slots &old_slot) {
    const uint32_t T = std::min(16u, std::thread::hardware_concurrency());
    if (T < 2) return false;
    const size_t cap = slot_.size(), NO = old_slot.size();
    uint32_t lr = 0;   // log2 of the regions: 8 per thread
    while ((1u << lr) < 8 * T && (cap >> (lr + 1)) >= 4096) ++lr;
    const uint32_t R = 1u << lr;
    uint32_t lcap = 0;
    while ((size_t(1) << lcap) < cap) ++lcap;
    auto region = [&](size_t home) { return (uint32_t)(home >> (lcap - lr)); };
    std::vector<size_t> cnt((size_t)T * R, 0);
    auto chunk = [&](uint32_t t, size_t &lo, size_t &hi) { lo = NO * t / T; hi = NO * (t + 1) / T; };
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < T; ++t)
      pool.emplace_back([&, t] {
        // first touch of the new (calloc'd) table: each thread its slice, in order
        const size_t a = cap * t / T, b = cap * (t + 1) / T;
        std::memset(static_cast<void *>(&slot_[a]), 0, (b - a) * sizeof(value_type));
        size_t lo, hi;
        chunk(t, lo, hi);
        size_t *c = cnt.data() + (size_t)t * R;
        for (size_t i = lo; i < hi; ++i)
          if (old_slot[i].state == FULL) c[region(WantHash()(old_slot[i].first) & mask())]++;
      });
    for (std::thread &th : pool) th.join();
    pool.clear();
    std::vector<size_t> rstart(R + 1, 0);
    size_t run = 0;
    for (uint32_t r = 0; r < R; ++r) {
      rstart[r] = run;
      for (uint32_t t = 0; t < T; ++t) {
        const size_t v = cnt[(size_t)t * R + r];
        cnt[(size_t)t * R + r] = run;
        run += v;
      }
    }
    rstart[R] = run;
    std::vector<uint32_t> idx(run);   // old slots, region after region
    for (uint32_t t = 0; t < T; ++t)
      pool.emplace_back([&, t] {
        size_t lo, hi;
        chunk(t, lo, hi);
        size_t *c = cnt.data() + (size_t)t * R;
        for (size_t i = lo; i < hi; ++i)
          if (old_slot[i].state == FULL) idx[c[region(WantHash()(old_slot[i].first) & mask())]++] = (uint32_t)i;
      });
    for (std::thread &th : pool) th.join();
    pool.clear();
    std::vector<std::vector<uint32_t>> spill(T);
    std::vector<size_t> placed(T, 0);
    const size_t rsz = cap >> lr;
    for (uint32_t t = 0; t < T; ++t)
      pool.emplace_back([&, t] {
        for (uint32_t r = t; r < R; r += T) {
          const size_t end = (size_t)(r + 1) * rsz;
          for (size_t k = rstart[r]; k < rstart[r + 1]; ++k) {
            const value_type &v = old_slot[idx[k]];
            size_t j = WantHash()(v.first) & mask();
            while (j < end && slot_[j].state != EMPTY) ++j;
            if (j == end) { spill[t].push_back(idx[k]); continue; }
            slot_[j] = v;
            placed[t]++;
          }
        }
      });
    for (std::thread &th : pool) th.join();
    for (uint32_t t = 0; t < T; ++t) n_ += placed[t];
    used_ = n_;
    for (const std::vector<uint32_t> &sp : spill)
      for (uint32_t i : sp) {
        const value_type &v = old_slot[i];
        size_t j = WantHash()(v.first) & mask();
        while (slot_[j].state != EMPTY) j = (j + 1) & mask();
        slot_[j] = v;
        ++n_;
        ++used_;
      }
    return true;
  }
  Slots slot_;
  size_t n_ = 0, used_ = 0;   // entries; entries + tombstones
};

struct Listen {
  uint32_t dst;
  uint8_t proto, has_port;
  uint16_t port;
};

struct Info {   // PacketInfo words (usn_internal.h)
  uint32_t w[4];
  bool operator==(const Info &o) const {
    return w[0] == o.w[0] && w[1] == o.w[1] && w[2] == o.w[2] && w[3] == o.w[3];
  }
  uint32_t kind() const { return w[0] & 0xFFu; }
  uint32_t proto() const { return (w[0] >> 8) & 0xFFu; }
  bool has_ports() const { return (w[0] >> 16) & 1u; }
  uint32_t src() const { return w[1]; }
  uint32_t dst() const { return w[2]; }
  uint32_t sport() const { return w[3] & 0xFFFFu; }
  uint32_t dport() const { return w[3] >> 16; }
};

struct FragKey {
  uint16_t id;
  uint8_t proto;
  uint32_t src, dst;
  uint64_t smac, dmac;
  bool operator==(const FragKey &o) const {
    return id == o.id && proto == o.proto && src == o.src && dst == o.dst && smac == o.smac &&
           dmac == o.dmac;
  }
};
struct FragHash {
  size_t operator()(const FragKey &k) const {
    uint64_t h = k.smac * 0x9E3779B97F4A7C15ull ^ (k.dmac + 0x632BE59BD9B4E019ull);
    h ^= ((uint64_t)k.src << 32 | k.dst) * 0xC2B2AE3D27D4EB4Full;
    h ^= ((uint64_t)k.id << 8 | k.proto) * 0x165667B19E3779F9ull;
    return (size_t)(h ^ (h >> 29));
  }
};
struct FragVal {
  Info info;
  uint64_t smac, dmac;
};

struct Ep {
  bool used = false;
  int kind = 0;
  int for_nic = -1;
  std::vector<Listen> listening;
  uint64_t listen_ver = 0;   // usn_ctx::listen_gen at the last change of `listening`
  int next_dhcp = -1;
};

/* carried decision cache of one source endpoint */
/* A/B and test knobs from the environment are read only by the test build
 * (USN_TEST_HOOKS=1: build/test/libusn.so, which tools/abl.py's variants
 * and the tests that force failures load).  The product library reads no
 * environment variable: test_knob is nullptr there for every name. */
#ifndef USN_TEST_HOOKS
#define USN_TEST_HOOKS 0
#endif
static const char *test_knob(const char *name) {
#if USN_TEST_HOOKS
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

/* host-time checkpoints of usn_classify_multi (test build only:
 * tools/hostprof.py reads them through usn_debug_host_prof) */
#if USN_TEST_HOOKS
uint64_t g_hprof[16];
inline uint64_t hprof_now() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define HPROF_DECL uint64_t hp_t_ = hprof_now();
#define HPROF(k) do { const uint64_t t_ = hprof_now(); g_hprof[k] += t_ - hp_t_; hp_t_ = t_; } while (0)
#else
#define HPROF_DECL
#define HPROF(k) do { } while (0)
#endif

struct Chain {
  bool device_chain = false;        // previous result on the device is authoritative
  uint32_t replica = 0;             // where the source's last batch was classified
  const usn_tile_hdr *tiles = nullptr;
  uint32_t ntiles = 0;
  const usn_summary *summary = nullptr;
  uint32_t state = 0, dst = 0;      // explicit state when !device_chain
  uint32_t info[4] = {0, 0, 0, 0};
  /* recorded on the stream of the source's last batch, one per replica
   * (created on that replica's device): chain_to_host waits for it before it
   * reads that batch's summary and tile headers */
  hipEvent_t done[USN_MAX_REPLICAS] = {};
};

struct ParsedH {   // host-side extract_pkt_info result
  int status;      // 0 fail (reason in `reason`), 1 ok
  uint32_t reason;
  Info info;
  uint64_t smac, dmac;
};

}  // namespace

/* One device copy of the shared state (a usn_ctx group has one per GPU):
 * the rule image and bridge set at the version it last uploaded, and the
 * device scratch of a tx batch classified on it. */
struct Replica {
  int device = 0;
  int n_cu = 0;
  uint4 *d_table = nullptr;
  size_t d_table_cap = 0;
  uint64_t table_version = 0;    // image version on the device (0 = none)
  void *d_patch = nullptr;       // an image patch: {values}{unit indices}
  size_t d_patch_cap = 0;
  uint64_t *d_bridge = nullptr;
  size_t d_bridge_cap = 0;
  unsigned long long *d_bridge_set = nullptr;   // open addressing, bit 63 = used
  size_t d_bridge_set_cap = 0;
  uint64_t bridge_version = 0;
  /* tx scratch.  Epoch-tagged (aux granules, the learning sets): shared by
   * the batches in flight.  What usn_finalize of a batch reads after the
   * next batch has launched (its counters, its learned list, its gathered
   * state) lives in one of two slots, alternating (usn_ctx::txq) */
  unsigned long long *aux = nullptr;   // TXA_GRANULES per tile, tagged with the epoch
  uint32_t aux_tiles = 0;
  unsigned long long *macset = nullptr, *ruleset = nullptr;
  uint32_t set_slots = 0;
  struct TxSlot {
    uint4 *learned = nullptr;
    uint64_t learned_frames = 0;
    uint32_t learned_cap = 0;
    uint32_t *counters = nullptr;       // TxArgs::counters
    hipEvent_t txstate_ev = nullptr;    // the batch's gathered state (usn_ctx::h_txstate) landed
  } txs[2];
  uint32_t *listen = nullptr;
  size_t listen_cap = 0;
  int listen_src = -1;           // the endpoint / version whose listening triples `listen` holds
  uint64_t listen_ver = 0;
  uint32_t epoch = 0;
  /* usn_set_lists_async: the scatter's stream, ordered after each classify
   * launch by the `classified` event */
  hipStream_t side = nullptr;
  hipEvent_t classified = nullptr;
  /* rx launches' completion (recorded after their scatter on the caller's
   * stream): usn_finalize of an rx batch waits for its own launch, not for
   * the later batches queued behind it.  A ring of events: a slot reused by
   * a later launch on the same stream only makes that wait longer; one
   * re-recorded on another stream no longer orders the batch's launch, so
   * each slot keeps the generation and stream of its last record (rx_wait) */
  static constexpr uint32_t RX_EVS = 64;
  hipEvent_t rx_ev[RX_EVS] = {};
  uint64_t rx_ev_gen[RX_EVS] = {};
  hipStream_t rx_ev_stream[RX_EVS] = {};
  // this device's addresses of the context's host-mapped rx / tx state
  // (hipHostGetDevicePointer once, not per call)
  uint32_t *d_rxstate = nullptr, *d_txstate = nullptr;
  uint32_t rx_ev_next = 0;
};

/* The completion events of rx and tx launches (usn_finalize waits for its
 * own launch on them).  An event between back-to-back launches of one stream
 * costs the next launch 1-2 % of a c5 call and 2-3 % of a c4 one (the A/B
 * harness, one stream: 160.3 -> 162.3 us per 8M ring, profiles/r05/r05w);
 * without the system-scope fence it is the same within noise (r05v), so the
 * events keep it (the host reads what they order: the launch's state words,
 * then the results through copies). */
#ifndef USN_BIND_MAX_TILES   /* 2M frames: c3's calls of 4 x 256K are bound, c2's 8 x 1M are not */
#define USN_BIND_MAX_TILES 2048u
#endif
#ifndef USN_DONE_EV_FLAGS
#define USN_DONE_EV_FLAGS hipEventDisableTiming
#endif
constexpr size_t TXSTATE_BYTES = USN_TX_RINGS * USN_TXS_WORDS * 4;   // a tx launch's gathered state per slot

struct usn_ctx {
  int device = 0;        // the selected replica's device (plumbing calls)
  uint32_t sel = 0;      // selected replica (usn_replica_select)
  int t512 = -1;   // USN_T512 env (A/B): -1 by table size, 0 never, 1 always
  /* launch completion (A/B, test build: USN_RX_EV 0 none for rx --
   * usn_finalize syncs the stream --, 1 recorded behind the scatter, 2 the
   * same without the system-scope fence, 3 with a device-scope release, 4
   * bound to the scatter's dispatch, 5 bound for launches of at most
   * USN_BIND_MAX_TILES tiles, else recorded (the product's); USN_RX_STATE=0: no host-mapped state gather, the
   * finalize reads summary and tile headers), and usn_event_create's flags
   * (USN_TIMING_EV: 0 default, 1 device-scope release, 2 no system fence) */
  int rx_ev_mode = 5;
  bool rx_state_on = true;
  unsigned timing_ev_flags = hipEventDefault;
  int tx512 = 1;   // USN_TX_T512 env (A/B): the tx kernel at 512 threads per tile (c4tx 1M:
                   // 51.2 vs 53.2 us at 256; two rounds per lane, 64 VGPRs, 4 workgroups per CU)
  double ph_load = USN_PH_LOAD;   // perfect-hash image geometry (env knobs)
  uint32_t ph_group = USN_PH_GROUP;
  std::mutex mu;
  std::vector<Ep> eps = std::vector<Ep>(USN_MAX_ENDPOINTS);
  uint32_t n_ep = 0;   // max id + 1
  RuleMap rules;
  std::vector<uint64_t> bridge;
  std::unordered_map<FragKey, FragVal, FragHash> frags;
  std::vector<Chain> chains = std::vector<Chain>(USN_MAX_ENDPOINTS);
  std::vector<Replica> reps;
  /* host image of the device rule table (perfect hash, usn_internal.h),
   * rebuilt from the registry when it changed; every replica uploads the
   * current version before its next batch (the table-version fence) */
  bool table_dirty = true;
  uint64_t table_version = 0;
  std::vector<uint4> img;          // the whole image in 16-byte units
  usn_ph_table img_t[4] = {};  // K1, K2, U, X (usn_internal.h)
  uint32_t img_base = 0;       // units of the K1/K2 part; U and X follow
  uint32_t img_udisp = 0;      // first unit of U's and X's displacements
  uint32_t probe_mask = 0;   // tables holding rules (ClassifyArgs::probe_mask)
  bool proj = test_knob("USN_NO_PROJ") == nullptr;   // A/B: build U and X
  /* incremental image updates between full builds (AddMatch / RemoveMatch /
   * a few learned rules): the registry keys changed since the image was last
   * brought up to date, each table's displacement groups (slot indices from
   * the table's first slot; built on first use after a full build), its
   * keys, and the 16-byte units patched since the last full build, with the
   * image version that patched them (what a replica uploads) */
  bool incremental = test_knob("USN_IMG_FULL") == nullptr;   // A/B: every change rebuilds
  std::vector<WantKey> img_delta;
  bool img_groups_ok = false;
  std::vector<std::vector<uint32_t>> img_groups[4];
  uint32_t img_nkeys[4] = {0, 0, 0, 0};
  double img_load01 = USN_PH_LOAD;   // slot load K1 / K2 were built at
  uint64_t img_full_version = 0;
  std::vector<std::pair<uint64_t, uint32_t>> img_patches;
  uint64_t img_builds = 0, img_updates = 0;   // full builds / incremental updates (diagnostics)
  bool bridge_dirty = true;
  uint64_t bridge_version = 0;
  std::vector<unsigned long long> bridge_set;
  uint32_t bridge_mask = 0;
  /* tx batches in flight: classified, not finalized, so the registry is not
   * final (every registry call returns USN_EBUSY).  At most two launches
   * (each one ring, or up to USN_TX_RINGS consecutive rings in one grid), of one source, on
   * one stream and replica: launch k + 1 may be enqueued before launch k's
   * rings are finalized (the device is not left idle while the host
   * finalizes).  Launch k + 1 ran against the state launch k started from;
   * when a finalize of launch k's rings changed that state (it learned, or
   * ran a host tail), launch k + 1's first ring is decided again on the host
   * from its first frame (tx_redo_next).  Ring k of a launch saw ring k - 1's
   * learning on the device: it is redone only after ring k - 1 ran a host
   * tail (or was redone). */
  struct Tx {
    const uint32_t *decisions = nullptr;
    const void *launch_dec = nullptr;   // ring 0's decisions (usn_ctx::txstate_for)
    int src = -1;
    uint32_t replica = 0, slot = 0, epoch = 0;
    uint32_t ring = 0, rings = 1;       // this ring of the launch's
    uint32_t voff = 0;                  // the launch's frame index of the ring's frame 0
    uint64_t launch = 0;
    hipStream_t stream = nullptr;
  };
  std::deque<Tx> txq;
  uint32_t tx_next_slot = 0;
  uint64_t tx_launches = 0;
  bool tx_chg = false;           // a finalize changed the state since the latest tx launch
  bool tx_redo_next = false;     // the next batch in txq is redone on the host from frame 0
  bool tx_cout_valid = false;    // ... from this carried cache (the previous batch's host tail)
  uint32_t tx_cout[6] = {0, 0, 0, 0, 0, 0};   // {state, dst, info[4]}
  /* pinned staging for usn_finalize's small reads (summary, tile headers,
   * tx counters): async copies and one stream sync instead of three
   * synchronous pageable copies */
  uint8_t *h_stage = nullptr;
  size_t h_stage_cap = 0;
  uint8_t *h_patch = nullptr;    // pinned: an image patch (upload_table)
  size_t h_patch_cap = 0;
  uint32_t *h_lists = nullptr;   // pinned: the host lists of a batch with many listed tiles
  size_t h_lists_cap = 0;
  uint4 *h_items = nullptr;      // pinned: a tx batch's learned list
  size_t h_items_cap = 0;
  uint64_t h_items_for = 0;      // the launch whose list h_items holds (every ring reads it)
  /* host frame reader: frames whose ports lie past the batch window */
  usn_frame_reader reader = nullptr;
  void *reader_user = nullptr;
  /* the replica each classified result (keyed by its decisions array) was
   * classified on: usn_finalize acts on the batch's own replica, not on the
   * replica of the source's latest batch */
  /* per classified batch (by its decisions): the replica it ran on and its
   * bin count (endpoints can be added before its usn_finalize: the batch's
   * scratch, count rows and lists keep the bins it was classified with) */
  struct BatchRec {
    uint32_t rep, nbins;
    uint32_t slot, epoch;   // its rx state slot (RX_SLOTS: none) and launch tag
    hipEvent_t done;        // rx: recorded after its launch's scatter (Replica::rx_ev), or null
    uint32_t ev_idx;        // ... its slot in Replica::rx_ev
    uint64_t ev_gen;        // ... and the record's generation (rx_wait)
    hipStream_t stream;     // the stream the launch ran on
  };
  std::unordered_map<const void *, BatchRec> batch_rep;
  uint64_t rx_ev_gen = 0;   // Replica::rx_ev records so far (their generations)
  /* usn_set_lists_async: lists built on the replica's side stream; each
   * result's `lists done` event (keyed by its decisions array, created on
   * its replica's device) */
  bool lists_async = false;
  struct ListsEv { hipEvent_t ev = nullptr; int device = -1; bool pending = false; };
  std::unordered_map<const void *, ListsEv> lists_ev;
  /* the scatter's scan: a tag per launch for its range granules (random
   * start), and the result scratches whose granules were zeroed */
  uint32_t scan_epoch = (uint32_t)std::random_device{}();
  /* per scratch: the bind tag and geometry (frames, bins) its granules were
   * last zeroed for (one entry per scratch, not per geometry) */
  struct Zeroed { uint32_t tag; uint64_t geo; };
  std::unordered_map<const void *, Zeroed> scan_zeroed;
  uint64_t listen_gen = 0;   // Ep::listen_ver source
  /* a tx batch's summary flags, counters and class totals, written into
   * host-mapped memory by the scatter's first chunk (usn_finalize of a
   * batch that learned nothing reads only these) */
  uint8_t *h_txstate = nullptr;      // 2 slots x TXSTATE_BYTES
  size_t h_txstate_cap = 0;
  const void *txstate_for[2] = {nullptr, nullptr};   // the result (decisions) each slot holds
  /* an rx batch's state for usn_finalize (ScatterBatch::rx_state), written
   * by its scatter into host-mapped memory: RX_SLOTS slots of 8 words, dealt
   * round-robin to the batches of each classify call (BatchRec::slot) */
  static constexpr uint32_t RX_SLOTS = 1024;
  uint32_t *h_rxstate = nullptr;
  uint32_t rx_next_slot = 0;
};

namespace {

uint32_t next_pow2(uint32_t v) {
  uint32_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

/* Which table of the device image a registry key belongs to: key1
 * (to_match_want_with_src(true), pkt.rs:96-113) always has src and both
 * ports or neither -> K1; key2 has neither src nor src_port -> K2.  A rule of
 * any other shape can never be hit by a frame and is left out (-1). */
int image_table(const WantKey &k) {
  if (k.present == USN_WANT_SRC || k.present == (USN_WANT_SRC | USN_WANT_DPORT | USN_WANT_SPORT))
    return 0;
  if (k.present == 0 || k.present == USN_WANT_DPORT) return 1;
  return -1;
}

/* a registry key whose rule was added, removed or changed: the image is
 * brought up to date before the next batch (refresh_image) */
void note_change(usn_ctx *c, const WantKey &k) {
  if (c->table_dirty) return;
  c->img_delta.push_back(k);
  // more changes than refresh_image would apply in place (or a registry-only
  // context that never refreshes): the next refresh rebuilds; stop queueing
  if (c->img_delta.size() > 4096u + ((size_t)c->img_nkeys[0] + c->img_nkeys[1]) / 8) {
    c->table_dirty = true;
    c->img_delta.clear();
    c->img_delta.shrink_to_fit();
  }
}

/* registry insert */
void rule_insert(usn_ctx *c, const WantKey &k, Rule r) {
  c->rules[k] = r;
  note_change(c, k);
}

/* USN_PROFILE_HOST=1 (test build): per-stage wall times of the host stages on stderr */
struct StageClock {
  bool on = test_knob("USN_PROFILE_HOST") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  const char *name;
  explicit StageClock(const char *n) : name(n) {}
  void mark(const char *what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "%s %-10s %8.3f ms\n", name, what,
                 std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

/* the registry slot of k: a random line in a table of 10^7..10^8 B */
void prefetch_rule(const usn_ctx *c, const WantKey &k) { c->rules.prefetch(k); }

/* ---- perfect-hash image (hash and displace) ---------------------------------
 * n keys go to m = n / USN_PH_LOAD slots through g = n / USN_PH_GROUP groups.
 * Groups are placed largest first; each takes the smallest displacement d
 * that sends all its keys to free, distinct slots (usn_ph_slot).  Lookups
 * then read one displacement and exactly one slot. */
/* A/B knobs, read at context creation: USN_PH_LOAD (slot load), USN_PH_GROUP
 * (keys per displacement) */
double ph_load_knob() {
  const char *e = test_knob("USN_PH_LOAD");
  const double v = e ? std::atof(e) : USN_PH_LOAD;
  return v > 0.05 && v < 0.99 ? v : USN_PH_LOAD;
}
uint32_t ph_group_knob() {
  const char *e = test_knob("USN_PH_GROUP");
  const int v = e ? std::atoi(e) : USN_PH_GROUP;
  return v >= 1 && v <= 32 ? (uint32_t)v : USN_PH_GROUP;
}

struct PhKey {
  PhKey() {}       // no value-initialisation: vectors of 10^6 keys are resized, then filled
  uint4 e;         // the slot: K1/K2 x, y, z, meta | NICOWNER | owner << 16; U: usn_internal.h
  uint4 k;         // the hashed key (x, y, z, meta): K1/K2 the packed key, U (dst, 0, E, 0)
  uint32_t h2, grp;
};

/* Place the n keys of one shard into its m slots and g displacements
 * (group = mulhi(h1 << shift, g)); the outputs are this shard's part of the
 * table's arrays. */
bool ph_place(PhKey *keys, uint32_t n, uint32_t m, uint32_t g, uint32_t seed, uint32_t shift,
              const uint4 &empty, uint4 *slots, uint16_t *disp) {
  for (uint32_t i = 0; i < n; ++i) {
    PhKey &k = keys[i];
    k.grp = usn_mulhi32(usn_ph_h1(k.k.x, k.k.y, k.k.z, k.k.w, seed) << shift, g);
    k.h2 = usn_key_hash2(k.k.x, k.k.y, k.k.z, k.k.w, seed);
  }
  /* members of each group (counting sort), then groups by size, largest first */
  std::vector<uint32_t> start(g + 1, 0), member(n);
  for (uint32_t i = 0; i < n; ++i) start[keys[i].grp + 1]++;
  uint32_t maxsz = 0;
  for (uint32_t i = 0; i < g; ++i) maxsz = std::max(maxsz, start[i + 1]);
  for (uint32_t i = 0; i < g; ++i) start[i + 1] += start[i];
  {
    std::vector<uint32_t> fill(start.begin(), start.end() - 1);
    for (uint32_t i = 0; i < n; ++i) member[fill[keys[i].grp]++] = i;
  }
  std::vector<uint32_t> bysz(maxsz + 2, 0), order(g);
  for (uint32_t i = 0; i < g; ++i) bysz[maxsz - (start[i + 1] - start[i]) + 1]++;
  for (uint32_t s = 0; s <= maxsz; ++s) bysz[s + 1] += bysz[s];
  for (uint32_t i = 0; i < g; ++i) order[bysz[maxsz - (start[i + 1] - start[i])]++] = i;
  std::fill(slots, slots + m, empty);
  std::fill(disp, disp + g, (uint16_t)0);
  std::vector<uint64_t> used((m + 63) / 64, 0);   // a bit per slot: stays in L1/L2
  uint32_t pos[64], h2[64];
  for (uint32_t gi : order) {
    const uint32_t a = start[gi], sz = start[gi + 1] - a;
    if (sz == 0) break;             // the rest are empty
    if (sz > 64) return false;
    for (uint32_t j = 0; j < sz; ++j) h2[j] = keys[member[a + j]].h2;
    uint32_t d = 0;
    for (; d < 65536; ++d) {
      bool ok = true;
      for (uint32_t j = 0; j < sz && ok; ++j) {
        const uint32_t p = usn_ph_slot(h2[j], d, m);
        if ((used[p >> 6] >> (p & 63)) & 1u) { ok = false; break; }
        for (uint32_t q = 0; q < j; ++q)
          if (pos[q] == p) { ok = false; break; }
        pos[j] = p;
      }
      if (ok) break;
    }
    if (d == 65536) return false;
    disp[gi] = (uint16_t)d;
    for (uint32_t j = 0; j < sz; ++j) {
      used[pos[j] >> 6] |= 1ull << (pos[j] & 63);
      slots[pos[j]] = keys[member[a + j]].e;
    }
  }
  return true;
}

/* up to this many keys per shard (one shard: c1-c5 never shard) */
#ifndef USN_PH_SHARD_KEYS
#define USN_PH_SHARD_KEYS 65536u
#endif
#ifndef USN_PH_THREADS
#define USN_PH_THREADS 16u
#endif

/* run f(0..jobs) over up to `threads` threads */
template <class F>
void parallel_for(uint32_t jobs, uint32_t threads, F f) {
  threads = std::max(1u, std::min(threads, jobs));
  if (threads == 1) {
    for (uint32_t j = 0; j < jobs; ++j) f(j);
    return;
  }
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (uint32_t j = t; j < jobs; j += threads) f(j);
    });
  for (std::thread &th : pool) th.join();
}

/* one table of the image: shards, m, g, seed and its slots / displacements
 * (shard after shard).  The keys are partitioned by shard in parallel (shard
 * ids, per-chunk counts, scatter) and every shard is placed straight into
 * its part of `slots` / `disp`. */
bool ph_build(std::vector<PhKey> &keys, usn_ph_table &t, std::vector<uint4> &slots,
              std::vector<uint16_t> &disp, double load0, uint32_t group, uint32_t threads,
              const uint4 &empty = make_uint4(0, 0, 0, 0), uint32_t shard_keys = USN_PH_SHARD_KEYS) {
  const uint32_t n = (uint32_t)keys.size();
  t = usn_ph_table{};
  slots.clear();
  disp.clear();
  if (n == 0) return true;
  uint32_t shift = 0;
  while ((n >> shift) > shard_keys && shift < 16) ++shift;
  const uint32_t S = 1u << shift;
  double load = load0;
  std::vector<PhKey> part;   // the keys, shard after shard (S > 1)
  std::vector<uint32_t> off(S + 1, 0);
  StageClock clk("ph_build");
  for (uint32_t attempt = 0; attempt < 12; ++attempt) {
    if (attempt && attempt % 3 == 0) load *= 0.9;
    const uint32_t seed = 0x9E3779B9u * (attempt + 1);
    PhKey *base = keys.data();
    if (S == 1) {
      off[0] = 0;
      off[1] = n;
    } else {
      const uint32_t C = std::max(1u, std::min(threads, n / 4096 + 1));   // chunks
      std::vector<uint16_t> sid(n);
      std::vector<uint32_t> cnt((size_t)C * S, 0);
      parallel_for(C, threads, [&](uint32_t ch) {
        const uint32_t lo = (uint32_t)((uint64_t)n * ch / C), hi = (uint32_t)((uint64_t)n * (ch + 1) / C);
        uint32_t *c = cnt.data() + (size_t)ch * S;
        for (uint32_t i = lo; i < hi; ++i) {
          const PhKey &k = keys[i];
          sid[i] = (uint16_t)usn_ph_shard(usn_ph_h1(k.k.x, k.k.y, k.k.z, k.k.w, seed), shift);
          c[sid[i]]++;
        }
      });
      // chunk-major offsets within each shard keep the keys' order (deterministic)
      uint32_t run = 0;
      for (uint32_t sh = 0; sh < S; ++sh) {
        off[sh] = run;
        for (uint32_t ch = 0; ch < C; ++ch) {
          const uint32_t v = cnt[(size_t)ch * S + sh];
          cnt[(size_t)ch * S + sh] = run;
          run += v;
        }
      }
      off[S] = run;
      part.resize(n);
      parallel_for(C, threads, [&](uint32_t ch) {
        const uint32_t lo = (uint32_t)((uint64_t)n * ch / C), hi = (uint32_t)((uint64_t)n * (ch + 1) / C);
        uint32_t *c = cnt.data() + (size_t)ch * S;
        for (uint32_t i = lo; i < hi; ++i) part[c[sid[i]]++] = keys[i];
      });
      base = part.data();
    }
    clk.mark("partition");
    uint32_t maxc = 0;
    for (uint32_t sh = 0; sh < S; ++sh) maxc = std::max(maxc, off[sh + 1] - off[sh]);
    // at least 64 slots, and groups for the keys the slots hold at `load`: a
    // small table takes keys in place (refresh_image) before it is rebuilt
    const uint32_t m = std::max<uint32_t>({maxc + 1, (uint32_t)((double)maxc / load) + 1, 64u});
    const uint32_t g = std::max<uint32_t>({1u, (maxc + group - 1) / group,
                                           (uint32_t)(m * load / group)});
    // the probes multiply shard ids by m and g in 24 bits (usn_mul24)
    if (m >= (1u << 24) || g >= (1u << 24) || S > (1u << 16)) return false;
    slots.resize((size_t)S * m);
    disp.resize((size_t)S * g);
    std::vector<uint8_t> ok(S, 0);
    parallel_for(S, threads, [&](uint32_t sh) {
      ok[sh] = ph_place(base + off[sh], off[sh + 1] - off[sh], m, g, seed, shift, empty,
                        slots.data() + (size_t)sh * m, disp.data() + (size_t)sh * g) ? 1 : 0;
    });
    clk.mark("place");
    if (std::find(ok.begin(), ok.end(), 0) != ok.end()) continue;
    t.m = m;
    t.g = g;
    t.seed = seed;
    t.shift = shift;
    return true;
  }
  slots.clear();
  disp.clear();
  return false;
}

/* U and X keys (usn_internal.h) from the K1 / K2 keys: one U slot per
 * projection with the K2 owner and one K1 rule inline; the projection's
 * further K1 rules go to X.  Rules no frame can hit (ports on a protocol that
 * has none, pkt.rs protocol_has_ports) are left out. */
#ifndef USN_U_MAX_KEYS   /* above: U's displacements would not fit LDS, U is not built */
#define USN_U_MAX_KEYS 131072u
#endif
void proj_keys(const std::vector<PhKey> *keys, std::vector<PhKey> &ukeys, std::vector<PhKey> &xkeys) {
  struct Ent { uint32_t dst, e, o1, o2, src, sport; bool more; };
  std::vector<Ent> ents;
  ents.reserve(keys[0].size() + keys[1].size());
  // projection -> entry: flat open addressing (E < 2^19, so ~0 is never a key)
  const uint32_t cap = next_pow2(2 * (uint32_t)(keys[0].size() + keys[1].size()) + 16);
  std::vector<std::pair<uint64_t, uint32_t>> at(cap, {~0ull, 0u});
  auto code = [](const uint4 &e) {
    return (e.w & USN_SLOT_NICOWNER) ? USN_U_NIC : (e.w >> 16);
  };
  for (int t = 1; t >= 0; --t)   // K2 first: a projection's slot exists before its K1 rules look for it
    for (const PhKey &k : keys[t]) {
      const uint32_t proto = k.e.w & 0xFFu, present = (k.e.w >> 8) & 7u;
      const uint32_t has = (present & USN_WANT_DPORT) ? 1u : 0u;
      if (has && usn_u_pidx(proto) == 7u) continue;   // never matched
      const uint32_t E = usn_u_e(proto, has, k.e.z & 0xFFFFu);
      const uint64_t pk = (uint64_t)k.e.x << 32 | E;
      uint32_t h = usn_key_hash(k.e.x, 0u, E, 0u) & (cap - 1);
      while (at[h].first != ~0ull && at[h].first != pk) h = (h + 1) & (cap - 1);
      uint32_t i;
      if (at[h].first == ~0ull) {
        i = (uint32_t)ents.size();
        at[h] = {pk, i};
        ents.push_back(Ent{k.e.x, E, USN_U_NONE, USN_U_NONE, 0u, 0u, false});
      } else {
        i = at[h].second;
      }
      Ent &en = ents[i];
      if (t == 1) {
        en.o2 = code(k.e);
      } else if (en.o1 == USN_U_NONE) {
        en.o1 = code(k.e);
        en.src = k.e.y;
        en.sport = has ? (k.e.z >> 16) : 0u;
      } else {
        en.more = true;
        xkeys.push_back(k);
      }
    }
  ukeys.resize(ents.size());
  for (size_t i = 0; i < ents.size(); ++i) {
    const Ent &en = ents[i];
    PhKey &u = ukeys[i];
    u.e = make_uint4(en.dst, en.src, en.sport | en.o1 << 16 | (en.more ? USN_U_MORE : 0u), en.e | en.o2 << 19);
    u.k = make_uint4(en.dst, 0u, en.e, 0u);
    u.h2 = u.grp = 0;
  }
}

/* The host image of the registry: [K1 slots][K2 slots][K1 disp][K2 disp][pad]
 * (table_units), then, when built, [U slots][X slots][U disp][X disp][pad];
 * each part starts on a 16-byte unit. */
int build_image(usn_ctx *c) {
  StageClock clk("build_image");
  std::vector<PhKey> keys[4];
  const uint32_t hw = std::max(1u, std::min(USN_PH_THREADS, std::thread::hardware_concurrency()));
  {
    // the registry scanned in chunks over threads: count per chunk and table,
    // then each chunk writes its keys at its offsets (the serial order)
    const size_t NS = c->rules.slots();
    const uint32_t C = (uint32_t)std::max<size_t>(1, std::min<size_t>(hw, NS / 65536 + 1));
    std::vector<uint32_t> cnt((size_t)C * 2, 0);
    auto chunk = [&](uint32_t ch, size_t &lo, size_t &hi) { lo = NS * ch / C; hi = NS * (ch + 1) / C; };
    parallel_for(C, hw, [&](uint32_t ch) {
      size_t lo, hi;
      chunk(ch, lo, hi);
      for (size_t i = lo; i < hi; ++i)
        if (const auto *kv = c->rules.at_slot(i)) {
          const int t = image_table(kv->first);
          if (t >= 0) cnt[(size_t)ch * 2 + t]++;
        }
    });
    uint32_t tot[2] = {0, 0};
    for (uint32_t ch = 0; ch < C; ++ch)
      for (int t = 0; t < 2; ++t) {
        const uint32_t v = cnt[(size_t)ch * 2 + t];
        cnt[(size_t)ch * 2 + t] = tot[t];
        tot[t] += v;
      }
    keys[0].resize(tot[0]);
    keys[1].resize(tot[1]);
    parallel_for(C, hw, [&](uint32_t ch) {
      size_t lo, hi;
      chunk(ch, lo, hi);
      uint32_t at[2] = {cnt[(size_t)ch * 2], cnt[(size_t)ch * 2 + 1]};
      for (size_t i = lo; i < hi; ++i) {
        const auto *kv = c->rules.at_slot(i);
        if (!kv) continue;
        const WantKey &k = kv->first;
        const int t = image_table(k);
        if (t < 0) continue;
        const uint16_t owner = kv->second.owner;
        const bool nic = c->eps[owner].used && c->eps[owner].kind == USN_EP_NIC;
        PhKey &pk = keys[t][at[t]++];
        pk.e = make_uint4(k.dst, k.src, (uint32_t)k.dport | ((uint32_t)k.sport << 16),
                          usn_key_meta(k.proto, k.present) | (nic ? USN_SLOT_NICOWNER : 0u) |
                              ((uint32_t)owner << 16));
        pk.k = make_uint4(pk.e.x, pk.e.y, pk.e.z, pk.e.w & USN_KEY_META_MASK);
        pk.h2 = pk.grp = 0;
      }
    });
  }
  bool proj = c->proj && (keys[0].size() + keys[1].size()) > 0 &&
              keys[0].size() + keys[1].size() <= USN_U_MAX_KEYS;
  if (proj) proj_keys(keys, keys[2], keys[3]);
  if (keys[2].empty()) {   // no rule a frame can hit: nothing for U to answer
    proj = false;
    keys[3].clear();
  }
  clk.mark("keys");
  std::vector<uint4> slots[4];
  std::vector<uint16_t> disp[4];
  usn_ph_table t[4] = {};
  bool placed[4] = {false, false, !proj, !proj};
  {
    // the tables side by side, each over its shards
    const uint32_t nt = proj ? 4u : 2u;
    // beyond U's range the K1/K2 displacements never go to LDS (TM_GLOBAL): half
    // the keys per displacement there places twice as fast (1.19 M rules: 102
    // -> 49 ms of placement on 8 threads) for twice the (L2-resident) bytes
    const bool global_only = keys[0].size() + keys[1].size() > USN_U_MAX_KEYS;
    // K1 / K2 at the slot load whose image still fits the classify kernel's
    // LDS copy (LDS_TABLE_MAX_BYTES, 32 KiB) when the default's would not: c3's
    // 1024 rules fit at 0.65, not at 0.5 (then read from L2: 47.5 vs 37.0 us
    // per 512K frames, profiles/r03/r03f_bench.log)
    double load01 = c->ph_load;
    {
      const double n12 = (double)(keys[0].size() + keys[1].size());
      auto kib = [&](double ld) { return (n12 / ld + n12 / c->ph_group / 8 + 136) * 16 / 1024; };
      if (kib(load01) > 31.0)
        for (double ld : {0.55, 0.6, 0.65, 0.7})
          if (ld > load01 && kib(ld) <= 31.0) { load01 = ld; break; }
    }
    c->img_load01 = load01;
    auto one = [&](uint32_t i, uint32_t threads) {
      const uint4 empty = i == 2 ? make_uint4(0, 0, 0, USN_U_EMPTY_W) : make_uint4(0, 0, 0, 0);
      // U and X in shards of up to 16K keys: placed in parallel (an AddMatch
      // rebuilds the image before the next batch)
      const uint32_t shard_keys = i >= 2 ? 16384u : USN_PH_SHARD_KEYS;
      const uint32_t grp0 = (global_only && i < 2) ? std::min(c->ph_group, 5u) : c->ph_group;
      for (uint32_t grp = grp0;; grp /= 2) {   // large groups may not place: smaller ones do
        if (ph_build(keys[i], t[i], slots[i], disp[i], i < 2 ? load01 : c->ph_load, grp, threads, empty,
                     shard_keys)) {
          placed[i] = true;
          break;
        }
        if (grp <= 1) break;
      }
    };
    uint32_t busy = 0;
    for (uint32_t i = 0; i < nt; ++i) busy += keys[i].empty() ? 0u : 1u;
    if (hw > 1 && busy > 1) {
      const uint32_t per = std::max(1u, hw / busy);
      std::vector<std::thread> pool;
      for (uint32_t i = 1; i < nt; ++i) pool.emplace_back(one, i, per);
      one(0, per);
      for (std::thread &th : pool) th.join();
    } else {
      for (uint32_t i = 0; i < nt; ++i) one(i, hw);
    }
  }
  if (!placed[0] || !placed[1] || !placed[2] || !placed[3]) return USN_ENOMEM;
  clk.mark("place");
  // 8 u16 displacements per 16-byte unit
  auto units = [](size_t n16) { return (uint32_t)((n16 + 7) / 8); };
  const uint32_t u0 = (uint32_t)slots[0].size(), u1 = (uint32_t)slots[1].size();
  const uint32_t d0 = units(disp[0].size()), d1 = units(disp[1].size());
  const uint32_t base = u0 + u1 + d0 + d1 + 1;
  // X's displacements take at least one unit: a lane that skips X still reads one inside the LDS copy
  const uint32_t u2 = (uint32_t)slots[2].size(), u3 = (uint32_t)slots[3].size();
  const uint32_t d2 = units(disp[2].size()), d3 = std::max(1u, units(disp[3].size()));
  const uint32_t total = proj ? base + u2 + u3 + d2 + d3 + 1 : base;
  c->img.assign(total, make_uint4(0, 0, 0, 0));
  std::copy(slots[0].begin(), slots[0].end(), c->img.begin());
  std::copy(slots[1].begin(), slots[1].end(), c->img.begin() + u0);
  uint16_t *dp = reinterpret_cast<uint16_t *>(c->img.data() + u0 + u1);
  std::copy(disp[0].begin(), disp[0].end(), dp);
  std::copy(disp[1].begin(), disp[1].end(), dp + (size_t)d0 * 8);
  t[0].slot_off = 0;
  t[1].slot_off = u0;
  t[0].disp_off = (u0 + u1) * 8;
  t[1].disp_off = (u0 + u1 + d0) * 8;
  if (proj) {
    std::copy(slots[2].begin(), slots[2].end(), c->img.begin() + base);
    std::copy(slots[3].begin(), slots[3].end(), c->img.begin() + base + u2);
    uint16_t *up = reinterpret_cast<uint16_t *>(c->img.data() + base + u2 + u3);
    std::copy(disp[2].begin(), disp[2].end(), up);
    std::copy(disp[3].begin(), disp[3].end(), up + (size_t)d2 * 8);
    t[2].slot_off = base;
    t[3].slot_off = base + u2;
    t[2].disp_off = (base + u2 + u3) * 8;
    t[3].disp_off = (base + u2 + u3 + d2) * 8;
  }
  for (int i = 0; i < 4; ++i) c->img_t[i] = t[i];
  c->img_base = base;
  c->img_udisp = proj ? base + u2 + u3 : base;
  c->probe_mask = (keys[0].empty() ? 0u : 1u) | (keys[1].empty() ? 0u : 2u) | (proj ? 4u : 0u);
  c->table_dirty = false;
  ++c->table_version;
  for (int i = 0; i < 4; ++i) c->img_nkeys[i] = (uint32_t)keys[i].size();
  c->img_delta.clear();
  c->img_groups_ok = false;
  c->img_full_version = c->table_version;
  c->img_patches.clear();
  ++c->img_builds;
  clk.mark("image");
  return USN_OK;
}

/* ---- incremental image updates ---------------------------------------------
 * An AddMatch or RemoveMatch changes one key: rather than rebuilding the
 * image (c5: 15-35 ms; the reference's insert is one HashMap insert,
 * main.rs:266-298), the key's slot is written in place, or, for a new key
 * whose slot under its group's displacement is taken, its group is placed
 * again (a new displacement that sends every member to a free slot); the
 * projection slot in U and the X table follow the same way.  Anything
 * else -- a group that cannot be placed, a table past IMG_MAX_LOAD or empty
 * at the last build, a change of the U build condition, more changes than
 * IMG_MAX_DELTA -- rebuilds the whole image.  The replicas upload only the
 * patched units (upload_table). */
#define IMG_MAX_LOAD 0.6
int g_img_fail = 0;   // diagnostics: why the last in-place insert failed (table * 10 + cause)
bool img_occupied(int i, const uint4 &e) {
  return i == 2 ? e.w != USN_U_EMPTY_W : (e.w & USN_SLOT_VALID) != 0;
}
uint4 img_empty(int i) { return i == 2 ? make_uint4(0, 0, 0, USN_U_EMPTY_W) : make_uint4(0, 0, 0, 0); }
uint4 img_hkey(int i, const uint4 &e) {   // the hashed key of an occupied slot
  return i == 2 ? make_uint4(e.x, 0u, e.w & USN_U_EMASK, 0u)
                : make_uint4(e.x, e.y, e.z, e.w & USN_KEY_META_MASK);
}
void img_patch(usn_ctx *c, uint32_t unit) { c->img_patches.emplace_back(c->table_version + 1, unit); }
uint16_t *img_disp(usn_ctx *c) { return reinterpret_cast<uint16_t *>(c->img.data()); }

void img_groups_build(usn_ctx *c) {
  for (int i = 0; i < 4; ++i) {
    const usn_ph_table &T = c->img_t[i];
    auto &G = c->img_groups[i];
    G.assign(T.m ? (size_t)T.g << T.shift : 0, {});
    if (!T.m) continue;
    const size_t slots = (size_t)T.m << T.shift;
    for (size_t q = 0; q < slots; ++q) {
      const uint4 &e = c->img[T.slot_off + q];
      if (!img_occupied(i, e)) continue;
      const uint4 k = img_hkey(i, e);
      G[usn_ph_group(usn_ph_h1(k.x, k.y, k.z, k.w, T.seed), T.shift, T.g)].push_back((uint32_t)q);
    }
  }
  c->img_groups_ok = true;
}

/* the image unit holding key k of table i, or -1 */
int64_t img_find(const usn_ctx *c, int i, const uint4 &k) {
  const usn_ph_table &T = c->img_t[i];
  if (!T.m) return -1;
  const uint32_t h1 = usn_ph_h1(k.x, k.y, k.z, k.w, T.seed);
  const uint32_t G = usn_ph_group(h1, T.shift, T.g);
  const uint16_t d = reinterpret_cast<const uint16_t *>(c->img.data())[T.disp_off + G];
  const size_t u = T.slot_off + (size_t)usn_ph_shard(h1, T.shift) * T.m +
                   usn_ph_slot(usn_key_hash2(k.x, k.y, k.z, k.w, T.seed), d, T.m);
  const uint4 &e = c->img[u];
  if (!img_occupied(i, e)) return -1;
  const uint4 h = img_hkey(i, e);
  return (h.x == k.x && h.y == k.y && h.z == k.z && h.w == k.w) ? (int64_t)u : -1;
}

/* a displacement group of table i being placed again: its entries (the
 * members, plus a new one) and their slots under the displacement found */
struct GroupMove {
  uint32_t G = 0, sh = 0;
  size_t n = 0;
  uint4 ent[64];
  uint32_t hh[64], pos[64];
  uint32_t d = 0;
  const GroupMove *avoid = nullptr;   // another group's move whose target slots are taken
};
bool img_group_collect(usn_ctx *c, int i, uint32_t G, const uint4 *extra, uint32_t extra_h2,
                       GroupMove &mv) {
  const usn_ph_table &T = c->img_t[i];
  const std::vector<uint32_t> &mem = c->img_groups[i][G];
  mv.G = G;
  mv.sh = G / T.g;
  mv.n = mem.size() + (extra ? 1 : 0);
  if (mv.n > 64) return false;
  for (size_t j = 0; j < mem.size(); ++j) {
    mv.ent[j] = c->img[T.slot_off + mem[j]];
    const uint4 mk = img_hkey(i, mv.ent[j]);
    mv.hh[j] = usn_key_hash2(mk.x, mk.y, mk.z, mk.w, T.seed);
  }
  if (extra) {
    mv.ent[mv.n - 1] = *extra;
    mv.hh[mv.n - 1] = extra_h2;
  }
  return true;
}
/* the first displacement that sends every entry of mv to a distinct slot
 * that is free or the group's own (and not a target of mv.avoid); with
 * `one`, the displacements blocked by exactly one other key are collected */
bool img_group_search(usn_ctx *c, int i, GroupMove &mv, const GroupMove *avoid,
                      std::vector<std::pair<uint32_t, uint32_t>> *one) {
  const usn_ph_table &T = c->img_t[i];
  const std::vector<uint32_t> &mem = c->img_groups[i][mv.G];
  const size_t base = T.slot_off + (size_t)mv.sh * T.m;
  auto own = [&](uint32_t p) {
    return std::find(mem.begin(), mem.end(), (uint32_t)(mv.sh * T.m + p)) != mem.end();
  };
  for (uint32_t d = 0; d < 65536; ++d) {
    uint32_t blockers = 0, blocker = 0;
    bool ok = true;
    for (size_t j = 0; j < mv.n && ok; ++j) {
      const uint32_t p = usn_ph_slot(mv.hh[j], d, T.m);
      for (size_t q = 0; q < j; ++q)
        if (mv.pos[q] == p) { ok = false; break; }
      if (!ok) break;
      mv.pos[j] = p;
      if (avoid && avoid->sh == mv.sh)
        for (size_t q = 0; q < avoid->n; ++q)
          if (avoid->pos[q] == p) { ok = false; break; }
      if (!ok) break;
      if (img_occupied(i, c->img[base + p]) && !own(p)) {
        blocker = p;
        if (++blockers > (one ? 1u : 0u)) ok = false;
      }
    }
    if (!ok) continue;
    if (blockers == 0) { mv.d = d; return true; }
    if (one && one->size() < 64) one->emplace_back(d, blocker);
  }
  return false;
}
/* the group's old slots emptied, its entries written at mv.pos, its
 * displacement set (every unit patched) */
void img_group_commit(usn_ctx *c, int i, const GroupMove &mv) {
  const usn_ph_table &T = c->img_t[i];
  std::vector<uint32_t> &mem = c->img_groups[i][mv.G];
  const size_t base = T.slot_off + (size_t)mv.sh * T.m;
  const uint4 empty = img_empty(i);
  for (uint32_t q : mem) {
    c->img[T.slot_off + q] = empty;
    img_patch(c, (uint32_t)(T.slot_off + q));
  }
  mem.clear();
  for (size_t j = 0; j < mv.n; ++j) {
    c->img[base + mv.pos[j]] = mv.ent[j];
    img_patch(c, (uint32_t)(base + mv.pos[j]));
    mem.push_back((uint32_t)(mv.sh * T.m + mv.pos[j]));
  }
  img_disp(c)[T.disp_off + mv.G] = (uint16_t)mv.d;
  img_patch(c, (T.disp_off + mv.G) / 8);
}

/* key k of table i gets slot content e (inserted or overwritten) */
bool img_upsert(usn_ctx *c, int i, const uint4 &k, const uint4 &e) {
  const int64_t at = img_find(c, i, k);
  if (at >= 0) {
    c->img[at] = e;
    img_patch(c, (uint32_t)at);
    return true;
  }
  const usn_ph_table &T = c->img_t[i];
  const double max_load = std::max(IMG_MAX_LOAD, (i < 2 ? c->img_load01 : c->ph_load) + 0.05);
  if (!T.m || c->img_nkeys[i] + 1 > max_load * (double)((size_t)T.m << T.shift)) {
    g_img_fail = i * 10 + 1;
    return false;
  }
  const uint32_t h1 = usn_ph_h1(k.x, k.y, k.z, k.w, T.seed);
  const uint32_t G = usn_ph_group(h1, T.shift, T.g), sh = usn_ph_shard(h1, T.shift);
  const size_t base = T.slot_off + (size_t)sh * T.m;   // the shard's first unit
  uint16_t *D = img_disp(c);
  const uint32_t h2 = usn_key_hash2(k.x, k.y, k.z, k.w, T.seed);
  std::vector<uint32_t> &mem = c->img_groups[i][G];   // from the table's first slot
  const uint32_t p0 = usn_ph_slot(h2, D[T.disp_off + G], T.m);
  if (!img_occupied(i, c->img[base + p0])) {   // free under the group's displacement
    c->img[base + p0] = e;
    img_patch(c, (uint32_t)(base + p0));
    mem.push_back((uint32_t)(sh * T.m + p0));
    c->img_nkeys[i]++;
    return true;
  }
  // the group again with a new displacement (img_group_search); if none
  // exists, one that blocks on a single key of another group, which that
  // group gives up by taking a new displacement itself
  GroupMove mv;
  if (!img_group_collect(c, i, G, &e, h2, mv)) { g_img_fail = i * 10 + 2; return false; }
  std::vector<std::pair<uint32_t, uint32_t>> one;   // (d, blocking slot) with a single blocker
  if (img_group_search(c, i, mv, nullptr, &one)) {
    img_group_commit(c, i, mv);
    c->img_nkeys[i]++;
    return true;
  }
  for (const auto &cand : one) {
    mv.d = cand.first;
    for (size_t j = 0; j < mv.n; ++j) mv.pos[j] = usn_ph_slot(mv.hh[j], mv.d, T.m);
    const uint4 bk = img_hkey(i, c->img[base + cand.second]);
    const uint32_t GB = usn_ph_group(usn_ph_h1(bk.x, bk.y, bk.z, bk.w, T.seed), T.shift, T.g);
    if (GB == G) continue;
    GroupMove mb;
    if (!img_group_collect(c, i, GB, nullptr, 0, mb)) continue;
    mb.avoid = &mv;   // not into the slots G takes (the blocker's among them)
    if (!img_group_search(c, i, mb, &mv, nullptr)) continue;
    img_group_commit(c, i, mb);
    img_group_commit(c, i, mv);
    c->img_nkeys[i]++;
    return true;
  }
  g_img_fail = i * 10 + 3;
  return false;
}

/* key k of table i leaves the image (if it is there) */
void img_erase(usn_ctx *c, int i, const uint4 &k) {
  const int64_t at = img_find(c, i, k);
  if (at < 0) return;
  const usn_ph_table &T = c->img_t[i];
  const uint32_t G = usn_ph_group(usn_ph_h1(k.x, k.y, k.z, k.w, T.seed), T.shift, T.g);
  std::vector<uint32_t> &mem = c->img_groups[i][G];
  mem.erase(std::find(mem.begin(), mem.end(), (uint32_t)(at - T.slot_off)));
  c->img[at] = img_empty(i);
  img_patch(c, (uint32_t)at);
  c->img_nkeys[i]--;
}

/* one registry key, brought into the image as build_image would place it
 * (K1 / K2 slot; U's projection slot and X as proj_keys builds them) */
bool img_apply_key(usn_ctx *c, const WantKey &k) {
  const int t = image_table(k);
  if (t < 0) return true;                        // no frame can hit it: not in the image
  auto it = c->rules.find(k);
  const bool present = it != c->rules.end();
  const uint16_t owner = present ? it->second.owner : 0;
  const bool nic = present && c->eps[owner].used && c->eps[owner].kind == USN_EP_NIC;
  const uint4 e = make_uint4(k.dst, k.src, (uint32_t)k.dport | ((uint32_t)k.sport << 16),
                             usn_key_meta(k.proto, k.present) | (nic ? USN_SLOT_NICOWNER : 0u) |
                                 ((uint32_t)owner << 16));
  const uint4 hk = make_uint4(e.x, e.y, e.z, e.w & USN_KEY_META_MASK);
  if (present) {
    if (!img_upsert(c, t, hk, e)) return false;
  } else {
    img_erase(c, t, hk);
  }
  if (!(c->probe_mask & 4u)) return true;
  const uint32_t has = (k.present & USN_WANT_DPORT) ? 1u : 0u;
  if (has && usn_u_pidx(k.proto) == 7u) return true;   // never matched (proj_keys skips it)
  const uint32_t E = usn_u_e(k.proto, has, k.dport);
  const uint4 uk = make_uint4(k.dst, 0u, E, 0u);
  const uint32_t code = !present ? USN_U_NONE : nic ? USN_U_NIC : owner;
  const int64_t at = img_find(c, 2, uk);
  if (t == 1) {                                  // key2: the projection's K2 owner
    if (at >= 0) {
      uint4 u = c->img[at];
      u.w = E | code << 19;
      c->img[at] = u;
      img_patch(c, (uint32_t)at);
      return true;
    }
    if (!present) return true;
    return img_upsert(c, 2, uk, make_uint4(k.dst, 0u, USN_U_NONE << 16, E | code << 19));
  }
  const uint32_t sport = has ? k.sport : 0u;     // key1: inline, or in X
  if (at < 0) {
    if (!present) return true;
    return img_upsert(c, 2, uk, make_uint4(k.dst, k.src, sport | code << 16, E | USN_U_NONE << 19));
  }
  uint4 u = c->img[at];
  const uint32_t o1 = (u.z >> 16) & 0x1FFFu;
  const bool inline_is_k = o1 != USN_U_NONE && u.y == k.src && (u.z & 0xFFFFu) == sport;
  if (inline_is_k) {                             // update or empty the inline rule (MORE stays)
    u.z = (u.z & USN_U_MORE) | (present ? (sport | code << 16) : (USN_U_NONE << 16));
    if (!present) u.y = 0;
    c->img[at] = u;
    img_patch(c, (uint32_t)at);
    return true;
  }
  if (!present) {
    if (c->img_t[3].m) img_erase(c, 3, hk);
    return true;
  }
  if (c->img_t[3].m && img_find(c, 3, hk) >= 0) return img_upsert(c, 3, hk, e);
  if (o1 == USN_U_NONE) {                        // the inline place is free
    u.y = k.src;
    u.z = (u.z & USN_U_MORE) | sport | code << 16;
    c->img[at] = u;
    img_patch(c, (uint32_t)at);
    return true;
  }
  u.z |= USN_U_MORE;
  c->img[at] = u;
  img_patch(c, (uint32_t)at);
  return img_upsert(c, 3, hk, e);                // (X empty at the last build: rebuild)
}

#define IMG_MAX_DELTA 4096u
#define IMG_MAX_PATCHES (1u << 16)
/* the host image brought up to date with the registry: the changed keys in
 * place, or a full build */
int refresh_image(usn_ctx *c) {
  if (c->table_dirty || c->img.empty()) return build_image(c);
  if (c->img_delta.empty()) return USN_OK;
  const size_t total = (size_t)c->img_nkeys[0] + c->img_nkeys[1];
  if (!c->incremental || c->img_delta.size() > IMG_MAX_DELTA + total / 8 ||
      c->img_patches.size() > IMG_MAX_PATCHES)
    return build_image(c);
  if (!c->img_groups_ok) img_groups_build(c);
  static const bool verbose = test_knob("USN_PROFILE_HOST") != nullptr;
  for (const WantKey &k : c->img_delta)
    if (!img_apply_key(c, k)) {
      if (verbose)
        std::fprintf(stderr, "refresh_image: key (table %d, cause %d) not placed in place: rebuild (keys %u %u %u %u)\n",
                     image_table(k), g_img_fail, c->img_nkeys[0], c->img_nkeys[1], c->img_nkeys[2], c->img_nkeys[3]);
      return build_image(c);
    }
  // the U build condition of build_image, with the counts the keys now have
  const uint32_t n12 = c->img_nkeys[0] + c->img_nkeys[1];
  const bool want_proj = c->proj && n12 > 0 && n12 <= USN_U_MAX_KEYS;
  if (want_proj != ((c->probe_mask & 4u) != 0) ||
      (n12 > USN_U_MAX_KEYS) != (total > USN_U_MAX_KEYS)) {  // K1/K2 group size changes there
    if (verbose) std::fprintf(stderr, "refresh_image: U build condition changed: rebuild\n");
    return build_image(c);
  }
  c->img_delta.clear();
  ++c->table_version;
  ++c->img_updates;
  return USN_OK;
}

/* the image probe as the device computes it (usn_device.hip ph_probe) */
uint32_t image_probe(const usn_ctx *c, int table, uint32_t x, uint32_t y, uint32_t z, uint32_t meta) {
  const usn_ph_table &t = c->img_t[table];
  if (!t.m) return 0;
  const uint32_t h1 = usn_ph_h1(x, y, z, meta, t.seed);
  const uint32_t grp = usn_ph_group(h1, t.shift, t.g);
  const uint16_t d = reinterpret_cast<const uint16_t *>(c->img.data())[t.disp_off + grp];
  const uint4 s = c->img[t.slot_off + usn_ph_shard(h1, t.shift) * t.m +
                         usn_ph_slot(usn_key_hash2(x, y, z, meta, t.seed), d, t.m)];
  const bool hit = s.x == x && s.y == y && s.z == z && ((s.w ^ meta) & USN_KEY_META_MASK) == 0;
  return hit ? s.w : 0u;
}

/* get_endpoint's two lookups for a parsed IPv4 frame through U (and X) as the
 * device computes them: w[0] = key1's slot meta word, w[1] = key2's (0 = miss) */
void image_probe_u(const usn_ctx *c, uint32_t dst, uint32_t src, uint32_t proto, uint32_t has,
                   uint32_t dport, uint32_t sport, uint32_t w[2]) {
  w[0] = w[1] = 0;
  const usn_ph_table &t = c->img_t[2];
  if (!(c->probe_mask & 4u) || !t.m) return;
  const uint32_t E = usn_u_e(proto, has, dport);
  const uint32_t h1 = usn_ph_h1(dst, 0u, E, 0u, t.seed);
  const uint16_t d = reinterpret_cast<const uint16_t *>(c->img.data())[t.disp_off + usn_ph_group(h1, t.shift, t.g)];
  const uint4 s = c->img[t.slot_off + usn_ph_shard(h1, t.shift) * t.m +
                         usn_ph_slot(usn_key_hash2(dst, 0u, E, 0u, t.seed), d, t.m)];
  if (s.x != dst || (s.w & USN_U_EMASK) != E) return;
  const uint32_t o1 = (s.z >> 16) & 0x1FFFu, sp = has ? sport : 0u;
  const bool in1 = o1 != USN_U_NONE && s.y == src && (s.z & 0xFFFFu) == sp;
  w[0] = in1 ? usn_u_meta(o1) : 0u;
  if (!in1 && (s.z & USN_U_MORE))
    w[0] = image_probe(c, 3, dst, src, has ? (dport | sport << 16) : 0u,
                       usn_key_meta(proto, has ? (USN_WANT_DPORT | USN_WANT_SRC | USN_WANT_SPORT) : USN_WANT_SRC));
  w[1] = usn_u_meta(s.w >> 19);
}

/* the replica's device table at the current image version; no batch still
 * in flight on that device may read the old one */
int upload_table(usn_ctx *c, Replica &R) {
  { const int s = refresh_image(c); if (s) return s; }
  if (R.table_version == c->table_version) return USN_OK;
  StageClock clk("upload_table");
  const size_t bytes = c->img.size() * sizeof(uint4);
  HIPCHK(hipSetDevice(R.device));
  HIPCHK(hipDeviceSynchronize());   // no batch in flight on this device reads the old image
  if (R.d_table && R.table_version >= c->img_full_version && bytes <= R.d_table_cap) {
    // the replica holds this build's image at an older version: the units
    // patched since, in runs of consecutive units
    // patched units, then one copy of {values}{indices} and one patch launch
    std::vector<uint32_t> u;
    for (const auto &pv : c->img_patches)
      if (pv.first > R.table_version) u.push_back(pv.second);
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    const size_t pb = u.size() * (sizeof(uint4) + 4);
    if (pb > c->h_patch_cap) {
      if (c->h_patch) HIPCHK(hipHostFree(c->h_patch));
      c->h_patch = nullptr;
      HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c->h_patch), pb, hipHostMallocDefault));
      c->h_patch_cap = pb;
    }
    if (pb > R.d_patch_cap) {
      if (R.d_patch) HIPCHK(hipFree(R.d_patch));
      R.d_patch = nullptr;
      HIPCHK(hipMalloc(&R.d_patch, pb));
      R.d_patch_cap = pb;
    }
    uint4 *hv = reinterpret_cast<uint4 *>(c->h_patch);
    uint32_t *hi = reinterpret_cast<uint32_t *>(hv + u.size());
    for (size_t k = 0; k < u.size(); ++k) { hv[k] = c->img[u[k]]; hi[k] = u[k]; }
    HIPCHK(hipMemcpyAsync(R.d_patch, c->h_patch, pb, hipMemcpyHostToDevice, nullptr));
    HIPCHK(usn::launch_patch(R.d_table, R.d_patch, (uint32_t)u.size(), nullptr));
    HIPCHK(hipStreamSynchronize(nullptr));
    R.table_version = c->table_version;
    bool all = true;   // every replica current: the log starts afresh
    for (const Replica &Q : c->reps) all &= Q.table_version == c->table_version;
    if (all) c->img_patches.clear();
    clk.mark("patch");
    return USN_OK;
  }
  if (bytes > R.d_table_cap) {
    if (R.d_table) HIPCHK(hipFree(R.d_table));
    R.d_table = nullptr;
    HIPCHK(hipMalloc(&R.d_table, bytes));
    R.d_table_cap = bytes;
  }
  HIPCHK(hipMemcpy(R.d_table, c->img.data(), bytes, hipMemcpyHostToDevice));
  R.table_version = c->table_version;
  clk.mark("upload");
  return USN_OK;
}

/* membership set of innerl2bridge (endpoint.rs:195, 254) for tx_scan */
void build_bridge_set(usn_ctx *c) {
  const uint32_t slots = next_pow2(std::max<uint32_t>(16, 2 * (uint32_t)c->bridge.size()));
  c->bridge_set.assign(slots, 0ull);
  for (uint64_t m : c->bridge) {
    uint32_t h = usn_mac_hash(m) & (slots - 1);
    while ((c->bridge_set[h] >> 63) && (c->bridge_set[h] & 0xFFFFFFFFFFFFull) != m)
      h = (h + 1) & (slots - 1);
    c->bridge_set[h] = (1ull << 63) | m;
  }
  c->bridge_mask = slots - 1;
  c->bridge_dirty = false;
  ++c->bridge_version;
}

int upload_bridge(usn_ctx *c, Replica &R) {
  if (c->bridge_dirty) build_bridge_set(c);
  if (R.bridge_version == c->bridge_version) return USN_OK;
  HIPCHK(hipSetDevice(R.device));
  HIPCHK(hipDeviceSynchronize());
  const size_t bytes = std::max<size_t>(8, c->bridge.size() * 8);
  if (bytes > R.d_bridge_cap) {
    if (R.d_bridge) HIPCHK(hipFree(R.d_bridge));
    R.d_bridge = nullptr;
    HIPCHK(hipMalloc(&R.d_bridge, bytes));
    R.d_bridge_cap = bytes;
  }
  if (!c->bridge.empty())
    HIPCHK(hipMemcpy(R.d_bridge, c->bridge.data(), c->bridge.size() * 8, hipMemcpyHostToDevice));
  const size_t sb = c->bridge_set.size() * 8ull;
  if (sb > R.d_bridge_set_cap) {
    if (R.d_bridge_set) HIPCHK(hipFree(R.d_bridge_set));
    R.d_bridge_set = nullptr;
    HIPCHK(hipMalloc(&R.d_bridge_set, sb));
    R.d_bridge_set_cap = sb;
  }
  HIPCHK(hipMemcpy(R.d_bridge_set, c->bridge_set.data(), sb, hipMemcpyHostToDevice));
  R.bridge_version = c->bridge_version;
  return USN_OK;
}

void cache_clear(usn_ctx *c, int ep) {
  if (ep < 0 || ep >= USN_MAX_ENDPOINTS) return;
  Chain &ch = c->chains[ep];
  ch = Chain();   // last_pkt = None
}

/* ---- host restatement of the per-frame path for the ordered stage -------- */
uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
uint64_t mac48(const uint8_t *p) {
  uint64_t m = 0;
  for (int i = 0; i < 6; ++i) m |= (uint64_t)p[i] << (8 * i);
  return m;
}

/* extract_pkt_info (pkt.rs:158-218) including the fragment map side effects */
ParsedH host_parse(usn_ctx *c, const uint8_t *b, uint32_t len) {
  ParsedH r{};
  r.status = 0;
  r.reason = USN_R_PARSE;
  if (len < 14) return r;
  r.dmac = mac48(b);
  r.smac = mac48(b + 6);
  const uint16_t et = be16(b + 12);
  if (et == 0x0806) { r.status = 1; r.info.w[0] = USN_INFO_ARP; return r; }
  if (et == 0x888E) { r.status = 1; r.info.w[0] = USN_INFO_EAPOL; return r; }
  if (et != 0x0800) return r;
  const uint8_t *p = b + 14;
  const uint32_t n = len - 14;
  if (n < 20) return r;
  const uint32_t hl = (p[0] & 0x0Fu) * 4, tl = be16(p + 2);
  if (n < hl || hl > tl || n < tl) return r;
  const uint16_t ff = be16(p + 6);
  FragKey fk{be16(p + 4), p[9], be32(p + 12), be32(p + 16), r.smac, r.dmac};
  if (ff & 0x1FFF) {
    auto it = c->frags.find(fk);
    if (it == c->frags.end()) { r.reason = USN_R_FRAGMISS; return r; }
    r.status = 1;
    r.info = it->second.info;
    r.smac = it->second.smac;
    r.dmac = it->second.dmac;
    return r;
  }
  const uint32_t proto = p[9];
  const bool pp = proto == 6 || proto == 17 || proto == 0x21 || proto == 0x84 || proto == 0x88;
  const bool ports = pp && (tl - hl) > 4;
  r.info.w[0] = USN_INFO_IPV4 | (proto << 8) | ((ports ? 1u : 0u) << 16);
  r.info.w[1] = be32(p + 12);
  r.info.w[2] = be32(p + 16);
  r.info.w[3] = ports ? ((uint32_t)be16(p + hl) | ((uint32_t)be16(p + hl + 2) << 16)) : 0u;
  r.status = 1;
  if (!(ff & 0x4000) && (ff & 0x2000)) c->frags[fk] = FragVal{r.info, r.smac, r.dmac};
  return r;
}

int registry_get(const usn_ctx *c, const WantKey &k) {
  auto it = c->rules.find(k);
  return it == c->rules.end() ? -1 : (int)it->second.owner;
}

bool bridge_has(const usn_ctx *c, uint64_t mac) {
  return std::find(c->bridge.begin(), c->bridge.end(), mac) != c->bridge.end();
}

struct CacheState {
  bool valid = false;
  Info info{};
  uint32_t dst = 0;
};

/* find_forward (endpoint.rs:172-296) for one frame; updates registry, bridge,
 * fragment map, next_dhcp and the source's cache state. */
uint32_t host_step(usn_ctx *c, int src, const uint8_t *frame, uint32_t len, CacheState &st,
                   bool &learned) {
  learned = false;
  Ep &S = c->eps[src];
  const bool incoming = S.kind == USN_EP_NIC;
  ParsedH p = host_parse(c, frame, len);
  if (!p.status) return usn_mkdec(USN_CLS_DROP, p.reason, 0xFFFF);
  if (st.valid && st.info == p.info) return st.dst | USN_F_CACHE;
  st.valid = false;
  if (!incoming && !(p.smac & 1) && !bridge_has(c, p.smac)) {
    c->bridge.push_back(p.smac);
    c->bridge_dirty = true;
    learned = true;
  }
  const uint32_t kind = p.info.kind();
  if (kind == USN_INFO_ARP || kind == USN_INFO_EAPOL) return usn_mkdec(USN_CLS_FLOOD, 0, 0xFFFF);
  if ((p.info.dst() >> 24) == 127) return usn_mkdec(USN_CLS_DROP, USN_R_LOOPBACK, 0xFFFF);
  st.valid = true;
  st.info = p.info;
  const bool ports = p.info.has_ports();
  const uint32_t proto = p.info.proto();
  if (!incoming) {
    WantKey w;   // to_want (pkt.rs:78-95)
    w.dst = p.info.src();
    w.src = p.info.dst();
    w.proto = (uint8_t)proto;
    w.present = USN_WANT_SRC | (ports ? (USN_WANT_DPORT | USN_WANT_SPORT) : 0);
    w.dport = ports ? (uint16_t)p.info.sport() : 0;
    w.sport = ports ? (uint16_t)p.info.dport() : 0;
    bool listening = false;
    for (const Listen &l : S.listening)
      if (l.dst == w.dst && l.proto == w.proto && l.has_port == (ports ? 1 : 0) &&
          (!ports || l.port == w.dport)) { listening = true; break; }
    if (!listening) {
      // is_unspecified(): smoltcp 0.7.0's 0.0.0.0/8 range test (src[0] == 0), pkt.rs:46
      const bool dhcp_req = proto == 17 && (p.info.src() >> 24) == 0 && ports && p.info.sport() == 68 &&
                            p.info.dport() == 67 && (p.info.dst() & 0xFF) == 255;
      if (dhcp_req) {
        if (S.for_nic >= 0) {
          c->eps[S.for_nic].next_dhcp = src;
          cache_clear(c, S.for_nic);
          st.valid = false;
        }
      } else if (!c->rules.count(w)) {
        if (S.for_nic >= 0) cache_clear(c, S.for_nic);
        rule_insert(c, w, Rule{(uint16_t)src, 0});
        learned = true;
      }
    }
  }
  uint32_t d;
  if (!incoming && !bridge_has(c, p.dmac)) {
    d = usn_mkdec(USN_CLS_NIC, 0, (uint32_t)S.for_nic);
  } else {
    WantKey k1;
    k1.dst = p.info.dst();
    k1.src = p.info.src();
    k1.proto = (uint8_t)proto;
    k1.present = USN_WANT_SRC | (ports ? (USN_WANT_DPORT | USN_WANT_SPORT) : 0);
    k1.dport = ports ? (uint16_t)p.info.dport() : 0;
    k1.sport = ports ? (uint16_t)p.info.sport() : 0;
    int e = registry_get(c, k1);
    if (e < 0) {
      WantKey k2 = k1;
      k2.src = 0;
      k2.sport = 0;
      k2.present = ports ? USN_WANT_DPORT : 0;
      e = registry_get(c, k2);
    }
    bool excl = false;
    if (e >= 0 && (c->eps[e].kind == USN_EP_NIC || e == src)) { excl = true; e = -1; }
    if (e >= 0) {
      d = usn_mkdec(USN_CLS_EP, 0, (uint32_t)e);
    } else if (proto == 17 && ports && p.info.sport() == 67 && p.info.dport() == 68) {
      if (S.next_dhcp >= 0) {
        d = usn_mkdec(USN_CLS_EP, 0, (uint32_t)S.next_dhcp) | USN_F_DHCP;
        S.next_dhcp = -1;
        st.valid = false;
      } else {
        d = usn_mkdec(USN_CLS_DROP, USN_R_DHCP_NONE, 0xFFFF);
      }
    } else {
      d = usn_mkdec(USN_CLS_DROP, excl ? USN_R_EXCLUDED : USN_R_NOMATCH, 0xFFFF);
    }
  }
  st.dst = d & USN_PARITY_MASK;
  return d;
}

}  // namespace

/* ========================================================================== */
namespace usn {
/* scratch of the per-endpoint scatter for one batch of n frames and nbins
 * bins: cnt[ntiles][nbw] u16 | agg[nchunks][nbw] u32 | tot[nbw] u32 |
 * gran[nranges][nbw] u64 | diag u32.  agg and gran are sized
 * for one-tile chunks: a launch picks its chunk length (launch_scatter) */
struct ScatterGeom {
  uint32_t nbw, ntiles;
  size_t cnt, agg, tot, gran, diag, total;
};
static ScatterGeom scatter_geom(uint64_t n, uint32_t nbins) {
  ScatterGeom g;
  g.nbw = (nbins + 7u) & ~7u;
  g.ntiles = (uint32_t)((n + USN_TILE - 1) / USN_TILE);
  const size_t ranges = (g.ntiles + USN_SCAN_RANGE_MIN - 1) / USN_SCAN_RANGE_MIN;
  size_t o = 0;
  auto a256 = [](size_t v) { return (v + 255) & ~(size_t)255; };
  g.cnt = o; o = a256(o + (size_t)g.ntiles * g.nbw * 2);
  g.agg = o; o = a256(o + (size_t)g.ntiles * g.nbw * 4);
  g.tot = o; o = a256(o + (size_t)g.nbw * 4);
  g.gran = o; o = a256(o + ranges * g.nbw * 8);
  g.diag = o; o = a256(o + 4);
  g.total = o;
  return g;
}
size_t scatter_scratch_bytes(uint64_t n, uint32_t nbins) { return scatter_geom(n, nbins).total; }
/* the scratch's layout follows the result's capacity (cap = usn_result.n),
 * not the batch's frames: a result keeps one geometry per bin count however
 * its batches vary (the granules are zeroed once per bind and bin count) */
void scatter_carve(void *scratch, uint64_t cap, uint64_t n, uint32_t nbins, uint32_t tc, uint32_t cpt,
                   ScatterBatch &sb, uint16_t **cnt) {
  const ScatterGeom g = scatter_geom(cap, nbins);
  const uint32_t ntiles = (uint32_t)((n + USN_TILE - 1) / USN_TILE);
  uint8_t *p = static_cast<uint8_t *>(scratch);
  *cnt = reinterpret_cast<uint16_t *>(p + g.cnt);
  sb.cnt = *cnt;
  sb.agg = reinterpret_cast<uint32_t *>(p + g.agg);
  sb.tot = reinterpret_cast<uint32_t *>(p + g.tot);
  sb.gran = reinterpret_cast<unsigned long long *>(p + g.gran);
  sb.diag = reinterpret_cast<uint32_t *>(p + g.diag);
  sb.n = (uint32_t)n;
  sb.ntiles = ntiles;
  sb.tc = tc;
  sb.nchunks = (ntiles + tc - 1) / tc;
  sb.nranges = (sb.nchunks + 16 * cpt - 1) / (16 * cpt);
}
/* the scan's diag word of a batch's scratch (bit 0: a wait timed out) */
uint32_t *scatter_diag(void *scratch, uint64_t cap, uint32_t nbins) {
  return reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(scratch) + scatter_geom(cap, nbins).diag);
}
/* How a launch's lists are built (launch_scatter): chunk length, scan
 * threads' chunks, and whether the scan launch is skipped.
 *  - chunk length: about one chunk per CU -- the longest chunk up to the LDS
 *    shape's that still gives every CU one (A/B at 1024 tiles, a tx ring or
 *    c3's call, profiles/r04/r04j: scan + scatter 21.3 / 16.7 / 16.1 / 17.6
 *    us at chunks of 1 / 2 / 4 / 8 tiles; c5 and c2 keep 8).  tc_knob (A/B)
 *    is taken as it is, at most the shape's;
 *  - noscan: batches of at most one chunk each (a daemon's drained rings):
 *    the scatter's one chunk per batch has the whole batch;
 *  - selfscan: every chunk resident at once and all chunks together reading
 *    at most selfscan_kb KiB of count rows (each reads its whole batch's):
 *    each chunk sums them itself (profiles/r04/r04n: c3's calls, 9.4 MB,
 *    lists 15.1 -> 11.8 us; a 1M c4 ring, 138 MB, 15.5 -> 33.7 us);
 *  - cpt: 4 chunks per scan thread (a workgroup per 64 chunks) while that
 *    gives >= 256 workgroups, else fewer (profiles/r03/r03i: c5 16M 56.6 /
 *    57.3 / 60.3 us at 4 / 2 / 1; c2 8M 32.1 / 30.4 / 29.4). */
ScatterPlan scatter_plan(const uint32_t *ntiles, uint32_t count, uint32_t nbins, uint32_t cus,
                         uint32_t tc_knob, uint32_t cpt_knob, uint32_t selfscan_kb) {
  ScatterPlan p{};
  const ScatterShape sh = scatter_shape(nbins);
  const uint32_t nbw = (nbins + 7u) & ~7u;
  uint32_t launch_tiles = 0, max_tiles = 0;
  for (uint32_t k = 0; k < count; ++k) {
    launch_tiles += ntiles[k];
    max_tiles = std::max(max_tiles, ntiles[k]);
  }
  uint32_t tc = tc_knob ? std::min(tc_knob, sh.tc) : sh.tc;
  p.noscan = max_tiles <= tc;
  if (!p.noscan && !tc_knob) {
    const uint32_t per = std::max(1u, launch_tiles / std::max(cus, 1u));
    while (tc > 1 && tc > per) tc /= 2;
  }
  p.tc = tc;
  uint32_t chunks = 0;
  size_t self_bytes = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const uint32_t ch = (ntiles[k] + tc - 1) / tc;
    chunks += ch;
    self_bytes += (size_t)ch * ntiles[k] * nbw * 2;
  }
  p.selfscan = !p.noscan && nbw <= 2 * 512 && chunks <= std::max(cus, 1u) &&
               self_bytes <= (size_t)selfscan_kb * 1024 && scatter_lds(nbins, tc, true) <= 64u * 1024u;
  const uint32_t nbb = (nbw + USN_SCAN_BLK - 1) / USN_SCAN_BLK;
  uint32_t cpt = 4;
  while (cpt > 1 && (chunks / (16 * cpt)) * nbb < 256) cpt /= 2;
  p.cpt = cpt_knob ? cpt_knob : cpt;
  return p;
}

/* the granule and diag part of a batch's scratch (zeroed on its first use
 * with this geometry) */
void scatter_tail(void *scratch, uint64_t cap, uint32_t nbins, void **p, size_t *bytes) {
  const ScatterGeom g = scatter_geom(cap, nbins);
  *p = static_cast<uint8_t *>(scratch) + g.gran;
  *bytes = g.total - g.gran;
}
}  // namespace usn

extern "C" {

int usn_abi_version(void) { return USN_ABI_VERSION; }
int usn_last_hip_error(void) { return g_last_hip; }

const char *usn_strerror(int s) {
  switch (s) {
    case USN_OK: return "ok";
    case USN_EINVAL: return "invalid argument";
    case USN_ENOMEM: return "out of memory";
    case USN_EEXIST: return "exists";
    case USN_ENOENT: return "not found";
    case USN_EPERM: return "not permitted";
    case USN_EHIP: return "HIP runtime error";
    case USN_ENODEV: return "no gfx950 device";
    case USN_ERANGE: return "out of range";
    case USN_EBUSY: return "a tx batch awaits usn_finalize";
    case USN_ELIST: return "per-endpoint lists inconsistent with the decisions";
    default: return "unknown";
  }
}

int usn_ctx_create(int hip_device, usn_ctx **out) {
  if (!out) return USN_EINVAL;
  *out = nullptr;
  if (hip_device == USN_HOST_ONLY) {   // registry only: the control plane without a GPU
    usn_ctx *c = new (std::nothrow) usn_ctx();
    if (!c) return USN_ENOMEM;
    c->device = -1;
    c->ph_load = ph_load_knob();
    c->ph_group = ph_group_knob();
    *out = c;
    return USN_OK;
  }
  return usn_ctx_create_group(&hip_device, 1, out);
}

int usn_ctx_create_group(const int *hip_devices, uint32_t n, usn_ctx **out) {
  if (!out || !hip_devices || n == 0 || n > USN_MAX_REPLICAS) return USN_EINVAL;
  *out = nullptr;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  std::vector<Replica> reps(n);
  for (uint32_t i = 0; i < n; ++i) {
    const int d = hip_devices[i];
    if (d < 0 || d >= ndev) return USN_ENODEV;
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, d));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return USN_ENODEV;
    reps[i].device = d;
    reps[i].n_cu = prop.multiProcessorCount;
  }
  HIPCHK(hipSetDevice(hip_devices[0]));
  usn_ctx *c = new (std::nothrow) usn_ctx();
  if (!c) return USN_ENOMEM;
  c->reps.swap(reps);
  c->device = hip_devices[0];
  if (const char *e = test_knob("USN_T512")) c->t512 = std::atoi(e) ? 1 : 0;
  if (const char *e = test_knob("USN_TX_T512")) c->tx512 = std::atoi(e) ? 1 : 0;
  c->ph_load = ph_load_knob();
  c->ph_group = ph_group_knob();
  if (const char *e = test_knob("USN_RX_EV")) c->rx_ev_mode = std::atoi(e);
  if (const char *e = test_knob("USN_RX_STATE")) c->rx_state_on = std::atoi(e) != 0;
  if (const char *e = test_knob("USN_TIMING_EV"))
    c->timing_ev_flags = std::atoi(e) == 1 ? hipEventReleaseToDevice
                       : std::atoi(e) == 2 ? hipEventDisableSystemFence : hipEventDefault;
  *out = c;
  return USN_OK;
}

int usn_ctx_replicas(usn_ctx *c) {
  if (!c) return USN_EINVAL;
  return (int)c->reps.size();
}

int usn_replica_select(usn_ctx *c, uint32_t replica) {
  if (!c) return USN_EINVAL;
  if (c->reps.empty()) return USN_ENODEV;
  if (replica >= c->reps.size()) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->sel = replica;
  c->device = c->reps[replica].device;
  HIPCHK(hipSetDevice(c->device));
  return USN_OK;
}

int usn_replica_device(usn_ctx *c, uint32_t replica) {
  if (!c) return USN_EINVAL;
  if (replica >= c->reps.size()) return USN_EINVAL;
  return c->reps[replica].device;
}

void usn_ctx_destroy(usn_ctx *c) {
  if (!c) return;
  for (Replica &R : c->reps) {
    (void)hipSetDevice(R.device);
    (void)hipDeviceSynchronize();
    for (void *p : {(void *)R.d_table, R.d_patch, (void *)R.d_bridge, (void *)R.d_bridge_set,
                    (void *)R.aux, (void *)R.macset, (void *)R.ruleset, (void *)R.txs[0].learned,
                    (void *)R.txs[0].counters, (void *)R.txs[1].learned, (void *)R.txs[1].counters,
                    (void *)R.listen})
      if (p) (void)hipFree(p);
  }
  for (auto &kv : c->lists_ev)
    if (kv.second.ev) {
      (void)hipSetDevice(kv.second.device);
      (void)hipEventDestroy(kv.second.ev);
    }
  for (Replica &R : c->reps) {
    (void)hipSetDevice(R.device);
    if (R.classified) (void)hipEventDestroy(R.classified);
    for (hipEvent_t e : R.rx_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto &x : R.txs)
      if (x.txstate_ev) (void)hipEventDestroy(x.txstate_ev);
    if (R.side) (void)hipStreamDestroy(R.side);
  }
  for (Chain &ch : c->chains)
    for (uint32_t k = 0; k < USN_MAX_REPLICAS; ++k)
      if (ch.done[k]) {
        (void)hipSetDevice(c->reps[k].device);
        (void)hipEventDestroy(ch.done[k]);
      }
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->h_patch) (void)hipHostFree(c->h_patch);
  if (c->h_txstate) (void)hipHostFree(c->h_txstate);
  if (c->h_rxstate) (void)hipHostFree(c->h_rxstate);
  if (c->h_lists) (void)hipHostFree(c->h_lists);
  if (c->h_items) (void)hipHostFree(c->h_items);
  delete c;
}

int usn_endpoint_add(usn_ctx *c, uint16_t id, int kind, int32_t for_nic) {
  if (!c || id >= USN_MAX_ENDPOINTS || kind < USN_EP_NIC || kind > USN_EP_UDS) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  if (c->eps[id].used) return USN_EEXIST;
  if ((kind == USN_EP_NIC) != (for_nic < 0)) return USN_EINVAL;   // main.rs:157-159
  if (for_nic >= 0 && (for_nic >= USN_MAX_ENDPOINTS || !c->eps[for_nic].used ||
                       c->eps[for_nic].kind != USN_EP_NIC))
    return USN_EINVAL;
  Ep &e = c->eps[id];
  e = Ep();
  e.used = true;
  e.kind = kind;
  e.for_nic = for_nic;
  e.listen_ver = ++c->listen_gen;
  c->n_ep = std::max<uint32_t>(c->n_ep, (uint32_t)id + 1);
  c->chains[id] = Chain();
  return USN_OK;
}

int usn_endpoint_remove(usn_ctx *c, uint16_t id) {
  if (!c || id >= USN_MAX_ENDPOINTS) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  if (!c->eps[id].used) return USN_ENOENT;
  for (auto it = c->rules.begin(); it != c->rules.end();) {   // match_register.retain
    if (it->second.owner == id) {
      it = c->rules.erase(it);
      c->table_dirty = true;
    } else {
      ++it;
    }
  }
  c->eps[id] = Ep();
  c->chains[id] = Chain();
  return USN_OK;
}

int usn_add_match(usn_ctx *c, const usn_want *w, uint16_t owner, int sticky) {
  if (!c || !w || owner >= USN_MAX_ENDPOINTS) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  Ep &e = c->eps[owner];
  if (!e.used) return USN_ENOENT;
  const WantKey k = canon(*w);
  if (c->rules.count(k)) return 0;                                   // main.rs:272-274
  e.listen_ver = ++c->listen_gen;
  e.listening.push_back(Listen{k.dst, k.proto, (uint8_t)((k.present & USN_WANT_DPORT) ? 1 : 0),
                               k.dport});                            // main.rs:276-279
  if (e.for_nic < 0) return USN_EPERM;                                // main.rs:287-289 panics
  cache_clear(c, e.for_nic);                                          // main.rs:280-286
  rule_insert(c, k, Rule{owner, (uint8_t)(sticky ? 1 : 0)});
  return 1;
}

int usn_remove_match(usn_ctx *c, const usn_want *w, uint16_t requester) {
  if (!c || !w) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  const WantKey k = canon(*w);
  auto it = c->rules.find(k);
  if (it == c->rules.end()) return 0;
  if (it->second.owner != requester) return USN_EPERM;               // main.rs:612-616
  c->rules.erase(it);
  note_change(c, k);
  return 1;
}

int usn_rule_count(usn_ctx *c) {
  if (!c) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  return (int)c->rules.size();
}

int usn_rules_get(usn_ctx *c, usn_want *w, uint16_t *owner, uint8_t *sticky, uint32_t cap) {
  if (!c) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  uint32_t n = 0;
  for (const auto &kv : c->rules) {
    if (n >= cap) break;
    if (w) {
      usn_want &o = w[n];
      std::memset(&o, 0, sizeof o);
      o.dst_addr = kv.first.dst;
      o.src_addr = kv.first.src;
      o.dst_port = kv.first.dport;
      o.src_port = kv.first.sport;
      o.protocol = kv.first.proto;
      o.present = kv.first.present;
    }
    if (owner) owner[n] = kv.second.owner;
    if (sticky) sticky[n] = kv.second.sticky;
    ++n;
  }
  return (int)n;
}

int usn_lookup(usn_ctx *c, const usn_want *w) {
  if (!c || !w) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  const int e = registry_get(c, canon(*w));
  return e < 0 ? USN_ENOENT : e;
}

int usn_bridge_add(usn_ctx *c, const uint8_t mac[6]) {
  if (!c || !mac) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  c->bridge.push_back(mac48(mac));
  c->bridge_dirty = true;
  return USN_OK;
}

int usn_bridge_set(usn_ctx *c, const uint8_t (*macs)[6], uint32_t n) {
  if (!c || (n && !macs)) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  c->bridge.clear();
  for (uint32_t i = 0; i < n; ++i) c->bridge.push_back(mac48(macs[i]));
  c->bridge_dirty = true;
  return USN_OK;
}

int usn_table_build(usn_ctx *c, const usn_rule *rules, uint32_t n) {
  if (!c || (n && !rules)) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  for (uint32_t i = 0; i < n; ++i)
    if (rules[i].endpoint >= USN_MAX_ENDPOINTS || !c->eps[rules[i].endpoint].used)
      return USN_ENOENT;
  c->rules.clear();
  c->rules.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    usn_want w;
    std::memset(&w, 0, sizeof w);
    w.dst_addr = rules[i].dst_addr;
    w.src_addr = rules[i].src_addr;
    w.dst_port = rules[i].dst_port;
    w.src_port = rules[i].src_port;
    w.protocol = rules[i].protocol;
    w.present = rules[i].present & 7u;
    c->rules.emplace(canon(w), Rule{rules[i].endpoint,
                                    (uint8_t)((rules[i].present & USN_RULE_STICKY) ? 1 : 0)});
  }
  for (int e = 0; e < USN_MAX_ENDPOINTS; ++e)
    if (c->eps[e].used && c->eps[e].kind == USN_EP_NIC) cache_clear(c, e);
  c->table_dirty = true;
  return (int)c->rules.size();
}

int usn_bridge_count(usn_ctx *c) {
  if (!c) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  return (int)c->bridge.size();
}

int usn_frag_clear(usn_ctx *c) {
  if (!c) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  c->frags.clear();
  return USN_OK;
}

int usn_set_frame_reader(usn_ctx *c, usn_frame_reader fn, void *user) {
  if (!c) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  c->reader = fn;
  c->reader_user = user;
  return USN_OK;
}

/* Test hook (not in the public header): the device image's lookup of one
 * packed key, computed on the host image (table 0 = K1, 1 = K2).  Builds
 * the image if the registry changed.  Returns the slot's meta word, 0 = miss. */
int64_t usn_debug_image_probe(usn_ctx *c, int table, uint32_t x, uint32_t y, uint32_t z,
                              uint32_t meta) {
  if (!c || table < 0 || table > 1) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  { const int s = refresh_image(c); if (s) return s; }
  return (int64_t)image_probe(c, table, x, y, z, meta);
}

/* Test hook: get_endpoint's lookups for one parsed IPv4 frame, through U / X
 * (out[0], out[1]) and through K1 / K2 (out[2], out[3]), each normalised to
 * 0 (miss), 0x10000 | owner, or 0x11FFE (a NIC owns the rule).  Returns 1
 * when U is built, 0 when not. */
int usn_debug_image_probe_rx(usn_ctx *c, uint32_t dst, uint32_t src, uint32_t proto, uint32_t has,
                             uint32_t dport, uint32_t sport, uint32_t *out4) {
  if (!c || !out4) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  { const int s = refresh_image(c); if (s) return s; }
  auto norm = [](uint32_t w) {
    return w == 0 ? 0u : 0x10000u | ((w & USN_SLOT_NICOWNER) ? USN_U_NIC : (w >> 16));
  };
  uint32_t wu[2];
  image_probe_u(c, dst, src, proto, has, dport, sport, wu);
  const uint32_t w1 = image_probe(c, 0, dst, src, has ? (dport | sport << 16) : 0u,
                                  usn_key_meta(proto, has ? (USN_WANT_DPORT | USN_WANT_SRC | USN_WANT_SPORT)
                                                          : USN_WANT_SRC));
  const uint32_t w2 = image_probe(c, 1, dst, 0u, has ? dport : 0u, usn_key_meta(proto, has ? USN_WANT_DPORT : 0u));
  out4[0] = norm(wu[0]); out4[1] = norm(wu[1]); out4[2] = norm(w1); out4[3] = norm(w2);
  return (c->probe_mask & 4u) ? 1 : 0;
}

/* Test hook: the image's geometry {m0, g0, m1, g1, units, probe_mask, mU, mX,
 * gU, gX} (slots and groups of each table, all shards). */
int usn_debug_image_info(usn_ctx *c, uint32_t *out6) {
  if (!c || !out6) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  { const int s = refresh_image(c); if (s) return s; }
  for (int i = 0; i < 2; ++i) {   // totals over the shards
    out6[2 * i] = c->img_t[i].m << c->img_t[i].shift;
    out6[2 * i + 1] = c->img_t[i].g << c->img_t[i].shift;
  }
  out6[4] = (uint32_t)c->img.size(); out6[5] = c->probe_mask;
  out6[6] = c->img_t[2].m << c->img_t[2].shift;
  out6[7] = c->img_t[3].m << c->img_t[3].shift;
  out6[8] = c->img_t[2].g << c->img_t[2].shift;
  out6[9] = c->img_t[3].g << c->img_t[3].shift;
  return USN_OK;
}

/* Test hook: {full image builds, incremental updates, registry changes not
 * yet in the image, image version} -- after bringing the image up to date
 * when `refresh` is set */
/* test hook (tests/test_scatter_plan.py, no GPU): the list plan of a launch
 * of `count` batches of ntiles[k] tiles and nbins bins on `cus` CUs, with the
 * default knobs: out4 = {chunk tiles, scan chunks per thread, noscan, selfscan} */
int usn_debug_scatter_plan(const uint32_t *ntiles, uint32_t count, uint32_t nbins, uint32_t cus,
                           uint32_t *out4) {
  if (!ntiles || !out4 || count == 0 || count > USN_MAX_MULTI || nbins == 0 || nbins > USN_MAX_BINS)
    return USN_EINVAL;
  const usn::ScatterPlan p = usn::scatter_plan(ntiles, count, nbins, cus, 0, 0, 16384);
  out4[0] = p.tc;
  out4[1] = p.cpt;
  out4[2] = p.noscan ? 1u : 0u;
  out4[3] = p.selfscan ? 1u : 0u;
  return USN_OK;
}

int usn_debug_image_stats(usn_ctx *c, int refresh, uint64_t *out4) {
  if (!c || !out4) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (refresh) { const int s = refresh_image(c); if (s) return s; }
  out4[0] = c->img_builds;
  out4[1] = c->img_updates;
  out4[2] = c->img_delta.size();
  out4[3] = c->table_version;
  return USN_OK;
}

/* Test hook: the tx scratch state of the selected replica's latest launch:
 * counters[0..7] (learned, flags, sets used, timed-out epoch, and the
 * host-stage frames of rings 0..3 ONLY; a launch takes up to USN_TX_RINGS = 8
 * rings, whose host-stage counters [4 + k] for k >= 4 and learned items
 * [12 + k] (usn_kernels.h USN_TXC_*) this hook does not expose), epoch. */
int usn_debug_tx_state(usn_ctx *c, uint32_t *out10) {
  if (!c || !out10 || c->reps.empty()) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  Replica &R = c->reps[c->sel];
  std::memset(out10, 0, 10 * sizeof(uint32_t));
  const uint32_t slot = c->txq.empty() ? (c->tx_next_slot ^ 1u) : c->txq.back().slot;   // the latest
  if (R.txs[slot].counters) {
    HIPCHK(hipSetDevice(R.device));
    HIPCHK(hipMemcpy(out10, R.txs[slot].counters, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  out10[8] = R.epoch;
  return USN_OK;
}

int usn_cache_clear(usn_ctx *c, uint16_t ep) {
  if (!c || ep >= USN_MAX_ENDPOINTS) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->txq.empty()) return USN_EBUSY;
  cache_clear(c, ep);
  return USN_OK;
}

/* ---- result layout ------------------------------------------------------- */
static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }


struct Layout {
  size_t dec, index, bin_off, tiles, summary, host, scratch, total;
};
static Layout layout_for(uint64_t n, uint32_t nbins) {
  const uint64_t nt = (n + USN_TILE - 1) / USN_TILE;
  Layout L;
  size_t off = 0;
  L.dec = off; off = align256(off + n * 4);
  L.index = off; off = align256(off + (n + USN_TILE) * 4);   // + a tile of sink slots (the scatter's
                                                           // lanes past a ragged tile's end)
  L.bin_off = off; off = align256(off + (size_t)(USN_MAX_BINS + 1) * 4);
  L.tiles = off; off = align256(off + nt * sizeof(usn_tile_hdr));
  L.summary = off; off = align256(off + sizeof(usn_summary));
  L.host = off; off = align256(off + nt * USN_TILE * 4);
  L.scratch = off; off = align256(off + usn::scatter_scratch_bytes(n, nbins));
  L.total = off;
  return L;
}

size_t usn_result_bytes(uint64_t n) { return layout_for(n, USN_MAX_BINS).total; }
size_t usn_result_bytes_ep(uint64_t n, uint32_t max_endpoints) {
  if (max_endpoints > USN_MAX_ENDPOINTS) max_endpoints = USN_MAX_ENDPOINTS;
  return layout_for(n, max_endpoints + 3).total;
}

int usn_result_bind(void *mem, size_t bytes, uint64_t n, usn_result *out) {
  if (!mem || !out || n == 0) return USN_EINVAL;
  const Layout L = layout_for(n, 3);   // the fixed part and the smallest scratch
  if (bytes < L.total) return USN_ERANGE;
  // the most bins the scratch holds
  uint32_t lo = 3, hi = USN_MAX_BINS;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) / 2;
    if (L.scratch + usn::scatter_scratch_bytes(n, mid) <= bytes) lo = mid; else hi = mid - 1;
  }
  uint8_t *b = static_cast<uint8_t *>(mem);
  out->decisions = reinterpret_cast<uint32_t *>(b + L.dec);
  out->index = reinterpret_cast<uint32_t *>(b + L.index);
  out->bin_off = reinterpret_cast<uint32_t *>(b + L.bin_off);
  out->tiles = reinterpret_cast<usn_tile_hdr *>(b + L.tiles);
  out->summary = reinterpret_cast<usn_summary *>(b + L.summary);
  out->host_list = reinterpret_cast<uint32_t *>(b + L.host);
  out->scratch = b + L.scratch;
  out->n = n;
  out->max_bins = lo;
  static std::atomic<uint32_t> tags{0};
  uint32_t t;
  do t = tags.fetch_add(1, std::memory_order_relaxed) + 1; while (t == 0);
  out->bind_tag = t;
  return USN_OK;
}

/* ---- the hot path ----------------------------------------------------------- */
/* a batch's bins (nbins = endpoints + 3) in its classify args, and the
 * count rows carved for them */
static void set_bins(const usn_result *r, uint64_t n, uint32_t nbins, usn::ClassifyArgs &a) {
  a.nbins = nbins;
  a.n_ep = nbins - 3;
  a.nbits = 1;
  while ((1u << a.nbits) < a.nbins) ++a.nbits;
  usn::ScatterBatch sb;
  usn::scatter_carve(r->scratch, r->n, n, nbins, 1, 1, sb, &a.cnt);
  a.nbw = (nbins + 7u) & ~7u;
}

static int fill_args(usn_ctx *c, const Replica &R, const usn_batch *b, const usn_result *r,
                     ClassifyArgs &a) {
  std::memset(&a, 0, sizeof a);
  a.frames = b->frames;
  a.stride = b->stride;
  a.offsets = b->offsets;
  a.lens = b->lens;
  a.n = b->n;
  a.ntiles = (uint32_t)((b->n + USN_TILE - 1) / USN_TILE);
  a.window = b->window ? b->window : USN_WINDOW;
  a.decisions = r->decisions;
  a.tiles = r->tiles;
  a.summary = r->summary;
  a.host_list = r->host_list;
  a.table = R.d_table;
  a.table_units = c->img_base;
  a.disp_unit = c->img_t[1].slot_off + (c->img_t[1].m << c->img_t[1].shift);
  for (int i = 0; i < 4; ++i) a.ph[i] = c->img_t[i];
  a.u_disp_unit = c->img_udisp;
  a.u_end_unit = (uint32_t)c->img.size();
  a.bridge = R.d_bridge;
  a.n_bridge = (uint32_t)c->bridge.size();
  const Ep &S = c->eps[b->src_endpoint];
  a.src = b->src_endpoint;
  a.src_is_nic = S.kind == USN_EP_NIC;
  a.for_nic = S.for_nic < 0 ? 0xFFFFu : (uint32_t)S.for_nic;
  a.next_dhcp_set = S.next_dhcp >= 0 ? 1u : 0u;
  a.n_ep = c->n_ep;
  a.nbins = c->n_ep + 3;
  a.nbits = 1;
  while ((1u << a.nbits) < a.nbins) ++a.nbits;
  a.probe_mask = c->probe_mask;
  usn::ScatterBatch sb;
  usn::scatter_carve(r->scratch, r->n, b->n, a.nbins, 1, 1, sb, &a.cnt);
  a.nbw = (a.nbins + 7u) & ~7u;
  return USN_OK;
}

/* the per-endpoint scatter of `count` classified batches (after their
 * classify / tx launch, or after finalize recounted patched tiles) */
/* a launch's tag: the scan's granules and a batch's rx state carry it (0 is
 * what zeroed granules hold) */
static uint32_t next_epoch(usn_ctx *c) {
  if (++c->scan_epoch == 0) c->scan_epoch = 1;
  return c->scan_epoch;
}

/* the lists' plan of a launch (usn::scatter_plan, with the A/B knobs of the
 * test build) */
static usn::ScatterPlan plan_lists(usn_ctx *c, const usn::ClassifyArgs *as, uint32_t count) {
  uint32_t ntl[USN_MAX_MULTI];
  for (uint32_t k = 0; k < count; ++k) ntl[k] = as[k].ntiles;
  int cus = 256;   // the replica's CUs, queried once
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
      for (Replica &R : c->reps)
        if (R.device == dev) {
          if (!R.n_cu) (void)hipDeviceGetAttribute(&R.n_cu, hipDeviceAttributeMultiprocessorCount, dev);
          if (R.n_cu > 0) cus = R.n_cu;
          break;
        }
    }
  }
  static const uint32_t tc_knob = [] {   // A/B: USN_SCATTER_TC=1|2|4|8 (at most the shape's)
    const char *e = test_knob("USN_SCATTER_TC");
    const int v = e ? std::atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4 || v == 8) ? (uint32_t)v : 0u;
  }();
  static const uint32_t cpt_knob = [] {   // A/B: USN_SCAN_CPT=1|2|4
    const char *e = test_knob("USN_SCAN_CPT");
    const int v = e ? std::atoi(e) : 0;
    return (v == 1 || v == 2 || v == 4) ? (uint32_t)v : 0u;
  }();
  static const uint32_t selfscan_kb = [] {   // A/B: USN_SELFSCAN_KB (row KiB all chunks read; 0 off)
    const char *e = test_knob("USN_SELFSCAN_KB");
    return e ? (uint32_t)std::atoi(e) : 16384u;
  }();
  return usn::scatter_plan(ntl, count, as[0].nbins, (uint32_t)std::max(cus, 1), tc_knob, cpt_knob,
                           selfscan_kb);
}

/* the per-endpoint scatter of `count` classified batches (after their
 * classify / tx launch, or after finalize recounted patched tiles); epoch:
 * the launch's tag when its classify took one; rx_state: the batches' state
 * slots for usn_finalize (host-mapped) */
static int launch_scatter(usn_ctx *c, const usn::ClassifyArgs *as, const usn_result *r,
                          uint32_t count, hipStream_t s, uint32_t *txs_out = nullptr,
                          const uint32_t *txs_counters = nullptr, uint32_t epoch = 0,
                          uint32_t *const *rx_state = nullptr, hipEvent_t done = nullptr) {
  usn::ScatterArgs x;
  std::memset(&x, 0, sizeof x);
  x.count = count;
  x.nbins = as[0].nbins;
  x.nbw = as[0].nbw;
  x.n_ep = as[0].n_ep;
  x.nbits = as[0].nbits;
  const usn::ScatterPlan pl = plan_lists(c, as, count);
  const uint32_t tc = pl.tc;
  x.tc = tc;
  static const bool slow_rank = test_knob("USN_SCATTER_SLOW_RANK") != nullptr;
  x.flags = (slow_rank ? USN_SCF_SLOW_RANK : 0u) | (pl.noscan ? USN_SCF_NOSCAN : 0u) |
            (pl.selfscan ? USN_SCF_SELFSCAN : 0u);
  x.nbb = (x.nbw + USN_SCAN_BLK - 1) / USN_SCAN_BLK;
  x.cpt = pl.cpt;
  x.txs_out = txs_out;
  x.txs_counters = txs_counters;
  if (!epoch) epoch = next_epoch(c);   // (the classify of this launch took one already)
  x.epoch = epoch;
  for (uint32_t k = 0; k < count; ++k) {
    usn::ScatterBatch &sb = x.b[k];
    uint16_t *cnt;
    usn::scatter_carve(r[k].scratch, r[k].n, as[k].n, x.nbins, tc, x.cpt, sb, &cnt);
    sb.decisions = r[k].decisions;
    sb.index = r[k].index;
    sb.bin_off = r[k].bin_off;
    sb.rx_state = rx_state ? rx_state[k] : nullptr;
    sb.summary = r[k].summary;
    x.chunk_base[k + 1] = x.chunk_base[k] + sb.nchunks;
    x.range_base[k + 1] = x.range_base[k] + sb.nranges;
    // granules of a scratch never used before may hold anything: zero them
    // after every bind, and again when the geometry moves them (their place
    // depends on the result's capacity and the bins)
    const uint64_t geo = (r[k].n << 16) ^ x.nbins;
    auto zi = c->scan_zeroed.find(r[k].scratch);
    if (zi == c->scan_zeroed.end() || zi->second.tag != r[k].bind_tag || zi->second.geo != geo) {
      c->scan_zeroed[r[k].scratch] = usn_ctx::Zeroed{r[k].bind_tag, geo};
      void *p;
      size_t bytes;
      usn::scatter_tail(r[k].scratch, r[k].n, x.nbins, &p, &bytes);
      HIPCHK(hipMemsetAsync(p, 0, bytes, s));
    }
  }
#if USN_TEST_HOOKS
  // test hook (tests/test_gpu_scatter.py, the test build only, read once per
  // process): USN_DEBUG_CORRUPT=1 sets bin 0 of batch 0's first count row to
  // 257, =2 makes frame 0's decision name endpoint 0x0FF0 (past every
  // batch's bins); the scatter must report either (usn_finalize: USN_ELIST)
  static const int corrupt = [] {
    const char *e = test_knob("USN_DEBUG_CORRUPT");
    return e ? std::atoi(e) : 0;
  }();
  if (corrupt == 1) HIPCHK(hipMemsetAsync(const_cast<uint16_t *>(x.b[0].cnt), 0x01, 2, s));
  if (corrupt == 2) HIPCHK(hipMemsetD32Async(r[0].decisions, (int)((1u << 16) | 0x0FF0u), 1, s));
#endif
  HIPCHK(usn_t512::launch_scatter(x, s, done));
  return USN_OK;
}

/* 512 threads per tile (two rounds per lane: both rounds' probes batched per
 * wave, displacements in LDS) for every layout, except when only the
 * 256-thread build can keep the image in LDS (its header stage is half as
 * big).  A/B, c4 (4096 rules, displacements in LDS), 8M frames per launch:
 * 161.8 us at 256 threads, 130.7 at 512 (profiles/r02h). */
static bool use_t512(uint32_t nbins, uint32_t units) {
  if (usn_t512::table_fits_lds(nbins, units)) return true;
  return !usn::table_fits_lds(nbins, units);
}

static int check_batch(usn_ctx *c, const usn_batch *b, const usn_result *r) {
  if (!b || !r || !b->frames || !b->lens || b->n == 0 || r->n < b->n) return USN_EINVAL;
  if ((b->stride == 0) == (b->offsets == nullptr)) return USN_EINVAL;
  const uint32_t window = b->window ? b->window : USN_WINDOW;
  if (window < USN_WINDOW) return USN_EINVAL;   // the header loads read 64 bytes
  if (b->stride && (b->stride % 16 != 0 || b->stride < window)) return USN_EINVAL;
  if (((uintptr_t)b->frames & 15) != 0) return USN_EINVAL;
  if (b->n > 0xFFFFFFFFull) return USN_ERANGE;
  if (b->src_endpoint >= USN_MAX_ENDPOINTS || !c->eps[b->src_endpoint].used) return USN_EINVAL;
  if (!r->scratch || !r->index || !r->bin_off || r->max_bins < c->n_ep + 3) return USN_ERANGE;
  return USN_OK;
}

/* device scratch of a tx batch of n frames on replica R; the epoch-tagged
 * sets are cleared only when (re)allocated or when the 16-bit epoch wraps */
static int tx_prepare(Replica &T, uint64_t n, uint32_t ntiles, uint32_t slot, bool in_flight) {
  Replica::TxSlot &X = T.txs[slot];
  if (n > X.learned_frames) {
    if (X.learned) HIPCHK(hipFree(X.learned));
    X.learned = nullptr;
    HIPCHK(hipMalloc(&X.learned, n * 4 * sizeof(uint4)));   // <= 2 items of 2 x uint4 per frame
    X.learned_frames = n;
    X.learned_cap = (uint32_t)(2 * n);
  }
  // below, buffers the batch in flight uses are replaced or cleared: only
  // after it has drained (rare: growth, or the 16-bit epoch wrapping)
  const uint32_t slots = next_pow2((uint32_t)std::max<uint64_t>(1024, 2 * n));   // load <= 1/2
  if (in_flight && (ntiles > T.aux_tiles || slots > T.set_slots || T.epoch + 1 > 0xFFFFu))
    HIPCHK(hipDeviceSynchronize());
  if (ntiles > T.aux_tiles) {   // zeroed: no flag holds an epoch yet
    if (T.aux) HIPCHK(hipFree(T.aux));
    T.aux = nullptr;
    // granules, then the packed EARLY words (TxArgs::early)
    HIPCHK(hipMalloc(&T.aux, (size_t)ntiles * usn::TXA_TILE_BYTES));
    HIPCHK(hipMemset(T.aux, 0, (size_t)ntiles * usn::TXA_TILE_BYTES));
    T.aux_tiles = ntiles;
  }
  if (!X.counters) {
    HIPCHK(hipMalloc(&X.counters, USN_TXC_WORDS * sizeof(uint32_t)));
    HIPCHK(hipMemset(X.counters, 0, USN_TXC_WORDS * sizeof(uint32_t)));
  }
  bool clear = false;
  if (slots > T.set_slots) {
    if (T.macset) HIPCHK(hipFree(T.macset));
    if (T.ruleset) HIPCHK(hipFree(T.ruleset));
    T.macset = nullptr; T.ruleset = nullptr;
    HIPCHK(hipMalloc(&T.macset, (size_t)slots * 2 * 8));
    HIPCHK(hipMalloc(&T.ruleset, (size_t)slots * 4 * 8));
    T.set_slots = slots;
    clear = true;
  }
  if (++T.epoch > 0xFFFFu) clear = true;
  if (clear) {
    HIPCHK(hipMemset(T.macset, 0, (size_t)T.set_slots * 2 * 8));
    HIPCHK(hipMemset(T.ruleset, 0, (size_t)T.set_slots * 4 * 8));
    HIPCHK(hipMemset(T.aux, 0, (size_t)T.aux_tiles * usn::TXA_TILE_BYTES));   // epoch-tagged flags
    // the slots' timeout marks (counters[3]: the epoch of a batch whose waits
    // timed out) hold epochs of the cycle that ends here (the device drained)
    for (auto &x : T.txs)
      if (x.counters) HIPCHK(hipMemset(x.counters + 3, 0, sizeof(uint32_t)));
    T.epoch = 1;
  }
  return USN_OK;
}

/* S.listening as {dst, proto | has_port << 8 | port << 16} words on the
 * device (uploaded when they changed since this replica's last tx batch) */
static int tx_listen(Replica &T, int src, const Ep &S, uint32_t &n_listen) {
  n_listen = (uint32_t)S.listening.size();
  if (T.listen_src == src && T.listen_ver == S.listen_ver) return USN_OK;
  std::vector<uint32_t> v;
  for (const Listen &l : S.listening) {
    v.push_back(l.dst);
    v.push_back((uint32_t)l.proto | ((uint32_t)l.has_port << 8) | ((uint32_t)l.port << 16));
  }
  if (v.empty()) return USN_OK;
  if (v.size() * 4 > T.listen_cap) {
    if (T.listen) HIPCHK(hipFree(T.listen));
    T.listen = nullptr;
    HIPCHK(hipMalloc(&T.listen, v.size() * 4));
    T.listen_cap = v.size() * 4;
  }
  HIPCHK(hipMemcpy(T.listen, v.data(), v.size() * 4, hipMemcpyHostToDevice));
  T.listen_src = src;
  T.listen_ver = S.listen_ver;
  return USN_OK;
}

/* A source's carried cache whose last batch ran on another replica (another
 * device): resolve it on the host from that batch's summary and tile headers,
 * as the kernel's resolve_carry would. */
static int chain_to_host(usn_ctx *c, Chain &ch) {
  HIPCHK(hipSetDevice(c->reps[ch.replica].device));
  // that batch may still be in flight on its (non-blocking) stream
  if (ch.done[ch.replica]) HIPCHK(hipEventSynchronize(ch.done[ch.replica]));
  usn_summary ps;
  HIPCHK(hipMemcpy(&ps, ch.summary, sizeof ps, hipMemcpyDeviceToHost));
  uint32_t st = 0, dst = 0, info[4] = {0, 0, 0, 0};
  if (ps.flags & USN_S_COUT) {
    st = ps.cout_state; dst = ps.cout_dst;
    std::memcpy(info, ps.cout_info, 16);
  } else {
    std::vector<usn_tile_hdr> th(ch.ntiles);
    if (ch.ntiles)
      HIPCHK(hipMemcpy(th.data(), ch.tiles, ch.ntiles * sizeof(usn_tile_hdr), hipMemcpyDeviceToHost));
    int best = -1;
    for (uint32_t t = 0; t < ch.ntiles; ++t)
      if (th[t].last_state & USN_TS_HAS) best = (int)t;
    if (best >= 0) {
      const usn_tile_hdr &h = th[best];
      if ((h.last_state & USN_TS_RETAINED) && !(h.last_state & USN_TS_UNKNOWN)) {
        st = USN_CS_VALID; dst = h.last_dst;
        std::memcpy(info, h.last_info, 16);
      }
    } else {
      st = ps.cin_state; dst = ps.cin_dst;
      std::memcpy(info, ps.cin_info, 16);
    }
  }
  ch.device_chain = false;
  ch.state = st;
  ch.dst = dst;
  std::memcpy(ch.info, info, 16);
  return USN_OK;
}

/* wait for an rx batch's own launch (classify + lists on its stream): its
 * completion event, unless the event's slot has since been re-recorded on
 * another stream (more than Replica::RX_EVS rx launches in flight over two or
 * more streams), which no longer orders this launch: then the device drains */
static int rx_wait(usn_ctx *c, const usn_ctx::BatchRec &rec) {
  Replica &R = c->reps[rec.rep];
  HIPCHK(hipSetDevice(R.device));
  if (R.rx_ev_gen[rec.ev_idx] == rec.ev_gen || R.rx_ev_stream[rec.ev_idx] == rec.stream)
    HIPCHK(hipEventSynchronize(rec.done));
  else
    HIPCHK(hipDeviceSynchronize());
  return USN_OK;
}

int usn_result_release(usn_ctx *c, const usn_result *r) {
  if (!c || !r || !r->decisions) return USN_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  for (const usn_ctx::Tx &t : c->txq)
    if (t.decisions == r->decisions) return USN_EBUSY;
  // an rx batch classified into r and not finalized: its kernels may still be
  // writing r, and the carried cache below is read from them
  const auto br = c->batch_rep.find(r->decisions);
  if (br != c->batch_rep.end() && br->second.done) { int e = rx_wait(c, br->second); if (e) return e; }
  const auto le = c->lists_ev.find(r->decisions);
  if (le != c->lists_ev.end() && le->second.ev) {   // lists on the side stream (after the classify)
    HIPCHK(hipSetDevice(le->second.device));
    HIPCHK(hipEventSynchronize(le->second.ev));   // the lists may still be built into r
  }
  for (Chain &ch : c->chains)   // a carried cache read from this result's tile headers
    if (ch.device_chain && ch.summary == r->summary) {
      const int s = chain_to_host(c, ch);
      if (s) return s;
    }
  if (br != c->batch_rep.end()) c->batch_rep.erase(br);
  if (le != c->lists_ev.end()) {
    if (le->second.ev) {
      HIPCHK(hipSetDevice(le->second.device));
      HIPCHK(hipEventDestroy(le->second.ev));
    }
    c->lists_ev.erase(le);
  }
  c->scan_zeroed.erase(r->scratch);
  for (const void *&t : c->txstate_for)
    if (t == r->decisions) t = nullptr;
  return USN_OK;
}

int usn_classify_multi(usn_ctx *c, const usn_batch *b, usn_result *r, uint32_t count,
                       void *stream) {
  if (!c || !b || !r || count == 0 || count > USN_MAX_MULTI) return USN_EINVAL;
  if (c->reps.empty()) return USN_ENODEV;
  HPROF_DECL
  std::lock_guard<std::mutex> g(c->mu);
  bool tx = false;
  for (uint32_t k = 0; k < count; ++k) {
    int st = check_batch(c, &b[k], &r[k]);
    if (st) return st;
    tx |= c->eps[b[k].src_endpoint].kind != USN_EP_NIC;
  }
  if (tx) {   // a tx launch changes shared state: one ring of a source, or up to 8 consecutive rings
    if (count > USN_TX_RINGS) return USN_EINVAL;
    uint64_t vend = 0;   // the launch's frame index (ring k after ring k - 1's tiles)
    for (uint32_t k = 0; k < count; ++k) {
      for (uint32_t j = 0; j < k; ++j)
        if (r[j].decisions == r[k].decisions || r[j].scratch == r[k].scratch) return USN_EINVAL;
      if (b[k].src_endpoint != b[0].src_endpoint) return USN_EINVAL;
      vend += k + 1 < count ? (b[k].n + USN_TILE - 1) / USN_TILE * USN_TILE : b[k].n;
    }
    if (vend >= 0xFFFFFFFFull) return USN_ERANGE;   // ... stays below 2^32 - 1
  } else {
    for (uint32_t k = 0; k < count; ++k)
      for (uint32_t j = 0; j < k; ++j)
        if (b[j].src_endpoint == b[k].src_endpoint) return USN_EINVAL;   // one batch per source
  }
  const uint32_t rep = c->sel;
  /* while tx batches are in flight: only the next ring(s) of the same source,
   * on the same stream and replica, and at most two launches in flight */
  if (!c->txq.empty()) {
    const usn_ctx::Tx &p = c->txq.back();
    if (!tx || c->txq.front().launch != p.launch || p.src != b[0].src_endpoint || p.replica != rep ||
        p.stream != (hipStream_t)stream)
      return USN_EBUSY;
    for (const usn_ctx::Tx &q : c->txq)
      for (uint32_t k = 0; k < count; ++k)
        if (q.decisions == r[k].decisions) return USN_EBUSY;
  }
  Replica &R = c->reps[rep];
  HPROF(1);
  /* the table-version fence: this replica sees every registry and bridge
   * change made before this call */
  { int s = upload_table(c, R); if (s) return s; }
  { int s = upload_bridge(c, R); if (s) return s; }
  for (uint32_t k = 0; k < count; ++k) {
    Chain &ch = c->chains[b[k].src_endpoint];
    if (ch.device_chain && ch.replica != rep) { int s = chain_to_host(c, ch); if (s) return s; }
  }
  HIPCHK(hipSetDevice(R.device));
  HPROF(2);
  usn::MultiArgs m;
  std::memset(&m, 0, sizeof m);
  m.count = count;
  for (uint32_t k = 0; k < count; ++k) {
    ClassifyArgs &a = m.b[k];
    fill_args(c, R, &b[k], &r[k], a);
    Chain &ch = c->chains[b[k].src_endpoint];
    if (ch.device_chain) {
      a.carry_mode = usn::CARRY_CHAIN;
      a.prev_tiles = ch.tiles;
      a.prev_ntiles = ch.ntiles;
      a.prev_summary = ch.summary;
    } else {
      a.carry_mode = usn::CARRY_EXPLICIT;
      a.cin_state = ch.state;
      a.cin_dst = ch.dst;
      std::memcpy(a.cin_info, ch.info, sizeof ch.info);
    }
    m.tile_base[k + 1] = m.tile_base[k] + a.ntiles;
  }
  HPROF(3);
  uint32_t slot = 0;
  uint32_t epoch = 0;        // rx: the launch tag (classify and lists)
  uint32_t rx_slot[USN_MAX_MULTI];
  uint32_t *rx_state[USN_MAX_MULTI];
  hipEvent_t rx_done = nullptr;   // rx, lists on the caller's stream: the launch's completion
  uint32_t rx_ev_idx = 0;
  if (tx) {
    const usn_batch &tb = b[0];
    slot = c->tx_next_slot;
    uint64_t n_all = 0;
    for (uint32_t k = 0; k < count; ++k) n_all += b[k].n;
    int st = tx_prepare(R, n_all, m.tile_base[count], slot, !c->txq.empty());
    if (st) return st;
    usn::TxArgs t;
    std::memset(&t, 0, sizeof t);
    t.rings = count;
    for (uint32_t k = 0; k < count; ++k) t.a[k] = m.b[k];
    for (uint32_t k = 0; k <= count; ++k) t.tile_base[k] = m.tile_base[k];
    st = tx_listen(R, tb.src_endpoint, c->eps[tb.src_endpoint], t.n_listen);
    if (st) return st;
    t.aux = R.aux;
    t.early = reinterpret_cast<uint32_t *>(R.aux + (size_t)R.aux_tiles * TXA_GRANULES);
    t.macset = R.macset;
    t.ruleset = R.ruleset;
    t.macset_mask = t.ruleset_mask = R.set_slots - 1;
    t.epoch = R.epoch;
    t.learned = R.txs[slot].learned;
    t.counters = R.txs[slot].counters;
    t.learned_cap = R.txs[slot].learned_cap;
    t.bridge_set = R.d_bridge_set;
    t.bridge_mask = c->bridge_mask;
    t.listen = R.listen;
    t.next_dhcp_set = t.a[0].next_dhcp_set;
    if (c->tx512) HIPCHK(usn_t512::launch_tx(t, (hipStream_t)stream));
    else HIPCHK(usn::launch_tx(t, (hipStream_t)stream));   // tile 0 zeroes t.counters[0..2]
    const uint64_t launch = ++c->tx_launches;
    for (uint32_t k = 0; k < count; ++k) {
      usn_ctx::Tx p;
      p.decisions = r[k].decisions;
      p.launch_dec = r[0].decisions;
      p.src = tb.src_endpoint;
      p.replica = rep;
      p.slot = slot;
      p.epoch = R.epoch;
      p.ring = k;
      p.rings = count;
      p.voff = m.tile_base[k] * USN_TILE;
      p.launch = launch;
      p.stream = (hipStream_t)stream;
      c->txq.push_back(p);
    }
    c->tx_chg = false;
    c->tx_next_slot ^= 1u;
  } else {
    /* a result whose lists are still being built on the side stream is not
     * overwritten before they are done */
    for (uint32_t k = 0; k < count; ++k) {
      auto it = c->lists_ev.find(r[k].decisions);
      if (it != c->lists_ev.end() && it->second.pending) {
        HIPCHK(hipStreamWaitEvent((hipStream_t)stream, it->second.ev, 0));
        it->second.pending = false;
      }
    }
    /* the batches' state for usn_finalize: a slot of host-mapped memory each,
     * written by the scatter (ScatterBatch::rx_state) */
    if (!c->h_rxstate)
      HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c->h_rxstate), usn_ctx::RX_SLOTS * 32,
                           hipHostMallocMapped | hipHostMallocCoherent));
    if (!R.d_rxstate) HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&R.d_rxstate), c->h_rxstate, 0));
    uint32_t *const d_rx = R.d_rxstate;
    epoch = next_epoch(c);
    for (uint32_t k = 0; k < count; ++k) {
      m.b[k].epoch = epoch;
      if (!c->rx_state_on) { rx_slot[k] = usn_ctx::RX_SLOTS; rx_state[k] = nullptr; continue; }
      rx_slot[k] = c->rx_next_slot++ % usn_ctx::RX_SLOTS;
      volatile uint32_t *h = c->h_rxstate + rx_slot[k] * 8;
      h[0] = 0;   // (the tag, until the scatter writes it)
      h[2] = 0;   // (set by any scatter chunk that finds inconsistent lists)
      rx_state[k] = d_rx + rx_slot[k] * 8;
    }
    HPROF(4);
    if (c->t512 == 1 || (c->t512 < 0 && use_t512(m.b[0].nbins, m.b[0].table_units)))
      HIPCHK(usn_t512::launch_classify(m, (hipStream_t)stream));   // large table in L2
    else
      HIPCHK(usn::launch_classify(m, (hipStream_t)stream));
    HPROF(5);
  }
  if (tx || !c->lists_async) {
    uint32_t *txs = nullptr;
    if (tx) {   // what usn_finalize reads first: written into host memory by the scatter's chunk 0
      if (!c->h_txstate) {
        HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c->h_txstate), 2 * TXSTATE_BYTES,
                             hipHostMallocMapped | hipHostMallocCoherent));
        c->h_txstate_cap = 2 * TXSTATE_BYTES;
      }
      if (!R.d_txstate) HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void **>(&R.d_txstate), c->h_txstate, 0));
      txs = R.d_txstate + slot * (TXSTATE_BYTES / 4);
      // word 11: set by any scatter chunk that finds inconsistent lists (the
      // slot's previous batch is final: its usn_finalize synchronised)
      reinterpret_cast<volatile uint32_t *>(c->h_txstate + slot * TXSTATE_BYTES)[11] = 0;
    }
    if (!tx && c->rx_ev_mode) {
      rx_ev_idx = R.rx_ev_next++ % Replica::RX_EVS;
      hipEvent_t &e = R.rx_ev[rx_ev_idx];
      if (!e)
        HIPCHK(hipEventCreateWithFlags(&e, USN_DONE_EV_FLAGS |
                                               (c->rx_ev_mode == 2 ? hipEventDisableSystemFence
                                                : c->rx_ev_mode == 3 ? hipEventReleaseToDevice : 0u)));
      R.rx_ev_gen[rx_ev_idx] = ++c->rx_ev_gen;
      R.rx_ev_stream[rx_ev_idx] = (hipStream_t)stream;
      rx_done = e;
    }
    hipEvent_t done = rx_done;   // the launch's completion: rx_ev, or the tx slot's
    if (tx) {
      Replica::TxSlot &X = R.txs[slot];
      if (!X.txstate_ev) HIPCHK(hipEventCreateWithFlags(&X.txstate_ev, USN_DONE_EV_FLAGS));
      done = X.txstate_ev;
    }
    /* The completion event bound to the scatter's own dispatch
     * (hipExtLaunchKernel's stop event, mode 4, the product's): recorded
     * behind it instead (hipEventRecord), it is a marker packet between this
     * launch and the next, which cost c3's calls of 4 x 256K frames 3.6 % and
     * their two-stream steps 5 % (profiles/r06/r06c, r06d).  Bound, it cost
     * the two-stream steps of c2's 8M-frame calls 1-1.5 % in the same A/Bs:
     * so bound for launches of at most USN_BIND_MAX_TILES tiles (mode 5) */
    HPROF(6);
    const bool bind = done && (c->rx_ev_mode == 4 ||
                               (c->rx_ev_mode == 5 && m.tile_base[count] <= USN_BIND_MAX_TILES));
    int st = launch_scatter(c, m.b, r, count, (hipStream_t)stream, txs, tx ? R.txs[slot].counters : nullptr,
                            epoch, tx ? nullptr : rx_state, bind ? done : nullptr);
    if (st) return st;
    if (done && !bind) HIPCHK(hipEventRecord(done, (hipStream_t)stream));
    if (tx) c->txstate_for[slot] = r[0].decisions;
    HPROF(7);
  } else {
    // the scatter on the side stream, after this launch; the caller's stream
    // goes on to the next batch (usn_finalize / usn_lists_wait join them)
    if (!R.side) HIPCHK(hipStreamCreateWithFlags(&R.side, hipStreamNonBlocking));
    if (!R.classified) HIPCHK(hipEventCreateWithFlags(&R.classified, hipEventDisableTiming));
    HIPCHK(hipEventRecord(R.classified, (hipStream_t)stream));
    HIPCHK(hipStreamWaitEvent(R.side, R.classified, 0));
    int st = launch_scatter(c, m.b, r, count, R.side, nullptr, nullptr, epoch, rx_state);
    if (st) return st;
    for (uint32_t k = 0; k < count; ++k) {
      usn_ctx::ListsEv &le = c->lists_ev[r[k].decisions];
      if (le.ev && le.device != R.device) {
        (void)hipSetDevice(le.device);
        (void)hipEventDestroy(le.ev);
        le.ev = nullptr;
        HIPCHK(hipSetDevice(R.device));
      }
      if (!le.ev) {
        HIPCHK(hipEventCreateWithFlags(&le.ev, hipEventDisableTiming));
        le.device = R.device;
      }
      HIPCHK(hipEventRecord(le.ev, R.side));
      le.pending = true;
    }
  }
  for (uint32_t k = 0; k < count; ++k) {
    Chain &ch = c->chains[b[k].src_endpoint];
    ch.device_chain = true;
    ch.replica = rep;
    ch.tiles = r[k].tiles;
    ch.ntiles = m.b[k].ntiles;
    ch.summary = r[k].summary;
    if (c->reps.size() > 1) {   // only a move to another replica reads the chain on the host
      if (!ch.done[rep]) HIPCHK(hipEventCreateWithFlags(&ch.done[rep], hipEventDisableTiming));
      HIPCHK(hipEventRecord(ch.done[rep], (hipStream_t)stream));
    }
    c->batch_rep[r[k].decisions] =
        usn_ctx::BatchRec{rep, m.b[k].nbins, tx ? usn_ctx::RX_SLOTS : rx_slot[k], epoch, rx_done,
                          rx_ev_idx, rx_done ? c->rx_ev_gen : 0, (hipStream_t)stream};
  }
  HPROF(8);
#if USN_TEST_HOOKS
  g_hprof[15] += 1;
#endif
  return USN_OK;
}

#if USN_TEST_HOOKS
/* test build only (not in include/usn_classify.h): the accumulated host ns
 * per checkpoint of usn_classify_multi, [15] = calls */
int usn_debug_host_prof(uint64_t *out16, int reset) {
  for (int k = 0; k < 16; ++k) out16[k] = g_hprof[k];
  if (reset) std::memset(g_hprof, 0, sizeof g_hprof);
  return USN_OK;
}
#endif

int usn_classify(usn_ctx *c, const usn_batch *b, usn_result *r, void *stream) {
  return usn_classify_multi(c, b, r, 1, stream);
}

/* ---- ordered host stage --------------------------------------------------- */
namespace {

uint32_t batch_window(const usn_batch *b) { return b->window ? b->window : USN_WINDOW; }

/* internal: finalize_tx refused before any side effect for want of a frame
 * reader (usn_finalize returns USN_EINVAL and keeps the batch pending) */
constexpr int USN_EAGAIN_READER = -1000;

/* extract_pkt_info would read the L4 ports (pkt.rs:177-186, bytes 14+hl ..
 * 17+hl) past the first `have` bytes of this frame: the kernel's status 5 */
bool ports_past(const uint8_t *f, uint32_t len, uint32_t have) {
  if (len < 34 || be16(f + 12) != 0x0800) return false;
  const uint32_t n = len - 14, hl = (f[14] & 0x0Fu) * 4, tl = be16(f + 16);
  if (n < hl || hl > tl || n < tl || (be16(f + 20) & 0x1FFF)) return false;
  const uint32_t proto = f[23];
  const bool pp = proto == 6 || proto == 17 || proto == 0x21 || proto == 0x84 || proto == 0x88;
  return pp && (tl - hl) > 4 && 18 + hl > have;
}

/* frames the device left to the host because their ports lie past the
 * window need the host frame reader */
bool needs_reader(const std::vector<uint32_t> &dec, const std::vector<uint32_t> &hosts) {
  for (uint32_t j : hosts)
    if (USN_DEC_REASON(dec[j]) == USN_R_WINDOW && (dec[j] & USN_F_HOST)) return true;
  return false;
}

struct HostView {   // lazily fetched device data of one batch
  usn_ctx *c;
  const usn_batch *b;
  const usn_result *r;
  hipStream_t s;
  std::vector<uint32_t> dec;     // decisions (fetched whole on first need)
  std::vector<uint16_t> lens;
  bool have_dec = false, have_lens = false;

  int fetch_dec() {
    if (have_dec) return USN_OK;
    dec.resize(b->n);
    HIPCHK(hipMemcpy(dec.data(), r->decisions, b->n * 4, hipMemcpyDeviceToHost));
    have_dec = true;
    return USN_OK;
  }
  int fetch_lens() {
    if (have_lens) return USN_OK;
    lens.resize(b->n);
    HIPCHK(hipMemcpy(lens.data(), b->lens, b->n * 2, hipMemcpyDeviceToHost));
    have_lens = true;
    return USN_OK;
  }
  /* the bytes of frame i that extract_pkt_info reads: the batch window from
   * the device, or, when its ports lie past the window, min(len, 80) bytes
   * from the host frame reader (usn_set_frame_reader) */
  int frame(uint64_t i, std::vector<uint8_t> &buf, uint32_t &len) {
    int s = fetch_lens();
    if (s) return s;
    len = lens[i];
    uint64_t off;
    if (b->offsets) HIPCHK(hipMemcpy(&off, b->offsets + i, 8, hipMemcpyDeviceToHost));
    else off = i * b->stride;
    const uint32_t have = std::min<uint32_t>(batch_window(b), USN_WINDOW_MAX);
    buf.assign(USN_WINDOW_MAX, 0);
    HIPCHK(hipMemcpy(buf.data(), b->frames + off, have, hipMemcpyDeviceToHost));
    if (ports_past(buf.data(), len, have)) {
      if (!c->reader) return USN_EINVAL;
      const int got = c->reader(c->reader_user, b->src_endpoint, i, buf.data(), USN_WINDOW_MAX);
      if (got < 0 || (uint32_t)got < std::min<uint32_t>(len, USN_WINDOW_MAX)) return USN_EINVAL;
    }
    return USN_OK;
  }
};

bool touches(uint32_t d) {
  return !(USN_DEC_CLASS(d) == USN_CLS_DROP &&
           (USN_DEC_REASON(d) == USN_R_PARSE || USN_DEC_REASON(d) == USN_R_FRAGMISS));
}
bool retains(uint32_t d) {
  return USN_DEC_CLASS(d) != USN_CLS_FLOOD && USN_DEC_REASON(d) != USN_R_LOOPBACK;
}

/* the per-tile host lists of a result, merged in frame order: one copy per
 * listed tile, or one bulk copy of the whole area when many tiles list frames */
/* summary + tile headers (+ the tx counters when cnt) of a classified batch,
 * through the context's pinned staging buffer on stream s */
/* the batch's lists are not valid (usn_kernels.h USN_DIAG_*): a scan wait
 * timed out (never seen; the kernel gave up after 200 ms), or the scatter
 * found counts that disagree with the decisions.  Reported once, loudly; the
 * word is cleared for the scratch's next batch. */
int lists_failed(uint32_t diag, uint32_t *d_diag, hipStream_t s) {
  if (!diag) return USN_OK;
  HIPCHK(hipMemsetAsync(d_diag, 0, 4, s));
  HIPCHK(hipStreamSynchronize(s));
  if (diag & USN_DIAG_LISTS) return USN_ELIST;
  g_last_hip = (int)hipErrorLaunchTimeOut;
  return USN_EHIP;
}
/* the same after a scatter that usn_finalize launched itself (the stream is
 * synchronised by the caller) */
int lists_check(uint32_t *d_diag, hipStream_t s) {
  uint32_t dg = 0;
  HIPCHK(hipMemcpyAsync(&dg, d_diag, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return lists_failed(dg, d_diag, s);
}

int fetch_batch_state(usn_ctx *c, const usn_result *r, uint32_t ntiles, hipStream_t s,
                      usn_summary &sum, std::vector<usn_tile_hdr> &th, uint32_t *cnt,
                      const uint32_t *d_counters = nullptr, uint32_t *d_diag = nullptr) {
  const size_t tb = (size_t)ntiles * sizeof(usn_tile_hdr);
  constexpr size_t CB = USN_TXC_WORDS * 4;
  const size_t need = sizeof(usn_summary) + tb + CB + 4;
  if (need > c->h_stage_cap) {
    if (c->h_stage) HIPCHK(hipHostFree(c->h_stage));
    c->h_stage = nullptr;
    c->h_stage_cap = 0;
    const size_t cap = std::max<size_t>(need, 64 * 1024);
    HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c->h_stage), cap, hipHostMallocDefault));
    c->h_stage_cap = cap;
  }
  uint8_t *p = c->h_stage;
  HIPCHK(hipMemcpyAsync(p, r->summary, sizeof(usn_summary), hipMemcpyDeviceToHost, s));
  if (tb) HIPCHK(hipMemcpyAsync(p + sizeof(usn_summary), r->tiles, tb, hipMemcpyDeviceToHost, s));
  if (cnt)
    HIPCHK(hipMemcpyAsync(p + sizeof(usn_summary) + tb, d_counters, CB, hipMemcpyDeviceToHost, s));
  if (d_diag) HIPCHK(hipMemcpyAsync(p + sizeof(usn_summary) + tb + CB, d_diag, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::memcpy(&sum, p, sizeof sum);
  th.resize(ntiles);
  if (tb) std::memcpy(th.data(), p + sizeof(usn_summary), tb);
  if (cnt) std::memcpy(cnt, p + sizeof(usn_summary) + tb, CB);
  if (d_diag) {
    uint32_t dg;
    std::memcpy(&dg, p + sizeof(usn_summary) + tb + CB, 4);
    return lists_failed(dg, d_diag, s);
  }
  return USN_OK;
}

int fetch_host_lists(usn_ctx *c, const usn_result *r, const std::vector<usn_tile_hdr> &th,
                     std::vector<uint32_t> &hosts, hipStream_t s) {
  const uint32_t ntiles = (uint32_t)th.size();
  uint32_t listed = 0;
  size_t total = 0;
  for (const usn_tile_hdr &h : th) {
    listed += h.n_host ? 1u : 0u;
    total += h.n_host;
  }
  hosts.clear();
  hosts.reserve(total);
  if (listed > 32) {   // every tile's list area in one copy, through pinned memory
    const size_t bytes = (size_t)ntiles * USN_TILE * 4;
    if (bytes > c->h_lists_cap) {
      if (c->h_lists) HIPCHK(hipHostFree(c->h_lists));
      c->h_lists = nullptr;
      c->h_lists_cap = 0;
      const size_t cap = bytes + bytes / 2;   // batch sizes vary: no re-pin every time
      HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c->h_lists), cap, hipHostMallocDefault));
      c->h_lists_cap = cap;
    }
    HIPCHK(hipMemcpyAsync(c->h_lists, r->host_list, bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const uint32_t *all = c->h_lists;
    for (uint32_t t = 0; t < ntiles; ++t)
      hosts.insert(hosts.end(), all + (size_t)t * USN_TILE, all + (size_t)t * USN_TILE + th[t].n_host);
  } else {
    for (uint32_t t = 0; t < ntiles; ++t) {
      if (!th[t].n_host) continue;
      const size_t at = hosts.size();
      hosts.resize(at + th[t].n_host);
      HIPCHK(hipMemcpy(hosts.data() + at, r->host_list + (size_t)t * USN_TILE,
                       th[t].n_host * 4, hipMemcpyDeviceToHost));
    }
  }
  /* frame order: a tile lists only its own frames (in atomic order), so the
   * tiles' segments are already in order and each is ordered by itself, by a
   * 1024-bit map when it is long.  Anything else falls back to a full sort. */
  size_t at = 0;
  bool full_sort = false;
  for (uint32_t t = 0; t < ntiles && !full_sort; ++t) {
    const uint32_t m = th[t].n_host;
    if (!m) continue;
    uint32_t *seg = hosts.data() + at;
    at += m;
    const uint64_t lo = (uint64_t)t * USN_TILE;
    uint64_t bits[USN_TILE / 64] = {0};
    uint32_t pop = 0;
    for (uint32_t k = 0; k < m; ++k) {
      const uint64_t o = (uint64_t)seg[k] - lo;
      if (seg[k] < lo || o >= USN_TILE) { full_sort = true; break; }
      pop += (bits[o >> 6] >> (o & 63) & 1) ? 0u : 1u;
      bits[o >> 6] |= 1ull << (o & 63);
    }
    if (full_sort) break;
    if (m < 64 || pop != m) {   // short, or a frame listed twice (not expected)
      std::sort(seg, seg + m);
      continue;
    }
    uint32_t k = 0;
    for (uint32_t w = 0; w < USN_TILE / 64; ++w)
      for (uint64_t bb = bits[w]; bb; bb &= bb - 1)
        seg[k++] = (uint32_t)(lo + w * 64 + (uint32_t)__builtin_ctzll(bb));
  }
  if (full_sort) std::sort(hosts.begin(), hosts.end());
  return USN_OK;
}

}  // namespace

/* the cache a batch's device chain carries out: its last tile with a
 * touching frame, else what it carried in (as resolve_carry / chain_to_host) */
static void device_cout(const std::vector<usn_tile_hdr> &th, const usn_summary &sum, CacheState &cs) {
  cs.valid = false;
  cs.dst = 0;
  std::memset(cs.info.w, 0, 16);
  for (size_t t = th.size(); t > 0; --t) {
    const usn_tile_hdr &h = th[t - 1];
    if (!(h.last_state & USN_TS_HAS)) continue;
    if ((h.last_state & USN_TS_RETAINED) && !(h.last_state & USN_TS_UNKNOWN)) {
      cs.valid = true;
      cs.dst = h.last_dst;
      std::memcpy(cs.info.w, h.last_info, 16);
    }
    return;
  }
  cs.valid = sum.cin_state & USN_CS_VALID;
  cs.dst = sum.cin_dst;
  std::memcpy(cs.info.w, sum.cin_info, 16);
}
static bool same_cache(const CacheState &a, const CacheState &b) {
  if (a.valid != b.valid) return false;
  return !a.valid || (a.dst == b.dst && std::memcmp(a.info.w, b.info.w, 16) == 0);
}

/* Ordered host stage of a tx batch.  Frames before the first F_HOST frame h
 * are final on the device: apply what they learned in frame order (bridge
 * MACs, answer rules with the NIC cache reset, first fragments into the map).
 * From h on, find_forward runs sequentially on the host (endpoint.rs:172-296)
 * from the cache state just before h.  An overflow of the device sets
 * (counters[1]) makes h = 0.  `redo`: the batch ran while the batch before
 * it (pipelined, usn_ctx::txq) had not been finalized, and that finalize
 * changed the state this batch started from: h = 0, from the carried cache
 * usn_ctx::tx_cout when the batch before ran a host tail (else the one the
 * device resolved).  *changed: this finalize changed the state a batch
 * launched after this one started from (registry, bridge, DHCP steering, or
 * a carried cache other than the device chain's). */
static int finalize_tx(usn_ctx *c, const usn_batch *b, usn_result *r, hipStream_t s,
                       usn_finalize_info *info, const usn_ctx::Tx &txp, bool redo, bool *changed,
                       bool *tail) {
  StageClock clk("finalize_tx");
  *changed = false;
  *tail = redo;
  // the previous batch's carried-out cache (its host tail), for a redo of this
  // one.  Consumed here: every return below pops the batch (usn_finalize),
  // except USN_EAGAIN_READER, which puts it back
  const bool cout_in = c->tx_cout_valid;
  uint32_t cin_redo[6];
  std::memcpy(cin_redo, c->tx_cout, sizeof cin_redo);
  c->tx_cout_valid = false;
  const uint64_t n = b->n;
  const uint32_t ntiles = (uint32_t)((n + USN_TILE - 1) / USN_TILE);
  const int src = b->src_endpoint;
  Ep &S = c->eps[src];
  Replica &R = c->reps[txp.replica];
  Replica::TxSlot &X = R.txs[txp.slot];
  const int nd_src0 = S.next_dhcp, nd_nic0 = S.for_nic >= 0 ? c->eps[S.for_nic].next_dhcp : -1;
  usn_summary sum;
  std::vector<usn_tile_hdr> th;
  uint32_t cnt[USN_TXC_WORDS];
  if (c->txstate_for[txp.slot] == txp.launch_dec && X.txstate_ev) {   // gathered behind the launch
    HIPCHK(hipEventSynchronize(X.txstate_ev));
    if (txp.ring + 1 == txp.rings) c->txstate_for[txp.slot] = nullptr;
    const volatile uint32_t *q =
        reinterpret_cast<const volatile uint32_t *>(c->h_txstate + txp.slot * TXSTATE_BYTES);
    uint32_t v[12];
    for (int k = 0; k < 11; ++k) v[k] = q[USN_TXS_WORDS * txp.ring + k];
    v[11] = q[11];   // (ring 0's block: any chunk of the launch)
    { const int e = lists_failed(v[10] | v[11], usn::scatter_diag(r->scratch, r->n, c->n_ep + 3), s); if (e) return e; }
    if (!redo && v[1] == 0 && v[2] == 0 && v[4] != txp.epoch && v[5] == 0) {
      // nothing learned, nothing for the host stage, no timeout: the
      // results are final; class totals from bin_off (EP bins, NIC, FLOOD, DROP)
      usn_finalize_info fi;
      std::memset(&fi, 0, sizeof fi);
      fi.flags = v[0];
      fi.class_count[USN_CLS_EP] = v[6];
      fi.class_count[USN_CLS_NIC] = v[7] - v[6];
      fi.class_count[USN_CLS_FLOOD] = v[8] - v[7];
      fi.class_count[USN_CLS_DROP] = v[9] - v[8];
      if (info) *info = fi;
      return USN_OK;
    }
  }
  {
    const int e = fetch_batch_state(c, r, ntiles, s, sum, th, cnt, X.counters,
                                    usn::scatter_diag(r->scratch, r->n, c->n_ep + 3));
    if (e) return e;
  }
  // a tile wait of the kernel timed out (counters[3] = this epoch), or the
  // batch is redone: the whole batch goes to the host stage
  if (cnt[3] == txp.epoch) cnt[1] |= 8u;
  if (redo) cnt[1] |= 16u;
  uint32_t items_here = cnt[0];   // learned by this ring's frames
  if (txp.ring) items_here = cnt[USN_TXC_LEARNED + txp.ring];
  else
    for (uint32_t k = 1; k < txp.rings; ++k) items_here -= cnt[USN_TXC_LEARNED + k];
  clk.mark("state");
  usn_finalize_info fi;
  std::memset(&fi, 0, sizeof fi);
  fi.flags = sum.flags;
  for (uint32_t t = 0; t < ntiles; ++t)
    for (int k = 0; k < 4; ++k) fi.class_count[k] += th[t].class_count[k];
  std::vector<uint32_t> hosts;
  int st = fetch_host_lists(c, r, th, hosts, s);
  if (st) return st;
  clk.mark("summary");
  if (hosts.empty() && items_here == 0 && cnt[1] == 0) {   // nothing learned, nothing ordered
    if (info) *info = fi;
    return USN_OK;
  }
  HostView hv{c, b, r, s, {}, {}, false, false};
  st = hv.fetch_dec();
  if (st) return st;
  if (!c->reader && needs_reader(hv.dec, hosts)) {   // before any side effect: the batch stays
    c->tx_cout_valid = cout_in;                      // pending, and its retry redoes it from
    return USN_EAGAIN_READER;                        // the same carried cache
  }
  clk.mark("decisions");
  uint64_t h = n;
  if (cnt[1]) h = 0;
  else
    for (uint32_t j : hosts)
      if (hv.dec[j] & USN_F_HOST) { h = j; break; }
  /* learned items and first fragments before h, in frame order */
  const uint32_t nl = items_here ? std::min(cnt[0], X.learned_cap) : 0u;
  const uint4 *items = nullptr;   // the learned list (the launch's), through pinned memory
  if (nl && c->h_items_for == txp.launch) {
    items = c->h_items;           // an earlier ring of this launch fetched it
  } else if (nl) {
    c->h_items_for = 0;
    const size_t bytes = (size_t)nl * 2 * sizeof(uint4);
    if (bytes > c->h_items_cap) {
      if (c->h_items) HIPCHK(hipHostFree(c->h_items));
      c->h_items = nullptr;
      c->h_items_cap = 0;
      const size_t cap = bytes + bytes / 2;   // counts vary per batch: no re-pin every time
      HIPCHK(hipHostMalloc(reinterpret_cast<void **>(&c->h_items), cap, hipHostMallocDefault));
      c->h_items_cap = cap;
    }
    HIPCHK(hipMemcpyAsync(c->h_items, X.learned, bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    items = c->h_items;
    c->h_items_for = txp.launch;
  }
  clk.mark("items");
  struct Ev { uint64_t idx; uint32_t kind; uint4 key; };   // kind 0 mac, 1 rule, 2 frag1
  std::vector<Ev> evs;
  evs.reserve(nl + hosts.size());
  c->rules.reserve(c->rules.size() + nl);
  clk.mark("reserve");
  for (uint32_t k = 0; k < nl; ++k) {   // (launch frame index -> this ring's)
    const uint32_t x = items[2 * k].x;
    if (x >= txp.voff && x - txp.voff < h) evs.push_back(Ev{x - txp.voff, items[2 * k].y, items[2 * k + 1]});
  }
  for (uint32_t j : hosts)
    if (j < h && (hv.dec[j] & USN_F_FRAG1)) evs.push_back(Ev{j, 2, make_uint4(0, 0, 0, 0)});
  /* frame order; within a frame the fragment map first (kind 2, 1, 0).
   * (idx, kind) is unique, so an LSD radix sort of idx*4 + 2-kind over the
   * events' positions is exact (and ~20x std::sort at 10^5 learned items) */
  {
    std::vector<uint64_t> key(evs.size()), tmp(evs.size());
    uint64_t kmax = 0;
    for (size_t k = 0; k < evs.size(); ++k) {
      const uint64_t o = evs[k].idx * 4 + (2 - evs[k].kind);
      key[k] = (o << 30) | k;
      kmax = std::max(kmax, o);
    }
    for (uint32_t sh = 30; sh < 64 && (kmax >> (sh - 30)); sh += 11) {
      uint32_t cnt[2049] = {0};
      for (uint64_t v : key) cnt[((v >> sh) & 2047u) + 1]++;
      for (int d = 0; d < 2048; ++d) cnt[d + 1] += cnt[d];
      for (uint64_t v : key) tmp[cnt[(v >> sh) & 2047u]++] = v;
      key.swap(tmp);
    }
    std::vector<Ev> sorted(evs.size());
    for (size_t k = 0; k < evs.size(); ++k) sorted[k] = evs[key[k] & ((1u << 30) - 1)];
    evs.swap(sorted);
  }
  std::vector<uint8_t> buf;
  clk.mark("sort");
  /* Every device read comes first: the frames the apply loop parses (first
   * fragments), the last cache-touching frame before h and the frames
   * [h, n).  A failure there leaves the registry, bridge and maps untouched
   * (the batch's results stay unusable; nothing was learned). */
  const uint32_t W = USN_WINDOW_MAX;
  auto fetch = [&](uint64_t i, uint8_t *dst, uint32_t &l) -> int {
    const int e = hv.frame(i, buf, l);
    if (e) return e;
    std::memcpy(dst, buf.data(), W);
    return USN_OK;
  };
  std::vector<uint8_t> frag_bytes;      // kind-2 events' frames, in event order
  std::vector<uint32_t> frag_lens;
  for (const Ev &e : evs)
    if (e.kind == 2) {
      frag_bytes.resize(frag_bytes.size() + W);
      frag_lens.push_back(0);
      st = fetch(e.idx, frag_bytes.data() + frag_bytes.size() - W, frag_lens.back());
      if (st) return st;
    }
  uint64_t walk = n;                    // the last touching frame before h, if it retains
  std::vector<uint8_t> walk_bytes(W);
  uint32_t walk_len = 0;
  bool walk_none = false;               // a touching frame left last_pkt = None
  std::vector<uint8_t> seq;             // frames [h, n), W bytes each
  std::vector<uint32_t> seq_len;
  if (h < n) {
    for (uint64_t k = h; k > 0; --k) {
      const uint32_t d = hv.dec[k - 1];
      if (!touches(d)) continue;
      if (!retains(d)) { walk_none = true; break; }
      walk = k - 1;
      st = fetch(walk, walk_bytes.data(), walk_len);
      if (st) return st;
      break;
    }
    const bool strided = b->stride != 0;
    const uint32_t width =
        strided ? (uint32_t)std::min<uint64_t>(std::min<uint64_t>(b->stride, batch_window(b)), W) : 0;
    st = hv.fetch_lens();
    if (st) return st;
    seq.assign((size_t)(n - h) * W, 0);
    seq_len.assign(n - h, 0);
    if (strided)
      HIPCHK(hipMemcpy2D(seq.data(), W, b->frames + h * b->stride, b->stride, width, n - h,
                         hipMemcpyDeviceToHost));
    for (uint64_t j = h; j < n; ++j) {
      uint8_t *fp = seq.data() + (size_t)(j - h) * W;
      if (strided && (hv.lens[j] <= width || width == W || !ports_past(fp, hv.lens[j], width))) {
        seq_len[j - h] = hv.lens[j];
      } else {
        st = fetch(j, fp, seq_len[j - h]);
        if (st) return st;
      }
    }
  }
  clk.mark("frames");
  auto ev_key = [](const Ev &e) {
    WantKey w;
    w.dst = e.key.x;
    w.src = e.key.y;
    w.dport = (uint16_t)(e.key.z & 0xFFFFu);
    w.sport = (uint16_t)(e.key.z >> 16);
    w.proto = (uint8_t)(e.key.w & 0xFFu);
    w.present = (uint8_t)((e.key.w >> 8) & 7u);
    return w;
  };
  constexpr size_t PF = 16;   // registry slots are random in a table of 10^6: prefetch ahead
  for (size_t k = 0; k < std::min(PF, evs.size()); ++k)
    if (evs[k].kind == 1) prefetch_rule(c, ev_key(evs[k]));
  size_t kf = 0;
  for (size_t ke = 0; ke < evs.size(); ++ke) {
    const Ev &e = evs[ke];
    if (ke + PF < evs.size() && evs[ke + PF].kind == 1) prefetch_rule(c, ev_key(evs[ke + PF]));
    if (e.kind == 2) {                                   // extract_pkt_info side effect
      (void)host_parse(c, frag_bytes.data() + kf * W, frag_lens[kf]);
      ++kf;
    } else if (e.kind == 0) {                            // endpoint.rs:195-197
      const uint64_t m = (uint64_t)e.key.x | ((uint64_t)e.key.y << 32);
      if (!bridge_has(c, m)) { c->bridge.push_back(m); c->bridge_dirty = true; fi.n_learned++; }
    } else {                                             // endpoint.rs:233-252
      const WantKey w = ev_key(e);
      if (!c->rules.count(w)) {
        if (S.for_nic >= 0) cache_clear(c, S.for_nic);
        rule_insert(c, w, Rule{(uint16_t)src, 0});
        fi.n_learned++;
      }
    }
  }
  clk.mark("apply");
  if (h < n) {
    /* cache state just before h: carried in, then the last touching frame */
    CacheState cs;
    cs.valid = sum.cin_state & USN_CS_VALID;
    cs.dst = sum.cin_dst;
    std::memcpy(cs.info.w, sum.cin_info, 16);
    if (redo && cout_in) {   // h = 0: the previous batch's host tail left this cache
      cs.valid = cin_redo[0] & USN_CS_VALID;
      cs.dst = cin_redo[1];
      std::memcpy(cs.info.w, cin_redo + 2, 16);
    }
    if (walk_none) cs.valid = false;
    if (walk < n) {
      ParsedH p = host_parse(c, walk_bytes.data(), walk_len);
      cs.valid = true;
      cs.info = p.info;
      cs.dst = hv.dec[walk] & USN_PARITY_MASK;
    }
    std::vector<uint32_t> out(n - h);
    for (uint64_t j = h; j < n; ++j) {
      bool learned = false;
      uint32_t d = host_step(c, src, seq.data() + (size_t)(j - h) * W, seq_len[j - h], cs, learned) |
                   USN_F_HOST;
      if (learned) { d |= USN_F_LEARN; fi.n_learned++; }
      const uint32_t old = hv.dec[j];
      if ((old & USN_PARITY_MASK) != (d & USN_PARITY_MASK)) fi.n_patched++;
      fi.class_count[USN_DEC_CLASS(old)]--;
      fi.class_count[USN_DEC_CLASS(d)]++;
      out[j - h] = d;
    }
    fi.n_host = (uint32_t)(n - h);
    *tail = true;
    /* the registry is final from here on; a HIP failure below leaves this
     * batch's device results unpatched (reported, not retried) */
    HIPCHK(hipMemcpy(r->decisions + h, out.data(), out.size() * 4, hipMemcpyHostToDevice));
    ClassifyArgs a;
    fill_args(c, R, b, r, a);
    HIPCHK(usn::launch_recount(a, (uint32_t)(h / USN_TILE), ntiles, s));
    st = launch_scatter(c, &a, r, 1, s);
    if (st) return st;
    usn_summary o = sum;
    o.flags |= USN_S_COUT;
    o.cout_state = cs.valid ? USN_CS_VALID : 0u;
    o.cout_dst = cs.dst;
    std::memcpy(o.cout_info, cs.info.w, 16);
    HIPCHK(hipMemcpy(r->summary, &o, sizeof o, hipMemcpyHostToDevice));
    HIPCHK(hipStreamSynchronize(s));
    st = lists_check(usn::scatter_diag(r->scratch, r->n, c->n_ep + 3), s);
    if (st) return st;
    // what a batch launched after this one took as its carried cache: the
    // device chain's (this batch's tile headers); the host tail's may differ
    CacheState dev;
    device_cout(th, sum, dev);
    *changed = !same_cache(cs, dev);
    c->tx_cout_valid = true;
    c->tx_cout[0] = cs.valid ? USN_CS_VALID : 0u;
    c->tx_cout[1] = cs.dst;
    std::memcpy(c->tx_cout + 2, cs.info.w, 16);
  }
  *changed = *changed || fi.n_learned > 0 || S.next_dhcp != nd_src0 ||
             (S.for_nic >= 0 && c->eps[S.for_nic].next_dhcp != nd_nic0);
  if (info) *info = fi;
  return USN_OK;
}

int usn_finalize(usn_ctx *c, const usn_batch *b, usn_result *r, void *stream,
                 usn_finalize_info *info) {
  if (!c || !b || !r || b->n == 0 || b->src_endpoint >= USN_MAX_ENDPOINTS) return USN_EINVAL;
  if (c->reps.empty()) return USN_ENODEV;
  std::lock_guard<std::mutex> g(c->mu);
  // the oldest tx batch in flight (finalized in order)
  const bool txb = !c->txq.empty() && c->txq.front().src == b->src_endpoint &&
                   c->txq.front().decisions == r->decisions;
  const auto br = c->batch_rep.find(r->decisions);
  const uint32_t rep = txb ? c->txq.front().replica
                     : br != c->batch_rep.end() ? br->second.rep : c->chains[b->src_endpoint].replica;
  // the bins the batch was classified with (an rx batch's endpoints may have
  // grown since; a tx batch blocks every registry change until it is final)
  const uint32_t nb0 = br != c->batch_rep.end() ? br->second.nbins : c->n_ep + 3;
  HIPCHK(hipSetDevice(c->reps[rep].device));
  hipStream_t s = (hipStream_t)stream;
  // (a tx batch waits for its own launches only: the next ring may already
  // be queued behind them on the stream; so does an rx batch whose launch
  // recorded its completion, and the host-stage path below orders its copies
  // on the stream itself)
  if (!txb) {
    if (br != c->batch_rep.end() && br->second.done) { int e = rx_wait(c, br->second); if (e) return e; }
    else HIPCHK(hipStreamSynchronize(s));
  }
  {  // lists built on the side stream (usn_set_lists_async)
    auto it = c->lists_ev.find(r->decisions);
    if (it != c->lists_ev.end() && it->second.pending) {
      HIPCHK(hipEventSynchronize(it->second.ev));
      it->second.pending = false;
    }
  }
  if (c->eps[b->src_endpoint].used && c->eps[b->src_endpoint].kind != USN_EP_NIC) {
    if (txb) {
      const usn_ctx::Tx p = c->txq.front();
      // its state is copied on `s`: the stream the batch's launches are on
      if (p.stream != s) return USN_EINVAL;
      bool changed = false, tail = false;
      const int st = finalize_tx(c, b, r, s, info, p, c->tx_redo_next, &changed, &tail);
      // refused before any side effect (a frame needs the frame reader and
      // none is set): the batch stays pending, so a call after
      // usn_set_frame_reader applies what it learned
      if (st == USN_EAGAIN_READER) return USN_EINVAL;
      c->txq.pop_front();
      c->tx_chg = c->tx_chg || changed || st != USN_OK;
      // the next ring in flight: the next ring of this launch saw this ring's device
      // results (redone when the host decided part of this ring, or it
      // failed); a later launch started from the state before the finalizes
      // since it was enqueued (redone when one of them changed it)
      if (c->txq.empty()) c->tx_redo_next = false;
      else if (c->txq.front().launch == p.launch) c->tx_redo_next = tail || st != USN_OK;
      else c->tx_redo_next = c->tx_chg;
      return st;
    }
    if (!c->txq.empty()) return USN_EBUSY;   // a later ring in flight (in order), or another source
    /* an already finalized tx batch: its results are final */
    const uint32_t nt = (uint32_t)((b->n + USN_TILE - 1) / USN_TILE);
    std::vector<usn_tile_hdr> th(nt);
    HIPCHK(hipMemcpy(th.data(), r->tiles, nt * sizeof(usn_tile_hdr), hipMemcpyDeviceToHost));
    usn_finalize_info fi;
    std::memset(&fi, 0, sizeof fi);
    for (uint32_t t = 0; t < nt; ++t)
      for (int k = 0; k < 4; ++k) fi.class_count[k] += th[t].class_count[k];
    if (info) *info = fi;
    return USN_OK;
  }
  /* NIC batch: its scatter left the batch's state in host-mapped memory
   * (summary flags, whether any tile listed frames for the host stage, the
   * class totals, the lists' diag word).  With nothing for the host stage the
   * device results are final: no copy of the summary and the tile headers
   * (37 us per 1M-frame ring, profiles/r05/r05b) */
  if (br != c->batch_rep.end() && br->second.slot < usn_ctx::RX_SLOTS) {
    const volatile uint32_t *h = c->h_rxstate + br->second.slot * 8;
    if (h[0] == br->second.epoch) {
      const uint32_t lists = h[2] | h[7];
      if (lists) return lists_failed(lists, usn::scatter_diag(r->scratch, r->n, nb0), s);
      if (h[1] == 0 && h[3] == 0) {
        usn_finalize_info fi;
        std::memset(&fi, 0, sizeof fi);
        fi.class_count[USN_CLS_EP] = h[4];
        fi.class_count[USN_CLS_NIC] = h[5] - h[4];
        fi.class_count[USN_CLS_FLOOD] = h[6] - h[5];
        fi.class_count[USN_CLS_DROP] = (uint32_t)b->n - h[6];
        if (info) *info = fi;
        return USN_OK;   // device results are final; the device chain carries the cache
      }
    }
  }
  const uint32_t ntiles = (uint32_t)((b->n + USN_TILE - 1) / USN_TILE);
  usn_summary sum;
  std::vector<usn_tile_hdr> th;
  {
    const int e = fetch_batch_state(c, r, ntiles, s, sum, th, nullptr, nullptr,
                                    usn::scatter_diag(r->scratch, r->n, nb0));
    if (e) return e;
  }
  usn_finalize_info fi;
  std::memset(&fi, 0, sizeof fi);
  fi.flags = sum.flags;
  for (uint32_t t = 0; t < ntiles; ++t)
    for (int k = 0; k < 4; ++k) fi.class_count[k] += th[t].class_count[k];
  std::vector<uint32_t> hosts;
  {
    const int e = fetch_host_lists(c, r, th, hosts, s);
    if (e) return e;
  }
  const bool stale_walk = (sum.flags & USN_S_STALE) && sum.first_break < b->n;
  if (hosts.empty() && !stale_walk && !(sum.flags & USN_S_STALE_EXTENDS)) {
    if (info) *info = fi;
    return USN_OK;   // device results are final; the device chain carries the cache
  }
  // the host stage may name an endpoint added since the classify: its lists
  // then need today's bins.  Refused here, before any side effect, when the
  // result cannot hold them (a retry would otherwise repeat the map, DHCP
  // and cache steps).
  if (c->n_ep + 3 > nb0 && c->n_ep + 3 > r->max_bins) return USN_ERANGE;
  const int src = b->src_endpoint;
  HostView hv{c, b, r, s, {}, {}, false, false};
  int st = hv.fetch_dec();
  if (st) return st;
  if (!c->reader && needs_reader(hv.dec, hosts)) return USN_EINVAL;   // before any side effect
  std::vector<uint8_t> buf;
  uint32_t len = 0;
  std::vector<char> dirty(ntiles, 0);
  bool new_ep = false;   // a resolved decision names an endpoint id >= the batch's n_ep
  CacheState cs;
  cs.valid = sum.cin_state & USN_CS_VALID;
  cs.dst = sum.cin_dst;
  std::memcpy(cs.info.w, sum.cin_info, 16);
  const CacheState carried = cs;
  uint64_t pos = 0;   // cache state `cs` is the state just before frame `pos`

  /* advance cs over device-final frames [pos, j) */
  auto advance = [&](uint64_t j) -> int {
    for (uint64_t k = j; k > pos; --k) {
      const uint32_t d = hv.dec[k - 1];
      if (!touches(d)) continue;
      if (!retains(d)) { cs.valid = false; break; }
      int e = hv.frame(k - 1, buf, len);
      if (e) return e;
      ParsedH p = host_parse(c, buf.data(), len);   // no map side effect: not a first fragment
      cs.valid = true;
      cs.info = p.info;
      cs.dst = d & USN_PARITY_MASK;
      break;
    }
    pos = j;
    return USN_OK;
  };
  auto resolve = [&](uint64_t j) -> int {
    int e = advance(j);
    if (e) return e;
    e = hv.frame(j, buf, len);
    if (e) return e;
    bool learned;
    const uint32_t d = host_step(c, src, buf.data(), len, cs, learned) | USN_F_HOST;
    const uint32_t old = hv.dec[j];
    // every resolved frame counts, host-listed or walked in a stale prefix
    if (USN_DEC_CLASS(d) == USN_CLS_EP && (d & 0xFFFFu) + 3 >= nb0) new_ep = true;
    if ((old & USN_PARITY_MASK) != (d & USN_PARITY_MASK)) {
      fi.n_patched++;
      fi.class_count[USN_DEC_CLASS(old)]--;
      fi.class_count[USN_DEC_CLASS(d)]++;
      dirty[j / USN_TILE] = 1;
    }
    if (old != d) {
      hv.dec[j] = d;
      HIPCHK(hipMemcpy(r->decisions + j, &d, 4, hipMemcpyHostToDevice));
    }
    fi.n_host++;
    pos = j + 1;
    return USN_OK;
  };

  size_t hi = 0;
  /* stale prefix that the device could not close inside tile 0 */
  if (stale_walk || (sum.flags & USN_S_STALE_EXTENDS)) {
    uint64_t j = (sum.flags & USN_S_STALE_EXTENDS) ? std::min<uint64_t>(USN_TILE, b->n)
                                                   : sum.first_break;
    // frames before j are final (device override or host frames among them)
    while (hi < hosts.size() && hosts[hi] < j) {
      st = resolve(hosts[hi++]);
      if (st) return st;
    }
    st = advance(j);
    if (st) return st;
    // walk while the stale entry is still the cached one
    while (j < b->n && cs.valid && cs.info == carried.info && cs.dst == carried.dst) {
      if (hi < hosts.size() && hosts[hi] == j) ++hi;
      st = resolve(j);
      if (st) return st;
      ++j;
    }
  }
  while (hi < hosts.size()) {
    st = resolve(hosts[hi++]);
    if (st) return st;
  }
  st = advance(b->n);
  if (st) return st;
  /* patched tiles: recount their bin rows, then the lists again, with the
   * bins the batch was classified with -- unless a decision of the host stage
   * names an endpoint added since (then every tile, with today's bins) */
  const uint32_t nb = new_ep ? c->n_ep + 3 : nb0;   // <= max_bins: checked before any side effect
  if (nb != nb0) std::fill(dirty.begin(), dirty.end(), 1);
  ClassifyArgs a;
  fill_args(c, c->reps[rep], b, r, a);
  set_bins(r, b->n, nb, a);
  bool any = false;
  for (uint32_t t = 0; t < ntiles;) {
    if (!dirty[t]) { ++t; continue; }
    uint32_t e = t;
    while (e < ntiles && dirty[e]) ++e;
    HIPCHK(usn::launch_recount(a, t, e, s));
    any = true;
    t = e;
  }
  if (any) {
    st = launch_scatter(c, &a, r, 1, s);
    if (st) return st;
  }
  /* carried-out cache: authoritative from now on */
  usn_summary out = sum;
  out.n_ep = nb - 3;
  out.n_bins = nb;
  if (nb != nb0) c->batch_rep[r->decisions].nbins = nb;
  out.flags |= USN_S_COUT;
  out.cout_state = cs.valid ? USN_CS_VALID : 0u;
  out.cout_dst = cs.dst;
  std::memcpy(out.cout_info, cs.info.w, 16);
  HIPCHK(hipMemcpy(r->summary, &out, sizeof out, hipMemcpyHostToDevice));
  HIPCHK(hipStreamSynchronize(s));
  if (any) {
    st = lists_check(usn::scatter_diag(r->scratch, r->n, nb), s);
    if (st) return st;
  }
  if (info) *info = fi;
  return USN_OK;
}

/* diagnostics (tools/scatter_bench.py): the per-endpoint scatter of `count`
 * batches classified together, again, on `stream` (no classify) */
int usn_debug_scatter(usn_ctx *c, const usn_batch *b, usn_result *r, uint32_t count, void *stream) {
  if (!c || !b || !r || count == 0 || count > USN_MAX_MULTI) return USN_EINVAL;
  if (c->reps.empty()) return USN_ENODEV;
  std::lock_guard<std::mutex> g(c->mu);
  Replica &R = c->reps[c->sel];
  HIPCHK(hipSetDevice(R.device));
  usn::ClassifyArgs as[USN_MAX_MULTI];
  for (uint32_t k = 0; k < count; ++k) fill_args(c, R, &b[k], &r[k], as[k]);
  return launch_scatter(c, as, r, count, (hipStream_t)stream);
}

/* diagnostics: scatter chunks on the selected replica's device whose
 * optimistic ranks were not stably sorted and were ranked again (the
 * kernel's step 5; expected 0), since the library was loaded */
int64_t usn_debug_scatter_fallbacks(usn_ctx *c) {
  if (!c) return USN_EINVAL;
  if (c->reps.empty()) return USN_ENODEV;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->reps[c->sel].device));
  HIPCHK(hipDeviceSynchronize());
  const uint32_t v = usn_t512::scatter_fallbacks();
  return v == 0xFFFFFFFFu ? (int64_t)USN_EHIP : (int64_t)v;
}

int usn_set_lists_async(usn_ctx *c, int on) {
  if (!c) return USN_EINVAL;
  if (c->reps.empty()) return USN_ENODEV;
  std::lock_guard<std::mutex> g(c->mu);
  c->lists_async = on != 0;
  return USN_OK;
}

int usn_lists_wait(usn_ctx *c, const usn_result *r, void *stream) {
  if (!c || !r) return USN_EINVAL;
  if (c->reps.empty()) return USN_ENODEV;
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->lists_ev.find(r->decisions);
  if (it == c->lists_ev.end() || !it->second.ev) return USN_OK;   // built on the batch's stream
  HIPCHK(hipSetDevice(it->second.device));
  HIPCHK(hipStreamWaitEvent((hipStream_t)stream, it->second.ev, 0));
  return USN_OK;
}

/* ---- device plumbing ------------------------------------------------------- */
int usn_dev_alloc(usn_ctx *c, size_t bytes, void **p) {
  if (!c || !p) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMalloc(p, bytes));
  return USN_OK;
}
int usn_dev_free(usn_ctx *c, void *p) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipFree(p));
  return USN_OK;
}
int usn_host_alloc_pinned(usn_ctx *c, size_t bytes, void **p) {
  if (!c || !p) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipHostMalloc(p, bytes, hipHostMallocDefault));
  return USN_OK;
}
int usn_host_free_pinned(usn_ctx *c, void *p) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipHostFree(p));
  return USN_OK;
}
int usn_memcpy_h2d(usn_ctx *c, void *d, const void *h, size_t n, void *s) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, (hipStream_t)s));
  return USN_OK;
}
int usn_memcpy_d2h(usn_ctx *c, void *h, const void *d, size_t n, void *s) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, (hipStream_t)s));
  return USN_OK;
}
int usn_memset_d(usn_ctx *c, void *d, int v, size_t n, void *s) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipMemsetAsync(d, v, n, (hipStream_t)s));
  return USN_OK;
}
int usn_stream_create(usn_ctx *c, void **s) {
  if (!c || !s) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipSetDevice(c->device));
  hipStream_t st;
  HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  *s = st;
  return USN_OK;
}
int usn_stream_destroy(usn_ctx *c, void *s) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipStreamDestroy((hipStream_t)s));
  return USN_OK;
}
int usn_stream_sync(usn_ctx *c, void *s) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipStreamSynchronize((hipStream_t)s));
  return USN_OK;
}
int usn_device_sync(usn_ctx *c) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipDeviceSynchronize());
  return USN_OK;
}
int usn_event_create(usn_ctx *c, void **ev) {
  if (!c || !ev) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  hipEvent_t e;
  HIPCHK(hipEventCreateWithFlags(&e, c->timing_ev_flags));
  *ev = e;
  return USN_OK;
}
int usn_event_destroy(usn_ctx *c, void *ev) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipEventDestroy((hipEvent_t)ev));
  return USN_OK;
}
int usn_event_record(usn_ctx *c, void *ev, void *s) {
  if (!c) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipEventRecord((hipEvent_t)ev, (hipStream_t)s));
  return USN_OK;
}
int usn_event_elapsed_ms(usn_ctx *c, void *a, void *b, float *ms) {
  if (!c || !ms) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipEventSynchronize((hipEvent_t)b));
  HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
  return USN_OK;
}

int usn_stream_wait_event(usn_ctx *c, void *s, void *ev) {
  if (!c || !ev) return USN_EINVAL;
  if (c->device < 0) return USN_ENODEV;
  HIPCHK(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)ev, 0));
  return USN_OK;
}

}  // extern "C"
