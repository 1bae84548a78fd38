/*
 * usnetd.cpp -- the usnetd daemon around the MI355X match path.
 *
 * Keeps the reference's external contract (/root/reference/src/main.rs):
 *   - the control socket /run/usnetd.socket (AF_UNIX SOCK_DGRAM, mode 0770,
 *     optional ALLOW_GID group, :886-903) and its JSON message set with the
 *     reference's replies and silences (act_on, :403-633);
 *   - RequestUDS: a SOCK_DGRAM socketpair whose far end is handed to the
 *     client with SCM_RIGHTS after a "$" payload (:415-466);
 *   - the 90 s cleanup (fragment map clear + GC of the kernel host ring's
 *     non-sticky rules against /proc/net/{tcp,udp}, :1070-1110) driven by a
 *     timer thread over <socket>timer (:673-701), "end" on SIGINT/SIGTERM;
 *   - client liveness through /proc/<pid>/cmdline (:1050-1057);
 *   - configuration from the environment or a dotenv CONFFILE: INTERFACES,
 *     ALLOW_GID, DEBUG_PORTS, STATIC_PIPES, ADD_MACS, NO_HOST_RINGS,
 *     NO_ZERO_COPY, PCAP_LOG, RUST_LOG (:818-866).
 * and replaces the per-frame loop (Endpoint::forward + find_forward,
 * src/endpoint.rs:114-296) by batches: every poll round drains the readable
 * endpoints, classifies their frames on the GPU through the C ABI
 * (usn_classify / usn_classify_multi + usn_finalize, include/usn_classify.h)
 * and writes each frame to its decision's target in frame order.
 *
 * NIC access: netmap and macvtap need a kernel module / root and are out of
 * scope here.  A NIC (and its kernel host ring) is an AF_UNIX datagram
 * "wire": the daemon binds <dir>/<iface>.nic and sends frames for the
 * network to <dir>/<iface>.wire; the host ring binds <dir>/<iface>.host and
 * sends to <dir>/<iface>.kernel.  <dir> = USNETD_NIC_DIR (default: the
 * socket's directory).  USNETD_CONTROL_ONLY=1 runs the control plane on a
 * registry-only context (no GPU, no frame forwarding).
 */
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <netinet/in.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstddef>
#include <tuple>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/usn_classify.h"
#include "messages.hpp"

namespace usnd {

/* ---- logging (RUST_LOG levels) ---------------------------------------------- */
static int g_level = 1;   // 0 error, 1 warn, 2 info, 3 debug
static void logf(int lvl, const char *fmt, ...) {
  if (lvl > g_level) return;
  static const char *names[] = {"ERROR", "WARN", "INFO", "DEBUG"};
  std::fprintf(stderr, "[usnetd %s] ", names[lvl]);
  va_list ap;
  va_start(ap, fmt);
  std::vfprintf(stderr, fmt, ap);
  va_end(ap);
  std::fputc('\n', stderr);
}
#define LOGE(...) logf(0, __VA_ARGS__)
#define LOGW(...) logf(1, __VA_ARGS__)
#define LOGI(...) logf(2, __VA_ARGS__)
#define LOGD(...) logf(3, __VA_ARGS__)

static std::string env(const char *k, const char *dflt = nullptr) {
  const char *v = std::getenv(k);
  return v ? std::string(v) : (dflt ? std::string(dflt) : std::string());
}
static bool has_env(const char *k) { return std::getenv(k) != nullptr; }

static std::vector<std::string> split(const std::string &s, char c) {
  std::vector<std::string> out;
  std::string cur;
  for (char x : s) {
    if (x == c) { out.push_back(cur); cur.clear(); }
    else cur += x;
  }
  out.push_back(cur);
  return out;
}

static bool make_addr(const std::string &path, sockaddr_un &a, socklen_t &len) {
  std::memset(&a, 0, sizeof a);
  a.sun_family = AF_UNIX;
  if (path.size() >= sizeof a.sun_path) return false;
  std::memcpy(a.sun_path, path.data(), path.size());
  len = (socklen_t)(offsetof(sockaddr_un, sun_path) + path.size() + 1);
  return true;
}

/* dotenv: KEY=VALUE lines fill variables that are not set already */
static bool load_dotenv(const std::string &file) {
  std::ifstream in(file);
  if (!in) return false;
  std::string line;
  while (std::getline(in, line)) {
    size_t a = line.find_first_not_of(" \t");
    if (a == std::string::npos || line[a] == '#') continue;
    if (line.compare(a, 7, "export ") == 0) a += 7;
    const size_t eq = line.find('=', a);
    if (eq == std::string::npos) continue;
    std::string k = line.substr(a, eq - a), v = line.substr(eq + 1);
    while (!k.empty() && (k.back() == ' ' || k.back() == '\t')) k.pop_back();
    while (!v.empty() && (v.back() == '\r' || v.back() == ' ' || v.back() == '\t')) v.pop_back();
    if (v.size() >= 2 && ((v.front() == '"' && v.back() == '"') || (v.front() == '\'' && v.back() == '\'')))
      v = v.substr(1, v.size() - 2);
    setenv(k.c_str(), v.c_str(), 0);
  }
  return true;
}

/* ---- devices ------------------------------------------------------------------ */
struct Dev {
  int kind = USN_EP_NIC;      // USN_EP_NIC / USN_EP_HOST / USN_EP_UDS
  uint16_t id = 0;            // usn endpoint id (decision word)
  int for_nic = -1;
  std::string iface;          // get_nic() / get_host_ring()
  std::string client_path;    // RequestUDS clients
  int fd = -1;
  sockaddr_un peer{};         // NIC / host ring: where frames are sent
  socklen_t peer_len = 0;
  int txfd = -1;              // NIC / host ring: socket connected to `peer` (lazily)
  uint32_t rep = 0;           // the device replica its rings are classified on
  /* two result buffers per source: the carried cache reads the previous one */
  void *res[2] = {nullptr, nullptr};
  usn_result rb[2] = {};      // bound once per allocation (a bind per round re-zeroes scratch)
  int cur = 0;
  uint64_t frames_in = 0, frames_out = 0;
};
using DevP = std::shared_ptr<Dev>;

struct Change {
  enum { Add, Remove, Cleanup } type;
  DevP dev;
};

struct PcapWriter {
  FILE *f = nullptr;
  bool open(const std::string &path) {
    f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const uint32_t hdr[6] = {0xA1B2C3D4u, 0x00040002u, 0, 0, 65535, 1};   // Ethernet
    std::fwrite(hdr, 4, 6, f);
    return true;
  }
  void packet(const uint8_t *p, uint32_t len) {
    if (!f) return;
    timeval tv;
    gettimeofday(&tv, nullptr);
    const uint32_t rec[4] = {(uint32_t)tv.tv_sec, (uint32_t)tv.tv_usec, len, len};
    std::fwrite(rec, 4, 4, f);
    std::fwrite(p, 1, len, f);
  }
  void flush() { if (f) std::fflush(f); }
};

static std::atomic<bool> g_signal{false};
static void on_signal(int) { g_signal.store(true); }

class Daemon {
 public:
  int run(int argc, char **argv);

 private:
  std::string sock_path_, nic_dir_;
  int ctl_fd_ = -1;
  usn_ctx *ctx_ = nullptr;
  bool data_path_ = true, test_dump_ = false;
  std::vector<DevP> devices_;   // all_devices without the control socket
  std::vector<std::pair<uint64_t, DevP>> pipe_monitor_;
  std::vector<Change> changes_;
  std::vector<char> used_ids_ = std::vector<char>(USN_MAX_ENDPOINTS, 0);
  PcapWriter pcap_;
  uint64_t class_count_[4] = {0, 0, 0, 0};
  bool end_ = false;
  uint32_t ep_limit_ = 0;   // max endpoint id ever added + 1: the context's n_ep (it never shrinks)
  unsigned cleanup_secs_ = 90;
  int write_wait_ms_ = 5;     // USNETD_WRITE_WAIT_MS: back-pressure before a frame is dropped

  /* data path buffers, one set per device replica (USNETD_HIP_DEVICES) */
  static const uint32_t HDR = 128;        // header window stride on the device
  /* per source in h_out: the summary, bin_off[USN_MAX_BINS + 1], then index[n] */
  static const size_t OUT_BINS = 128;
  static const size_t OUT_HEAD = OUT_BINS + (size_t)(USN_MAX_BINS + 1) * 4;
  uint32_t max_batch_ = 4096;             // frames per source per round
  struct RepBuf {
    void *stream = nullptr;
    uint8_t *h_hdr = nullptr, *d_hdr = nullptr;   // headers of the round (pinned / device)
    uint16_t *h_lens = nullptr, *d_lens = nullptr;
    uint32_t cap = 0;                             // frames
    uint8_t *h_out = nullptr;                     // pinned: summary, bin offsets, lists per source
    size_t out_cap = 0;
  };
  std::vector<RepBuf> reps_;
  uint32_t next_rep_ = 0;                 // endpoints are spread over the replicas round-robin
  std::vector<uint8_t> arena_;            // full frames of the round
  std::vector<size_t> off_;
  std::vector<uint32_t> len_;

  int alloc_id() {
    for (int i = 0; i < USN_MAX_ENDPOINTS; ++i)
      if (!used_ids_[i]) { used_ids_[i] = 1; return i; }
    return -1;
  }
  DevP by_id(uint32_t id) {
    for (auto &d : devices_) if (d->id == id) return d;
    return nullptr;
  }
  bool setup_config();
  bool bind_control();
  DevP add_nic(const std::string &iface);
  DevP add_host_ring(const std::string &iface, const DevP &nic);
  bool register_dev(const DevP &d);
  void remove_dev(const DevP &d);
  bool iface_ipv4(const std::string &iface, uint32_t &ip);
  bool want_of(const WantMsg &m, usn_want &w);
  void reply(const std::string &client_path, const std::string &msg);
  DevP find_by_client_path(const std::string &p);
  DevP find_nic(const std::string &iface);
  void act_on(const ClientMessage &m, const std::string &client_path);
  void control_readable();
  void cleanup();
  void dump(const std::string &client_path);
  void apply_changes();
  /* data path */
  bool data_path_init();
  void forward_round(const std::vector<DevP> &ready);
  int write_frames(const DevP &t, const std::vector<uint32_t> &idx);
  bool select(uint32_t rep);
};

/* ---- configuration ------------------------------------------------------------- */
bool Daemon::iface_ipv4(const std::string &iface, uint32_t &ip) {
  std::string over = "USNETD_IFACE_IP_" + iface;
  for (char &c : over) if (!isalnum((unsigned char)c)) c = '_';
  if (has_env(over.c_str())) return parse_ipv4(env(over.c_str()), ip);
  ifaddrs *ifa = nullptr;
  if (getifaddrs(&ifa) != 0) return false;
  bool ok = false;
  for (ifaddrs *p = ifa; p; p = p->ifa_next)
    if (p->ifa_addr && p->ifa_addr->sa_family == AF_INET && iface == p->ifa_name) {
      ip = ntohl(reinterpret_cast<sockaddr_in *>(p->ifa_addr)->sin_addr.s_addr);
      ok = true;
      break;
    }
  freeifaddrs(ifa);
  return ok;
}

bool Daemon::register_dev(const DevP &d) {
  /* every endpoint's rings go to one replica, round-robin: the registry is
   * shared, so a sending endpoint may learn on any of them */
  if (!reps_.empty()) d->rep = next_rep_++ % (uint32_t)reps_.size();
  const int st = usn_endpoint_add(ctx_, d->id, d->kind, d->for_nic);
  if (st != USN_OK) {
    LOGE("usn_endpoint_add(%u): %s", d->id, usn_strerror(st));
    return false;
  }
  devices_.push_back(d);
  ep_limit_ = std::max<uint32_t>(ep_limit_, (uint32_t)d->id + 1);
  LOGI("added endpoint %u (kind %d)", d->id, d->kind);
  return true;
}

DevP Daemon::add_nic(const std::string &iface) {
  auto d = std::make_shared<Dev>();
  d->kind = USN_EP_NIC;
  d->iface = iface;
  const int id = alloc_id();
  if (id < 0) return nullptr;
  d->id = (uint16_t)id;
  if (data_path_) {
    d->fd = socket(AF_UNIX, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    sockaddr_un a;
    socklen_t len;
    const std::string p = nic_dir_ + "/" + iface + ".nic";
    unlink(p.c_str());
    if (d->fd < 0 || !make_addr(p, a, len) || bind(d->fd, (sockaddr *)&a, len) != 0) {
      LOGE("cannot bind NIC wire %s: %s", p.c_str(), std::strerror(errno));
      return nullptr;
    }
    make_addr(nic_dir_ + "/" + iface + ".wire", d->peer, d->peer_len);
  }
  return register_dev(d) ? d : nullptr;
}

DevP Daemon::add_host_ring(const std::string &iface, const DevP &nic) {
  auto d = std::make_shared<Dev>();
  d->kind = USN_EP_HOST;
  d->iface = iface;
  d->for_nic = nic->id;
  const int id = alloc_id();
  if (id < 0) return nullptr;
  d->id = (uint16_t)id;
  if (data_path_) {
    d->fd = socket(AF_UNIX, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    sockaddr_un a;
    socklen_t len;
    const std::string p = nic_dir_ + "/" + iface + ".host";
    unlink(p.c_str());
    if (d->fd < 0 || !make_addr(p, a, len) || bind(d->fd, (sockaddr *)&a, len) != 0) {
      LOGE("cannot bind host ring %s: %s", p.c_str(), std::strerror(errno));
      return nullptr;
    }
    make_addr(nic_dir_ + "/" + iface + ".kernel", d->peer, d->peer_len);
  }
  return register_dev(d) ? d : nullptr;
}

/* Want::new_from_want_msg (pkt.rs:228-260) */
bool Daemon::want_of(const WantMsg &m, usn_want &w) {
  std::memset(&w, 0, sizeof w);
  if (m.dst.v6 || (m.has_src && m.src.v6)) {
    // the reference panics ("unimplemented"); the daemon logs and ignores
    LOGE("IPv6 match rules are not supported");
    return false;
  }
  if (!parse_ipv4(m.dst.text, w.dst_addr)) return false;
  if (m.has_src) {
    if (!parse_ipv4(m.src.text, w.src_addr)) w.src_addr = 0;   // :242-247 .ok() -> None
    else w.present |= USN_WANT_SRC;
  }
  if (m.has_dport) { w.dst_port = m.dport; w.present |= USN_WANT_DPORT; }
  if (m.has_sport) { w.src_port = m.sport; w.present |= USN_WANT_SPORT; }
  w.protocol = m.protocol;
  return true;
}

static bool parse_port_list(const std::string &list,
                            std::vector<std::tuple<std::string, uint8_t, int, std::string>> &out) {
  for (const std::string &entry : split(list, ',')) {
    auto parts = split(entry, ':');
    if (parts.size() < 2) return false;
    uint8_t proto;
    int port = -1;
    size_t k = 2;
    if (parts[1] == "ICMP") {
      proto = 1;
    } else if (parts[1] == "TCP" || parts[1] == "UDP") {
      proto = parts[1] == "TCP" ? 6 : 17;
      if (parts.size() < 3) return false;
      char *end = nullptr;
      const long v = std::strtol(parts[2].c_str(), &end, 10);
      if (parts[2].empty() || *end || v < 0 || v > 65535) return false;
      port = (int)v;
      k = 3;
    } else {
      return false;
    }
    std::string remote = parts.size() > k ? parts[k] : std::string();
    if (parts.size() > k + 1) return false;
    out.emplace_back(parts[0], proto, port, remote);
  }
  return true;
}

bool Daemon::setup_config() {
  if (!has_env("INTERFACES")) {
    LOGE("INTERFACES env var not specified");
    return false;
  }
  const bool host_rings = env("NO_HOST_RINGS") != "true";
  if (has_env("ADD_MACS")) {
    std::vector<std::array<uint8_t, 6>> macs;
    for (const std::string &m : split(env("ADD_MACS"), ',')) {
      auto b = split(m, ':');
      if (b.size() != 6) { LOGE("bad MAC %s", m.c_str()); return false; }
      std::array<uint8_t, 6> mac;
      for (int i = 0; i < 6; ++i) mac[i] = (uint8_t)std::strtoul(b[i].c_str(), nullptr, 16);
      usn_bridge_add(ctx_, mac.data());
    }
  }
  for (const std::string &iface : split(env("INTERFACES"), ',')) {
    DevP nic = add_nic(iface);
    if (!nic) return false;
    if (host_rings && !add_host_ring(iface, nic)) return false;
  }
  std::vector<std::tuple<std::string, uint8_t, int, std::string>> ports;
  if (has_env("DEBUG_PORTS")) {
    if (!parse_port_list(env("DEBUG_PORTS"), ports)) {
      LOGE("cannot parse DEBUG_PORTS");
      return false;
    }
    for (auto &t : ports) {   // add_debug_match_for_kernel (main.rs:300-309)
      uint32_t ip;
      if (!iface_ipv4(std::get<0>(t), ip)) { LOGE("no IPv4 on %s", std::get<0>(t).c_str()); return false; }
      DevP host;
      for (auto &d : devices_) if (d->kind == USN_EP_HOST && d->iface == std::get<0>(t)) host = d;
      if (!host) { LOGE("host ring not found"); return false; }
      usn_want w;
      std::memset(&w, 0, sizeof w);
      w.dst_addr = ip;
      w.protocol = std::get<1>(t);
      if (std::get<2>(t) >= 0) { w.dst_port = (uint16_t)std::get<2>(t); w.present |= USN_WANT_DPORT; }
      if (!std::get<3>(t).empty()) {
        if (!parse_ipv4(std::get<3>(t), w.src_addr)) { LOGE("bad remote IP"); return false; }
        w.present |= USN_WANT_SRC;
      }
      usn_add_match(ctx_, &w, host->id, 1);
    }
  }
  if (has_env("STATIC_PIPES")) {   // main.rs:940-957: needs netmap
    LOGE("compiled without netmap support, cannot add STATIC_PIPES");
    return false;
  }
  if (has_env("PCAP_LOG") && !pcap_.open(env("PCAP_LOG"))) {
    LOGE("cannot open PCAP_LOG file");
    return false;
  }
  return true;
}

bool Daemon::bind_control() {
  unlink(sock_path_.c_str());
  ctl_fd_ = socket(AF_UNIX, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  sockaddr_un a;
  socklen_t len;
  if (ctl_fd_ < 0 || !make_addr(sock_path_, a, len) || bind(ctl_fd_, (sockaddr *)&a, len) != 0) {
    LOGE("Cannot bind service socket %s: %s", sock_path_.c_str(), std::strerror(errno));
    return false;
  }
  if (has_env("ALLOW_GID")) {
    const long gid = std::strtol(env("ALLOW_GID").c_str(), nullptr, 10);
    if (chown(sock_path_.c_str(), (uid_t)-1, (gid_t)gid) != 0) {
      LOGE("chown to set group failed");
      return false;
    }
  }
  if (chmod(sock_path_.c_str(), 0770) != 0) {
    LOGE("chmod 770 failed");
    return false;
  }
  return true;
}

/* ---- control plane (act_on, main.rs:403-633) -------------------------------------- */
void Daemon::reply(const std::string &client_path, const std::string &msg) {
  sockaddr_un a;
  socklen_t len;
  if (!make_addr(client_path, a, len) ||
      sendto(ctl_fd_, msg.data(), msg.size(), 0, (sockaddr *)&a, len) != (ssize_t)msg.size())
    LOGE("cannot send to %s", client_path.c_str());
}

DevP Daemon::find_by_client_path(const std::string &p) {
  for (auto &d : devices_) if (d->client_path == p && !p.empty()) return d;
  return nullptr;
}

DevP Daemon::find_nic(const std::string &iface) {
  for (auto &d : devices_) if (d->kind == USN_EP_NIC && d->iface == iface) return d;
  return nullptr;
}

void Daemon::act_on(const ClientMessage &m, const std::string &client_path) {
  switch (m.type) {
    case ClientMessage::RequestUDS: {
      DevP nic = find_nic(m.iface);
      if (!nic) {
        reply(client_path, "ER");
        LOGE("nic %s not found", m.iface.c_str());
        return;
      }
      int sv[2];
      if (socketpair(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0, sv) != 0) {
        LOGE("no unix datagram pair created");
        return;
      }
      char payload = '$';
      iovec iov{&payload, 1};
      alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(int))];
      std::memset(cbuf, 0, sizeof cbuf);
      sockaddr_un a;
      socklen_t alen;
      make_addr(client_path, a, alen);
      msghdr mh{};
      mh.msg_name = &a;
      mh.msg_namelen = alen;
      mh.msg_iov = &iov;
      mh.msg_iovlen = 1;
      mh.msg_control = cbuf;
      mh.msg_controllen = sizeof cbuf;
      cmsghdr *cm = CMSG_FIRSTHDR(&mh);
      cm->cmsg_level = SOL_SOCKET;
      cm->cmsg_type = SCM_RIGHTS;
      cm->cmsg_len = CMSG_LEN(sizeof(int));
      std::memcpy(CMSG_DATA(cm), &sv[1], sizeof(int));
      if (sendmsg(ctl_fd_, &mh, 0) < 0) {
        LOGE("sndmsg failed: %s", std::strerror(errno));
        close(sv[0]);
        close(sv[1]);
        return;
      }
      close(sv[1]);   // the handover end now lives in the client
      fcntl(sv[0], F_SETFL, fcntl(sv[0], F_GETFL) | O_NONBLOCK);
      auto d = std::make_shared<Dev>();
      d->kind = USN_EP_UDS;
      d->for_nic = nic->id;
      d->client_path = client_path;
      d->fd = sv[0];
      const int id = alloc_id();
      if (id < 0) { LOGE("endpoint ids exhausted"); close(sv[0]); return; }
      d->id = (uint16_t)id;
      pipe_monitor_.emplace_back(m.pid, d);
      changes_.push_back(Change{Change::Add, d});
      return;
    }
    case ClientMessage::RequestNetmapPipe:   // built without netmap (main.rs:467-477)
      reply(client_path, "ER");
      return;
    case ClientMessage::AddMatch: {
      DevP d = find_by_client_path(client_path);
      if (!d) { LOGE("AddMatch: endpoint for %s not found", client_path.c_str()); return; }
      usn_want w;
      if (!want_of(m.want, w)) { LOGE("AddMatch: error parsing ip addr"); return; }
      const int st = usn_add_match(ctx_, &w, d->id, 0);
      if (st == 1) reply(client_path, "OK");
      else if (st == 0) reply(client_path, "ER");
      else LOGE("AddMatch: %s", usn_strerror(st));   // the reference panics (no NIC)
      return;
    }
    case ClientMessage::QueryUsedPorts: {   // main.rs:549-577
      const int n = usn_rule_count(ctx_);
      std::vector<usn_want> ws(std::max(n, 1));
      std::vector<uint16_t> own(std::max(n, 1));
      std::vector<uint8_t> st(std::max(n, 1));
      const int got = usn_rules_get(ctx_, ws.data(), own.data(), st.data(), (uint32_t)std::max(n, 0));
      std::vector<PortTriple> listening, connected;
      for (int i = 0; i < got; ++i) {
        if (!(ws[i].present & USN_WANT_DPORT)) continue;
        PortTriple t{ws[i].protocol, ws[i].dst_addr, ws[i].dst_port};
        ((ws[i].present & USN_WANT_SRC) ? connected : listening).push_back(t);
      }
      reply(client_path, encode_used_ports(listening, connected));
      return;
    }
    case ClientMessage::DeleteClient: {
      DevP d = find_by_client_path(client_path);
      if (d) {
        LOGI("got delete event from client");
        changes_.push_back(Change{Change::Remove, d});
      }
      return;
    }
    case ClientMessage::RemoveMatch: {   // main.rs:603-625: never answered
      DevP d = find_by_client_path(client_path);
      if (!d) return;
      usn_want w;
      if (!want_of(m.want, w)) { LOGW("could not convert to want msg"); return; }
      const int owner = usn_lookup(ctx_, &w);
      if (owner >= 0 && owner != d->id) {
        LOGW("want rule does not belong to client which requests removal");
        return;
      }
      if (owner < 0) LOGW("could not find rule to remove");
      usn_remove_match(ctx_, &w, d->id);
      return;
    }
    case ClientMessage::QueryUsedPortsAnswer:
      LOGW("received answer message from client, ignoring");
      return;
  }
}

void Daemon::dump(const std::string &client_path) {
  std::string out = "{\"endpoints\":[";
  for (size_t i = 0; i < devices_.size(); ++i) {
    const Dev &d = *devices_[i];
    if (i) out += ',';
    out += "[" + std::to_string(d.id) + "," + std::to_string(d.kind) + "," +
           std::to_string(d.for_nic) + ",";
    json_quote(out, d.iface);
    out += ',';
    json_quote(out, d.client_path);
    out += "," + std::to_string(d.frames_in) + "," + std::to_string(d.frames_out) + "]";
  }
  out += "],\"rules\":[";
  const int n = usn_rule_count(ctx_);
  std::vector<usn_want> ws(std::max(n, 1));
  std::vector<uint16_t> own(std::max(n, 1));
  std::vector<uint8_t> st(std::max(n, 1));
  const int got = usn_rules_get(ctx_, ws.data(), own.data(), st.data(), (uint32_t)std::max(n, 0));
  for (int i = 0; i < got; ++i) {
    if (i) out += ',';
    out += "[" + std::to_string(ws[i].dst_addr) + "," + std::to_string(ws[i].src_addr) + "," +
           std::to_string(ws[i].dst_port) + "," + std::to_string(ws[i].src_port) + "," +
           std::to_string(ws[i].protocol) + "," + std::to_string(ws[i].present) + "," +
           std::to_string(own[i]) + "," + std::to_string(st[i]) + "]";
  }
  out += "],\"bridge\":" + std::to_string(usn_bridge_count(ctx_)) + ",\"class_count\":[";
  for (int k = 0; k < 4; ++k) out += (k ? "," : "") + std::to_string(class_count_[k]);
  out += "]}";
  reply(client_path, out);
}

/* One datagram per poll round, as the reference (main.rs:990-1025): the
 * endpoint changes a message causes are applied before the next one is read. */
void Daemon::control_readable() {
  char buf[4000];   // client_buf (main.rs:980)
  {
    sockaddr_un from;
    socklen_t flen = sizeof from;
    const ssize_t len = recvfrom(ctl_fd_, buf, sizeof buf, 0, (sockaddr *)&from, &flen);
    if (len < 0) return;
    if (flen <= offsetof(sockaddr_un, sun_path) || from.sun_path[0] == '\0') {
      LOGE("no client path");
      return;
    }
    const std::string client_path(from.sun_path, strnlen(from.sun_path, sizeof from.sun_path));
    const std::string text(buf, (size_t)len);
    ClientMessage m;
    if (decode_message(text, m)) {
      act_on(m, client_path);
    } else if (text == "cleanup") {
      changes_.push_back(Change{Change::Cleanup, nullptr});
    } else if (text == "end") {
      end_ = true;
      return;
    } else if (test_dump_ && text == "dump") {
      dump(client_path);
    } else {
      LOGE("no json: %s", text.c_str());
    }
  }
}

static std::set<uint16_t> read_ports_from(const char *file, bool &ok) {
  std::set<uint16_t> ports;
  std::ifstream in(file);
  ok = (bool)in;
  std::string line;
  std::getline(in, line);   // header
  while (std::getline(in, line)) {
    auto parts = split(line, ':');
    if (parts.size() < 3) continue;
    const std::string hex = split(parts[2], ' ')[0];
    ports.insert((uint16_t)std::strtoul(hex.c_str(), nullptr, 16));
  }
  return ports;
}

void Daemon::cleanup() {   // EntryChange::Cleanup (main.rs:1070-1110)
  usn_frag_clear(ctx_);
  bool ok_t, ok_u;
  const auto tcp = read_ports_from("/proc/net/tcp", ok_t);
  const auto udp = read_ports_from("/proc/net/udp", ok_u);
  if (!ok_t || !ok_u) { LOGE("cannot open /proc/net/tcp|udp"); return; }
  const int n = usn_rule_count(ctx_);
  std::vector<usn_want> ws(std::max(n, 1));
  std::vector<uint16_t> own(std::max(n, 1));
  std::vector<uint8_t> st(std::max(n, 1));
  const int got = usn_rules_get(ctx_, ws.data(), own.data(), st.data(), (uint32_t)std::max(n, 0));
  int removed = 0;
  for (int i = 0; i < got; ++i) {
    DevP d = by_id(own[i]);
    if (!d || d->kind != USN_EP_HOST || st[i]) continue;
    bool drop = true;   // no dst_port, or a protocol without a /proc/net table
    if (ws[i].present & USN_WANT_DPORT) {
      if (ws[i].protocol == 6) drop = !tcp.count(ws[i].dst_port);
      else if (ws[i].protocol == 17) drop = !udp.count(ws[i].dst_port);
    }
    if (drop && usn_remove_match(ctx_, &ws[i], own[i]) == 1) ++removed;
  }
  LOGI("cleanup: %d host-ring rules released; classes drop/ep/nic/flood = %llu/%llu/%llu/%llu",
       removed, (unsigned long long)class_count_[0], (unsigned long long)class_count_[1],
       (unsigned long long)class_count_[2], (unsigned long long)class_count_[3]);
  pcap_.flush();
}

void Daemon::remove_dev(const DevP &d) {
  auto it = std::find(devices_.begin(), devices_.end(), d);
  if (it == devices_.end()) { LOGI("double remove call"); return; }
  usn_endpoint_remove(ctx_, d->id);   // match_register.retain (main.rs:1062-1064)
  pipe_monitor_.erase(std::remove_if(pipe_monitor_.begin(), pipe_monitor_.end(),
                                     [&](const std::pair<uint64_t, DevP> &p) { return p.second == d; }),
                      pipe_monitor_.end());
  if (d->res[0] || d->res[1]) {
    select(d->rep);
    for (int k = 0; k < 2; ++k)
      if (d->res[k]) {
        usn_result_release(ctx_, &d->rb[k]);
        usn_dev_free(ctx_, d->res[k]);
      }
  }
  if (d->fd >= 0) close(d->fd);
  if (d->txfd >= 0) close(d->txfd);
  used_ids_[d->id] = 0;
  devices_.erase(it);
  LOGI("cleared endpoint %u", d->id);
}

void Daemon::apply_changes() {
  if (!changes_.empty())   // liveness of the clients (main.rs:1050-1057)
    for (auto &pm : pipe_monitor_) {
      const std::string probe = "/proc/" + std::to_string(pm.first) + "/cmdline";
      if (access(probe.c_str(), R_OK) != 0) changes_.push_back(Change{Change::Remove, pm.second});
    }
  while (!changes_.empty()) {   // popped from the back, as the reference does
    Change c = changes_.back();
    changes_.pop_back();
    if (c.type == Change::Add) {
      if (!register_dev(c.dev)) { close(c.dev->fd); used_ids_[c.dev->id] = 0; }
    } else if (c.type == Change::Remove) {
      remove_dev(c.dev);
    } else {
      cleanup();
    }
  }
}

/* ---- data path ------------------------------------------------------------------- */
bool Daemon::select(uint32_t rep) {
  const int st = usn_replica_select(ctx_, rep);
  if (st != USN_OK) LOGE("usn_replica_select(%u): %s", rep, usn_strerror(st));
  return st == USN_OK;
}

bool Daemon::data_path_init() {
  const int n = usn_ctx_replicas(ctx_);
  if (n <= 0) return false;
  reps_.resize((size_t)n);
  for (int r = 0; r < n; ++r)
    if (!select((uint32_t)r) || usn_stream_create(ctx_, &reps_[r].stream) != USN_OK) return false;
  return true;
}

/* Endpoint writes (EndpointDevice::write) of the frames `idx` (arena
 * indices, in order) by sendmmsg.  A full peer queue gets up to
 * USNETD_WRITE_WAIT_MS for room; frames that still do not fit are dropped
 * with a debug log (a full tx ring).  Returns 1 when the client has vanished
 * (Error::Unaddressable, endpoint.rs:90-105): it is removed after the round. */
int Daemon::write_frames(const DevP &t, const std::vector<uint32_t> &idx) {
  if (idx.empty()) return 0;
  int fd = t->fd;
  if (t->kind != USN_EP_UDS) {   // the wire / kernel side, connected for flow control
    if (t->txfd < 0) {
      t->txfd = socket(AF_UNIX, SOCK_DGRAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
      if (t->txfd >= 0 && connect(t->txfd, (sockaddr *)&t->peer, t->peer_len) != 0) {
        close(t->txfd);
        t->txfd = -1;
      }
      if (t->txfd < 0) { LOGD("no peer for endpoint %u", t->id); return 0; }
    }
    fd = t->txfd;
  }
  static const size_t VLEN = 256;
  std::vector<mmsghdr> msgs(std::min(idx.size(), VLEN));
  std::vector<iovec> iov(msgs.size());
  size_t done = 0;
  int budget = write_wait_ms_;
  while (done < idx.size()) {
    const size_t k = std::min(idx.size() - done, VLEN);
    for (size_t j = 0; j < k; ++j) {
      const uint32_t i = idx[done + j];
      iov[j].iov_base = arena_.data() + off_[i];
      iov[j].iov_len = len_[i];
      std::memset(&msgs[j], 0, sizeof msgs[j]);
      msgs[j].msg_hdr.msg_iov = &iov[j];
      msgs[j].msg_hdr.msg_iovlen = 1;
    }
    const int r = sendmmsg(fd, msgs.data(), (unsigned)k, MSG_DONTWAIT | MSG_NOSIGNAL);
    if (r > 0) {
      done += (size_t)r;
      t->frames_out += (uint64_t)r;
      continue;
    }
    const int e = errno;
    if (e == EAGAIN && budget > 0) {
      const auto t0 = std::chrono::steady_clock::now();
      pollfd pf{fd, POLLOUT, 0};
      poll(&pf, 1, budget);
      budget -= (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                    std::chrono::steady_clock::now() - t0).count() + 1;
      continue;
    }
    if (e == EAGAIN) {
      LOGD("endpoint %u: queue full, %zu frames dropped", t->id, idx.size() - done);
      return 0;
    }
    LOGD("Write error %s for endpoint %u", std::strerror(e), t->id);
    if (t->kind == USN_EP_UDS && (e == ECONNREFUSED || e == EPIPE || e == ENOTCONN || e == ECONNRESET))
      return 1;
    if (t->kind != USN_EP_UDS && (e == ECONNREFUSED || e == ENOTCONN)) {   // peer went away
      close(t->txfd);
      t->txfd = -1;
      return 0;
    }
    ++done;   // this frame cannot be sent (e.g. EMSGSIZE): skip it
  }
  return 0;
}

void Daemon::forward_round(const std::vector<DevP> &ready) {
  /* 1. drain every readable endpoint, in device order */
  struct Src {
    DevP dev;
    uint32_t start, n;     // arena frames [start, start + n)
    uint32_t dstart;       // first window in its replica's device buffer
    size_t out_off;        // summary / bin offsets / index in the replica's h_out
    usn_batch b;
    usn_result res;
  };
  std::vector<Src> srcs;
  arena_.clear();
  off_.clear();
  len_.clear();
  static thread_local std::vector<uint8_t> buf(1 << 16);
  for (const DevP &d : ready) {
    Src s{};
    s.dev = d;
    s.start = (uint32_t)len_.size();
    while (s.n < max_batch_) {
      const ssize_t r = recv(d->fd, buf.data(), buf.size(), MSG_DONTWAIT);
      if (r < 0) break;
      pcap_.packet(buf.data(), (uint32_t)r);
      off_.push_back(arena_.size());
      len_.push_back((uint32_t)r);
      arena_.insert(arena_.end(), buf.begin(), buf.begin() + r);
      ++s.n;
    }
    d->frames_in += s.n;
    if (s.n) srcs.push_back(s);
  }
  if (srcs.empty()) return;
  /* 2. per replica: the header windows + lengths of its sources to its device */
  const uint32_t R = (uint32_t)reps_.size();
  std::vector<uint32_t> total(R, 0);
  std::vector<size_t> outb(R, 0);
  for (Src &s : srcs) {
    const uint32_t r = s.dev->rep;
    s.dstart = total[r];
    total[r] += s.n;
    s.out_off = outb[r];
    outb[r] += OUT_HEAD + (size_t)s.n * 4;
  }
  for (uint32_t r = 0; r < R; ++r) {
    RepBuf &B = reps_[r];
    if (!total[r]) continue;
    if (!select(r)) { end_ = true; return; }
    if (total[r] > B.cap) {
      if (B.h_hdr) {
        usn_host_free_pinned(ctx_, B.h_hdr);
        usn_host_free_pinned(ctx_, B.h_lens);
        usn_dev_free(ctx_, B.d_hdr);
        usn_dev_free(ctx_, B.d_lens);
        B.h_hdr = B.d_hdr = nullptr;
        B.h_lens = B.d_lens = nullptr;
      }
      B.cap = std::max<uint32_t>(total[r], 4096);
      if (usn_host_alloc_pinned(ctx_, (size_t)B.cap * HDR + 64, (void **)&B.h_hdr) ||
          usn_host_alloc_pinned(ctx_, (size_t)B.cap * 2, (void **)&B.h_lens) ||
          usn_dev_alloc(ctx_, (size_t)B.cap * HDR + 64, (void **)&B.d_hdr) ||
          usn_dev_alloc(ctx_, (size_t)B.cap * 2, (void **)&B.d_lens)) {
        LOGE("data path buffers of replica %u: out of memory", r);
        B.cap = 0;
        end_ = true;
        return;
      }
    }
    if (outb[r] > B.out_cap) {
      if (B.h_out) usn_host_free_pinned(ctx_, B.h_out);
      B.h_out = nullptr;
      B.out_cap = 0;
      if (usn_host_alloc_pinned(ctx_, outb[r], (void **)&B.h_out)) {
        LOGE("result staging of replica %u: out of memory", r);
        end_ = true;
        return;
      }
      B.out_cap = outb[r];
    }
  }
  for (Src &s : srcs) {
    RepBuf &B = reps_[s.dev->rep];
    for (uint32_t j = 0; j < s.n; ++j) {
      const uint32_t i = s.start + j, w = s.dstart + j;
      const uint32_t c = std::min<uint32_t>(len_[i], HDR);
      std::memcpy(B.h_hdr + (size_t)w * HDR, arena_.data() + off_[i], c);
      std::memset(B.h_hdr + (size_t)w * HDR + c, 0, HDR - c);
      B.h_lens[w] = (uint16_t)std::min<uint32_t>(len_[i], 0xFFFF);
    }
  }
  for (uint32_t r = 0; r < R; ++r) {
    if (!total[r]) continue;
    RepBuf &B = reps_[r];
    select(r);
    usn_memcpy_h2d(ctx_, B.d_hdr, B.h_hdr, (size_t)total[r] * HDR, B.stream);
    usn_memcpy_h2d(ctx_, B.d_lens, B.h_lens, (size_t)total[r] * 2, B.stream);
  }
  /* 3. batches and result buffers (two per source: the carried cache reads
   *    the previous batch's result) */
  for (Src &s : srcs) {
    RepBuf &B = reps_[s.dev->rep];
    usn_batch &b = s.b;
    std::memset(&b, 0, sizeof b);
    b.frames = B.d_hdr + (size_t)s.dstart * HDR;
    b.stride = HDR;
    b.window = HDR;                // whole 128-byte windows: never past USN_WINDOW_MAX
    b.lens = B.d_lens + s.dstart;
    b.n = s.n;
    b.src_endpoint = s.dev->id;
    Dev &d = *s.dev;
    d.cur ^= 1;
    if (!d.res[d.cur]) {
      select(d.rep);
      if (usn_dev_alloc(ctx_, usn_result_bytes(max_batch_), &d.res[d.cur]) != USN_OK) {
        LOGE("result buffer of endpoint %u: out of memory", d.id);
        end_ = true;
        return;
      }
      usn_result_bind(d.res[d.cur], usn_result_bytes(max_batch_), max_batch_, &d.rb[d.cur]);
    }
    s.res = d.rb[d.cur];
  }
  /* 4. classify in device order.  A run of consecutive NIC rings changes no
   *    shared state: its rings go to their replicas' GPUs at once (up to 8
   *    per launch), then are finalized in order.  A sending endpoint's ring
   *    learns (endpoint.rs:194-253), so it is classified and finalized alone
   *    before anything after it. */
  int st = USN_OK;
  for (size_t k = 0; k < srcs.size() && st == USN_OK;) {
    size_t e = k + 1;
    if (srcs[k].dev->kind == USN_EP_NIC)
      while (e < srcs.size() && srcs[e].dev->kind == USN_EP_NIC) ++e;
    for (uint32_t r = 0; r < R && st == USN_OK; ++r) {
      std::vector<usn_batch> bs;
      std::vector<usn_result> rs;
      auto flush = [&]() {
        if (bs.empty()) return;
        st = usn_classify_multi(ctx_, bs.data(), rs.data(), (uint32_t)bs.size(), reps_[r].stream);
        bs.clear();
        rs.clear();
      };
      for (size_t j = k; j < e && st == USN_OK; ++j) {
        if (srcs[j].dev->rep != r) continue;
        if (bs.empty() && !select(r)) { st = USN_EINVAL; break; }
        bs.push_back(srcs[j].b);
        rs.push_back(srcs[j].res);
        if (bs.size() == 8) flush();
      }
      if (st == USN_OK) flush();
    }
    for (size_t j = k; j < e && st == USN_OK; ++j) {
      Src &s = srcs[j];
      RepBuf &B = reps_[s.dev->rep];
      usn_finalize_info info;
      std::memset(&info, 0, sizeof info);
      st = usn_finalize(ctx_, &s.b, &s.res, B.stream, &info);
      if (st != USN_OK) break;
      for (int c = 0; c < 4; ++c) class_count_[c] += info.class_count[c];
      /* the per-endpoint lists: summary (n_ep), bin offsets, index */
      uint8_t *o = B.h_out + s.out_off;
      select(s.dev->rep);
      usn_memcpy_d2h(ctx_, o, s.res.summary, sizeof(usn_summary), B.stream);
      // bin_off entries the batch can use: its bins are at most today's
      // n_ep + 3 (not the whole USN_MAX_BINS + 1 array per source)
      const size_t nbo = std::min<size_t>((size_t)ep_limit_ + 4, USN_MAX_BINS + 1);
      usn_memcpy_d2h(ctx_, o + OUT_BINS, s.res.bin_off, nbo * 4, B.stream);
      usn_memcpy_d2h(ctx_, o + OUT_HEAD, s.res.index, (size_t)s.n * 4, B.stream);
    }
    k = e;
  }
  if (st != USN_OK) {
    LOGE("classify failed: %s (hip %d)", usn_strerror(st), usn_last_hip_error());
    end_ = true;
    return;
  }
  for (uint32_t r = 0; r < R; ++r)
    if (total[r]) { select(r); usn_stream_sync(ctx_, reps_[r].stream); }
  /* 5. deliver, source by source, each target's frames in frame order with
   *    one sendmmsg stream per target: its list of the device-wide scatter
   *    (usn_result.index, grouped by bin), with FLOOD (mirror_to_all,
   *    endpoint.rs:340-363: every endpoint but the source) and Target::Nic
   *    merged in by frame index */
  std::vector<DevP> unaddressable;
  std::vector<std::vector<uint32_t>> per(USN_MAX_ENDPOINTS);
  std::vector<uint32_t> nic, flood, merged, tmp;
  std::vector<uint16_t> touched;
  for (const Src &s : srcs) {
    const uint8_t *o = reps_[s.dev->rep].h_out + s.out_off;
    const usn_summary *sum = reinterpret_cast<const usn_summary *>(o);
    const uint32_t *bin_off = reinterpret_cast<const uint32_t *>(o + OUT_BINS);
    const uint32_t *index = reinterpret_cast<const uint32_t *>(o + OUT_HEAD);
    const uint32_t bn = sum->n_ep;
    auto list = [&](uint32_t bin, std::vector<uint32_t> &dst) {
      for (uint32_t p = bin_off[bin]; p < bin_off[bin + 1]; ++p) dst.push_back(s.start + index[p]);
    };
    nic.clear();
    flood.clear();
    touched.clear();
    list(bn, nic);
    list(bn + 1, flood);
    for (uint32_t bin = 0; bin < bn; ++bin) {
      if (bin_off[bin] == bin_off[bin + 1]) continue;
      touched.push_back((uint16_t)bin);
      list(bin, per[bin]);
    }
    const uint32_t nic_id = (uint32_t)s.dev->for_nic;   // Target::Nic of a sending endpoint
    for (const DevP &t : devices_) {
      const bool fl = !flood.empty() && t != s.dev;
      const bool ni = !nic.empty() && t->id == nic_id;
      std::vector<uint32_t> &mine = per[t->id];
      if (mine.empty() && !fl && !ni) continue;
      const std::vector<uint32_t> *out = &mine;
      if (fl || ni) {   // merge the sorted lists by frame index
        const std::vector<uint32_t> &x = fl ? flood : nic;
        merged.resize(mine.size() + x.size());
        std::merge(mine.begin(), mine.end(), x.begin(), x.end(), merged.begin());
        if (fl && ni) {
          tmp.resize(merged.size() + nic.size());
          std::merge(merged.begin(), merged.end(), nic.begin(), nic.end(), tmp.begin());
          merged.swap(tmp);
        }
        out = &merged;
      }
      if (write_frames(t, *out)) unaddressable.push_back(t);
    }
    for (uint16_t b : touched) per[b].clear();
  }
  std::sort(unaddressable.begin(), unaddressable.end());
  unaddressable.erase(std::unique(unaddressable.begin(), unaddressable.end()), unaddressable.end());
  for (const DevP &t : unaddressable) changes_.push_back(Change{Change::Remove, t});
}

/* ---- main loop --------------------------------------------------------------------- */
int Daemon::run(int argc, char **argv) {
  if (argc > 1 && !load_dotenv(argv[1])) {
    std::fprintf(stderr, "could not open configuration file %s\n", argv[1]);
    return 1;
  }
  {
    const std::string lv = env("RUST_LOG", env("USNETD_LOG", "warn").c_str());
    g_level = lv == "error" ? 0 : lv == "info" ? 2 : (lv == "debug" || lv == "trace") ? 3 : 1;
  }
  sock_path_ = env("USNETD_SOCKET", "/run/usnetd.socket");
  {
    const size_t sl = sock_path_.rfind('/');
    nic_dir_ = env("USNETD_NIC_DIR", sl == std::string::npos ? "." : sock_path_.substr(0, sl).c_str());
  }
  data_path_ = env("USNETD_CONTROL_ONLY") != "1";
  test_dump_ = env("USNETD_TEST_DUMP") == "1";
  if (has_env("USNETD_CLEANUP_SECS"))
    cleanup_secs_ = (unsigned)std::max(1L, std::strtol(env("USNETD_CLEANUP_SECS").c_str(), nullptr, 10));
  if (has_env("USNETD_WRITE_WAIT_MS"))
    write_wait_ms_ = std::max(0, std::atoi(env("USNETD_WRITE_WAIT_MS").c_str()));
  if (has_env("USNETD_MAX_BATCH"))
    max_batch_ = (uint32_t)std::max(1L, std::strtol(env("USNETD_MAX_BATCH").c_str(), nullptr, 10));
  /* USNETD_HIP_DEVICES=0,1,...: one registry, a device replica per GPU; the
   * NICs' rings are spread over them (USNETD_HIP_DEVICE: a single GPU) */
  std::vector<int> devs;
  if (data_path_) {
    if (has_env("USNETD_HIP_DEVICES")) {
      for (const std::string &x : split(env("USNETD_HIP_DEVICES"), ','))
        if (!x.empty()) devs.push_back(std::atoi(x.c_str()));
    } else {
      devs.push_back(std::atoi(env("USNETD_HIP_DEVICE", "0").c_str()));
    }
  }
  int st = data_path_ ? usn_ctx_create_group(devs.data(), (uint32_t)devs.size(), &ctx_)
                      : usn_ctx_create(USN_HOST_ONLY, &ctx_);
  if (st != USN_OK) {
    LOGE("usn_ctx_create: %s -- the match path needs a gfx950 GPU "
         "(USNETD_CONTROL_ONLY=1 runs the control plane alone)", usn_strerror(st));
    return 1;
  }
  if (data_path_ && !data_path_init()) { LOGE("data path init failed"); return 1; }
  if (!bind_control() || !setup_config()) return 1;

  signal(SIGINT, on_signal);
  signal(SIGTERM, on_signal);
  signal(SIGPIPE, SIG_IGN);
  const std::string timer_path = sock_path_ + "timer";
  const unsigned secs = cleanup_secs_;
  std::thread timer([timer_path, secs, this]() {   // cleanup() thread (main.rs:673-701)
    unlink(timer_path.c_str());
    const int fd = socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0);
    sockaddr_un a, to;
    socklen_t al = 0, tl = 0;
    make_addr(timer_path, a, al);
    make_addr(sock_path_, to, tl);
    if (fd < 0 || bind(fd, (sockaddr *)&a, al) != 0) { LOGE("Cannot bind timer socket"); return; }
    unsigned counter = 0;
    for (;;) {
      std::this_thread::sleep_for(std::chrono::seconds(1));
      ++counter;
      const char *msg = nullptr;
      if (g_signal.load()) msg = "end";
      else if (counter == secs) { counter = 0; msg = "cleanup"; }
      if (msg) {
        sendto(fd, msg, std::strlen(msg), 0, (sockaddr *)&to, tl);
        if (!std::strcmp(msg, "end")) break;
      }
    }
    close(fd);
    unlink(timer_path.c_str());
  });
  LOGI("usnetd ready on %s (%s)", sock_path_.c_str(), data_path_ ? "GPU data path" : "control only");
  while (!end_) {
    std::vector<pollfd> pf;
    pf.push_back(pollfd{ctl_fd_, POLLIN, 0});
    std::vector<DevP> polled;
    if (data_path_)
      for (auto &d : devices_)
        if (d->fd >= 0) { pf.push_back(pollfd{d->fd, POLLIN, 0}); polled.push_back(d); }
    if (poll(pf.data(), pf.size(), -1) < 0) {
      if (errno == EINTR) continue;
      LOGE("poll error: %s", std::strerror(errno));
      continue;
    }
    if (pf[0].revents & POLLIN) control_readable();
    std::vector<DevP> ready;
    for (size_t i = 1; i < pf.size(); ++i)
      if (pf[i].revents & POLLIN) ready.push_back(polled[i - 1]);
    if (!ready.empty() && !end_) forward_round(ready);
    apply_changes();
  }
  LOGI("Clean shutdown");
  g_signal.store(true);
  timer.join();
  for (auto &d : std::vector<DevP>(devices_)) remove_dev(d);
  unlink(sock_path_.c_str());
  usn_ctx_destroy(ctx_);
  return 0;
}

}  // namespace usnd

int main(int argc, char **argv) {
  usnd::Daemon d;
  return d.run(argc, argv);
}
