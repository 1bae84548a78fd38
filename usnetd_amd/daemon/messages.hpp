/*
 * messages.hpp -- the control-socket message set of usnetd and its serde
 * encoding, restated for C++.
 *
 * Types (/root/reference/src/lib.rs:6-33): ClientMessage is an externally
 * tagged serde enum:
 *   unit     "DeleteClient", "QueryUsedPorts"            (or {"X": null})
 *   tuple    {"RequestUDS": ["eth0", 1234]}, {"RequestNetmapPipe": [..]}
 *   newtype  {"AddMatch": WantMsg}, {"RemoveMatch": WantMsg}
 *   struct   {"QueryUsedPortsAnswer": {"listening": [...], "connected": [...]}}
 * WantMsg {dst_addr: ClientMessageIp, dst_port: Option<u16>, src_addr:
 * Option<ClientMessageIp>, src_port: Option<u16>, protocol: u8}; a derived
 * serde struct is read from a map (any order, unknown keys ignored,
 * duplicate keys rejected, missing Option fields = None) or from a sequence
 * of exactly its fields in order.  ClientMessageIp is {"Ipv4": "a.b.c.d"} or
 * {"Ipv6": "..."}.  Unsigned fields take only integer literals in range.
 */
#ifndef USND_MESSAGES_HPP
#define USND_MESSAGES_HPP

#include <cstdint>
#include <string>
#include <vector>

#include "json.hpp"

namespace usnd {

struct IpMsg {
  bool v6 = false;
  std::string text;
};

struct WantMsg {
  IpMsg dst;
  bool has_dport = false, has_src = false, has_sport = false;
  uint16_t dport = 0, sport = 0;
  IpMsg src;
  uint8_t protocol = 0;
};

struct ClientMessage {
  enum Type {
    RequestNetmapPipe, RequestUDS, DeleteClient, AddMatch, RemoveMatch, QueryUsedPorts,
    QueryUsedPortsAnswer
  } type = DeleteClient;
  std::string iface;   // RequestNetmapPipe / RequestUDS
  uint64_t pid = 0;
  WantMsg want;        // AddMatch / RemoveMatch
};

namespace detail {

inline bool as_u(const Json &v, uint64_t max, uint64_t &out) {
  if (v.kind != Json::Number || !v.is_uint || v.u > max) return false;
  out = v.u;
  return true;
}

inline bool as_ip(const Json &v, IpMsg &ip) {
  if (v.kind != Json::Object || v.o.size() != 1) return false;
  const auto &kv = v.o[0];
  if (kv.second.kind != Json::String) return false;
  if (kv.first == "Ipv4") ip.v6 = false;
  else if (kv.first == "Ipv6") ip.v6 = true;
  else return false;
  ip.text = kv.second.s;
  return true;
}

inline bool opt_u16(const Json &v, bool &has, uint16_t &out) {
  if (v.kind == Json::Null) { has = false; return true; }
  uint64_t u;
  if (!as_u(v, 0xFFFF, u)) return false;
  has = true;
  out = (uint16_t)u;
  return true;
}

inline bool opt_ip(const Json &v, bool &has, IpMsg &ip) {
  if (v.kind == Json::Null) { has = false; return true; }
  has = true;
  return as_ip(v, ip);
}

inline bool want_from(const Json &v, WantMsg &w) {
  static const char *names[5] = {"dst_addr", "dst_port", "src_addr", "src_port", "protocol"};
  const Json *f[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  if (v.kind == Json::Array) {
    if (v.a.size() != 5) return false;
    for (int k = 0; k < 5; ++k) f[k] = &v.a[k];
  } else if (v.kind == Json::Object) {
    for (const auto &kv : v.o)
      for (int k = 0; k < 5; ++k)
        if (kv.first == names[k]) {
          if (f[k]) return false;        // duplicate field
          f[k] = &kv.second;
        }
    if (!f[0] || !f[4]) return false;    // required: dst_addr, protocol
  } else {
    return false;
  }
  if (!as_ip(*f[0], w.dst)) return false;
  if (f[1] && !opt_u16(*f[1], w.has_dport, w.dport)) return false;
  if (f[2] && !opt_ip(*f[2], w.has_src, w.src)) return false;
  if (f[3] && !opt_u16(*f[3], w.has_sport, w.sport)) return false;
  uint64_t p;
  if (!as_u(*f[4], 0xFF, p)) return false;
  w.protocol = (uint8_t)p;
  return true;
}

/* Vec<(u8, ClientMessageIp, u16)> */
inline bool triples(const Json &v) {
  if (v.kind != Json::Array) return false;
  for (const Json &t : v.a) {
    uint64_t u;
    IpMsg ip;
    if (t.kind != Json::Array || t.a.size() != 3 || !as_u(t.a[0], 0xFF, u) ||
        !as_ip(t.a[1], ip) || !as_u(t.a[2], 0xFFFF, u))
      return false;
  }
  return true;
}

}  // namespace detail

/* serde_json::from_str::<ClientMessage>: false where serde would fail */
inline bool decode_message(const std::string &text, ClientMessage &m) {
  Json v;
  if (!JsonReader(text).parse(v)) return false;
  std::string tag;
  const Json *body = nullptr;
  if (v.kind == Json::String) {
    tag = v.s;
  } else if (v.kind == Json::Object && v.o.size() == 1) {
    tag = v.o[0].first;
    body = &v.o[0].second;
  } else {
    return false;
  }
  if (tag == "DeleteClient" || tag == "QueryUsedPorts") {
    if (body && body->kind != Json::Null) return false;
    m.type = tag == "DeleteClient" ? ClientMessage::DeleteClient : ClientMessage::QueryUsedPorts;
    return true;
  }
  if (!body) return false;   // a non-unit variant named by a bare string
  if (tag == "RequestUDS" || tag == "RequestNetmapPipe") {
    if (body->kind != Json::Array || body->a.size() != 2 || body->a[0].kind != Json::String)
      return false;
    if (!detail::as_u(body->a[1], UINT64_MAX, m.pid)) return false;
    m.iface = body->a[0].s;
    m.type = tag == "RequestUDS" ? ClientMessage::RequestUDS : ClientMessage::RequestNetmapPipe;
    return true;
  }
  if (tag == "AddMatch" || tag == "RemoveMatch") {
    m.type = tag == "AddMatch" ? ClientMessage::AddMatch : ClientMessage::RemoveMatch;
    return detail::want_from(*body, m.want);
  }
  if (tag == "QueryUsedPortsAnswer") {
    const Json *l = nullptr, *c = nullptr;
    if (body->kind == Json::Array) {
      if (body->a.size() != 2) return false;
      l = &body->a[0];
      c = &body->a[1];
    } else if (body->kind == Json::Object) {
      for (const auto &kv : body->o) {
        if (kv.first == "listening") { if (l) return false; l = &kv.second; }
        if (kv.first == "connected") { if (c) return false; c = &kv.second; }
      }
    } else {
      return false;
    }
    if (!l || !c || !detail::triples(*l) || !detail::triples(*c)) return false;
    m.type = ClientMessage::QueryUsedPortsAnswer;
    return true;
  }
  return false;
}

/* smoltcp 0.7.0 Ipv4Address::from_str (recalled): four
 * dot-separated decimal octets of 1-3 digits each, value < 256, nothing else. */
inline bool parse_ipv4(const std::string &s, uint32_t &out) {
  size_t i = 0;
  uint32_t v = 0;
  for (int oct = 0; oct < 4; ++oct) {
    if (oct) {
      if (i >= s.size() || s[i] != '.') return false;
      ++i;
    }
    uint32_t n = 0;
    int digits = 0;
    while (i < s.size() && digits < 3 && s[i] >= '0' && s[i] <= '9') {
      n = n * 10 + (uint32_t)(s[i] - '0');
      ++i;
      ++digits;
    }
    if (!digits || n >= 256) return false;
    v = (v << 8) | n;
  }
  if (i != s.size()) return false;
  out = v;
  return true;
}

inline std::string ipv4_text(uint32_t a) {
  return std::to_string(a >> 24) + "." + std::to_string((a >> 16) & 255) + "." +
         std::to_string((a >> 8) & 255) + "." + std::to_string(a & 255);
}

struct PortTriple {
  uint8_t proto;
  uint32_t addr;
  uint16_t port;
};

/* serde_json::to_string(&ClientMessage::QueryUsedPortsAnswer{..}) */
inline std::string encode_used_ports(const std::vector<PortTriple> &listening,
                                     const std::vector<PortTriple> &connected) {
  std::string out = "{\"QueryUsedPortsAnswer\":{\"listening\":[";
  auto list = [&out](const std::vector<PortTriple> &v) {
    for (size_t i = 0; i < v.size(); ++i) {
      if (i) out += ',';
      out += '[' + std::to_string(v[i].proto) + ",{\"Ipv4\":";
      json_quote(out, ipv4_text(v[i].addr));
      out += "}," + std::to_string(v[i].port) + ']';
    }
  };
  list(listening);
  out += "],\"connected\":[";
  list(connected);
  out += "]}}";
  return out;
}

}  // namespace usnd

#endif
