// kredis-server: see store.hpp for scope.
//
//   kredis-server [--bind 127.0.0.1] [--port 6379]
//                 [--sentinel NAME HOST PORT] [--replica HOST:PORT]...
//                 [--redis-version X.Y]   (5.0: no LMOVE/BLMOVE, integer
//                                          blocking timeouts, no SCAN TYPE)
//
// Semantics follow Redis 7 for every implemented command (reply types,
// WRONGTYPE, negative list indices, LMOVE/BLMOVE direction arguments, SET
// EX/PX/NX/XX, SCAN MATCH/COUNT/TYPE).  Blocking pops park the client;
// any list push re-serves parked clients in FIFO order.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <stdexcept>
#include <list>
#include <memory>

#include "store.hpp"

namespace kredis {

// SIGTERM/SIGINT end the event loop normally (destructors and, in the
// sanitizer build, LeakSanitizer's exit check run)
volatile sig_atomic_t g_terminate = 0;

int64_t now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000 + ts.tv_nsec / 1000000;
}

// Redis-style glob: * ? [abc] [^a-z] and backslash escapes.
bool glob_match(const char* p, size_t plen, const char* s, size_t slen) {
  while (plen > 0) {
    switch (*p) {
      case '*': {
        while (plen > 1 && p[1] == '*') { ++p; --plen; }
        if (plen == 1) return true;
        for (size_t i = 0; i <= slen; ++i)
          if (glob_match(p + 1, plen - 1, s + i, slen - i)) return true;
        return false;
      }
      case '?':
        if (slen == 0) return false;
        ++s; --slen;
        break;
      case '[': {
        if (slen == 0) return false;
        ++p; --plen;
        bool negate = false, match = false;
        if (plen > 0 && *p == '^') { negate = true; ++p; --plen; }
        while (plen > 0 && *p != ']') {
          if (*p == '\\' && plen >= 2) {
            ++p; --plen;
            if (*p == *s) match = true;
          } else if (plen >= 3 && p[1] == '-') {
            char lo = p[0], hi = p[2];
            if (lo > hi) std::swap(lo, hi);
            if (*s >= lo && *s <= hi) match = true;
            p += 2; plen -= 2;
          } else if (*p == *s) {
            match = true;
          }
          ++p; --plen;
        }
        if (negate) match = !match;
        if (!match) return false;
        ++s; --slen;
        break;
      }
      case '\\':
        if (plen >= 2) { ++p; --plen; }
        // fallthrough
      default:
        if (slen == 0 || *p != *s) return false;
        ++s; --slen;
        break;
    }
    ++p; --plen;
  }
  return slen == 0;
}

namespace {

std::string upper(std::string s) {
  for (auto& c : s) c = static_cast<char>(toupper(static_cast<unsigned char>(c)));
  return s;
}

bool parse_ll(const std::string& s, long long* out) {
  if (s.empty() || s.size() > 20) return false;
  char* end = nullptr;
  errno = 0;
  long long v = strtoll(s.c_str(), &end, 10);
  if (errno || *end != '\0') return false;
  *out = v;
  return true;
}

bool parse_double(const std::string& s, double* out) {
  if (s.empty()) return false;
  char* end = nullptr;
  double v = strtod(s.c_str(), &end);
  if (*end != '\0') return false;
  *out = v;
  return true;
}

struct Client {
  int fd = -1;
  std::string in;
  std::string out;
  int db = 0;
  bool in_multi = false;
  std::vector<Args> queued;
  bool multi_error = false;
  std::string name;
  bool closing = false;
  // blocking state
  bool blocked = false;
  Args blocked_cmd;
  std::vector<std::string> blocked_keys;
  int64_t deadline = 0;   // 0 = forever
  uint64_t id = 0;
};

const char* kWrongType =
    "WRONGTYPE Operation against a key holding the wrong kind of value";

class Server {
 public:
  Server(int dbs, SentinelConfig sentinel, std::string version = "7.2.0")
      : dbs_(dbs), sentinel_(std::move(sentinel)), started_(now_ms()),
        version_text_(std::move(version)) {
    int major = 0, minor = 0;
    sscanf(version_text_.c_str(), "%d.%d", &major, &minor);
    version_ = major * 100 + minor;
  }

  int run(const std::string& bind_addr, int port);

 private:
  using Handler = std::function<void(Client&, const Args&, Reply&)>;

  // keyspace
  Db& db(Client& c) { return dbs_[c.db]; }
  bool alive(Db& d, const std::string& key);
  Value* lookup(Db& d, const std::string& key, Value::Type type, bool* wrong);
  Value& create(Db& d, const std::string& key, Value::Type type);
  void drop_if_empty(Db& d, const std::string& key);
  bool remove(Db& d, const std::string& key);

  // dispatch
  void register_commands();
  void execute(Client& c, const Args& args, Reply& r, bool from_exec);
  bool try_pop_move(Client& c, const Args& args, Reply& r, bool blocking_ok);
  void serve_blocked(const std::string& key);
  void unblock_timeouts();
  void touched_list(const std::string& key) { touched_.push_back(key); }

  // networking
  void on_readable(Client& c);
  void process_input(Client& c);
  void flush(Client& c);
  void close_client(int fd);

  std::vector<Db> dbs_;
  SentinelConfig sentinel_;
  int64_t started_;
  // the Redis version this server answers as (--redis-version): below 6.2
  // LMOVE/BLMOVE are unknown, below 6.0 blocking timeouts are integers and
  // SCAN has no TYPE -- a server of the reference's redis~=3.5.3 era
  std::string version_text_;
  int version_ = 702;           // major * 100 + minor
  bool parse_timeout(const std::string& s, double* out) const {
    if (version_ >= 600) return parse_double(s, out);
    long long v;
    if (!parse_ll(s, &v)) return false;
    *out = static_cast<double>(v);
    return true;
  }
  const char* timeout_error() const {
    return version_ >= 600 ? "ERR timeout is not a float or out of range"
                           : "ERR timeout is not an integer or out of range";
  }
  long long commands_ = 0;
  std::unordered_map<std::string, Handler> table_;
  std::map<int, std::unique_ptr<Client>> clients_;
  std::list<int> blocked_order_;           // fds of parked clients, FIFO
  std::vector<std::string> touched_;
  int epfd_ = -1;
  uint64_t next_id_ = 1;
  bool shutdown_ = false;
};

bool Server::alive(Db& d, const std::string& key) {
  auto e = d.expires.find(key);
  if (e != d.expires.end() && now_ms() >= e->second) {
    d.expires.erase(e);
    d.keys.erase(key);
    ++d.version;
    return false;
  }
  return d.keys.count(key) > 0;
}

Value* Server::lookup(Db& d, const std::string& key, Value::Type type,
                      bool* wrong) {
  *wrong = false;
  if (!alive(d, key)) return nullptr;
  Value& v = d.keys[key];
  if (v.type != type) {
    *wrong = true;
    return nullptr;
  }
  return &v;
}

Value& Server::create(Db& d, const std::string& key, Value::Type type) {
  auto ins = d.keys.try_emplace(key);
  if (ins.second) ++d.version;
  Value& v = ins.first->second;
  v = Value();
  v.type = type;
  return v;
}

void Server::drop_if_empty(Db& d, const std::string& key) {
  auto it = d.keys.find(key);
  if (it == d.keys.end()) return;
  const Value& v = it->second;
  bool empty = (v.type == Value::LIST && v.list.empty()) ||
               (v.type == Value::HASH && v.hash.empty()) ||
               (v.type == Value::SET && v.set.empty());
  if (empty) {
    d.keys.erase(it);
    d.expires.erase(key);
    ++d.version;
  }
}

bool Server::remove(Db& d, const std::string& key) {
  d.expires.erase(key);
  if (d.keys.erase(key) == 0) return false;
  ++d.version;
  return true;
}

#define WRONG_OR(expr)         \
  do {                         \
    if (wrong) {               \
      r.error(kWrongType);     \
      return;                  \
    }                          \
    expr;                      \
  } while (0)

void Server::register_commands() {
  auto& t = table_;
  t["PING"] = [](Client&, const Args& a, Reply& r) {
    if (a.size() > 1) r.bulk(a[1]); else r.simple("PONG");
  };
  t["ECHO"] = [](Client&, const Args& a, Reply& r) { r.bulk(a.at(1)); };
  t["AUTH"] = [](Client&, const Args&, Reply& r) { r.simple("OK"); };
  t["QUIT"] = [](Client& c, const Args&, Reply& r) {
    r.simple("OK");
    c.closing = true;
  };
  t["SELECT"] = [this](Client& c, const Args& a, Reply& r) {
    long long i;
    if (!parse_ll(a.at(1), &i) || i < 0 || i >= (long long)dbs_.size()) {
      r.error("ERR DB index is out of range");
      return;
    }
    c.db = static_cast<int>(i);
    r.simple("OK");
  };
  t["DBSIZE"] = [this](Client& c, const Args&, Reply& r) {
    Db& d = db(c);
    long long n = 0;
    std::vector<std::string> keys;
    for (auto& kv : d.keys) keys.push_back(kv.first);
    for (auto& k : keys) n += alive(d, k);
    r.integer(n);
  };
  t["FLUSHDB"] = [this](Client& c, const Args&, Reply& r) {
    db(c).keys.clear();
    db(c).expires.clear();
    ++db(c).version;
    r.simple("OK");
  };
  t["FLUSHALL"] = [this](Client&, const Args&, Reply& r) {
    for (auto& d : dbs_) { d.keys.clear(); d.expires.clear(); ++d.version; }
    r.simple("OK");
  };
  t["TIME"] = [](Client&, const Args&, Reply& r) {
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    r.array(2);
    r.bulk(std::to_string(ts.tv_sec));
    r.bulk(std::to_string(ts.tv_nsec / 1000));
  };
  t["INFO"] = [this](Client&, const Args&, Reply& r) {
    std::string s = "# Server\r\nredis_version:" + version_text_ + "-kredis\r\n";
    s += std::string("redis_mode:") +
         (sentinel_.enabled() ? "sentinel" : "standalone") + "\r\n";
    s += "uptime_in_seconds:" + std::to_string((now_ms() - started_) / 1000) +
         "\r\n# Clients\r\nconnected_clients:" +
         std::to_string(clients_.size()) + "\r\nblocked_clients:" +
         std::to_string(blocked_order_.size()) + "\r\n# Replication\r\nrole:" +
         (sentinel_.enabled() ? "sentinel" : "master") +
         "\r\n# Stats\r\ntotal_commands_processed:" +
         std::to_string(commands_) + "\r\n# Keyspace\r\n";
    for (size_t i = 0; i < dbs_.size(); ++i) {
      if (!dbs_[i].keys.empty()) {
        s += "db" + std::to_string(i) + ":keys=" +
             std::to_string(dbs_[i].keys.size()) + ",expires=" +
             std::to_string(dbs_[i].expires.size()) + "\r\n";
      }
    }
    r.bulk(s);
  };
  t["CLIENT"] = [](Client& c, const Args& a, Reply& r) {
    std::string sub = upper(a.at(1));
    if (sub == "SETNAME") { c.name = a.at(2); r.simple("OK"); }
    else if (sub == "GETNAME") { if (c.name.empty()) r.null_bulk(); else r.bulk(c.name); }
    else if (sub == "ID") r.integer(static_cast<long long>(c.id));
    else r.simple("OK");
  };
  t["COMMAND"] = [](Client&, const Args&, Reply& r) { r.array(0); };
  t["CONFIG"] = [](Client&, const Args&, Reply& r) { r.array(0); };
  t["SHUTDOWN"] = [this](Client&, const Args&, Reply& r) {
    shutdown_ = true;
    r.simple("OK");
  };

  // ---- keys
  t["KEYS"] = [this](Client& c, const Args& a, Reply& r) {
    Db& d = db(c);
    std::vector<std::string> keys;
    for (auto& kv : d.keys) keys.push_back(kv.first);
    std::vector<std::string> out;
    for (auto& k : keys)
      if (alive(d, k) && glob_match(a.at(1).data(), a[1].size(), k.data(), k.size()))
        out.push_back(k);
    std::sort(out.begin(), out.end());
    r.array(out.size());
    for (auto& k : out) r.bulk(k);
  };
  t["EXISTS"] = [this](Client& c, const Args& a, Reply& r) {
    long long n = 0;
    for (size_t i = 1; i < a.size(); ++i) n += alive(db(c), a[i]);
    r.integer(n);
  };
  t["DEL"] = [this](Client& c, const Args& a, Reply& r) {
    long long n = 0;
    for (size_t i = 1; i < a.size(); ++i)
      if (alive(db(c), a[i])) n += remove(db(c), a[i]);
    r.integer(n);
  };
  t["UNLINK"] = t["DEL"];
  t["TYPE"] = [this](Client& c, const Args& a, Reply& r) {
    if (!alive(db(c), a.at(1))) { r.simple("none"); return; }
    static const char* names[] = {"string", "list", "hash", "set"};
    r.simple(names[db(c).keys[a[1]].type]);
  };
  auto set_deadline = [this](Client& c, const std::string& key, int64_t ms,
                             Reply& r) {
    if (!alive(db(c), key)) { r.integer(0); return; }
    db(c).expires[key] = now_ms() + ms;
    r.integer(1);
  };
  t["EXPIRE"] = [set_deadline](Client& c, const Args& a, Reply& r) {
    long long s;
    if (!parse_ll(a.at(2), &s)) { r.error("ERR value is not an integer or out of range"); return; }
    set_deadline(c, a[1], s * 1000, r);
  };
  t["PEXPIRE"] = [set_deadline](Client& c, const Args& a, Reply& r) {
    long long s;
    if (!parse_ll(a.at(2), &s)) { r.error("ERR value is not an integer or out of range"); return; }
    set_deadline(c, a[1], s, r);
  };
  t["PERSIST"] = [this](Client& c, const Args& a, Reply& r) {
    if (!alive(db(c), a.at(1))) { r.integer(0); return; }
    r.integer(db(c).expires.erase(a[1]) ? 1 : 0);
  };
  auto remaining = [this](Client& c, const std::string& key, int64_t scale,
                          Reply& r) {
    if (!alive(db(c), key)) { r.integer(-2); return; }
    auto e = db(c).expires.find(key);
    if (e == db(c).expires.end()) { r.integer(-1); return; }
    int64_t ms = std::max<int64_t>(0, e->second - now_ms());
    r.integer(scale == 1 ? ms : (ms + 500) / 1000);
  };
  t["TTL"] = [remaining](Client& c, const Args& a, Reply& r) { remaining(c, a.at(1), 1000, r); };
  t["PTTL"] = [remaining](Client& c, const Args& a, Reply& r) { remaining(c, a.at(1), 1, r); };
  t["RENAME"] = [this](Client& c, const Args& a, Reply& r) {
    Db& d = db(c);
    if (!alive(d, a.at(1))) { r.error("ERR no such key"); return; }
    Value v = std::move(d.keys[a[1]]);
    auto e = d.expires.find(a[1]);
    bool had = e != d.expires.end();
    int64_t deadline = had ? e->second : 0;
    remove(d, a[1]);
    remove(d, a.at(2));
    d.keys[a[2]] = std::move(v);
    ++d.version;
    if (had) d.expires[a[2]] = deadline;
    if (d.keys[a[2]].type == Value::LIST) touched_list(a[2]);
    r.simple("OK");
  };
  t["SCAN"] = [this](Client& c, const Args& a, Reply& r) {
    long long cursor;
    if (!parse_ll(a.at(1), &cursor) || cursor < 0) { r.error("ERR invalid cursor"); return; }
    std::string match, type;
    long long count = 10;
    for (size_t i = 2; i + 1 < a.size(); i += 2) {
      std::string opt = upper(a[i]);
      if (opt == "MATCH") match = a[i + 1];
      else if (opt == "COUNT") { if (!parse_ll(a[i + 1], &count) || count < 1) { r.error("ERR syntax error"); return; } }
      else if (opt == "TYPE" && version_ >= 600) type = a[i + 1];
      else { r.error("ERR syntax error"); return; }
    }
    Db& d = db(c);
    if (d.sorted_version != d.version) {
      d.sorted.clear();
      d.sorted.reserve(d.keys.size());
      for (auto& kv : d.keys) d.sorted.emplace_back(scan_hash(kv.first), kv.first);
      std::sort(d.sorted.begin(), d.sorted.end());
      d.sorted_version = d.version;
    }
    // alive() below may expire keys (bumping the version) but only SCAN
    // rebuilds `sorted`, so this reference stays valid for the call
    const auto& keys = d.sorted;
    static const char* names[] = {"string", "list", "hash", "set"};
    std::vector<std::string> out;
    size_t i = std::lower_bound(keys.begin(), keys.end(),
                                std::make_pair(static_cast<uint64_t>(cursor),
                                               std::string())) - keys.begin();
    size_t end = std::min(keys.size(), i + static_cast<size_t>(count));
    // never split keys of one hash value across pages: the next cursor is
    // a hash, so they would be returned twice
    while (end < keys.size() && end > i && keys[end].first == keys[end - 1].first) ++end;
    for (; i < end; ++i) {
      const std::string& k = keys[i].second;
      if (!alive(d, k)) continue;
      if (!match.empty() && !glob_match(match.data(), match.size(), k.data(), k.size())) continue;
      if (!type.empty() && type != names[d.keys[k].type]) continue;
      out.push_back(k);
    }
    r.array(2);
    r.bulk(end >= keys.size() ? "0" : std::to_string(keys[end].first));
    r.array(out.size());
    for (auto& k : out) r.bulk(k);
  };

  // ---- strings
  t["GET"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::STR, &wrong);
    WRONG_OR(if (v) r.bulk(v->str); else r.null_bulk());
  };
  t["SET"] = [this](Client& c, const Args& a, Reply& r) {
    const std::string& key = a.at(1);
    int64_t ttl = -1;
    bool nx = false, xx = false;
    for (size_t i = 3; i < a.size(); ++i) {
      std::string opt = upper(a[i]);
      long long n;
      if ((opt == "EX" || opt == "PX") && i + 1 < a.size() && parse_ll(a[i + 1], &n)) {
        ttl = opt == "EX" ? n * 1000 : n;
        ++i;
      } else if (opt == "NX") nx = true;
      else if (opt == "XX") xx = true;
      else { r.error("ERR syntax error"); return; }
    }
    bool exists = alive(db(c), key);
    if ((nx && exists) || (xx && !exists)) { r.null_bulk(); return; }
    remove(db(c), key);
    create(db(c), key, Value::STR).str = a.at(2);
    if (ttl >= 0) db(c).expires[key] = now_ms() + ttl;
    r.simple("OK");
  };
  t["SETNX"] = [this](Client& c, const Args& a, Reply& r) {
    if (alive(db(c), a.at(1))) { r.integer(0); return; }
    create(db(c), a[1], Value::STR).str = a.at(2);
    r.integer(1);
  };
  t["MGET"] = [this](Client& c, const Args& a, Reply& r) {
    r.array(a.size() - 1);
    for (size_t i = 1; i < a.size(); ++i) {
      bool wrong;
      Value* v = lookup(db(c), a[i], Value::STR, &wrong);
      if (v) r.bulk(v->str); else r.null_bulk();
    }
  };
  t["MSET"] = [this](Client& c, const Args& a, Reply& r) {
    if (a.size() < 3 || a.size() % 2 == 0) { r.error("ERR wrong number of arguments for 'mset' command"); return; }
    for (size_t i = 1; i + 1 < a.size(); i += 2) {
      remove(db(c), a[i]);
      create(db(c), a[i], Value::STR).str = a[i + 1];
    }
    r.simple("OK");
  };
  auto incr = [this](Client& c, const std::string& key, long long by, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), key, Value::STR, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    long long cur = 0;
    if (v && !parse_ll(v->str, &cur)) { r.error("ERR value is not an integer or out of range"); return; }
    if (!v) v = &create(db(c), key, Value::STR);
    cur += by;
    v->str = std::to_string(cur);
    r.integer(cur);
  };
  t["INCR"] = [incr](Client& c, const Args& a, Reply& r) { incr(c, a.at(1), 1, r); };
  t["DECR"] = [incr](Client& c, const Args& a, Reply& r) { incr(c, a.at(1), -1, r); };
  t["INCRBY"] = [incr](Client& c, const Args& a, Reply& r) {
    long long n;
    if (!parse_ll(a.at(2), &n)) { r.error("ERR value is not an integer or out of range"); return; }
    incr(c, a[1], n, r);
  };
  t["DECRBY"] = [incr](Client& c, const Args& a, Reply& r) {
    long long n;
    if (!parse_ll(a.at(2), &n)) { r.error("ERR value is not an integer or out of range"); return; }
    incr(c, a[1], -n, r);
  };

  // ---- lists
  auto push = [this](Client& c, const Args& a, Reply& r, bool left) {
    if (a.size() < 3) { r.error("ERR wrong number of arguments"); return; }
    bool wrong;
    Value* v = lookup(db(c), a[1], Value::LIST, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    if (!v) v = &create(db(c), a[1], Value::LIST);
    for (size_t i = 2; i < a.size(); ++i) {
      if (left) v->list.push_front(a[i]); else v->list.push_back(a[i]);
    }
    r.integer(static_cast<long long>(v->list.size()));
    touched_list(a[1]);
  };
  t["LPUSH"] = [push](Client& c, const Args& a, Reply& r) { push(c, a, r, true); };
  t["RPUSH"] = [push](Client& c, const Args& a, Reply& r) { push(c, a, r, false); };
  auto pop = [this](Client& c, const Args& a, Reply& r, bool left) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::LIST, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    if (a.size() > 2) {
      long long n;
      if (!parse_ll(a[2], &n) || n < 0) { r.error("ERR value is out of range, must be positive"); return; }
      if (!v) { r.null_array(); return; }
      std::vector<std::string> out;
      while (n-- > 0 && !v->list.empty()) {
        if (left) { out.push_back(v->list.front()); v->list.pop_front(); }
        else { out.push_back(v->list.back()); v->list.pop_back(); }
      }
      drop_if_empty(db(c), a[1]);
      r.array(out.size());
      for (auto& s : out) r.bulk(s);
      return;
    }
    if (!v || v->list.empty()) { r.null_bulk(); return; }
    std::string s;
    if (left) { s = v->list.front(); v->list.pop_front(); }
    else { s = v->list.back(); v->list.pop_back(); }
    drop_if_empty(db(c), a[1]);
    r.bulk(s);
  };
  t["LPOP"] = [pop](Client& c, const Args& a, Reply& r) { pop(c, a, r, true); };
  t["RPOP"] = [pop](Client& c, const Args& a, Reply& r) { pop(c, a, r, false); };
  t["LLEN"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::LIST, &wrong);
    WRONG_OR(r.integer(v ? static_cast<long long>(v->list.size()) : 0));
  };
  t["LRANGE"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::LIST, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    long long start, stop;
    if (!parse_ll(a.at(2), &start) || !parse_ll(a.at(3), &stop)) { r.error("ERR value is not an integer or out of range"); return; }
    long long n = v ? static_cast<long long>(v->list.size()) : 0;
    if (start < 0) start = std::max(0LL, n + start);
    if (stop < 0) stop = n + stop;
    stop = std::min(stop, n - 1);
    if (start > stop) { r.array(0); return; }
    r.array(static_cast<size_t>(stop - start + 1));
    for (long long i = start; i <= stop; ++i) r.bulk(v->list[static_cast<size_t>(i)]);
  };
  t["LINDEX"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::LIST, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    long long i;
    if (!parse_ll(a.at(2), &i)) { r.error("ERR value is not an integer or out of range"); return; }
    long long n = v ? static_cast<long long>(v->list.size()) : 0;
    if (i < 0) i += n;
    if (i < 0 || i >= n) { r.null_bulk(); return; }
    r.bulk(v->list[static_cast<size_t>(i)]);
  };
  t["LSET"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::LIST, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    if (!v) { r.error("ERR no such key"); return; }
    long long i;
    if (!parse_ll(a.at(2), &i)) { r.error("ERR value is not an integer or out of range"); return; }
    long long n = static_cast<long long>(v->list.size());
    if (i < 0) i += n;
    if (i < 0 || i >= n) { r.error("ERR index out of range"); return; }
    v->list[static_cast<size_t>(i)] = a.at(3);
    r.simple("OK");
  };
  t["LREM"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::LIST, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    long long count;
    if (!parse_ll(a.at(2), &count)) { r.error("ERR value is not an integer or out of range"); return; }
    if (!v) { r.integer(0); return; }
    const std::string& val = a.at(3);
    long long removed = 0;
    if (count >= 0) {
      for (auto it = v->list.begin(); it != v->list.end() && (count == 0 || removed < count);) {
        if (*it == val) { it = v->list.erase(it); ++removed; } else ++it;
      }
    } else {
      for (size_t i = v->list.size(); i-- > 0 && removed < -count;) {
        if (v->list[i] == val) { v->list.erase(v->list.begin() + i); ++removed; }
      }
    }
    drop_if_empty(db(c), a[1]);
    r.integer(removed);
  };
  t["LTRIM"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::LIST, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    long long start, stop;
    if (!parse_ll(a.at(2), &start) || !parse_ll(a.at(3), &stop)) { r.error("ERR value is not an integer or out of range"); return; }
    if (v) {
      long long n = static_cast<long long>(v->list.size());
      if (start < 0) start = std::max(0LL, n + start);
      if (stop < 0) stop = n + stop;
      stop = std::min(stop, n - 1);
      std::deque<std::string> kept;
      for (long long i = start; i <= stop; ++i) kept.push_back(v->list[static_cast<size_t>(i)]);
      v->list.swap(kept);
      drop_if_empty(db(c), a[1]);
    }
    r.simple("OK");
  };
  // LMOVE / RPOPLPUSH / blocking variants share try_pop_move.
  auto moves = [this](Client& c, const Args& a, Reply& r) { try_pop_move(c, a, r, true); };
  for (const char* name : {"LMOVE", "RPOPLPUSH", "BLMOVE", "BRPOPLPUSH", "BLPOP", "BRPOP"})
    t[name] = moves;
  if (version_ < 602) {          // LMOVE / BLMOVE arrived in Redis 6.2
    t.erase("LMOVE");
    t.erase("BLMOVE");
  }

  // ---- hashes
  t["HSET"] = [this](Client& c, const Args& a, Reply& r) {
    if (a.size() < 4 || a.size() % 2 != 0) { r.error("ERR wrong number of arguments for 'hset' command"); return; }
    bool wrong;
    Value* v = lookup(db(c), a[1], Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    if (!v) v = &create(db(c), a[1], Value::HASH);
    long long added = 0;
    for (size_t i = 2; i + 1 < a.size(); i += 2) {
      added += v->hash.count(a[i]) == 0;
      v->hash[a[i]] = a[i + 1];
    }
    r.integer(added);
  };
  t["HMSET"] = [this](Client& c, const Args& a, Reply& r) {
    Reply tmp;
    table_["HSET"](c, a, tmp);
    if (!tmp.data().empty() && tmp.data()[0] == '-') r.data() += tmp.data();
    else r.simple("OK");
  };
  t["HSETNX"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    if (!v) v = &create(db(c), a[1], Value::HASH);
    if (v->hash.count(a.at(2))) { r.integer(0); return; }
    v->hash[a[2]] = a.at(3);
    r.integer(1);
  };
  t["HGET"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    if (!v) { r.null_bulk(); return; }
    auto it = v->hash.find(a.at(2));
    if (it == v->hash.end()) r.null_bulk(); else r.bulk(it->second);
  };
  t["HMGET"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    r.array(a.size() - 2);
    for (size_t i = 2; i < a.size(); ++i) {
      if (!v) { r.null_bulk(); continue; }
      auto it = v->hash.find(a[i]);
      if (it == v->hash.end()) r.null_bulk(); else r.bulk(it->second);
    }
  };
  t["HGETALL"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    if (!v) { r.array(0); return; }
    r.array(v->hash.size() * 2);
    for (auto& kv : v->hash) { r.bulk(kv.first); r.bulk(kv.second); }
  };
  t["HDEL"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    long long n = 0;
    if (v) for (size_t i = 2; i < a.size(); ++i) n += v->hash.erase(a[i]);
    drop_if_empty(db(c), a[1]);
    r.integer(n);
  };
  t["HLEN"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    WRONG_OR(r.integer(v ? static_cast<long long>(v->hash.size()) : 0));
  };
  t["HEXISTS"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    WRONG_OR(r.integer(v && v->hash.count(a.at(2)) ? 1 : 0));
  };
  t["HINCRBY"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    long long by, cur = 0;
    if (!parse_ll(a.at(3), &by)) { r.error("ERR value is not an integer or out of range"); return; }
    if (!v) v = &create(db(c), a[1], Value::HASH);
    auto it = v->hash.find(a[2]);
    if (it != v->hash.end() && !parse_ll(it->second, &cur)) { r.error("ERR hash value is not an integer"); return; }
    cur += by;
    v->hash[a[2]] = std::to_string(cur);
    r.integer(cur);
  };
  t["HKEYS"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    r.array(v ? v->hash.size() : 0);
    if (v) for (auto& kv : v->hash) r.bulk(kv.first);
  };
  t["HVALS"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::HASH, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    r.array(v ? v->hash.size() : 0);
    if (v) for (auto& kv : v->hash) r.bulk(kv.second);
  };

  // ---- sets
  t["SADD"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::SET, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    if (!v) v = &create(db(c), a[1], Value::SET);
    long long n = 0;
    for (size_t i = 2; i < a.size(); ++i) n += v->set.insert(a[i]).second;
    r.integer(n);
  };
  t["SREM"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::SET, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    long long n = 0;
    if (v) for (size_t i = 2; i < a.size(); ++i) n += v->set.erase(a[i]);
    drop_if_empty(db(c), a[1]);
    r.integer(n);
  };
  t["SMEMBERS"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::SET, &wrong);
    if (wrong) { r.error(kWrongType); return; }
    std::vector<std::string> out;
    if (v) out.assign(v->set.begin(), v->set.end());
    std::sort(out.begin(), out.end());
    r.array(out.size());
    for (auto& s : out) r.bulk(s);
  };
  t["SCARD"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::SET, &wrong);
    WRONG_OR(r.integer(v ? static_cast<long long>(v->set.size()) : 0));
  };
  t["SISMEMBER"] = [this](Client& c, const Args& a, Reply& r) {
    bool wrong;
    Value* v = lookup(db(c), a.at(1), Value::SET, &wrong);
    WRONG_OR(r.integer(v && v->set.count(a.at(2)) ? 1 : 0));
  };

  // ---- pub/sub + scripting stubs
  t["PUBLISH"] = [](Client&, const Args&, Reply& r) { r.integer(0); };
  t["EVAL"] = [](Client&, const Args&, Reply& r) {
    r.error("ERR scripting is not supported by kredis");
  };
  t["EVALSHA"] = t["EVAL"];
  t["SCRIPT"] = [](Client&, const Args& a, Reply& r) {
    if (a.size() > 1 && upper(a[1]) == "KILL")
      r.error("NOTBUSY No scripts in execution right now.");
    else
      r.error("ERR scripting is not supported by kredis");
  };

  // ---- sentinel personality
  t["SENTINEL"] = [this](Client&, const Args& a, Reply& r) {
    if (!sentinel_.enabled()) {
      r.error("ERR unknown command 'sentinel', with args beginning with: ");
      return;
    }
    std::string sub = upper(a.at(1));
    auto state = [&r](const std::string& name, const std::string& ip, int port,
                      const char* flags) {
      r.array(10);
      r.bulk("name"); r.bulk(name);
      r.bulk("ip"); r.bulk(ip);
      r.bulk("port"); r.bulk(std::to_string(port));
      r.bulk("flags"); r.bulk(flags);
      r.bulk("role-reported"); r.bulk(std::string(flags) == "master" ? "master" : "slave");
    };
    if (sub == "MASTERS") {
      r.array(1);
      state(sentinel_.name, sentinel_.host, sentinel_.port, "master");
    } else if (sub == "SLAVES" || sub == "REPLICAS") {
      if (a.at(2) != sentinel_.name) { r.error("ERR No such master with that name"); return; }
      r.array(sentinel_.replicas.size());
      for (auto& rep : sentinel_.replicas)
        state(rep.first + ":" + std::to_string(rep.second), rep.first, rep.second, "slave");
    } else if (sub == "GET-MASTER-ADDR-BY-NAME") {
      if (a.at(2) != sentinel_.name) { r.null_bulk(); return; }
      r.array(2);
      r.bulk(sentinel_.host);
      r.bulk(std::to_string(sentinel_.port));
    } else {
      r.error("ERR Unknown sentinel subcommand");
    }
  };
}

// Pops/moves for LMOVE, RPOPLPUSH, BLMOVE, BRPOPLPUSH, BLPOP, BRPOP.
// Returns true when a reply was produced (false = the client is parked).
bool Server::try_pop_move(Client& c, const Args& a, Reply& r, bool blocking_ok) {
  const std::string cmd = upper(a.at(0));
  Db& d = db(c);
  bool is_move = cmd == "LMOVE" || cmd == "RPOPLPUSH" || cmd == "BLMOVE" ||
                 cmd == "BRPOPLPUSH";
  bool blocking = cmd[0] == 'B';
  double timeout = 0;
  std::vector<std::string> srcs;
  std::string dst;
  bool from_left = false, to_left = true;
  if (is_move) {
    srcs.push_back(a.at(1));
    dst = a.at(2);
    if (cmd == "LMOVE" || cmd == "BLMOVE") {
      std::string wf = upper(a.at(3)), wt = upper(a.at(4));
      if ((wf != "LEFT" && wf != "RIGHT") || (wt != "LEFT" && wt != "RIGHT")) {
        r.error("ERR syntax error");
        return true;
      }
      from_left = wf == "LEFT";
      to_left = wt == "LEFT";
      if (cmd == "BLMOVE" && !parse_timeout(a.at(5), &timeout)) {
        r.error(timeout_error());
        return true;
      }
    } else {
      from_left = false;
      to_left = true;
      if (cmd == "BRPOPLPUSH" && !parse_timeout(a.at(3), &timeout)) {
        r.error(timeout_error());
        return true;
      }
    }
  } else {
    if (a.size() < 3) { r.error("ERR wrong number of arguments"); return true; }
    for (size_t i = 1; i + 1 < a.size(); ++i) srcs.push_back(a[i]);
    if (!parse_timeout(a.back(), &timeout)) {
      r.error(timeout_error());
      return true;
    }
    from_left = cmd == "BLPOP";
  }
  if (timeout < 0) { r.error("ERR timeout is negative"); return true; }
  for (const auto& src : srcs) {
    bool wrong;
    Value* v = lookup(d, src, Value::LIST, &wrong);
    if (wrong) { r.error(kWrongType); return true; }
    if (!v || v->list.empty()) continue;
    if (is_move) {
      bool wrong_dst;
      Value* t = lookup(d, dst, Value::LIST, &wrong_dst);
      if (wrong_dst) { r.error(kWrongType); return true; }
      std::string item;
      if (from_left) { item = v->list.front(); v->list.pop_front(); }
      else { item = v->list.back(); v->list.pop_back(); }
      drop_if_empty(d, src);
      if (!t) t = &create(d, dst, Value::LIST);
      if (to_left) t->list.push_front(item); else t->list.push_back(item);
      touched_list(dst);
      r.bulk(item);
    } else {
      std::string item;
      if (from_left) { item = v->list.front(); v->list.pop_front(); }
      else { item = v->list.back(); v->list.pop_back(); }
      drop_if_empty(d, src);
      r.array(2);
      r.bulk(src);
      r.bulk(item);
    }
    return true;
  }
  if (!blocking || !blocking_ok || c.in_multi) {
    if (blocking && !is_move) r.null_array(); else r.null_bulk();
    return true;
  }
  c.blocked = true;
  c.blocked_cmd = a;
  c.blocked_keys = srcs;
  c.deadline = timeout > 0 ? now_ms() + static_cast<int64_t>(timeout * 1000) : 0;
  blocked_order_.push_back(c.fd);
  return false;
}

void Server::serve_blocked(const std::string& key) {
  (void)key;
  bool progress = true;
  while (progress) {
    progress = false;
    for (auto it = blocked_order_.begin(); it != blocked_order_.end();) {
      auto cit = clients_.find(*it);
      if (cit == clients_.end()) { it = blocked_order_.erase(it); continue; }
      Client& c = *cit->second;
      bool ready = false;
      for (auto& k : c.blocked_keys) {
        bool wrong;
        Value* v = lookup(dbs_[c.db], k, Value::LIST, &wrong);
        if (wrong || (v && !v->list.empty())) { ready = true; break; }
      }
      if (!ready) { ++it; continue; }
      Reply r;
      c.blocked = false;
      it = blocked_order_.erase(it);
      try_pop_move(c, c.blocked_cmd, r, false);
      c.out += r.data();
      flush(c);
      progress = true;
      break;   // the keyspace changed: rescan from the oldest waiter
    }
  }
}

void Server::unblock_timeouts() {
  const int64_t now = now_ms();
  for (auto it = blocked_order_.begin(); it != blocked_order_.end();) {
    auto cit = clients_.find(*it);
    if (cit == clients_.end()) { it = blocked_order_.erase(it); continue; }
    Client& c = *cit->second;
    if (c.deadline && now >= c.deadline) {
      const std::string cmd = upper(c.blocked_cmd[0]);
      c.blocked = false;
      c.out += (cmd == "BLPOP" || cmd == "BRPOP") ? "*-1\r\n" : "$-1\r\n";
      it = blocked_order_.erase(it);
      flush(c);
      process_input(c);   // pipelined commands queued behind the block
    } else {
      ++it;
    }
  }
}

void Server::execute(Client& c, const Args& args, Reply& r, bool from_exec) {
  ++commands_;
  const std::string cmd = upper(args[0]);
  if (c.in_multi && !from_exec && cmd != "EXEC" && cmd != "DISCARD" &&
      cmd != "MULTI" && cmd != "WATCH") {
    if (!table_.count(cmd)) {
      c.multi_error = true;
      r.error("ERR unknown command '" + args[0] + "'");
      return;
    }
    c.queued.push_back(args);
    r.simple("QUEUED");
    return;
  }
  if (cmd == "MULTI") {
    if (c.in_multi) { r.error("ERR MULTI calls can not be nested"); return; }
    c.in_multi = true;
    c.queued.clear();
    c.multi_error = false;
    r.simple("OK");
    return;
  }
  if (cmd == "DISCARD") {
    if (!c.in_multi) { r.error("ERR DISCARD without MULTI"); return; }
    c.in_multi = false;
    c.queued.clear();
    r.simple("OK");
    return;
  }
  if (cmd == "EXEC") {
    if (!c.in_multi) { r.error("ERR EXEC without MULTI"); return; }
    auto queued = std::move(c.queued);
    c.queued.clear();
    if (c.multi_error) {
      c.in_multi = false;
      r.error("EXECABORT Transaction discarded because of previous errors.");
      return;
    }
    r.array(queued.size());
    for (auto& q : queued) execute(c, q, r, true);
    c.in_multi = false;
    return;
  }
  if (cmd == "WATCH" || cmd == "UNWATCH") { r.simple("OK"); return; }
  auto it = table_.find(cmd);
  if (it == table_.end()) {
    r.error("ERR unknown command '" + args[0] + "', with args beginning with: ");
    return;
  }
  try {
    it->second(c, args, r);
  } catch (const std::out_of_range&) {
    r.error("ERR wrong number of arguments for '" + args[0] + "' command");
  }
}

void Server::flush(Client& c) {
  while (!c.out.empty()) {
    ssize_t n = send(c.fd, c.out.data(), c.out.size(), MSG_NOSIGNAL);
    if (n > 0) {
      c.out.erase(0, static_cast<size_t>(n));
    } else if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT;
      ev.data.fd = c.fd;
      epoll_ctl(epfd_, EPOLL_CTL_MOD, c.fd, &ev);
      return;
    } else {
      c.closing = true;
      return;
    }
  }
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = c.fd;
  epoll_ctl(epfd_, EPOLL_CTL_MOD, c.fd, &ev);
}

// Parse as many complete commands as the input holds and run them.
void Server::process_input(Client& c) {
  while (!c.blocked && !c.closing && !c.in.empty()) {
    Args args;
    size_t pos = 0;
    if (c.in[0] == '*') {
      size_t eol = c.in.find("\r\n");
      if (eol == std::string::npos) return;
      long long n;
      if (!parse_ll(c.in.substr(1, eol - 1), &n) || n < 0 || n > 1024 * 1024) {
        c.out += "-ERR Protocol error: invalid multibulk length\r\n";
        c.closing = true;
        return;
      }
      pos = eol + 2;
      bool complete = true;
      for (long long i = 0; i < n; ++i) {
        if (pos >= c.in.size()) { complete = false; break; }
        if (c.in[pos] != '$') {
          c.out += "-ERR Protocol error: expected '$'\r\n";
          c.closing = true;
          return;
        }
        size_t e = c.in.find("\r\n", pos);
        if (e == std::string::npos) { complete = false; break; }
        long long len;
        if (!parse_ll(c.in.substr(pos + 1, e - pos - 1), &len) || len < 0 ||
            len > 512LL * 1024 * 1024) {
          c.out += "-ERR Protocol error: invalid bulk length\r\n";
          c.closing = true;
          return;
        }
        if (c.in.size() < e + 2 + static_cast<size_t>(len) + 2) { complete = false; break; }
        args.push_back(c.in.substr(e + 2, static_cast<size_t>(len)));
        pos = e + 2 + static_cast<size_t>(len) + 2;
      }
      if (!complete) return;
    } else {
      size_t eol = c.in.find('\n');
      if (eol == std::string::npos) return;
      std::string line = c.in.substr(0, eol);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      pos = eol + 1;
      size_t i = 0;
      while (i < line.size()) {
        while (i < line.size() && line[i] == ' ') ++i;
        size_t j = i;
        while (j < line.size() && line[j] != ' ') ++j;
        if (j > i) args.push_back(line.substr(i, j - i));
        i = j;
      }
    }
    c.in.erase(0, pos);
    if (args.empty()) continue;
    Reply r;
    touched_.clear();
    execute(c, args, r, false);
    c.out += r.data();
    if (!touched_.empty()) {
      auto keys = touched_;
      touched_.clear();
      for (auto& k : keys) serve_blocked(k);
    }
  }
  flush(c);
}

void Server::on_readable(Client& c) {
  char buf[65536];
  while (true) {
    ssize_t n = recv(c.fd, buf, sizeof(buf), 0);
    if (n > 0) {
      c.in.append(buf, static_cast<size_t>(n));
      if (static_cast<size_t>(n) < sizeof(buf)) break;
    } else if (n == 0) {
      c.closing = true;
      return;
    } else {
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      c.closing = true;
      return;
    }
  }
  process_input(c);
}

void Server::close_client(int fd) {
  epoll_ctl(epfd_, EPOLL_CTL_DEL, fd, nullptr);
  close(fd);
  blocked_order_.remove(fd);
  clients_.erase(fd);
}

int Server::run(const std::string& bind_addr, int port) {
  register_commands();
  int lfd = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, bind_addr.c_str(), &addr.sin_addr) != 1) {
    fprintf(stderr, "bad bind address %s\n", bind_addr.c_str());
    return 2;
  }
  if (bind(lfd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 ||
      listen(lfd, 512) != 0) {
    perror("bind/listen");
    return 2;
  }
  socklen_t alen = sizeof(addr);
  getsockname(lfd, reinterpret_cast<sockaddr*>(&addr), &alen);
  fcntl(lfd, F_SETFL, fcntl(lfd, F_GETFL) | O_NONBLOCK);
  epfd_ = epoll_create1(0);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd;
  epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd, &ev);
  printf("kredis-server listening on %s:%d\n", bind_addr.c_str(),
         ntohs(addr.sin_port));
  fflush(stdout);
  std::vector<epoll_event> events(256);
  while (!shutdown_ && !g_terminate) {
    // sleep until the nearest blocked client's deadline (1 ms resolution),
    // so a BLMOVE with a 5 ms bound returns after 5 ms, not the next 10 ms
    int timeout = 1000;
    if (!blocked_order_.empty()) {
      const int64_t now = now_ms();
      for (int bfd : blocked_order_) {
        auto bit = clients_.find(bfd);
        if (bit == clients_.end() || !bit->second->deadline) continue;
        const int64_t left = bit->second->deadline - now;
        timeout = static_cast<int>(std::max<int64_t>(
            0, std::min<int64_t>(timeout, left)));
      }
    }
    int n = epoll_wait(epfd_, events.data(), static_cast<int>(events.size()),
                       timeout);
    if (n < 0 && errno != EINTR) break;
    for (int i = 0; i < n; ++i) {
      int fd = events[i].data.fd;
      if (fd == lfd) {
        while (true) {
          int cfd = accept(lfd, nullptr, nullptr);
          if (cfd < 0) break;
          fcntl(cfd, F_SETFL, fcntl(cfd, F_GETFL) | O_NONBLOCK);
          setsockopt(cfd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          auto cl = std::make_unique<Client>();
          cl->fd = cfd;
          cl->id = next_id_++;
          epoll_event cev{};
          cev.events = EPOLLIN;
          cev.data.fd = cfd;
          epoll_ctl(epfd_, EPOLL_CTL_ADD, cfd, &cev);
          clients_[cfd] = std::move(cl);
        }
        continue;
      }
      auto it = clients_.find(fd);
      if (it == clients_.end()) continue;
      Client& c = *it->second;
      if (events[i].events & (EPOLLERR | EPOLLHUP)) c.closing = true;
      if (!c.closing && (events[i].events & EPOLLIN)) on_readable(c);
      if (!c.closing && (events[i].events & EPOLLOUT)) flush(c);
      if (c.closing && c.out.empty()) close_client(fd);
      else if (c.closing) { flush(c); close_client(fd); }
    }
    if (!blocked_order_.empty()) unblock_timeouts();
  }
  close(lfd);
  return 0;
}

}  // namespace

}  // namespace kredis

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  signal(SIGTERM, [](int) { kredis::g_terminate = 1; });
  signal(SIGINT, [](int) { kredis::g_terminate = 1; });
  std::string bind_addr = "127.0.0.1";
  int port = 6379;
  kredis::SentinelConfig sentinel;
  std::string version = "7.2.0";
  for (int i = 1; i < argc; ++i) {
    std::string arg = argv[i];
    if (arg == "--port" && i + 1 < argc) port = atoi(argv[++i]);
    else if (arg == "--bind" && i + 1 < argc) bind_addr = argv[++i];
    else if (arg == "--redis-version" && i + 1 < argc) version = argv[++i];
    else if (arg == "--sentinel" && i + 3 < argc) {
      sentinel.name = argv[++i];
      sentinel.host = argv[++i];
      sentinel.port = atoi(argv[++i]);
    } else if (arg == "--replica" && i + 1 < argc) {
      std::string hp = argv[++i];
      size_t colon = hp.rfind(':');
      if (colon == std::string::npos) { fprintf(stderr, "--replica HOST:PORT\n"); return 2; }
      sentinel.replicas.emplace_back(hp.substr(0, colon), atoi(hp.c_str() + colon + 1));
    } else if (arg == "--help" || arg == "-h") {
      printf("kredis-server [--bind ADDR] [--port N] [--sentinel NAME HOST PORT] "
             "[--replica HOST:PORT]... [--redis-version X.Y]\n");
      return 0;
    } else {
      fprintf(stderr, "unknown argument %s\n", arg.c_str());
      return 2;
    }
  }
  kredis::Server server(16, sentinel, version);
  return server.run(bind_addr, port);
}
