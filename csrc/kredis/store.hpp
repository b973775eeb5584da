// kredis: a single-threaded, epoll-driven RESP2 server holding the subset
// of Redis the autoscaler stack uses (strings, lists, hashes, sets, TTLs,
// SCAN/KEYS globbing, MULTI/EXEC, blocking list moves, a SENTINEL
// personality).  There is no redis-server on the GPU boxes and no network
// to fetch one; this binary is the work bus for benchmarks and multi-process
// integration runs.
#pragma once

#include <stdint.h>

#include <deque>
#include <map>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace kredis {

using Args = std::vector<std::string>;

struct Value {
  enum Type { STR, LIST, HASH, SET } type = STR;
  std::string str;
  std::deque<std::string> list;
  std::unordered_map<std::string, std::string> hash;
  std::unordered_set<std::string> set;
};

struct Db {
  std::unordered_map<std::string, Value> keys;
  std::unordered_map<std::string, int64_t> expires;   // monotonic ms
  // SCAN walks the keys in (hash, key) order and its cursor is a position
  // in *hash space*, not an index: deleting or adding keys between pages
  // cannot shift a key that was present all along past the cursor (Redis's
  // guarantee).  The ordered copy is rebuilt only when the key set changed
  // (version bumps on every insert / removal).
  uint64_t version = 0;
  uint64_t sorted_version = ~0ull;
  std::vector<std::pair<uint64_t, std::string>> sorted;
};

// RESP reply builder.
class Reply {
 public:
  void simple(const std::string& s) { out_ += "+" + s + "\r\n"; }
  void error(const std::string& s) { out_ += "-" + s + "\r\n"; }
  void integer(long long v) { out_ += ":" + std::to_string(v) + "\r\n"; }
  void bulk(const std::string& s) {
    out_ += "$" + std::to_string(s.size()) + "\r\n";
    out_ += s;
    out_ += "\r\n";
  }
  void null_bulk() { out_ += "$-1\r\n"; }
  void null_array() { out_ += "*-1\r\n"; }
  void array(size_t n) { out_ += "*" + std::to_string(n) + "\r\n"; }
  std::string& data() { return out_; }
  bool empty() const { return out_.empty(); }
  void clear() { out_.clear(); }

 private:
  std::string out_;
};

bool glob_match(const char* pat, size_t plen, const char* str, size_t slen);

// SCAN position of a key: 64-bit FNV-1a folded into [1, 2^63) (cursor 0
// is reserved for "start" / "done").
inline uint64_t scan_hash(const std::string& key) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char ch : key) {
    h ^= ch;
    h *= 1099511628211ull;
  }
  return (h >> 1) | 1ull;
}

int64_t now_ms();

struct SentinelConfig {
  std::string name;
  std::string host;
  int port = 0;
  std::vector<std::pair<std::string, int>> replicas;
  bool enabled() const { return !name.empty(); }
};

}  // namespace kredis
