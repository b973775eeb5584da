// kiosk-rccl-slim: a one-ISA, uncompressed, debug-stripped copy of RCCL's
// device code, so that a fresh worker process stops paying for the other
// twelve GPU targets on every node-communicator generation.
//
// Why (profiles/r5_fence_lag): ROCm 7.2's librccl.so
// carries one compressed offload bundle (CCOB v3, zstd) of 571 MB that
// inflates to 5.29 GB: thirteen code objects, gfx950 the LAST of them
// (4.72 GB into the stream), each with ~460 MB of DWARF.  The HIP runtime
// digests a fat binary lazily, at the first use of one of its kernels, i.e.
// inside the first ncclCommInitRank of every process: it inflates the whole
// stream to find gfx950, then loads a 569 MB ELF.  A worker forked from the
// zygote (which registered RCCL before any HIP call) therefore paid ~1.1 s
// of zstd plus the code-object load in every generation, 1.75 s in all,
// while the fenced set lagged READY.
//
// What this writes: a copy of the library whose `.hip_fatbin` section holds
// an *uncompressed* bundle with the host entry and the one gfx950 code
// object, stripped of its .debug_* sections (569 MB -> 108 MB; the loadable
// segments are byte-identical).  The section keeps its offset and size (the
// ELF layout, relocations and the __hip_fatbin_wrapper pointer are
// untouched); the unused tail is a file hole.  The HIP runtime then finds
// the code object in place, without inflating anything.
//
// usage: kiosk-rccl-slim --src LIB --out PATH [--isa gfx950] [--no-strip]
// Prints one JSON line (sizes, timings) on success; exit 2 on any failure
// (the caller keeps the stock library).
#include <dlfcn.h>
#include <elf.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

constexpr char kBundleMagic[] = "__CLANG_OFFLOAD_BUNDLE__";   // 24 bytes
constexpr size_t kBundleMagicLen = 24;
constexpr char kCompressedMagic[] = "CCOB";
constexpr size_t kCodeObjectAlign = 4096;

struct Entry {
  uint64_t offset = 0;
  uint64_t size = 0;
  std::string id;
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

template <typename T>
T load(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

// ---------------------------------------------------------------------------
// bundle header: magic, u64 count, count x {u64 offset, u64 size, u64 idlen,
// id}.  Returns false while `n` bytes are not enough to hold all of it.
bool parse_bundle_header(const uint8_t* p, size_t n, std::vector<Entry>* out,
                         size_t* header_len) {
  if (n < kBundleMagicLen + 8) return false;
  if (std::memcmp(p, kBundleMagic, kBundleMagicLen) != 0) {
    throw std::runtime_error("not a clang offload bundle");
  }
  const uint64_t count = load<uint64_t>(p + kBundleMagicLen);
  if (count == 0 || count > 4096) throw std::runtime_error("bad entry count");
  size_t pos = kBundleMagicLen + 8;
  std::vector<Entry> entries;
  for (uint64_t i = 0; i < count; ++i) {
    if (pos + 24 > n) return false;
    Entry e;
    e.offset = load<uint64_t>(p + pos);
    e.size = load<uint64_t>(p + pos + 8);
    const uint64_t idlen = load<uint64_t>(p + pos + 16);
    if (idlen > 4096) throw std::runtime_error("bad entry id length");
    pos += 24;
    if (pos + idlen > n) return false;
    e.id.assign(reinterpret_cast<const char*>(p + pos), idlen);
    pos += idlen;
    entries.push_back(e);
  }
  *out = entries;
  *header_len = pos;
  return true;
}

// "hipv4-amdgcn-amd-amdhsa--gfx950[:feature...]": the processor and its
// target features.
bool entry_matches(const std::string& id, const std::string& isa, int* rank) {
  const std::string tag = "amdgcn-amd-amdhsa--";
  const size_t at = id.find(tag);
  if (at == std::string::npos) return false;
  const std::string target = id.substr(at + tag.size());
  const std::string proc = target.substr(0, target.find(':'));
  if (proc != isa) return false;
  if (target.find("xnack+") != std::string::npos) return false;   // XNACK off
  *rank = target == isa ? 0 : 1;   // a generic entry before a feature one
  return true;
}

const Entry* pick(const std::vector<Entry>& entries, const std::string& isa) {
  const Entry* best = nullptr;
  int best_rank = 99;
  for (const auto& e : entries) {
    int rank = 0;
    if (entry_matches(e.id, isa, &rank) && rank < best_rank) {
      best = &e;
      best_rank = rank;
    }
  }
  if (!best) throw std::runtime_error("no " + isa + " entry in the bundle");
  return best;
}

// ---------------------------------------------------------------------------
// zstd through dlopen (the image ships libzstd.so.1 but no header)
struct ZBuf {
  void* ptr;
  size_t size;
  size_t pos;
};

struct Zstd {
  void* handle = nullptr;
  void* (*create)() = nullptr;
  size_t (*init)(void*) = nullptr;
  size_t (*stream)(void*, ZBuf*, ZBuf*) = nullptr;
  size_t (*free_)(void*) = nullptr;
  unsigned (*is_error)(size_t) = nullptr;
  const char* (*error_name)(size_t) = nullptr;

  Zstd() {
    handle = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!handle) throw std::runtime_error("libzstd.so.1 not found");
    create = reinterpret_cast<void* (*)()>(dlsym(handle, "ZSTD_createDStream"));
    init = reinterpret_cast<size_t (*)(void*)>(dlsym(handle, "ZSTD_initDStream"));
    stream = reinterpret_cast<size_t (*)(void*, ZBuf*, ZBuf*)>(
        dlsym(handle, "ZSTD_decompressStream"));
    free_ = reinterpret_cast<size_t (*)(void*)>(dlsym(handle, "ZSTD_freeDStream"));
    is_error = reinterpret_cast<unsigned (*)(size_t)>(dlsym(handle, "ZSTD_isError"));
    error_name = reinterpret_cast<const char* (*)(size_t)>(
        dlsym(handle, "ZSTD_getErrorName"));
    if (!create || !init || !stream || !free_ || !is_error || !error_name) {
      throw std::runtime_error("libzstd.so.1 lacks the streaming API");
    }
  }
};

// Inflates a CCOB payload only as far as the selected entry's last byte;
// returns that entry's bytes and the inflated byte count.
std::vector<uint8_t> inflate_entry(const uint8_t* payload, size_t len,
                                   const std::string& isa, Entry* chosen,
                                   uint64_t* inflated) {
  Zstd z;
  void* ds = z.create();
  z.init(ds);
  ZBuf in{const_cast<uint8_t*>(payload), len, 0};
  std::vector<uint8_t> chunk(8u << 20);
  std::vector<uint8_t> head;   // the bundle header, until it parses
  std::vector<Entry> entries;
  bool have_header = false;
  uint64_t total = 0, want_lo = 0, want_hi = 0;
  std::vector<uint8_t> entry;
  while (true) {
    ZBuf out{chunk.data(), chunk.size(), 0};
    const size_t ret = z.stream(ds, &out, &in);
    if (z.is_error(ret)) {
      z.free_(ds);
      throw std::runtime_error(std::string("zstd: ") + z.error_name(ret));
    }
    uint64_t a = total;
    const uint64_t b = total + out.pos;
    const uint8_t* bytes = chunk.data();
    if (!have_header) {
      head.insert(head.end(), chunk.data(), chunk.data() + out.pos);
      size_t hlen = 0;
      if (parse_bundle_header(head.data(), head.size(), &entries, &hlen)) {
        have_header = true;
        *chosen = *pick(entries, isa);
        want_lo = chosen->offset;
        want_hi = chosen->offset + chosen->size;
        entry.reserve(chosen->size);
        // everything inflated so far ([0, b)) is scanned for the entry
        a = 0;
        bytes = head.data();
      }
    }
    if (have_header) {
      const uint64_t lo = std::max(a, want_lo), hi = std::min(b, want_hi);
      if (hi > lo) {
        entry.insert(entry.end(), bytes + (lo - a), bytes + (hi - a));
      }
      if (bytes == head.data()) {
        std::vector<uint8_t>().swap(head);
      }
      if (entry.size() == chosen->size) {
        total = b;
        break;   // the rest of the stream is other targets: never inflated
      }
    }
    total = b;
    if (out.pos == 0 && in.pos >= in.size) break;
  }
  z.free_(ds);
  if (!have_header || entry.size() != chosen->size) {
    throw std::runtime_error("compressed bundle ended before the entry");
  }
  *inflated = total;
  return entry;
}

// ---------------------------------------------------------------------------
// Drop the .debug_* sections of a code object (ELF64).  They are never
// loaded, so only the file shrinks: allocated sections, program headers and
// every byte the loader maps stay where they were.
std::vector<uint8_t> strip_debug(const std::vector<uint8_t>& in) {
  if (in.size() < sizeof(Elf64_Ehdr) ||
      std::memcmp(in.data(), ELFMAG, SELFMAG) != 0 ||
      in[EI_CLASS] != ELFCLASS64) {
    throw std::runtime_error("code object is not ELF64");
  }
  const auto eh = load<Elf64_Ehdr>(in.data());
  if (eh.e_shentsize != sizeof(Elf64_Shdr) || eh.e_shnum == 0 ||
      eh.e_shoff + uint64_t(eh.e_shnum) * sizeof(Elf64_Shdr) > in.size() ||
      eh.e_shstrndx >= eh.e_shnum) {
    throw std::runtime_error("bad section header table");
  }
  // every offset below comes from the (untrusted) code object: checked
  // against the buffer before it is dereferenced
  const uint64_t size = in.size();
  auto fits = [size](uint64_t off, uint64_t len) {
    return off <= size && len <= size - off;
  };
  if (eh.e_phnum &&
      (eh.e_phentsize != sizeof(Elf64_Phdr) ||
       !fits(eh.e_phoff, uint64_t(eh.e_phnum) * sizeof(Elf64_Phdr)))) {
    throw std::runtime_error("bad program header table");
  }
  std::vector<Elf64_Shdr> sh(eh.e_shnum);
  std::memcpy(sh.data(), in.data() + eh.e_shoff, eh.e_shnum * sizeof(Elf64_Shdr));
  const Elf64_Shdr& strsec = sh[eh.e_shstrndx];
  if (!fits(strsec.sh_offset, strsec.sh_size)) {
    throw std::runtime_error("section name table out of bounds");
  }
  auto name = [&](const Elf64_Shdr& s) {
    // bounded by the string table, never past its end
    if (s.sh_name >= strsec.sh_size) return std::string();
    const char* at = reinterpret_cast<const char*>(in.data() +
                                                   strsec.sh_offset + s.sh_name);
    return std::string(at, strnlen(at, strsec.sh_size - s.sh_name));
  };
  std::vector<int> remap(eh.e_shnum, -1);
  std::vector<int> kept;
  int last_alloc = 0, first_drop = eh.e_shnum;
  uint64_t loaded_end = eh.e_phoff + uint64_t(eh.e_phnum) * eh.e_phentsize;
  for (int i = 0; i < eh.e_shnum; ++i) {
    const bool alloc = sh[i].sh_flags & SHF_ALLOC;
    const bool drop = !alloc && name(sh[i]).rfind(".debug", 0) == 0;
    if (sh[i].sh_type != SHT_NOBITS && !fits(sh[i].sh_offset, sh[i].sh_size)) {
      throw std::runtime_error("section " + std::to_string(i) +
                               " out of bounds");
    }
    if (alloc) {
      last_alloc = i;
      if (sh[i].sh_type != SHT_NOBITS) {
        loaded_end = std::max<uint64_t>(loaded_end, sh[i].sh_offset + sh[i].sh_size);
      }
    }
    if (drop) {
      first_drop = std::min(first_drop, i);
      continue;
    }
    remap[i] = static_cast<int>(kept.size());
    kept.push_back(i);
  }
  if (first_drop == eh.e_shnum) return in;   // nothing to strip
  if (first_drop < last_alloc) {
    // an allocated section after a dropped one would change the indices
    // that .dynsym (inside a loaded segment) refers to
    throw std::runtime_error("debug section before an allocated one");
  }
  for (int i = 0; i < eh.e_phnum; ++i) {
    const auto ph = load<Elf64_Phdr>(in.data() + eh.e_phoff + i * sizeof(Elf64_Phdr));
    if (!fits(ph.p_offset, ph.p_filesz)) {
      throw std::runtime_error("segment out of bounds");
    }
    loaded_end = std::max<uint64_t>(loaded_end, ph.p_offset + ph.p_filesz);
  }
  if (loaded_end > size) throw std::runtime_error("loaded image out of bounds");
  std::vector<uint8_t> out(in.begin(), in.begin() + loaded_end);
  std::vector<Elf64_Shdr> new_sh;
  for (int i : kept) {
    Elf64_Shdr s = sh[i];
    const bool alloc = s.sh_flags & SHF_ALLOC;
    if (!alloc && s.sh_type != SHT_NOBITS) {
      const uint64_t align = std::max<uint64_t>(1, s.sh_addralign);
      out.resize((out.size() + align - 1) / align * align, 0);
      const uint64_t at = out.size();
      out.insert(out.end(), in.begin() + s.sh_offset,
                 in.begin() + s.sh_offset + s.sh_size);
      if (s.sh_type == SHT_SYMTAB) {
        // section symbols and defined symbols name a section index
        for (uint64_t off = 0; off + sizeof(Elf64_Sym) <= s.sh_size;
             off += sizeof(Elf64_Sym)) {
          auto sym = load<Elf64_Sym>(out.data() + at + off);
          if (sym.st_shndx != SHN_UNDEF && sym.st_shndx < SHN_LORESERVE) {
            const int to = sym.st_shndx < eh.e_shnum ? remap[sym.st_shndx] : -1;
            sym.st_shndx = to < 0 ? SHN_ABS : static_cast<uint16_t>(to);
            std::memcpy(out.data() + at + off, &sym, sizeof(sym));
          }
        }
      }
      s.sh_offset = at;
    }
    if (s.sh_link && s.sh_link < eh.e_shnum) {
      s.sh_link = remap[s.sh_link] < 0 ? 0 : remap[s.sh_link];
    }
    if ((s.sh_type == SHT_REL || s.sh_type == SHT_RELA) && s.sh_info &&
        s.sh_info < eh.e_shnum && !(s.sh_flags & SHF_ALLOC)) {
      s.sh_info = remap[s.sh_info] < 0 ? 0 : remap[s.sh_info];
    }
    new_sh.push_back(s);
  }
  out.resize((out.size() + 7) / 8 * 8, 0);
  Elf64_Ehdr neh = eh;
  neh.e_shoff = out.size();
  neh.e_shnum = static_cast<uint16_t>(new_sh.size());
  neh.e_shstrndx = static_cast<uint16_t>(remap[eh.e_shstrndx]);
  const auto* raw = reinterpret_cast<const uint8_t*>(new_sh.data());
  out.insert(out.end(), raw, raw + new_sh.size() * sizeof(Elf64_Shdr));
  std::memcpy(out.data(), &neh, sizeof(neh));
  return out;
}

// ---------------------------------------------------------------------------
struct Source {
  int fd = -1;
  const uint8_t* data = nullptr;
  size_t size = 0;
  ~Source() {
    if (data) munmap(const_cast<uint8_t*>(data), size);
    if (fd >= 0) close(fd);
  }
};

void write_all(int fd, const uint8_t* p, size_t n, off_t at) {
  while (n) {
    const ssize_t w = pwrite(fd, p, std::min<size_t>(n, 1u << 30), at);
    if (w <= 0) throw std::runtime_error("write failed");
    p += w;
    n -= static_cast<size_t>(w);
    at += w;
  }
}

int run(int argc, char** argv) {
  std::string src, out, isa = "gfx950";
  bool strip = true;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--src" && i + 1 < argc) src = argv[++i];
    else if (a == "--out" && i + 1 < argc) out = argv[++i];
    else if (a == "--isa" && i + 1 < argc) isa = argv[++i];
    else if (a == "--no-strip") strip = false;
    else throw std::runtime_error("unknown argument " + a);
  }
  if (src.empty() || out.empty()) {
    throw std::runtime_error("usage: kiosk-rccl-slim --src LIB --out PATH "
                             "[--isa gfx950] [--no-strip]");
  }
  const double t0 = now_ms();
  Source s;
  s.fd = open(src.c_str(), O_RDONLY | O_CLOEXEC);
  if (s.fd < 0) throw std::runtime_error("cannot open " + src);
  struct stat st;
  if (fstat(s.fd, &st) != 0) throw std::runtime_error("stat failed");
  s.size = static_cast<size_t>(st.st_size);
  void* map = mmap(nullptr, s.size, PROT_READ, MAP_PRIVATE, s.fd, 0);
  if (map == MAP_FAILED) throw std::runtime_error("mmap failed");
  s.data = static_cast<const uint8_t*>(map);
  if (s.size < sizeof(Elf64_Ehdr) || std::memcmp(s.data, ELFMAG, SELFMAG) != 0 ||
      s.data[EI_CLASS] != ELFCLASS64) {
    throw std::runtime_error(src + " is not an ELF64 library");
  }
  const auto eh = load<Elf64_Ehdr>(s.data);
  if (eh.e_shoff + uint64_t(eh.e_shnum) * sizeof(Elf64_Shdr) > s.size ||
      eh.e_shstrndx >= eh.e_shnum) {
    throw std::runtime_error("bad section header table");
  }
  const auto* shdrs = reinterpret_cast<const Elf64_Shdr*>(s.data + eh.e_shoff);
  const Elf64_Shdr& strsec = shdrs[eh.e_shstrndx];
  if (strsec.sh_offset > s.size || strsec.sh_size > s.size - strsec.sh_offset) {
    throw std::runtime_error("section name table out of bounds");
  }
  const Elf64_Shdr* fat = nullptr;
  static const char kFat[] = ".hip_fatbin";
  for (int i = 0; i < eh.e_shnum; ++i) {
    // a name is compared only within the string table
    if (shdrs[i].sh_name >= strsec.sh_size ||
        strsec.sh_size - shdrs[i].sh_name < sizeof(kFat)) {
      continue;
    }
    const char* nm = reinterpret_cast<const char*>(s.data + strsec.sh_offset +
                                                   shdrs[i].sh_name);
    if (std::memcmp(nm, kFat, sizeof(kFat)) == 0) fat = &shdrs[i];
  }
  if (!fat || fat->sh_offset > s.size || fat->sh_size > s.size - fat->sh_offset) {
    throw std::runtime_error("no .hip_fatbin section");
  }
  const uint8_t* sec = s.data + fat->sh_offset;
  const size_t sec_size = fat->sh_size;
  Entry chosen;
  std::vector<uint8_t> code;
  uint64_t inflated = 0;
  bool compressed = false;
  int version = 0;
  if (sec_size >= 8 && std::memcmp(sec, kCompressedMagic, 4) == 0) {
    compressed = true;
    version = load<uint16_t>(sec + 4);
    const uint16_t method = load<uint16_t>(sec + 6);
    size_t header = 0, total = sec_size;
    if (version == 1) {
      header = 20;
    } else if (version == 2) {
      header = 24;
      total = load<uint32_t>(sec + 8);
    } else if (version == 3) {
      header = 32;
      total = static_cast<size_t>(load<uint64_t>(sec + 8));
    } else {
      throw std::runtime_error("unknown compressed bundle version");
    }
    if (method != 1) throw std::runtime_error("bundle is not zstd-compressed");
    if (total > sec_size || total < header) total = sec_size;
    code = inflate_entry(sec + header, total - header, isa, &chosen, &inflated);
  } else {
    std::vector<Entry> entries;
    size_t hlen = 0;
    if (!parse_bundle_header(sec, sec_size, &entries, &hlen)) {
      throw std::runtime_error("truncated bundle header");
    }
    chosen = *pick(entries, isa);
    if (chosen.offset + chosen.size > sec_size) {
      throw std::runtime_error("entry outside the section");
    }
    code.assign(sec + chosen.offset, sec + chosen.offset + chosen.size);
  }
  const double t_inflate = now_ms();
  const size_t code_bytes = code.size();
  if (strip) code = strip_debug(code);
  const double t_strip = now_ms();

  // the new bundle: host entry (empty) + the one device code object
  const std::string host_id = "host-x86_64-unknown-linux-gnu-";
  std::vector<uint8_t> bundle(kBundleMagic, kBundleMagic + kBundleMagicLen);
  auto put64 = [&](uint64_t v) {
    const auto* b = reinterpret_cast<const uint8_t*>(&v);
    bundle.insert(bundle.end(), b, b + 8);
  };
  put64(2);
  const uint64_t co_off = kCodeObjectAlign;
  put64(co_off);
  put64(0);
  put64(host_id.size());
  bundle.insert(bundle.end(), host_id.begin(), host_id.end());
  put64(co_off);
  put64(code.size());
  put64(chosen.id.size());
  bundle.insert(bundle.end(), chosen.id.begin(), chosen.id.end());
  if (bundle.size() > co_off) throw std::runtime_error("bundle header too big");
  bundle.resize(co_off, 0);
  bundle.insert(bundle.end(), code.begin(), code.end());
  if (bundle.size() > sec_size) {
    throw std::runtime_error("the slim bundle does not fit the section");
  }

  const std::string tmp = out + ".tmp." + std::to_string(getpid());
  const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0755);
  if (fd < 0) throw std::runtime_error("cannot create " + tmp);
  try {
    if (ftruncate(fd, static_cast<off_t>(s.size)) != 0) {
      throw std::runtime_error("ftruncate failed");
    }
    write_all(fd, s.data, fat->sh_offset, 0);
    write_all(fd, bundle.data(), bundle.size(), static_cast<off_t>(fat->sh_offset));
    const size_t tail = fat->sh_offset + sec_size;
    write_all(fd, s.data + tail, s.size - tail, static_cast<off_t>(tail));
    if (close(fd) != 0) throw std::runtime_error("close failed");
  } catch (...) {
    close(fd);
    unlink(tmp.c_str());
    throw;
  }
  if (rename(tmp.c_str(), out.c_str()) != 0) {
    unlink(tmp.c_str());
    throw std::runtime_error("rename failed");
  }
  const double t_end = now_ms();
  std::printf(
      "{\"src\": \"%s\", \"out\": \"%s\", \"isa\": \"%s\", \"entry\": \"%s\", "
      "\"compressed\": %s, \"bundle_version\": %d, \"section_bytes\": %zu, "
      "\"inflated_bytes\": %llu, \"code_object_bytes\": %zu, "
      "\"slim_code_object_bytes\": %zu, \"inflate_ms\": %.1f, "
      "\"strip_ms\": %.1f, \"write_ms\": %.1f}\n",
      src.c_str(), out.c_str(), isa.c_str(), chosen.id.c_str(),
      compressed ? "true" : "false", version, sec_size,
      static_cast<unsigned long long>(inflated), code_bytes, code.size(),
      t_inflate - t0, t_strip - t_inflate, t_end - t_strip);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  try {
    return run(argc, argv);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "kiosk-rccl-slim: %s\n", e.what());
    return 2;
  }
}
