// Cross-process ring of fixed-width metric rows in a shared-memory file (/dev/shm).
//
// The node's ONE device-counter process (rocmdash/runtime/counterd.py) owns every GPU's
// rocprofiler-sdk counting context - and with it the runtime's one busy-polling
// completion thread - and publishes each GPU's counter rows here; every rank process
// maps its GPU's file read-only (ShmSource, node_counters.cpp) instead of configuring
// counting itself. VERDICT r04 item 3: 8 counting contexts in 8 rank processes kept
// ~8 cores busy per node.
//
// Same single-producer seqlock protocol as SeriesRing (ring.h), with the control words
// in the shared mapping: the producer announces row h in `wpos` (release fence) before
// writing it and publishes `head` = h + 1 (release) after; a reader copies a row, then
// (acquire fence) re-reads `wpos`: rows <= wpos - 1 - cap may have been overwritten
// while it copied and are dropped. The 64-bit atomics are lock-free and address-free,
// so they order across processes. A producer that starts again writes a NEW file and
// renames it over the old path (readers re-open on a new inode / generation).
//
// Layout: [header 4096 B][ts: cap x u64][rows: cap x width x f32].
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace rocmdash {

struct ShmRingHeader {
  uint64_t magic;
  uint32_t version;
  uint32_t width;
  uint64_t cap;
  uint64_t generation;
  double hz;
  int32_t producer_pid;
  int32_t lane;                                 // the publisher's lane generation (re-admissions)
  char kind[16];
  char backend[48];
  alignas(64) std::atomic<uint64_t> head;       // rows completely written
  alignas(64) std::atomic<uint64_t> wpos;       // rows whose writing has started
  alignas(64) std::atomic<uint64_t> beat_ns;    // producer's last tick (CLOCK_REALTIME)
  std::atomic<uint64_t> failures;               // reads that produced no row
  std::atomic<uint64_t> read_ns_total;          // summed duration of the producer's reads
};
static_assert(sizeof(ShmRingHeader) <= 4096, "header must fit its page");
// The node supervisor reads these words from Python (rocmdash/runtime/lanes.py) without
// loading the extension: keep the offsets in step with RING_HEADER_OFFSETS there.
static_assert(offsetof(ShmRingHeader, producer_pid) == 40 && offsetof(ShmRingHeader, lane) == 44, "header layout");
static_assert(offsetof(ShmRingHeader, head) == 128 && offsetof(ShmRingHeader, beat_ns) == 256, "header layout");
static_assert(offsetof(ShmRingHeader, failures) == 264 && offsetof(ShmRingHeader, read_ns_total) == 272, "header layout");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics must be lock-free");

class ShmRing {
 public:
  static constexpr uint64_t kMagic = 0x31474e5248534452ull;  // "RDSHRNG1"
  static constexpr uint32_t kVersion = 1;
  static constexpr size_t kHeader = 4096;

  static size_t bytes_for(uint32_t width, uint64_t cap) { return kHeader + cap * 8 + cap * width * 4; }

  // Producer: create `path` (via a temporary file renamed over it).
  static ShmRing create(const std::string& path, uint32_t width, uint64_t cap, double hz, const std::string& kind,
                        const std::string& backend, uint64_t generation, int32_t lane = 0) {
    if (width == 0 || cap < 2 || (cap & (cap - 1))) throw std::invalid_argument("shm ring: bad width / capacity");
    const std::string tmp = path + ".tmp." + std::to_string(getpid()) + "." + std::to_string(lane);
    int fd = ::open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) throw std::runtime_error("shm ring: cannot create " + tmp);
    const size_t n = bytes_for(width, cap);
    if (ftruncate(fd, off_t(n)) != 0) {
      ::close(fd);
      throw std::runtime_error("shm ring: ftruncate " + tmp);
    }
    void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("shm ring: mmap " + tmp);
    std::memset(p, 0, kHeader);
    auto* h = new (p) ShmRingHeader();
    h->magic = kMagic;
    h->version = kVersion;
    h->width = width;
    h->cap = cap;
    h->generation = generation;
    h->hz = hz;
    h->producer_pid = int32_t(getpid());
    h->lane = lane;
    std::strncpy(h->kind, kind.c_str(), sizeof h->kind - 1);
    std::strncpy(h->backend, backend.c_str(), sizeof h->backend - 1);
    h->head.store(0, std::memory_order_relaxed);
    h->wpos.store(0, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);
    if (::rename(tmp.c_str(), path.c_str()) != 0) {
      munmap(p, n);
      throw std::runtime_error("shm ring: rename to " + path);
    }
    return ShmRing(p, n);
  }

  // Reader: map `path` read-only. Throws when it does not exist or is not a ring.
  static ShmRing open(const std::string& path, ino_t* inode = nullptr) {
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("shm ring: cannot open " + path);
    struct stat st;
    if (fstat(fd, &st) != 0 || size_t(st.st_size) < kHeader) {
      ::close(fd);
      throw std::runtime_error("shm ring: " + path + " is too small");
    }
    void* p = mmap(nullptr, size_t(st.st_size), PROT_READ, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("shm ring: mmap " + path);
    auto* h = static_cast<const ShmRingHeader*>(p);
    if (h->magic != kMagic || h->version != kVersion || size_t(st.st_size) < bytes_for(h->width, h->cap)) {
      munmap(p, size_t(st.st_size));
      throw std::runtime_error("shm ring: " + path + " is not a rocmdash ring");
    }
    if (inode) *inode = st.st_ino;
    return ShmRing(p, size_t(st.st_size));
  }

  ShmRing() = default;
  ShmRing(ShmRing&& o) noexcept { *this = std::move(o); }
  ShmRing& operator=(ShmRing&& o) noexcept {
    if (this != &o) {
      unmap();
      base_ = o.base_;
      bytes_ = o.bytes_;
      o.base_ = nullptr;
      o.bytes_ = 0;
    }
    return *this;
  }
  ShmRing(const ShmRing&) = delete;
  ShmRing& operator=(const ShmRing&) = delete;
  ~ShmRing() { unmap(); }

  bool valid() const { return base_ != nullptr; }
  ShmRingHeader* header() const { return static_cast<ShmRingHeader*>(base_); }
  uint32_t width() const { return header()->width; }
  uint64_t cap() const { return header()->cap; }
  uint64_t head() const { return header()->head.load(std::memory_order_acquire); }

  void push(const float* row, uint64_t t_ns) {
    ShmRingHeader* h = header();
    const uint64_t i = h->head.load(std::memory_order_relaxed);
    const uint64_t idx = i & (h->cap - 1);
    h->wpos.store(i + 1, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_release);
    auto* d = reinterpret_cast<uint32_t*>(rows() + idx * h->width);
    const auto* s = reinterpret_cast<const uint32_t*>(row);
    for (uint32_t k = 0; k < h->width; ++k) __atomic_store_n(d + k, s[k], __ATOMIC_RELAXED);
    __atomic_store_n(ts() + idx, t_ns, __ATOMIC_RELAXED);
    h->head.store(i + 1, std::memory_order_release);
  }

  // Copy row i (< head) into out; false if it was (possibly) overwritten meanwhile.
  bool read(uint64_t i, float* out, uint64_t* t_ns) const {
    const ShmRingHeader* h = header();
    const uint64_t idx = i & (h->cap - 1);
    auto* d = reinterpret_cast<uint32_t*>(out);
    const auto* s = reinterpret_cast<const uint32_t*>(rows() + idx * h->width);
    for (uint32_t k = 0; k < h->width; ++k) d[k] = __atomic_load_n(s + k, __ATOMIC_RELAXED);
    const uint64_t t = __atomic_load_n(ts() + idx, __ATOMIC_RELAXED);
    std::atomic_thread_fence(std::memory_order_acquire);
    const uint64_t w = h->wpos.load(std::memory_order_relaxed);
    if (w > h->cap && w - 1 - h->cap >= i) return false;
    if (t_ns) *t_ns = t;
    return true;
  }

 private:
  ShmRing(void* p, size_t n) : base_(p), bytes_(n) {}
  void unmap() {
    if (base_) munmap(base_, bytes_);
    base_ = nullptr;
  }
  uint64_t* ts() const { return reinterpret_cast<uint64_t*>(static_cast<char*>(base_) + kHeader); }
  float* rows() const { return reinterpret_cast<float*>(static_cast<char*>(base_) + kHeader + header()->cap * 8); }

  void* base_ = nullptr;
  size_t bytes_ = 0;
};

}  // namespace rocmdash
