// Single-producer / multi-consumer broadcast ring in POSIX shared memory: the control plane
// of the layer-sharded pipeline (parallel/transport.py).
//
// All stage processes of a pipeline live on one 8-GPU node, so the head's per-tick step
// metadata does not need sockets: the head writes each tick's packed StepMeta ONCE into the
// next slot of a mapped ring and bumps a sequence number; every stage reads it from the same
// pages. Cost per tick on the head: one memcpy of a few KB + one release store, independent
// of the number of stages (the gloo control plane it replaces posted 2 * (N - 1) socket
// sends per tick).
//
// Flow control: the head may run at most `slots` messages ahead of the slowest consumer
// (each consumer publishes its read cursor on its own cache line). Waits spin briefly, then
// back off to short sleeps, and give up when the peer process is gone (kill(pid, 0)) or the
// timeout expires, so a dead head / dead stage turns into an error instead of a hang.
//
// C ABI for ctypes.
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace {

constexpr uint64_t kMagic = 0x444c4952494e4731ull;  // "DLIRING1"
constexpr int kMaxConsumers = 64;

struct alignas(64) Cursor {
  std::atomic<uint64_t> v;
  char pad[64 - sizeof(std::atomic<uint64_t>)];
};

struct alignas(64) RingHeader {
  uint64_t magic;
  uint64_t slots;
  uint64_t slot_bytes;      // payload capacity per slot
  uint64_t consumers;
  int64_t producer_pid;
  std::atomic<uint32_t> closed;
  char pad0[64 - 5 * 8 - 4];
  Cursor head;                              // messages published
  Cursor tail[kMaxConsumers];               // messages consumed, per consumer
  Cursor consumer_pid[kMaxConsumers];
};

struct SlotHeader {
  std::atomic<uint64_t> seq;                // message index + 1 once the payload is complete
  uint64_t len;
};

struct Ring {
  int fd = -1;
  size_t map_bytes = 0;
  uint8_t* base = nullptr;
  RingHeader* hdr = nullptr;
  std::string name;
  bool owner = false;
  uint64_t stride = 0;
  uint64_t read_cursor = 0;                 // consumer side: next message to read
  int consumer = -1;
};

inline Ring* R(void* h) { return reinterpret_cast<Ring*>(h); }

inline uint64_t stride_of(uint64_t slot_bytes) {
  return (sizeof(SlotHeader) + slot_bytes + 63) & ~uint64_t(63);
}

inline SlotHeader* slot_at(Ring* r, uint64_t idx) {
  return reinterpret_cast<SlotHeader*>(r->base + sizeof(RingHeader) +
                                       (idx % r->hdr->slots) * r->stride);
}

inline double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// A process that exited but was not reaped yet (a zombie: its parent — a launcher blocked
// elsewhere — has not waited for it) still answers kill(pid, 0): read its state too.
inline bool pid_alive(int64_t pid) {
  if (pid <= 0) return true;
  if (!(kill((pid_t)pid, 0) == 0 || errno == EPERM)) return false;
  char path[64], buf[512];
  snprintf(path, sizeof path, "/proc/%lld/stat", (long long)pid);
  FILE* f = fopen(path, "r");
  if (!f) return true;                             // no procfs: trust kill()
  const size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');              // "pid (comm) S ..." — comm may hold ')'
  return !(rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X'));
}

// Adaptive wait: spin briefly (the common case: the message is already there), then yield,
// then sleep with a growing period capped at 200 us (a waiting stage must not steal the
// CPU the head's scheduler runs on). Returns false on
// timeout / dead peer.
struct Backoff {
  int n = 0;
  double t0 = now_s();
  bool wait(double timeout_s, int64_t peer_pid) {
    ++n;
    if (n < 256) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
      return true;
    }
    if (n < 272) { sched_yield(); return true; }
    const long us = n < 1000 ? 10 : (n < 4000 ? 50 : 200);
    timespec ts{0, us * 1000};
    nanosleep(&ts, nullptr);
    if ((n & 63) == 0) {
      if (timeout_s > 0 && now_s() - t0 > timeout_s) return false;
      if (!pid_alive(peer_pid)) return false;
    }
    return true;
  }
};

}  // namespace

extern "C" {

// Producer: create (replacing any stale segment of the same name).
void* dli_ring_create(const char* name, long long slots, long long slot_bytes, int consumers) {
  if (slots < 2 || slot_bytes < 8 || consumers < 0 || consumers > kMaxConsumers) return nullptr;
  auto* r = new Ring();
  r->name = name;
  shm_unlink(name);
  r->fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (r->fd < 0) { delete r; return nullptr; }
  r->stride = stride_of((uint64_t)slot_bytes);
  r->map_bytes = sizeof(RingHeader) + (size_t)slots * r->stride;
  if (ftruncate(r->fd, (off_t)r->map_bytes) != 0) {
    close(r->fd); shm_unlink(name); delete r; return nullptr;
  }
  void* m = mmap(nullptr, r->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, r->fd, 0);
  if (m == MAP_FAILED) { close(r->fd); shm_unlink(name); delete r; return nullptr; }
  r->base = (uint8_t*)m;
  r->hdr = reinterpret_cast<RingHeader*>(m);
  std::memset(m, 0, sizeof(RingHeader));
  r->hdr->slots = (uint64_t)slots;
  r->hdr->slot_bytes = (uint64_t)slot_bytes;
  r->hdr->consumers = (uint64_t)consumers;
  r->hdr->producer_pid = (int64_t)getpid();
  for (long long i = 0; i < slots; ++i) {
    auto* s = slot_at(r, (uint64_t)i);
    s->seq.store(0, std::memory_order_relaxed);
    s->len = 0;
  }
  r->owner = true;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  reinterpret_cast<std::atomic<uint64_t>*>(&r->hdr->magic)->store(kMagic,
                                                                  std::memory_order_release);
  return r;
}

// Consumer `index` in [0, consumers): attach to an existing ring.
void* dli_ring_open(const char* name, int index) {
  auto* r = new Ring();
  r->name = name;
  r->fd = shm_open(name, O_RDWR, 0600);
  if (r->fd < 0) { delete r; return nullptr; }
  struct stat sb;
  if (fstat(r->fd, &sb) != 0 || (size_t)sb.st_size < sizeof(RingHeader)) {
    close(r->fd); delete r; return nullptr;
  }
  r->map_bytes = (size_t)sb.st_size;
  void* m = mmap(nullptr, r->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, r->fd, 0);
  if (m == MAP_FAILED) { close(r->fd); delete r; return nullptr; }
  r->base = (uint8_t*)m;
  r->hdr = reinterpret_cast<RingHeader*>(m);
  const uint64_t magic =
      reinterpret_cast<std::atomic<uint64_t>*>(&r->hdr->magic)->load(std::memory_order_acquire);
  if (magic != kMagic || index < 0 || (uint64_t)index >= r->hdr->consumers ||
      sizeof(RingHeader) + r->hdr->slots * stride_of(r->hdr->slot_bytes) > r->map_bytes) {
    munmap(m, r->map_bytes); close(r->fd); delete r; return nullptr;
  }
  r->stride = stride_of(r->hdr->slot_bytes);
  r->consumer = index;
  r->read_cursor = r->hdr->tail[index].v.load(std::memory_order_acquire);
  r->hdr->consumer_pid[index].v.store((uint64_t)getpid(), std::memory_order_release);
  return r;
}

// Producer: after every consumer has opened, remove the name (the mapping stays valid).
int dli_ring_unlink(void* h) {
  auto* r = R(h);
  if (!r || r->name.empty()) return -1;
  return shm_unlink(r->name.c_str());
}

long long dli_ring_slot_bytes(void* h) { return (long long)R(h)->hdr->slot_bytes; }

// Publish one message. 0 = ok, -1 = too large, -2 = timeout / a consumer died, -3 = closed.
int dli_ring_publish(void* h, const void* data, long long n, double timeout_s) {
  auto* r = R(h);
  auto* hd = r->hdr;
  if (n < 0 || (uint64_t)n > hd->slot_bytes) return -1;
  const uint64_t seq = hd->head.v.load(std::memory_order_relaxed);
  // wait until the slowest consumer has read the message that used this slot last
  for (uint64_t c = 0; c < hd->consumers; ++c) {
    Backoff b;
    while (seq >= hd->slots &&
           hd->tail[c].v.load(std::memory_order_acquire) + hd->slots <= seq) {
      if (hd->closed.load(std::memory_order_relaxed)) return -3;
      if (!b.wait(timeout_s, (int64_t)hd->consumer_pid[c].v.load(std::memory_order_relaxed)))
        return -2;
    }
  }
  SlotHeader* s = slot_at(r, seq);
  std::memcpy(reinterpret_cast<uint8_t*>(s) + sizeof(SlotHeader), data, (size_t)n);
  s->len = (uint64_t)n;
  s->seq.store(seq + 1, std::memory_order_release);
  hd->head.v.store(seq + 1, std::memory_order_release);
  return 0;
}

// Consume the next message into `out` (capacity `cap`). Returns its length, -1 if `cap` is
// too small (the message stays unread), -2 on timeout / dead producer, -3 if closed and
// drained.
long long dli_ring_consume(void* h, void* out, long long cap, double timeout_s) {
  auto* r = R(h);
  auto* hd = r->hdr;
  const uint64_t want = r->read_cursor;
  SlotHeader* s = slot_at(r, want);
  Backoff b;
  while (s->seq.load(std::memory_order_acquire) != want + 1) {
    if (hd->closed.load(std::memory_order_acquire) &&
        hd->head.v.load(std::memory_order_acquire) <= want)
      return -3;
    if (!b.wait(timeout_s, hd->producer_pid)) return -2;
  }
  const uint64_t n = s->len;
  if ((long long)n > cap) return -1;
  std::memcpy(out, reinterpret_cast<uint8_t*>(s) + sizeof(SlotHeader), (size_t)n);
  r->read_cursor = want + 1;
  hd->tail[r->consumer].v.store(want + 1, std::memory_order_release);
  return (long long)n;
}

// Length of the next message without consuming it (-2 timeout / dead producer, -3 closed).
long long dli_ring_peek_len(void* h, double timeout_s) {
  auto* r = R(h);
  auto* hd = r->hdr;
  const uint64_t want = r->read_cursor;
  SlotHeader* s = slot_at(r, want);
  Backoff b;
  while (s->seq.load(std::memory_order_acquire) != want + 1) {
    if (hd->closed.load(std::memory_order_acquire) &&
        hd->head.v.load(std::memory_order_acquire) <= want)
      return -3;
    if (!b.wait(timeout_s, hd->producer_pid)) return -2;
  }
  return (long long)s->len;
}

long long dli_ring_published(void* h) {
  return (long long)R(h)->hdr->head.v.load(std::memory_order_acquire);
}

long long dli_ring_min_consumed(void* h) {
  auto* hd = R(h)->hdr;
  uint64_t m = hd->head.v.load(std::memory_order_acquire);
  for (uint64_t c = 0; c < hd->consumers; ++c) {
    const uint64_t t = hd->tail[c].v.load(std::memory_order_acquire);
    if (t < m) m = t;
  }
  return (long long)m;
}

// Liveness of the ring's processes (the pipeline watchdog polls this every ~0.2 s, so a
// stage that dies is noticed in well under a second instead of when a wait times out):
// -1 all alive, consumer index c (>= 0) if consumer c's process is gone, 1000 if the
// producer's is. Consumers that never opened (pid 0) count as alive.
int dli_ring_dead(void* h) {
  auto* hd = R(h)->hdr;
  if (!pid_alive(hd->producer_pid)) return 1000;
  for (uint64_t c = 0; c < hd->consumers; ++c) {
    const int64_t pid = (int64_t)hd->consumer_pid[c].v.load(std::memory_order_acquire);
    if (pid > 0 && !pid_alive(pid)) return (int)c;
  }
  return -1;
}

void dli_ring_close(void* h) {
  auto* r = R(h);
  if (r && r->hdr) r->hdr->closed.store(1, std::memory_order_release);
}

void dli_ring_destroy(void* h) {
  auto* r = R(h);
  if (!r) return;
  if (r->base) munmap(r->base, r->map_bytes);
  if (r->fd >= 0) close(r->fd);
  if (r->owner && !r->name.empty()) shm_unlink(r->name.c_str());
  delete r;
}

}  // extern "C"
