// Lockstep board in POSIX shared memory: the per-step control exchange of the expert-parallel
// ranks of one node (parallel/expert.py ExpertParallelEngine._exchange) and the doorbell its
// idle ranks sleep on (worker/service.py ExpertService).
//
// Every EP step, each rank publishes (has work, tokens of its next forward, stop bit) and needs
// every other rank's triple before it launches the forward (the MoE all-to-all sizes its
// regions from them). Over gloo that is an all_gather of sockets per step; here each rank
// writes its triple into its own cache line of a mapped segment and bumps its sequence
// number, then waits until every slot carries that sequence: one store + N loads per step,
// no syscall while the peers keep up. Values are double-buffered by sequence parity: a rank
// can run at most one exchange ahead of the slowest reader (it needs everyone's publish of
// step s to finish step s, and a slow rank publishes s only after it read s - 1), so the
// buffer it overwrites has always been read.
//
// Waits spin briefly, then sleep on a futex (the shared `arrivals` word every publish bumps)
// and re-check peer liveness (kill(pid, 0) + /proc state) so a dead rank turns into an error,
// not a hang. The doorbell: a rank with nothing to do (no rank has work) sleeps in
// dli_board_wait_bell until any process rings it (a request arrived on some rank, or a stop
// was requested): 0 % CPU while the group idles, instead of an exchange every few ms.
//
// C ABI for ctypes.
#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

namespace {

constexpr uint64_t kMagic = 0x444c494c4f434b31ull;  // "DLILOCK1"
constexpr int kMaxRanks = 64;
constexpr int kVals = 4;                             // int64 words per rank per step

struct alignas(64) Slot {
  std::atomic<uint64_t> seq;                         // exchanges published by this rank
  std::atomic<int64_t> pid;
  int64_t vals[2][kVals];                            // [seq parity][word]
};                                                   // 128 B: every slot on lines of its own

struct alignas(64) BoardHeader {
  uint64_t magic;
  uint64_t world;
  std::atomic<uint32_t> arrivals;                    // futex word: bumped by every publish
  std::atomic<uint32_t> bell;                        // futex word: bumped by every ring
  std::atomic<uint32_t> closed;
  char pad[64 - 16 - 12];
  Slot slots[kMaxRanks];
};

struct Board {
  int fd = -1;
  size_t bytes = 0;
  BoardHeader* hdr = nullptr;
  std::string name;
  int rank = -1;
  uint64_t seq = 0;                                  // exchanges completed by this rank
  int dead = -1;
};

inline Board* B(void* h) { return reinterpret_cast<Board*>(h); }

inline double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

inline bool pid_alive(int64_t pid) {
  if (pid <= 0) return true;
  if (!(kill((pid_t)pid, 0) == 0 || errno == EPERM)) return false;
  char path[64], buf[512];
  snprintf(path, sizeof path, "/proc/%lld/stat", (long long)pid);
  FILE* f = fopen(path, "r");
  if (!f) return true;
  const size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');
  return !(rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X'));
}

// futex wait on a word of the shared mapping (not FUTEX_PRIVATE: the waiters are processes)
inline void futex_wait(std::atomic<uint32_t>* w, uint32_t expect, double secs) {
  timespec ts;
  ts.tv_sec = (time_t)secs;
  ts.tv_nsec = (long)((secs - (double)ts.tv_sec) * 1e9);
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expect, &ts, nullptr, 0);
}

inline void futex_wake_all(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, 0x7fffffff, nullptr, nullptr, 0);
}

Board* map_board(const char* name, bool create, int world) {
  auto* b = new Board();
  b->name = name;
  b->bytes = sizeof(BoardHeader);
  if (create) {
    shm_unlink(name);
    b->fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (b->fd < 0 || ftruncate(b->fd, (off_t)b->bytes) != 0) {
      if (b->fd >= 0) { close(b->fd); shm_unlink(name); }
      delete b;
      return nullptr;
    }
  } else {
    b->fd = shm_open(name, O_RDWR, 0600);
    struct stat sb;
    if (b->fd < 0 || fstat(b->fd, &sb) != 0 || (size_t)sb.st_size < b->bytes) {
      if (b->fd >= 0) close(b->fd);
      delete b;
      return nullptr;
    }
  }
  void* m = mmap(nullptr, b->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, b->fd, 0);
  if (m == MAP_FAILED) {
    close(b->fd);
    if (create) shm_unlink(name);
    delete b;
    return nullptr;
  }
  b->hdr = reinterpret_cast<BoardHeader*>(m);
  if (create) {
    std::memset(m, 0, b->bytes);
    b->hdr->world = (uint64_t)world;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    reinterpret_cast<std::atomic<uint64_t>*>(&b->hdr->magic)->store(kMagic,
                                                                    std::memory_order_release);
  } else if (reinterpret_cast<std::atomic<uint64_t>*>(&b->hdr->magic)->load(
                 std::memory_order_acquire) != kMagic) {
    munmap(m, b->bytes);
    close(b->fd);
    delete b;
    return nullptr;
  }
  return b;
}

}  // namespace

extern "C" {

// Rank 0: create the segment (replacing a stale one of the same name) for `world` ranks.
void* dli_board_create(const char* name, int world) {
  if (world < 1 || world > kMaxRanks) return nullptr;
  return map_board(name, true, world);
}

// Attach (every rank, rank 0's create handle included, calls dli_board_join once).
void* dli_board_open(const char* name) { return map_board(name, false, 0); }

// Register this process as rank `rank`: its pid becomes visible to the liveness checks.
int dli_board_join(void* h, int rank) {
  auto* b = B(h);
  if (rank < 0 || (uint64_t)rank >= b->hdr->world) return -1;
  b->rank = rank;
  b->seq = b->hdr->slots[rank].seq.load(std::memory_order_acquire);
  b->hdr->slots[rank].pid.store((int64_t)getpid(), std::memory_order_release);
  return 0;
}

// After every rank has opened, remove the name (the mappings stay valid).
int dli_board_unlink(void* h) { return shm_unlink(B(h)->name.c_str()); }

int dli_board_world(void* h) { return (int)B(h)->hdr->world; }

// One lockstep exchange: publish this rank's kVals words, wait until every rank published the
// same exchange, copy all of them to out[world * kVals]. 0 ok; -1 timeout; -2 a peer process
// is gone (dli_board_dead says which); -3 the board was closed.
int dli_board_exchange(void* h, const long long* mine, long long* out, double timeout_s) {
  auto* b = B(h);
  BoardHeader* H = b->hdr;
  const int W = (int)H->world, me = b->rank;
  if (me < 0) return -4;
  const uint64_t s = b->seq + 1, par = s & 1;
  Slot& ms = H->slots[me];
  for (int j = 0; j < kVals; ++j) ms.vals[par][j] = mine[j];
  ms.seq.store(s, std::memory_order_release);
  H->arrivals.fetch_add(1, std::memory_order_acq_rel);
  futex_wake_all(&H->arrivals);
  const double t0 = now_s();
  int spins = 0;
  for (int r = 0; r < W; ++r) {
    while (H->slots[r].seq.load(std::memory_order_acquire) < s) {
      if (H->closed.load(std::memory_order_acquire)) return -3;
      if (++spins < 2048) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
        continue;
      }
      const uint32_t a = H->arrivals.load(std::memory_order_acquire);
      if (H->slots[r].seq.load(std::memory_order_acquire) >= s) break;
      futex_wait(&H->arrivals, a, 0.05);
      // a peer that published and then exited is not a failure: re-check its slot first
      if (H->slots[r].seq.load(std::memory_order_acquire) >= s) break;
      if (!pid_alive(H->slots[r].pid.load(std::memory_order_acquire))) {
        b->dead = r;
        return -2;
      }
      if (timeout_s > 0 && now_s() - t0 > timeout_s) return -1;
    }
  }
  for (int r = 0; r < W; ++r)
    for (int j = 0; j < kVals; ++j) out[r * kVals + j] = H->slots[r].vals[par][j];
  b->seq = s;
  return 0;
}

// Doorbell: the current value, a ring (wakes every sleeper), and a bounded sleep until the
// value differs from `seen` (returns the value read last).
unsigned dli_board_bell(void* h) { return B(h)->hdr->bell.load(std::memory_order_acquire); }

void dli_board_ring(void* h) {
  auto* H = B(h)->hdr;
  H->bell.fetch_add(1, std::memory_order_acq_rel);
  futex_wake_all(&H->bell);
}

unsigned dli_board_wait_bell(void* h, unsigned seen, double timeout_s) {
  auto* H = B(h)->hdr;
  const double t0 = now_s();
  for (;;) {
    const unsigned v = H->bell.load(std::memory_order_acquire);
    if (v != seen || H->closed.load(std::memory_order_acquire)) return v;
    const double left = timeout_s - (now_s() - t0);
    if (left <= 0) return v;
    futex_wait(&H->bell, seen, left < 0.5 ? left : 0.5);
  }
}

// The rank a failed exchange found dead (-1: none), or any rank whose process is gone now.
int dli_board_dead(void* h) {
  auto* b = B(h);
  if (b->dead >= 0) return b->dead;
  for (int r = 0; r < (int)b->hdr->world; ++r) {
    const int64_t pid = b->hdr->slots[r].pid.load(std::memory_order_acquire);
    if (pid > 0 && !pid_alive(pid)) return r;
  }
  return -1;
}

// Wake everything blocked on the board for good (teardown / failure).
void dli_board_close(void* h) {
  auto* H = B(h)->hdr;
  H->closed.store(1, std::memory_order_release);
  H->bell.fetch_add(1, std::memory_order_acq_rel);
  futex_wake_all(&H->bell);
  futex_wake_all(&H->arrivals);
}

void dli_board_destroy(void* h) {
  auto* b = B(h);
  if (!b) return;
  if (b->hdr) munmap(b->hdr, b->bytes);
  if (b->fd >= 0) close(b->fd);
  delete b;
}

}  // extern "C"
