// Device-memory mailbox transport between the processes of one node (hipIpc): the
// pipeline / expert-parallel data plane without RCCL ("loopback transport
// (same C++ interface): stage-ranks on one GPU exchange via device memcpy / IPC handles").
// The reference has no data plane at all — its "shards" exchange nothing
// (master/dashboard/views.py:318-355, worker/app.py:332-372).
//
// Every directed edge src -> dst owns one mailbox in dst's HBM plus two flag words that
// work as binary semaphores: READY (in dst's flag page) and FREE (in src's page, initially
// 1). A message goes
//
//   src stream: wait FREE == 1; FREE = 0; put kernel (mailbox <- header + payload); READY = 1
//   dst stream: wait READY == 1; READY = 0; get kernel (target <- payload, header checked); FREE = 1
//
// (waits = one-lane wait kernels with a wall-clock budget, signals = release-store kernels;
// DLI_IPC_SYNC=stream uses hipStreamWaitValue64 / hipStreamWriteValue64 outside graph
// capture instead, unbounded). The put kernel's stores are xGMI peer writes on an 8-GPU
// node, local stores when the ranks share one GPU. No sequence number lives on the host, so
// an exchange captured in a hipGraph is correct on every replay, and eager and captured
// exchanges interleave freely. The sender runs at most one message ahead per edge, which the
// anti-diagonal pipeline schedule never needs to exceed: every wait depends on a strictly
// earlier tick, so it cannot deadlock.
//
// All of it is enqueued on the caller's stream (the stage's compute stream): the send is
// ordered after the kernels that produced the payload and the receive before the kernels
// that read the target, with no events, no side stream and no host wait. Matching is strictly
// FIFO per edge, the same rule RCCL applies (tags are ignored), so a schedule that works
// here has RCCL's ordering.
//
// Flag words live either in device memory (exported with the mailbox) or in a POSIX
// shared-memory page registered with HIP ("host" flags): then the host can observe how far
// every queue has got and ABORT a ring whose peer died by setting every flag it could be
// waiting on (dli_ipc_abort), which a device-only wait could never be released from.
//
// Memory model across GPUs. A sender writes the peer's mailbox over xGMI; the receiver then
// reads it from its own HBM. With ordinary (coarse-grained) allocations the receiver's L2
// may still hold lines of the PREVIOUS message it read from the same mailbox (a peer's
// remote write does not invalidate them, and a coarse-grained local line is not invalidated
// at a kernel boundary), so mailboxes and flag pages are allocated UNCACHED
// (hipExtMallocWithFlags hipDeviceMallocUncached, the kind RCCL uses for its own flags and
// LL buffers): no XCD's L2 ever holds a copy, every load and store goes to memory. Flags are
// written with system-scope release stores after the payload kernel and polled with
// system-scope acquire loads. DLI_IPC_MEM = uncached (default) | fine | coarse selects the
// allocation (coarse = the round-3 layout, for A/B only); the kind in use is reported by
// dli_ipc_mem_kind.
//
// Every message carries a 16-byte header {sequence, bytes}. Each rank keeps a 64-bit
// counter per edge and direction in its own device memory, advanced by the copy kernels
// themselves (so a captured exchange advances it on every replay): the sender stamps
// ++seq_out[peer], the receiver checks header.seq == ++seq_in[peer]. A stale mailbox (an old
// message read again) or a lost / duplicated message sets bit 2 of the error word instead of
// silently yielding wrong activations. (Sizes are not compared on the device: a captured
// decode graph moves its padded bucket while the eager peer moves the live rows; the CPU
// model of the protocol, parallel/fifo.py, does assert equal sizes of the unpadded schedule.)
//
// Error word: bit 0 = a bounded wait ran out of budget (a peer stopped signalling), bit 1 =
// sequence / size mismatch, bit 2 = aborted. It lives twice: in pinned host memory (the host
// polls it every pipeline tick with a plain load, no HIP call) and in the flag page (the
// device mirror that wait and signal kernels test first). Once set the endpoint is
// sticky-failed: every later wait returns at once and no signal is sent, so a broken ring
// drains its queues in microseconds and the host fails the session (HTTP 503) instead of
// serving tokens computed from stale data.
//
// C ABI (ctypes): 0 / >= 0 on success, negative hipError_t (or -1000 - reason) on failure.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

constexpr size_t kFlagStride = 16;   // words between flags (128 B: one flag per line)
constexpr long long kHdr = 16;       // message header {sequence, bytes} in front of a payload
enum : uint64_t { kErrWait = 1, kErrSeq = 2, kErrAbort = 4 };

struct Edge {                        // one peer, both directions
  // outbound (me -> peer)
  uint8_t* peer_mailbox = nullptr;   // peer's mailbox for my messages (mapped)
  uint64_t* peer_ready = nullptr;    // peer's READY word for me (mapped)
  uint64_t* my_free = nullptr;       // my FREE word for this edge (peer sets it)
  long long out_bytes = 0;           // mailbox payload capacity
  // inbound (peer -> me)
  uint8_t* my_mailbox = nullptr;
  uint64_t* my_ready = nullptr;
  uint64_t* peer_free = nullptr;     // the peer's FREE word for messages to me (mapped)
  long long in_bytes = 0;
};

// error bookkeeping shared by every kernel of an endpoint
struct ErrRef {
  uint64_t* dev;                     // device mirror (flag page): tested by wait / signal
  uint64_t* host;                    // pinned host word (device address): polled by the host
};

// The device mirror takes the read-modify-write; the pinned host word only a plain
// system-scope store of the accumulated bits (a device atomic on host memory needs PCIe
// AtomicOps from the root complex, which a host may not provide). Bits only ever grow, so a
// racing store can at worst drop another raiser's bit — or the abort bit dli_ipc_abort set on
// the host before its flag copy reached the device mirror — from the host copy, never clear
// the word: the host's per-tick poll still sees a nonzero error, and dli_ipc_error ORs the
// endpoint's host-side sticky abort flag back in, so "aborted" is never lost.
__device__ __forceinline__ void raise_err(ErrRef e, uint64_t bit) {
  const uint64_t v =
      __hip_atomic_fetch_or(e.dev, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) | bit;
  __hip_atomic_store(e.host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Sender: payload -> peer mailbox (after the header), header {++seq, bytes}. A plain
// vectorised copy on the caller's stream keeps a hop to one launch on the compute queue
// (hipMemcpyAsync between IPC-mapped buffers may be routed to an SDMA engine, measured at
// ~40 GB/s for 4 MB messages on one MI355X: profiles/r3/ipc_probe_*.jsonl).
__global__ void __launch_bounds__(256) ipc_put_kernel(uint8_t* __restrict__ mbox,
                                                      const uint8_t* __restrict__ src,
                                                      long long bytes, int vec,
                                                      uint64_t* __restrict__ seq_out,
                                                      ErrRef err) {
  // a failed / aborted endpoint writes nothing more into a peer's memory (the peer may be
  // gone): one load of the error mirror, uniform over the grid
  if (__hip_atomic_load(err.dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) return;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    const uint64_t s = *seq_out + 1;
    *seq_out = s;
    reinterpret_cast<uint64_t*>(mbox)[0] = s;
    reinterpret_cast<uint64_t*>(mbox)[1] = (uint64_t)bytes;
  }
  if (vec) {                       // 16-B aligned source: uint4 copy, 4 loads in flight
    const uint4* s4 = reinterpret_cast<const uint4*>(src);
    uint4* d4 = reinterpret_cast<uint4*>(mbox + kHdr);
    const long n16 = bytes / 16;
    for (; i + 3 * stride < n16; i += 4 * stride) {
      const uint4 a = s4[i], b = s4[i + stride], c = s4[i + 2 * stride], d = s4[i + 3 * stride];
      d4[i] = a;
      d4[i + stride] = b;
      d4[i + 2 * stride] = c;
      d4[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) d4[i] = s4[i];
    i = n16 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x;   // the 4-B tail
  }
  const uint32_t* s1 = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d1 = reinterpret_cast<uint32_t*>(mbox + kHdr);
  for (const long n4 = bytes / 4; i < n4; i += stride) d1[i] = s1[i];
}

// Receiver: mailbox payload -> target, the header's sequence number checked against
// ++seq_in. Sizes may legitimately differ by bucket padding (a stage's captured decode graph
// receives / sends its whole padded bucket while the eager side moves the live rows), so the
// copy takes min(sent, expected) bytes: padding rows keep stale values, which nothing reads.
__global__ void __launch_bounds__(256) ipc_get_kernel(uint8_t* __restrict__ dst,
                                                      const uint8_t* __restrict__ mbox,
                                                      long long bytes, int vec,
                                                      uint64_t* __restrict__ seq_in, ErrRef err) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t* h = reinterpret_cast<const uint64_t*>(mbox);
  if (i == 0) {
    const uint64_t s = *seq_in + 1;
    *seq_in = s;
    if (h[0] != s) raise_err(err, kErrSeq);
  }
  const long long sent = (long long)h[1];
  bytes = sent < bytes ? sent : bytes;
  if (vec) {
    const uint4* s4 = reinterpret_cast<const uint4*>(mbox + kHdr);
    uint4* d4 = reinterpret_cast<uint4*>(dst);
    const long n16 = bytes / 16;
    for (; i + 3 * stride < n16; i += 4 * stride) {
      const uint4 a = s4[i], b = s4[i + stride], c = s4[i + 2 * stride], d = s4[i + 3 * stride];
      d4[i] = a;
      d4[i + stride] = b;
      d4[i + 2 * stride] = c;
      d4[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) d4[i] = s4[i];
    i = n16 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  }
  const uint32_t* s1 = reinterpret_cast<const uint32_t*>(mbox + kHdr);
  uint32_t* d1 = reinterpret_cast<uint32_t*>(dst);
  for (const long n4 = bytes / 4; i < n4; i += stride) d1[i] = s1[i];
}

// ---- expert-parallel all-to-all on the mailboxes: row counts live on the device -------
// A dispatch message on edge s -> p is [int64 count | uint64 sequence | ids int32 x cap |
// rows x row_bytes] (return messages use the same offsets, no ids). Only `count` rows move;
// the grid is sized for the mailbox capacity and threads past the count exit, so no routing
// value is ever read on the host and the whole exchange can be captured in a graph. The
// receiver clamps the count to the region it reserved for the source (recv_cap): rows past
// it are dropped and flagged (kErrSeq), never written past the region.
__device__ __forceinline__ long ep_ids_off() { return 16; }
__device__ __forceinline__ long ep_rows_off(int cap) {
  return 16 + (((long)cap * 4 + 15) / 16) * 16;
}

__global__ void __launch_bounds__(256) ep_put_kernel(uint8_t* __restrict__ mbox, int cap,
                                                     const int* __restrict__ count,
                                                     const uint4* __restrict__ x, int row16,
                                                     const int* __restrict__ ids,
                                                     uint64_t* __restrict__ seq_out,
                                                     ErrRef err) {
  if (__hip_atomic_load(err.dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) return;
  const int n = min(*count, cap);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint64_t s = *seq_out + 1;
    *seq_out = s;
    reinterpret_cast<long long*>(mbox)[0] = n;
    reinterpret_cast<uint64_t*>(mbox)[1] = s;
  }
  int* mid = reinterpret_cast<int*>(mbox + ep_ids_off());
  uint4* mrow = reinterpret_cast<uint4*>(mbox + ep_rows_off(cap));
  const long stride = (long)gridDim.x * blockDim.x;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (ids != nullptr)
    for (long i = tid; i < n; i += stride) mid[i] = ids[i];
  const long total = (long)n * row16;
  for (long i = tid; i < total; i += stride) mrow[i] = x[i];
}

__global__ void __launch_bounds__(256) ep_get_kernel(const uint8_t* __restrict__ mbox, int cap,
                                                     uint4* __restrict__ x, int row16,
                                                     int* __restrict__ ids, int fill,
                                                     int maxn, int* __restrict__ count_out,
                                                     uint64_t* __restrict__ seq_in, ErrRef err) {
  const long long hn = *reinterpret_cast<const long long*>(mbox);
  const int n = (int)min(min(hn, (long long)cap), (long long)maxn);
  const int* mid = reinterpret_cast<const int*>(mbox + ep_ids_off());
  const uint4* mrow = reinterpret_cast<const uint4*>(mbox + ep_rows_off(cap));
  const long stride = (long)gridDim.x * blockDim.x;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid == 0) {
    const uint64_t s = *seq_in + 1;
    *seq_in = s;
    if (reinterpret_cast<const uint64_t*>(mbox)[1] != s || hn > maxn || hn < 0)
      raise_err(err, kErrSeq);
    if (count_out != nullptr) *count_out = n;
  }
  if (ids != nullptr)
    for (long i = tid; i < fill; i += stride) ids[i] = i < n ? mid[i] : -1;
  const long total = (long)n * row16;
  for (long i = tid; i < total; i += stride) x[i] = mrow[i];
}

// the rank's own bucket: send region -> receive region (ids -1 past the count), at most
// maxn rows (the destination region)
__global__ void __launch_bounds__(256) ep_local_kernel(const int* __restrict__ count,
                                                       const uint4* __restrict__ xs, int row16,
                                                       const int* __restrict__ ids_s,
                                                       uint4* __restrict__ xd,
                                                       int* __restrict__ ids_d, int fill,
                                                       int maxn, int* __restrict__ count_out) {
  const int n = min(*count, maxn);
  const long stride = (long)gridDim.x * blockDim.x;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (count_out != nullptr && tid == 0) *count_out = n;
  if (ids_d != nullptr)
    for (long i = tid; i < fill; i += stride) ids_d[i] = i < n ? ids_s[i] : -1;
  const long total = (long)n * row16;
  for (long i = tid; i < total; i += stride) xd[i] = xs[i];
}

// Semaphore waits / signals as kernels: the default (bounded waits), and always while a
// stream is being captured into a hipGraph (stream write/wait-value operations captured
// into a graph were measured to lose their ordering against the copy kernels on replay:
// profiles/r3/ipc_probe_*.jsonl, check "graph"). One lane polls the flag and the error
// mirror with system-scope acquire loads and a wall-clock budget. A wait that runs out of
// budget raises kErrWait and leaves the flag alone; once the error word is set every later
// wait returns at once and no signal is sent (sticky failure: the queue drains).
__global__ void ipc_wait_kernel(uint64_t* flag, ErrRef err, unsigned long long budget) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  while (true) {
    if (__hip_atomic_load(err.dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) return;
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 1ull) break;
    __builtin_amdgcn_s_sleep(4);
    if (wall_clock64() - t0 > budget) {
      raise_err(err, kErrWait);
      return;
    }
  }
  __hip_atomic_store(flag, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void ipc_signal_kernel(uint64_t* flag, ErrRef err) {
  if (threadIdx.x != 0) return;
  if (__hip_atomic_load(err.dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) return;
  __hip_atomic_store(flag, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void ipc_bump_kernel(uint64_t* ctr, uint64_t d) { if (threadIdx.x == 0) *ctr += d; }

enum MemKind { kCoarse = 0, kFine = 1, kUncached = 2 };

struct Endpoint {
  int world = 0, rank = 0;
  int sync_mode = 1;                  // 1: wait / signal kernels (bounded); 0: stream ops
  unsigned long long wait_budget = 0; // wall-clock ticks a wait kernel polls at most
  long long khz = 100000;             // wall clock rate
  ErrRef err{nullptr, nullptr};       // device addresses of the two error words
  uint64_t* err_host = nullptr;       // pinned host error word (host address)
  // set by dli_ipc_abort on the host only and ORed into dli_ipc_error: a device raise that
  // lands on err_host between the abort's fetch_or and its flag copy overwrites the word with
  // the device mirror's bits (plain store), which would drop "aborted" from the report
  std::atomic<uint64_t> host_sticky{0};
  uint64_t* seq = nullptr;            // device: seq_out[world], seq_in[world]
  bool host_flags = false;
  int mem_kind = kUncached;
  hipStream_t abort_stream = nullptr; // device-flag abort: its own (SDMA) queue
  uint64_t* abort_src = nullptr;      // pinned page of FREE/READY = 1 patterns + error bit
  uint8_t* mailbox = nullptr;        // local, all inbound edges
  size_t mailbox_bytes = 0;
  uint64_t* flags = nullptr;         // local flag page (device or registered host memory)
  uint64_t* flags_dev = nullptr;     // its device address
  size_t flag_bytes = 0;
  std::vector<long long> cap;        // mailbox payload bytes per edge [src * world + dst]
  std::vector<Edge> edge;
  std::vector<void*> opened;         // mapped peer allocations (device flags / mailboxes)
  std::vector<uint64_t*> host_pages; // host flag mode: every rank's page, mapped here
  std::string shm_prefix;
  uint64_t sends = 0, recvs = 0, bytes_out = 0;
};

inline Endpoint* E(void* h) { return reinterpret_cast<Endpoint*>(h); }
inline int herr(hipError_t e) { return e == hipSuccess ? 0 : -(int)e; }

// flag page of rank r: READY[src] for every src, then FREE[dst] for every dst, then the
// device error mirror
inline size_t ready_word(int src) { return (size_t)src * kFlagStride; }
inline size_t free_word(const Endpoint* e, int dst) {
  return ((size_t)e->world + dst) * kFlagStride;
}
inline size_t err_word(const Endpoint* e) { return 2 * (size_t)e->world * kFlagStride; }
inline long long slot_bytes(long long cap) { return cap > 0 ? kHdr + ((cap + 15) / 16) * 16 : 0; }
inline size_t mailbox_off(const Endpoint* e, int dst, int src) {
  size_t off = 0;
  for (int s = 0; s < src; ++s) off += (size_t)slot_bytes(e->cap[s * e->world + dst]);
  return off;
}

// Shared device memory of the requested kind that can be exported with hipIpcGetMemHandle;
// falls back towards coarse-grained (the kind actually used is returned in *kind).
hipError_t alloc_shared(void** p, size_t bytes, int* kind) {
  const char* m = getenv("DLI_IPC_MEM");
  int want = kUncached;
  if (m != nullptr && std::string(m) == "fine") want = kFine;
  if (m != nullptr && std::string(m) == "coarse") want = kCoarse;
  for (int k = want; k >= kCoarse; --k) {
    hipError_t r;
    if (k == kUncached) r = hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
    else if (k == kFine) r = hipExtMallocWithFlags(p, bytes, hipDeviceMallocFinegrained);
    else r = hipMalloc(p, bytes);
    if (r != hipSuccess) { (void)hipGetLastError(); continue; }
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, *p) != hipSuccess) {   // not exportable: next kind
      (void)hipGetLastError();
      (void)hipFree(*p);
      *p = nullptr;
      continue;
    }
    *kind = k;
    return hipSuccess;
  }
  return hipErrorOutOfMemory;
}

std::string page_name(const std::string& prefix, int r) {
  return prefix + "_" + std::to_string(r);
}

uint64_t* map_host_page(const std::string& name, size_t bytes, bool create) {
  int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) return nullptr;
  if (create && ftruncate(fd, (off_t)bytes) != 0) {
    close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  if (hipHostRegister(p, bytes, hipHostRegisterMapped) != hipSuccess) {
    munmap(p, bytes);
    return nullptr;
  }
  return reinterpret_cast<uint64_t*>(p);
}

uint64_t* dev_addr(uint64_t* host) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) return nullptr;
  return reinterpret_cast<uint64_t*>(d);
}

void set_word(uint64_t* w, uint64_t v) {
  reinterpret_cast<std::atomic<uint64_t>*>(w)->store(v, std::memory_order_release);
}

unsigned blocks_for(long n16) {
  long b = (n16 + 4 * 256 - 1) / (4 * 256);
  return (unsigned)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
}

// wait until *w == 1 then reset it (bounded kernel, or a stream op); signal *w = 1
int wait_flag(Endpoint* e, hipStream_t s, uint64_t* w) {
  if (e->sync_mode == 1 || capturing(s)) {
    ipc_wait_kernel<<<1, 64, 0, s>>>(w, e->err, e->wait_budget);
    return herr(hipGetLastError());
  }
  int r = herr(hipStreamWaitValue64(s, w, 1, hipStreamWaitValueEq));
  return r ? r : herr(hipStreamWriteValue64(s, w, 0, 0));
}
int signal_flag(Endpoint* e, hipStream_t s, uint64_t* w) {
  if (e->sync_mode == 1 || capturing(s)) {
    ipc_signal_kernel<<<1, 64, 0, s>>>(w, e->err);
    return herr(hipGetLastError());
  }
  return herr(hipStreamWriteValue64(s, w, 1, 0));
}

}  // namespace

extern "C" {

int dli_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// Allocate this rank's inbound mailboxes and flag page. cap: world x world matrix of mailbox
// payload bytes (row = src, col = dst; 0 = no edge), identical on every rank. host_prefix:
// shm page name prefix (rank r's page is "<prefix>_<r>"), or "" for device flags.
void* dli_ipc_create(int world, int rank, const long long* cap, const char* host_prefix) {
  if (world < 1 || rank < 0 || rank >= world) return nullptr;
  auto* e = new Endpoint();
  e->world = world;
  e->rank = rank;
  e->cap.assign(cap, cap + (size_t)world * world);
  e->edge.resize(world);
  e->host_flags = host_prefix != nullptr && host_prefix[0] != '\0';
  for (int s = 0; s < world; ++s) e->mailbox_bytes += (size_t)slot_bytes(e->cap[s * world + rank]);
  auto fail = [&]() -> void* {
    if (e->mailbox) (void)hipFree(e->mailbox);
    if (e->seq) (void)hipFree(e->seq);
    if (e->err_host) (void)hipHostFree(e->err_host);
    delete e;
    return nullptr;
  };
  if (e->mailbox_bytes &&
      (alloc_shared(reinterpret_cast<void**>(&e->mailbox), e->mailbox_bytes, &e->mem_kind) !=
           hipSuccess ||
       hipMemset(e->mailbox, 0, e->mailbox_bytes) != hipSuccess))
    return fail();
  if (hipMalloc(reinterpret_cast<void**>(&e->seq), 2 * (size_t)world * 8) != hipSuccess ||
      hipMemset(e->seq, 0, 2 * (size_t)world * 8) != hipSuccess)
    return fail();
  if (hipHostMalloc(reinterpret_cast<void**>(&e->err_host), 64,
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return fail();
  std::memset(e->err_host, 0, 64);
  e->err.host = dev_addr(e->err_host);
  e->flag_bytes = (((2 * (size_t)world + 1) * kFlagStride * 8 + 4095) / 4096) * 4096;
  const char* sm = getenv("DLI_IPC_SYNC");
  e->sync_mode = (sm != nullptr && std::string(sm) == "stream") ? 0 : 1;
  {
    int khz = 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
      khz = 100000;
    e->khz = khz;
    // the budget covers the longest legitimate gap between a peer's send and this rank's
    // receive (a long prefill on a shared GPU, a first-use library load): 120 s by default,
    // DLI_IPC_WAIT_S per deployment. A dead peer is caught long before by the pipeline
    // watchdog (process liveness on the control ring), which aborts the endpoint.
    const char* bs = getenv("DLI_IPC_WAIT_S");
    const double secs = bs ? atof(bs) : 120.0;
    e->wait_budget = (unsigned long long)(secs * 1000.0 * khz);
  }
  // FREE words start at 1 (every mailbox empty), READY words and the error mirror at 0
  std::vector<uint64_t> init(e->flag_bytes / 8, 0);
  for (int d = 0; d < world; ++d) init[free_word(e, d)] = 1;
  if (e->host_flags) {
    e->shm_prefix = host_prefix;
    const std::string name = page_name(e->shm_prefix, rank);
    shm_unlink(name.c_str());
    uint64_t* p = map_host_page(name, e->flag_bytes, true);
    if (p == nullptr) return fail();
    std::memcpy(p, init.data(), e->flag_bytes);
    e->flags = p;
    e->flags_dev = dev_addr(p);
    e->host_pages.assign(world, nullptr);
    e->host_pages[rank] = p;
  } else {
    int k = kCoarse;
    if (alloc_shared(reinterpret_cast<void**>(&e->flags), e->flag_bytes, &k) != hipSuccess ||
        hipMemcpy(e->flags, init.data(), e->flag_bytes, hipMemcpyHostToDevice) != hipSuccess)
      return fail();
    if (e->mailbox_bytes == 0) e->mem_kind = k;
    e->flags_dev = e->flags;
    if (hipStreamCreateWithFlags(&e->abort_stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&e->abort_src), e->flag_bytes,
                      hipHostMallocDefault) != hipSuccess) {
      e->abort_stream = nullptr;
      e->abort_src = nullptr;
    } else {
      std::memset(e->abort_src, 0, e->flag_bytes);
      for (size_t i = 0; i < 2 * (size_t)world; ++i) e->abort_src[i * kFlagStride] = 1;
      e->abort_src[err_word(e)] = kErrAbort;
    }
  }
  e->err.dev = e->flags_dev + err_word(e);
  (void)hipDeviceSynchronize();
  return e;
}

// This rank's IPC handles into `out` (2 * dli_ipc_handle_bytes()): the mailbox (zeros if it
// has none) and, in device-flag mode, the flag page (zeros in host-flag mode).
int dli_ipc_handles(void* h, void* out) {
  auto* e = E(h);
  const size_t hb = sizeof(hipIpcMemHandle_t);
  auto* o = reinterpret_cast<uint8_t*>(out);
  std::memset(o, 0, 2 * hb);
  if (e->mailbox) {
    hipIpcMemHandle_t mh;
    const int r = herr(hipIpcGetMemHandle(&mh, e->mailbox));
    if (r) return r;
    std::memcpy(o, &mh, hb);
  }
  if (!e->host_flags) {
    hipIpcMemHandle_t fh;
    const int r = herr(hipIpcGetMemHandle(&fh, e->flags));
    if (r) return r;
    std::memcpy(o + hb, &fh, hb);
  }
  return 0;
}

// Map every connected peer's mailbox + flags. handles: world * 2 * handle_bytes, rank-major,
// as written by dli_ipc_handles on each rank.
int dli_ipc_connect(void* h, const void* handles) {
  auto* e = E(h);
  const size_t hb = sizeof(hipIpcMemHandle_t);
  const auto* base = reinterpret_cast<const uint8_t*>(handles);
  const int W = e->world, me = e->rank;
  for (int p = 0; p < W; ++p) {
    if (p == me) continue;
    const bool out = e->cap[me * W + p] > 0, in = e->cap[p * W + me] > 0;
    if (!out && !in) continue;
    uint8_t* pmail = nullptr;
    uint64_t* pflags = nullptr;
    if (out) {
      hipIpcMemHandle_t mh;
      std::memcpy(&mh, base + (size_t)p * 2 * hb, hb);
      void* ptr = nullptr;
      const int r = herr(hipIpcOpenMemHandle(&ptr, mh, hipIpcMemLazyEnablePeerAccess));
      if (r) return r;
      e->opened.push_back(ptr);
      pmail = reinterpret_cast<uint8_t*>(ptr);
    }
    if (e->host_flags) {
      uint64_t* hp = map_host_page(page_name(e->shm_prefix, p), e->flag_bytes, false);
      if (hp == nullptr) return -1001;
      e->host_pages[p] = hp;
      pflags = dev_addr(hp);
      if (pflags == nullptr) return -1002;
    } else {
      hipIpcMemHandle_t fh;
      std::memcpy(&fh, base + (size_t)p * 2 * hb + hb, hb);
      void* ptr = nullptr;
      const int r = herr(hipIpcOpenMemHandle(&ptr, fh, hipIpcMemLazyEnablePeerAccess));
      if (r) return r;
      e->opened.push_back(ptr);
      pflags = reinterpret_cast<uint64_t*>(ptr);
    }
    Edge& g = e->edge[p];
    if (out) {
      g.out_bytes = e->cap[me * W + p];
      g.peer_mailbox = pmail + mailbox_off(e, p, me);
      g.peer_ready = pflags + ready_word(me);
      g.my_free = e->flags_dev + free_word(e, p);
    }
    if (in) {
      g.in_bytes = e->cap[p * W + me];
      g.my_mailbox = e->mailbox + mailbox_off(e, me, p);
      g.my_ready = e->flags_dev + ready_word(p);
      g.peer_free = pflags + free_word(e, me);
    }
  }
  return 0;
}

// One exchange, enqueued on `stream`: every send, then every receive (see the protocol at
// the top). A message larger than its edge's mailbox is refused (-1003) before anything is
// enqueued; a zero-byte message still hands the mailbox over once (header only).
int dli_ipc_exchange(void* h, void* stream, int n_send, void* const* send_ptrs,
                     const long long* send_bytes, const int* send_peers, int n_recv,
                     void* const* recv_ptrs, const long long* recv_bytes,
                     const int* recv_peers) {
  auto* e = E(h);
  auto s = (hipStream_t)stream;
  for (int i = 0; i < n_send; ++i) {
    const Edge& g = e->edge[send_peers[i]];
    if (g.peer_ready == nullptr || send_bytes[i] > g.out_bytes) return -1003;
    if ((uintptr_t)send_ptrs[i] % 4 || send_bytes[i] % 4) return -1007;
  }
  for (int i = 0; i < n_recv; ++i) {
    const Edge& g = e->edge[recv_peers[i]];
    if (g.my_ready == nullptr || recv_bytes[i] > g.in_bytes) return -1003;
    if ((uintptr_t)recv_ptrs[i] % 4 || recv_bytes[i] % 4) return -1007;
  }
  int r = 0;
  for (int i = 0; i < n_send && r == 0; ++i) {
    const int p = send_peers[i];
    const Edge& g = e->edge[p];
    const long long nb = send_bytes[i];
    const int vec = (uintptr_t)send_ptrs[i] % 16 == 0;
    r = wait_flag(e, s, g.my_free);
    if (!r) {
      ipc_put_kernel<<<blocks_for(vec ? nb / 16 : nb / 64), 256, 0, s>>>(
          g.peer_mailbox, reinterpret_cast<const uint8_t*>(send_ptrs[i]), nb, vec, e->seq + p,
          e->err);
      r = herr(hipGetLastError());
    }
    if (!r) r = signal_flag(e, s, g.peer_ready);
    e->sends++;
    e->bytes_out += (uint64_t)nb;
  }
  for (int i = 0; i < n_recv && r == 0; ++i) {
    const int p = recv_peers[i];
    const Edge& g = e->edge[p];
    const long long nb = recv_bytes[i];
    const int vec = (uintptr_t)recv_ptrs[i] % 16 == 0;
    r = wait_flag(e, s, g.my_ready);
    if (!r) {
      ipc_get_kernel<<<blocks_for(vec ? nb / 16 : nb / 64), 256, 0, s>>>(
          reinterpret_cast<uint8_t*>(recv_ptrs[i]), g.my_mailbox, nb, vec,
          e->seq + e->world + p, e->err);
      r = herr(hipGetLastError());
    }
    if (!r) r = signal_flag(e, s, g.peer_free);
    e->recvs++;
  }
  return r;
}

// Expert-parallel dispatch (ret = 0) or return (ret = 1) over the mailboxes, enqueued on
// `stream`. Rows are row_bytes long (a multiple of 16).
//   dispatch: the rows for peer p are send_x + send_base[p] rows (count on the device at
//     send_cnt[p], global expert ids at send_e + send_base[p]); the rows from source q land
//     in recv_x + recv_base[q] rows (region capacity recv_cap[q]; ids -> recv_e +
//     recv_base[q], -1 past the count; count -> recv_cnt[q] on the device).
//   return: the roles swap: the recv_cnt[q] result rows at recv_x + recv_base[q] go back to
//     q, and peer p's results for my rows land at send_x + send_base[p] (no ids), at most
//     send_cap rows per peer.
// cap_rows[p] / in_cap_rows[q]: capacity in rows of the mailbox of edge me -> p / q -> me
// (sized by the caller with dli_ipc_ep_bytes). Every received count is clamped to the
// region it lands in; an over-long message raises the sequence error bit.
int dli_ipc_ep(void* h, void* stream, int ret, int row_bytes, void* send_x, int* send_e,
               const int* send_base, int* send_cnt, void* recv_x, int* recv_e,
               const int* recv_base, const int* recv_cap, int* recv_cnt, const int* cap_rows,
               const int* in_cap_rows, int send_cap) {
  auto* e = E(h);
  auto s = (hipStream_t)stream;
  const int W = e->world, me = e->rank;
  const int row16 = row_bytes / 16;
  if (row_bytes % 16) return -1006;
  auto ep_bytes = [&](long cap) { return 16 + (cap * 4 + 15) / 16 * 16 + cap * row_bytes; };
  for (int p = 0; p < W; ++p) {
    if (p == me) continue;
    const Edge& g = e->edge[p];
    if (g.peer_mailbox == nullptr || g.my_mailbox == nullptr) return -1003;
    if (ep_bytes(cap_rows[p]) > g.out_bytes || ep_bytes(in_cap_rows[p]) > g.in_bytes)
      return -1003;
  }
  auto blocks = [&](long rows) { return blocks_for(rows * row16); };
  uint64_t* seq_out = e->seq;
  uint64_t* seq_in = e->seq + W;
  auto* sx = reinterpret_cast<uint8_t*>(send_x);
  auto* rx = reinterpret_cast<uint8_t*>(recv_x);
  const long rb = row_bytes;
  int r = 0;
  if (!ret) {
    for (int p = 0; p < W && r == 0; ++p) {
      if (p == me) continue;
      const Edge& g = e->edge[p];
      r = wait_flag(e, s, g.my_free);
      if (r) break;
      ep_put_kernel<<<blocks(cap_rows[p]), 256, 0, s>>>(
          g.peer_mailbox, cap_rows[p], send_cnt + p,
          reinterpret_cast<const uint4*>(sx + (long)send_base[p] * rb), row16,
          send_e + send_base[p], seq_out + p, e->err);
      r = herr(hipGetLastError());
      if (!r) r = signal_flag(e, s, g.peer_ready);
      e->sends++;
    }
    if (r == 0) {
      ep_local_kernel<<<blocks(recv_cap[me]), 256, 0, s>>>(
          send_cnt + me, reinterpret_cast<const uint4*>(sx + (long)send_base[me] * rb), row16,
          send_e + send_base[me], reinterpret_cast<uint4*>(rx + (long)recv_base[me] * rb),
          recv_e + recv_base[me], recv_cap[me], recv_cap[me], recv_cnt + me);
      r = herr(hipGetLastError());
    }
    for (int q = 0; q < W && r == 0; ++q) {
      if (q == me) continue;
      const Edge& g = e->edge[q];
      r = wait_flag(e, s, g.my_ready);
      if (r) break;
      ep_get_kernel<<<blocks(recv_cap[q]), 256, 0, s>>>(
          g.my_mailbox, in_cap_rows[q], reinterpret_cast<uint4*>(rx + (long)recv_base[q] * rb),
          row16, recv_e + recv_base[q], recv_cap[q], recv_cap[q], recv_cnt + q, seq_in + q,
          e->err);
      r = herr(hipGetLastError());
      if (!r) r = signal_flag(e, s, g.peer_free);
      e->recvs++;
    }
    return r;
  }
  for (int q = 0; q < W && r == 0; ++q) {
    if (q == me) continue;
    const Edge& g = e->edge[q];
    r = wait_flag(e, s, g.my_free);
    if (r) break;
    ep_put_kernel<<<blocks(recv_cap[q]), 256, 0, s>>>(
        g.peer_mailbox, cap_rows[q], recv_cnt + q,
        reinterpret_cast<const uint4*>(rx + (long)recv_base[q] * rb), row16, nullptr,
        seq_out + q, e->err);
    r = herr(hipGetLastError());
    if (!r) r = signal_flag(e, s, g.peer_ready);
    e->sends++;
  }
  if (r == 0) {
    ep_local_kernel<<<blocks(recv_cap[me]), 256, 0, s>>>(
        recv_cnt + me, reinterpret_cast<const uint4*>(rx + (long)recv_base[me] * rb), row16,
        nullptr, reinterpret_cast<uint4*>(sx + (long)send_base[me] * rb), nullptr, 0, send_cap,
        nullptr);
    r = herr(hipGetLastError());
  }
  for (int p = 0; p < W && r == 0; ++p) {
    if (p == me) continue;
    const Edge& g = e->edge[p];
    r = wait_flag(e, s, g.my_ready);
    if (r) break;
    ep_get_kernel<<<blocks(in_cap_rows[p]), 256, 0, s>>>(
        g.my_mailbox, in_cap_rows[p], reinterpret_cast<uint4*>(sx + (long)send_base[p] * rb),
        row16, nullptr, 0, send_cap, nullptr, seq_in + p, e->err);
    r = herr(hipGetLastError());
    if (!r) r = signal_flag(e, s, g.peer_free);
    e->recvs++;
  }
  return r;
}

// Mailbox payload bytes an expert-parallel edge of `cap_rows` rows needs.
long long dli_ipc_ep_bytes(int cap_rows, int row_bytes) {
  return 16 + ((long long)cap_rows * 4 + 15) / 16 * 16 + (long long)cap_rows * row_bytes;
}

// Host flag mode: 1 when a message from `peer` sits in my mailbox, not yet taken by my queue
// (a host-side progress probe); -1 in device-flag mode.
long long dli_ipc_pending(void* h, int peer) {
  auto* e = E(h);
  if (!e->host_flags) return -1;
  return (long long)reinterpret_cast<std::atomic<uint64_t>*>(e->flags + ready_word(peer))
      ->load(std::memory_order_acquire);
}

// Release whatever this rank's queue waits on (a dead peer): set every READY and FREE word
// of this rank to 1 and the error mirror to "aborted", so every wait kernel already queued
// returns at once and no further signal is sent (sticky). A stream-op wait (DLI_IPC_SYNC=
// stream) resets its word after each wait, so a caller draining such a stream repeats this
// until the stream is idle. Host flags: CPU stores. Device flags: an H2D copy of the pattern
// on the endpoint's own non-blocking stream (a DMA queue, not the blocked compute queue),
// polled for up to timeout_s; -1004 when it did not complete.
int dli_ipc_abort(void* h, double timeout_s) {
  auto* e = E(h);
  const size_t n = 2 * (size_t)e->world;
  e->host_sticky.fetch_or(kErrAbort, std::memory_order_release);
  reinterpret_cast<std::atomic<uint64_t>*>(e->err_host)->fetch_or(kErrAbort);
  if (e->host_flags) {
    for (size_t i = 0; i < n; ++i) set_word(e->flags + i * kFlagStride, 1);
    set_word(e->flags + err_word(e), kErrAbort);
    return 0;
  }
  if (e->abort_stream == nullptr) return -1005;
  int r = herr(hipMemcpyAsync(e->flags, e->abort_src, e->flag_bytes, hipMemcpyHostToDevice,
                              e->abort_stream));
  if (r) return r;
  const auto t0 = std::chrono::steady_clock::now();
  while (hipStreamQuery(e->abort_stream) == hipErrorNotReady) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      return -1004;
    usleep(200);
  }
  return 0;
}

// The error bits (kErrWait | kErrSeq | kErrAbort) set so far: one load of a pinned host word,
// cheap enough to poll every pipeline tick.
int dli_ipc_error(void* h) {
  auto* e = E(h);
  return (int)(reinterpret_cast<std::atomic<uint64_t>*>(e->err_host)->load(
                   std::memory_order_acquire) |
               e->host_sticky.load(std::memory_order_acquire));
}

// Bounded-wait budget in seconds (wait kernels enqueued after the call).
void dli_ipc_set_wait(void* h, double secs) {
  auto* e = E(h);
  e->wait_budget = (unsigned long long)(secs * 1000.0 * (double)e->khz);
}

// Test hook: advance this rank's outbound sequence counter for `peer` by `d` on `stream`, so
// the next message on that edge carries a wrong sequence number (the receiver must flag it).
int dli_ipc_debug_bump_seq(void* h, void* stream, int peer, long long d) {
  auto* e = E(h);
  if (peer < 0 || peer >= e->world) return -1;
  ipc_bump_kernel<<<1, 64, 0, (hipStream_t)stream>>>(e->seq + peer, (uint64_t)d);
  return herr(hipGetLastError());
}

// 0 coarse-grained, 1 fine-grained, 2 uncached: the allocation the mailboxes use
int dli_ipc_mem_kind(void* h) { return E(h)->mem_kind; }

void dli_ipc_stats(void* h, long long* out3) {
  auto* e = E(h);
  out3[0] = (long long)e->sends;
  out3[1] = (long long)e->recvs;
  out3[2] = (long long)e->bytes_out;
}

int dli_ipc_host_flags(void* h) { return E(h)->host_flags ? 1 : 0; }

void dli_ipc_destroy(void* h) {
  auto* e = E(h);
  if (e == nullptr) return;
  for (void* p : e->opened) (void)hipIpcCloseMemHandle(p);
  if (e->host_flags) {
    for (auto* p : e->host_pages) {
      if (p == nullptr) continue;
      (void)hipHostUnregister(p);
      munmap(p, e->flag_bytes);
    }
    shm_unlink(page_name(e->shm_prefix, e->rank).c_str());
  } else if (e->flags) {
    (void)hipFree(e->flags);
  }
  if (e->abort_stream) (void)hipStreamDestroy(e->abort_stream);
  if (e->abort_src) (void)hipHostFree(e->abort_src);
  if (e->mailbox) (void)hipFree(e->mailbox);
  if (e->seq) (void)hipFree(e->seq);
  if (e->err_host) (void)hipHostFree(e->err_host);
  delete e;
}

}  // extern "C"
