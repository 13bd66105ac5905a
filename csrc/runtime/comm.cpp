// RCCL point-to-point for the pipeline data plane, called directly ("RCCL ...
// called directly from a C++ comm module"; the reference has no data plane at all — its
// "shards" exchange nothing, master/dashboard/views.py:318-355).
//
// One communicator per pipeline (ranks = stages). Sends and receives of a tick are enqueued
// inside one ncclGroupStart/End on the CALLER's stream — the stage's compute stream — so the
// transfer is ordered after the kernels that produced the send buffer and before the ones
// that read the receive buffer with no events, no side stream and no host wait (torch's
// process-group path runs them on a separate RCCL stream and joins it with an event).
//
// The RCCL entry points are resolved at run time from the librccl.so.1 already mapped into
// the process (torch links it), so the pipeline and torch.distributed share ONE RCCL
// instance; a process without it loaded falls back to dlopen by name.
//
// C ABI (ctypes): >= 0 on success; a negative value is -(ncclResult_t) or -100 when RCCL
// could not be loaded.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) =
      nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};

RcclApi* api() {
  static RcclApi a;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);   // torch's instance
    if (h == nullptr) h = dlopen("librccl.so.1", RTLD_NOW);
    if (h == nullptr) h = dlopen("librccl.so", RTLD_NOW);
    if (h == nullptr) return;
    auto sym = [h](const char* n) { return dlsym(h, n); };
    a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(sym("ncclGetUniqueId"));
    a.comm_init_rank = reinterpret_cast<decltype(a.comm_init_rank)>(sym("ncclCommInitRank"));
    a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(sym("ncclCommDestroy"));
    a.comm_abort = reinterpret_cast<decltype(a.comm_abort)>(sym("ncclCommAbort"));
    a.async_error =
        reinterpret_cast<decltype(a.async_error)>(sym("ncclCommGetAsyncError"));
    a.send = reinterpret_cast<decltype(a.send)>(sym("ncclSend"));
    a.recv = reinterpret_cast<decltype(a.recv)>(sym("ncclRecv"));
    a.group_start = reinterpret_cast<decltype(a.group_start)>(sym("ncclGroupStart"));
    a.group_end = reinterpret_cast<decltype(a.group_end)>(sym("ncclGroupEnd"));
    a.error_string = reinterpret_cast<decltype(a.error_string)>(sym("ncclGetErrorString"));
    a.ok = a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.send && a.recv &&
           a.group_start && a.group_end;
  });
  return &a;
}

inline int rc(ncclResult_t r) { return r == ncclSuccess ? 0 : -(int)r; }

}  // namespace

extern "C" {

int dli_comm_available() { return api()->ok ? 1 : 0; }

const char* dli_comm_error_string(int code) {
  auto* a = api();
  if (!a->ok || a->error_string == nullptr) return "RCCL not loaded";
  return a->error_string((ncclResult_t)(code < 0 ? -code : code));
}

// 128-byte unique id of a new communicator (rank 0 creates it and ships it to the others).
int dli_comm_unique_id(void* out_id) {
  auto* a = api();
  if (!a->ok) return -100;
  ncclUniqueId id;
  const int r = rc(a->get_unique_id(&id));
  if (r == 0) std::memcpy(out_id, &id, sizeof(id));
  return r;
}

int dli_comm_id_bytes() { return (int)sizeof(ncclUniqueId); }

// Collective over all `nranks` processes (each on its own current HIP device).
int dli_comm_init(void** out_comm, const void* id_bytes, int nranks, int rank) {
  auto* a = api();
  if (!a->ok) return -100;
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  ncclComm_t c = nullptr;
  const int r = rc(a->comm_init_rank(&c, nranks, id, rank));
  *out_comm = r == 0 ? (void*)c : nullptr;
  return r;
}

int dli_comm_destroy(void* comm) {
  auto* a = api();
  if (!a->ok || comm == nullptr) return 0;
  return rc(a->comm_destroy((ncclComm_t)comm));
}

// Failure handling ("RCCL async-error polling (ncclCommGetAsyncError) with
// communicator abort + rebuild"). dli_comm_async_error: 0 healthy, else -(ncclResult_t) of
// the communicator's asynchronous error (a peer died, a network / xGMI fault). The pipeline
// watchdog polls it next to the stage liveness probe. dli_comm_abort: ncclCommAbort — frees
// the communicator WITHOUT waiting for the peers and makes its kernels still queued on a
// stream return, so a stage blocked on a dead neighbour drains; a new communicator is then
// built for the re-formed ring.
int dli_comm_async_error(void* comm) {
  auto* a = api();
  if (!a->ok || comm == nullptr || a->async_error == nullptr) return 0;
  ncclResult_t e = ncclSuccess;
  const int r = rc(a->async_error((ncclComm_t)comm, &e));
  return r != 0 ? r : rc(e);
}

int dli_comm_abort(void* comm) {
  auto* a = api();
  if (!a->ok || comm == nullptr) return 0;
  if (a->comm_abort == nullptr) return -100;
  return rc(a->comm_abort((ncclComm_t)comm));
}

// One tick's exchange: n_send buffers to their peers and n_recv buffers from theirs, grouped
// (deadlock-free in any order across ranks) and enqueued on `stream`.
int dli_comm_exchange(void* comm, void* stream, int n_send, void* const* send_ptrs,
                      const long long* send_bytes, const int* send_peers, int n_recv,
                      void* const* recv_ptrs, const long long* recv_bytes,
                      const int* recv_peers) {
  auto* a = api();
  if (!a->ok) return -100;
  auto c = (ncclComm_t)comm;
  auto s = (hipStream_t)stream;
  int r = rc(a->group_start());
  if (r != 0) return r;
  for (int i = 0; i < n_send && r == 0; ++i)
    r = rc(a->send(send_ptrs[i], (size_t)send_bytes[i], ncclUint8, send_peers[i], c, s));
  for (int i = 0; i < n_recv && r == 0; ++i)
    r = rc(a->recv(recv_ptrs[i], (size_t)recv_bytes[i], ncclUint8, recv_peers[i], c, s));
  const int e = rc(a->group_end());
  return r != 0 ? r : e;
}

}  // extern "C"
