// Safetensors shard loader: mmap -> pinned staging ring -> hipMemcpyAsync into HBM.
//
// The reference worker loads whole HF checkpoints with `from_pretrained` then `.to(DEVICE)`
// (worker/app.py:121-124). Here each pipeline stage reads only its own per-stage shard file
// (shard/writer.py) and streams tensors straight into pre-allocated device buffers: the file
// is memory-mapped, copied in 32 MiB pieces into a ring of pinned host buffers
// (hipHostMalloc) and pushed with hipMemcpyAsync on the caller's stream; a ring slot is
// reused only after the event recorded behind its copy has completed, so host memcpy and
// DMA overlap. No tensor is ever materialised twice in host RAM.
//
// C ABI for ctypes; returns >= 0 on success.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct TensorInfo {
  std::string name, dtype;
  std::vector<long long> shape;
  long long begin = 0, end = 0;
};

struct StFile {
  int fd = -1;
  size_t size = 0;
  const uint8_t* map = nullptr;
  size_t data_off = 0;
  std::vector<TensorInfo> tensors;
};

// ---- minimal JSON reader for the safetensors header --------------------------------------
struct Json {
  const char* p;
  const char* e;
  void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
  bool eat(char c) { ws(); if (p < e && *p == c) { ++p; return true; } return false; }
  bool str(std::string& out) {
    ws();
    if (p >= e || *p != '"') return false;
    ++p;
    out.clear();
    while (p < e && *p != '"') {
      if (*p == '\\' && p + 1 < e) { out.push_back(p[1]); p += 2; continue; }
      out.push_back(*p++);
    }
    if (p >= e) return false;
    ++p;
    return true;
  }
  bool num(long long& v) {  // bounded: the header is not NUL-terminated
    ws();
    const char* q = p;
    bool neg = false;
    if (q < e && *q == '-') { neg = true; ++q; }
    if (q >= e || *q < '0' || *q > '9') return false;
    unsigned long long acc = 0;
    for (; q < e && *q >= '0' && *q <= '9'; ++q) {
      if (acc > (1ull << 62)) return false;       // absurd value: reject, never overflow
      acc = acc * 10 + (unsigned)(*q - '0');
    }
    v = neg ? -(long long)acc : (long long)acc;
    p = q;
    return true;
  }
  bool skip() {  // skip any value
    ws();
    if (p >= e) return false;
    if (*p == '"') { std::string s; return str(s); }
    if (*p == '{' || *p == '[') {
      const char open = *p, close = open == '{' ? '}' : ']';
      int depth = 0;
      bool in_str = false;
      for (; p < e; ++p) {
        if (in_str) { if (*p == '\\') ++p; else if (*p == '"') in_str = false; continue; }
        if (*p == '"') in_str = true;
        else if (*p == open) ++depth;
        else if (*p == close && --depth == 0) { ++p; return true; }
      }
      return false;
    }
    while (p < e && *p != ',' && *p != '}' && *p != ']') ++p;
    return true;
  }
};

bool parse_header(StFile& f, const char* js, size_t n) {
  Json j{js, js + n};
  if (!j.eat('{')) return false;
  if (j.eat('}')) return true;
  do {
    std::string key;
    if (!j.str(key) || !j.eat(':')) return false;
    if (key == "__metadata__") { if (!j.skip()) return false; continue; }
    TensorInfo t;
    t.name = key;
    if (!j.eat('{')) return false;
    do {
      std::string k;
      if (!j.str(k) || !j.eat(':')) return false;
      if (k == "dtype") {
        if (!j.str(t.dtype)) return false;
      } else if (k == "shape") {
        if (!j.eat('[')) return false;
        if (!j.eat(']')) {
          do { long long v; if (!j.num(v)) return false; t.shape.push_back(v); } while (j.eat(','));
          if (!j.eat(']')) return false;
        }
      } else if (k == "data_offsets") {
        if (!j.eat('[') || !j.num(t.begin) || !j.eat(',') || !j.num(t.end) || !j.eat(']'))
          return false;
      } else if (!j.skip()) {
        return false;
      }
    } while (j.eat(','));
    if (!j.eat('}')) return false;
    f.tensors.push_back(std::move(t));
  } while (j.eat(','));
  return j.eat('}');
}

constexpr size_t kPiece = 32ull << 20;
constexpr int kRing = 3;

struct Staging {
  void* buf[kRing] = {nullptr, nullptr, nullptr};
  hipEvent_t ev[kRing];
  bool used[kRing] = {false, false, false};
  int next = 0;
  bool ok = false;
  Staging() {
    ok = true;
    for (int i = 0; i < kRing; ++i) {
      if (hipHostMalloc(&buf[i], kPiece, hipHostMallocDefault) != hipSuccess) ok = false;
      if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) ok = false;
    }
  }
  ~Staging() {
    for (int i = 0; i < kRing; ++i) {
      if (used[i]) hipEventSynchronize(ev[i]);
      if (buf[i]) hipHostFree(buf[i]);
      hipEventDestroy(ev[i]);
    }
  }
};

inline StFile* H(void* h) { return reinterpret_cast<StFile*>(h); }

}  // namespace

extern "C" {

void* dli_st_open(const char* path) {
  auto* f = new StFile();
  f->fd = open(path, O_RDONLY);
  if (f->fd < 0) { delete f; return nullptr; }
  struct stat sb;
  if (fstat(f->fd, &sb) != 0 || sb.st_size < 8) { close(f->fd); delete f; return nullptr; }
  f->size = (size_t)sb.st_size;
  void* m = mmap(nullptr, f->size, PROT_READ, MAP_PRIVATE, f->fd, 0);
  if (m == MAP_FAILED) { close(f->fd); delete f; return nullptr; }
  f->map = (const uint8_t*)m;
  uint64_t hlen = 0;
  std::memcpy(&hlen, f->map, 8);
  bool ok = hlen <= f->size - 8 && parse_header(*f, (const char*)f->map + 8, hlen);
  if (ok) {
    f->data_off = 8 + hlen;
    const long long avail = (long long)(f->size - f->data_off);
    for (const auto& t : f->tensors)            // every tensor must lie inside the file
      if (t.begin < 0 || t.end < t.begin || t.end > avail) { ok = false; break; }
  }
  if (!ok) {
    munmap((void*)f->map, f->size); close(f->fd); delete f; return nullptr;
  }
  return f;
}

void dli_st_close(void* h) {
  auto* f = H(h);
  if (!f) return;
  if (f->map) munmap((void*)f->map, f->size);
  if (f->fd >= 0) close(f->fd);
  delete f;
}

int dli_st_count(void* h) { return (int)H(h)->tensors.size(); }

int dli_st_info(void* h, int i, char* name, int name_cap, char* dtype, int dtype_cap,
                long long* shape, int* ndim, long long* nbytes) {
  auto* f = H(h);
  if (i < 0 || i >= (int)f->tensors.size()) return -1;
  const auto& t = f->tensors[i];
  snprintf(name, name_cap, "%s", t.name.c_str());
  snprintf(dtype, dtype_cap, "%s", t.dtype.c_str());
  const int nd = (int)t.shape.size();
  for (int d = 0; d < nd && d < 8; ++d) shape[d] = t.shape[d];
  *ndim = nd;
  *nbytes = t.end - t.begin;
  return 0;
}

int dli_st_find(void* h, const char* name) {
  auto* f = H(h);
  for (size_t i = 0; i < f->tensors.size(); ++i)
    if (f->tensors[i].name == name) return (int)i;
  return -1;
}

int dli_st_copy_to_host(void* h, int i, void* dst) {
  auto* f = H(h);
  if (i < 0 || i >= (int)f->tensors.size()) return -1;
  const auto& t = f->tensors[i];
  std::memcpy(dst, f->map + f->data_off + t.begin, (size_t)(t.end - t.begin));
  return 0;
}

// Streams tensors idx[0..n) into dsts[0..n) (device pointers) on `stream`.
// Returns total bytes, or -(hip error) on failure. Waits for its own staging before return.
long long dli_st_load_to_device(void* h, const int* idx, void* const* dsts, int n,
                                hipStream_t stream) {
  auto* f = H(h);
  Staging s;
  if (!s.ok) return -1;
  long long total = 0;
  for (int k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= (int)f->tensors.size()) return -2;
    const auto& t = f->tensors[idx[k]];
    const uint8_t* src = f->map + f->data_off + t.begin;
    uint8_t* dst = (uint8_t*)dsts[k];
    size_t left = (size_t)(t.end - t.begin), off = 0;
    while (left > 0) {
      const size_t piece = left < kPiece ? left : kPiece;
      const int slot = s.next;
      s.next = (s.next + 1) % kRing;
      if (s.used[slot]) {
        hipError_t e = hipEventSynchronize(s.ev[slot]);
        if (e != hipSuccess) return -(long long)e;
      }
      std::memcpy(s.buf[slot], src + off, piece);
      hipError_t e = hipMemcpyAsync(dst + off, s.buf[slot], piece, hipMemcpyHostToDevice, stream);
      if (e != hipSuccess) return -(long long)e;
      e = hipEventRecord(s.ev[slot], stream);
      if (e != hipSuccess) return -(long long)e;
      s.used[slot] = true;
      off += piece;
      left -= piece;
      total += (long long)piece;
    }
  }
  for (int i = 0; i < kRing; ++i)
    if (s.used[i]) hipEventSynchronize(s.ev[i]);
  for (int i = 0; i < kRing; ++i) s.used[i] = false;
  return total;
}

// Bytes [byte_off, byte_off + nbytes) of tensor i into dst (a row range of a row-major
// tensor, e.g. one rank's vocabulary slice of the LM head): device = 1 streams through the
// pinned ring with hipMemcpyAsync on `stream`, device = 0 is a host memcpy.
long long dli_st_load_range(void* h, int i, long long byte_off, long long nbytes, void* dst,
                            hipStream_t stream, int device) {
  auto* f = H(h);
  if (i < 0 || i >= (int)f->tensors.size()) return -2;
  const auto& t = f->tensors[i];
  if (byte_off < 0 || nbytes < 0 || byte_off + nbytes > t.end - t.begin) return -3;
  const uint8_t* src = f->map + f->data_off + t.begin + byte_off;
  if (!device) {
    std::memcpy(dst, src, (size_t)nbytes);
    return nbytes;
  }
  Staging s;
  if (!s.ok) return -1;
  size_t left = (size_t)nbytes, off = 0;
  while (left > 0) {
    const size_t piece = left < kPiece ? left : kPiece;
    const int slot = s.next;
    s.next = (s.next + 1) % kRing;
    if (s.used[slot]) {
      hipError_t e = hipEventSynchronize(s.ev[slot]);
      if (e != hipSuccess) return -(long long)e;
    }
    std::memcpy(s.buf[slot], src + off, piece);
    hipError_t e = hipMemcpyAsync((uint8_t*)dst + off, s.buf[slot], piece, hipMemcpyHostToDevice,
                                  stream);
    if (e != hipSuccess) return -(long long)e;
    e = hipEventRecord(s.ev[slot], stream);
    if (e != hipSuccess) return -(long long)e;
    s.used[slot] = true;
    off += piece;
    left -= piece;
  }
  for (int k = 0; k < kRing; ++k)
    if (s.used[k]) hipEventSynchronize(s.ev[k]);
  for (int k = 0; k < kRing; ++k) s.used[k] = false;
  return nbytes;
}

}  // extern "C"
