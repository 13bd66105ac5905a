// Continuous-batching scheduler core (host C++): one microbatch's running sequences as a
// struct-of-arrays mirror, and the two per-tick operations of the decode fast path
//
//   schedule: allocate KV blocks for every row's new token, then write the step's packed
//             metadata (the pipeline control-plane wire format of engine/batch.py
//             StepMeta.pack: seq ids | input ids | positions | slots | seq lens | context
//             lens | block tables trimmed to the widest | temperature | top-k | top-p |
//             64-bit Philox seeds) straight into one int32 buffer;
//   update:   apply the sampled tokens (history, last id, context, output count) and report
//             the rows that finished (length budget, model length, EOS).
//
// The reference worker served one request at a time (gunicorn sync worker,
// worker/Dockerfile:45); here the pipeline head schedules 512-row microbatches every tick of
// a ~1 ms decode step, so this path must cost tens of microseconds, not the ~0.5 ms of the
// equivalent numpy code. Python (engine/scheduler.py) keeps the Sequence objects and the
// rare paths (admission, preemption, stop tokens, lookahead).
//
// C ABI for ctypes.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

extern "C" int dli_bm_decode_prepare(void* h, const long long* seqs, const int* ctx, int n,
                                     int* slots, int* tables, int max_blocks);

namespace {

struct MB {
  int n = 0;
  std::vector<long long> sid, seed;
  std::vector<int> ctx, out_cnt, budget, last, topk;
  std::vector<float> temp, topp;
  std::vector<unsigned char> eos_ok;
  std::vector<int> hist;           // n x cap, tokens generated since the mirror was built
  int cap = 0, k = 0;
  int eos = -1, max_model_len = 0;
  std::vector<int> slots_tmp, tables_tmp;
};

inline MB* H(void* h) { return reinterpret_cast<MB*>(h); }

inline uint64_t splitmix_row_seed(long long seq_seed, long long index) {
  // == sequence.row_seed / scheduler.row_seeds (splitmix64 of (seed, output index))
  uint64_t z = (uint64_t)seq_seed * 0x9E3779B97F4A7C15ull + (uint64_t)index +
               0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace

extern "C" {

void* dli_mb_create(int n, const long long* sid, const int* ctx, const int* out_cnt,
                    const int* budget, const int* last, const float* temp, const int* topk,
                    const float* topp, const long long* seed, const unsigned char* eos_ok,
                    int eos, int max_model_len, int hist_cap) {
  if (n < 0) return nullptr;
  auto* m = new MB();
  m->n = n;
  m->sid.assign(sid, sid + n);
  m->seed.assign(seed, seed + n);
  m->ctx.assign(ctx, ctx + n);
  m->out_cnt.assign(out_cnt, out_cnt + n);
  m->budget.assign(budget, budget + n);
  m->last.assign(last, last + n);
  m->topk.assign(topk, topk + n);
  m->temp.assign(temp, temp + n);
  m->topp.assign(topp, topp + n);
  m->eos_ok.assign(eos_ok, eos_ok + n);
  m->cap = std::max(1, hist_cap);
  m->hist.assign((size_t)n * m->cap, 0);
  m->eos = eos;
  m->max_model_len = max_model_len;
  return m;
}

void dli_mb_destroy(void* h) { delete H(h); }

int dli_mb_rows(void* h) { return H(h)->n; }
int dli_mb_steps(void* h) { return H(h)->k; }

// Words of the packed payload for a given table width.
long long dli_mb_payload_words(void* h, int table_cols) {
  const long long S = H(h)->n;
  return S + 3 * S + 2 * S + S * (long long)table_cols + 3 * S + 2 * S;
}

// Decode step for every row. Returns payload words written (*out_cols = table columns on the
// wire), -(i + 1) if row i could not get a KV block (caller preempts and retries), or
// -(n + 1) if a table exceeds table_width / the payload does not fit.
long long dli_mb_schedule(void* h, void* bm, int table_width, int* payload,
                          long long cap_words, int* out_cols) {
  auto* m = H(h);
  const int S = m->n;
  if (S == 0) { *out_cols = 0; return 0; }
  m->slots_tmp.resize(S);
  m->tables_tmp.resize((size_t)S * table_width);
  const int widest = dli_bm_decode_prepare(bm, m->sid.data(), m->ctx.data(), S,
                                           m->slots_tmp.data(), m->tables_tmp.data(),
                                           table_width);
  if (widest < 0) return widest;
  const int cols = std::max(1, widest);
  const long long words = dli_mb_payload_words(h, cols);
  if (words > cap_words) return -(S + 1);
  int* o = payload;
  for (int i = 0; i < S; ++i) o[i] = (int)m->sid[i];
  o += S;
  std::memcpy(o, m->last.data(), sizeof(int) * S);                        // input ids
  o += S;
  for (int i = 0; i < S; ++i) o[i] = m->ctx[i] - 1;                       // positions
  o += S;
  std::memcpy(o, m->slots_tmp.data(), sizeof(int) * S);                   // slots
  o += S;
  for (int i = 0; i < S; ++i) o[i] = 1;                                   // seq lens
  o += S;
  std::memcpy(o, m->ctx.data(), sizeof(int) * S);                         // context lens
  o += S;
  for (int i = 0; i < S; ++i)                                             // tables
    std::memcpy(o + (size_t)i * cols, m->tables_tmp.data() + (size_t)i * table_width,
                sizeof(int) * cols);
  o += (size_t)S * cols;
  std::memcpy(o, m->temp.data(), sizeof(float) * S);
  o += S;
  std::memcpy(o, m->topk.data(), sizeof(int) * S);
  o += S;
  std::memcpy(o, m->topp.data(), sizeof(float) * S);
  o += S;
  for (int i = 0; i < S; ++i) {
    const uint64_t z = splitmix_row_seed(m->seed[i], m->out_cnt[i]);
    std::memcpy(o + 2 * i, &z, 8);
  }
  *out_cols = cols;
  return words;
}

// Apply one step's tokens (one per row, in row order). Writes the finished rows (ascending)
// to done_idx and their reasons to done_stop (1 = EOS stop, 0 = length) and returns how many.
int dli_mb_update(void* h, const int* tokens, int n, int* done_idx, int* done_stop) {
  auto* m = H(h);
  if (n != m->n) return -1;
  if (m->k >= m->cap) {                          // grow the history (rare: budget estimate)
    const int nc = m->cap * 2;
    std::vector<int> nh((size_t)m->n * nc, 0);
    for (int i = 0; i < m->n; ++i)
      std::memcpy(nh.data() + (size_t)i * nc, m->hist.data() + (size_t)i * m->cap,
                  sizeof(int) * m->k);
    m->hist.swap(nh);
    m->cap = nc;
  }
  int nd = 0;
  for (int i = 0; i < n; ++i) {
    const int t = tokens[i];
    m->hist[(size_t)i * m->cap + m->k] = t;
    m->last[i] = t;
    m->out_cnt[i] += 1;
    m->ctx[i] += 1;
    const bool stop = m->eos_ok[i] && t == m->eos;
    const bool len = m->out_cnt[i] >= m->budget[i] || m->ctx[i] >= m->max_model_len;
    if (stop || len) {
      done_idx[nd] = i;
      done_stop[nd] = stop ? 1 : 0;
      ++nd;
    }
  }
  m->k += 1;
  return nd;
}

// Tokens generated by `row` since the mirror was built (returns the count).
int dli_mb_row_history(void* h, int row, int* out) {
  auto* m = H(h);
  if (row < 0 || row >= m->n) return -1;
  std::memcpy(out, m->hist.data() + (size_t)row * m->cap, sizeof(int) * m->k);
  return m->k;
}

// Whole history [n, k] (row-major) into out; returns k.
int dli_mb_history(void* h, int* out) {
  auto* m = H(h);
  for (int i = 0; i < m->n; ++i)
    std::memcpy(out + (size_t)i * m->k, m->hist.data() + (size_t)i * m->cap,
                sizeof(int) * m->k);
  return m->k;
}

// Remove rows drop[0..nd) (ascending); the remaining rows keep their order.
int dli_mb_compact(void* h, const int* drop, int nd) {
  auto* m = H(h);
  int w = 0, j = 0;
  for (int i = 0; i < m->n; ++i) {
    if (j < nd && drop[j] == i) { ++j; continue; }
    if (w != i) {
      m->sid[w] = m->sid[i]; m->seed[w] = m->seed[i]; m->ctx[w] = m->ctx[i];
      m->out_cnt[w] = m->out_cnt[i]; m->budget[w] = m->budget[i]; m->last[w] = m->last[i];
      m->topk[w] = m->topk[i]; m->temp[w] = m->temp[i]; m->topp[w] = m->topp[i];
      m->eos_ok[w] = m->eos_ok[i];
      std::memcpy(m->hist.data() + (size_t)w * m->cap, m->hist.data() + (size_t)i * m->cap,
                  sizeof(int) * m->k);
    }
    ++w;
  }
  m->n = w;
  return w;
}

}  // extern "C"
