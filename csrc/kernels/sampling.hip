// On-device token sampling with HF `generate` semantics — SURVEY.md §2.4 K13/K14.
//
// HF warper order (transformers/generation/utils.py): Temperature -> TopK -> TopP -> softmax
// -> multinomial. One 512-thread workgroup per row (vocab up to ~256k), no full-vocab sort:
//   * greedy (temperature <= 0 or top_k == 1): block argmax (first index on ties, like torch).
//   * top_k <= 0 and top_p >= 1: exact Gumbel-max sampling over the whole row in one pass.
//   * otherwise: radix select (8-bit digits, early exit) finds the bin holding the k-th
//     largest logit; every element at or above it (<= CAP) is gathered into LDS, bitonic-
//     sorted, cut to the top-k (ties kept, as HF's `scores < kth` mask keeps them), then
//     temperature-softmax, top-p truncation (keep j while the mass of strictly larger tokens
//     < top_p, i.e. HF's `cumsum_asc <= 1-top_p` removal) and an inverse-CDF draw.
// top_k is capped at CAP (2048). Randomness: Philox4x32-10 keyed by a per-row 64-bit seed
// supplied by the engine (seed = f(request seed, output index)), so a request samples the
// same tokens regardless of how it is batched.
#include "common.h"

#define SMP_THREADS 512
#define SMP_CAP 2048

__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Philox4x32-10
__device__ __forceinline__ uint4 philox(uint2 key, uint4 ctr) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0; key.y += W1;
  }
  return ctr;
}
__device__ __forceinline__ float u01(uint32_t x) {           // (0, 1)
  return ((x >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

struct ArgMax { float v; int i; };
__device__ __forceinline__ ArgMax amax(ArgMax a, ArgMax b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}
__device__ ArgMax block_argmax(ArgMax a, float* sv, int* si) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, 64), __shfl_xor(a.i, o, 64)};
    a = amax(a, b);
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) { sv[w] = a.v; si[w] = a.i; }
  __syncthreads();
  ArgMax r{sv[0], si[0]};
  for (int i = 1; i < nw; ++i) r = amax(r, ArgMax{sv[i], si[i]});
  return r;
}

// inclusive block scan of one float per thread (512 threads)
__device__ float block_scan(float v, float* tmp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  __syncthreads();
  if (lane == 63) tmp[w] = v;
  __syncthreads();
  float add = 0.f;
  for (int i = 0; i < w; ++i) add += tmp[i];
  (void)nw;
  return v + add;
}

// Radix-select digit step: the largest bin d whose suffix count S(d) = sum_{b >= d} hist[b]
// reaches k_rem (bins walked from 255 down), as one block scan over the 256 bins instead of
// a serial walk by one thread (up to 256 dependent LDS reads per pass). sel = {digit, count
// strictly above the digit's bin, count in it}; with S(0) < k_rem (fewer than k_rem keys):
// {0, S(0), 0}, so sel[1] + sel[2] < k_rem tells that case apart.
// All threads call it (block_scan barriers).
__device__ __forceinline__ void find_digit(const uint32_t* hist, uint32_t k_rem, float* tmp,
                                           uint32_t* sel) {
  const int tid = threadIdx.x;
  const uint32_t h = tid < 256 ? hist[255 - tid] : 0u;
  const uint32_t S = (uint32_t)block_scan((float)h, tmp);     // exact: counts < 2^24
  if (tid < 256) {
    const bool hit = S >= k_rem && S - h < k_rem;
    if (hit || (tid == 255 && S < k_rem)) {
      sel[0] = 255u - (uint32_t)tid;
      sel[1] = hit ? S - h : S;
      sel[2] = hit ? h : 0u;
    }
  }
}

// k-th largest non-zero key of keys[0..n) (LDS), 8-bit digits. Key 0 (an all-ones NaN
// pattern) marks an empty slot and is never counted. Returns 0 when fewer than k keys exist.
__device__ uint32_t radix_kth(const uint32_t* keys, int n, uint32_t k, uint32_t* hist,
                              float* tmp, uint32_t* sel) {
  uint32_t prefix = 0, pmask = 0, k_rem = k;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int e = threadIdx.x; e < n; e += blockDim.x) {
      const uint32_t key = keys[e];
      if (key != 0u && (key & pmask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    find_digit(hist, k_rem, tmp, sel);
    __syncthreads();
    if (k_rem > sel[1] + sel[2]) return 0u;                    // fewer than k keys
    k_rem -= sel[1];
    prefix |= sel[0] << shift;
    pmask |= 255u << shift;
  }
  return prefix;
}

// Logits arrive as fp32 or as bf16 (u16: the LM head's output in the model dtype, as HF's
// `lm_head(hidden).float()` produces them); every comparison runs on the exact fp32 value.
__device__ __forceinline__ float ldv(const float* x, int i) { return x[i]; }
__device__ __forceinline__ float ldv(const u16* x, int i) { return bf2f(x[i]); }

// Visit every element of a row with 16-B loads, 4 loads in flight per thread (the sampler is
// one workgroup per row, so memory-level parallelism per CU comes from ILP, not occupancy).
template <typename F>
__device__ __forceinline__ void row_scan(const u16* __restrict__ x, int V, F&& f) {
  const int tid = threadIdx.x, nt = blockDim.x;
  int done = 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const int V8 = V >> 3;
    const uint4* x8 = reinterpret_cast<const uint4*>(x);
    auto eight = [&](const uint4 v, int base) {
      f(__uint_as_float(v.x << 16), base);     f(__uint_as_float(v.x & 0xffff0000u), base + 1);
      f(__uint_as_float(v.y << 16), base + 2); f(__uint_as_float(v.y & 0xffff0000u), base + 3);
      f(__uint_as_float(v.z << 16), base + 4); f(__uint_as_float(v.z & 0xffff0000u), base + 5);
      f(__uint_as_float(v.w << 16), base + 6); f(__uint_as_float(v.w & 0xffff0000u), base + 7);
    };
    int i = tid;
    for (; i + 3 * nt < V8; i += 4 * nt) {
      const uint4 a = x8[i], b = x8[i + nt], c = x8[i + 2 * nt], d = x8[i + 3 * nt];
      eight(a, 8 * i); eight(b, 8 * (i + nt)); eight(c, 8 * (i + 2 * nt)); eight(d, 8 * (i + 3 * nt));
    }
    for (; i < V8; i += nt) eight(x8[i], 8 * i);
    done = V8 * 8;
  }
  for (int j = done + tid; j < V; j += nt) f(bf2f(x[j]), j);
}

template <typename F>
__device__ __forceinline__ void row_scan(const float* __restrict__ x, int V, F&& f) {
  const int tid = threadIdx.x, nt = blockDim.x;
  int done = 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const int V4 = V >> 2;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    int i = tid;
    for (; i + 3 * nt < V4; i += 4 * nt) {
      const float4 a = x4[i], b = x4[i + nt], c = x4[i + 2 * nt], d = x4[i + 3 * nt];
      f(a.x, 4 * i); f(a.y, 4 * i + 1); f(a.z, 4 * i + 2); f(a.w, 4 * i + 3);
      const int ib = 4 * (i + nt), ic = 4 * (i + 2 * nt), id = 4 * (i + 3 * nt);
      f(b.x, ib); f(b.y, ib + 1); f(b.z, ib + 2); f(b.w, ib + 3);
      f(c.x, ic); f(c.y, ic + 1); f(c.z, ic + 2); f(c.w, ic + 3);
      f(d.x, id); f(d.y, id + 1); f(d.z, id + 2); f(d.w, id + 3);
    }
    for (; i < V4; i += nt) {
      const float4 a = x4[i];
      f(a.x, 4 * i); f(a.y, 4 * i + 1); f(a.z, 4 * i + 2); f(a.w, 4 * i + 3);
    }
    done = V4 * 4;
  }
  for (int j = done + tid; j < V; j += nt) f(x[j], j);
}

// ---------------------------------------------------------------------------------------
// Small batches (B <= SMP_SPLIT_MAX_B): one workgroup per row leaves ~255 CUs idle while it
// walks a 128k-entry row several times (~45 us at batch 1, profiles/r3/b1_p). Two phases
// instead: sample_chunk_kernel splits each row into P chunks (P workgroups per row); a chunk
// keeps every logit >= its own Keff-th largest (radix select in LDS), in index order, in a
// CAPC-slot candidate list (pads: -inf). The row's top-Keff is contained in the union of the
// chunks' lists, which keep index order, so sample_kernel then runs its unchanged algorithm
// over the P*CAPC candidates (ties still break on the lower vocab index) and maps the pick
// back to a vocab id. Rows whose Keff exceeds CAPC, plain-temperature rows and rows where a
// chunk had more than CAPC ties at its threshold (overflow flag) read the full row as before.
#define SMP_CAPC 64
#define SMP_CHUNK_MAX 4096
#define SMP_SPLIT_MAX_B 8                       // default largest two-phase batch
#define SMP_SPLIT_CAP_B 1024                    // largest batch dli_sample_set_split_max_b takes
static int g_smp_max_b = SMP_SPLIT_MAX_B;

__device__ __forceinline__ bool smp_split_ok(float T, int K, float P) {
  const bool greedy = T <= 0.f || K == 1;
  return greedy || (K >= 1 && K <= SMP_CAPC);      // K <= 0 means 'no top-k': whole row
}

template <typename LT>
__global__ void __launch_bounds__(256) sample_chunk_kernel(
    float* __restrict__ cand_v, int* __restrict__ cand_i, int* __restrict__ overflow,
    const LT* __restrict__ logits, long row_stride, int V, int L,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p) {
  __shared__ uint32_t keys[SMP_CHUNK_MAX];
  __shared__ uint32_t hist[256];
  __shared__ float tmp[16];
  __shared__ uint32_t sel[3];
  const int row = blockIdx.y, c = blockIdx.x, tid = threadIdx.x, P = gridDim.x;
  const float T = temperature[row];
  const int K = top_k[row];
  if (!smp_split_ok(T, K, top_p[row])) return;        // sample_kernel reads the full row
  const int keff = (T <= 0.f || K == 1) ? 1 : K;
  const int lo = c * L, n = max(0, min(V, lo + L) - lo);
  const LT* x = logits + (long)row * row_stride + lo;
  for (int e = tid; e < n; e += 256) keys[e] = f2key(ldv(x, e));
  __syncthreads();
  // the chunk's keff-th largest key (0: fewer than keff entries -> keep them all)
  const uint32_t tau = n > 0 ? radix_kth(keys, n, (uint32_t)min(keff, n), hist, tmp, sel) : 0u;
  // ordered compaction: thread t owns a contiguous slice, a block scan of the counts gives
  // each survivor its slot
  const int per = (n + 255) / 256, b0 = min(n, tid * per), b1 = min(n, b0 + per);
  int cnt = 0;
  for (int e = b0; e < b1; ++e) cnt += keys[e] >= tau && keys[e] != 0u;
  const int incl = (int)block_scan((float)cnt, tmp);   // exact: counts < 2^24
  int pos = incl - cnt;
  const long base = ((long)row * P + c) * SMP_CAPC;
  for (int e = b0; e < b1; ++e)
    if (keys[e] >= tau && keys[e] != 0u) {
      if (pos < SMP_CAPC) { cand_v[base + pos] = key2f(keys[e]); cand_i[base + pos] = lo + e; }
      ++pos;
    }
  __shared__ int s_total;
  if (tid == 255) s_total = incl;
  __syncthreads();
  if (s_total > SMP_CAPC) {
    if (tid == 0) overflow[row] = 1;                   // the row falls back to the full scan
  }
  for (int e = s_total + tid; e < SMP_CAPC; e += 256) {
    cand_v[base + e] = -INFINITY;
    cand_i[base + e] = 0;
  }
}

template <typename LT>
__global__ void __launch_bounds__(SMP_THREADS) sample_kernel(
    int* __restrict__ out_tokens, const LT* __restrict__ logits, long row_stride, int V,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const long long* __restrict__ seeds,
    const float* __restrict__ cand_v, const int* __restrict__ cand_i,
    int* __restrict__ overflow, int ncand) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t ckey[2 * SMP_CAP];      // fast path: 512 threads x top-8 candidates
  __shared__ int cidx[2 * SMP_CAP];
  __shared__ uint32_t skey[512];
  __shared__ int sidx[512];
  __shared__ float cprob[SMP_CAP];
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ uint32_t s_sel[3], s_cnt;
  const int row = blockIdx.x, tid = threadIdx.x;
  const LT* xl = logits + (long)row * row_stride;
  const float* xc = nullptr;                     // two-phase mode: the row's candidate list
  const float T = temperature[row];
  const int K = top_k[row];
  const float P = top_p[row];
  const unsigned long long sd = (unsigned long long)seeds[row];
  const uint2 key = make_uint2((uint32_t)sd, (uint32_t)(sd >> 32));
  // two-phase small-batch mode: read the row's candidate list unless a chunk overflowed
  const int Vfull = V;
  const int* map = nullptr;
  if (cand_v != nullptr && smp_split_ok(T, K, P)) {
    if (overflow[row] == 0) {
      xc = cand_v + (long)row * ncand;
      map = cand_i + (long)row * ncand;
      V = ncand;
    }
    __syncthreads();                                          // every thread read the flag
    if (tid == 0) overflow[row] = 0;                          // zero for the next call
  }
  auto vocab_id = [&](int j) { return map != nullptr ? map[j] : j; };
  // every pass over the row: the candidate list (fp32) or the logits row (fp32 / bf16)
  auto scan = [&](int n, auto&& f) {
    if (xc != nullptr) row_scan(xc, n, f);
    else row_scan(xl, n, f);
  };

  if (T <= 0.f || K == 1) {                                  // greedy
    ArgMax a{-INFINITY, 0x7fffffff};
    scan(V, [&](float v, int i) { a = amax(a, ArgMax{v, i}); });
    a = block_argmax(a, sv, si);
    if (tid == 0) out_tokens[row] = a.i < V ? vocab_id(a.i) : 0;
    return;
  }
  const float invT = 1.f / T;
  if (K <= 0 && P >= 1.f) {                                  // plain temperature: Gumbel-max
    ArgMax a{-INFINITY, 0x7fffffff};
    for (int base = tid * 4; base < V; base += blockDim.x * 4) {
      const uint4 r = philox(key, make_uint4((uint32_t)(base >> 2), 0u, 0x5a5a5a5au, 0u));
      const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = base + j;
        if (i < V) {
          const float g = -__logf(-__logf(u01(rr[j])));
          a = amax(a, ArgMax{(xc != nullptr ? xc[i] : ldv(xl, i)) * invT + g, i});
        }
      }
    }
    a = block_argmax(a, sv, si);
    if (tid == 0) out_tokens[row] = a.i < V ? a.i : 0;
    return;
  }
  int Keff = (K <= 0 || K > SMP_CAP) ? SMP_CAP : K;
  if (Keff > Vfull) Keff = Vfull;

  int n = 0;
  bool fast_ok = false;
  // ---- fast path, no full-row select:
  //  (1) tau0 = the Keff-th largest of the 512 per-thread maxima over the row's first
  //      quarter. At least Keff elements are >= tau0, so tau0 <= the row's Keff-th largest.
  //  (2) one pass over the row; each thread keeps its top-8 (key, index) in registers
  //      (static-index insertion network) among the elements >= tau0 only. Unguarded, the
  //      network ran for nearly every element: some lane of the wave almost always had a
  //      new local top-8 entry, and the whole wave pays for it.
  //  The Keff-th largest of the candidates (tau) is exact iff no thread dropped an element
  //  >= tau, i.e. every thread's 8th kept key is < tau — one block-wide OR. Otherwise the
  //  full radix select below.
  if (Keff <= 256) {
    uint32_t mk = 0u;
    scan((V >> 4) << 2, [&](float v, int) { mk = max(mk, f2key(v)); });
    ckey[tid] = mk;
    __syncthreads();
    const uint32_t tau0 = radix_kth(ckey, SMP_THREADS, (uint32_t)Keff, hist, sv, s_sel);
    uint32_t tk[8];
    int ti[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { tk[j] = 0u; ti[j] = 0x7fffffff; }
    scan(V, [&](float v, int i) {
      uint32_t k = f2key(v);
      if (k >= tau0 && k > tk[7]) {
        int id = i;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (k > tk[j]) {
            const uint32_t t = tk[j]; tk[j] = k; k = t;
            const int u = ti[j]; ti[j] = id; id = u;
          }
        }
      }
    });
    __syncthreads();                              // every thread is past radix_kth's reads
#pragma unroll
    for (int j = 0; j < 8; ++j) { ckey[tid * 8 + j] = tk[j]; cidx[tid * 8 + j] = ti[j]; }
    __syncthreads();
    // key of the Keff-th largest candidate (0: fewer than Keff candidates)
    const uint32_t tau = radix_kth(ckey, 8 * SMP_THREADS, (uint32_t)Keff, hist, sv, s_sel);
    const int dropped = __syncthreads_or(tk[7] >= tau ? 1 : 0);
    fast_ok = tau != 0u && !dropped;
    if (fast_ok) {
      if (tid == 0) s_cnt = 0;
      __syncthreads();
      for (int e = tid; e < 8 * SMP_THREADS; e += blockDim.x) {
        if (ckey[e] >= tau) {
          const uint32_t pos = atomicAdd(&s_cnt, 1u);
          if (pos < 512) { skey[pos] = ckey[e]; sidx[pos] = cidx[e]; }
        }
      }
      __syncthreads();
      if (s_cnt > 512) {
        fast_ok = false;                          // absurd tie count: take the slow path
      } else {
        n = (int)s_cnt;
        for (int e = tid; e < n; e += blockDim.x) { ckey[e] = skey[e]; cidx[e] = sidx[e]; }
      }
      __syncthreads();
    }
  }
  if (!fast_ok) {
  // ---- radix select on order-preserving keys (largest first), 8-bit digits
  uint32_t prefix = 0, pmask = 0, k_rem = (uint32_t)Keff, above_total = 0;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    scan(V, [&](float v, int) {
      const uint32_t k = f2key(v);
      if ((k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    });
    __syncthreads();
    find_digit(hist, k_rem, sv, s_sel);
    __syncthreads();
    k_rem -= s_sel[1];
    above_total += s_sel[1];
    prefix |= s_sel[0] << shift;
    pmask |= 255u << shift;
    if (above_total + s_sel[2] <= SMP_CAP) break;
  }
  // ---- gather everything at or above the boundary bin. When that is more than SMP_CAP
  // (the 4 passes ran out: prefix is the exact CAP-th key, and its ties overflow), keep every
  // key strictly above it and the lowest-index ties: a deterministic set, whatever the order
  // of the atomics below (bf16 logits tie often)
  const bool overflow_ties = above_total + s_sel[2] > SMP_CAP;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  scan(V, [&](float v, int i) {
    const uint32_t k = f2key(v);
    if (overflow_ties ? k > prefix : (k & pmask) >= prefix) {
      const uint32_t pos = atomicAdd(&s_cnt, 1u);
      if (pos < SMP_CAP) { ckey[pos] = k; cidx[pos] = i; }
    }
  });
  __syncthreads();
  n = (int)min(s_cnt, (uint32_t)SMP_CAP);
  if (overflow_ties) {
    // ordered compaction of the ties over contiguous per-thread slices of the row
    const uint32_t need = (uint32_t)SMP_CAP - (uint32_t)n;
    const int per = (V + SMP_THREADS - 1) / SMP_THREADS;
    const int lo = min(V, tid * per), hi = min(V, lo + per);
    auto val = [&](int e) { return xc != nullptr ? xc[e] : ldv(xl, e); };
    uint32_t n_eq = 0;
    for (int e = lo; e < hi; ++e) n_eq += f2key(val(e)) == prefix;
    __syncthreads();                              // sv reuse by block_scan
    uint32_t before = (uint32_t)block_scan((float)n_eq, sv) - n_eq;   // exact: < 2^24
    for (int e = lo; e < hi && before < need; ++e) {
      if (f2key(val(e)) == prefix) {
        ckey[n + before] = prefix;
        cidx[n + before] = e;
        ++before;
      }
    }
    __syncthreads();
    n = SMP_CAP;
  }
  }
  int npow = 1;
  while (npow < n) npow <<= 1;
  for (int i = n + tid; i < npow; i += blockDim.x) { ckey[i] = 0u; cidx[i] = 0x7fffffff; }
  __syncthreads();
  // ---- bitonic sort descending by key (ties: smaller index first)
  for (int size = 2; size <= npow; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < npow / 2; i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = ((lo & size) == 0);
        const uint32_t a = ckey[lo], b = ckey[hi];
        const int ia = cidx[lo], ib = cidx[hi];
        const bool a_first = (a > b) || (a == b && ia < ib);
        if (a_first != desc) {
          ckey[lo] = b; ckey[hi] = a; cidx[lo] = ib; cidx[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  // ---- top-k cut (ties with the k-th value kept)
  const int kk = min(Keff, n);
  const uint32_t tau = ckey[kk - 1];
  int m = kk;
  while (m < n && ckey[m] == tau) ++m;
  // ---- temperature softmax over the m survivors, top-p, inverse CDF
  const float xmax = key2f(ckey[0]);
  constexpr int PER = SMP_CAP / SMP_THREADS;                 // 4 consecutive entries / thread
  float loc[PER], lsum = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int e = tid * PER + j;
    loc[j] = e < m ? __expf((key2f(ckey[e]) - xmax) * invT) : 0.f;
    lsum += loc[j];
  }
  const float incl = block_scan(lsum, sv);
  float run = incl - lsum;
#pragma unroll
  for (int j = 0; j < PER; ++j) { run += loc[j]; cprob[tid * PER + j] = run; }
  __syncthreads();
  const float Z = cprob[m - 1];
  // keep entries whose exclusive prefix < P * Z: c = 1 + (first j < m-1 with cprob[j] >= lim,
  // else m-1); then the draw j = first j < c-1 with cprob[j] > u, else c-1. Both "first
  // index" searches run over all threads with an LDS atomicMin (was one thread's serial walk)
  const float lim = P * Z;
  if (tid == 0) s_cnt = (uint32_t)(m - 1);
  __syncthreads();
  for (int e = tid; e < m - 1; e += blockDim.x)
    if (cprob[e] >= lim) atomicMin(&s_cnt, (uint32_t)e);
  __syncthreads();
  const int c = (int)s_cnt + 1;
  const float zk = cprob[c - 1];
  const uint4 r = philox(key, make_uint4(0xfffffffu, 1u, 0xa5a5a5a5u, 7u));
  const float u = u01(r.x) * zk;
  __syncthreads();                                // s_cnt read by every thread
  if (tid == 0) s_cnt = (uint32_t)(c - 1);
  __syncthreads();
  for (int e = tid; e < c - 1; e += blockDim.x)
    if (cprob[e] > u) atomicMin(&s_cnt, (uint32_t)e);
  __syncthreads();
  if (tid == 0) out_tokens[row] = vocab_id(cidx[s_cnt]);
}

// Bytes of the two-phase workspace dli_sample takes for a batch of B rows (0: one phase).
extern "C" long dli_sample_workspace_bytes(int B, int V) {
  if (B <= 0 || B > g_smp_max_b) return 0;
  return (long)g_smp_max_b * 4 + (long)B * 64 * SMP_CAPC * 8;
}

// Largest batch that samples in two phases (default SMP_SPLIT_MAX_B = 8; A/B runs raise it:
// the workspace layout follows it, so set it before the first workspace is sized). Returns
// the previous value.
extern "C" int dli_sample_set_split_max_b(int b) {
  const int old = g_smp_max_b;
  if (b >= 1 && b <= SMP_SPLIT_CAP_B) g_smp_max_b = b;
  return old;
}

// ws: nullable; when given (>= dli_sample_workspace_bytes, its first g_smp_max_b ints
// zero before the first call — the kernels leave them zero), batches of B <= 8 rows sample in
// two phases (above).
template <typename LT>
static int launch_sample(int* out_tokens, const LT* logits, long row_stride, int B, int V,
                         const float* temperature, const int* top_k, const float* top_p,
                         const long long* seeds, void* ws, hipStream_t st) {
  if (B <= 0) return 0;
  if (ws != nullptr && B <= g_smp_max_b) {
    // P chunks per row: >= 256 workgroups in all, each chunk <= SMP_CHUNK_MAX entries
    int P = 1;
    while (P < 64 && (B * P < 256 || (V + P - 1) / P > SMP_CHUNK_MAX)) P <<= 1;
    const int L = (((V + P - 1) / P) + 3) & ~3;
    if (L <= SMP_CHUNK_MAX) {
      int* overflow = static_cast<int*>(ws);
      float* cand_v = reinterpret_cast<float*>(overflow + g_smp_max_b);
      int* cand_i = reinterpret_cast<int*>(cand_v + (long)B * 64 * SMP_CAPC);
      sample_chunk_kernel<LT><<<dim3(P, B), 256, 0, st>>>(cand_v, cand_i, overflow, logits,
                                                          row_stride, V, L, temperature, top_k,
                                                          top_p);
      sample_kernel<LT><<<B, SMP_THREADS, 0, st>>>(out_tokens, logits, row_stride, V,
                                                  temperature, top_k, top_p, seeds, cand_v,
                                                  cand_i, overflow, P * SMP_CAPC);
      DLI_RETURN_LAUNCH();
    }
  }
  sample_kernel<LT><<<B, SMP_THREADS, 0, st>>>(out_tokens, logits, row_stride, V, temperature,
                                              top_k, top_p, seeds, nullptr, nullptr, nullptr, 0);
  DLI_RETURN_LAUNCH();
}

extern "C" int dli_sample(int* out_tokens, const float* logits, long row_stride, int B, int V,
                          const float* temperature, const int* top_k, const float* top_p,
                          const long long* seeds, void* ws, hipStream_t st) {
  return launch_sample(out_tokens, logits, row_stride, B, V, temperature, top_k, top_p, seeds,
                       ws, st);
}

// the same over bf16 logits (row_stride in elements)
extern "C" int dli_sample_bf16(int* out_tokens, const void* logits, long row_stride, int B,
                               int V, const float* temperature, const int* top_k,
                               const float* top_p, const long long* seeds, void* ws,
                               hipStream_t st) {
  return launch_sample(out_tokens, static_cast<const u16*>(logits), row_stride, B, V,
                       temperature, top_k, top_p, seeds, ws, st);
}

// ---------------------------------------------------------------------------------------
// Per-row top-c of fp32 logits (the vocab-parallel LM head's candidates,
// parallel/pipeline.py): one 512-thread workgroup per row.
//   1. radix select over the row in global memory (4 passes of 8-bit digits on order-
//      preserving keys): tau = key of the c-th largest element, n_gt = count above tau;
//   2. ordered compaction: thread t owns a contiguous slice of the row, so a block scan of
//      per-thread counts writes the winners (every key > tau, then the first c - n_gt keys
//      == tau in index order) already in ascending index order — the order the candidate
//      merge on rank 0 requires (ranks concatenate ascending vocab slices).
// Replaces torch.topk + torch.sort + gather on the pipeline's hot path.
template <typename T>
__global__ void __launch_bounds__(SMP_THREADS) topk_rows_kernel(
    float* __restrict__ out_v, int* __restrict__ out_i, const T* __restrict__ x,
    long row_stride, int V, int c, int id_offset) {
  __shared__ uint32_t hist[256];
  __shared__ float sv[16];
  __shared__ uint32_t s_sel[3];
  const int row = blockIdx.x, tid = threadIdx.x;
  const T* xr = x + (long)row * row_stride;
  uint32_t prefix = 0, pmask = 0, k_rem = (uint32_t)c;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    row_scan(xr, V, [&](float v, int) {
      const uint32_t k = f2key(v);
      if ((k & pmask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    });
    __syncthreads();
    find_digit(hist, k_rem, sv, s_sel);
    __syncthreads();
    k_rem -= s_sel[1];
    prefix |= s_sel[0] << shift;
    pmask |= 255u << shift;
    __syncthreads();
  }
  const uint32_t tau = prefix;                 // c-th largest key; k_rem of its ties are taken
  // ---- ordered compaction over contiguous per-thread slices
  const int per = (V + SMP_THREADS - 1) / SMP_THREADS;
  const int lo = min(V, tid * per), hi = min(V, lo + per);
  uint32_t n_gt = 0, n_eq = 0;
  for (int e = lo; e < hi; ++e) {
    const uint32_t k = f2key(ldv(xr, e));
    n_gt += k > tau;
    n_eq += k == tau;
  }
  const float gt_incl = block_scan((float)n_gt, sv);        // exact: counts < 2^24
  __syncthreads();
  const float eq_incl = block_scan((float)n_eq, sv);
  uint32_t eq_before = (uint32_t)eq_incl - n_eq;            // ties in earlier slices
  uint32_t before = (uint32_t)gt_incl - n_gt + min(eq_before, k_rem);
  for (int e = lo; e < hi && before < (uint32_t)c; ++e) {
    const float v = ldv(xr, e);
    const uint32_t k = f2key(v);
    bool take = k > tau;
    if (k == tau) { take = eq_before < k_rem; ++eq_before; }
    if (take) {
      out_v[(long)row * c + before] = v;
      out_i[(long)row * c + before] = e + id_offset;
      ++before;
    }
  }
}

extern "C" int dli_topk_rows(float* out_v, int* out_i, const float* x, long row_stride, int rows,
                             int V, int c, int id_offset, hipStream_t st) {
  if (rows <= 0) return 0;
  if (c < 1 || c > V || V > (1 << 24)) return (int)hipErrorInvalidValue;
  topk_rows_kernel<float><<<rows, SMP_THREADS, 0, st>>>(out_v, out_i, x, row_stride, V, c,
                                                         id_offset);
  DLI_RETURN_LAUNCH();
}

extern "C" int dli_topk_rows_bf16(float* out_v, int* out_i, const void* x, long row_stride,
                                  int rows, int V, int c, int id_offset, hipStream_t st) {
  if (rows <= 0) return 0;
  if (c < 1 || c > V || V > (1 << 24)) return (int)hipErrorInvalidValue;
  topk_rows_kernel<u16><<<rows, SMP_THREADS, 0, st>>>(out_v, out_i, static_cast<const u16*>(x),
                                                       row_stride, V, c, id_offset);
  DLI_RETURN_LAUNCH();
}
