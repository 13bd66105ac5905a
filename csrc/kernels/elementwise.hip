// Memory-bound elementwise kernels: embedding gather (K1), SiLU·mul over the 16-row
// interleaved gate/up activation (K10 unfused form), tanh-GELU (+bias) and bias add (GPT-2).
// All move 16 B per lane (cdna_hip_programming.md Guideline 13).
#include "common.h"

// x[t] = table[ids[t]] (+ pos_table[positions[t]])  — one 8-element chunk per lane
__global__ void __launch_bounds__(256) embedding_kernel(
    u16* __restrict__ out, const int* __restrict__ ids, const u16* __restrict__ table,
    const u16* __restrict__ pos_table, const int* __restrict__ positions, int T, int dim) {
  const int chunks = dim >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)T * chunks) return;
  const int t = (int)(gid / chunks), c = (int)(gid % chunks);
  const u16* src = table + (long)ids[t] * dim + c * 8;
  if (pos_table == nullptr) {
    *reinterpret_cast<uint4*>(out + (long)t * dim + c * 8) = *reinterpret_cast<const uint4*>(src);
  } else {
    float a[8], b[8];
    load8(src, a);
    load8(pos_table + (long)positions[t] * dim + c * 8, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += b[j];
    store8(out + (long)t * dim + c * 8, a);
  }
}

extern "C" int dli_embedding(void* out, const int* ids, const void* table, const void* pos_table,
                             const int* positions, int T, int dim, hipStream_t st) {
  if (T <= 0) return 0;
  if (dim % 8) return (int)hipErrorInvalidValue;
  const long total = (long)T * (dim / 8);
  embedding_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>(
      (u16*)out, ids, (const u16*)table, (const u16*)pos_table, positions, T, dim);
  DLI_RETURN_LAUNCH();
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// gu [T, 2F] in 16-row-group interleave -> out [T, F]; each lane: 8 output features.
__global__ void __launch_bounds__(256) silu_mul_kernel(u16* __restrict__ out,
                                                        const u16* __restrict__ gu, int T, int F) {
  const int chunks = F >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)T * chunks) return;
  const int t = (int)(gid / chunks), c = (int)(gid % chunks);
  const int f0 = c * 8;                       // output features [f0, f0+8) lie in one 16-group
  const int grp = f0 >> 4, in = f0 & 15;
  const u16* row = gu + (long)t * 2 * F;
  float g[8], u[8], o[8];
  load8(row + grp * 32 + in, g);
  load8(row + grp * 32 + 16 + in, u);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = silu(g[j]) * u[j];
  store8(out + (long)t * F + f0, o);
}

extern "C" int dli_silu_mul(void* out, const void* gu, int T, int F, hipStream_t st) {
  if (T <= 0) return 0;
  if (F % 16) return (int)hipErrorInvalidValue;
  const long total = (long)T * (F / 8);
  silu_mul_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>((u16*)out, (const u16*)gu, T, F);
  DLI_RETURN_LAUNCH();
}

__device__ __forceinline__ float gelu_tanh_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

// y = act(x + bias) in place; act: 0 = identity, 1 = gelu_tanh
__global__ void __launch_bounds__(256) bias_act_kernel(u16* __restrict__ x,
                                                        const u16* __restrict__ bias, int T, int N,
                                                        int act) {
  const int chunks = N >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)T * chunks) return;
  const int t = (int)(gid / chunks), c = (int)(gid % chunks);
  u16* p = x + (long)t * N + c * 8;
  float v[8];
  load8(p, v);
  if (bias) {
    float b[8];
    load8(bias + c * 8, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += b[j];
  }
  if (act == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_tanh_f(v[j]);
  }
  store8(p, v);
}

extern "C" int dli_bias_act(void* x, const void* bias, int T, int N, int act, hipStream_t st) {
  if (T <= 0) return 0;
  if (N % 8) return (int)hipErrorInvalidValue;
  const long total = (long)T * (N / 8);
  bias_act_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>((u16*)x, (const u16*)bias, T, N,
                                                               act);
  DLI_RETURN_LAUNCH();
}

// Lookahead input ids (engine/llm_engine.py): ids[i] = feed[src[i]] where src[i] >= 0, i.e. the
// token the in-flight step sampled for that sequence; src[i] < 0 keeps the host-provided id.
// One launch instead of a clamp / gather / compare / select / copy chain of torch ops.
__global__ void __launch_bounds__(256) feed_ids_kernel(int* __restrict__ ids,
                                                       const int* __restrict__ src,
                                                       const int* __restrict__ feed, int n,
                                                       int n_feed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = src[i];
  if (s >= 0 && s < n_feed) ids[i] = feed[s];
}

extern "C" int dli_feed_ids(int* ids, const int* src, const int* feed, int n, int n_feed,
                            hipStream_t st) {
  if (n <= 0) return 0;
  feed_ids_kernel<<<(n + 255) / 256, 256, 0, st>>>(ids, src, feed, n, n_feed);
  DLI_RETURN_LAUNCH();
}

// Read `bytes` of device memory and discard it: pulls a weight matrix into the memory-side
// Infinity Cache (256 MB) ahead of the GEMM that streams it, from a side stream while the
// main stream runs latency-bound work (decode attention, norms). 4 x 16 B in flight per lane;
// the xor keeps the loads alive (the guarded store never happens for real data patterns).
__global__ void __launch_bounds__(256) prefetch_kernel(const uint4* __restrict__ p, long n16,
                                                       unsigned* __restrict__ sink) {
  unsigned acc = 0;
  const long stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;
}

extern "C" int dli_prefetch(const void* p, long bytes, int max_wgs, void* sink, hipStream_t st) {
  const long n16 = bytes / 16;
  if (n16 <= 0) return 0;
  if (((uintptr_t)p & 15) || sink == nullptr) return (int)hipErrorInvalidValue;
  long wgs = (n16 + 1023) / 1024;
  if (max_wgs <= 0) max_wgs = 256;
  if (wgs > max_wgs) wgs = max_wgs;
  prefetch_kernel<<<(int)wgs, 256, 0, st>>>((const uint4*)p, n16, (unsigned*)sink);
  DLI_RETURN_LAUNCH();
}
