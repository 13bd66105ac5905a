// Mixture-of-experts routing / permutation kernels (Mixtral) — SURVEY.md §2.4 K15/K16.
//   route   : softmax over E router logits -> top-k -> renormalise (HF MixtralSparseMoeBlock)
//   align   : per-expert counts, exclusive offsets, permuted position of every (token, slot)
//   gather  : x_perm[p] = x[src[p]]            (16-B row copies)
//   combine : out[t] = sum_slot w[t,slot] * y_perm[pos[t,slot]]   (fp32 sum, bf16 out)
// The expert MLPs themselves run as grouped GEMMs (gemm.hip, grid.z = expert).
#include "common.h"

// One wave per token, lane e holds expert e (E <= 64): softmax max / sum and each of the k
// argmax rounds are wave-wide shuffle reductions, so no per-thread logits array (the former
// float p[64] per thread spilled to scratch).
__global__ void __launch_bounds__(256) moe_route_kernel(float* __restrict__ topk_w,
                                                        int* __restrict__ topk_ids,
                                                        const u16* __restrict__ logits, int T,
                                                        int E, int k) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;                                  // wave-uniform
  const float x = lane < E ? bf2f(logits[(long)t * E + lane]) : -INFINITY;
  route_pick(x, lane, E, k, t, topk_w, topk_ids);
}

// The Mixtral gate in one pass: the E <= 8 router logits of a token are dot products of its
// hidden row with the E router rows (a 512 x 8 GEMM through MFMA tiles took a 128 x 128 tile
// per 8 columns, a split-K reduce and a route kernel: ~24 us per layer at batch 512). One
// workgroup per token: thread i takes the 16-B chunks i, i + 256, ... of the row (fp32
// sums, wave-reduced, the 4 waves' partials added in LDS in wave order); the logits are
// rounded to bf16 as the GEMM's output was, and wave 0 picks as moe_route_kernel. (A wave per
// token, 128 workgroups, walked its 8 chunks one HBM round trip at a time: 14.9 us.)
template <int EM, int NCH>
__global__ void __launch_bounds__(256) moe_router_kernel(float* __restrict__ topk_w,
                                                         int* __restrict__ topk_ids,
                                                         const u16* __restrict__ h, int ldh,
                                                         const u16* __restrict__ wr, int T,
                                                         int E, int D, int k) {
  __shared__ float part[4][EM];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int t = blockIdx.x;
  const u16* hr = h + (long)t * ldh;
  float acc[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) acc[e] = 0.f;
  // NCH > 0 (D = 2048 NCH): each thread's NCH 16-B chunks of the hidden row and of every
  // expert row are all requested before any is used, in straight-line code (rows past E
  // re-read row E - 1, unused). A loop over the chunks, or one that left at E, had the
  // compiler wait on each load as it came: one round trip per load, 13.4 us per call.
  if constexpr (NCH > 0) {
    uint4 xv[NCH], wv[NCH][EM];
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      const int c = threadIdx.x + 256 * u;
      xv[u] = *reinterpret_cast<const uint4*>(hr + 8 * c);
#pragma unroll
      for (int e = 0; e < EM; ++e)
        wv[u][e] = *reinterpret_cast<const uint4*>(wr + (long)min(e, E - 1) * D + 8 * c);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < NCH; ++u) {
      float x[8];
      unpack8bf(xv[u], x);
#pragma unroll
      for (int e = 0; e < EM; ++e) {
        float w[8];
        unpack8bf(wv[u][e], w);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[e] = fmaf(x[j], w[j], acc[e]);
      }
    }
  } else {
    for (int c = threadIdx.x; c < D / 8; c += 256) {
      float x[8];
      load8(hr + 8 * c, x);
#pragma unroll
      for (int e = 0; e < EM; ++e) {
        float w[8];
        load8(wr + (long)min(e, E - 1) * D + 8 * c, w);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[e] = fmaf(x[j], w[j], acc[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    const float s = wave_sum(acc[e]);
    if (lane == 0) part[wv][e] = s;
  }
  __syncthreads();
  if (wv != 0) return;
  float lg = -INFINITY;
  if (lane < E && lane < EM)
    lg = bf2f(f2bf(((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]));
  route_pick(lg, lane, E, k, t, topk_w, topk_ids);
}

extern "C" int dli_moe_router(float* topk_w, int* topk_ids, const void* h, int ldh,
                              const void* wr, int T, int E, int D, int k, hipStream_t st) {
  if (T <= 0) return 0;
  if (E > 8 || k > E || D % 8 || ldh % 8 || ((uintptr_t)h & 15) || ((uintptr_t)wr & 15))
    return (int)hipErrorInvalidValue;
#define DLI_ROUTER(NCH) moe_router_kernel<8, NCH><<<T, 256, 0, st>>>(topk_w, topk_ids, \
      (const u16*)h, ldh, (const u16*)wr, T, E, D, k)
  if (D == 4096) DLI_ROUTER(2);
  else if (D == 2048) DLI_ROUTER(1);
  else DLI_ROUTER(0);
#undef DLI_ROUTER
  DLI_RETURN_LAUNCH();
}

extern "C" int dli_moe_route(float* topk_w, int* topk_ids, const void* logits, int T, int E, int k,
                             hipStream_t st) {
  if (T <= 0) return 0;
  if (E > 64 || k > E) return (int)hipErrorInvalidValue;
  moe_route_kernel<<<(T + 3) / 4, 256, 0, st>>>(topk_w, topk_ids, (const u16*)logits, T, E, k);
  DLI_RETURN_LAUNCH();
}

// Single workgroup of 1024 threads (n = T*k routed slots: counting and placement are
// block-strided, LDS atomics; the expert-offset scan is one wave's shuffle scan). ids: [n]
// expert ids; experts outside [e0, e0+E_local) are dropped (pos = -1). offsets:
// [E_local + 1]; pos: [n]; src: [n] (token of each permuted row).
__global__ void __launch_bounds__(1024) moe_align_kernel(int* __restrict__ offsets,
                                                         int* __restrict__ pos,
                                                         int* __restrict__ src,
                                                         const int* __restrict__ ids, int n,
                                                         int k, int e0, int E_local) {
  __shared__ int cnt[256];
  __shared__ int off[257];
  for (int i = threadIdx.x; i < E_local; i += blockDim.x) cnt[i] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i] - e0;
    if (e >= 0 && e < E_local) atomicAdd(&cnt[e], 1);
  }
  __syncthreads();
  if (threadIdx.x < 64) {                              // exclusive scan by the first wave
    const int lane = threadIdx.x;
    int run = 0;
    for (int base = 0; base < E_local; base += 64) {
      const int e = base + lane;
      const int c = e < E_local ? cnt[e] : 0;
      int incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      if (e < E_local) off[e] = run + incl - c;
      run += __shfl(incl, 63, 64);
    }
    if (lane == 0) off[E_local] = run;
  }
  __syncthreads();
  for (int e = threadIdx.x; e <= E_local; e += blockDim.x) {
    offsets[e] = off[e];
    if (e < E_local) cnt[e] = 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i] - e0;
    if (e >= 0 && e < E_local) {
      const int p = off[e] + atomicAdd(&cnt[e], 1);
      pos[i] = p;
      src[p] = i / k;
    } else {
      pos[i] = -1;
    }
  }
}

extern "C" int dli_moe_align(int* offsets, int* pos, int* src, const int* ids, int n, int k,
                             int e0, int E_local, hipStream_t st) {
  if (E_local > 256) return (int)hipErrorInvalidValue;
  moe_align_kernel<<<1, 1024, 0, st>>>(offsets, pos, src, ids, n, k, e0, E_local);
  DLI_RETURN_LAUNCH();
}

// rows p >= *count (the routed total, offsets[E_local]) are left untouched: src is undefined there
__global__ void __launch_bounds__(256) moe_gather_kernel(u16* __restrict__ out,
                                                         const u16* __restrict__ x,
                                                         const int* __restrict__ src, int P,
                                                         int dim, const int* __restrict__ count) {
  const int chunks = dim >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)P * chunks) return;
  const int p = (int)(gid / chunks), c = (int)(gid % chunks);
  if (count != nullptr && p >= *count) return;
  *reinterpret_cast<uint4*>(out + (long)p * dim + c * 8) =
      *reinterpret_cast<const uint4*>(x + (long)src[p] * dim + c * 8);
}

extern "C" int dli_moe_gather(void* out, const void* x, const int* src, int P, int dim,
                              const int* count, hipStream_t st) {
  if (P <= 0) return 0;
  if (dim % 8) return (int)hipErrorInvalidValue;
  const long total = (long)P * (dim / 8);
  moe_gather_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>((u16*)out, (const u16*)x, src, P,
                                                                dim, count);
  DLI_RETURN_LAUNCH();
}

__global__ void __launch_bounds__(256) moe_combine_kernel(u16* __restrict__ out,
                                                          const u16* __restrict__ y,
                                                          const float* __restrict__ w,
                                                          const int* __restrict__ pos, int T,
                                                          int k, int dim) {
  const int chunks = dim >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)T * chunks) return;
  const int t = (int)(gid / chunks), c = (int)(gid % chunks);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    const int p = pos[t * k + j];
    if (p < 0) continue;
    float v[8];
    load8(y + (long)p * dim + c * 8, v);
    const float ww = w[t * k + j];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += ww * v[q];
  }
  store8(out + (long)t * dim + c * 8, acc);
}

extern "C" int dli_moe_combine(void* out, const void* y, const float* w, const int* pos, int T,
                               int k, int dim, hipStream_t st) {
  if (T <= 0) return 0;
  if (dim % 8) return (int)hipErrorInvalidValue;
  const long total = (long)T * (dim / 8);
  moe_combine_kernel<<<(int)((total + 255) / 256), 256, 0, st>>>((u16*)out, (const u16*)y, w, pos,
                                                                 T, k, dim);
  DLI_RETURN_LAUNCH();
}

// The combine fused with the down projection's split-K reduce: the grouped down GEMM leaves
// S fp16 x 1/16 partial slabs [S, rows, dim] (EPI_SLAB16, permuted rows) instead of a bf16 y;
// each (token, pick) row is summed over the slabs in slab order, rounded to bf16 exactly as
// the bf16 GEMM output would be, weighted and accumulated as in moe_combine_kernel. The
// expert output never makes the bf16 round trip through memory and no reduce kernel runs.
template <int S>
__global__ void __launch_bounds__(256) moe_combine_slabs_kernel(
    u16* __restrict__ out, const u16* __restrict__ ws, long slab_stride,
    const float* __restrict__ w, const int* __restrict__ pos, int T, int k, int dim) {
  const int chunks = dim >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)T * chunks) return;
  const int t = (int)(gid / chunks), c = (int)(gid % chunks);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    const int p = pos[t * k + j];
    if (p < 0) continue;
    uint4 u[S];
#pragma unroll
    for (int s = 0; s < S; ++s)
      u[s] = *reinterpret_cast<const uint4*>(ws + s * slab_stride + (long)p * dim + c * 8);
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float f[8];
      unpack8h(u[s], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += f[q];
    }
    const float ww = w[t * k + j];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += ww * bf2f(f2bf(v[q]));
  }
  store8(out + (long)t * dim + c * 8, acc);
}

// The combine above, then the next layer's input norm in the same pass (one workgroup per
// token, 512 threads x 8 columns = dim 4096): m = bf16(sum_j w_j bf16(sum_s P_s[pos_j]))
// (what moe_combine_slabs_kernel stores), residual = bf16(residual + m), out =
// rmsnorm(residual) * nw — the combine's bf16 output and the separate add + RMSNorm kernel
// (norm_kernel, 7.5 us per layer at batch 512) go away. nw null: the residual add only (a
// stage's last layer).
template <int S>
__global__ void __launch_bounds__(512) moe_combine_add_rmsnorm_kernel(
    u16* __restrict__ out, u16* __restrict__ residual, const u16* __restrict__ ws,
    long slab_stride, const float* __restrict__ w, const int* __restrict__ pos, int k, int dim,
    const u16* __restrict__ nw, float eps) {
  __shared__ float red[16];
  const int t = blockIdx.x, c = threadIdx.x;
  const long off = (long)t * dim + c * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < k; ++j) {
    const int p = pos[t * k + j];
    if (p < 0) continue;
    uint4 u[S];
#pragma unroll
    for (int s = 0; s < S; ++s)
      u[s] = *reinterpret_cast<const uint4*>(ws + s * slab_stride + (long)p * dim + c * 8);
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float f[8];
      unpack8h(u[s], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] += f[q];
    }
    const float ww = w[t * k + j];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] += ww * bf2f(f2bf(v[q]));
  }
  float r[8], x[8], ss = 0.f;
  load8(residual + off, r);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    x[q] = bf2f(f2bf(r[q] + bf2f(f2bf(acc[q]))));
    ss += x[q] * x[q];
  }
  store8(residual + off, x);
  if (nw == nullptr) return;                         // uniform
  const float rstd = rsqrtf(block_sum(ss, red) / dim + eps);
  float wn[8], o[8];
  load8(nw + c * 8, wn);
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = x[q] * rstd * wn[q];
  store8(out + off, o);
}

extern "C" int dli_moe_combine_add_rmsnorm(void* out, void* residual, const void* ws, int splits,
                                           int rows, const float* w, const int* pos, int T,
                                           int k, int dim, const void* nw, float eps,
                                           hipStream_t st) {
  if (T <= 0) return 0;
  if (dim != 4096) return (int)hipErrorInvalidValue;
  const long stride = (long)rows * dim;
#define DLI_MCN(S) moe_combine_add_rmsnorm_kernel<S><<<T, 512, 0, st>>>(                   \
      (u16*)out, (u16*)residual, (const u16*)ws, stride, w, pos, k, dim, (const u16*)nw, eps)
  switch (splits) {
    case 2: DLI_MCN(2); break;
    case 4: DLI_MCN(4); break;
    case 8: DLI_MCN(8); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef DLI_MCN
  DLI_RETURN_LAUNCH();
}

// ws: the fp16 slabs of a grouped split-K GEMM over `rows` permuted rows (slab stride rows x dim)
extern "C" int dli_moe_combine_slabs(void* out, const void* ws, int splits, int rows,
                                     const float* w, const int* pos, int T, int k, int dim,
                                     hipStream_t st) {
  if (T <= 0) return 0;
  if (dim % 8) return (int)hipErrorInvalidValue;
  const long total = (long)T * (dim / 8);
  const int blocks = (int)((total + 255) / 256);
  const long stride = (long)rows * dim;
#define DLI_MCS(S) moe_combine_slabs_kernel<S><<<blocks, 256, 0, st>>>(               \
      (u16*)out, (const u16*)ws, stride, w, pos, T, k, dim)
  switch (splits) {
    case 2: DLI_MCS(2); break;
    case 4: DLI_MCS(4); break;
    case 8: DLI_MCS(8); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef DLI_MCS
  DLI_RETURN_LAUNCH();
}

// Expert-parallel dispatch pack (parallel/expert.py): every (token t, pick j) row goes to
// the bucket of the rank that holds its expert:
//   dest = id / e_per,  pos[t*k + j] = base[dest] + atomicAdd(&fill[dest], 1),
//   send_x[pos] = x[t], send_e[pos] = id (global expert id; unused rows keep -1).
// Decode: base[d] = d * C with C = T * min(k, e_per), which bounds a bucket exactly (a
// token's top-k experts are distinct), so no row is dropped and the all-to-all sizes are
// known on the host without reading the routing. Prefill: base = exclusive prefix of the
// exact per-destination counts. Slot order within a bucket is arbitrary; results do not
// depend on it (the expert GEMM treats rows independently, the combine sums each token's
// picks in j order). One 256-thread workgroup per (t, j): lane 0 claims the slot, the block
// copies the row with 16-B vectors.
__global__ void __launch_bounds__(256) ep_pack_kernel(u16* __restrict__ send_x,
                                                      int* __restrict__ send_e,
                                                      int* __restrict__ pos,
                                                      int* __restrict__ fill,
                                                      const int* __restrict__ base,
                                                      const u16* __restrict__ x,
                                                      const int* __restrict__ ids, int k, int D,
                                                      int e_per) {
  __shared__ int s_pos;
  const int r = blockIdx.x;                      // = t * k + j
  const int t = r / k;
  if (threadIdx.x == 0) {
    const int id = ids[r];
    const int dest = id / e_per;
    const int p = base[dest] + atomicAdd(&fill[dest], 1);
    pos[r] = p;
    send_e[p] = id;
    s_pos = p;
  }
  __syncthreads();
  const int p = s_pos;
  const int chunks = D >> 3;
  for (int c = threadIdx.x; c < chunks; c += blockDim.x)
    *reinterpret_cast<uint4*>(send_x + (long)p * D + c * 8) =
        *reinterpret_cast<const uint4*>(x + (long)t * D + c * 8);
}

extern "C" int dli_ep_pack(void* send_x, int* send_e, int* pos, int* fill, const int* base,
                           const void* x, const int* ids, int T, int k, int D, int e_per,
                           hipStream_t st) {
  if (T <= 0) return 0;
  if (D % 8 || e_per <= 0) return (int)hipErrorInvalidValue;
  ep_pack_kernel<<<T * k, 256, 0, st>>>((u16*)send_x, send_e, pos, fill, base, (const u16*)x,
                                         ids, k, D, e_per);
  DLI_RETURN_LAUNCH();
}
