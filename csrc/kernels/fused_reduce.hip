// Split-K partial-sum reductions fused with the elementwise op that follows the GEMM, so a
// decode layer runs 2 fewer kernels and never re-reads the bf16 GEMM output:
//
//  dli_splitk_add_rmsnorm : out = rmsnorm(residual += sum_s P_s) * w     (O-proj, down-proj)
//                           (w == null: residual += sum_s P_s only, for a stage's last layer)
//  dli_splitk_rope_cache  : qkv = bf16(sum_s P_s); RoPE on q,k in place; k,v -> paged cache
//
// P_s are the [M, N] slabs written by a GEMM called with C == nullptr: fp32, or (fmt 1, the
// EPI_SLAB16 epilogue of the MFMA families) fp16 scaled by 1/16. The sum is fp32 in slab
// order 0..S-1 and rounded to bf16 before the residual add / rotation, exactly as the bf16
// GEMM output would be.
#include "common.h"
#include <stdlib.h>

// SPL > 0: the split count is a compile-time constant, so every partial of a thread is
// loaded before the first add (SPL x VPT x 2 16-B loads in flight per lane instead of 2 x VPT);
// SPL == 0 reads `splits` partials in a runtime loop.
template <int VPT, int SPL, bool S16 = false>
__global__ void __launch_bounds__(512) splitk_add_rmsnorm_kernel(
    u16* __restrict__ out, u16* __restrict__ residual, const float* __restrict__ ws, int splits,
    int M, int N, const u16* __restrict__ w, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = N >> 3;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (S16) {                        // fp16 slabs: one 16-B load per slab
        const u16* ws16 = reinterpret_cast<const u16*>(ws);
        uint4 pu[SPL];
#pragma unroll
        for (int s = 0; s < SPL; ++s)
          pu[s] = *reinterpret_cast<const uint4*>(ws16 + ((long)s * M + row) * N + vi * 8);
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          float f[8];
          unpack8h(pu[s], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += f[j];
        }
      } else if constexpr (SPL > 0) {
        float4 pa[SPL], pb[SPL];
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          const float4* p = reinterpret_cast<const float4*>(ws + ((long)s * M + row) * N + vi * 8);
          pa[s] = p[0];
          pb[s] = p[1];
        }
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          acc[0] += pa[s].x; acc[1] += pa[s].y; acc[2] += pa[s].z; acc[3] += pa[s].w;
          acc[4] += pb[s].x; acc[5] += pb[s].y; acc[6] += pb[s].z; acc[7] += pb[s].w;
        }
      } else {
        for (int s = 0; s < splits; ++s) {
          const float4* p = reinterpret_cast<const float4*>(ws + ((long)s * M + row) * N + vi * 8);
          const float4 a = p[0], b = p[1];
          acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
          acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
        }
      }
      float r[8];
      u16* rp = residual + (long)row * N + vi * 8;
      load8(rp, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(r[j] + bf2f(f2bf(acc[j]))));
      store8(rp, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  if (w == nullptr) return;
  const float rstd = rsqrtf(block_sum(ss, red) / N + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      float wv[8], o[8];
      load8(w + vi * 8, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rstd * wv[j];
      store8(out + (long)row * N + vi * 8, o);
    }
  }
}

template <int VPT>
static int launch_add_rmsnorm(u16* o, u16* r, const float* ws, int splits, int M, int N,
                              const u16* wp, float eps, int threads, int fmt, hipStream_t st) {
  if (fmt == 1) {                                  // fp16 slabs: the planner's 2 / 4 / 8 splits
    switch (splits) {
      case 2: splitk_add_rmsnorm_kernel<VPT, 2, true><<<M, threads, 0, st>>>(o, r, ws, 2, M, N, wp, eps); break;
      case 4: splitk_add_rmsnorm_kernel<VPT, 4, true><<<M, threads, 0, st>>>(o, r, ws, 4, M, N, wp, eps); break;
      case 8: splitk_add_rmsnorm_kernel<VPT, 8, true><<<M, threads, 0, st>>>(o, r, ws, 8, M, N, wp, eps); break;
      default: return (int)hipErrorInvalidValue;
    }
    DLI_RETURN_LAUNCH();
  }
  // the register-resident partials of SPL x VPT cap the unrolled variants at 8 slabs, so
  // they exist for rows up to 4096 wide (VPT <= 2) and the split counts the planner offers
  // (2/4/8); wider rows and other counts take the runtime-split loop (SPL = 0)
  switch (VPT <= 2 ? splits : 0) {
    case 2: splitk_add_rmsnorm_kernel<VPT, 2><<<M, threads, 0, st>>>(o, r, ws, 2, M, N, wp, eps); break;
    case 4: splitk_add_rmsnorm_kernel<VPT, 4><<<M, threads, 0, st>>>(o, r, ws, 4, M, N, wp, eps); break;
    case 8: splitk_add_rmsnorm_kernel<VPT, 8><<<M, threads, 0, st>>>(o, r, ws, 8, M, N, wp, eps); break;
    default: splitk_add_rmsnorm_kernel<VPT, 0><<<M, threads, 0, st>>>(o, r, ws, splits, M, N, wp, eps);
  }
  DLI_RETURN_LAUNCH();
}

// The Mixtral O-projection reduce with the MoE gate fused in (fp16 slabs, rows of N = 512 x 8
// columns: one 8-column vector per thread, 8 waves): residual += sum_s P_s; out =
// rmsnorm(residual) * w; then the E <= 8 router logits of the bf16 output row (each thread's
// 8 columns against the E router rows, requested with the slabs; per-wave sums added in LDS
// in wave order), rounded to bf16, softmax, top-k (route_pick) — the separate gate kernel
// (moe_router_kernel, 9 us per layer at batch 512) and its launch go away.
template <int SPL>
__global__ void __launch_bounds__(512) splitk_add_rmsnorm_route_kernel(
    u16* __restrict__ out, u16* __restrict__ residual, const u16* __restrict__ ws16, int M,
    int N, const u16* __restrict__ w, float eps, const u16* __restrict__ wr, int E, int k,
    float* __restrict__ topk_w, int* __restrict__ topk_ids) {
  constexpr int EM = 8;
  __shared__ float red[16];
  __shared__ float part[8][EM];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const long off = (long)row * N + tid * 8;
  uint4 pu[SPL], rv, wvv, ru[EM];
#pragma unroll
  for (int s = 0; s < SPL; ++s)
    pu[s] = *reinterpret_cast<const uint4*>(ws16 + (long)s * M * N + off);
  rv = *reinterpret_cast<const uint4*>(residual + off);
  wvv = *reinterpret_cast<const uint4*>(w + tid * 8);
#pragma unroll
  for (int e = 0; e < EM; ++e)
    ru[e] = *reinterpret_cast<const uint4*>(wr + (long)min(e, E - 1) * N + tid * 8);
  __builtin_amdgcn_sched_barrier(0);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < SPL; ++s) {
    float f[8];
    unpack8h(pu[s], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += f[j];
  }
  float r[8], v[8], ss = 0.f;
  unpack8bf(rv, r);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = bf2f(f2bf(r[j] + bf2f(f2bf(acc[j]))));
    ss += v[j] * v[j];
  }
  store8(residual + off, v);
  const float rstd = rsqrtf(block_sum(ss, red) / N + eps);
  float wn[8], o[8];
  unpack8bf(wvv, wn);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f(f2bf(v[j] * rstd * wn[j]));   // as stored
  store8(out + off, o);
  float lg[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    float we[8];
    unpack8bf(ru[e], we);
    float d = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) d = fmaf(o[j], we[j], d);
    lg[e] = wave_sum(d);
  }
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < EM; ++e) part[wv][e] = lg[e];
  }
  __syncthreads();
  if (wv != 0) return;
  float x = -INFINITY;
  if (lane < E && lane < EM) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += part[q][lane];
    x = bf2f(f2bf(t));
  }
  route_pick(x, lane, E, k, row, topk_w, topk_ids);
}

// N = 4096 (512 threads x 8), fp16 slabs, E <= 8
extern "C" int dli_splitk_add_rmsnorm_route(void* out, void* residual, const void* ws,
                                            int splits, int M, int N, const void* w, float eps,
                                            const void* wr, int E, int k, float* topk_w,
                                            int* topk_ids, hipStream_t st) {
  if (M <= 0) return 0;
  if (N != 4096 || E > 8 || k > E || w == nullptr || ((uintptr_t)wr & 15))
    return (int)hipErrorInvalidValue;
#define DLI_SRR(S) splitk_add_rmsnorm_route_kernel<S><<<M, 512, 0, st>>>((u16*)out, \
      (u16*)residual, (const u16*)ws, M, N, (const u16*)w, eps, (const u16*)wr, E, k, topk_w, \
      topk_ids)
  switch (splits) {
    case 2: DLI_SRR(2); break;
    case 4: DLI_SRR(4); break;
    case 8: DLI_SRR(8); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef DLI_SRR
  DLI_RETURN_LAUNCH();
}

// fmt: 0 = fp32 slabs, 1 = fp16 x 1/16 slabs (EPI_SLAB16)
extern "C" int dli_splitk_add_rmsnorm(void* out, void* residual, const float* ws, int splits,
                                      int M, int N, const void* w, float eps, int fmt,
                                      hipStream_t st) {
  if (M <= 0) return 0;
  if (N % 8 || fmt < 0 || fmt > 1) return (int)hipErrorInvalidValue;
  const int nvec = N / 8;
  // threads per row (one workgroup per row): 512, i.e. one 8-column vector per lane at
  // N = 4096 (same-box A/B with the GEMMs that feed it, M = 512: O + reduce 33.85-33.92 ->
  // 33.4 us, down + reduce 70.5-70.8 -> 69.95 us; profiles/r3/reduce_threads/)
  constexpr int cap = 512;
  int threads = ((nvec + 63) / 64) * 64;
  if (threads > cap) threads = cap;
  const int vpt = (nvec + threads - 1) / threads;
  auto o = (u16*)out; auto r = (u16*)residual; auto wp = (const u16*)w;
  switch (vpt) {
    case 1: return launch_add_rmsnorm<1>(o, r, ws, splits, M, N, wp, eps, threads, fmt, st);
    case 2: return launch_add_rmsnorm<2>(o, r, ws, splits, M, N, wp, eps, threads, fmt, st);
    case 3: case 4: return launch_add_rmsnorm<4>(o, r, ws, splits, M, N, wp, eps, threads, fmt, st);
    case 5: case 6: case 7: case 8:
      return launch_add_rmsnorm<8>(o, r, ws, splits, M, N, wp, eps, threads, fmt, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// one lane: 8 dims of the first half of a head + the matching 8 of the second half. SPL > 0:
// compile-time split count, every partial's loads issued before the first add (and the
// position / cos-sin loads ahead of them); SPL == 0: runtime loop.
template <int SPL, bool S16 = false>
__global__ void __launch_bounds__(256) splitk_rope_cache_kernel(
    u16* __restrict__ qkv, const float* __restrict__ ws, int splits, int T, int N,
    const int* __restrict__ positions, const int* __restrict__ slot_mapping,
    const float* __restrict__ cos_sin, u16* __restrict__ k_cache, u16* __restrict__ v_cache,
    int hq, int hkv, int hd, int block_size, int use_rope) {
  const int lanes_per_head = hd >> 4;
  const int heads = hq + 2 * hkv;
  const long total = (long)T * heads * lanes_per_head;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int c = (int)(gid % lanes_per_head);
  const long th = gid / lanes_per_head;
  const int h = (int)(th % heads);
  const int t = (int)(th / heads);
  const int half = hd >> 1, d0 = c * 8;
  const long col1 = (long)h * hd + d0, col2 = col1 + half;
  const bool is_q = h < hq, is_k = !is_q && h < hq + hkv;
  const bool rope = use_rope && (is_q || is_k);
  const int pos = rope ? positions[t] : 0;
  float x1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, x2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto add4 = [](float* x, const float4& a, const float4& b) {
    x[0] += a.x; x[1] += a.y; x[2] += a.z; x[3] += a.w;
    x[4] += b.x; x[5] += b.y; x[6] += b.z; x[7] += b.w;
  };
  if constexpr (S16) {                             // fp16 slabs: one 16-B load per half-row
    const u16* ws16 = reinterpret_cast<const u16*>(ws);
    uint4 pu[SPL], pv[SPL];
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
      const u16* base = ws16 + ((long)s * T + t) * N;
      pu[s] = *reinterpret_cast<const uint4*>(base + col1);
      pv[s] = *reinterpret_cast<const uint4*>(base + col2);
    }
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
      float f1[8], f2[8];
      unpack8h(pu[s], f1);
      unpack8h(pv[s], f2);
#pragma unroll
      for (int j = 0; j < 8; ++j) { x1[j] += f1[j]; x2[j] += f2[j]; }
    }
  } else if constexpr (SPL > 0) {
    float4 pa[SPL], pb[SPL], pe[SPL], pf[SPL];
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
      const float* base = ws + ((long)s * T + t) * N;
      const float4* p1 = reinterpret_cast<const float4*>(base + col1);
      const float4* p2 = reinterpret_cast<const float4*>(base + col2);
      pa[s] = p1[0]; pb[s] = p1[1]; pe[s] = p2[0]; pf[s] = p2[1];
    }
#pragma unroll
    for (int s = 0; s < SPL; ++s) { add4(x1, pa[s], pb[s]); add4(x2, pe[s], pf[s]); }
  } else {
    for (int s = 0; s < splits; ++s) {
      const float* base = ws + ((long)s * T + t) * N;
      const float4* p1 = reinterpret_cast<const float4*>(base + col1);
      const float4* p2 = reinterpret_cast<const float4*>(base + col2);
      add4(x1, p1[0], p1[1]);
      add4(x2, p2[0], p2[1]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { x1[j] = bf2f(f2bf(x1[j])); x2[j] = bf2f(f2bf(x2[j])); }
  if (rope) {
    const float* cs = cos_sin + (long)pos * hd;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float co = cs[d0 + j], si = cs[half + d0 + j];
      const float o1 = x1[j] * co - x2[j] * si, o2 = x2[j] * co + x1[j] * si;
      x1[j] = bf2f(f2bf(o1));
      x2[j] = bf2f(f2bf(o2));
    }
  }
  u16* row = qkv + (long)t * N;
  store8(row + col1, x1);
  store8(row + col2, x2);
  if (is_q || k_cache == nullptr) return;
  const int slot = slot_mapping[t];
  if (slot < 0) return;
  const int blk = slot / block_size, off = slot - blk * block_size;
  // K and V share the token-major [blk, head, off, hd] layout: whole-row 16-B stores
  u16* dst = is_k ? k_cache + (((long)blk * hkv + (h - hq)) * block_size + off) * hd
                  : v_cache + (((long)blk * hkv + (h - hq - hkv)) * block_size + off) * hd;
  store8(dst + d0, x1);
  store8(dst + half + d0, x2);
}

extern "C" int dli_splitk_rope_cache(void* qkv, const float* ws, int splits, int T, int N,
                                     const int* positions, const int* slot_mapping,
                                     const float* cos_sin, void* k_cache, void* v_cache, int hq,
                                     int hkv, int hd, int block_size, int use_rope, int fmt,
                                     hipStream_t st) {
  if (T <= 0) return 0;
  if (hd % 16 || N != (hq + 2 * hkv) * hd || fmt < 0 || fmt > 1 ||
      (fmt == 1 && splits != 2 && splits != 4 && splits != 8))
    return (int)hipErrorInvalidValue;
  const long total = (long)T * (hq + 2 * hkv) * (hd / 16);
  const int blocks = (int)((total + 255) / 256);
#define DLI_SRC(S, F) splitk_rope_cache_kernel<S, F><<<blocks, 256, 0, st>>>(             \
      (u16*)qkv, ws, splits, T, N, positions, slot_mapping, cos_sin, (u16*)k_cache,        \
      (u16*)v_cache, hq, hkv, hd, block_size, use_rope)
  if (fmt == 1) {
    switch (splits) {
      case 2: DLI_SRC(2, true); break;
      case 4: DLI_SRC(4, true); break;
      default: DLI_SRC(8, true);
    }
  } else {
    switch (splits) {
      case 2: DLI_SRC(2, false); break;
      case 4: DLI_SRC(4, false); break;
      default: DLI_SRC(0, false);
    }
  }
#undef DLI_SRC
  DLI_RETURN_LAUNCH();
}
