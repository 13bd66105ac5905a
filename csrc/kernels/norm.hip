// RMSNorm / LayerNorm (+ fused residual add) for gfx950 — SURVEY.md §2.4 K2/K3.
//
// Memory-bound: one workgroup per row, 16-B vector loads (8 x bf16 per lane), the row is
// held in registers between the reduction and the normalised write (one HBM read of x and
// of the residual, one write of each). fp32 statistics, bf16 I/O.
#include "common.h"

template <int VPT, bool LAYERNORM, bool ADD_RES>
__global__ void __launch_bounds__(256) norm_kernel(
    u16* __restrict__ out, u16* __restrict__ residual, const u16* __restrict__ x,
    const u16* __restrict__ w, const u16* __restrict__ b, int dim, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = dim >> 3;
  const u16* xr = x + (size_t)row * dim;
  u16* rr = residual ? residual + (size_t)row * dim : nullptr;
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      load8(xr + vi * 8, v[i]);
      if (ADD_RES) {
        float r[8];
        load8(rr + vi * 8, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
        // residual stream is kept in bf16 (as HF does for bf16 models): round, then normalise
        // the rounded value so the next layer sees exactly what is stored.
        store8(rr + vi * 8, v[i]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j]));
      } else if (residual) {
        store8(rr + vi * 8, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += LAYERNORM ? v[i][j] : v[i][j] * v[i][j];
    }
  }
  float mean = 0.f, rstd;
  if (LAYERNORM) {
    mean = block_sum(s, red) / dim;
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int vi = threadIdx.x + i * blockDim.x;
      if (vi < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { float d = v[i][j] - mean; s2 += d * d; }
      }
    }
    __syncthreads();
    rstd = rsqrtf(block_sum(s2, red) / dim + eps);
  } else {
    rstd = rsqrtf(block_sum(s, red) / dim + eps);
  }
  u16* orow = out + (size_t)row * dim;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      float wv[8], o[8];
      load8(w + vi * 8, wv);
      if (LAYERNORM) {
        float bv[8];
        load8(b + vi * 8, bv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * wv[j] + bv[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rstd * wv[j];
      }
      store8(orow + vi * 8, o);
    }
  }
}

template <bool LN, bool ADD>
static int launch_norm(void* out, void* residual, const void* x, const void* w, const void* b,
                       int rows, int dim, float eps, hipStream_t st) {
  if (dim % 8 != 0 || rows <= 0) return rows == 0 ? 0 : (int)hipErrorInvalidValue;
  const int nvec = dim / 8;
  int threads = ((nvec + 63) / 64) * 64;
  if (threads > 256) threads = 256;
  const int vpt = (nvec + threads - 1) / threads;
  dim3 g(rows), blk(threads);
  auto o = (u16*)out; auto r = (u16*)residual; auto xi = (const u16*)x;
  auto wi = (const u16*)w; auto bi = (const u16*)b;
  switch (vpt) {
    case 1: norm_kernel<1, LN, ADD><<<g, blk, 0, st>>>(o, r, xi, wi, bi, dim, eps); break;
    case 2: norm_kernel<2, LN, ADD><<<g, blk, 0, st>>>(o, r, xi, wi, bi, dim, eps); break;
    case 3: norm_kernel<3, LN, ADD><<<g, blk, 0, st>>>(o, r, xi, wi, bi, dim, eps); break;
    case 4: norm_kernel<4, LN, ADD><<<g, blk, 0, st>>>(o, r, xi, wi, bi, dim, eps); break;
    case 5: case 6: case 7: case 8:
      norm_kernel<8, LN, ADD><<<g, blk, 0, st>>>(o, r, xi, wi, bi, dim, eps); break;
    default: return (int)hipErrorInvalidValue;  // dim > 16384
  }
  DLI_RETURN_LAUNCH();
}

// out = rmsnorm(x) * w ; if residual != null it receives a copy of x (first-layer form).
extern "C" int dli_rmsnorm(void* out, void* residual_copy, const void* x, const void* w, int rows,
                           int dim, float eps, hipStream_t st) {
  return launch_norm<false, false>(out, residual_copy, x, w, nullptr, rows, dim, eps, st);
}

// residual += x (bf16, in place); out = rmsnorm(residual) * w
extern "C" int dli_fused_add_rmsnorm(void* out, void* residual, const void* x, const void* w,
                                     int rows, int dim, float eps, hipStream_t st) {
  return launch_norm<false, true>(out, residual, x, w, nullptr, rows, dim, eps, st);
}

extern "C" int dli_layernorm(void* out, void* residual_copy, const void* x, const void* w,
                             const void* b, int rows, int dim, float eps, hipStream_t st) {
  return launch_norm<true, false>(out, residual_copy, x, w, b, rows, dim, eps, st);
}

extern "C" int dli_fused_add_layernorm(void* out, void* residual, const void* x, const void* w,
                                       const void* b, int rows, int dim, float eps,
                                       hipStream_t st) {
  return launch_norm<true, true>(out, residual, x, w, b, rows, dim, eps, st);
}
