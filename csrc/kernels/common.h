// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of distributed_llm_inferencing_amd.
//
// Conventions used by every kernel in this directory:
//  * wave = 64 lanes; block sizes are multiples of 64.
//  * bf16 tensors are moved as 16-byte vectors (8 x bf16) wherever the row allows it.
//  * fp32 accumulation everywhere; f32->bf16 through __float2bfloat16, which lowers to
//    v_cvt_pk_bf16_f32 on gfx950 (round-to-nearest-even, NaN-preserving).
//  * every launcher is `extern "C" int dli_*(..., hipStream_t)` returning a hipError_t.
// Comments cite cdna_hip_programming.md and MI355X_MICROARCH.md: the CDNA4 programming guide
// and the measured MI355X microarchitecture notes of the build image (/opt/skills/guides/),
// not files of this repository.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define DLI_WAVE 64

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16;

struct alignas(16) U16x8 { u16 v[8]; };
struct alignas(8) U16x4 { u16 v[4]; };

__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ u16 f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<u16*>(&b);
}

__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// 8 bf16 (one 16-B word) -> fp32
__device__ __forceinline__ void unpack8bf(const uint4 v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ void load8(const u16* p, float* f) {
  unpack8bf(*reinterpret_cast<const uint4*>(p), f);
}

__device__ __forceinline__ void store8(u16* p, const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]); v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]); v.w = pack2bf(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// MoE gate (moe.hip moe_route / moe_router kernels, fused_reduce.hip add + RMSNorm + gate):
// softmax over the E logits (lane e < E holds logit e, the others -inf) -> top-k (HF: lowest
// index on ties) -> renormalised weights; one wave per token
__device__ __forceinline__ void route_pick(float x, int lane, int E, int k, int t,
                                           float* __restrict__ topk_w,
                                           int* __restrict__ topk_ids) {
  const float mx = wave_max(x);
  float p = lane < E ? __expf(x - mx) : 0.f;
  const float s = wave_sum(p);
  float mine = 0.f, wsum = 0.f;                        // lane j keeps the j-th pick's weight
  for (int j = 0; j < k; ++j) {
    float bv = lane < E ? p : -3.f;
    int bi = lane;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {                 // argmax, lowest index on ties (HF)
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    const float w = bv / s;
    wsum += w;
    if (lane == j) { mine = w; topk_ids[t * k + j] = bi; }
    if (lane == bi) p = -2.f;                          // taken
  }
  if (lane < k) topk_w[t * k + lane] = mine / wsum;
}


// XCD-aware bijective remap of a linear block id (cdna_hip_programming.md §5 'XCD swizzle must be
// bijective'): consecutive logical tiles land on the same XCD (shared L2). Speed only.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

#define DLI_RETURN_LAUNCH() return (int)hipGetLastError()

// fp16 split-K partials (the EPI_SLAB16 GEMM epilogue and its consumers): value x 1/16 in
// fp16 (RNE), read back x 16 — half the bytes of fp32 slabs, |partial| up to ~1e6 in range
constexpr float SLAB16_SCALE = 0.0625f, SLAB16_UNSCALE = 16.f;
__device__ __forceinline__ uint32_t pack2h(float a, float b) {
  const _Float16 ha = (_Float16)a, hb = (_Float16)b;
  return (uint32_t)__builtin_bit_cast(uint16_t, ha) |
         ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
__device__ __forceinline__ float h2f(uint32_t bits16) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
}
// 8 fp16 slab values (one 16-B load) -> fp32, unscaled
__device__ __forceinline__ void unpack8h(const uint4 u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = h2f(w[i] & 0xffffu) * SLAB16_UNSCALE;
    f[2 * i + 1] = h2f(w[i] >> 16) * SLAB16_UNSCALE;
  }
}

