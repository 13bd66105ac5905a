// Shared pieces of the bf16 MFMA GEMM families (gemm_tiles.hip, gemm8p.hip, gemm4w.hip,
// gemv.hip; dispatched by gemm.hip's dli_gemm): epilogue stores, split-K slab stores, the
// counted-vmcnt helpers, the split-K tile mapping and the split-K reduce kernel.
// Every kernel computes C[M,N] = A[M,K] . W[N,K]^T with the W fragment as MFMA operand A
// (transposed accumulators, see below). Static / inline only: each family is its own
// translation unit.
#pragma once
#include "common.h"
#include <type_traits>


#define BK 64

enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_SILU = 2, EPI_BIAS_GELU = 3, EPI_BIAS = 4,
       // slab-only split-K call (C == nullptr, splits > 1) whose partials are stored as fp16
       // scaled by 1/16 instead of fp32 (half the bytes the GEMM writes and its consumer
       // reads; the scale keeps |partial| up to ~1e6 in range). Tiles and 8-phase families.
       EPI_SLAB16 = 5 };

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }
// tanh-approximate GELU, branch-free: 0.5 (1 + tanh(y)) = sigmoid(2 y). tanhf's range
// branches made a 256-accumulator epilogue too large to unroll, and the rolled loop indexed
// the accumulators dynamically: hipcc demoted them to scratch and copied them out of the
// AGPRs inside the K loop, where no hazard padding follows an inline-asm MFMA
__device__ __forceinline__ float gelu_f(float x) {
  const float y2 = 1.5957691216057308f * (x + 0.044715f * x * x * x);
  return x / (1.f + __expf(-y2));
}

template <int EPI>
__device__ __forceinline__ void store_pair_or_one(void* C, int ldc, int row, int col, float v,
                                                  const u16* bias) {
  if (EPI == EPI_F32) {
    ((float*)C)[(long)row * ldc + col] = v;
  } else {
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) v += bf2f(bias[col]);
    if (EPI == EPI_BIAS_GELU) v = gelu_f(v);
    ((u16*)C)[(long)row * ldc + col] = f2bf(v);
  }
}

// fp32 split-K partial stores: 0 plain (the line stays dirty in the XCD's L2 and is written
// back at the kernel boundary, /opt/skills/guides/MI355X_MICROARCH.md price row 'boundary'), 1 nontemporal,
// 2 sc1 (write-through: the bytes leave L2 while the GEMM still computes), 3 sc0 sc1.
// One copy per translation unit (device code is not relocatable across files, -fno-gpu-rdc):
// every GEMM family sets its own through set_slab_store_tu(), dli_gemm_set_slab_store sets all.
static __device__ int g_slab_store = 0;
static inline int set_slab_store_tu(int mode) {
  int old = 0;
  (void)hipMemcpyFromSymbol(&old, HIP_SYMBOL(g_slab_store), sizeof(int));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_slab_store), &mode, sizeof(int));
  return old;
}
__device__ __forceinline__ void slab_store(float* p, float v, int mode) {
  if (mode == 1) {
    __builtin_nontemporal_store(v, p);
  } else if (mode == 2) {
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else if (mode == 3) {
    asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  } else {
    *p = v;
  }
}

// ---- transposed accumulators. Every MFMA kernel in this file passes the W fragment as MFMA
// operand A and the activation fragment as operand B, i.e. it computes C^T = W . A^T. A
// 16x16 output block then lands as: lane (fq = lane / 16, fr = lane % 16) holds
// C[16 i + fr][16 j + 4 fq + r] for r = 0..3 — four CONSECUTIVE columns of one row — so an
// epilogue writes one 16-B (fp32 slab / logits) or 8-B (bf16) vector per block instead of
// four 4-B / 2-B scalars. The epilogue store tail of a short-K split GEMM is issue-bound
// (cdna_hip_programming.md T21: halving the store instructions at equal bytes halved it);
// the fragments read from LDS, the MFMA count and the slab layout are unchanged.
__device__ __forceinline__ void slab_store4(float* p, f32x4 v, int mode) {
  if (mode == 1) {
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
  } else if (mode == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else if (mode == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  } else {
    *reinterpret_cast<f32x4*>(p) = v;
  }
}

// the fp32 partial quad (store modes 0-3); the 4-wave family calls it directly (its
// accumulator-pinned epilogue has no register room for the probe modes)
__device__ __forceinline__ void slab_quad_fp32(float* p, f32x4 v, int mode, bool vec, int left) {
  if (vec) {
    slab_store4(p, v, mode);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r < left) slab_store(p + r, v[r], mode);
  }
}

// fp16 (x 1/16) partial quad of the EPI_SLAB16 slab image: p = &fp32-indexed slab[row][col]
// (the element index into a [splits][M][N] image based at ws), one 8-B store
__device__ __forceinline__ void slab_quad16(float* p, f32x4 v, bool vec, int left,
                                            const float* ws) {
  u16* q = (u16*)ws + (p - ws);
  if (vec) {
    uint2 pk;
    pk.x = pack2h(v[0] * SLAB16_SCALE, v[1] * SLAB16_SCALE);
    pk.y = pack2h(v[2] * SLAB16_SCALE, v[3] * SLAB16_SCALE);
    *reinterpret_cast<uint2*>(q) = pk;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r < left) q[r] = (u16)(pack2h(v[r] * SLAB16_SCALE, 0.f) & 0xffffu);
  }
}

// one split-K partial quad: p = &slab[row][col]; vec = (N % 4 == 0), so col + 3 < N.
// Probe modes (dli_gemm_set_slab_store): 4 = bf16 partials at the same element index of a
// bf16 [splits][M][N] image based at ws, 5 = no store (timing only: the consumer reads junk)
__device__ __forceinline__ void slab_quad(float* p, f32x4 v, int mode, bool vec, int left,
                                          const float* ws) {
  if (mode == 5) return;
  if (mode == 4) {
    u16* q = (u16*)ws + (p - ws);
    if (vec) {
      uint2 pk;
      pk.x = pack2bf(v[0], v[1]);
      pk.y = pack2bf(v[2], v[3]);
      *reinterpret_cast<uint2*>(q) = pk;
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (r < left) q[r] = f2bf(v[r]);
    }
    return;
  }
  slab_quad_fp32(p, v, mode, vec, left);
}

// four consecutive output columns [col, col + 4) of one row; vec = (N % 4 == 0 && ldc % 4
// == 0): one 16-B (fp32) / 8-B (bf16) store, else per-column stores for the row's tail
template <int EPI>
__device__ __forceinline__ void store_quad(void* C, int ldc, int row, int col, int N, f32x4 v,
                                           const u16* bias, bool vec) {
  if (!vec) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (col + r < N) store_pair_or_one<EPI>(C, ldc, row, col + r, v[r], bias);
    return;
  }
  if (EPI == EPI_F32) {
    *reinterpret_cast<f32x4*>((float*)C + (long)row * ldc + col) = v;
    return;
  }
  float o[4] = {v[0], v[1], v[2], v[3]};
  if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
    const uint2 b = *reinterpret_cast<const uint2*>(bias + col);
    o[0] += __uint_as_float(b.x << 16); o[1] += __uint_as_float(b.x & 0xffff0000u);
    o[2] += __uint_as_float(b.y << 16); o[3] += __uint_as_float(b.y & 0xffff0000u);
  }
  if (EPI == EPI_BIAS_GELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = gelu_f(o[r]);
  }
  uint2 pk;
  pk.x = pack2bf(o[0], o[1]);
  pk.y = pack2bf(o[2], o[3]);
  *reinterpret_cast<uint2*>((u16*)C + (long)row * ldc + col) = pk;
}

// the vector epilogue needs every row start and column quad aligned: N and ldc multiples
// of 4, C (and the bias) 16-B (fp32) / 8-B (bf16) aligned (C may be a column view)
template <int EPI>
__device__ __forceinline__ bool out_vec(const void* C, int ldc, int N, const u16* bias) {
  const uintptr_t mis = ((uintptr_t)C | (uintptr_t)bias) & (EPI == EPI_F32 ? 15 : 7);
  return ((N | ldc) & 3) == 0 && mis == 0;
}

// SiLU(gate) * up of one gate block g and its up block u (same lane, same row): the four
// features [f, f + 4) of the 16-row-interleaved gate/up layout
__device__ __forceinline__ void store_silu_quad(void* C, int ldc, int row, int f, f32x4 g,
                                                f32x4 u, bool vec) {
  float o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = silu_f(g[r]) * u[r];
  u16* p = (u16*)C + (long)row * ldc + f;
  if (vec) {
    uint2 pk;
    pk.x = pack2bf(o[0], o[1]);
    pk.y = pack2bf(o[2], o[3]);
    *reinterpret_cast<uint2*>(p) = pk;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r] = f2bf(o[r]);
  }
}

// s_waitcnt vmcnt(N) with expcnt/lgkmcnt left at their maxima (gfx9 encoding)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// s_waitcnt vmcnt(INSTR * ahead) for a wave-uniform ahead in [0, MAXA]: retire everything
// but the `ahead` youngest tiles of INSTR LDS-DMA instructions each
template <int INSTR, int MAXA>
__device__ __forceinline__ void wait_ahead(int ahead) {
  static_assert(MAXA <= 4 && INSTR * MAXA < 64, "vmcnt range");
  if constexpr (MAXA >= 4) { if (ahead >= 4) { wait_vmcnt<INSTR * 4>(); return; } }
  if constexpr (MAXA >= 3) { if (ahead == 3) { wait_vmcnt<INSTR * 3>(); return; } }
  if constexpr (MAXA >= 2) { if (ahead == 2) { wait_vmcnt<INSTR * 2>(); return; } }
  if constexpr (MAXA >= 1) { if (ahead == 1) { wait_vmcnt<INSTR>(); return; } }
  wait_vmcnt<0>();
}

// Block -> (output tile, K split). Without split-K: the XCD remap over tiles (n-major order,
// so an XCD's tiles share W panels). With split-K, (split, tile) is one split-major index
// remapped over the whole grid, so an XCD's blocks work on ONE K slice: its L2 fetches that
// slice of A once instead of every XCD fetching all of A (rocprofv3 TCC_EA0_RDREQ_*: the
// down projection at M=512, split 8, read 224 MB per call for 132 MB of operands).
// The hardware places linear block id L = y * gridDim.x + x on XCD L % 8.
__device__ __forceinline__ void split_tile(int nwg, bool grouped, int& tile, int& ks) {
  if (grouped || gridDim.y == 1) {
    tile = xcd_remap(blockIdx.x, nwg);
    ks = blockIdx.y;
    return;
  }
  const int total = nwg * (int)gridDim.y;
  const int lg = xcd_remap((int)(blockIdx.y * gridDim.x + blockIdx.x), total);
  ks = lg / nwg;
  tile = lg - ks * nwg;
}

// split-K reduction + epilogue: one thread per output element group of 4 columns
template <int EPI>
static __global__ void __launch_bounds__(256) splitk_reduce_kernel(void* __restrict__ C, int ldc,
                                                            const float* __restrict__ ws, int M,
                                                            int N, int splits,
                                                            const u16* __restrict__ bias) {
  const int outN = (EPI == EPI_SILU) ? N / 2 : N;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)M * outN) return;
  const int row = (int)(gid / outN), col = (int)(gid % outN);
  if (EPI == EPI_SILU) {
    const int grp = col >> 4, in = col & 15;
    const long gi = (long)row * N + grp * 32 + in, ui = gi + 16;
    float g = 0.f, u = 0.f;
    for (int s = 0; s < splits; ++s) { g += ws[(long)s * M * N + gi]; u += ws[(long)s * M * N + ui]; }
    ((u16*)C)[(long)row * ldc + col] = f2bf(silu_f(g) * u);
  } else {
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += ws[(long)s * M * N + (long)row * N + col];
    store_pair_or_one<EPI>(C, ldc, row, col, v, bias);
  }
}


// the dispatch signature every family shares: (tile_cfg) -> that family's launcher, or
// DLI_NOT_MINE when the tile id belongs to another family
#define DLI_GEMM_ARGS const void *A, int lda, const void *W, int ldw, void *C, int ldc, int M, \
                      int N, int K, int splits, const void *bias, void *ws, const int *go,  \
                      int groups, hipStream_t st
#define DLI_GEMM_PASS A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st
constexpr int DLI_NOT_MINE = -0x4d494e45;

int gemm_tiles_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS);
int gemm_8p_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS);
int gemm_4w_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS);
int gemm_4wp_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS);
int gemm_gemv_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS);
int gemm_tiles_set_slab_store(int mode);
int gemm_8p_set_slab_store(int mode);
int gemm_4w_set_slab_store(int mode);

// EPI -> template argument, for a family's dispatch<EPI>(tile_cfg, ...); the families with
// an fp16 slab store (tiles, 8-phase) take DLI_EPI_SWITCH_S16
#define DLI_EPI_SWITCH_S16(FN)                                                     \
  if (epi == EPI_SLAB16) {                                                         \
    if (C != nullptr || splits < 2) return (int)hipErrorInvalidValue;              \
    return FN<EPI_SLAB16>(tile_cfg, DLI_GEMM_PASS);                                \
  }                                                                                \
  DLI_EPI_SWITCH(FN)

#define DLI_EPI_SWITCH(FN)                                                         \
  switch (epi) {                                                                   \
    case EPI_BF16: return FN<EPI_BF16>(tile_cfg, DLI_GEMM_PASS);                   \
    case EPI_F32: return FN<EPI_F32>(tile_cfg, DLI_GEMM_PASS);                     \
    case EPI_SILU: return FN<EPI_SILU>(tile_cfg, DLI_GEMM_PASS);                   \
    case EPI_BIAS_GELU: return FN<EPI_BIAS_GELU>(tile_cfg, DLI_GEMM_PASS);         \
    case EPI_BIAS: return FN<EPI_BIAS>(tile_cfg, DLI_GEMM_PASS);                   \
    default: return (int)hipErrorInvalidValue;                                     \
  }
