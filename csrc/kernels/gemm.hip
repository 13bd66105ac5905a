// bf16 GEMM on CDNA4 matrix cores: C[M,N] = A[M,K] . W[N,K]^T (+ fused epilogue).
// SURVEY.md §2.4 K4/K9-K12 (dense projections) and K16 (MoE grouped GEMM).
//
// Structure (cdna_hip_programming.md §5):
//  * WM x WN waves (2x2 = 256 threads, or 2x4 / 4x2 = 512 threads for 256-wide tiles); block
//    tile BM x BN x 64; wave tile (BM/WM) x (BN/WN) built from v_mfma_f32_16x16x32_bf16 (the bf16 shape that holds the higher clock on random
//    data, MI355X_MICROARCH.md 'DVFS give-back' item 7).
//  * global -> LDS by global_load_lds_dwordx4 (16 B per lane, no VGPR round trip), 2 LDS
//    buffers: the next K-tile's DMA is issued before the current tile's ds_reads + MFMAs.
//  * LDS rows are 128 B (64 bf16); the 16-B chunk c of row r is stored at physical chunk
//    c ^ ((r >> 1) & 7). glds writes lane-linearly, so the permutation is applied to the
//    per-lane GLOBAL source address and the same XOR on the ds_read_b128 address (rule 21);
//    verified conflict-free for all four ds_read_b128 lane groups of the 16x16x32 A/B maps.
//  * XCD-aware bijective block remap (T1) with n-major tile order so consecutive tiles share
//    one W panel in an XCD's L2; split-K grids are remapped split-major so an XCD's blocks
//    share one K slice of A and W (split_tile).
//  * split-K over grid.y writes fp32 slabs; a second pass reduces and applies the epilogue.
//  * grouped mode (MoE): grid.z = expert; rows of group g are [off[g], off[g+1]) of A/C,
//    weights W + g*N*ldw. Rows past the group end are skipped. Split-K composes with it
//    (slab rows are the permuted rows), for long-K expert GEMMs with few row tiles.
// Epilogues: 0 bf16 store, 1 fp32 store (logits), 2 SiLU(gate)*up over the 16-row-interleaved
// gate/up weight (output width N/2), 3 bias + tanh-GELU, 4 bias.
#include "common.h"
#include <type_traits>

#define BK 64

enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_SILU = 2, EPI_BIAS_GELU = 3, EPI_BIAS = 4 };

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
// back at the kernel boundary, MI355X_MICROARCH.md price row 'boundary'), 1 nontemporal,
// 2 sc1 (write-through: the bytes leave L2 while the GEMM still computes), 3 sc0 sc1.
__device__ int g_slab_store = 0;
extern "C" int dli_gemm_set_slab_store(int mode) {
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

// one split-K partial quad: p = &slab[row][col]; vec = (N % 4 == 0), so col + 3 < N
__device__ __forceinline__ void slab_quad(float* p, f32x4 v, int mode, bool vec, int left) {
  if (vec) {
    slab_store4(p, v, mode);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r < left) slab_store(p + r, v[r], mode);
  }
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

template <int BM, int BN, int EPI, int NS, int WM, int WN>
__global__ void __launch_bounds__(64 * WM * WN) gemm_bf16_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws, const int* __restrict__ group_off) {
  constexpr int NW = WM * WN;                      // waves: WM along M x WN along N
  constexpr int TM = BM / WM, TN = BN / WN;        // wave tile
  constexpr int MI = TM / 16, NI = TN / 16;        // 16x16 MFMA blocks per wave
  constexpr int A_BYTES = BM * BK * 2, W_BYTES = BN * BK * 2;
  constexpr int BUF = A_BYTES + W_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // ---- tile coordinates
  int row0 = 0, Mg = M;
  const u16* Wg = W;
  if (group_off != nullptr) {
    row0 = group_off[blockIdx.z];
    Mg = group_off[blockIdx.z + 1] - row0;
    Wg = W + (long)blockIdx.z * N * ldw;
  }
  const int tiles_m = (M + BM - 1) / BM;           // M = max rows per group in grouped mode
  const int tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int tile, ks;
  split_tile(nwg, group_off != nullptr, tile, ks);
  const int tn = tile / tiles_m, tm = tile % tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mg) return;                             // grouped: empty tile (block-uniform)
  const int kb = ks * k_split_len;
  const int nk = min(k_split_len, K - kb) / BK;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const u16* Ab = A + (long)row0 * lda;

  // ---- per-lane glds source pointers (row clamped in range; swizzled chunk)
  // one glds wave-instruction stages 8 rows x 128 B; all NW waves share each tile
  constexpr int A_INSTR = BM / (8 * NW), W_INSTR = BN / (8 * NW);
  static_assert(A_INSTR * 8 * NW == BM && W_INSTR * 8 * NW == BN, "tile vs waves");
  const u16* a_src[A_INSTR];
  const u16* w_src[W_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int r = (i * NW + wid) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = min(m0 + r, Mg - 1);
    a_src[i] = Ab + (long)gr * lda + kb + c * 8;
  }
#pragma unroll
  for (int i = 0; i < W_INSTR; ++i) {
    const int r = (i * NW + wid) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = min(n0 + r, N - 1);
    w_src[i] = Wg + (long)gr * ldw + kb + c * 8;
  }
  auto stage = [&](int buf, int kt) {
    char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(a_src[i] + kt * BK),
                                       (lds_void*)(base + (i * NW + wid) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < W_INSTR; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(w_src[i] + kt * BK),
                                       (lds_void*)(base + A_BYTES + (i * NW + wid) * 1024), 16,
                                       0, 0);
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment read offsets (bytes, within a buffer), chunk XOR applied per k-step
  const int fr = lane & 15, fq = lane >> 4;
  int a_row[MI], w_row[NI];
#pragma unroll
  for (int i = 0; i < MI; ++i) a_row[i] = wm * TM + i * 16 + fr;
#pragma unroll
  for (int j = 0; j < NI; ++j) w_row[j] = wn * TN + j * 16 + fr;

  auto compute = [&](int buf) {
    const char* abuf = smem + buf * BUF;
    const char* wbuf = abuf + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + fq;
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int r = a_row[i];
        af[i] = *reinterpret_cast<const bf16x8*>(abuf + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int r = w_row[j];
        bfr[j] = *reinterpret_cast<const bf16x8*>(wbuf + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  if (NS == 2) {
    // 2 LDS buffers: the next tile's DMA overlaps this tile's MFMAs; drained every K-step
    if (nk > 0) stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // NS >= 3 LDS buffers, NS - 2 tiles kept in flight ACROSS the barrier
    // (cdna_hip_programming.md §5 'Pipelining across barriers'): a counted vmcnt retires
    // tile kt only (the tiles issued after it stay in flight), then a raw s_barrier (a
    // __syncthreads() would emit vmcnt(0) and drain the DMA); the restaged buffer
    // (kt + NS - 1) % NS was last read in iteration kt - 1, which every wave has finished.
    // Deeper rings (NS 4-6 on the 128x64 / 128x96 / 128x128 / 128x192 decode tiles) were
    // measured and not kept: equal or slower at M = 512 (profiles/r3/deep_ring/).
    constexpr int INSTR = A_INSTR + W_INSTR;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nk) stage(s, s);
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = min(nk - 1 - kt, NS - 2);     // tiles issued after kt (uniform)
      wait_ahead<INSTR, NS - 2>(ahead);
      __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      if (kt + NS - 1 < nk) {
        int nb = cur + NS - 1;
        if (nb >= NS) nb -= NS;
        stage(nb, kt + NS - 1);
      }
      compute(cur);
      cur = (cur + 1 == NS) ? 0 : cur + 1;
    }
    wait_vmcnt<0>();
  }

  // ---- epilogue (transposed accumulators):
  // acc[i][j][r] = C[m0 + wm*TM + 16i + fr][n0 + wn*TN + 16j + 4fq + r]
  const bool split = gridDim.y > 1;
  if (split) {
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = m0 + wm * TM + 16 * i + fr;
      if (row >= Mg) continue;
      float* srow = slab + (long)(row0 + row) * N;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = n0 + wn * TN + 16 * j + 4 * fq;
        if (col < N) slab_quad(srow + col, acc[i][j], sm, vec, N - col);
      }
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {
    // column blocks j (even) = gate, j+1 = up of the same 16 features
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = m0 + wm * TM + 16 * i + fr;
      if (row >= Mg) continue;
#pragma unroll
      for (int j = 0; j < NI; j += 2) {
        const int gcol = n0 + wn * TN + 16 * j;         // first gate row of the pair
        if (gcol < N)
          store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][j],
                          acc[i][j + 1], vec);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int row = m0 + wm * TM + 16 * i + fr;
    if (row >= Mg) continue;
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int col = n0 + wn * TN + 16 * j + 4 * fq;
      if (col < N) store_quad<EPI>(C, ldc, row0 + row, col, N, acc[i][j], bias, vec);
    }
  }
}

// ---------------------------------------------------------------------------------------
// 256x256 "8-phase ping-pong" GEMM (cdna_hip_programming.md §5 'The 256² 8-phase template',
// T3+T4+T5; MI355X_MICROARCH.md 'Two waves per SIMD' items 1, 7, 9).
//
// 8 waves = 2 groups of 4 (g = wid >> 2 = the wave's 128-row half of the tile; one wave of
// each group per SIMD). Every K-tile (BK = 64) is 4 phases; a phase is a LOAD segment
// (this phase's ds_reads + one quarter of a later K-tile's glds + a counted vmcnt) and a
// MATRIX segment (16 MFMAs, one 64x32 quadrant of the wave's 128x64 output), separated by
// raw s_barriers. Group 1 runs one barrier behind group 0, so on every SIMD one wave is in
// its matrix segment while its partner is in its load segment.
//
//   phase | ds_read_b128 (this K-tile)        | MFMAs          | glds issued
//   0     | A rows 0-63 of the half, B 0-31   | acc[0-3][0-1]  | slot 3 of K-tile T+1
//   1     | B cols 32-63                      | acc[0-3][2-3]  | slot 0 of K-tile T+2
//   2     | A rows 64-127                     | acc[4-7][2-3]  | slot 1 of K-tile T+2
//   3     | -                                 | acc[4-7][0-1]  | slot 2 of K-tile T+2
//
// LDS: 2 buffers x (A 256x64 + W 256x64) bf16 = 128 KiB (1 workgroup / CU), 128-B rows with
// the chunk XOR swizzle of gemm_bf16_kernel. Staging slots per group (2 glds per lane each):
// group 0 stages A rows 0-63 / 64-127 and the even 32-row W chunks, group 1 A rows
// 128-191 / 192-255 and the odd W chunks. With segments numbered s (group 0 loads in even
// s, group 1 in odd s) every slot is restaged >= 2 segments after its last ds_read of the
// K-tile two back (WAR) and retired by its issuer's vmcnt >= 1 barrier before its first
// ds_read (RAW) when every load segment leaves the last 3 segments' glds in flight:
// vmcnt(6) in steady state, fewer when the K loop's tail issues nothing.
template <int EPI, int VAR = 0>
__global__ void __launch_bounds__(512) gemm8p_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws, const int* __restrict__ group_off) {
  constexpr int BM = 256, BN = 256;
  constexpr int A_BYTES = BM * BK * 2, BUF = 2 * A_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int row0 = 0, Mg = M;
  const u16* Wg = W;
  if (group_off != nullptr) {
    row0 = group_off[blockIdx.z];
    Mg = group_off[blockIdx.z + 1] - row0;
    Wg = W + (long)blockIdx.z * N * ldw;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = (N + BN - 1) / BN;
  int tile, ks;
  split_tile(tiles_m * tiles_n, group_off != nullptr, tile, ks);
  int tn, tm;
  constexpr int GM = (VAR & 8) ? 4 : (VAR & 16) ? 8 : 1;
  if (GM > 1) {
    // grouped order: an XCD's ~32 consecutive tiles cover GM tile-rows x 32/GM tile-columns,
    // so its CUs share both A and W panels in its L2 (n-major order shares W only)
    const int per_group = GM * tiles_n;
    const int first_m = (tile / per_group) * GM;
    const int gsz = min(tiles_m - first_m, GM);
    const int in_g = tile % per_group;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
  } else {
    tn = tile / tiles_m;
    tm = tile % tiles_m;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mg) return;
  const int kb = ks * k_split_len;
  const int nk = min(k_split_len, K - kb) / BK;
  const u16* Ab = A + (long)row0 * lda;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid >> 2, gw = wid & 3;           // group (= M half), wave in group (= N quarter)

  // ---- staging: slot s (0..3) x instruction i (0..1): element offset of this lane's source
  // and the wave-uniform LDS byte offset of the 1-KiB piece (8 rows x 128 B)
  int src[4][2];
  int dst[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int rb, is_a;
      if ((s & 1) == 0) { rb = 64 * (2 * g + (s >> 1)) + 32 * i + 8 * gw; is_a = 1; }
      else { rb = 64 * (2 * (s >> 1) + i) + 32 * g + 8 * gw; is_a = 0; }
      const int r = rb + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      if (is_a) src[s][i] = min(m0 + r, Mg - 1) * lda + kb + c * 8;
      else src[s][i] = min(n0 + r, N - 1) * ldw + kb + c * 8;
      dst[s][i] = (is_a ? 0 : A_BYTES) + rb * 128;
    }
  // deep plan (VAR & 4): per group, A region h (2 glds) and all 4 W chunks of its parity (4 glds)
  int srcB[4], dstB[4];
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4) {
    const int rb = 64 * c4 + 32 * g + 8 * gw;
    const int r = rb + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    srcB[c4] = min(n0 + r, N - 1) * ldw + kb + c * 8;
    dstB[c4] = A_BYTES + rb * 128;
  }
  auto issue_a = [&](int h, int kt) {             // h: A rows 64h..64h+63 of the group's half
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(Ab + src[2 * h][i] + kt * BK),
                                       (lds_void*)(lds + dst[2 * h][i]), 16, 0, 0);
  };
  auto issue_b = [&](int kt) {
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4)
      __builtin_amdgcn_global_load_lds((gbl_void*)(Wg + srcB[c4] + kt * BK),
                                       (lds_void*)(lds + dstB[c4]), 16, 0, 0);
  };
  auto issue = [&](auto S, int kt) {
    constexpr int s = decltype(S)::value;
    const u16* base = (s & 1) ? Wg : Ab;
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(base + src[s][i] + kt * BK),
                                       (lds_void*)(lds + dst[s][i]), 16, 0, 0);
  };

  // ---- fragments
  const int fr = lane & 15, fq = lane >> 4;
  auto read_frag = [&](const char* part, int row, int kk) -> bf16x8 {
    const int c = kk * 4 + fq;
    return *reinterpret_cast<const bf16x8*>(part + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: K-tiles 0 and 1 in full
  if (nk > 0) {
    issue(std::integral_constant<int, 0>{}, 0); issue(std::integral_constant<int, 1>{}, 0);
    issue(std::integral_constant<int, 2>{}, 0); issue(std::integral_constant<int, 3>{}, 0);
  }
  if (nk > 1) {
    issue(std::integral_constant<int, 0>{}, 1); issue(std::integral_constant<int, 1>{}, 1);
    issue(std::integral_constant<int, 2>{}, 1); issue(std::integral_constant<int, 3>{}, 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (g == 1) {                                    // stagger: group 1 runs one segment behind
    __builtin_amdgcn_s_barrier();
    if (VAR & 256) __builtin_amdgcn_s_setprio(1);  // static priority for the younger half
  }

  const int last_issue_seg = 4 * nk - 8;          // load segments 1..last issue glds
  bf16x8 a0[4][2], a1[4][2], b0[2][2], b1[2][2];

  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  auto wait_deep = [&](int u) {                   // keep the last 5 load segments' glds in flight
    int cnt = 0;
#pragma unroll
    for (int d = 0; d < 5; ++d) {
      const int v = u - d;
      const int q = v & 3;
      if (v >= 1 && q != 0 && (v >> 2) + 2 < nk) cnt += (q == 2) ? 4 : 2;
    }
    switch (cnt) {                                 // wave-uniform
      case 0: wait_vmcnt<0>(); break;
      case 2: wait_vmcnt<2>(); break;
      case 4: wait_vmcnt<4>(); break;
      case 6: wait_vmcnt<6>(); break;
      case 8: wait_vmcnt<8>(); break;
      case 10: wait_vmcnt<10>(); break;
      default: wait_vmcnt<12>(); break;
    }
  };
  auto wait_issued = [&](int u) {
    if (VAR & 4) { wait_deep(u); return; }
    if (VAR & 512) {
      // one counted wait per K-tile (the 8-phase template's schedule): at phase 3 of K-tile
      // T every DMA of T+1 is retired; only T+2's slots 0-2 (issued in phases 1-3) stay in
      // flight. Phases 0-2 do not wait at all.
      if ((u & 3) == 3) {
        if ((u >> 2) + 2 < nk) wait_vmcnt<6>();
        else wait_vmcnt<0>();
      }
      return;
    }
    const int lo = max(1, u - 2), hi = min(u, last_issue_seg);
    const int cnt = hi >= lo ? hi - lo + 1 : 0;    // wave-uniform
    if (cnt >= 3) wait_vmcnt<6>();
    else if (cnt == 2) wait_vmcnt<4>();
    else if (cnt == 1) wait_vmcnt<2>();
    else wait_vmcnt<0>();
  };

  for (int kt = 0; kt < nk; ++kt) {
    const char* abuf = smem + (kt & 1) * BUF;
    const char* wbuf = abuf + A_BYTES;
    const int arow = g * 128 + fr, wrow = gw * 64 + fr;
    const int u0 = 4 * kt;
    auto phase = [&](auto P) {
      constexpr int p = decltype(P)::value;
      auto reads = [&]() {
        if (p == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) a0[i][kk] = read_frag(abuf, arow + 16 * i, kk);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) b0[j][kk] = read_frag(wbuf, wrow + 16 * j, kk);
        } else if (p == 1) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) b1[j][kk] = read_frag(wbuf, wrow + 32 + 16 * j, kk);
        } else if (p == 2) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) a1[i][kk] = read_frag(abuf, arow + 64 + 16 * i, kk);
        }
      };
      auto stage = [&]() {
        if (p == 0) {
          if (!(VAR & 4) && kt >= 1 && kt + 1 < nk) issue(std::integral_constant<int, 3>{}, kt + 1);
        } else if (kt + 2 < nk) {
          if (VAR & 4) {
            if (p == 1) issue_a(0, kt + 2);
            else if (p == 2) issue_b(kt + 2);
            else issue_a(1, kt + 2);
          } else {
            issue(std::integral_constant<int, (p + 3) & 3>{}, kt + 2);
          }
        }
      };
      if (VAR & 64) { stage(); reads(); }
      else { reads(); stage(); }
      if (!(VAR & 32)) wait_issued(u0 + p);
      barrier();
      if (!(VAR & 256)) __builtin_amdgcn_s_setprio(1);
      const bf16x8 (&af)[4][2] = (p < 2) ? a0 : a1;
      const bf16x8 (&bf)[2][2] = (p == 0 || p == 3) ? b0 : b1;
      constexpr int I0 = (p < 2) ? 0 : 4, J0 = (p == 0 || p == 3) ? 0 : 2;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                bf[j][kk], af[i][kk], acc[I0 + i][J0 + j], 0, 0, 0);
      if (!(VAR & 256)) __builtin_amdgcn_s_setprio(0);
      barrier();
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    phase(std::integral_constant<int, 3>{});
  }
  if (g == 0) {                                    // balance group 1's stagger barrier
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue (transposed accumulators):
  // acc[I][J][r] = C[m0 + 128g + 16I + fr][n0 + 64gw + 16J + 4fq + r]
  const int wr0 = m0 + 128 * g, wc0 = n0 + 64 * gw;
  if (gridDim.y > 1) {
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
      float* srow = slab + (long)(row0 + row) * N;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wc0 + 16 * j + 4 * fq;
        if (col < N) slab_quad(srow + col, acc[i][j], sm, vec, N - col);
      }
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const int gcol = wc0 + 16 * j;
        if (gcol < N)
          store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][j],
                          acc[i][j + 1], vec);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wr0 + 16 * i + fr;
    if (row >= Mg) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc0 + 16 * j + 4 * fq;
      if (col < N) store_quad<EPI>(C, ldc, row0 + row, col, N, acc[i][j], bias, vec);
    }
  }
}

// ---------------------------------------------------------------------------------------
// 256x224 ping-pong GEMM: the 8-phase schedule of gemm8p_kernel for N-tiles of 224 columns,
// so a GEMM whose N is a multiple of 7 x 32 fills the chip where 256-wide tiles leave CUs
// idle: the Llama-3 gate/up projection at M = 512 (N = 28672) is 2 x 128 = 256 tiles on 256
// CUs instead of 224 (one workgroup per CU at 128 KiB of LDS).
//
// Waves: group g = wid >> 2 = the tile's 128-row half (one wave of each group per SIMD,
// group 1 one barrier behind); in a group, wave (wm, wn) = (w4 >> 1, w4 & 1) owns rows
// 128 g + 64 wm .. +63 and columns 112 wn .. +111: 4 x 7 MFMA blocks, as gemm8p's 8 x 4.
// K-tile T (BK = 64) = 4 phases, each a LOAD segment (ds_reads of T, LDS-DMA of T+2) and a
// MATRIX segment (MFMAs):
//   phase | reads                              | MFMAs              | DMA for T+2
//   0     | A rows +0..31 (both kk), B +0..63  | 2 x 4 blocks       | -
//   1     | B +64..111                         | 2 x 3 blocks       | A "h0", B "h0"
//   2     | A rows +32..63                     | 2 x 3 blocks       | B "h1"
//   3     | -                                  | 2 x 4 blocks       | A "h1"
// (A h0 = rows r % 64 < 32, h1 the rest; B h0 = rows 0-63 and 112-175, h1 = rows 64-111,
// 176-223 and 224-255: the next tile's rows, staged so every wave DMAs 2 pieces per region,
// never read.) Every LOAD segment retires its ds_reads (lgkmcnt(0)) before its barrier, so a
// region is restaged in the phase after its last reading phase — after group 1's read too.
// Phase 3 waits (counted vmcnt: T+2's 8 DMAs stay in flight) for every DMA of T+1, retired
// for all readers by the barrier closing the segment. SiLU pairs are 16-column blocks (2p,
// 2p+1); the pair (6, 7) straddles the two waves of a row band and meets through LDS.
template <int EPI>
__global__ void __launch_bounds__(512) gemm8p224_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws, const int* __restrict__ group_off) {
  constexpr int BM = 256, BN = 224;
  constexpr int A_BYTES = BM * BK * 2, BUF = 2 * A_BYTES;     // A 256 rows + B image 256 rows
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int row0 = 0, Mg = M;
  const u16* Wg = W;
  if (group_off != nullptr) {
    row0 = group_off[blockIdx.z];
    Mg = group_off[blockIdx.z + 1] - row0;
    Wg = W + (long)blockIdx.z * N * ldw;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = (N + BN - 1) / BN;
  int tile, ks;
  split_tile(tiles_m * tiles_n, group_off != nullptr, tile, ks);
  constexpr int GM = 4;                            // grouped tile order (see gemm8p_kernel)
  const int per_group = GM * tiles_n;
  const int first_m = (tile / per_group) * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_g = tile % per_group;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mg) return;
  const int kb = ks * k_split_len;
  const int nk = min(k_split_len, K - kb) / BK;
  const u16* Ab = A + (long)row0 * lda;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid >> 2, w4 = wid & 3, wm = w4 >> 1, wn = w4 & 1;

  // ---- LDS-DMA pieces (8 rows x 128 B; lane L lands at row L/8, physical chunk L%8, so it
  // loads logical chunk (L%8) ^ ((r >> 1) & 7)). Region pieces (16 per region, wave wid
  // takes region pieces wid and wid + 8): A h0 piece q -> rows 64 (q >> 2) + 8 (q & 3),
  // A h1 -> the same + 32; B h0 piece q -> rows 8q (q < 8) or 112 + 8 (q - 8); B h1 piece q
  // -> rows 64 + 8q (q < 6), 176 + 8 (q - 6) (q < 12), 224 + 8 (q - 12).
  auto piece_row = [](int region, int q) {
    switch (region) {
      case 0: return 64 * (q >> 2) + 8 * (q & 3);
      case 1: return 64 * (q >> 2) + 8 * (q & 3) + 32;
      case 2: return q < 8 ? 8 * q : 112 + 8 * (q - 8);
      default: return q < 6 ? 64 + 8 * q : (q < 12 ? 176 + 8 * (q - 6) : 224 + 8 * (q - 12));
    }
  };
  int src[4][2], dst[4][2];                        // [region: A h0, A h1, B h0, B h1][piece]
#pragma unroll
  for (int rg = 0; rg < 4; ++rg)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rb = piece_row(rg, wid + 8 * i);
      const int r = rb + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      if (rg < 2) src[rg][i] = min(m0 + r, Mg - 1) * lda + kb + c * 8;
      else src[rg][i] = min(n0 + r, N - 1) * ldw + kb + c * 8;
      dst[rg][i] = (rg < 2 ? 0 : A_BYTES) + rb * 128;
    }
  auto dma = [&](auto RG, int kt) {
    constexpr int rg = decltype(RG)::value;
    const u16* base = rg < 2 ? Ab : Wg;
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(base + src[rg][i] + kt * BK),
                                       (lds_void*)(lds + dst[rg][i]), 16, 0, 0);
  };
  auto dma_all = [&](int kt) {
    dma(std::integral_constant<int, 0>{}, kt); dma(std::integral_constant<int, 1>{}, kt);
    dma(std::integral_constant<int, 2>{}, kt); dma(std::integral_constant<int, 3>{}, kt);
  };

  const int fr = lane & 15, fq = lane >> 4;
  auto read_frag = [&](const char* part, int row, int kk) -> bf16x8 {
    const int c = kk * 4 + fq;
    return *reinterpret_cast<const bf16x8*>(part + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  };
  f32x4 acc[4][7];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: K-tiles 0 and 1 whole
  if (nk > 0) dma_all(0);
  if (nk > 1) { dma_all(1); wait_vmcnt<8>(); }
  else wait_vmcnt<0>();
  __syncthreads();
  if (g == 1) {                                    // stagger: group 1 runs one segment behind
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);                 // static priority for the younger half
  }
  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  const int arow = 128 * g + 64 * wm + fr, brow = 112 * wn + fr;
  bf16x8 a0[2][2], a1[2][2], b0[4][2], b1[3][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* abuf = smem + (kt & 1) * BUF;
    const char* bbuf = abuf + A_BYTES;
    auto phase = [&](auto P) {
      constexpr int p = decltype(P)::value;
      if (p == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a0[i][kk] = read_frag(abuf, arow + 16 * i, kk);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b0[j][kk] = read_frag(bbuf, brow + 16 * j, kk);
      } else if (p == 1) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b1[j][kk] = read_frag(bbuf, brow + 64 + 16 * j, kk);
        if (kt + 2 < nk) { dma(std::integral_constant<int, 0>{}, kt + 2);
                           dma(std::integral_constant<int, 2>{}, kt + 2); }
      } else if (p == 2) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a1[i][kk] = read_frag(abuf, arow + 32 + 16 * i, kk);
        if (kt + 2 < nk) dma(std::integral_constant<int, 3>{}, kt + 2);
      } else {
        if (kt + 2 < nk) { dma(std::integral_constant<int, 1>{}, kt + 2); wait_vmcnt<8>(); }
        else wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0): this segment's reads done
      barrier();
      const bf16x8 (&af)[2][2] = (p < 2) ? a0 : a1;
      constexpr int I0 = (p < 2) ? 0 : 2;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (p == 0 || p == 3) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[I0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  b0[j][kk], af[i][kk], acc[I0 + i][j], 0, 0, 0);
          } else {
#pragma unroll
            for (int j = 0; j < 3; ++j)
              acc[I0 + i][4 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  b1[j][kk], af[i][kk], acc[I0 + i][4 + j], 0, 0, 0);
          }
        }
      barrier();
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    phase(std::integral_constant<int, 3>{});
  }
  if (g == 0) __builtin_amdgcn_s_barrier();       // balance group 1's stagger barrier

  // ---- epilogue (transposed accumulators):
  // acc[i][j][r] = C[m0 + 128 g + 64 wm + 16 i + fr][n0 + 112 wn + 16 j + 4 fq + r]
  const int wr0 = m0 + 128 * g + 64 * wm, wc0 = n0 + 112 * wn;
  if (gridDim.y > 1) {
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
      float* srow = slab + (long)(row0 + row) * N;
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const int col = wc0 + 16 * j + 4 * fq;
        if (col < N) slab_quad(srow + col, acc[i][j], sm, vec, N - col);
      }
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {
    // block 6 of wave wn = 0 (gate) pairs with block 0 of wave wn = 1 (up): through LDS
    __syncthreads();                               // every wave is past its last LDS read
    float* xch = reinterpret_cast<float*>(smem) + (2 * g + wm) * 1024;   // 64 x 16 fp32
    if (wn == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<f32x4*>(xch + (16 * i + fr) * 16 + 4 * fq) = acc[i][0];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
      // own pairs: wave 0 blocks (0,1) (2,3) (4,5) + (6, partner's 0); wave 1 (1,2) (3,4)
      // (5,6) (compile-time block indices in each branch: no runtime-indexed registers)
      if (wn == 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int gcol = wc0 + 32 * q;
          if (gcol < N)
            store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][2 * q],
                            acc[i][2 * q + 1], vec);
        }
        const int gcol = wc0 + 16 * 6;
        if (gcol < N) {
          const f32x4 up = *reinterpret_cast<const f32x4*>(xch + (16 * i + fr) * 16 + 4 * fq);
          store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][6], up, vec);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int gcol = wc0 + 16 + 32 * q;
          if (gcol < N)
            store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][2 * q + 1],
                            acc[i][2 * q + 2], vec);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wr0 + 16 * i + fr;
    if (row >= Mg) continue;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int col = wc0 + 16 * j + 4 * fq;
      if (col < N) store_quad<EPI>(C, ldc, row0 + row, col, N, acc[i][j], bias, vec);
    }
  }
}

// ---------------------------------------------------------------------------------------
// 256x128 ping-pong GEMM: the 8-phase schedule of gemm8p224_kernel for 128-column N-tiles.
// Where 256-column tiles leave most of the chip idle or need deep K splits: the Mixtral
// grouped down projection (N = 4096, one 256-row tile per expert: 8 x 16 = 128 workgroups of
// 256x256 / 152 of 256x224, here 8 x 32 = 256), and the dense N = 4096 projections at
// M = 512 (64 tiles: split-K 4 fills 256 CUs with half the fp32 slab bytes of 32 tiles x 8).
//
// Waves: group g = wid >> 2 = the tile's 128-row half (one wave of each group per SIMD,
// group 1 one barrier behind); wave (wm, wn) = (w4 >> 1, w4 & 1) of a group owns rows
// 128 g + 64 wm .. +63 and columns 64 wn .. +63: 4 x 4 MFMA blocks.
//   phase | reads                              | MFMAs             | DMA for T+2
//   0     | A rows +0..31 (both kk), B +0..31  | rows 0-31, cols 0-31   | -
//   1     | B +32..63                          | rows 0-31, cols 32-63  | A h0
//   2     | A rows +32..63                     | rows 32-63, cols 32-63 | B
//   3     | -                                  | rows 32-63, cols 0-31  | A h1, then a counted
//                                                                         wait for T+1's DMAs
// (A h0 = rows r % 64 < 32, h1 the rest; B = all 128 rows, last read in phase 1.) LDS:
// 2 x (A 256 x 64 + B 128 x 64) bf16 = 96 KiB. SiLU pairs (2p, 2p+1) stay inside a wave.
template <int EPI>
__global__ void __launch_bounds__(512) gemm8p128_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws, const int* __restrict__ group_off) {
  constexpr int BM = 256, BN = 128;
  constexpr int A_BYTES = BM * BK * 2, BUF = A_BYTES + BN * BK * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int row0 = 0, Mg = M;
  const u16* Wg = W;
  if (group_off != nullptr) {
    row0 = group_off[blockIdx.z];
    Mg = group_off[blockIdx.z + 1] - row0;
    Wg = W + (long)blockIdx.z * N * ldw;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = (N + BN - 1) / BN;
  int tile, ks;
  split_tile(tiles_m * tiles_n, group_off != nullptr, tile, ks);
  constexpr int GM = 4;                            // grouped tile order (see gemm8p_kernel)
  const int per_group = GM * tiles_n;
  const int first_m = (tile / per_group) * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_g = tile % per_group;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mg) return;
  const int kb = ks * k_split_len;
  const int nk = min(k_split_len, K - kb) / BK;
  const u16* Ab = A + (long)row0 * lda;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid >> 2, w4 = wid & 3, wm = w4 >> 1, wn = w4 & 1;

  // ---- LDS-DMA pieces (8 rows x 128 B; lane L lands at row L/8, physical chunk L%8, so it
  // loads logical chunk (L%8) ^ ((r >> 1) & 7)). 16 pieces per region, wave wid takes pieces
  // wid and wid + 8: A h0 piece q -> rows 64 (q >> 2) + 8 (q & 3), A h1 -> the same + 32,
  // B piece q -> rows 8 q.
  auto piece_row = [](int region, int q) {
    switch (region) {
      case 0: return 64 * (q >> 2) + 8 * (q & 3);
      case 1: return 64 * (q >> 2) + 8 * (q & 3) + 32;
      default: return 8 * q;
    }
  };
  int src[3][2], dst[3][2];                        // [region: A h0, A h1, B][piece]
#pragma unroll
  for (int rg = 0; rg < 3; ++rg)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rb = piece_row(rg, wid + 8 * i);
      const int r = rb + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      if (rg < 2) src[rg][i] = min(m0 + r, Mg - 1) * lda + kb + c * 8;
      else src[rg][i] = min(n0 + r, N - 1) * ldw + kb + c * 8;
      dst[rg][i] = (rg < 2 ? 0 : A_BYTES) + rb * 128;
    }
  auto dma = [&](auto RG, int kt) {
    constexpr int rg = decltype(RG)::value;
    const u16* base = rg < 2 ? Ab : Wg;
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(base + src[rg][i] + kt * BK),
                                       (lds_void*)(lds + dst[rg][i]), 16, 0, 0);
  };
  auto dma_all = [&](int kt) {
    dma(std::integral_constant<int, 0>{}, kt); dma(std::integral_constant<int, 1>{}, kt);
    dma(std::integral_constant<int, 2>{}, kt);
  };

  const int fr = lane & 15, fq = lane >> 4;
  auto read_frag = [&](const char* part, int row, int kk) -> bf16x8 {
    const int c = kk * 4 + fq;
    return *reinterpret_cast<const bf16x8*>(part + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: K-tiles 0 and 1 whole
  if (nk > 0) dma_all(0);
  if (nk > 1) { dma_all(1); wait_vmcnt<6>(); }
  else wait_vmcnt<0>();
  __syncthreads();
  if (g == 1) {                                    // stagger: group 1 runs one segment behind
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);                 // static priority for the younger half
  }
  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  const int arow = 128 * g + 64 * wm + fr, brow = 64 * wn + fr;
  bf16x8 a0[2][2], a1[2][2], b0[2][2], b1[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* abuf = smem + (kt & 1) * BUF;
    const char* bbuf = abuf + A_BYTES;
    auto phase = [&](auto P) {
      constexpr int p = decltype(P)::value;
      if (p == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a0[i][kk] = read_frag(abuf, arow + 16 * i, kk);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b0[j][kk] = read_frag(bbuf, brow + 16 * j, kk);
      } else if (p == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b1[j][kk] = read_frag(bbuf, brow + 32 + 16 * j, kk);
        if (kt + 2 < nk) dma(std::integral_constant<int, 0>{}, kt + 2);
      } else if (p == 2) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a1[i][kk] = read_frag(abuf, arow + 32 + 16 * i, kk);
        if (kt + 2 < nk) dma(std::integral_constant<int, 2>{}, kt + 2);
      } else {
        if (kt + 2 < nk) { dma(std::integral_constant<int, 1>{}, kt + 2); wait_vmcnt<6>(); }
        else wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0): this segment's reads done
      barrier();
      const bf16x8 (&af)[2][2] = (p < 2) ? a0 : a1;
      const bf16x8 (&bf)[2][2] = (p == 0 || p == 3) ? b0 : b1;
      constexpr int I0 = (p < 2) ? 0 : 2, J0 = (p == 0 || p == 3) ? 0 : 2;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                bf[j][kk], af[i][kk], acc[I0 + i][J0 + j], 0, 0, 0);
      barrier();
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    phase(std::integral_constant<int, 3>{});
  }
  if (g == 0) __builtin_amdgcn_s_barrier();       // balance group 1's stagger barrier

  // ---- epilogue (transposed accumulators):
  // acc[i][j][r] = C[m0 + 128 g + 64 wm + 16 i + fr][n0 + 64 wn + 16 j + 4 fq + r]
  const int wr0 = m0 + 128 * g + 64 * wm, wc0 = n0 + 64 * wn;
  if (gridDim.y > 1) {
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
      float* srow = slab + (long)(row0 + row) * N;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wc0 + 16 * j + 4 * fq;
        if (col < N) slab_quad(srow + col, acc[i][j], sm, vec, N - col);
      }
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int gcol = wc0 + 32 * q;
        if (gcol < N)
          store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][2 * q],
                          acc[i][2 * q + 1], vec);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wr0 + 16 * i + fr;
    if (row >= Mg) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc0 + 16 * j + 4 * fq;
      if (col < N) store_quad<EPI>(C, ldc, row0 + row, col, N, acc[i][j], bias, vec);
    }
  }
}

// 16-B buffer load of `base` (a range-checked descriptor over `nbytes`: lanes past it read
// zeros) straight into LDS at the wave-uniform `lds` + 16 * lane; voff per lane, soff uniform
// CPOL: the load's cache-policy bits (0 default; 16 = sc1, device scope: the line is not
// allocated in the CU's vector L1, which an LDS-DMA stream never re-reads)
template <int CPOL = 0>
__device__ __forceinline__ void buf_lds16(const void* base, int nbytes, char* lds, int voff,
                                          int soff) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nbytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, soff, 0, CPOL);
}

// 16-B buffer load of `base` into registers (same range-checked descriptor as buf_lds16)
__device__ __forceinline__ uint4 buf_ld16(const void* base, int nbytes, int voff, int soff) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nbytes, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return uint4{v[0], v[1], v[2], v[3]};
}

// ---------------------------------------------------------------------------------------
// 256x256 GEMM with ONE wave per SIMD and 128x128 wave tiles ("4-wave"): the structure of
// the library kernels the prefill projections used to fall back to (hipBLASLt's
// MT256x256x64 solution for these shapes is 4 waves, MIWaveTile 16x4, 1 workgroup per CU).
// Against the 8-wave ping-pong (gemm8p_kernel: 128x64 per wave, two waves per SIMD) a
// 128x128 wave tile reads 1/3 fewer LDS bytes per MFMA (32 ds_read_b128 per 128 MFMAs per
// K-tile instead of 24 per 64) and issues half the barrier traffic; on MI355X under DVFS the
// energy per MFMA, not the cycle count, sets the clock the chip holds on random data
// (cdna_hip_programming.md §5.4 rule 28), and LDS read bytes are one of the terms.
//
// Waves (wm, wn) = (wid >> 1, wid & 1) own rows 128 wm .. +127 and columns 128 wn .. +127:
// acc[8][8] 16x16 blocks = 256 accumulator registers. LDS: 2 buffers x (A 256x64 + W 256x64)
// bf16 = 128 KiB, the chunk XOR swizzle of gemm_bf16_kernel, staged by LDS-DMA (each wave
// moves 64 rows of A and 64 rows of W per K-tile: 16 x 1 KiB). K-tile T = two 32-deep halves:
//   half 0: ds_read the kk=1 fragments of T (F1) | 64 MFMAs on F0 (kk=0 of T)
//   lgkmcnt(0) + vmcnt(0) (T+1 landed) + s_barrier     <- the only barrier of the K-tile
//   half 1: LDS-DMA T+2 into T's buffer; ds_read F0 = kk=0 of T+1 | 64 MFMAs on F1
// so the fragments a half multiplies were read during the previous half, and the barrier
// never leaves the matrix pipe without queued work beyond its own skew.
// VAR bits: 1 = stagger-U (workgroup t starts its K loop at K-tile t % 8 and wraps: the
// concurrent workgroups of a wave of the grid spread over memory channels), 8 / 16 = grouped
// tile order (GM 4 / 8 tile-rows per group, as gemm8p), 2 = all 16 next-half reads up front,
// 4 = all 16 LDS-DMA pieces of a K-tile up front (default: one per 4 MFMAs), 32 = deep W
// ring (3 W stages), 1024 = register staging, 2048 = sc1 loads, 4096 = the two-barrier K-tile
// (ktile2 below; tile 45, the default 4-wave tile), 8192 / 16384 = its other barrier
// placements, 32768 = column-major MFMA order, 65536 = per-piece voffset addressing.
// Diagnostics only: 64 = no LDS-DMA in the K loop, 128 = also no barrier / waits (wrong
// results, timing of the remaining work), 131072 = s_memtime stamps (correct results).
// Only tiles 34 (VAR 8), 41 (8 | 32) and 45 (8 | 4096) are built by default; the rest with
// DLI_GEMM_AB=1 (measurements: profiles/r4/gemm4w/).
template <int EPI, int VAR = 0>
__global__ void __launch_bounds__(256, 1) gemm4w_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws, const int* __restrict__ group_off) {
  constexpr int BM = 256, BN = 256;
  constexpr int A_BYTES = BM * BK * 2, BUF = 2 * A_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int row0 = 0, Mg = M;
  const u16* Wg = W;
  if (group_off != nullptr) {
    row0 = group_off[blockIdx.z];
    Mg = group_off[blockIdx.z + 1] - row0;
    Wg = W + (long)blockIdx.z * N * ldw;
  }
  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = (N + BN - 1) / BN;
  int tile, ks;
  split_tile(tiles_m * tiles_n, group_off != nullptr, tile, ks);
  int tn, tm;
  constexpr int GM = (VAR & 8) ? 4 : (VAR & 16) ? 8 : 1;
  if (GM > 1) {
    const int per_group = GM * tiles_n;
    const int first_m = (tile / per_group) * GM;
    const int gsz = min(tiles_m - first_m, GM);
    const int in_g = tile % per_group;
    tm = first_m + in_g % gsz;
    tn = in_g / gsz;
  } else {
    tn = tile / tiles_m;
    tm = tile % tiles_m;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mg) return;
  const int kb = ks * k_split_len;
  const int nk = min(k_split_len, K - kb) / BK;
  const int kst = (VAR & 1) ? (tile & 7) % max(nk, 1) : 0;   // stagger-U start K-tile
  const u16* Ab = A + (long)row0 * lda;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  // ---- staging by buffer LDS-DMA: piece i (0..7) of A / W = rows 64 wid + 8 i + lane / 8 of
  // the tile, swizzled chunk (lane & 7) ^ ((row >> 1) & 7) = (lane & 7) ^ ((lane >> 4) + 4 i)
  // & 7: only the parity of i changes the lane's offset, the rest is the scalar soffset
  // i * 8 rows + K-tile. Rows past the matrix read as zeros (buffer range check) instead of
  // needing a clamped address per row, so a lane keeps 4 offset VGPRs, not 16 pointers.
  // (the descriptors are built inside buf_lds16: a lambda capturing an
  // __amdgpu_buffer_rsrc_t made hipcc drop the kernel's host-side handle)
  const u16* a_base = Ab + (long)m0 * lda;
  const u16* w_base = Wg + (long)n0 * ldw;
  const int a_bytes = min(Mg - m0, BM) * lda * 2, w_bytes = min(N - n0, BN) * ldw * 2;
  const int prow = 64 * wid + (lane >> 3);
  const int ce = (lane & 7) ^ ((lane >> 4) & 7), co = (lane & 7) ^ (((lane >> 4) + 4) & 7);
  const int a_off[2] = {prow * lda * 2 + (kb + ce * 8) * 2, prow * lda * 2 + (kb + co * 8) * 2};
  const int w_off[2] = {prow * ldw * 2 + (kb + ce * 8) * 2, prow * ldw * 2 + (kb + co * 8) * 2};
  // LDS: 2 stages of {A 256x64, W 256x64} (128 KiB); with VAR 32 ("deep W") 2 A stages and
  // 3 W stages (160 KiB, the whole LDS): the weight panel, which a decode-sized GEMM streams
  // from HBM while A is L2-resident, is fetched one K-tile further ahead (a CU's stream rate
  // is its bytes in flight over the loaded memory latency)
  constexpr bool DEEP = (VAR & 32) != 0;
  auto abase = [&](int kt) -> char* {
    return DEEP ? smem + (kt & 1) * A_BYTES : smem + (kt & 1) * BUF;
  };
  auto wbase = [&](int kt, int ws) -> char* {      // ws = kt % 3 (DEEP)
    return DEEP ? smem + 2 * A_BYTES + ws * A_BYTES : smem + (kt & 1) * BUF + A_BYTES;
  };
  auto kpos = [&](int kt) {                        // stagger-U: physical K-tile of logical kt
    const int kp = kt + kst;
    return kp >= nk ? kp - nk : kp;
  };
  // one 1-KiB piece f (0..15: A pieces 0-7 of K-tile ka, W pieces 8-15 of K-tile kw into W
  // slot ws); a negative K-tile skips its pieces
  constexpr int CPOL = (VAR & 2048) ? 16 : 0;
  // VAR 65536 (VOFF, the library kernel's addressing): every piece keeps its whole byte
  // offset in its own VGPR (16 per lane) and the K-tile advances the descriptor's base
  // (SALU, once per K-tile and operand) instead of a per-piece soffset SGPR
  constexpr bool VOFF = (VAR & 65536) != 0;
  int va[8], vw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    va[i] = VOFF ? a_off[i & 1] + i * 16 * lda : 0;
    vw[i] = VOFF ? w_off[i & 1] + i * 16 * ldw : 0;
  }
  auto stage_piece = [&](int ka, int kw, int ws, int f) {
    const int i = f & 7;
    if (VOFF) {
      if (f < 8) {
        if (ka >= 0) {
          const int kp = kpos(ka) * BK;
          buf_lds16<CPOL>(a_base + kp, a_bytes - kp * 2, abase(ka) + (64 * wid + 8 * i) * 128,
                          va[i], 0);
        }
      } else if (kw >= 0) {
        const int kp = kpos(kw) * BK;
        buf_lds16<CPOL>(w_base + kp, w_bytes - kp * 2, wbase(kw, ws) + (64 * wid + 8 * i) * 128,
                        vw[i], 0);
      }
      return;
    }
    if (f < 8) {
      if (ka >= 0)
        buf_lds16<CPOL>(a_base, a_bytes, abase(ka) + (64 * wid + 8 * i) * 128, a_off[i & 1],
                        i * 16 * lda + kpos(ka) * (BK * 2));
    } else if (kw >= 0) {
      buf_lds16<CPOL>(w_base, w_bytes, wbase(kw, ws) + (64 * wid + 8 * i) * 128, w_off[i & 1],
                      i * 16 * ldw + kpos(kw) * (BK * 2));
    }
  };
  auto stage = [&](int ka, int kw, int ws) {
#pragma unroll
    for (int f = 0; f < 16; ++f) stage_piece(ka, kw, ws, f);
  };
  // VAR 1024 (register staging): piece f of K-tile k is loaded into stg[f] (buffer_load to
  // VGPRs, 64 per lane for a K-tile) and later written to LDS with one ds_write_b128 — the
  // load / write pair issues in a fraction of an LDS-DMA's cost among MFMAs with ONE wave
  // per SIMD (no partner wave hides the DMA issue, as the 8-wave ping-pong does)
  constexpr bool RS = (VAR & 1024) != 0;
  uint4 stg[16];
  auto rs_load = [&](int k, int f) {
    const int i = f & 7;
    if (f < 8) stg[f] = buf_ld16(a_base, a_bytes, a_off[i & 1], i * 16 * lda + kpos(k) * (BK * 2));
    else stg[f] = buf_ld16(w_base, w_bytes, w_off[i & 1], i * 16 * ldw + kpos(k) * (BK * 2));
  };
  auto rs_write = [&](int k, int f) {
    const int i = f & 7;
    char* dst = (f < 8 ? abase(k) : wbase(k, 0)) + (64 * wid + 8 * i) * 128 + lane * 16;
    *reinterpret_cast<uint4*>(dst) = stg[f];
  };

  const int fr = lane & 15, fq = lane >> 4;
  auto read_frag = [&](const char* part, int row, int kk) -> bf16x8 {
    const int c = kk * 4 + fq;
    return *reinterpret_cast<const bf16x8*>(part + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  };
  const int arow = wm * 128 + fr, wrow = wn * 128 + fr;

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  // one 32-deep half: 64 MFMAs on (acur, bcur) while the next half's 16 fragments are read
  // from (na, nw) into (anext, bnext). The MFMAs are inline asm with the accumulator pinned to
  // the AGPR file ("+a"): with 256 accumulators per lane the compiler's own MFMA selection
  // bounced them between VGPRs and AGPRs (1,000+ v_accvgpr moves per K-tile). hipcc pads no
  // hazard inside an asm statement (cdna_hip_programming.md §5.7): the fragments come from
  // ds_reads, whose completion hipcc waits for by register (lgkmcnt) before each statement;
  // an accumulator is read only as the next MFMA's C (no wait states) until the drain after
  // the loop. ka / kw >= 0: this half also stages those K-tiles, one LDS-DMA piece after
  // every 4th MFMA (16 pieces issued back to back held the matrix pipe for several hundred
  // cycles: an LDS-DMA issue costs ~60 cycles among MFMAs, MI355X_MICROARCH.md constants).
  auto half = [&](const bf16x8 (&acur)[8], const bf16x8 (&bcur)[8], bf16x8 (&anext)[8],
                  bf16x8 (&bnext)[8], const char* na, const char* nw, int nkk, bool more,
                  int ka, int kw, int ws, int rw = -1, int rl = -1)
      __attribute__((always_inline)) {
    if ((VAR & 2) && more) {                       // A/B: all 16 reads up front
#pragma unroll
      for (int i = 0; i < 8; ++i) anext[i] = read_frag(na, arow + 16 * i, nkk);
#pragma unroll
      for (int j = 0; j < 8; ++j) bnext[j] = read_frag(nw, wrow + 16 * j, nkk);
    }
    const bool dma = !(VAR & 4) && (ka >= 0 || kw >= 0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[i][j]) : "v"(bcur[j]), "v"(acur[i]));
        const int q = 8 * i + j;
        if (dma && (q & 3) == 1) {
          stage_piece(ka, kw, ws, q >> 2);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (RS && rw >= 0 && (q & 3) == 1) {        // write piece of rw, reload it with rl
          rs_write(rw, q >> 2);
          if (rl >= 0) rs_load(rl, q >> 2);
          __builtin_amdgcn_sched_barrier(0);
        }
        // one next-half fragment read after every 4th MFMA, pinned in place (the scheduler
        // hoisted all 16 above the first MFMA, whose lgkmcnt then waited on 2 of them), in
        // the order the next half consumes them: A0, B0..B7, A1..A7
        if (!(VAR & 2) && more && (q & 3) == 3) {
          const int f = q >> 2;
          if (f >= 1 && f <= 8) bnext[f - 1] = read_frag(nw, wrow + 16 * (f - 1), nkk);
          else { const int ia = f == 0 ? 0 : f - 8; anext[ia] = read_frag(na, arow + 16 * ia, nkk); }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
  };

  // ---- prologue. Plain: K-tiles 0 and 1 in flight. DEEP: A 0-1 and W 0-2 (issue order A0 W0
  // A1 W1 W2). Then the kk=0 fragments of K-tile 0 in registers.
  if (RS) {                                        // K-tiles 0, 1 into LDS, 2 in registers
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k < nk) {
#pragma unroll
        for (int f = 0; f < 16; ++f) rs_load(k, f);
#pragma unroll
        for (int f = 0; f < 16; ++f) rs_write(k, f);
      }
    }
    if (nk > 2) {
#pragma unroll
      for (int f = 0; f < 16; ++f) rs_load(2, f);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0): the writes landed
    barrier();
  } else {
    if (nk > 0) stage(0, 0, 0);
    if (nk > 1) stage(1, 1, 1);
    if (DEEP && nk > 2) stage(-1, 2, 2);
    if (DEEP && nk > 2) wait_vmcnt<24>();
    else if (nk > 1) wait_vmcnt<16>();
    else wait_vmcnt<0>();
    barrier();
  }
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  if (nk > 0 && (VAR & 32768)) {                   // column-major MFMA order (JM below)
    b0[0] = read_frag(wbase(0, 0), wrow, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = read_frag(abase(0), arow + 16 * i, 0);
#pragma unroll
    for (int j = 1; j < 8; ++j) b0[j] = read_frag(wbase(0, 0), wrow + 16 * j, 0);
  } else if (nk > 0) {
    a0[0] = read_frag(abase(0), arow, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) b0[j] = read_frag(wbase(0, 0), wrow + 16 * j, 0);
#pragma unroll
    for (int i = 1; i < 8; ++i) a0[i] = read_frag(abase(0), arow + 16 * i, 0);
  }

  // one K-tile; SA / SW (compile-time, so no branch sits inside an MFMA sequence): restage
  // A (K-tile kt + 2) / W (kt + 2, DEEP: kt + 3) during its second half
  int wsl = 0;                                      // W slot of kt (DEEP: kt % 3)
  auto ktile = [&](auto SA, auto SW, int kt) __attribute__((always_inline)) {
    constexpr bool sa = decltype(SA)::value, sw = decltype(SW)::value;
    const int ws1 = wsl == 2 ? 0 : wsl + 1;
    const char* ab = abase(kt);
    const char* wb = wbase(kt, wsl);
    // half 0: MFMAs on kk=0 of kt, reading kk=1 of kt
    half(a0, b0, a1, b1, ab, wb, 1, true, -1, -1, 0);
    // every wave's reads of these buffers retired; K-tile kt+1 landed for every wave: the
    // only younger DMAs may be DEEP's W of kt+2 (issued last in the previous K-tile)
    if (!(VAR & 128)) {
      __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0), seen by hipcc's counters
      if (RS) {
      } else if (DEEP && kt + 2 < nk) {
        wait_vmcnt<8>();
      } else {
        wait_vmcnt<0>();
      }
      barrier();
    }
    // half 1: MFMAs on kk=1 of kt, reading kk=0 of kt+1; restage kt's buffers (register
    // staging: write K-tile kt+2 from the registers, reload them with kt+3)
    const int ka = (sa && !(VAR & 64)) ? kt + 2 : -1;
    const int kw = (sw && !(VAR & 64)) ? kt + (DEEP ? 3 : 2) : -1;
    if (RS) {
      half(a1, b1, a0, b0, abase(kt + 1), wbase(kt + 1, ws1), 0, true, -1, -1, 0,
           sa ? kt + 2 : -1, sw ? kt + 3 : -1);
    } else {
      if ((VAR & 4) && (ka >= 0 || kw >= 0)) stage(ka, kw, wsl);
      half(a1, b1, a0, b0, abase(kt + 1), wbase(kt + 1, ws1), 0, true,
           (VAR & 4) ? -1 : ka, (VAR & 4) ? -1 : kw, wsl);
    }
    wsl = ws1;
  };
  // VAR 4096 ("two barriers", the buffer-release point moved forward): one K-tile = 128
  // MFMAs, 64 on F0 (kk=0, read during the previous K-tile) then 64 on F1:
  //   MFMAs 0-15: one F1(kt) fragment read after each        | frees buffer kt early
  //   after MFMA 19: lgkmcnt(0) + s_barrier (B1: every wave has read buffer kt)
  //   MFMAs 20-95: LDS-DMA of K-tile kt+2 into buffer kt, one piece per 5 MFMAs
  //   after MFMA 103: vmcnt(16) (K-tile kt+1 landed; kt+2 may fly) + s_barrier (B2)
  //   MFMAs 104-119: one F0(kt+1) fragment read after each
  // The DMA of kt+2 starts ~45 MFMAs earlier than in the one-barrier schedule and is waited
  // for ~1.5 K-tiles later (hides ~2,400 cycles of HBM latency instead of ~1,000-2,000),
  // and 16 DMAs spread over 80 MFMAs instead of 64. Plain (2-stage) ring only.
  constexpr bool TWO_B = (VAR & 4096) != 0;
  // With DEEP (3 W stages) the DMA of this K-tile is A(kt+2) and W(kt+3), both into kt's
  // slots; B2 may leave the previous tile's W pieces in flight too (vmcnt 24).
  static_assert(!(TWO_B && RS), "two-barrier schedule: LDS-DMA staging only");
  // SA / SW: this K-tile stages A(kt+2) / W(kt+2, DEEP: kt+3); PW: the previous K-tile
  // staged W (DEEP: its pieces may still fly at B2)
  // VAR 131072 (STAMP, diagnostic build only): s_memtime stamps around the two barriers and
  // the DMA window, summed over the K loop per segment and written by each workgroup's
  // first lane to the workspace (read the SHARES: every stamp drains the LDS reads)
  constexpr bool STAMP = (VAR & 131072) != 0;
  unsigned long long sseg[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long st_prev = 0;
  auto stamp = [&]() __attribute__((always_inline)) -> unsigned long long {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
  };
  auto mark = [&](int seg) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const unsigned long long t = stamp();
      sseg[seg] += t - st_prev;
      st_prev = t;
    }
  };
  auto ktile2 = [&](auto SA, auto SW, auto PW, bool more, int kt)
      __attribute__((always_inline)) {
    if constexpr (STAMP) st_prev = stamp();
    constexpr bool sa = decltype(SA)::value, sw = decltype(SW)::value;
    constexpr bool pw = DEEP && decltype(PW)::value;
    constexpr bool sd = sa || sw;
    const int ws1 = wsl == 2 ? 0 : wsl + 1;
    const char* ab = abase(kt);
    const char* wb = wbase(kt, wsl);
    const char* nab = abase(kt + 1);
    const char* nwb = wbase(kt + 1, ws1);
    // B1 / B2 positions: default 19 / 103; VAR 8192: 25 / 111; VAR 16384: 25 / after the
    // last MFMA with the 16 F0(kt+1) reads in one burst (the library kernel's placement)
    constexpr int QB1 = (VAR & (8192 | 16384)) ? 25 : 19;
    constexpr int QB2 = (VAR & 8192) ? 111 : (VAR & 16384) ? 127 : 103;
    // VAR 32768 (JM): MFMAs column-major within a half (acc[i][j] with j outer), so the
    // weight fragment — MFMA operand A — stays the same for 8 consecutive MFMAs (the
    // library kernel's order); fragment f of a half is then read in the order B0, A0..A7,
    // B1..B7 instead of A0, B0..B7, A1..A7
    constexpr bool JM = (VAR & 32768) != 0;
    auto read_fx = [&](int f, bf16x8 (&av)[8], bf16x8 (&bv)[8], const char* pa, const char* pw,
                       int kk) __attribute__((always_inline)) {
      if (JM) {
        if (f >= 1 && f <= 8) av[f - 1] = read_frag(pa, arow + 16 * (f - 1), kk);
        else { const int jb = f == 0 ? 0 : f - 8; bv[jb] = read_frag(pw, wrow + 16 * jb, kk); }
      } else {
        if (f >= 1 && f <= 8) bv[f - 1] = read_frag(pw, wrow + 16 * (f - 1), kk);
        else { const int ia = f == 0 ? 0 : f - 8; av[ia] = read_frag(pa, arow + 16 * ia, kk); }
      }
    };
    auto read_f0 = [&](int f) __attribute__((always_inline)) { read_fx(f, a0, b0, nab, nwb, 0); };
    auto step = [&](int q) __attribute__((always_inline)) {
      if (q < 16) {                                // F1(kt)
        read_fx(q, a1, b1, ab, wb, 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (q == QB1 && !(VAR & 128)) {
        mark(0);                                   // MFMAs 0..QB1 + the F1 reads
        __builtin_amdgcn_s_waitcnt(0xC07F);        // lgkmcnt(0)
        barrier();
        mark(1);                                   // B1
      }
      if (q == QB1 + 80) mark(2);                  // the DMA window
      if (sd && !(VAR & 64) && q > QB1 && q <= QB1 + 80 && (q - QB1 - 1) % 5 == 0) {
        stage_piece(sa ? kt + 2 : -1, sw ? kt + (DEEP ? 3 : 2) : -1, wsl, (q - QB1 - 1) / 5);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (q == QB2 && more && !(VAR & 128)) {
        mark(3);                                   // MFMAs after the DMA window
        constexpr int fly = (VAR & 64) ? 0 : 8 * ((sa ? 1 : 0) + (sw ? 1 : 0) + (pw ? 1 : 0));
        wait_vmcnt<fly>();
        barrier();
        mark(4);                                   // B2
      }
      if (q == 127) mark(5);                       // MFMAs after B2 + the F0 reads
      if (more) {                                  // F0(kt+1)
        if (QB2 == 127) {
          if (q == 127) {
#pragma unroll
            for (int f = 0; f < 16; ++f) read_f0(f);
            __builtin_amdgcn_sched_barrier(0);
          }
        } else if (q > QB2 && q <= QB2 + 16) {
          read_f0(q - QB2 - 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const int i = JM ? v : u, j = JM ? u : v;
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[i][j]) : "v"(b0[j]), "v"(a0[i]));
        step(8 * u + v);
      }
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const int i = JM ? v : u, j = JM ? u : v;
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[i][j]) : "v"(b1[j]), "v"(a1[i]));
        step(64 + 8 * u + v);
      }
  };

  using T_ = std::integral_constant<bool, true>;
  using F_ = std::integral_constant<bool, false>;
  int kt = 0;
  if (TWO_B && DEEP) {
    for (; kt + 3 < nk; ++kt) { ktile2(T_{}, T_{}, T_{}, true, kt); wsl = wsl == 2 ? 0 : wsl + 1; }
    if (kt + 2 < nk) { ktile2(T_{}, F_{}, T_{}, true, kt); wsl = wsl == 2 ? 0 : wsl + 1; ++kt; }
    for (; kt < nk; ++kt) { ktile2(F_{}, F_{}, F_{}, kt + 1 < nk, kt); wsl = wsl == 2 ? 0 : wsl + 1; }
  } else if (TWO_B) {
    for (; kt + 2 < nk; ++kt) ktile2(T_{}, T_{}, F_{}, true, kt);
    for (; kt < nk; ++kt) ktile2(F_{}, F_{}, F_{}, kt + 1 < nk, kt);
  } else if (DEEP || RS) {                         // RS: SA = write kt+2, SW = load kt+3
    for (; kt + 3 < nk; ++kt) ktile(T_{}, T_{}, kt);
    if (kt + 2 < nk) { ktile(T_{}, F_{}, kt); ++kt; }
  } else {
    for (; kt + 2 < nk; ++kt) ktile(T_{}, T_{}, kt);
  }
  if (!TWO_B) {
    if (kt + 1 < nk) { ktile(F_{}, F_{}, kt); ++kt; }
    if (nk > 0) {
      half(a0, b0, a1, b1, abase(kt), wbase(kt, wsl), 1, true, -1, -1, 0);
      half(a1, b1, a0, b0, smem, smem, 0, false, -1, -1, 0);
    }
  }
  // MFMA results -> any other reader: the XDL write-back wait states (§5.7 item 2), tied to
  // the last row of accumulators written so that no copy of them is hoisted above the pad
  if constexpr ((VAR & 32768) != 0) {              // column-major order: column 7 is last
    asm volatile("s_nop 15\n\ts_nop 15"
                 : "+a"(acc[0][7]), "+a"(acc[1][7]), "+a"(acc[2][7]), "+a"(acc[3][7]),
                   "+a"(acc[4][7]), "+a"(acc[5][7]), "+a"(acc[6][7]), "+a"(acc[7][7]));
  } else {
    asm volatile("s_nop 15\n\ts_nop 15"
                 : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]),
                   "+a"(acc[7][4]), "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));
  }
  // accumulators leave the AGPR file by one pinned copy each, ahead of any row / column
  // condition (an AGPR value read inside a divergent branch made hipcc move the whole
  // accumulator set through VGPRs in the K loop)
  auto vget = [&](const f32x4& a) -> f32x4 {
    f32x4 v;
    asm volatile("" : "=v"(v) : "0"(a));
    return v;
  };

  // ---- epilogue (transposed accumulators):
  // acc[I][J][r] = C[m0 + 128 wm + 16I + fr][n0 + 128 wn + 16J + 4fq + r]
  if constexpr (STAMP) {
    if (threadIdx.x == 0 && ws != nullptr) {
      unsigned long long* o = reinterpret_cast<unsigned long long*>(ws) + (long)blockIdx.x * 8;
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k] = sseg[k];
      o[6] = (unsigned long long)nk;
    }
  }
  const int wr0 = m0 + 128 * wm, wc0 = n0 + 128 * wn;
  if (gridDim.y > 1) {
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr0 + 16 * i + fr;
      float* srow = slab + (long)(row0 + min(row, Mg - 1)) * N;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const f32x4 v = vget(acc[i][j]);
        const int col = wc0 + 16 * j + 4 * fq;
        if (row < Mg && col < N) slab_quad(srow + col, v, sm, vec, N - col);
      }
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr0 + 16 * i + fr;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const f32x4 g = vget(acc[i][j]), u = vget(acc[i][j + 1]);
        const int gcol = wc0 + 16 * j;
        if (row < Mg && gcol < N)
          store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, g, u, vec);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wr0 + 16 * i + fr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 v = vget(acc[i][j]);
      const int col = wc0 + 16 * j + 4 * fq;
      if (row < Mg && col < N) store_quad<EPI>(C, ldc, row0 + row, col, N, v, bias, vec);
    }
  }
}

// split-K reduction + epilogue: one thread per output element group of 4 columns
template <int EPI>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(void* __restrict__ C, int ldc,
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

template <int BM, int BN, int EPI, int NS, int WM = 2, int WN = 2>
static int launch_cfg(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                      int N, int K, int splits, const void* bias, void* ws,
                      const int* group_off, int groups, hipStream_t st) {
  if (EPI == EPI_SILU && (BN / WN) % 32) return (int)hipErrorInvalidValue;  // gate/up pairs
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int ksl = K / splits;
  ksl = (ksl / BK) * BK;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  const size_t lds = NS * (size_t)(BM + BN) * BK * 2;
  static bool attr_done = false;                   // > 64 KiB dynamic LDS needs the opt-in
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm_bf16_kernel<BM, BN, EPI, NS, WM, WN>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  dim3 grid(tiles, splits, groups);
  gemm_bf16_kernel<BM, BN, EPI, NS, WM, WN><<<grid, 64 * WM * WN, lds, st>>>(
      (const u16*)A, lda, (const u16*)W, ldw, C, ldc, M, N, K, ksl, (const u16*)bias,
      (float*)ws, group_off);
  if (splits > 1 && C != nullptr) {       // C == nullptr: leave the fp32 partial slabs for a
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;   // fused consumer (fused_reduce.hip)
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

// measured on MI355X (scripts/bench_gemm8p.py, profiles/r1_gemm8p/, profiles/r2_s2/): grouped
// tile order (+6-14 % on prefill shapes), a static priority for waves 4-7 (+1.5-5 %) over
// per-cluster flips, and one counted vmcnt per K-tile instead of one per phase (VAR 512:
// +6 % on prefill shapes, +6-11 % on the decode gate/up, down and LM head); the
// deep-prefetch plan (VAR 4) and glds-before-ds_read order measured slower / equal, and so
// (within 1 %, profiles/r2_s2/gemm8p_wait/variants.log) did the template's B-before-A read
// order, an lgkmcnt(0) after the barrier and per-cluster priority flips
constexpr int GEMM8P_DEFAULT = 8 | 256 | 512;
constexpr int GEMM8P_PER_PHASE_WAITS = 8 | 256;     // round-1 schedule (tile 27, for A/Bs)

template <int EPI, int VAR = 0>
static int launch_8p(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                     int N, int K, int splits, const void* bias, void* ws, const int* group_off,
                     int groups, hipStream_t st) {
  if (EPI == EPI_SILU && N % 64) return (int)hipErrorInvalidValue;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  int ksl = K / splits;
  ksl = (ksl / BK) * BK;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  constexpr size_t lds = 2 * (size_t)(256 + 256) * BK * 2;
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm8p_kernel<EPI, VAR>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  dim3 grid(tiles, splits, groups);
  gemm8p_kernel<EPI, VAR><<<grid, 512, lds, st>>>((const u16*)A, lda, (const u16*)W, ldw, C, ldc, M,
                                             N, K, ksl, (const u16*)bias, (float*)ws, group_off);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI>
static int launch_8p224(const void* A, int lda, const void* W, int ldw, void* C, int ldc,
                        int M, int N, int K, int splits, const void* bias, void* ws,
                        const int* group_off, int groups, hipStream_t st) {
  if (EPI == EPI_SILU && N % 32) return (int)hipErrorInvalidValue;
  const int tiles = ((M + 255) / 256) * ((N + 223) / 224);
  int ksl = K / splits;
  ksl = (ksl / BK) * BK;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  constexpr size_t lds = 2 * (size_t)(256 + 256) * BK * 2;
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm8p224_kernel<EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  dim3 grid(tiles, splits, groups);
  gemm8p224_kernel<EPI><<<grid, 512, lds, st>>>((const u16*)A, lda, (const u16*)W, ldw, C, ldc,
                                                M, N, K, ksl, (const u16*)bias, (float*)ws,
                                                group_off);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI>
static int launch_8p128(const void* A, int lda, const void* W, int ldw, void* C, int ldc,
                        int M, int N, int K, int splits, const void* bias, void* ws,
                        const int* group_off, int groups, hipStream_t st) {
  if (EPI == EPI_SILU && N % 32) return (int)hipErrorInvalidValue;
  const int tiles = ((M + 255) / 256) * ((N + 127) / 128);
  int ksl = K / splits;
  ksl = (ksl / BK) * BK;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  constexpr size_t lds = 2 * (size_t)(256 + 128) * BK * 2;
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm8p128_kernel<EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  dim3 grid(tiles, splits, groups);
  gemm8p128_kernel<EPI><<<grid, 512, lds, st>>>((const u16*)A, lda, (const u16*)W, ldw, C, ldc,
                                                M, N, K, ksl, (const u16*)bias, (float*)ws,
                                                group_off);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI, int VAR>
static int launch_4w(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                     int N, int K, int splits, const void* bias, void* ws, const int* group_off,
                     int groups, hipStream_t st) {
  if (EPI == EPI_SILU && N % 32) return (int)hipErrorInvalidValue;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  int ksl = K / splits;
  ksl = (ksl / BK) * BK;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  constexpr size_t lds = ((VAR & 32) ? 5 : 4) * (size_t)256 * BK * 2;
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm4w_kernel<EPI, VAR>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  dim3 grid(tiles, splits, groups);
  gemm4w_kernel<EPI, VAR><<<grid, 256, lds, st>>>((const u16*)A, lda, (const u16*)W, ldw, C,
                                                  ldc, M, N, K, ksl, (const u16*)bias,
                                                  (float*)ws, group_off);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

// ---------------------------------------------------------------------------------------
// Skinny GEMM for M <= 4 rows (batch-1 / tiny-batch decode: SURVEY.md §7.4 "the decode
// skinny GEMM must approach the HBM roofline"): every weight byte is used M times, so the
// kernel is a weight stream, not an MFMA tile. A workgroup (4 waves) owns R = 4 * RW output
// rows of W over one K slice; in a wave, lane l covers the 8 K-elements [8 (l + 64 s),
// +8) of step s for its RW rows: RW 16-B nontemporal weight loads per step (the weights are
// read exactly once, MI355X_MICROARCH.md 'nt-weights'), two steps in flight, bf16 pairs
// accumulated by v_dot2c_f32_bf16 against x (M rows, L1/L2-resident). Lane partial sums
// are reduced across the wave with shuffles and staged in LDS; the epilogue then writes
// bf16 / fp32 / SiLU(gate)*up (the 16-row interleaved gate/up weight: a workgroup's 32 rows
// are 16 gate + 16 up features) or fp32 split-K slabs for the fused reduces. No MFMA, no
// LDS tiles, no padding rows: bytes moved = weights + M * K * 2 + outputs.
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

// bf16 pairs by __builtin_shufflevector: a __builtin_bit_cast of one element of a uint
// ext-vector was compiled (ROCm 7.2 clang) into the FIRST element for every lane pair
__device__ __forceinline__ float dot8_acc(const bf16x8v w, const bf16x8v x, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 0, 1),
                                        __builtin_shufflevector(x, x, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 2, 3),
                                        __builtin_shufflevector(x, x, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 4, 5),
                                        __builtin_shufflevector(x, x, 4, 5), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 6, 7),
                                        __builtin_shufflevector(x, x, 6, 7), acc, false);
  return acc;
}

// The weight stream of one workgroup: res[m][wid * RW + r] = sum over this K slice of
// A[m, :] . W[r0 + r, :] (r < RW), reduced across the wave and staged in LDS.
template <int MB, int RW, int UNROLL>
__device__ __forceinline__ void gemv_core(const u16* __restrict__ A, int lda,
                                          const u16* __restrict__ W, int ldw, int M, int N,
                                          int K, int k_split_len, int r0, int ks,
                                          float (&res)[MB][4 * RW]) {
  // r0: this wave's first weight row (rows r0 .. r0 + RW - 1 land in res[.][wid * RW ..])
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kb = ks * k_split_len;
  const int klen = min(k_split_len, K - kb);
  const int nchunk = klen >> 3;                     // 8-element chunks of the K slice
  const bf16x8v* wrow[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int n = min(r0 + r, N - 1);
    wrow[r] = reinterpret_cast<const bf16x8v*>(W + (long)n * ldw + kb);
  }
  const bf16x8v* xrow[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m)
    xrow[m] = reinterpret_cast<const bf16x8v*>(A + (long)min(m, M - 1) * lda + kb);
  float acc[MB][RW];
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[m][r] = 0.f;
  int c = lane;
  // UNROLL 64-chunk steps per iteration: UNROLL * RW weight loads in flight per lane (the
  // short projections of a batch-1 layer run only a few iterations, so depth, not
  // occupancy, hides the HBM latency)
  for (; c + 64 * (UNROLL - 1) < nchunk; c += 64 * UNROLL) {
    bf16x8v w[UNROLL][RW];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int r = 0; r < RW; ++r) w[u][r] = __builtin_nontemporal_load(wrow[r] + c + 64 * u);
#pragma unroll
    for (int m = 0; m < MB; ++m) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const bf16x8v xv = xrow[m][c + 64 * u];
#pragma unroll
        for (int r = 0; r < RW; ++r) acc[m][r] = dot8_acc(w[u][r], xv, acc[m][r]);
      }
    }
  }
  for (; c < nchunk; c += 64) {
    bf16x8v w0[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) w0[r] = __builtin_nontemporal_load(wrow[r] + c);
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      const bf16x8v x0 = xrow[m][c];
#pragma unroll
      for (int r = 0; r < RW; ++r) acc[m][r] = dot8_acc(w0[r], x0, acc[m][r]);
    }
  }
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const float v = wave_sum(acc[m][r]);
      if (lane == 0) res[m][wid * RW + r] = v;
    }
}

// H16 (SiLU*up only, RW = 4): 16 rows per workgroup as 8 gate + 8 up rows of one 32-row
// gate/up block (waves 0-1 the gate half h, waves 2-3 the matching up half), so the pairing
// runs at the 16-row grid (2x the workgroups of the 32-row tile; profiles/r4/b1/)
template <int MB, int RW, int EPI, int UNROLL, bool H16 = false>
__global__ void __launch_bounds__(256) gemv_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws) {
  constexpr int R = 4 * RW;
  static_assert(!H16 || (EPI == EPI_SILU && RW == 4), "H16 pairs 8 gate + 8 up rows");
  __shared__ float res[MB][R];
  const int n_base = blockIdx.x * R;
  const int ks = blockIdx.y;
  const int wid = threadIdx.x >> 6;
  const int blk = blockIdx.x >> 1, half = blockIdx.x & 1;
  // weight row of res column j
  auto row_of = [&](int j) {
    return H16 ? blk * 32 + (j < 8 ? half * 8 + j : 16 + half * 8 + (j - 8)) : n_base + j;
  };
  gemv_core<MB, RW, UNROLL>(A, lda, W, ldw, M, N, K, k_split_len, row_of(wid * RW), ks, res);
  __syncthreads();
  // epilogue: one thread per (row m, output column)
  if (ws != nullptr && gridDim.y > 1) {             // fp32 partial slab of this K slice
    for (int t = threadIdx.x; t < MB * R; t += 256) {
      const int m = t / R, j = t % R, n = row_of(j);
      if (m < M && n < N) ws[((long)ks * M + m) * N + n] = res[m][j];
    }
    return;
  }
  if (H16) {                                        // res 0-7 gate, 8-15 the matching up
    for (int t = threadIdx.x; t < MB * 8; t += 256) {
      const int m = t / 8, j = t % 8;
      const int f = blk * 16 + half * 8 + j;
      if (m < M && blk * 32 < N)
        ((u16*)C)[(long)m * ldc + f] = f2bf(silu_f(res[m][j]) * res[m][j + 8]);
    }
    return;
  }
  if (EPI == EPI_SILU) {                            // R = 32: rows 0-15 gate, 16-31 up
    for (int t = threadIdx.x; t < MB * 16; t += 256) {
      const int m = t / 16, j = t % 16;
      const int f = (n_base >> 5) * 16 + j;
      if (m < M && n_base + j < N)
        ((u16*)C)[(long)m * ldc + f] = f2bf(silu_f(res[m][j]) * res[m][j + 16]);
    }
    return;
  }
  for (int t = threadIdx.x; t < MB * R; t += 256) {
    const int m = t / R, j = t % R, n = n_base + j;
    if (m < M && n < N) store_pair_or_one<EPI>(C, ldc, m, n, res[m][j], bias);
  }
}

template <int MB, int RW, int EPI, int UNROLL = 2, bool H16 = false>
static int launch_gemv(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                       int N, int K, int splits, const void* bias, void* ws, hipStream_t st) {
  constexpr int R = 4 * RW;
  if (M > MB || (EPI == EPI_SILU && ((R != 32 && !H16) || N % 32)) || K % 8 || lda % 8 ||
      ldw % 8)
    return (int)hipErrorInvalidValue;
  int ksl = K / splits;
  ksl = (ksl / 8) * 8;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  dim3 grid((N + R - 1) / R, splits);
  gemv_kernel<MB, RW, EPI, UNROLL, H16><<<grid, 256, 0, st>>>((const u16*)A, lda, (const u16*)W, ldw, C, ldc,
                                                 M, N, K, ksl, (const u16*)bias,
                                                 splits > 1 ? (float*)ws : nullptr);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI>
static int dispatch_gemv(int tile_cfg, const void* A, int lda, const void* W, int ldw, void* C,
                         int ldc, int M, int N, int K, int splits, const void* bias, void* ws,
                         hipStream_t st) {
  // 30: 16 rows per workgroup, 31: 32 rows (the SiLU gate/up pairing needs 32), 32: 16 rows
  // with 4 K-steps in flight per lane (M = 1)
  const bool r32 = tile_cfg == 31;
  if (tile_cfg == 32)
    return M <= 1 ? launch_gemv<1, 4, EPI, 4>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : (int)hipErrorInvalidValue;
  // 33: 32 rows (SiLU gate/up pairs) with 4 K-steps in flight per lane (M = 1): 32 weight
  // loads of 16 B outstanding per lane instead of 16 (tile 31)
  if (tile_cfg == 33)
    return M <= 1 ? launch_gemv<1, 8, EPI, 4>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : (int)hipErrorInvalidValue;
  // 29: SiLU*up gate/up on the 16-row grid (8 gate + 8 up rows per workgroup); 4 K-steps
  // in flight per lane at M = 1 (tile 32's depth), 2 at M = 2..4 (tile 30's)
  if (tile_cfg == 29) {
    if constexpr (EPI == EPI_SILU) {
      if (M <= 1) return launch_gemv<1, 4, EPI, 4, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
      if (M <= 2) return launch_gemv<2, 4, EPI, 2, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
      if (M <= 4) return launch_gemv<4, 4, EPI, 2, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    }
    return (int)hipErrorInvalidValue;
  }
  if (M <= 1)
    return r32 ? launch_gemv<1, 8, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
               : launch_gemv<1, 4, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
  if (M <= 2)
    return r32 ? launch_gemv<2, 8, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
               : launch_gemv<2, 4, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
  if (M <= 4)
    return r32 ? launch_gemv<4, 8, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
               : launch_gemv<4, 4, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
  return (int)hipErrorInvalidValue;
}

template <int EPI>
static int dispatch_tile(int tile_cfg, const void* A, int lda, const void* W, int ldw, void* C,
                         int ldc, int M, int N, int K, int splits, const void* bias, void* ws,
                         const int* go, int groups, hipStream_t st) {
  switch (tile_cfg) {
#define DLI_CFG(id, bm, bn, ns) \
    case id: return launch_cfg<bm, bn, EPI, ns>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    DLI_CFG(0, 64, 64, 2) DLI_CFG(1, 64, 128, 2) DLI_CFG(2, 128, 128, 2) DLI_CFG(3, 128, 256, 2)
    DLI_CFG(4, 256, 128, 2)
    DLI_CFG(5, 64, 64, 3) DLI_CFG(6, 64, 128, 3) DLI_CFG(7, 128, 128, 3) DLI_CFG(8, 128, 256, 3)
    DLI_CFG(9, 256, 128, 3)
    DLI_CFG(10, 192, 128, 2) DLI_CFG(11, 192, 128, 3) DLI_CFG(12, 160, 128, 2)
#define DLI_CFG8(id, bm, bn, ns, wm, wn) \
    case id: return launch_cfg<bm, bn, EPI, ns, wm, wn>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 8 waves (512 threads): 256-wide tiles halve the L2 re-reads of A/W at M >= 256
    DLI_CFG8(13, 256, 256, 2, 2, 4) DLI_CFG8(14, 256, 128, 2, 4, 2) DLI_CFG8(15, 128, 256, 2, 2, 4)
    DLI_CFG8(16, 256, 128, 3, 4, 2) DLI_CFG8(17, 128, 256, 3, 2, 4)
    // grid-filling shapes for N = 6144 / 4096 at M = 512 (4 x 64 = 256 workgroups)
    DLI_CFG(18, 128, 96, 2) DLI_CFG(19, 128, 96, 3) DLI_CFG(20, 128, 64, 2) DLI_CFG(21, 128, 64, 3)
    // 256x256 8-phase ping-pong (gemm8p_kernel)
    case 22: return launch_8p<EPI, GEMM8P_DEFAULT>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 22 with the round-1 schedule (a counted vmcnt in every phase), for A/B runs
    case 27: return launch_8p<EPI, GEMM8P_PER_PHASE_WAITS>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 192-wide tiles: N = 6144 (fused QKV) = 32 column tiles, so M = 512 fills 256 CUs with
    // 4 x 32 x split 2 (128-row) or 2 x 32 x split 4 (256-row) workgroups of 8 waves
    DLI_CFG8(23, 128, 192, 3, 2, 4) DLI_CFG8(24, 128, 192, 2, 2, 4) DLI_CFG8(25, 256, 192, 2, 4, 2)
    // 256x224 ping-pong (gemm8p224_kernel): N = 28672 gate/up at M = 512 is 256 tiles
    case 26: return launch_8p224<EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 256x128 ping-pong (gemm8p128_kernel): Mixtral grouped down (8 x 32 tiles), N = 4096 at
    // M = 512 (64 tiles x split 4)
    case 28: return launch_8p128<EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 256x256, one wave per SIMD, 128x128 wave tiles (gemm4w_kernel): 34 grouped order,
    // 41 = 34 with the deep weight ring (3 W stages, 160 KiB LDS)
    case 34: return launch_4w<EPI, 8>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 41: return launch_4w<EPI, 8 | 32>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 45 = 34 with the two-barrier schedule: the prefill autotune's 4-wave candidate
    // (sc1 loads, VAR 2048, measured neutral: profiles/r4/gemm4w/s17_*)
    case 45: return launch_4w<EPI, 8 | 4096>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
#if DLI_GEMM_AB_VARIANTS
    // diagnostic: 48 = 45 with s_memtime stamps (per-workgroup segment sums into ws;
    // scripts/stamp_gemm4w.py, profiles/r4/gemm4w/s26_stamps_tile45.jsonl)
    case 48:
      if constexpr (EPI == EPI_BF16)
        return launch_4w<EPI, 8 | 4096 | 131072>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
      return (int)hipErrorInvalidValue;
    // 47 = 45 with the library's DMA addressing (a voffset VGPR per piece, soffset 0, the
    // descriptor base advanced per K-tile): -2 % .. +0.7 % (profiles/r4/gemm4w/s25_*)
    case 47: return launch_4w<EPI, 8 | 4096 | 65536>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 46 = 45 with column-major MFMA order (weight operand reused 8x, the library's order):
    // within 0.2 % of 45 (profiles/r4/gemm4w/s23_*)
    case 46: return launch_4w<EPI, 8 | 4096 | 32768>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // two-barrier variants measured no faster than 45 (profiles/r4/gemm4w/s18_*):
    // 49 / 50: 45 with the barriers at MFMA 25 / 111, and at 25 / after the last MFMA
    case 49: return launch_4w<EPI, 8 | 4096 | 8192>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 50: return launch_4w<EPI, 8 | 4096 | 16384>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 52 / 53: 45 with 8-row-tile groups / no grouping (tile order A/B)
    case 52: return launch_4w<EPI, 16 | 4096>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 53: return launch_4w<EPI, 4096>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // 51: 45 with the deep weight ring of 41 (W of K-tile kt+3 staged during kt)
    case 51: return launch_4w<EPI, 8 | 4096 | 32>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    // A/B variants measured slower everywhere (profiles/r4/gemm4w/; built only with
    // DLI_GEMM_AB=1, each is 5 more heavy instantiations): 35 stagger-U, 36 all next-half
    // reads up front, 37 both, 42 = 41 + stagger-U, 43 register staging, 44 = 43 +
    // stagger-U, 40 the K-tile's LDS-DMA in one burst; diagnostics (wrong results): 38 no
    // LDS-DMA in the K loop, 39 also no barrier
    case 35: return launch_4w<EPI, 8 | 1>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 36: return launch_4w<EPI, 8 | 2>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 37: return launch_4w<EPI, 8 | 3>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 42: return launch_4w<EPI, 8 | 32 | 1>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 43: return launch_4w<EPI, 8 | 1024>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 44: return launch_4w<EPI, 8 | 1024 | 1>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 40: return launch_4w<EPI, 8 | 4>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 38: return launch_4w<EPI, 8 | 64>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
    case 39: return launch_4w<EPI, 8 | 64 | 128>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, groups, st);
#endif
    // skinny weight-streaming GEMM for M <= 4 (no grouped mode)
    case 29: case 30: case 31: case 32: case 33:
      if (go != nullptr) return (int)hipErrorInvalidValue;
      return dispatch_gemv<EPI>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
#undef DLI_CFG8
#undef DLI_CFG
    default: return (int)hipErrorInvalidValue;
  }
}

// tile_cfg: 0=64x64 1=64x128 2=128x128 3=128x256 4=256x128 (2 LDS stages); 5..9 = the same
// tiles with 3 LDS stages (one tile in flight across the barrier); 10/11 = 192x128 with 2/3
// stages, 12 = 160x128 (MoE experts of ~130-190 rows in one pass); 13-17 = 8-wave tiles
// 256x256, 256x128, 128x256 (2 stages) and 256x128, 128x256 (3 stages); 18/19 = 128x96 and
// 20/21 = 128x64 with 2/3 stages; 22 = 256x256 8-phase ping-pong; 23/24 = 128x192 (3/2
// stages), 25 = 256x192, 8 waves; 26 = 256x224 ping-pong; 29-33 = the M <= 4 weight
// stream (16 / 32 rows per workgroup, dispatch_gemv). ws: fp32 [splits, M, N] when splits>1.
// group_off (nullable): int[groups+1] row offsets; M is then the max rows of any group.
extern "C" int dli_gemm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                        int N, int K, int epi, int tile_cfg, int splits, const void* bias,
                        void* ws, const int* group_off, int groups, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (((tile_cfg < 29 || tile_cfg > 33) && K % BK) || lda % 8 || ldw % 8 || splits < 1)
    return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU && N % 32) return (int)hipErrorInvalidValue;
  if (splits > 1 && ws == nullptr) return (int)hipErrorInvalidValue;
  if (groups < 1) groups = 1;
  switch (epi) {
    case EPI_BF16: return dispatch_tile<EPI_BF16>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, group_off, groups, st);
    case EPI_F32: return dispatch_tile<EPI_F32>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, group_off, groups, st);
    case EPI_SILU: return dispatch_tile<EPI_SILU>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, group_off, groups, st);
    case EPI_BIAS_GELU: return dispatch_tile<EPI_BIAS_GELU>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, group_off, groups, st);
    case EPI_BIAS: return dispatch_tile<EPI_BIAS>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, group_off, groups, st);
    default: return (int)hipErrorInvalidValue;
  }
}
