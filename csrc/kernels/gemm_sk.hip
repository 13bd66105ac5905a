// Skinny full-K MFMA GEMM for decode-sized M (tile ids 60-62): C[M,N] = A[M,K] . W[N,K]^T.
//
// Why (VERDICT r4 "What's weak" 2, profiles/r5/s09/tiles.log): at M = 512 the Llama-3-8B O /
// down / QKV projections have 2-3 M outputs, i.e. ~8k per CU. A 256x256 LDS tile then needs
// split-K 8 (down: 67 MB of fp32 slabs written and re-read, 13.6 us of reduce per layer) and
// the LDS-tiled 64x128 / 128x64 tiles run at 300-570 TF: their 4 waves share each staged
// K-tile, so every K-step pays an LDS round trip and a barrier for data that only ONE wave of
// the 64x128 block actually reuses.
//
// Here a workgroup owns one BM x BN output block over its whole K range and its 4 waves split
// that range 4 ways: wave w multiplies K-quarter w of the SAME block. No operand is shared
// between waves, so nothing goes through LDS in the K loop: each lane loads its MFMA
// fragments straight from global memory (L2-served: the XCD's workgroups are consecutive
// tiles of one N panel, n-major, so a W row is fetched once per XCD and an A row once per
// workgroup column), two K-steps of loads in flight per wave, no barrier until the end.
// The 4 partial blocks are then summed through LDS (each wave sums a quarter of the rows) and
// the epilogue writes bf16 / fp32 / SiLU(gate)*up / split-K slabs.
//
// Fragment layout (v_mfma_f32_16x16x32_bf16, W as operand A: C^T blocks, gemm_common.h):
// for a 64-deep K-step lane (fq = lane / 16, fr = lane % 16) loads the 32 contiguous bytes
// k = 16 fq .. 16 fq + 15 of row fr of each 16-row block (two 16-B loads; 4 lanes cover a
// row's 128-B line), and MFMA kk (0 / 1) consumes elements 8 kk .. 8 kk + 7 of them. Both
// operands use the same k permutation, so each MFMA pair still sums the step's 64 products.
#include "gemm_common.h"

template <int BM, int BN>
constexpr size_t sk_lds_bytes() { return (size_t)4 * BM * (BN + 4) * sizeof(float); }

template <int BM, int BN, int EPI>
__global__ void __launch_bounds__(256, 1) gemm_sk_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws) {
  constexpr int MI = BM / 16, NI = BN / 16;
  constexpr int ROW = BN + 4;                       // padded LDS row of a partial block (floats)
  extern __shared__ __attribute__((aligned(16))) float red[];

  const int tiles_m = (M + BM - 1) / BM;
  const int tiles_n = (N + BN - 1) / BN;
  int tile, ks;
  split_tile(tiles_m * tiles_n, false, tile, ks);
  const int tn = tile / tiles_m, tm = tile % tiles_m;   // n-major: an XCD shares W panels
  const int m0 = tm * BM, n0 = tn * BN;
  const int kb = ks * k_split_len;
  const int kw = min(k_split_len, K - kb) / 4;          // this wave's K range (launcher: % 64)
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int fr = lane & 15, fq = lane >> 4;
  const int k0 = kb + wid * kw;
  const int nsteps = kw / 64;

  const u16* ap[MI];
  const u16* wp[NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
    ap[i] = A + (long)min(m0 + 16 * i + fr, M - 1) * lda + k0 + 16 * fq;
#pragma unroll
  for (int j = 0; j < NI; ++j)
    wp[j] = W + (long)min(n0 + 16 * j + fr, N - 1) * ldw + k0 + 16 * fq;

  // accumulators pinned to the AGPR file by inline-asm MFMAs ("+a"): with the builtin, hipcc
  // hoisted both stages' reloads above the MFMAs and moved the 128 accumulator registers
  // between AGPRs every iteration (v_accvgpr_mov). hipcc pads no hazard inside an asm
  // statement: the fragments come from global loads, whose completion it waits for by
  // register before each statement; the accumulators are read only as the next MFMA's C until
  // the padded copy after the loop (gemm4w.h)
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // two register stages of fragments (compile-time indexed: no scratch)
  bf16x8 fa0[MI][2], fw0[NI][2], fa1[MI][2], fw1[NI][2];
  auto load = [&](bf16x8 (&fa)[MI][2], bf16x8 (&fw)[NI][2], int s) __attribute__((always_inline)) {
    const int o = s * 64;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {                // in the order the MFMAs consume them
#pragma unroll
      for (int j = 0; j < NI; ++j) fw[j][kk] = *reinterpret_cast<const bf16x8*>(wp[j] + o + 8 * kk);
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i][kk] = *reinterpret_cast<const bf16x8*>(ap[i] + o + 8 * kk);
    }
    __builtin_amdgcn_sched_barrier(0);             // the loads stay between the MFMA blocks
  };
  auto compute = [&](const bf16x8 (&fa)[MI][2], const bf16x8 (&fw)[NI][2])
      __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                       : "+a"(acc[i][j]) : "v"(fw[j][kk]), "v"(fa[i][kk]));
    __builtin_amdgcn_sched_barrier(0);
  };

  // the reloads are unconditional (an odd step count re-reads its last step into the idle
  // stage): a conditional reload made hipcc's waitcnt merge at the loop head wait on the
  // loads it had just issued
  load(fa0, fw0, 0);
  load(fa1, fw1, min(1, nsteps - 1));
  int s = 0;
  for (; s + 2 < nsteps; s += 2) {
    compute(fa0, fw0);
    load(fa0, fw0, s + 2);
    compute(fa1, fw1);
    load(fa1, fw1, min(s + 3, nsteps - 1));
  }
  if (s < nsteps) compute(fa0, fw0);
  if (s + 1 < nsteps) compute(fa1, fw1);
  // MFMA results -> the copies below: XDL write-back wait states, tied to the last row of
  // accumulators the MFMA order writes (kk = 1, i = MI - 1)
  static_assert(NI == 8 || NI == 6, "pin list");
  if constexpr (NI == 8) {
    asm volatile("s_nop 15\n\ts_nop 15"
                 : "+a"(acc[MI - 1][0]), "+a"(acc[MI - 1][1]), "+a"(acc[MI - 1][2]),
                   "+a"(acc[MI - 1][3]), "+a"(acc[MI - 1][4]), "+a"(acc[MI - 1][5]),
                   "+a"(acc[MI - 1][6]), "+a"(acc[MI - 1][7]));
  } else {
    asm volatile("s_nop 15\n\ts_nop 15"
                 : "+a"(acc[MI - 1][0]), "+a"(acc[MI - 1][1]), "+a"(acc[MI - 1][2]),
                   "+a"(acc[MI - 1][3]), "+a"(acc[MI - 1][4]), "+a"(acc[MI - 1][5]));
  }
  auto vget = [&](const f32x4& a) -> f32x4 {
    f32x4 v;
    asm volatile("" : "=v"(v) : "0"(a));
    return v;
  };

  // ---- the 4 waves' partial blocks -> LDS, row-major [BM][ROW]; lane holds
  // acc[i][j][r] = block[16 i + fr][16 j + 4 fq + r] (transposed accumulators)
  float* mine = red + wid * BM * ROW;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
      *reinterpret_cast<f32x4*>(mine + (16 * i + fr) * ROW + 16 * j + 4 * fq) = vget(acc[i][j]);
  __syncthreads();

  // ---- wave w sums rows [w BM / 4, (w + 1) BM / 4) of the 4 partials and writes them
  constexpr int RQ = BM / 4;
  auto sum4 = [&](int r, int c) -> f32x4 {
    const int o = r * ROW + c;
    f32x4 v = *reinterpret_cast<const f32x4*>(red + o);
#pragma unroll
    for (int q = 1; q < 4; ++q) v += *reinterpret_cast<const f32x4*>(red + q * BM * ROW + o);
    return v;
  };
  if (gridDim.y > 1) {                              // fp32 partial slab of this K split
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool v4 = (N & 3) == 0;
    for (int t = lane; t < RQ * (BN / 4); t += 64) {
      const int r = wid * RQ + t / (BN / 4), c = 4 * (t % (BN / 4));
      const int m = m0 + r, n = n0 + c;
      if (m < M && n < N) slab_quad(slab + (long)m * N + n, sum4(r, c), sm, v4, N - n);
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {                            // gate block 32p + e, up 32p + 16 + e
    for (int t = lane; t < RQ * (BN / 8); t += 64) {
      const int r = wid * RQ + t / (BN / 8), q = t % (BN / 8);
      const int c = 32 * (q >> 2) + 4 * (q & 3);
      const int m = m0 + r, n = n0 + c;
      if (m < M && n < N)
        store_silu_quad(C, ldc, m, ((n0 + c) >> 5) * 16 + 4 * (q & 3), sum4(r, c),
                        sum4(r, c + 16), vec);
    }
    return;
  }
  for (int t = lane; t < RQ * (BN / 4); t += 64) {
    const int r = wid * RQ + t / (BN / 4), c = 4 * (t % (BN / 4));
    const int m = m0 + r, n = n0 + c;
    if (m < M && n < N) store_quad<EPI>(C, ldc, m, n, N, sum4(r, c), bias, vec);
  }
}

template <int BM, int BN, int EPI>
static int launch_sk(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                     int N, int K, int splits, const void* bias, void* ws, const int* group_off,
                     hipStream_t st) {
  // every wave's K range a whole number of 64-deep steps; SiLU pairs need whole 32-col blocks
  if (group_off != nullptr || K % (256 * splits) || lda % 8 || ldw % 8 ||
      (EPI == EPI_SILU && (N % 32 || BN % 32)))
    return (int)hipErrorInvalidValue;
  constexpr size_t lds = sk_lds_bytes<BM, BN>();
  static_assert(lds <= 160 * 1024, "partial blocks must fit the LDS");
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm_sk_kernel<BM, BN, EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  dim3 grid(tiles, splits);
  gemm_sk_kernel<BM, BN, EPI><<<grid, 256, lds, st>>>(
      (const u16*)A, lda, (const u16*)W, ldw, C, ldc, M, N, K, K / splits, (const u16*)bias,
      (float*)ws);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI>
static int dispatch_sk(int tile_cfg, DLI_GEMM_ARGS) {
  (void)groups;
  switch (tile_cfg) {
    case 60: return launch_sk<64, 128, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, st);
    case 61: return launch_sk<64, 96, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, st);
    case 62: return launch_sk<32, 128, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, go, st);
    default: return DLI_NOT_MINE;
  }
}

int gemm_sk_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS) { DLI_EPI_SWITCH(dispatch_sk) }
int gemm_sk_set_slab_store(int mode) { return set_slab_store_tu(mode); }
