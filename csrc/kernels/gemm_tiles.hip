// Generic LDS-tiled MFMA GEMM family (tile ids 0-21, 23-25): WM x WN waves, BM x BN x 64
// block tiles, 2 or 3 LDS stages filled by LDS-DMA. Split-K writes fp32 slabs for the fused
// consumers (fused_reduce.hip) or reduces them with splitk_reduce_kernel.
#include "gemm_common.h"

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
  // grouped SiLU*up with a row index (dli_gemm_grouped_gather passes it as `bias`, which the
  // SiLU epilogue never reads): permuted row p of the group reads activation row arow[p], so
  // the MoE gate/up projection streams the token rows in place (no gathered copy)
  const int* arow = (EPI == EPI_SILU && group_off != nullptr)
                        ? reinterpret_cast<const int*>(bias) : nullptr;

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
    a_src[i] = (arow != nullptr ? A + (long)arow[row0 + gr] * lda : Ab + (long)gr * lda) + kb +
               c * 8;
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
        if (col >= N) continue;
        if (EPI == EPI_SLAB16) slab_quad16(srow + col, acc[i][j], vec, N - col, ws);
        else slab_quad(srow + col, acc[i][j], sm, vec, N - col, ws);
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

template <int EPI>
static int dispatch_tiles(int tile_cfg, DLI_GEMM_ARGS) {
  switch (tile_cfg) {
#define DLI_CFG(id, bm, bn, ns) \
    case id: return launch_cfg<bm, bn, EPI, ns>(DLI_GEMM_PASS);
    DLI_CFG(0, 64, 64, 2) DLI_CFG(1, 64, 128, 2) DLI_CFG(2, 128, 128, 2) DLI_CFG(3, 128, 256, 2)
    DLI_CFG(4, 256, 128, 2)
    DLI_CFG(5, 64, 64, 3) DLI_CFG(6, 64, 128, 3) DLI_CFG(7, 128, 128, 3) DLI_CFG(8, 128, 256, 3)
    DLI_CFG(9, 256, 128, 3)
    DLI_CFG(10, 192, 128, 2) DLI_CFG(11, 192, 128, 3) DLI_CFG(12, 160, 128, 2)
#define DLI_CFG8(id, bm, bn, ns, wm, wn) \
    case id: return launch_cfg<bm, bn, EPI, ns, wm, wn>(DLI_GEMM_PASS);
    // 8 waves (512 threads): 256-wide tiles halve the L2 re-reads of A/W at M >= 256
    DLI_CFG8(13, 256, 256, 2, 2, 4) DLI_CFG8(14, 256, 128, 2, 4, 2) DLI_CFG8(15, 128, 256, 2, 2, 4)
    DLI_CFG8(16, 256, 128, 3, 4, 2) DLI_CFG8(17, 128, 256, 3, 2, 4)
    // grid-filling shapes for N = 6144 / 4096 at M = 512 (4 x 64 = 256 workgroups)
    DLI_CFG(18, 128, 96, 2) DLI_CFG(19, 128, 96, 3) DLI_CFG(20, 128, 64, 2) DLI_CFG(21, 128, 64, 3)
    // 192-wide tiles: N = 6144 (fused QKV) = 32 column tiles, so M = 512 fills 256 CUs with
    // 4 x 32 x split 2 (128-row) or 2 x 32 x split 4 (256-row) workgroups of 8 waves
    DLI_CFG8(23, 128, 192, 3, 2, 4) DLI_CFG8(24, 128, 192, 2, 2, 4) DLI_CFG8(25, 256, 192, 2, 4, 2)
#undef DLI_CFG8
#undef DLI_CFG
    default: return DLI_NOT_MINE;
  }
}

int gemm_tiles_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS) { DLI_EPI_SWITCH_S16(dispatch_tiles) }
int gemm_tiles_set_slab_store(int mode) { return set_slab_store_tu(mode); }
