// bf16 GEMM on CDNA4 matrix cores: C[M,N] = A[M,K] . W[N,K]^T (+ fused epilogue).
// SURVEY.md §2.4 K4/K9-K12 (dense projections) and K16 (MoE grouped GEMM).
//
// Structure (cdna_hip_programming.md §5):
//  * WM x WN waves (2x2 = 256 threads, or 2x4 / 4x2 = 512 threads for 256-wide tiles); block
//    tile BM x BN x 64; wave tile (BM/WM) x (BN/WN) built from v_mfma_f32_16x16x32_bf16 (the bf16 shape that holds the higher clock on random
//    data, /opt/skills/guides/MI355X_MICROARCH.md 'DVFS give-back' item 7).
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
//
// Files: gemm_common.h (shared epilogue / split-K pieces), gemm_tiles.hip (ids 0-21, 23-25),
// gemm8p.hip (22, 26-28), gemm4w.h + gemm4w.hip (34, 41, 45), gemm4wp.hip (55: persistent
// 45), gemv.hip (29-33 and the fused
// batch-1 combine). The losing 4-wave A/B variants of round 4 are documented, not built
// (profiles/r4/gemm4w/).
#include "gemm_common.h"

extern "C" int dli_gemm_set_slab_store(int mode) {
  const int old = gemm_tiles_set_slab_store(mode);
  gemm_8p_set_slab_store(mode);
  gemm_4w_set_slab_store(mode);
  return old;
}

// one family's split-K slab store (0 plain, 1 nt, 2 sc1, 3 sc0 sc1): family 0 = the generic
// tiles (decode O / QKV), 1 = the 8-phase kernels (decode down), 2 = the 4-wave kernels
extern "C" int dli_gemm_set_slab_store_family(int family, int mode) {
  switch (family) {
    case 0: return gemm_tiles_set_slab_store(mode);
    case 1: return gemm_8p_set_slab_store(mode);
    case 2: return gemm_4w_set_slab_store(mode);
    default: return -1;
  }
}

// tile_cfg: 0=64x64 1=64x128 2=128x128 3=128x256 4=256x128 (2 LDS stages); 5..9 = the same
// tiles with 3 LDS stages (one tile in flight across the barrier); 10/11 = 192x128 with 2/3
// stages, 12 = 160x128 (MoE experts of ~130-190 rows in one pass); 13-17 = 8-wave tiles
// 256x256, 256x128, 128x256 (2 stages) and 256x128, 128x256 (3 stages); 18/19 = 128x96 and
// 20/21 = 128x64 with 2/3 stages; 22 = 256x256 8-phase ping-pong; 23/24 = 128x192 (3/2
// stages), 25 = 256x192, 8 waves; 26 = 256x224 ping-pong; 29-33 = the M <= 4 weight
// stream (16 / 32 rows per workgroup, dispatch_gemv); 55 = tile 45 persistent (one workgroup
// per CU walks its tiles, no split-K / grouped mode). ws: fp32 [splits, M, N] when splits>1.
// group_off (nullable): int[groups+1] row offsets; M is then the max rows of any group.
// Grouped SiLU*up GEMM whose permuted row p reads activation row arow[p] (the MoE gate/up
// projection without the gathered copy of its input rows): the generic tile family only,
// unsplit. M: the row bound per group, as dli_gemm's grouped mode.
extern "C" int dli_gemm_grouped_gather(const void* A, int lda, const void* W, int ldw, void* C,
                                       int ldc, int M, int N, int K, int tile_cfg,
                                       const int* arow, const int* group_off, int groups,
                                       hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  const bool generic = (tile_cfg >= 0 && tile_cfg <= 21) || (tile_cfg >= 23 && tile_cfg <= 25);
  if (!generic || arow == nullptr || group_off == nullptr || groups < 1 || K % BK || lda % 8 ||
      ldw % 8 || N % 32)
    return (int)hipErrorInvalidValue;
  const void* bias = arow;
  void* ws = nullptr;
  const int* go = group_off;
  const int splits = 1;
  return gemm_tiles_dispatch(EPI_SILU, tile_cfg, DLI_GEMM_PASS);
}

extern "C" int dli_gemm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                        int N, int K, int epi, int tile_cfg, int splits, const void* bias,
                        void* ws, const int* group_off, int groups, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (((tile_cfg < 29 || tile_cfg > 33) && K % BK) || lda % 8 || ldw % 8 || splits < 1)
    return (int)hipErrorInvalidValue;
  if (epi == EPI_SILU && N % 32) return (int)hipErrorInvalidValue;
  if (splits > 1 && ws == nullptr) return (int)hipErrorInvalidValue;
  if (groups < 1) groups = 1;
  const int* go = group_off;
  int r = gemm_tiles_dispatch(epi, tile_cfg, DLI_GEMM_PASS);
  if (r == DLI_NOT_MINE) r = gemm_8p_dispatch(epi, tile_cfg, DLI_GEMM_PASS);
  if (r == DLI_NOT_MINE) r = gemm_4w_dispatch(epi, tile_cfg, DLI_GEMM_PASS);
  if (r == DLI_NOT_MINE) r = gemm_4wp_dispatch(epi, tile_cfg, DLI_GEMM_PASS);
  if (r == DLI_NOT_MINE) r = gemm_gemv_dispatch(epi, tile_cfg, DLI_GEMM_PASS);
  return r == DLI_NOT_MINE ? (int)hipErrorInvalidValue : r;
}
