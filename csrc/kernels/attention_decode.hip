// Paged decode attention (one query token per sequence, GQA) on MFMA — SURVEY.md §2.4 K8.
//
// Work decomposition: one wave per (sequence, kv head, KV split) item, 4 independent items per
// workgroup; the wave walks the split's 32-token tiles. Per tile, with the GQA group of G <= 16 query
// heads padded to 16 MFMA columns:
//   S^T[tok, head] = K[tok, :] . Q[head, :]^T   (mfma_f32_16x16x32_bf16, K rows as the A
//                                                operand straight from the cache: 16-B loads)
//   online softmax along tokens (exp2 domain; max across the 4 lane groups = 2 shuffles)
//   O[head, d] += P[head, tok] . V[tok, d]       (the S^T accumulator IS the A operand with a
//                                                permuted token order, so P never leaves
//                                                registers; the V tile is staged row-major in
//                                                a per-wave LDS tile and read as the B operand
//                                                with the transposing ds_read_b64_tr_b16, as
//                                                in the prefill kernel)
// With >1 split the per-split (m, l, O) go to a workspace merged by a second kernel.
// decode_attn_fused_kernel (the decode-graph default) runs the same tile loop after a
// prologue that replaces dli_splitk_rope_cache: the QKV GEMM's split-K slabs are reduced,
// q/k rotated and k/v written to the paged cache inside the attention wave.
//
// Layouts: q rows of stride q_stride (the fused QKV buffer), k_cache and v_cache
// [nblk,Hkv,bs,hd] (token-major: the per-step cache write is a contiguous row),
// block_tables [B, max_blocks], out [B, Hq, hd].
#include "common.h"
#include <limits.h>
#include <stdlib.h>

#define DEC_WAVES 4
#define DEC_TILE 32

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// The tile loop shared by the plain and the fused kernel: one wave = one (sequence, kv head,
// split) item with its Q^T fragments already in registers.
// The tile loop over tokens [s_begin, s_end): leaves the unnormalised O rows in o_acc, the
// running max of head `col` in m_run and this lane's partial denominator in l_part.
// The first 64-block window of the block-table row of tokens [s_begin, s_end), one block id
// per lane (decode_attn_loop's bt_lane0): loaded by the caller so that the load can be
// issued ahead of the prologue's cache write and its fence.
__device__ __forceinline__ int decode_bt_window(const int* __restrict__ block_tables,
                                                int max_blocks, int b, int s_begin, int s_end,
                                                int block_size, int lane) {
  const int last_blk = max(s_end - 1, 0) / block_size;
  return block_tables[(long)b * max_blocks + min(s_begin / block_size + lane, last_blk)];
}

// [s_begin, s_end) of wave wv when WPI waves split a context of ctx tokens by whole tiles
template <int WPI>
__device__ __forceinline__ void decode_wg_range(int ctx, int wv, int& s_begin, int& s_end) {
  const int tiles = (ctx + DEC_TILE - 1) / DEC_TILE;
  const int per = (tiles + WPI - 1) / WPI;
  s_begin = min(ctx, wv * per * DEC_TILE);
  s_end = min(ctx, s_begin + per * DEC_TILE);
}

template <int HD>
__device__ __forceinline__ void decode_attn_loop(
    const bf16x8 (&qf)[HD / 32], u16* vt, int lane, int b, int kvh, int s_begin, int s_end,
    const u16* __restrict__ k_cache, const u16* __restrict__ v_cache,
    const int* __restrict__ block_tables, int max_blocks, int hkv, int block_size,
    float scale_log2, int bt_lane0, f32x4 (&o_acc)[HD / 16], float& m_run, float& l_part) {
  constexpr int DB = HD / 16;     // 16-wide output column blocks (= V pieces per lane)
  constexpr int KK = HD / 32;
  constexpr int VROW = HD + 16;   // padded LDS row of the V tile, in u16
  constexpr int VCH = HD / 8;     // 16-B chunks per V row
  const int col = lane & 15, grp = lane >> 4;
  const int* bt = block_tables + (long)b * max_blocks;
  // the split's block ids, one per lane, read once per 64-block window (token -> block by a
  // lane shuffle): the per-tile K/V loads no longer wait on a dependent block-table load
  const int last_blk = max(s_end - 1, 0) / block_size;
  int win = s_begin / block_size;
  int bt_lane = bt_lane0;
  const long kv_head_stride = (long)block_size * HD;           // elements per (blk, head)
  m_run = -INFINITY;                // running max for head `col` (replicated over groups)
  l_part = 0.f;                     // this lane's partial denominator for head `col`
#pragma unroll
  for (int i = 0; i < DB; ++i) o_acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int t0 = s_begin; t0 < s_end; t0 += DEC_TILE) {
    if ((min(t0 + DEC_TILE, s_end) - 1) / block_size - win >= 64) {   // wave-uniform
      win = t0 / block_size;
      bt_lane = bt[min(win + lane, last_blk)];
    }
    // ---- issue every global load of the tile up front (K fragments AND V fragments)
    uint4 kreg[2][KK];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      int tok = t0 + 16 * s + col;
      tok = tok < s_end ? tok : s_end - 1;                     // clamp: always-written rows
      const int blk = __shfl(bt_lane, tok / block_size - win, 64), off = tok % block_size;
      const u16* kp = k_cache + ((long)blk * hkv + kvh) * kv_head_stride + (long)off * HD;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        kreg[s][kk] = *reinterpret_cast<const uint4*>(kp + kk * 32 + grp * 8);
    }
    // V rows t0 .. t0+31 (row-major, 16-B chunks; piece lane + 64m = row r, chunk c)
    uint4 vreg[DB];
#pragma unroll
    for (int m = 0; m < DB; ++m) {
      const int piece = lane + 64 * m, r = piece / VCH, c = piece % VCH;
      const int tok = min(t0 + r, s_end - 1);                  // clamp: always-written rows
      const int blk = __shfl(bt_lane, tok / block_size - win, 64), off = tok % block_size;
      vreg[m] = *reinterpret_cast<const uint4*>(
          v_cache + ((long)blk * hkv + kvh) * kv_head_stride + (long)off * HD + c * 8);
    }
    // ---- S^T = K . Q^T for the two 16-token subtiles
    f32x4 s_acc[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      s_acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        s_acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            *reinterpret_cast<bf16x8*>(&kreg[s][kk]), qf[kk], s_acc[s], 0, 0, 0);
    }
    // lane holds S^T[tok = t0 + 16s + 4grp + r][head = col]
    float p[8];
    float tmax = -INFINITY;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tok = t0 + 16 * s + 4 * grp + r;
        const float v = tok < s_end ? s_acc[s][r] * scale_log2 : -INFINITY;
        p[s * 4 + r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = exp2f(m_run - m_new);                  // m_run=-inf -> 0
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { p[j] = exp2f(p[j] - m_new); psum += p[j]; }
    l_part = l_part * alpha + psum;
    // rescale O rows (heads 4grp + r) by their head's alpha (held by lane 4grp + r)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a = __shfl(alpha, 4 * grp + r, 64);
#pragma unroll
      for (int i = 0; i < DB; ++i) o_acc[i][r] *= a;
    }
    // stage the V tile in this wave's LDS rows (previous tile's reads retired below)
#pragma unroll
    for (int m = 0; m < DB; ++m) {
      const int piece = lane + 64 * m, r = piece / VCH, c = piece % VCH;
      *reinterpret_cast<uint4*>(vt + r * VROW + c * 8) = vreg[m];
    }
    // A operand: P[head=col][k = 8grp + j] in the permuted token order
    // pi(grp, j) = 16(j>>2) + 4grp + (j&3)
    bf16x8 pa;
#pragma unroll
    for (int j = 0; j < 8; ++j) pa[j] = (__bf16)p[j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // V tile writes landed (same wave)
    // B operand: rows (tokens) 4grp+q and 16+4grp+q, columns 16i + 4p, transposed by
    // ds_read_b64_tr_b16 (lane 4q+p of each 16-lane group names row q, columns 4p..4p+3)
    const int qrow = (lane >> 2) & 3, pcol = lane & 3;
#pragma unroll
    for (int i = 0; i < DB; ++i) {
      const u16* a0 = vt + (4 * grp + qrow) * VROW + 16 * i + 4 * pcol;
      const u16* a1 = vt + (16 + 4 * grp + qrow) * VROW + 16 * i + 4 * pcol;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(a0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(a1));
      s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o_acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, *reinterpret_cast<bf16x8*>(&w),
                                                        o_acc[i], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before next overwrite
  }
}

template <int HD>
__device__ __forceinline__ void decode_attn_core(
    const bf16x8 (&qf)[HD / 32], u16* vt, int lane, int b, int kvh, int split, int G, int ctx,
    int s_begin, int s_end, u16* __restrict__ out, const u16* __restrict__ k_cache,
    const u16* __restrict__ v_cache, const int* __restrict__ block_tables, int max_blocks,
    int hq, int hkv, int block_size, float scale_log2, int num_splits,
    float* __restrict__ ws_o, float* __restrict__ ws_ml, int bt_lane0 = INT_MIN) {
  constexpr int DB = HD / 16;
  const int col = lane & 15, grp = lane >> 4;
  f32x4 o_acc[DB];
  float m_run, l_part;
  if (bt_lane0 == INT_MIN)
    bt_lane0 = decode_bt_window(block_tables, max_blocks, b, s_begin, s_end, block_size, lane);
  decode_attn_loop<HD>(qf, vt, lane, b, kvh, s_begin, s_end, k_cache, v_cache, block_tables,
                       max_blocks, hkv, block_size, scale_log2, bt_lane0, o_acc, m_run, l_part);
  // ---- finalize: denominator of head `col`, then rows 4grp + r of O
  float l_tot = l_part + __shfl_xor(l_part, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int h = 4 * grp + r;
    const float lr = __shfl(l_tot, h, 64);
    const float mr = __shfl(m_run, h, 64);
    if (h >= G) continue;
    const int qh = kvh * G + h;
    const float inv = lr > 0.f ? 1.f / lr : 0.f;
    if (num_splits == 1) {
      u16* op = out + ((long)b * hq + qh) * HD;
#pragma unroll
      for (int i = 0; i < DB; ++i) op[16 * i + col] = f2bf(o_acc[i][r] * inv);
    } else {
      const long base = ((long)b * hq + qh) * num_splits + split;
      float* wo = ws_o + base * HD;
#pragma unroll
      for (int i = 0; i < DB; ++i) wo[16 * i + col] = o_acc[i][r] * inv;
      if (col == 0) {
        ws_ml[base * 2] = lr > 0.f ? mr : -INFINITY;
        ws_ml[base * 2 + 1] = lr;
      }
    }
  }}

// MINW = 4 waves per SIMD: <= 128 VGPRs, so every item of a 512-sequence batch (4096 waves)
// is resident at once (measured 7 % faster than the 166-VGPR / 2-waves build at ctx 66)
template <int HD, int MINW>
__global__ void __launch_bounds__(256, MINW) decode_attn_kernel(
    u16* __restrict__ out, const u16* __restrict__ q, int q_stride,
    const u16* __restrict__ k_cache, const u16* __restrict__ v_cache,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ context_lens,
    int B, int hq, int hkv, int block_size, float scale_log2, int num_splits, int split_tokens,
    float* __restrict__ ws_o, float* __restrict__ ws_ml) {
  constexpr int KK = HD / 32;     // MFMA k-steps over head_dim
  constexpr int VROW = HD + 16;   // padded LDS row of the V tile, in u16
  __shared__ __attribute__((aligned(16))) u16 vtile_all[DEC_WAVES][DEC_TILE * VROW];
  u16* vt = vtile_all[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  // one WAVE per work item (sequence, kv head, KV split): no LDS, no barriers, so every
  // resident wave of the chip streams a different (seq, head) pair concurrently
  const int item = blockIdx.x * DEC_WAVES + (threadIdx.x >> 6);
  if (item >= B * hkv * num_splits) return;                    // wave-uniform exit
  const int split = item % num_splits;
  const int bh = item / num_splits;
  const int kvh = bh % hkv, b = bh / hkv;
  const int col = lane & 15, grp = lane >> 4;
  const int G = hq / hkv;
  const int ctx = context_lens[b];
  const int s_begin = split * split_tokens;
  const int s_end = min(ctx, s_begin + split_tokens);

  // Q^T fragments (B operand): head = col, dims 32kk + 8grp .. +7
  bf16x8 qf[KK];
  {
    const bool valid = col < G;
    const u16* qp = q + (long)b * q_stride + (long)(kvh * G + (valid ? col : 0)) * HD;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      uint4 v = valid ? *reinterpret_cast<const uint4*>(qp + kk * 32 + grp * 8)
                      : make_uint4(0, 0, 0, 0);
      qf[kk] = *reinterpret_cast<bf16x8*>(&v);
    }
  }
  decode_attn_core<HD>(qf, vt, lane, b, kvh, split, G, ctx, s_begin, s_end, out, k_cache,
                       v_cache, block_tables, max_blocks, hq, hkv, block_size, scale_log2,
                       num_splits, ws_o, ws_ml);
}

// One (sequence, kv head) item per workgroup of WPI waves: wave wv walks the wv-th of WPI
// equal slices of the context's 32-token tiles, then the partial (m, l, O) merge through
// LDS (each wave's V-tile rows are reused for its O partial) and the workgroup writes the
// GQA group's output rows. Small batches: with one item per wave most of the chip idles and
// each wave pays one HBM round trip per tile of the whole context.
template <int WPI>
__device__ __forceinline__ void decode_attn_wg(
    const bf16x8 (&qf)[4], u16 (*vtile_all)[DEC_TILE * 144], float (*ml_all)[16][2], int wv,
    int lane, int b, int kvh, int G, int s_begin, int s_end, int bt_lane0,
    u16* __restrict__ out, const u16* __restrict__ k_cache, const u16* __restrict__ v_cache,
    const int* __restrict__ block_tables, int max_blocks, int hq, int hkv, int block_size,
    float scale_log2) {
  constexpr int HD = 128, DB = HD / 16;
  static_assert(16 * HD * 4 <= DEC_TILE * 144 * 2, "O partials fit a wave's V tile");
  const int col = lane & 15, grp = lane >> 4;
  f32x4 o_acc[DB];
  float m_run, l_part;
  decode_attn_loop<HD>(qf, vtile_all[wv], lane, b, kvh, s_begin, s_end, k_cache, v_cache,
                       block_tables, max_blocks, hkv, block_size, scale_log2, bt_lane0, o_acc,
                       m_run, l_part);
  float l_tot = l_part + __shfl_xor(l_part, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  float* po = reinterpret_cast<float*>(vtile_all[wv]);
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int i = 0; i < DB; ++i) po[(4 * grp + r) * HD + 16 * i + col] = o_acc[i][r];
  if (grp == 0) {
    ml_all[wv][col][0] = m_run;
    ml_all[wv][col][1] = l_tot;
  }
  __syncthreads();
  // merge: thread t -> head t / 16, dims 8 (t % 16) .. +7
  const int h = threadIdx.x >> 4, d0 = (threadIdx.x & 15) * 8;
  if (h >= G) return;
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < WPI; ++w) M = fmaxf(M, ml_all[w][h][0]);
  float den = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int w = 0; w < WPI; ++w) {
    const float mw = ml_all[w][h][0];
    const float e = mw == -INFINITY ? 0.f : exp2f(mw - M);
    den += e * ml_all[w][h][1];
    const float4* o4 = reinterpret_cast<const float4*>(
        reinterpret_cast<const float*>(vtile_all[w]) + h * HD + d0);
    const float4 a = o4[0], c = o4[1];
    acc[0] += e * a.x; acc[1] += e * a.y; acc[2] += e * a.z; acc[3] += e * a.w;
    acc[4] += e * c.x; acc[5] += e * c.y; acc[6] += e * c.z; acc[7] += e * c.w;
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  store8(out + ((long)b * hq + kvh * G + h) * HD + d0, acc);
}

// Small-batch form of decode_attn_kernel (head dim 128, one KV split): a workgroup per item.
__global__ void __launch_bounds__(256) decode_attn_wg_kernel(
    u16* __restrict__ out, const u16* __restrict__ q, int q_stride,
    const u16* __restrict__ k_cache, const u16* __restrict__ v_cache,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ context_lens,
    int B, int hq, int hkv, int block_size, float scale_log2) {
  constexpr int HD = 128, KK = HD / 32, VROW = HD + 16;
  __shared__ __attribute__((aligned(16))) u16 vtile_all[DEC_WAVES][DEC_TILE * VROW];
  __shared__ float ml_all[DEC_WAVES][16][2];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int item = blockIdx.x;
  const int kvh = item % hkv, b = item / hkv;
  const int col = lane & 15, grp = lane >> 4;
  const int G = hq / hkv;
  bf16x8 qf[KK];
  {
    const bool valid = col < G;
    const u16* qp = q + (long)b * q_stride + (long)(kvh * G + (valid ? col : 0)) * HD;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      uint4 v = valid ? *reinterpret_cast<const uint4*>(qp + kk * 32 + grp * 8)
                      : make_uint4(0, 0, 0, 0);
      qf[kk] = *reinterpret_cast<bf16x8*>(&v);
    }
  }
  int s_begin, s_end;
  decode_wg_range<DEC_WAVES>(context_lens[b], wv, s_begin, s_end);
  const int bt0 = decode_bt_window(block_tables, max_blocks, b, s_begin, s_end, block_size, lane);
  decode_attn_wg<DEC_WAVES>(qf, vtile_all, ml_all, wv, lane, b, kvh, G, s_begin, s_end, bt0,
                            out, k_cache, v_cache, block_tables, max_blocks, hq, hkv,
                            block_size, scale_log2);
}

// Fused variant for the decode graph (one KV split per item): the QKV GEMM's split-K fp32
// slabs go straight into the attention wave instead of through dli_splitk_rope_cache.
// Prologue of item (sequence b, kv head h): lane l sums the slabs of this token's k and v
// for dims l and l + 64 of head h, rounds to bf16, rotates k (RoPE) and writes both into
// the paged cache at slot_mapping[b]; then each lane builds its Q^T fragments (head col of
// the GQA group, dims 32kk + 8grp .. +7 and their RoPE partners 64 apart, which the same
// lane holds) from the slabs. Numerics equal the unfused kernels: sum -> bf16 -> rotate ->
// bf16. The q rows never go to memory, and one kernel per layer and its slab pass are gone.
//
// WPI = 1: one wave per (sequence, kv head) item, 4 items per workgroup (large batches).
// WPI = DEC_WAVES: one workgroup per item for small batches, where 4 items per workgroup
// leave most of the chip idle and each wave walks the whole context serially (one HBM round
// trip per 32-token tile): wave 0 writes the new k/v row, every wave builds the Q fragments,
// wave w takes the w-th quarter of the context's tiles, and the four partial (m, l, O) merge
// through LDS (the V-tile rows are reused for the O partials).
template <int SPL, int WPI, bool S16 = false>
__global__ void __launch_bounds__(256, 4) decode_attn_fused_kernel(
    u16* __restrict__ out, const void* __restrict__ src, int N,
    const int* __restrict__ positions, const int* __restrict__ slot_mapping,
    const float* __restrict__ cos_sin, u16* __restrict__ k_cache, u16* __restrict__ v_cache,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ context_lens,
    int B, int hq, int hkv, int block_size, float scale_log2) {
  constexpr int HD = 128, HALF = 64, KK = HD / 32, VROW = HD + 16, DB = HD / 16;
  // SPL > 0: src = the QKV GEMM's fp32 split-K slabs [SPL, B, N]; SPL == 0: the bf16 QKV rows
  // [B, N] of an unsplit GEMM (the same prologue minus the slab sum)
  // S16: the slabs are fp16 x 1/16 (EPI_SLAB16), read as 16-bit words
  const float* ws = static_cast<const float*>(src);
  const u16* qkv = static_cast<const u16*>(src);
  const u16* ws16 = static_cast<const u16*>(src);
  static_assert(WPI == 1 || WPI == DEC_WAVES, "one item per wave or per workgroup");
  __shared__ __attribute__((aligned(16))) u16 vtile_all[DEC_WAVES][DEC_TILE * VROW];
  __shared__ float ml_all[WPI > 1 ? WPI : 1][16][2];
  const int wv = threadIdx.x >> 6;
  u16* vt = vtile_all[wv];
  const int lane = threadIdx.x & 63;
  const int item = WPI > 1 ? (int)blockIdx.x : (int)blockIdx.x * DEC_WAVES + wv;
  if (item >= B * hkv) return;                                 // wave-uniform exit (WPI 1)
  const int kvh = item % hkv, b = item / hkv;
  const int col = lane & 15, grp = lane >> 4;
  const int G = hq / hkv;
  const int ctx = context_lens[b];
  const float* cs = cos_sin + (long)positions[b] * HD;
  const long rowoff = (long)b * N;
  const long splitstride = (long)B * N;
  // ---- Q^T fragments (first: their slab loads do not wait on the cache write below): head
  // col of the group, dims 32kk + 8grp .. +7 (kk < 2: first half, its RoPE partner is
  // fragment kk + 2 of the same lane)
  bf16x8 qf[KK];
  if (col < G) {
    const float* qp = ws + rowoff + (long)(kvh * G + col) * HD;
#pragma unroll
    for (int kp2 = 0; kp2 < KK / 2; ++kp2) {
      const int d1 = 32 * kp2 + 8 * grp;
      float x1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, x2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (SPL == 0) {
        const u16* qr = qkv + rowoff + (long)(kvh * G + col) * HD;
        load8(qr + d1, x1);
        load8(qr + HALF + d1, x2);
      }
      if constexpr (S16) {
        const u16* qh = ws16 + rowoff + (long)(kvh * G + col) * HD;
        uint4 ua[SPL], uc[SPL];
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          ua[s] = *reinterpret_cast<const uint4*>(qh + s * splitstride + d1);
          uc[s] = *reinterpret_cast<const uint4*>(qh + s * splitstride + HALF + d1);
        }
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          float fa[8], fc[8];
          unpack8h(ua[s], fa);
          unpack8h(uc[s], fc);
#pragma unroll
          for (int j = 0; j < 8; ++j) { x1[j] += fa[j]; x2[j] += fc[j]; }
        }
      }
#pragma unroll
      for (int s = 0; s < (S16 ? 0 : SPL); ++s) {
        const float4* a = reinterpret_cast<const float4*>(qp + s * splitstride + d1);
        const float4* c = reinterpret_cast<const float4*>(qp + s * splitstride + HALF + d1);
        const float4 a0 = a[0], a1 = a[1], c0 = c[0], c1 = c[1];
        x1[0] += a0.x; x1[1] += a0.y; x1[2] += a0.z; x1[3] += a0.w;
        x1[4] += a1.x; x1[5] += a1.y; x1[6] += a1.z; x1[7] += a1.w;
        x2[0] += c0.x; x2[1] += c0.y; x2[2] += c0.z; x2[3] += c0.w;
        x2[4] += c1.x; x2[5] += c1.y; x2[6] += c1.z; x2[7] += c1.w;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float q1 = bf2f(f2bf(x1[j])), q2 = bf2f(f2bf(x2[j]));
        const float co = cs[d1 + j], si = cs[HALF + d1 + j];
        qf[kp2][j] = (__bf16)(q1 * co - q2 * si);
        qf[kp2 + 2][j] = (__bf16)(q2 * co + q1 * si);
      }
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      uint4 z = make_uint4(0, 0, 0, 0);
      qf[kk] = *reinterpret_cast<bf16x8*>(&z);
    }
  }
  // the block-table window too: every load the tile loop's first tile waits on except the
  // new cache row is issued before the fence below
  int s_begin = 0, s_end = ctx;
  if constexpr (WPI > 1) decode_wg_range<WPI>(ctx, wv, s_begin, s_end);
  const int bt0 = decode_bt_window(block_tables, max_blocks, b, s_begin, s_end, block_size, lane);
  // ---- this token's k (rotated) and v -> paged cache (lane: dims lane, lane + 64)
  const int slot = slot_mapping[b];
  if (slot >= 0 && (WPI == 1 || wv == 0)) {
    const float* kp = ws + rowoff + (long)(hq + kvh) * HD;
    const float* vp = ws + rowoff + (long)(hq + hkv + kvh) * HD;
    float k1 = 0.f, k2 = 0.f, v1 = 0.f, v2 = 0.f;
    if constexpr (S16) {
      const u16* kh = ws16 + rowoff + (long)(hq + kvh) * HD;
      const u16* vh = ws16 + rowoff + (long)(hq + hkv + kvh) * HD;
#pragma unroll
      for (int s = 0; s < SPL; ++s) {
        k1 += h2f(kh[s * splitstride + lane]) * SLAB16_UNSCALE;
        k2 += h2f(kh[s * splitstride + HALF + lane]) * SLAB16_UNSCALE;
        v1 += h2f(vh[s * splitstride + lane]) * SLAB16_UNSCALE;
        v2 += h2f(vh[s * splitstride + HALF + lane]) * SLAB16_UNSCALE;
      }
    } else if constexpr (SPL > 0) {
#pragma unroll
      for (int s = 0; s < SPL; ++s) {
        k1 += kp[s * splitstride + lane];
        k2 += kp[s * splitstride + HALF + lane];
        v1 += vp[s * splitstride + lane];
        v2 += vp[s * splitstride + HALF + lane];
      }
    } else {
      const u16* kr = qkv + rowoff + (long)(hq + kvh) * HD;
      const u16* vr = qkv + rowoff + (long)(hq + hkv + kvh) * HD;
      k1 = bf2f(kr[lane]); k2 = bf2f(kr[HALF + lane]);
      v1 = bf2f(vr[lane]); v2 = bf2f(vr[HALF + lane]);
    }
    k1 = bf2f(f2bf(k1)); k2 = bf2f(f2bf(k2));
    const float co = cs[lane], si = cs[HALF + lane];
    const int blk = slot / block_size, off = slot - blk * block_size;
    const long dst = (((long)blk * hkv + kvh) * block_size + off) * HD;
    k_cache[dst + lane] = f2bf(k1 * co - k2 * si);
    k_cache[dst + HALF + lane] = f2bf(k2 * co + k1 * si);
    v_cache[dst + lane] = f2bf(v1);
    v_cache[dst + HALF + lane] = f2bf(v2);
  }
  // the tile loop below reads this row back (other lanes of this wave): order the stores
  // before those loads
  __threadfence_block();
  if constexpr (WPI == 1) {
    decode_attn_core<HD>(qf, vt, lane, b, kvh, 0, G, ctx, 0, ctx, out, k_cache, v_cache,
                         block_tables, max_blocks, hq, hkv, block_size, scale_log2, 1, nullptr,
                         nullptr, bt0);
  } else {
    __syncthreads();                       // wave 0's cache row visible to the other waves
    decode_attn_wg<WPI>(qf, vtile_all, ml_all, wv, lane, b, kvh, G, s_begin, s_end, bt0, out,
                        k_cache, v_cache, block_tables, max_blocks, hq, hkv, block_size,
                        scale_log2);
  }
}

// Software-pipelined variant: a wave walks a list of work units (item = (sequence, kv head,
// split), unit = one 32-token tile of it; an empty split is one empty unit) and issues the
// loads of unit u+1 before computing unit u, across item boundaries (the next item's Q and
// block-table window are fetched one unit ahead too). K goes to one of two register sets;
// V goes by LDS-DMA (global_load_lds_dwordx4) straight into one of two per-wave LDS tiles
// (256-B rows, chunk XOR swizzle for the transposed reads), so no VGPRs hold it. 2 waves per
// SIMD and a grid of 8 waves per CU, each wave taking items gw, gw + nw, ... The
// one-tile-per-round kernel above leaves every wave of the chip loading, then computing, in
// lockstep: 3 exposed HBM round trips at ctx ~66.
typedef __attribute__((address_space(3))) void dec_lds_void;
typedef const __attribute__((address_space(1))) void dec_gbl_void;

template <int HD>
__global__ void __launch_bounds__(256, 2) decode_attn_pipe_kernel(
    u16* __restrict__ out, const u16* __restrict__ q, int q_stride,
    const u16* __restrict__ k_cache, const u16* __restrict__ v_cache,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ context_lens,
    int B, int hq, int hkv, int block_size, float scale_log2, int num_splits, int split_tokens,
    float* __restrict__ ws_o, float* __restrict__ ws_ml) {
  static_assert(HD == 128, "pipelined decode attention: head_dim 128");
  constexpr int KK = HD / 32, DB = HD / 16;
  constexpr int VT_BYTES = DEC_TILE * HD * 2;                  // 8 KiB per V tile
  __shared__ __attribute__((aligned(16))) char vt_all[DEC_WAVES][2][VT_BYTES];
  const int wv = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63, col = lane & 15, grp = lane >> 4;
  const int G = hq / hkv;
  const int nitems = B * hkv * num_splits;
  const int nw = gridDim.x * DEC_WAVES;
  const long kv_head_stride = (long)block_size * HD;

  int p_item = blockIdx.x * DEC_WAVES + wv;
  if (p_item >= nitems) return;                                  // wave-uniform
  auto geom = [&](int it, int& b, int& kvh, int& split, int& sb, int& se) {
    split = it % num_splits;
    const int bh = it / num_splits;
    kvh = bh % hkv;
    b = bh / hkv;
    const int ctx = context_lens[b];
    sb = split * split_tokens;
    se = min(ctx, sb + split_tokens);
  };
  auto ntiles_of = [&](int sb, int se) { return se > sb ? (se - sb + DEC_TILE - 1) / DEC_TILE : 1; };
  auto load_q = [&](int b, int kvh, bf16x8* dst) {
    const bool valid = col < G;
    const u16* qp = q + (long)b * q_stride + (long)(kvh * G + (valid ? col : 0)) * HD;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      uint4 v = valid ? *reinterpret_cast<const uint4*>(qp + kk * 32 + grp * 8)
                      : make_uint4(0, 0, 0, 0);
      dst[kk] = *reinterpret_cast<bf16x8*>(&v);
    }
  };
  int pb, pkvh, psplit, psb, pse;
  geom(p_item, pb, pkvh, psplit, psb, pse);
  int p_tile = 0, p_nt = ntiles_of(psb, pse);
  int p_win = psb / block_size;
  int p_last_blk = max(pse - 1, 0) / block_size;
  int p_bt = block_tables[(long)pb * max_blocks + min(p_win + lane, p_last_blk)];
  bf16x8 qf_next[KK];
  load_q(pb, pkvh, qf_next);

  // V image: row r at 256 r, 16-B chunk c at physical chunk c ^ swz(r)
  auto vswz = [](int r) { return ((r & 3) << 2) | ((r >> 2) & 3); };
  uint4 ka[2][KK], kb[2][KK];
  // issue the loads of the prefetch cursor's unit; returns true if it issued any
  auto issue = [&](uint4 (&kr)[2][KK], int vbuf) -> bool {
    if (pse <= psb) return false;                                // empty unit: no loads
    const int t0 = psb + DEC_TILE * p_tile;
    if ((min(t0 + DEC_TILE, pse) - 1) / block_size - p_win >= 64) {   // wave-uniform
      p_win = t0 / block_size;
      p_bt = block_tables[(long)pb * max_blocks + min(p_win + lane, p_last_blk)];
    }
    const u16* kbase = k_cache + (long)pkvh * kv_head_stride;
    const u16* vbase = v_cache + (long)pkvh * kv_head_stride;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int tok = min(t0 + 16 * s + col, pse - 1);
      const int blk = __shfl(p_bt, tok / block_size - p_win, 64), off = tok % block_size;
      const u16* kp = kbase + (long)blk * hkv * kv_head_stride + (long)off * HD;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        kr[s][kk] = *reinterpret_cast<const uint4*>(kp + kk * 32 + grp * 8);
    }
    // 8 pieces of 4 rows: lane L of piece m lands at row 4m + L/16, physical chunk L%16
#pragma unroll
    for (int m = 0; m < DEC_TILE / 4; ++m) {
      const int r = 4 * m + (lane >> 4);
      const int c = (lane & 15) ^ vswz(r);
      const int tok = min(t0 + r, pse - 1);
      const int blk = __shfl(p_bt, tok / block_size - p_win, 64), off = tok % block_size;
      __builtin_amdgcn_global_load_lds(
          (dec_gbl_void*)(vbase + (long)blk * hkv * kv_head_stride + (long)off * HD + c * 8),
          (dec_lds_void*)&vt_all[wv][vbuf][m * 1024], 16, 0, 0);
    }
    return true;
  };
  auto advance = [&]() -> bool {
    if (++p_tile < p_nt) return true;
    p_item += nw;
    if (p_item >= nitems) return false;
    geom(p_item, pb, pkvh, psplit, psb, pse);
    p_tile = 0;
    p_nt = ntiles_of(psb, pse);
    p_win = psb / block_size;
    p_last_blk = max(pse - 1, 0) / block_size;
    p_bt = block_tables[(long)pb * max_blocks + min(p_win + lane, p_last_blk)];
    load_q(pb, pkvh, qf_next);
    return true;
  };

  int c_item = p_item, cb = pb, ckvh = pkvh, csplit = psplit, csb = psb, cse = pse;
  int c_tile = 0, c_nt = p_nt;
  bf16x8 qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) qf[kk] = qf_next[kk];
  float m_run = -INFINITY, l_part = 0.f;
  f32x4 o_acc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) o_acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto finalize = [&]() {
    float l_tot = l_part + __shfl_xor(l_part, 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 4 * grp + r;
      const float lr = __shfl(l_tot, h, 64);
      const float mr = __shfl(m_run, h, 64);
      if (h >= G) continue;
      const int qh = ckvh * G + h;
      const float inv = lr > 0.f ? 1.f / lr : 0.f;
      if (num_splits == 1) {
        u16* op = out + ((long)cb * hq + qh) * HD;
#pragma unroll
        for (int i = 0; i < DB; ++i) op[16 * i + col] = f2bf(o_acc[i][r] * inv);
      } else {
        const long base = ((long)cb * hq + qh) * num_splits + csplit;
        float* wo = ws_o + base * HD;
#pragma unroll
        for (int i = 0; i < DB; ++i) wo[16 * i + col] = o_acc[i][r] * inv;
        if (col == 0) {
          ws_ml[base * 2] = lr > 0.f ? mr : -INFINITY;
          ws_ml[base * 2 + 1] = lr;
        }
      }
    }
  };
  // compute cursor's unit from K registers kr and V tile vbuf; `later` = the next unit's
  // loads were issued after this unit's V DMA (then vmcnt(16) retires exactly this tile:
  // at least 16 vector-memory ops followed it; else vmcnt(0))
  const int qrow = (lane >> 2) & 3, pcol = lane & 3;
  auto compute = [&](uint4 (&kr)[2][KK], int vbuf, bool later) {
    if (cse > csb) {
      const int t0 = csb + DEC_TILE * c_tile;
      f32x4 s_acc[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        s_acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
          s_acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              *reinterpret_cast<bf16x8*>(&kr[s][kk]), qf[kk], s_acc[s], 0, 0, 0);
      }
      float p[8];
      float tmax = -INFINITY;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int tok = t0 + 16 * s + 4 * grp + r;
          const float v = tok < cse ? s_acc[s][r] * scale_log2 : -INFINITY;
          p[s * 4 + r] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float m_new = fmaxf(m_run, tmax);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);     // m_run=-inf -> 0
      m_run = m_new;
      float psum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { p[j] = __builtin_amdgcn_exp2f(p[j] - m_new); psum += p[j]; }
      l_part = l_part * alpha + psum;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = __shfl(alpha, 4 * grp + r, 64);
#pragma unroll
        for (int i = 0; i < DB; ++i) o_acc[i][r] *= a;
      }
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 8; ++j) pa[j] = (__bf16)p[j];
      if (later) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // this V tile landed
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const char* vt = vt_all[wv][vbuf];
#pragma unroll
      for (int i = 0; i < DB; ++i) {
        // rows 4grp + qrow and 16 + 4grp + qrow, columns 16i + 4pcol .. +3
        const int r0 = 4 * grp + qrow, r1 = 16 + r0, ch = 2 * i + (pcol >> 1);
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(vt + 256 * r0 + 16 * (ch ^ vswz(r0)) +
                                                       8 * (pcol & 1)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(vt + 256 * r1 + 16 * (ch ^ vswz(r1)) +
                                                       8 * (pcol & 1)));
        s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o_acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, *reinterpret_cast<bf16x8*>(&w),
                                                          o_acc[i], 0, 0, 0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // reads done before restaging
    }
    if (++c_tile == c_nt) {                                      // item done
      finalize();
      c_item += nw;
      if (c_item < nitems) {
        geom(c_item, cb, ckvh, csplit, csb, cse);
        c_tile = 0;
        c_nt = ntiles_of(csb, cse);
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) qf[kk] = qf_next[kk];
        m_run = -INFINITY;
        l_part = 0.f;
#pragma unroll
        for (int i = 0; i < DB; ++i) o_acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  issue(ka, 0);
  while (true) {
    bool more = advance();
    bool later = more && issue(kb, 1);
    compute(ka, 0, later);
    if (!more) break;
    more = advance();
    later = more && issue(ka, 0);
    compute(kb, 1, later);
    if (!more) break;
  }
}

// out[b, h, :] = sum_s w_s o_s / sum_s w_s,  w_s = exp2(m_s - M) * l_s
template <int HD>
__global__ void __launch_bounds__(256) decode_reduce_kernel(u16* __restrict__ out,
                                                            const float* __restrict__ ws_o,
                                                            const float* __restrict__ ws_ml,
                                                            int B, int hq, int num_splits) {
  const int per_row = HD / 8;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long)B * hq * per_row) return;
  const long bh = gid / per_row;
  const int d0 = (int)(gid % per_row) * 8;
  const float* ml = ws_ml + bh * num_splits * 2;
  float M = -INFINITY;
  for (int s = 0; s < num_splits; ++s) M = fmaxf(M, ml[2 * s]);
  float den = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (M != -INFINITY) {
    for (int s = 0; s < num_splits; ++s) {
      const float w = exp2f(ml[2 * s] - M) * ml[2 * s + 1];
      den += w;
      const float* o = ws_o + (bh * num_splits + s) * HD + d0;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += w * o[j];
    }
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  store8(out + bh * HD + d0, acc);
}

// pipelined (1), one-tile-per-round (0) or automatic (2, the default) decode kernel for hd 128
static int g_decode_pipe = 2;
extern "C" int dli_decode_set_pipe(int v) {
  const int old = g_decode_pipe;
  g_decode_pipe = v;
  return old;
}

// the mode the next dli_decode_attention call applies
extern "C" int dli_decode_get_pipe() { return g_decode_pipe; }

// a workgroup per (sequence, kv head) item while the items alone would leave most CUs idle
// (<= 256 items: B <= 32 at 8 kv heads), else a wave per item; tests force either form with
// dli_decode_set_form(1 = wave per item, DEC_WAVES = workgroup per item, 0 = automatic)
static int g_decode_form = 0;
extern "C" int dli_decode_set_form(int v) {
  const int old = g_decode_form;
  g_decode_form = v;
  return old;
}
static bool wg_form(long items) {
  return g_decode_form == DEC_WAVES || (g_decode_form != 1 && items <= 256);
}

extern "C" int dli_decode_attention(void* out, const void* q, int q_stride, const void* k_cache,
                                    const void* v_cache, const int* block_tables, int max_blocks,
                                    const int* context_lens, int B, int hq, int hkv, int hd,
                                    int block_size, float scale, int max_context, int num_splits,
                                    void* workspace, hipStream_t st) {
  if (B <= 0) return 0;
  if (hq % hkv || hq / hkv > 16 || block_size % 16 || (hd != 64 && hd != 128))
    return (int)hipErrorInvalidValue;
  if (num_splits < 1) num_splits = 1;
  if (num_splits > 1 && workspace == nullptr) return (int)hipErrorInvalidValue;
  int split_tokens = (max_context + num_splits - 1) / num_splits;
  split_tokens = ((split_tokens + DEC_TILE - 1) / DEC_TILE) * DEC_TILE;
  if (split_tokens <= 0) split_tokens = DEC_TILE;
  float* ws_o = (float*)workspace;
  float* ws_ml = ws_o ? ws_o + (long)B * hq * num_splits * hd : nullptr;
  const float scale_log2 = scale * 1.4426950408889634f;
  const long items = (long)B * hkv * num_splits;
  // 2 = automatic: the pipelined kernel for splits of >= 768 tokens (measured: +18 % at ctx
  // 1000, B 64; within 3 % slower at ctx 33-100, B 512, where the per-item dependent loads
  // (context length -> block table -> K/V) rather than tile rounds bound the time)
  const bool use_pipe = g_decode_pipe == 1 || (g_decode_pipe == 2 && split_tokens >= 768);
  if (hd == 128 && use_pipe) {
    // 8 waves per CU x 256 CUs; each wave walks items gw, gw + nw, ...
    const long wgs = (items + DEC_WAVES - 1) / DEC_WAVES;
    dim3 gp((int)(wgs < 512 ? wgs : 512));
    decode_attn_pipe_kernel<128><<<gp, 64 * DEC_WAVES, 0, st>>>(
        (u16*)out, (const u16*)q, q_stride, (const u16*)k_cache, (const u16*)v_cache,
        block_tables, max_blocks, context_lens, B, hq, hkv, block_size, scale_log2, num_splits,
        split_tokens, ws_o, ws_ml);
  } else if (hd == 128 && num_splits == 1 && wg_form(items)) {
    decode_attn_wg_kernel<<<(int)items, 64 * DEC_WAVES, 0, st>>>(
        (u16*)out, (const u16*)q, q_stride, (const u16*)k_cache, (const u16*)v_cache,
        block_tables, max_blocks, context_lens, B, hq, hkv, block_size, scale_log2);
  } else {
  dim3 grid((int)((items + DEC_WAVES - 1) / DEC_WAVES));
  if (hd == 128)
    decode_attn_kernel<128, 4><<<grid, 64 * DEC_WAVES, 0, st>>>(
        (u16*)out, (const u16*)q, q_stride, (const u16*)k_cache, (const u16*)v_cache,
        block_tables, max_blocks, context_lens, B, hq, hkv, block_size, scale_log2, num_splits,
        split_tokens, ws_o, ws_ml);
  else
    decode_attn_kernel<64, 1><<<grid, 64 * DEC_WAVES, 0, st>>>(
        (u16*)out, (const u16*)q, q_stride, (const u16*)k_cache, (const u16*)v_cache,
        block_tables, max_blocks, context_lens, B, hq, hkv, block_size, scale_log2, num_splits,
        split_tokens, ws_o, ws_ml);
  }
  if (num_splits > 1) {
    const long total = (long)B * hq * (hd / 8);
    const int blocks = (int)((total + 255) / 256);
    if (hd == 128)
      decode_reduce_kernel<128><<<blocks, 256, 0, st>>>((u16*)out, ws_o, ws_ml, B, hq, num_splits);
    else
      decode_reduce_kernel<64><<<blocks, 256, 0, st>>>((u16*)out, ws_o, ws_ml, B, hq, num_splits);
  }
  DLI_RETURN_LAUNCH();
}

// Fused split-K QKV reduce + RoPE + KV-cache write + decode attention (one KV split, head
// dim 128, RoPE models): ws = the QKV GEMM's fp32 slabs [splits, B, (hq + 2 hkv) * 128], or
// with splits == 0 the bf16 QKV rows [B, (hq + 2 hkv) * 128] of an unsplit GEMM.
// fmt: 0 = fp32 slabs (or the bf16 rows when splits == 0), 1 = fp16 x 1/16 slabs (EPI_SLAB16)
extern "C" int dli_decode_attention_fused(void* out, const void* ws, int splits,
                                          const int* positions, const int* slot_mapping,
                                          const float* cos_sin, void* k_cache, void* v_cache,
                                          const int* block_tables, int max_blocks,
                                          const int* context_lens, int B, int hq, int hkv,
                                          int hd, int block_size, float scale, int fmt,
                                          hipStream_t st) {
  if (B <= 0) return 0;
  if (hd != 128 || hq % hkv || hq / hkv > 16 || block_size % 16 ||
      (splits != 0 && splits != 2 && splits != 4) || fmt < 0 || fmt > 1 ||
      (fmt == 1 && splits == 0))
    return (int)hipErrorInvalidValue;
  const int N = (hq + 2 * hkv) * hd;
  const float scale_log2 = scale * 1.4426950408889634f;
  const long items = (long)B * hkv;
  const bool per_wg = wg_form(items);
  dim3 grid((int)(per_wg ? items : (items + DEC_WAVES - 1) / DEC_WAVES));
#define DLI_DAF(S, W, F) decode_attn_fused_kernel<S, W, F><<<grid, 64 * DEC_WAVES, 0, st>>>(   \
      (u16*)out, ws, N, positions, slot_mapping, cos_sin, (u16*)k_cache, (u16*)v_cache,      \
      block_tables, max_blocks, context_lens, B, hq, hkv, block_size, scale_log2)
  if (per_wg) {
    if (splits == 0) DLI_DAF(0, DEC_WAVES, false);
    else if (splits == 2) { if (fmt) DLI_DAF(2, DEC_WAVES, true); else DLI_DAF(2, DEC_WAVES, false); }
    else { if (fmt) DLI_DAF(4, DEC_WAVES, true); else DLI_DAF(4, DEC_WAVES, false); }
  } else {
    if (splits == 0) DLI_DAF(0, 1, false);
    else if (splits == 2) { if (fmt) DLI_DAF(2, 1, true); else DLI_DAF(2, 1, false); }
    else { if (fmt) DLI_DAF(4, 1, true); else DLI_DAF(4, 1, false); }
  }
#undef DLI_DAF
  DLI_RETURN_LAUNCH();
}

extern "C" long dli_decode_attention_workspace_bytes(int B, int hq, int hd, int num_splits) {
  if (num_splits <= 1) return 0;
  return (long)B * hq * num_splits * (hd + 2) * (long)sizeof(float);
}
