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
//
// Layouts: q rows of stride q_stride (the fused QKV buffer), k_cache and v_cache
// [nblk,Hkv,bs,hd] (token-major: the per-step cache write is a contiguous row),
// block_tables [B, max_blocks], out [B, Hq, hd].
#include "common.h"

#define DEC_WAVES 4
#define DEC_TILE 32

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

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
  constexpr int DB = HD / 16;     // 16-wide output column blocks (= V pieces per lane)
  constexpr int VROW = HD + 16;   // padded LDS row of the V tile, in u16
  constexpr int VCH = HD / 8;     // 16-B chunks per V row
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
  const int* bt = block_tables + (long)b * max_blocks;
  // the split's block ids, one per lane, read once per 64-block window (token -> block by a
  // lane shuffle): the per-tile K/V loads no longer wait on a dependent block-table load
  const int last_blk = max(s_end - 1, 0) / block_size;
  int win = s_begin / block_size;
  int bt_lane = bt[min(win + lane, last_blk)];
  const long kv_head_stride = (long)block_size * HD;           // elements per (blk, head)
  float m_run = -INFINITY;          // running max for head `col` (replicated over groups)
  float l_part = 0.f;               // this lane's partial denominator for head `col`
  f32x4 o_acc[DB];
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

extern "C" long dli_decode_attention_workspace_bytes(int B, int hq, int hd, int num_splits) {
  if (num_splits <= 1) return 0;
  return (long)B * hq * num_splits * (hd + 2) * (long)sizeof(float);
}
