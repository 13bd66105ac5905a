// Paged decode attention (one query token per sequence, GQA) on MFMA — SURVEY.md §2.4 K8.
//
// Work decomposition: workgroup = (kv head, sequence, KV split); 4 waves; each wave walks
// 32-token tiles of the split round-robin. Per tile, with the GQA group of G <= 16 query
// heads padded to 16 MFMA columns:
//   S^T[tok, head] = K[tok, :] . Q[head, :]^T   (mfma_f32_16x16x32_bf16, K rows as the A
//                                                operand straight from the cache: 16-B loads)
//   online softmax along tokens (exp2 domain; max across the 4 lane groups = 2 shuffles)
//   O[head, d] += P[head, tok] . V[tok, d]       (the S^T accumulator IS the A operand with a
//                                                permuted token order, so P never leaves
//                                                registers; V^T is stored token-contiguous in
//                                                the cache so the B operand is two 8-B loads)
// The 4 waves' (m, l, O) are merged through LDS; with >1 split the partials go to a
// workspace reduced by a second kernel.
//
// Layouts: q rows of stride q_stride (the fused QKV buffer), k_cache [nblk,Hkv,bs,hd],
// v_cache [nblk,Hkv,hd,bs], block_tables [B, max_blocks], out [B, Hq, hd].
#include "common.h"

#define DEC_WAVES 4
#define DEC_TILE 32

template <int HD>
__global__ void __launch_bounds__(256) decode_attn_kernel(
    u16* __restrict__ out, const u16* __restrict__ q, int q_stride,
    const u16* __restrict__ k_cache, const u16* __restrict__ v_cache,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ context_lens,
    int hq, int hkv, int block_size, float scale_log2, int num_splits, int split_tokens,
    float* __restrict__ ws_o, float* __restrict__ ws_ml) {
  constexpr int KK = HD / 32;     // MFMA k-steps over head_dim
  constexpr int DB = HD / 16;     // 16-wide output column blocks
  const int kvh = blockIdx.x, b = blockIdx.y, split = blockIdx.z;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int G = hq / hkv;
  const int ctx = context_lens[b];
  const int s_begin = split * split_tokens;
  const int s_end = min(ctx, s_begin + split_tokens);

  __shared__ float sh_o[DEC_WAVES][16][HD];
  __shared__ float sh_m[DEC_WAVES][16], sh_l[DEC_WAVES][16];

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
  const long kv_head_stride = (long)block_size * HD;           // elements per (blk, head)
  float m_run = -INFINITY;          // running max for head `col` (replicated over groups)
  float l_part = 0.f;               // this lane's partial denominator for head `col`
  f32x4 o_acc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) o_acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int t0 = s_begin + wid * DEC_TILE; t0 < s_end; t0 += DEC_WAVES * DEC_TILE) {
    // ---- issue every global load of the tile up front (K fragments AND V fragments) so the
    // tile pays one HBM round trip instead of two (V used to wait for the softmax)
    uint4 kreg[2][KK];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      int tok = t0 + 16 * s + col;
      tok = tok < s_end ? tok : s_end - 1;                     // clamp: always-written rows
      const int blk = bt[tok / block_size], off = tok % block_size;
      const u16* kp = k_cache + ((long)blk * hkv + kvh) * kv_head_stride + (long)off * HD;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        kreg[s][kk] = *reinterpret_cast<const uint4*>(kp + kk * 32 + grp * 8);
    }
    // V rows: tokens t0 + pi(grp, j), pi(grp, j) = 16(j>>2) + 4grp + (j&3), from V^T [d][tok]
    const int tokA = min(t0 + 4 * grp, s_end - 1) & ~3;         // 4-aligned, in-range rows
    const int tokB = min(t0 + 16 + 4 * grp, s_end - 1) & ~3;
    const int blkA = bt[tokA / block_size], offA = tokA % block_size;
    const int blkB = bt[tokB / block_size], offB = tokB % block_size;
    const u16* vA = v_cache + ((long)blkA * hkv + kvh) * kv_head_stride + offA;
    const u16* vB = v_cache + ((long)blkB * hkv + kvh) * kv_head_stride + offB;
    uint4 vreg[DB];
#pragma unroll
    for (int i = 0; i < DB; ++i) {
      const long drow = (long)(16 * i + col) * block_size;
      const uint2 a = *reinterpret_cast<const uint2*>(vA + drow);
      const uint2 c = *reinterpret_cast<const uint2*>(vB + drow);
      vreg[i] = make_uint4(a.x, a.y, c.x, c.y);
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
    // A operand: P[head=col][k = 8grp + j] in the permuted token order pi(grp, j)
    bf16x8 pa;
#pragma unroll
    for (int j = 0; j < 8; ++j) pa[j] = (__bf16)p[j];
#pragma unroll
    for (int i = 0; i < DB; ++i)
      o_acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, *reinterpret_cast<bf16x8*>(&vreg[i]),
                                                        o_acc[i], 0, 0, 0);
  }
  // total denominator for head `col`
  float l_tot = l_part + __shfl_xor(l_part, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (grp == 0) { sh_m[wid][col] = m_run; sh_l[wid][col] = l_tot; }
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) sh_o[wid][4 * grp + r][16 * i + col] = o_acc[i][r];
  __syncthreads();

  // merge the 4 waves: each thread produces 8 consecutive output dims of one head
  const int per_head = HD / 8;
  for (int idx = threadIdx.x; idx < G * per_head; idx += blockDim.x) {
    const int h = idx / per_head, d0 = (idx % per_head) * 8;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < DEC_WAVES; ++w) M = fmaxf(M, sh_m[w][h]);
    float den = 0.f, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (M != -INFINITY) {
#pragma unroll
      for (int w = 0; w < DEC_WAVES; ++w) {
        const float f = exp2f(sh_m[w][h] - M);
        den += f * sh_l[w][h];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f * sh_o[w][h][d0 + j];
      }
    }
    const float inv = den > 0.f ? 1.f / den : 0.f;
    const int qh = kvh * G + h;
    if (num_splits == 1) {
      float o8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o8[j] = acc[j] * inv;
      store8(out + ((long)b * hq + qh) * HD + d0, o8);
    } else {
      float* wo = ws_o + (((long)b * hq + qh) * num_splits + split) * HD + d0;
#pragma unroll
      for (int j = 0; j < 8; ++j) wo[j] = acc[j] * inv;
      if (d0 == 0) {
        float* ml = ws_ml + (((long)b * hq + qh) * num_splits + split) * 2;
        ml[0] = M;
        ml[1] = den;
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
  dim3 grid(hkv, B, num_splits);
  if (hd == 128)
    decode_attn_kernel<128><<<grid, 256, 0, st>>>(
        (u16*)out, (const u16*)q, q_stride, (const u16*)k_cache, (const u16*)v_cache,
        block_tables, max_blocks, context_lens, hq, hkv, block_size, scale_log2, num_splits,
        split_tokens, ws_o, ws_ml);
  else
    decode_attn_kernel<64><<<grid, 256, 0, st>>>(
        (u16*)out, (const u16*)q, q_stride, (const u16*)k_cache, (const u16*)v_cache,
        block_tables, max_blocks, context_lens, hq, hkv, block_size, scale_log2, num_splits,
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
