// Causal variable-length (packed) GQA prefill attention on MFMA — SURVEY.md §2.4 K7.
//
// Reads q/k/v straight out of the fused QKV activation (row stride = (Hq+2Hkv)*hd) after
// the in-place RoPE, so no separate K/V copies exist. A workgroup = 4 waves = 64 query rows
// of one query head (16 per wave); the workgroup streams 64-key tiles of K and V through
// LDS ONCE for all 4 waves (each wave used to fetch its own K rows from global memory: 4x
// the K/V traffic, O(L^2) bytes per head for long prompts):
//   stage      tile t+1 is loaded into registers while tile t is computed, then written
//              to LDS between two barriers (K rows padded to 272 B: conflict-free
//              ds_read_b128 of the A operand; V rows to hd*2+32 B for the transposing read)
//   S^T[key, q] = K . Q^T        mfma_f32_16x16x32_bf16, K rows as the A operand
//   softmax along keys           exp2 domain, online (flash) rescaling per tile
//   O[q, d] += P[q, key] . V     P re-used from the accumulator registers (permuted key
//                                order); V read as the B operand with the CDNA4 transposing
//                                ds_read_b64_tr_b16 (cdna_hip_programming.md T10)
// Causality: a wave skips the math of tiles entirely above its rows (it still helps stage
// them); the workgroup stops at its last row's bound.
// Chunked prefill (PAGED): the chunk's K/V have already been written to the paged cache
// (rope_cache), so keys come from the cache through the block table: a chunk of len queries
// at positions [ctx - len, ctx) attends over all ctx cached keys of its sequence (earlier
// chunks, a recomputed prefix) with the causal bound shifted by ctx - len.
// Grid: (ceil(max_len / 64), num_seqs, Hq).
#include "common.h"

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
#define PF_WAVES 4
#define PF_QROWS 16
#define PF_KT 64

template <int HD, bool PAGED>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) prefill_attn_kernel(
    u16* __restrict__ out, int out_stride, const u16* __restrict__ qkv, int row_stride,
    const int* __restrict__ cu_seqlens, int hq, int hkv, float scale_log2,
    const int* __restrict__ ctx_lens, const u16* __restrict__ k_cache,
    const u16* __restrict__ v_cache, const int* __restrict__ block_tables, int bt_stride,
    int block_size) {
  constexpr int KK = HD / 32, DB = HD / 16;
  constexpr int KROW = HD + 8;                     // K row in LDS (u16): 272 B for hd 128
  constexpr int VROW = HD + 16;                    // V row in LDS (u16): hd*2 + 32 B
  constexpr int CH = HD / 8;                       // 16-B chunks per row
  constexpr int PER = PF_KT * CH / 256;            // chunks per thread per tile (K or V)
  __shared__ __attribute__((aligned(16))) u16 ktile[PF_KT * KROW];
  __shared__ __attribute__((aligned(16))) u16 vtile[PF_KT * VROW];
  const int seq = blockIdx.y, h = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int s0 = cu_seqlens[seq], len = cu_seqlens[seq + 1] - s0;
  const int nkeys = PAGED ? ctx_lens[seq] : len;                 // keys visible to the chunk
  const int qoff = nkeys - len;                                  // position of query row 0
  const int wg_q0 = blockIdx.x * PF_WAVES * PF_QROWS;
  if (wg_q0 >= len) return;                                      // workgroup-uniform exit
  const int q0 = wg_q0 + wid * PF_QROWS;                         // this wave's first row
  const bool active = q0 < len;
  const int G = hq / hkv, kvh = h / G;
  const u16* qbase = qkv + (long)h * HD;
  const u16* kbase = qkv + (long)(hq + kvh) * HD;
  const u16* vbase = qkv + (long)(hq + hkv + kvh) * HD;
  const int* btab = PAGED ? block_tables + (long)seq * bt_stride : nullptr;
  const long head_off = (long)kvh * block_size * HD;             // (blk, head) panel offset

  bf16x8 qf[KK];
  {
    const int qr = min(q0 + col, len - 1);
    const u16* qp = qbase + (long)(s0 + qr) * row_stride;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      uint4 v = *reinterpret_cast<const uint4*>(qp + kk * 32 + grp * 8);
      qf[kk] = *reinterpret_cast<bf16x8*>(&v);
    }
  }
  const int my_q = qoff + q0 + col;        // position of the query row of this lane's column
  float m_run = -INFINITY, l_part = 0.f;
  f32x4 o_acc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) o_acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kend_wg = min(nkeys, qoff + wg_q0 + PF_WAVES * PF_QROWS);  // last row's bound
  const int kend_w = min(nkeys, qoff + q0 + PF_QROWS);                 // this wave's bound

  uint4 kreg[PER], vreg[PER];
#define PF_LOAD_TILE(K0)                                                              \
  _Pragma("unroll") for (int j = 0; j < PER; ++j) {                                   \
    const int i = tid + 256 * j;                                                      \
    const int r = i / CH, c = i % CH;                                                 \
    const int tok = min((K0) + r, nkeys - 1);                                         \
    if (PAGED) {                                                                      \
      const long e = (long)btab[tok / block_size] * hkv * block_size * HD + head_off +  \
                     (long)(tok % block_size) * HD + c * 8;                           \
      kreg[j] = *reinterpret_cast<const uint4*>(k_cache + e);                         \
      vreg[j] = *reinterpret_cast<const uint4*>(v_cache + e);                         \
    } else {                                                                          \
      const long row = s0 + tok;                                                      \
      kreg[j] = *reinterpret_cast<const uint4*>(kbase + row * row_stride + c * 8);    \
      vreg[j] = *reinterpret_cast<const uint4*>(vbase + row * row_stride + c * 8);    \
    }                                                                                 \
  }
  PF_LOAD_TILE(0)
  const int qrow = (lane >> 2) & 3, pcol = lane & 3;
  for (int k0 = 0; k0 < kend_wg; k0 += PF_KT) {
    __syncthreads();                                             // previous tile fully read
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + 256 * j;
      const int r = i / CH, c = i % CH;
      *reinterpret_cast<uint4*>(ktile + r * KROW + c * 8) = kreg[j];
      *reinterpret_cast<uint4*>(vtile + r * VROW + c * 8) = vreg[j];
    }
    __syncthreads();                                             // tile visible to all waves
    if (k0 + PF_KT < kend_wg) { PF_LOAD_TILE(k0 + PF_KT) }       // in flight during compute
    if (!active || k0 >= kend_w) continue;                       // tile above this wave's rows
    // ---- S^T = K . Q^T over four 16-key subtiles
    f32x4 s_acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u16* kp = ktile + (16 * s + col) * KROW;
      s_acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        s_acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            *reinterpret_cast<const bf16x8*>(kp + kk * 32 + grp * 8), qf[kk], s_acc[s], 0, 0, 0);
    }
    float p[16], tmax = -INFINITY;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * s + 4 * grp + r;
        const float v = (key <= my_q && key < nkeys) ? s_acc[s][r] * scale_log2 : -INFINITY;
        p[s * 4 + r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    // rows past the sequence end may see no valid key: keep them finite
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) { p[j] = exp2f(p[j] - m_use); psum += p[j]; }
    l_part = l_part * alpha + psum;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a = __shfl(alpha, 4 * grp + r, 64);
#pragma unroll
      for (int i = 0; i < DB; ++i) o_acc[i][r] *= a;
    }
    // ---- O += P . V, two 32-key halves; B operand rows: keys 32h + 4grp + q and
    // 32h + 16 + 4grp + q (the p[] key order), cols 16i + 4p via tr16 reads
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 8; ++j) pa[j] = (__bf16)p[8 * hh + j];
#pragma unroll
      for (int i = 0; i < DB; ++i) {
        const u16* a0 = vtile + (32 * hh + 4 * grp + qrow) * VROW + 16 * i + 4 * pcol;
        const u16* a1 = vtile + (32 * hh + 16 + 4 * grp + qrow) * VROW + 16 * i + 4 * pcol;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(a0));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(a1));
        s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o_acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, *reinterpret_cast<bf16x8*>(&w),
                                                          o_acc[i], 0, 0, 0);
      }
    }
  }
#undef PF_LOAD_TILE
  if (!active) return;
  float l_tot = l_part + __shfl_xor(l_part, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float iv = __shfl(inv, 4 * grp + r, 64);
    const int qr = q0 + 4 * grp + r;
    if (qr < len) {
      u16* op = out + (long)(s0 + qr) * out_stride + (long)h * HD;
#pragma unroll
      for (int i = 0; i < DB; ++i) op[16 * i + col] = f2bf(o_acc[i][r] * iv);
    }
  }
}

template <bool PAGED>
static int launch_prefill(void* out, int out_stride, const void* qkv, int row_stride,
                          const int* cu_seqlens, int num_seqs, int max_seqlen, int hq, int hkv,
                          int hd, float scale, const int* ctx_lens, const void* k_cache,
                          const void* v_cache, const int* block_tables, int bt_stride,
                          int block_size, hipStream_t st) {
  if (num_seqs <= 0 || max_seqlen <= 0) return 0;
  if (hq % hkv || (hd != 64 && hd != 128)) return (int)hipErrorInvalidValue;
  const int rows_per_wg = PF_WAVES * PF_QROWS;
  dim3 grid((max_seqlen + rows_per_wg - 1) / rows_per_wg, num_seqs, hq);
  const float sl2 = scale * 1.4426950408889634f;
  if (hd == 128)
    prefill_attn_kernel<128, PAGED><<<grid, 256, 0, st>>>(
        (u16*)out, out_stride, (const u16*)qkv, row_stride, cu_seqlens, hq, hkv, sl2, ctx_lens,
        (const u16*)k_cache, (const u16*)v_cache, block_tables, bt_stride, block_size);
  else
    prefill_attn_kernel<64, PAGED><<<grid, 256, 0, st>>>(
        (u16*)out, out_stride, (const u16*)qkv, row_stride, cu_seqlens, hq, hkv, sl2, ctx_lens,
        (const u16*)k_cache, (const u16*)v_cache, block_tables, bt_stride, block_size);
  DLI_RETURN_LAUNCH();
}

extern "C" int dli_prefill_attention(void* out, int out_stride, const void* qkv, int row_stride,
                                     const int* cu_seqlens, int num_seqs, int max_seqlen, int hq,
                                     int hkv, int hd, float scale, hipStream_t st) {
  return launch_prefill<false>(out, out_stride, qkv, row_stride, cu_seqlens, num_seqs,
                               max_seqlen, hq, hkv, hd, scale, nullptr, nullptr, nullptr,
                               nullptr, 0, 16, st);
}

// Chunked prefill: q from qkv rows [cu[s], cu[s+1]); keys 0..ctx_lens[s]-1 of sequence s
// from the paged caches [num_blocks, hkv, block_size, hd] through block_tables[s, :].
extern "C" int dli_prefill_attention_paged(void* out, int out_stride, const void* qkv,
                                           int row_stride, const int* cu_seqlens,
                                           const int* ctx_lens, const void* k_cache,
                                           const void* v_cache, const int* block_tables,
                                           int bt_stride, int num_seqs, int max_seqlen, int hq,
                                           int hkv, int hd, int block_size, float scale,
                                           hipStream_t st) {
  if (block_size <= 0) return (int)hipErrorInvalidValue;
  return launch_prefill<true>(out, out_stride, qkv, row_stride, cu_seqlens, num_seqs,
                              max_seqlen, hq, hkv, hd, scale, ctx_lens, k_cache, v_cache,
                              block_tables, bt_stride, block_size, st);
}
