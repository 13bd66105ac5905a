// Causal variable-length (packed) GQA prefill attention on MFMA — SURVEY.md §2.4 K7.
//
// Reads q/k/v straight out of the fused QKV activation (row stride = (Hq+2Hkv)*hd) after
// the in-place RoPE, so no separate K/V copies exist. Each wave owns 16 query rows of one
// query head and streams 32-key tiles (flash-attention online softmax):
//   S^T[key, q] = K . Q^T        mfma_f32_16x16x32_bf16, K rows as A operand (16-B loads)
//   softmax along keys           exp2 domain; per-q max over 2 lane groups (2 shuffles)
//   O[q, d] += P[q, key] . V     P re-used from the accumulator registers (permuted key
//                                order); V staged row-major in a per-wave LDS tile (rows
//                                padded to hd*2+32 B) and read as the B operand with the
//                                CDNA4 transposing ds_read_b64_tr_b16 (cdna_hip_programming.md T10)
// Grid: (ceil(max_len / 64), num_seqs, Hq); 4 independent waves per workgroup.
#include "common.h"

typedef short s16x4 __attribute__((ext_vector_type(4)));
#define PF_WAVES 4
#define PF_QROWS 16
#define PF_KT 32

template <int HD>
__global__ void __launch_bounds__(256) prefill_attn_kernel(
    u16* __restrict__ out, int out_stride, const u16* __restrict__ qkv, int row_stride,
    const int* __restrict__ cu_seqlens, int hq, int hkv, float scale_log2) {
  constexpr int KK = HD / 32, DB = HD / 16;
  constexpr int VROW = HD + 16;                    // padded LDS row, in u16 (HD*2 + 32 bytes)
  __shared__ __attribute__((aligned(16))) u16 vtile[PF_WAVES][PF_KT * VROW];
  const int seq = blockIdx.y, h = blockIdx.z;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;
  const int s0 = cu_seqlens[seq], len = cu_seqlens[seq + 1] - s0;
  const int q0 = (blockIdx.x * PF_WAVES + wid) * PF_QROWS;      // position within the sequence
  if (q0 >= len) return;                                         // wave-uniform exit
  const int G = hq / hkv, kvh = h / G;
  const u16* qbase = qkv + (long)h * HD;
  const u16* kbase = qkv + (long)(hq + kvh) * HD;
  const u16* vbase = qkv + (long)(hq + hkv + kvh) * HD;

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
  const int my_q = q0 + col;               // the query row this lane's S^T column belongs to
  float m_run = -INFINITY, l_part = 0.f;
  f32x4 o_acc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) o_acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16* vt = vtile[wid];
  const int kend = min(len, q0 + PF_QROWS);                      // causal bound for this wave

  for (int k0 = 0; k0 < kend; k0 += PF_KT) {
    // ---- stage V[k0 .. k0+32) row-major into LDS (each lane: 16-B pieces)
    constexpr int PIECES = PF_KT * HD / 8;                      // 16-B pieces per tile
#pragma unroll
    for (int i = lane; i < PIECES; i += 64) {
      const int r = i / (HD / 8), c = i % (HD / 8);
      const int key = min(k0 + r, len - 1);
      uint4 v = *reinterpret_cast<const uint4*>(vbase + (long)(s0 + key) * row_stride + c * 8);
      *reinterpret_cast<uint4*>(vt + r * VROW + c * 8) = v;
    }
    // ---- S^T = K . Q^T for two 16-key subtiles
    f32x4 s_acc[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int key = min(k0 + 16 * s + col, len - 1);
      const u16* kp = kbase + (long)(s0 + key) * row_stride;
      s_acc[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        uint4 kv = *reinterpret_cast<const uint4*>(kp + kk * 32 + grp * 8);
        s_acc[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&kv),
                                                          qf[kk], s_acc[s], 0, 0, 0);
      }
    }
    float p[8], tmax = -INFINITY;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = k0 + 16 * s + 4 * grp + r;
        const float v = (key <= my_q && key < len) ? s_acc[s][r] * scale_log2 : -INFINITY;
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
    for (int j = 0; j < 8; ++j) { p[j] = exp2f(p[j] - m_use); psum += p[j]; }
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // V tile writes landed (same wave)
    // B operand rows: keys 4grp+q (first read) and 16+4grp+q (second), cols 16db + 4p
    // tr16 addressing: lane 4q+p of each 16-lane group names row q, columns 4p..4p+3
    const int qrow = (lane >> 2) & 3, pcol = lane & 3;
#pragma unroll
    for (int i = 0; i < DB; ++i) {
      const u16* a0 = vt + (4 * grp + qrow) * VROW + 16 * i + 4 * pcol;
      const u16* a1 = vt + (16 + 4 * grp + qrow) * VROW + 16 * i + 4 * pcol;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(a0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(a1));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      s16x8 w = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o_acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, *reinterpret_cast<bf16x8*>(&w),
                                                        o_acc[i], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before next overwrite
  }
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

extern "C" int dli_prefill_attention(void* out, int out_stride, const void* qkv, int row_stride,
                                     const int* cu_seqlens, int num_seqs, int max_seqlen, int hq,
                                     int hkv, int hd, float scale, hipStream_t st) {
  if (num_seqs <= 0 || max_seqlen <= 0) return 0;
  if (hq % hkv || (hd != 64 && hd != 128)) return (int)hipErrorInvalidValue;
  const int rows_per_wg = PF_WAVES * PF_QROWS;
  dim3 grid((max_seqlen + rows_per_wg - 1) / rows_per_wg, num_seqs, hq);
  const float sl2 = scale * 1.4426950408889634f;
  if (hd == 128)
    prefill_attn_kernel<128><<<grid, 256, 0, st>>>((u16*)out, out_stride, (const u16*)qkv,
                                                   row_stride, cu_seqlens, hq, hkv, sl2);
  else
    prefill_attn_kernel<64><<<grid, 256, 0, st>>>((u16*)out, out_stride, (const u16*)qkv,
                                                  row_stride, cu_seqlens, hq, hkv, sl2);
  DLI_RETURN_LAUNCH();
}
