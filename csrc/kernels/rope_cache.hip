// RoPE (rotate-half, HF Llama convention) applied IN PLACE to q and k inside the fused QKV
// activation, fused with the paged KV-cache write — SURVEY.md §2.4 K5/K6.
//
// One lane owns 8 dims of the first half of a head and the matching 8 dims of the second
// half (16-B loads of each), so a head of 128 dims is 8 lanes and the rotation needs no
// cross-lane traffic. cos/sin come from a host-precomputed fp32 table [max_pos, hd]
// (cdna_hip_programming.md App. B: no on-device trig in memory-bound elementwise ops).
//
// Cache layouts (see ops/reference.py): k_cache and v_cache both [nblk, Hkv, bs, hd].
#include "common.h"

__global__ void __launch_bounds__(256) rope_cache_kernel(
    u16* __restrict__ qkv, int row_stride, const int* __restrict__ positions,
    const int* __restrict__ slot_mapping, const float* __restrict__ cos_sin,
    u16* __restrict__ k_cache, u16* __restrict__ v_cache, int T, int hq, int hkv, int hd,
    int block_size, int use_rope) {
  const int lanes_per_head = hd >> 4;            // each lane: 8 dims + their partner 8 dims
  const int heads = hq + 2 * hkv;
  const long total = (long)T * heads * lanes_per_head;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int c = (int)(gid % lanes_per_head);
  const long th = gid / lanes_per_head;
  const int h = (int)(th % heads);
  const int t = (int)(th / heads);
  const int half = hd >> 1;
  u16* base = qkv + (long)t * row_stride + (long)h * hd;
  const int d0 = c * 8;                         // dims [d0, d0+8) and [half+d0, half+d0+8)
  float x1[8], x2[8];
  load8(base + d0, x1);
  load8(base + half + d0, x2);
  const bool is_q = h < hq, is_k = !is_q && h < hq + hkv;
  if (use_rope && (is_q || is_k)) {
    const float* cs = cos_sin + (long)positions[t] * hd;
    float o1[8], o2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float co = cs[d0 + j], si = cs[half + d0 + j];
      o1[j] = x1[j] * co - x2[j] * si;
      o2[j] = x2[j] * co + x1[j] * si;
    }
    store8(base + d0, o1);
    store8(base + half + d0, o2);
    // cache receives exactly the bf16 values now stored in qkv
#pragma unroll
    for (int j = 0; j < 8; ++j) { x1[j] = bf2f(f2bf(o1[j])); x2[j] = bf2f(f2bf(o2[j])); }
  }
  if (is_q || k_cache == nullptr) return;
  const int slot = slot_mapping[t];
  if (slot < 0) return;
  const int blk = slot / block_size, off = slot - blk * block_size;
  // K and V share the token-major [blk, head, off, hd] layout: whole-row 16-B stores (a
  // transposed V made every decode step a 2-byte scatter, i.e. a read-modify-write of a
  // memory sector per element)
  u16* dst = is_k ? k_cache + (((long)blk * hkv + (h - hq)) * block_size + off) * hd
                  : v_cache + (((long)blk * hkv + (h - hq - hkv)) * block_size + off) * hd;
  store8(dst + d0, x1);
  store8(dst + half + d0, x2);
}

extern "C" int dli_rope_cache(void* qkv, int row_stride, const int* positions,
                              const int* slot_mapping, const float* cos_sin, void* k_cache,
                              void* v_cache, int T, int hq, int hkv, int hd, int block_size,
                              int use_rope, hipStream_t st) {
  if (T <= 0) return 0;
  if (hd % 16 != 0) return (int)hipErrorInvalidValue;
  const long total = (long)T * (hq + 2 * hkv) * (hd / 16);
  const int blocks = (int)((total + 255) / 256);
  rope_cache_kernel<<<blocks, 256, 0, st>>>((u16*)qkv, row_stride, positions, slot_mapping,
                                             cos_sin, (u16*)k_cache, (u16*)v_cache, T, hq, hkv,
                                             hd, block_size, use_rope);
  DLI_RETURN_LAUNCH();
}
