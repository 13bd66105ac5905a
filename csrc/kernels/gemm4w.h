// The 4-wave 256x256 MFMA GEMM (gemm4w_kernel: one wave per SIMD, 128x128 wave tiles,
// accumulators pinned in the AGPR file) and its launcher, shared by the production tiles
// (gemm4w.hip: 34, 41, 45).
#pragma once
#include "gemm_common.h"

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
// Only tiles 34 (VAR 8), 41 (8 | 32) and 45 (8 | 4096) are instantiated; the other VAR bits
// are the round-4 A/B variants, kept for diagnostics (measurements: profiles/r4/gemm4w/).
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
  // cycles: an LDS-DMA issue costs ~60 cycles among MFMAs, /opt/skills/guides/MI355X_MICROARCH.md constants).
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
        if (row < Mg && col < N) slab_quad_fp32(srow + col, v, sm & 3, vec, N - col);
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

