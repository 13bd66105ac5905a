// 8-wave "8-phase ping-pong" MFMA GEMMs (tile ids 22, 26, 28): 256x256 (gemm8p_kernel),
// 256x224 (gemm8p224_kernel) and 256x128 (gemm8p128_kernel) block tiles, two wave groups
// alternating MFMA and load segments (cdna_hip_programming.md §5 'The 256² 8-phase template').
#include "gemm_common.h"

// ---------------------------------------------------------------------------------------
// 256x256 "8-phase ping-pong" GEMM (cdna_hip_programming.md §5 'The 256² 8-phase template',
// T3+T4+T5; /opt/skills/guides/MI355X_MICROARCH.md 'Two waves per SIMD' items 1, 7, 9).
//
// 8 waves = 2 groups of 4 (g = wid >> 2 = the wave's 128-row half of the tile; one wave of
// each group per SIMD). Every K-tile (BK = 64) is 4 phases; a phase is a LOAD segment
// (this phase's ds_reads + one quarter of a later K-tile's glds + a counted vmcnt) and a
// MATRIX segment (16 MFMAs, one 64x32 quadrant of the wave's 128x64 output), separated by
// raw s_barriers. Group 1 runs one barrier behind group 0, so on every SIMD one wave is in
// its matrix segment while its partner is in its load segment.
//
//   phase | ds_read_b128 (this K-tile)        | MFMAs          | glds issued
//   0     | A rows 0-63 of the half, B 0-31   | acc[0-3][0-1]  | slot 3 of K-tile T+1
//   1     | B cols 32-63                      | acc[0-3][2-3]  | slot 0 of K-tile T+2
//   2     | A rows 64-127                     | acc[4-7][2-3]  | slot 1 of K-tile T+2
//   3     | -                                 | acc[4-7][0-1]  | slot 2 of K-tile T+2
//
// LDS: 2 buffers x (A 256x64 + W 256x64) bf16 = 128 KiB (1 workgroup / CU), 128-B rows with
// the chunk XOR swizzle of gemm_bf16_kernel. Staging slots per group (2 glds per lane each):
// group 0 stages A rows 0-63 / 64-127 and the even 32-row W chunks, group 1 A rows
// 128-191 / 192-255 and the odd W chunks. With segments numbered s (group 0 loads in even
// s, group 1 in odd s) every slot is restaged >= 2 segments after its last ds_read of the
// K-tile two back (WAR) and retired by its issuer's vmcnt >= 1 barrier before its first
// ds_read (RAW) when every load segment leaves the last 3 segments' glds in flight:
// vmcnt(6) in steady state, fewer when the K loop's tail issues nothing.
template <int EPI, int VAR = 0>
__global__ void __launch_bounds__(512) gemm8p_kernel(
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
    // grouped order: an XCD's ~32 consecutive tiles cover GM tile-rows x 32/GM tile-columns,
    // so its CUs share both A and W panels in its L2 (n-major order shares W only)
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
  const u16* Ab = A + (long)row0 * lda;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid >> 2, gw = wid & 3;           // group (= M half), wave in group (= N quarter)

  // ---- staging: slot s (0..3) x instruction i (0..1): element offset of this lane's source
  // and the wave-uniform LDS byte offset of the 1-KiB piece (8 rows x 128 B)
  int src[4][2];
  int dst[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int rb, is_a;
      if ((s & 1) == 0) { rb = 64 * (2 * g + (s >> 1)) + 32 * i + 8 * gw; is_a = 1; }
      else { rb = 64 * (2 * (s >> 1) + i) + 32 * g + 8 * gw; is_a = 0; }
      const int r = rb + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      if (is_a) src[s][i] = min(m0 + r, Mg - 1) * lda + kb + c * 8;
      else src[s][i] = min(n0 + r, N - 1) * ldw + kb + c * 8;
      dst[s][i] = (is_a ? 0 : A_BYTES) + rb * 128;
    }
  // deep plan (VAR & 4): per group, A region h (2 glds) and all 4 W chunks of its parity (4 glds)
  int srcB[4], dstB[4];
#pragma unroll
  for (int c4 = 0; c4 < 4; ++c4) {
    const int rb = 64 * c4 + 32 * g + 8 * gw;
    const int r = rb + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    srcB[c4] = min(n0 + r, N - 1) * ldw + kb + c * 8;
    dstB[c4] = A_BYTES + rb * 128;
  }
  auto issue_a = [&](int h, int kt) {             // h: A rows 64h..64h+63 of the group's half
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(Ab + src[2 * h][i] + kt * BK),
                                       (lds_void*)(lds + dst[2 * h][i]), 16, 0, 0);
  };
  auto issue_b = [&](int kt) {
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4)
      __builtin_amdgcn_global_load_lds((gbl_void*)(Wg + srcB[c4] + kt * BK),
                                       (lds_void*)(lds + dstB[c4]), 16, 0, 0);
  };
  auto issue = [&](auto S, int kt) {
    constexpr int s = decltype(S)::value;
    const u16* base = (s & 1) ? Wg : Ab;
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(base + src[s][i] + kt * BK),
                                       (lds_void*)(lds + dst[s][i]), 16, 0, 0);
  };

  // ---- fragments
  const int fr = lane & 15, fq = lane >> 4;
  auto read_frag = [&](const char* part, int row, int kk) -> bf16x8 {
    const int c = kk * 4 + fq;
    return *reinterpret_cast<const bf16x8*>(part + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: K-tiles 0 and 1 in full
  if (nk > 0) {
    issue(std::integral_constant<int, 0>{}, 0); issue(std::integral_constant<int, 1>{}, 0);
    issue(std::integral_constant<int, 2>{}, 0); issue(std::integral_constant<int, 3>{}, 0);
  }
  if (nk > 1) {
    issue(std::integral_constant<int, 0>{}, 1); issue(std::integral_constant<int, 1>{}, 1);
    issue(std::integral_constant<int, 2>{}, 1); issue(std::integral_constant<int, 3>{}, 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (g == 1) {                                    // stagger: group 1 runs one segment behind
    __builtin_amdgcn_s_barrier();
    if (VAR & 256) __builtin_amdgcn_s_setprio(1);  // static priority for the younger half
  }

  const int last_issue_seg = 4 * nk - 8;          // load segments 1..last issue glds
  bf16x8 a0[4][2], a1[4][2], b0[2][2], b1[2][2];

  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  auto wait_deep = [&](int u) {                   // keep the last 5 load segments' glds in flight
    int cnt = 0;
#pragma unroll
    for (int d = 0; d < 5; ++d) {
      const int v = u - d;
      const int q = v & 3;
      if (v >= 1 && q != 0 && (v >> 2) + 2 < nk) cnt += (q == 2) ? 4 : 2;
    }
    switch (cnt) {                                 // wave-uniform
      case 0: wait_vmcnt<0>(); break;
      case 2: wait_vmcnt<2>(); break;
      case 4: wait_vmcnt<4>(); break;
      case 6: wait_vmcnt<6>(); break;
      case 8: wait_vmcnt<8>(); break;
      case 10: wait_vmcnt<10>(); break;
      default: wait_vmcnt<12>(); break;
    }
  };
  auto wait_issued = [&](int u) {
    if (VAR & 4) { wait_deep(u); return; }
    if (VAR & 512) {
      // one counted wait per K-tile (the 8-phase template's schedule): at phase 3 of K-tile
      // T every DMA of T+1 is retired; only T+2's slots 0-2 (issued in phases 1-3) stay in
      // flight. Phases 0-2 do not wait at all.
      if ((u & 3) == 3) {
        if ((u >> 2) + 2 < nk) wait_vmcnt<6>();
        else wait_vmcnt<0>();
      }
      return;
    }
    const int lo = max(1, u - 2), hi = min(u, last_issue_seg);
    const int cnt = hi >= lo ? hi - lo + 1 : 0;    // wave-uniform
    if (cnt >= 3) wait_vmcnt<6>();
    else if (cnt == 2) wait_vmcnt<4>();
    else if (cnt == 1) wait_vmcnt<2>();
    else wait_vmcnt<0>();
  };

  for (int kt = 0; kt < nk; ++kt) {
    const char* abuf = smem + (kt & 1) * BUF;
    const char* wbuf = abuf + A_BYTES;
    const int arow = g * 128 + fr, wrow = gw * 64 + fr;
    const int u0 = 4 * kt;
    auto phase = [&](auto P) {
      constexpr int p = decltype(P)::value;
      auto reads = [&]() {
        if (p == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) a0[i][kk] = read_frag(abuf, arow + 16 * i, kk);
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) b0[j][kk] = read_frag(wbuf, wrow + 16 * j, kk);
        } else if (p == 1) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) b1[j][kk] = read_frag(wbuf, wrow + 32 + 16 * j, kk);
        } else if (p == 2) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) a1[i][kk] = read_frag(abuf, arow + 64 + 16 * i, kk);
        }
      };
      auto stage = [&]() {
        if (p == 0) {
          if (!(VAR & 4) && kt >= 1 && kt + 1 < nk) issue(std::integral_constant<int, 3>{}, kt + 1);
        } else if (kt + 2 < nk) {
          if (VAR & 4) {
            if (p == 1) issue_a(0, kt + 2);
            else if (p == 2) issue_b(kt + 2);
            else issue_a(1, kt + 2);
          } else {
            issue(std::integral_constant<int, (p + 3) & 3>{}, kt + 2);
          }
        }
      };
      if (VAR & 64) { stage(); reads(); }
      else { reads(); stage(); }
      if (!(VAR & 32)) wait_issued(u0 + p);
      barrier();
      if (!(VAR & 256)) __builtin_amdgcn_s_setprio(1);
      const bf16x8 (&af)[4][2] = (p < 2) ? a0 : a1;
      const bf16x8 (&bf)[2][2] = (p == 0 || p == 3) ? b0 : b1;
      constexpr int I0 = (p < 2) ? 0 : 4, J0 = (p == 0 || p == 3) ? 0 : 2;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                bf[j][kk], af[i][kk], acc[I0 + i][J0 + j], 0, 0, 0);
      if (!(VAR & 256)) __builtin_amdgcn_s_setprio(0);
      barrier();
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    phase(std::integral_constant<int, 3>{});
  }
  if (g == 0) {                                    // balance group 1's stagger barrier
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue (transposed accumulators):
  // acc[I][J][r] = C[m0 + 128g + 16I + fr][n0 + 64gw + 16J + 4fq + r]
  const int wr0 = m0 + 128 * g, wc0 = n0 + 64 * gw;
  if (gridDim.y > 1) {
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
      float* srow = slab + (long)(row0 + row) * N;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wc0 + 16 * j + 4 * fq;
        if (col >= N) continue;
        if (EPI == EPI_SLAB16) slab_quad16(srow + col, acc[i][j], vec, N - col, ws);
        else slab_quad(srow + col, acc[i][j], sm, vec, N - col, ws);
      }
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const int gcol = wc0 + 16 * j;
        if (gcol < N)
          store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][j],
                          acc[i][j + 1], vec);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = wr0 + 16 * i + fr;
    if (row >= Mg) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc0 + 16 * j + 4 * fq;
      if (col < N) store_quad<EPI>(C, ldc, row0 + row, col, N, acc[i][j], bias, vec);
    }
  }
}

// ---------------------------------------------------------------------------------------
// 256x224 ping-pong GEMM: the 8-phase schedule of gemm8p_kernel for N-tiles of 224 columns,
// so a GEMM whose N is a multiple of 7 x 32 fills the chip where 256-wide tiles leave CUs
// idle: the Llama-3 gate/up projection at M = 512 (N = 28672) is 2 x 128 = 256 tiles on 256
// CUs instead of 224 (one workgroup per CU at 128 KiB of LDS).
//
// Waves: group g = wid >> 2 = the tile's 128-row half (one wave of each group per SIMD,
// group 1 one barrier behind); in a group, wave (wm, wn) = (w4 >> 1, w4 & 1) owns rows
// 128 g + 64 wm .. +63 and columns 112 wn .. +111: 4 x 7 MFMA blocks, as gemm8p's 8 x 4.
// K-tile T (BK = 64) = 4 phases, each a LOAD segment (ds_reads of T, LDS-DMA of T+2) and a
// MATRIX segment (MFMAs):
//   phase | reads                              | MFMAs              | DMA for T+2
//   0     | A rows +0..31 (both kk), B +0..63  | 2 x 4 blocks       | -
//   1     | B +64..111                         | 2 x 3 blocks       | A "h0", B "h0"
//   2     | A rows +32..63                     | 2 x 3 blocks       | B "h1"
//   3     | -                                  | 2 x 4 blocks       | A "h1"
// (A h0 = rows r % 64 < 32, h1 the rest; B h0 = rows 0-63 and 112-175, h1 = rows 64-111,
// 176-223 and 224-255: the next tile's rows, staged so every wave DMAs 2 pieces per region,
// never read.) Every LOAD segment retires its ds_reads (lgkmcnt(0)) before its barrier, so a
// region is restaged in the phase after its last reading phase — after group 1's read too.
// Phase 3 waits (counted vmcnt: T+2's 8 DMAs stay in flight) for every DMA of T+1, retired
// for all readers by the barrier closing the segment. SiLU pairs are 16-column blocks (2p,
// 2p+1); the pair (6, 7) straddles the two waves of a row band and meets through LDS.
template <int EPI>
__global__ void __launch_bounds__(512) gemm8p224_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws, const int* __restrict__ group_off) {
  constexpr int BM = 256, BN = 224;
  constexpr int A_BYTES = BM * BK * 2, BUF = 2 * A_BYTES;     // A 256 rows + B image 256 rows
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
  constexpr int GM = 4;                            // grouped tile order (see gemm8p_kernel)
  const int per_group = GM * tiles_n;
  const int first_m = (tile / per_group) * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_g = tile % per_group;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mg) return;
  const int kb = ks * k_split_len;
  const int nk = min(k_split_len, K - kb) / BK;
  const u16* Ab = A + (long)row0 * lda;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid >> 2, w4 = wid & 3, wm = w4 >> 1, wn = w4 & 1;

  // ---- LDS-DMA pieces (8 rows x 128 B; lane L lands at row L/8, physical chunk L%8, so it
  // loads logical chunk (L%8) ^ ((r >> 1) & 7)). Region pieces (16 per region, wave wid
  // takes region pieces wid and wid + 8): A h0 piece q -> rows 64 (q >> 2) + 8 (q & 3),
  // A h1 -> the same + 32; B h0 piece q -> rows 8q (q < 8) or 112 + 8 (q - 8); B h1 piece q
  // -> rows 64 + 8q (q < 6), 176 + 8 (q - 6) (q < 12), 224 + 8 (q - 12).
  auto piece_row = [](int region, int q) {
    switch (region) {
      case 0: return 64 * (q >> 2) + 8 * (q & 3);
      case 1: return 64 * (q >> 2) + 8 * (q & 3) + 32;
      case 2: return q < 8 ? 8 * q : 112 + 8 * (q - 8);
      default: return q < 6 ? 64 + 8 * q : (q < 12 ? 176 + 8 * (q - 6) : 224 + 8 * (q - 12));
    }
  };
  int src[4][2], dst[4][2];                        // [region: A h0, A h1, B h0, B h1][piece]
#pragma unroll
  for (int rg = 0; rg < 4; ++rg)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rb = piece_row(rg, wid + 8 * i);
      const int r = rb + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      if (rg < 2) src[rg][i] = min(m0 + r, Mg - 1) * lda + kb + c * 8;
      else src[rg][i] = min(n0 + r, N - 1) * ldw + kb + c * 8;
      dst[rg][i] = (rg < 2 ? 0 : A_BYTES) + rb * 128;
    }
  auto dma = [&](auto RG, int kt) {
    constexpr int rg = decltype(RG)::value;
    const u16* base = rg < 2 ? Ab : Wg;
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(base + src[rg][i] + kt * BK),
                                       (lds_void*)(lds + dst[rg][i]), 16, 0, 0);
  };
  auto dma_all = [&](int kt) {
    dma(std::integral_constant<int, 0>{}, kt); dma(std::integral_constant<int, 1>{}, kt);
    dma(std::integral_constant<int, 2>{}, kt); dma(std::integral_constant<int, 3>{}, kt);
  };

  const int fr = lane & 15, fq = lane >> 4;
  auto read_frag = [&](const char* part, int row, int kk) -> bf16x8 {
    const int c = kk * 4 + fq;
    return *reinterpret_cast<const bf16x8*>(part + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  };
  f32x4 acc[4][7];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: K-tiles 0 and 1 whole
  if (nk > 0) dma_all(0);
  if (nk > 1) { dma_all(1); wait_vmcnt<8>(); }
  else wait_vmcnt<0>();
  __syncthreads();
  if (g == 1) {                                    // stagger: group 1 runs one segment behind
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);                 // static priority for the younger half
  }
  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  const int arow = 128 * g + 64 * wm + fr, brow = 112 * wn + fr;
  bf16x8 a0[2][2], a1[2][2], b0[4][2], b1[3][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* abuf = smem + (kt & 1) * BUF;
    const char* bbuf = abuf + A_BYTES;
    auto phase = [&](auto P) {
      constexpr int p = decltype(P)::value;
      if (p == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a0[i][kk] = read_frag(abuf, arow + 16 * i, kk);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b0[j][kk] = read_frag(bbuf, brow + 16 * j, kk);
      } else if (p == 1) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b1[j][kk] = read_frag(bbuf, brow + 64 + 16 * j, kk);
        if (kt + 2 < nk) { dma(std::integral_constant<int, 0>{}, kt + 2);
                           dma(std::integral_constant<int, 2>{}, kt + 2); }
      } else if (p == 2) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a1[i][kk] = read_frag(abuf, arow + 32 + 16 * i, kk);
        if (kt + 2 < nk) dma(std::integral_constant<int, 3>{}, kt + 2);
      } else {
        if (kt + 2 < nk) { dma(std::integral_constant<int, 1>{}, kt + 2); wait_vmcnt<8>(); }
        else wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0): this segment's reads done
      barrier();
      const bf16x8 (&af)[2][2] = (p < 2) ? a0 : a1;
      constexpr int I0 = (p < 2) ? 0 : 2;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (p == 0 || p == 3) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[I0 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  b0[j][kk], af[i][kk], acc[I0 + i][j], 0, 0, 0);
          } else {
#pragma unroll
            for (int j = 0; j < 3; ++j)
              acc[I0 + i][4 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  b1[j][kk], af[i][kk], acc[I0 + i][4 + j], 0, 0, 0);
          }
        }
      barrier();
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    phase(std::integral_constant<int, 3>{});
  }
  if (g == 0) __builtin_amdgcn_s_barrier();       // balance group 1's stagger barrier

  // ---- epilogue (transposed accumulators):
  // acc[i][j][r] = C[m0 + 128 g + 64 wm + 16 i + fr][n0 + 112 wn + 16 j + 4 fq + r]
  const int wr0 = m0 + 128 * g + 64 * wm, wc0 = n0 + 112 * wn;
  if (gridDim.y > 1) {
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
      float* srow = slab + (long)(row0 + row) * N;
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const int col = wc0 + 16 * j + 4 * fq;
        if (col >= N) continue;
        if (EPI == EPI_SLAB16) slab_quad16(srow + col, acc[i][j], vec, N - col, ws);
        else slab_quad(srow + col, acc[i][j], sm, vec, N - col, ws);
      }
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {
    // block 6 of wave wn = 0 (gate) pairs with block 0 of wave wn = 1 (up): through LDS
    __syncthreads();                               // every wave is past its last LDS read
    float* xch = reinterpret_cast<float*>(smem) + (2 * g + wm) * 1024;   // 64 x 16 fp32
    if (wn == 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<f32x4*>(xch + (16 * i + fr) * 16 + 4 * fq) = acc[i][0];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
      // own pairs: wave 0 blocks (0,1) (2,3) (4,5) + (6, partner's 0); wave 1 (1,2) (3,4)
      // (5,6) (compile-time block indices in each branch: no runtime-indexed registers)
      if (wn == 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int gcol = wc0 + 32 * q;
          if (gcol < N)
            store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][2 * q],
                            acc[i][2 * q + 1], vec);
        }
        const int gcol = wc0 + 16 * 6;
        if (gcol < N) {
          const f32x4 up = *reinterpret_cast<const f32x4*>(xch + (16 * i + fr) * 16 + 4 * fq);
          store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][6], up, vec);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int gcol = wc0 + 16 + 32 * q;
          if (gcol < N)
            store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][2 * q + 1],
                            acc[i][2 * q + 2], vec);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wr0 + 16 * i + fr;
    if (row >= Mg) continue;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int col = wc0 + 16 * j + 4 * fq;
      if (col < N) store_quad<EPI>(C, ldc, row0 + row, col, N, acc[i][j], bias, vec);
    }
  }
}

// ---------------------------------------------------------------------------------------
// 256x128 ping-pong GEMM: the 8-phase schedule of gemm8p224_kernel for 128-column N-tiles.
// Where 256-column tiles leave most of the chip idle or need deep K splits: the Mixtral
// grouped down projection (N = 4096, one 256-row tile per expert: 8 x 16 = 128 workgroups of
// 256x256 / 152 of 256x224, here 8 x 32 = 256), and the dense N = 4096 projections at
// M = 512 (64 tiles: split-K 4 fills 256 CUs with half the fp32 slab bytes of 32 tiles x 8).
//
// Waves: group g = wid >> 2 = the tile's 128-row half (one wave of each group per SIMD,
// group 1 one barrier behind); wave (wm, wn) = (w4 >> 1, w4 & 1) of a group owns rows
// 128 g + 64 wm .. +63 and columns 64 wn .. +63: 4 x 4 MFMA blocks.
//   phase | reads                              | MFMAs             | DMA for T+2
//   0     | A rows +0..31 (both kk), B +0..31  | rows 0-31, cols 0-31   | -
//   1     | B +32..63                          | rows 0-31, cols 32-63  | A h0
//   2     | A rows +32..63                     | rows 32-63, cols 32-63 | B
//   3     | -                                  | rows 32-63, cols 0-31  | A h1, then a counted
//                                                                         wait for T+1's DMAs
// (A h0 = rows r % 64 < 32, h1 the rest; B = all 128 rows, last read in phase 1.) LDS:
// 2 x (A 256 x 64 + B 128 x 64) bf16 = 96 KiB. SiLU pairs (2p, 2p+1) stay inside a wave.
template <int EPI>
__global__ void __launch_bounds__(512) gemm8p128_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws, const int* __restrict__ group_off) {
  constexpr int BM = 256, BN = 128;
  constexpr int A_BYTES = BM * BK * 2, BUF = A_BYTES + BN * BK * 2;
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
  constexpr int GM = 4;                            // grouped tile order (see gemm8p_kernel)
  const int per_group = GM * tiles_n;
  const int first_m = (tile / per_group) * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int in_g = tile % per_group;
  const int tm = first_m + in_g % gsz, tn = in_g / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  if (m0 >= Mg) return;
  const int kb = ks * k_split_len;
  const int nk = min(k_split_len, K - kb) / BK;
  const u16* Ab = A + (long)row0 * lda;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wid >> 2, w4 = wid & 3, wm = w4 >> 1, wn = w4 & 1;

  // ---- LDS-DMA pieces (8 rows x 128 B; lane L lands at row L/8, physical chunk L%8, so it
  // loads logical chunk (L%8) ^ ((r >> 1) & 7)). 16 pieces per region, wave wid takes pieces
  // wid and wid + 8: A h0 piece q -> rows 64 (q >> 2) + 8 (q & 3), A h1 -> the same + 32,
  // B piece q -> rows 8 q.
  auto piece_row = [](int region, int q) {
    switch (region) {
      case 0: return 64 * (q >> 2) + 8 * (q & 3);
      case 1: return 64 * (q >> 2) + 8 * (q & 3) + 32;
      default: return 8 * q;
    }
  };
  int src[3][2], dst[3][2];                        // [region: A h0, A h1, B][piece]
#pragma unroll
  for (int rg = 0; rg < 3; ++rg)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rb = piece_row(rg, wid + 8 * i);
      const int r = rb + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      if (rg < 2) src[rg][i] = min(m0 + r, Mg - 1) * lda + kb + c * 8;
      else src[rg][i] = min(n0 + r, N - 1) * ldw + kb + c * 8;
      dst[rg][i] = (rg < 2 ? 0 : A_BYTES) + rb * 128;
    }
  auto dma = [&](auto RG, int kt) {
    constexpr int rg = decltype(RG)::value;
    const u16* base = rg < 2 ? Ab : Wg;
    char* lds = smem + (kt & 1) * BUF;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((gbl_void*)(base + src[rg][i] + kt * BK),
                                       (lds_void*)(lds + dst[rg][i]), 16, 0, 0);
  };
  auto dma_all = [&](int kt) {
    dma(std::integral_constant<int, 0>{}, kt); dma(std::integral_constant<int, 1>{}, kt);
    dma(std::integral_constant<int, 2>{}, kt);
  };

  const int fr = lane & 15, fq = lane >> 4;
  auto read_frag = [&](const char* part, int row, int kk) -> bf16x8 {
    const int c = kk * 4 + fq;
    return *reinterpret_cast<const bf16x8*>(part + row * 128 + ((c ^ ((row >> 1) & 7)) << 4));
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- prologue: K-tiles 0 and 1 whole
  if (nk > 0) dma_all(0);
  if (nk > 1) { dma_all(1); wait_vmcnt<6>(); }
  else wait_vmcnt<0>();
  __syncthreads();
  if (g == 1) {                                    // stagger: group 1 runs one segment behind
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_s_setprio(1);                 // static priority for the younger half
  }
  auto barrier = [&]() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
  };
  const int arow = 128 * g + 64 * wm + fr, brow = 64 * wn + fr;
  bf16x8 a0[2][2], a1[2][2], b0[2][2], b1[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* abuf = smem + (kt & 1) * BUF;
    const char* bbuf = abuf + A_BYTES;
    auto phase = [&](auto P) {
      constexpr int p = decltype(P)::value;
      if (p == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a0[i][kk] = read_frag(abuf, arow + 16 * i, kk);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b0[j][kk] = read_frag(bbuf, brow + 16 * j, kk);
      } else if (p == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b1[j][kk] = read_frag(bbuf, brow + 32 + 16 * j, kk);
        if (kt + 2 < nk) dma(std::integral_constant<int, 0>{}, kt + 2);
      } else if (p == 2) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) a1[i][kk] = read_frag(abuf, arow + 32 + 16 * i, kk);
        if (kt + 2 < nk) dma(std::integral_constant<int, 2>{}, kt + 2);
      } else {
        if (kt + 2 < nk) { dma(std::integral_constant<int, 1>{}, kt + 2); wait_vmcnt<6>(); }
        else wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0): this segment's reads done
      barrier();
      const bf16x8 (&af)[2][2] = (p < 2) ? a0 : a1;
      const bf16x8 (&bf)[2][2] = (p == 0 || p == 3) ? b0 : b1;
      constexpr int I0 = (p < 2) ? 0 : 2, J0 = (p == 0 || p == 3) ? 0 : 2;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                bf[j][kk], af[i][kk], acc[I0 + i][J0 + j], 0, 0, 0);
      barrier();
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    phase(std::integral_constant<int, 3>{});
  }
  if (g == 0) __builtin_amdgcn_s_barrier();       // balance group 1's stagger barrier

  // ---- epilogue (transposed accumulators):
  // acc[i][j][r] = C[m0 + 128 g + 64 wm + 16 i + fr][n0 + 64 wn + 16 j + 4 fq + r]
  const int wr0 = m0 + 128 * g + 64 * wm, wc0 = n0 + 64 * wn;
  if (gridDim.y > 1) {
    float* slab = ws + (long)ks * M * N;
    const int sm = g_slab_store;
    const bool vec = (N & 3) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
      float* srow = slab + (long)(row0 + row) * N;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wc0 + 16 * j + 4 * fq;
        if (col >= N) continue;
        if (EPI == EPI_SLAB16) slab_quad16(srow + col, acc[i][j], vec, N - col, ws);
        else slab_quad(srow + col, acc[i][j], sm, vec, N - col, ws);
      }
    }
    return;
  }
  const bool vec = out_vec<EPI>(C, ldc, N, bias);
  if (EPI == EPI_SILU) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr0 + 16 * i + fr;
      if (row >= Mg) continue;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int gcol = wc0 + 32 * q;
        if (gcol < N)
          store_silu_quad(C, ldc, row0 + row, (gcol >> 5) * 16 + 4 * fq, acc[i][2 * q],
                          acc[i][2 * q + 1], vec);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wr0 + 16 * i + fr;
    if (row >= Mg) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc0 + 16 * j + 4 * fq;
      if (col < N) store_quad<EPI>(C, ldc, row0 + row, col, N, acc[i][j], bias, vec);
    }
  }
}

// 16-B buffer load of `base` (a range-checked descriptor over `nbytes`: lanes past it read
// zeros) straight into LDS at the wave-uniform `lds` + 16 * lane; voff per lane, soff uniform
// CPOL: the load's cache-policy bits (0 default; 16 = sc1, device scope: the line is not
// allocated in the CU's vector L1, which an LDS-DMA stream never re-reads)
// measured on MI355X (scripts/bench_gemm8p.py, profiles/r1_gemm8p/, profiles/r2_s2/): grouped
// tile order (+6-14 % on prefill shapes), a static priority for waves 4-7 (+1.5-5 %) over
// per-cluster flips, and one counted vmcnt per K-tile instead of one per phase (VAR 512:
// +6 % on prefill shapes, +6-11 % on the decode gate/up, down and LM head); the
// deep-prefetch plan (VAR 4) and glds-before-ds_read order measured slower / equal, and so
// (within 1 %, profiles/r2_s2/gemm8p_wait/variants.log) did the template's B-before-A read
// order, an lgkmcnt(0) after the barrier and per-cluster priority flips
constexpr int GEMM8P_DEFAULT = 8 | 256 | 512;

template <int EPI, int VAR = 0>
static int launch_8p(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                     int N, int K, int splits, const void* bias, void* ws, const int* group_off,
                     int groups, hipStream_t st) {
  if (EPI == EPI_SILU && N % 64) return (int)hipErrorInvalidValue;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  int ksl = K / splits;
  ksl = (ksl / BK) * BK;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  constexpr size_t lds = 2 * (size_t)(256 + 256) * BK * 2;
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm8p_kernel<EPI, VAR>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  dim3 grid(tiles, splits, groups);
  gemm8p_kernel<EPI, VAR><<<grid, 512, lds, st>>>((const u16*)A, lda, (const u16*)W, ldw, C, ldc, M,
                                             N, K, ksl, (const u16*)bias, (float*)ws, group_off);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI>
static int launch_8p224(const void* A, int lda, const void* W, int ldw, void* C, int ldc,
                        int M, int N, int K, int splits, const void* bias, void* ws,
                        const int* group_off, int groups, hipStream_t st) {
  if (EPI == EPI_SILU && N % 32) return (int)hipErrorInvalidValue;
  const int tiles = ((M + 255) / 256) * ((N + 223) / 224);
  int ksl = K / splits;
  ksl = (ksl / BK) * BK;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  constexpr size_t lds = 2 * (size_t)(256 + 256) * BK * 2;
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm8p224_kernel<EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  dim3 grid(tiles, splits, groups);
  gemm8p224_kernel<EPI><<<grid, 512, lds, st>>>((const u16*)A, lda, (const u16*)W, ldw, C, ldc,
                                                M, N, K, ksl, (const u16*)bias, (float*)ws,
                                                group_off);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI>
static int launch_8p128(const void* A, int lda, const void* W, int ldw, void* C, int ldc,
                        int M, int N, int K, int splits, const void* bias, void* ws,
                        const int* group_off, int groups, hipStream_t st) {
  if (EPI == EPI_SILU && N % 32) return (int)hipErrorInvalidValue;
  const int tiles = ((M + 255) / 256) * ((N + 127) / 128);
  int ksl = K / splits;
  ksl = (ksl / BK) * BK;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  constexpr size_t lds = 2 * (size_t)(256 + 128) * BK * 2;
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)gemm8p128_kernel<EPI>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_done = true;
  }
  dim3 grid(tiles, splits, groups);
  gemm8p128_kernel<EPI><<<grid, 512, lds, st>>>((const u16*)A, lda, (const u16*)W, ldw, C, ldc,
                                                M, N, K, ksl, (const u16*)bias, (float*)ws,
                                                group_off);
  if (splits > 1 && C != nullptr) {
    const int outN = (EPI == EPI_SILU) ? N / 2 : N;
    const long total = (long)M * outN;
    splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
        C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI>
static int dispatch_8p(int tile_cfg, DLI_GEMM_ARGS) {
  switch (tile_cfg) {
    // 256x256 8-phase ping-pong (gemm8p_kernel)
    case 22: return launch_8p<EPI, GEMM8P_DEFAULT>(DLI_GEMM_PASS);
    // 256x224 ping-pong (gemm8p224_kernel): N = 28672 gate/up at M = 512 is 256 tiles
    case 26: return launch_8p224<EPI>(DLI_GEMM_PASS);
    // 256x128 ping-pong (gemm8p128_kernel): Mixtral grouped down (8 x 32 tiles), N = 4096 at
    // M = 512 (64 tiles x split 4)
    case 28: return launch_8p128<EPI>(DLI_GEMM_PASS);
    default: return DLI_NOT_MINE;
  }
}

int gemm_8p_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS) { DLI_EPI_SWITCH_S16(dispatch_8p) }
int gemm_8p_set_slab_store(int mode) { return set_slab_store_tu(mode); }
