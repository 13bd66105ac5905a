// Weight-streaming skinny GEMM for M <= 4 rows (tile ids 29-33, 56-59) and the batch-1
// reduce-free forms (dli_gemv_fused: residual-adding epilogue, RMSNorm prologue).
#include "gemm_common.h"

// ---------------------------------------------------------------------------------------
// Skinny GEMM for M <= 4 rows (batch-1 / tiny-batch decode: SURVEY.md §7.4 "the decode
// skinny GEMM must approach the HBM roofline"): every weight byte is used M times, so the
// kernel is a weight stream, not an MFMA tile. A workgroup (4 waves) owns R = 4 * RW output
// rows of W over one K slice; in a wave, lane l covers the 8 K-elements [8 (l + 64 s),
// +8) of step s for its RW rows: RW 16-B nontemporal weight loads per step (the weights are
// read exactly once, /opt/skills/guides/MI355X_MICROARCH.md 'nt-weights'), two steps in flight, bf16 pairs
// accumulated by v_dot2c_f32_bf16 against x (M rows, L1/L2-resident). Lane partial sums
// are reduced across the wave with shuffles and staged in LDS; the epilogue then writes
// bf16 / fp32 / SiLU(gate)*up (the 16-row interleaved gate/up weight: a workgroup's 32 rows
// are 16 gate + 16 up features) or fp32 split-K slabs for the fused reduces. No MFMA, no
// LDS tiles, no padding rows: bytes moved = weights + M * K * 2 + outputs.
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

// bf16 pairs by __builtin_shufflevector: a __builtin_bit_cast of one element of a uint
// ext-vector was compiled (ROCm 7.2 clang) into the FIRST element for every lane pair
__device__ __forceinline__ float dot8_acc(const bf16x8v w, const bf16x8v x, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 0, 1),
                                        __builtin_shufflevector(x, x, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 2, 3),
                                        __builtin_shufflevector(x, x, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 4, 5),
                                        __builtin_shufflevector(x, x, 4, 5), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 6, 7),
                                        __builtin_shufflevector(x, x, 6, 7), acc, false);
  return acc;
}

struct NoPrologue {
  __device__ void issue() {}
  __device__ void complete() {}
};

// The weight stream of one workgroup: res[m][wid * RW + r] = sum over this K slice of
// A[m, :] . W[r0 + r, :] (r < RW), reduced across the wave and staged in LDS.
// PRE: the input rows are produced by `pro` (the RMSNorm prologue, into LDS): pro.issue()
// requests the residual rows and norm weight, then this lane's first UNROLL weight steps are
// requested (branch-free: clamped, the steps past the slice masked out of the sums), then
// pro.complete() waits for the ROW loads only (they
// are older than the weight loads, so the counted wait leaves the weight stream in flight),
// normalises into LDS and synchronises. The prologue's latency (rows from the Infinity
// Cache, a block reduction, LDS stores) thus runs under the first weight requests.
template <int MB, int RW, int UNROLL, bool PRE = false, class Pro = NoPrologue>
__device__ __forceinline__ void gemv_core(const u16* __restrict__ A, int lda,
                                          const u16* __restrict__ W, int ldw, int M, int N,
                                          int K, int k_split_len, int r0, int ks,
                                          float (&res)[MB][4 * RW], Pro& pro) {
  // r0: this wave's first weight row (rows r0 .. r0 + RW - 1 land in res[.][wid * RW ..])
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kb = ks * k_split_len;
  const int klen = min(k_split_len, K - kb);
  const int nchunk = klen >> 3;                     // 8-element chunks of the K slice
  const bf16x8v* wrow[RW];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int n = min(r0 + r, N - 1);
    wrow[r] = reinterpret_cast<const bf16x8v*>(W + (long)n * ldw + kb);
  }
  const bf16x8v* xrow[MB];
#pragma unroll
  for (int m = 0; m < MB; ++m)
    xrow[m] = reinterpret_cast<const bf16x8v*>(A + (long)min(m, M - 1) * lda + kb);
  float acc[MB][RW];
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int r = 0; r < RW; ++r) acc[m][r] = 0.f;
  int c = lane;
  if constexpr (PRE) {
    pro.issue();
    bf16x8v w[UNROLL][RW];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int r = 0; r < RW; ++r)
        w[u][r] = __builtin_nontemporal_load(wrow[r] + min(c + 64 * u, nchunk - 1));
    pro.complete();
#pragma unroll
    for (int m = 0; m < MB; ++m) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        // branch-free mask: a branch here made the compiler sink the x loads into it, each
        // behind a full vmcnt(0) wait (8 serial loads per iteration at UNROLL 8)
        const bool ok = c + 64 * u < nchunk;
        const bf16x8v xv = xrow[m][min(c + 64 * u, nchunk - 1)];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const float a = dot8_acc(w[u][r], xv, acc[m][r]);
          acc[m][r] = ok ? a : acc[m][r];
        }
      }
      // several rows: one row's LDS reads at a time (hoisting every row's 8 reads held
      // 128 VGPRs at MB = 4 and dropped the prologue GEMVs to 2 waves per SIMD)
      if constexpr (MB > 1) __builtin_amdgcn_sched_barrier(0);
    }
    c += 64 * UNROLL;
  }
  // UNROLL 64-chunk steps per iteration: UNROLL * RW weight loads in flight per lane (the
  // short projections of a batch-1 layer run only a few iterations, so depth, not
  // occupancy, hides the HBM latency). Full iterations address by immediate offsets from one
  // base; the last, partial one issues all its loads at once too (indices clamped, the
  // extra steps masked out of the sums by selects — a branch let the compiler sink the x
  // loads into it, each behind a vmcnt(0)): a step-at-a-time tail cost the K = 14336 down
  // projection 4 serial HBM round trips (28 steps a lane at UNROLL 8). Sums stay in step
  // order.
  for (; c + 64 * (UNROLL - 1) < nchunk; c += 64 * UNROLL) {
    bf16x8v w[UNROLL][RW];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int r = 0; r < RW; ++r) w[u][r] = __builtin_nontemporal_load(wrow[r] + c + 64 * u);
#pragma unroll
    for (int m = 0; m < MB; ++m) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const bf16x8v xv = xrow[m][c + 64 * u];
#pragma unroll
        for (int r = 0; r < RW; ++r) acc[m][r] = dot8_acc(w[u][r], xv, acc[m][r]);
      }
    }
  }
  if (c < nchunk) {
    bf16x8v w[UNROLL][RW];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int r = 0; r < RW; ++r)
        w[u][r] = __builtin_nontemporal_load(wrow[r] + min(c + 64 * u, nchunk - 1));
#pragma unroll
    for (int m = 0; m < MB; ++m) {
#pragma unroll
      for (int u = 0; u < UNROLL; ++u) {
        const bool ok = c + 64 * u < nchunk;
        const bf16x8v xv = xrow[m][min(c + 64 * u, nchunk - 1)];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const float a = dot8_acc(w[u][r], xv, acc[m][r]);
          acc[m][r] = ok ? a : acc[m][r];
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const float v = wave_sum(acc[m][r]);
      if (lane == 0) res[m][wid * RW + r] = v;
    }
}

// gemv-only epilogue: C is the residual, residual[m, n] = bf16(residual + bf16(acc)) (the
// rounding of splitk_add_rmsnorm: the GEMM result is rounded before the add). Full K per
// workgroup (splits 1): every output element has one writer and no slab round trip.
constexpr int EPI_RES = 16;

// The deferred RMSNorm of the consuming GEMV (PRO): x[m] = bf16(A[m] * rstd_m * nw) for the
// MB input rows into LDS (xs: [MB][K] bf16), one block reduction per row. issue(): every row
// vector and norm-weight vector of this thread requested (VPT 16-B vectors per row, indices
// clamped, K <= 256 * 8 * VPT); complete(): sums, scales, stores, barrier. Numerics as
// splitk_add_rmsnorm's output: (v * rstd) * w in fp32, rounded once.
template <int MB, int VPT>
struct NormPrologue {
  const u16* A;
  int lda;
  const u16* nw;
  float eps;
  int M, K;
  u16* xs;
  float* red;
  uint4 rv[MB][VPT], wv[VPT];
  __device__ __forceinline__ void issue() {
    const int nvec = K >> 3;
#pragma unroll
    for (int i = 0; i < VPT; ++i) {
      const int vi = min((int)threadIdx.x + 256 * i, nvec - 1);
#pragma unroll
      for (int m = 0; m < MB; ++m)
        rv[m][i] = *reinterpret_cast<const uint4*>(A + (long)min(m, M - 1) * lda + vi * 8);
      wv[i] = *reinterpret_cast<const uint4*>(nw + vi * 8);
    }
  }
  __device__ __forceinline__ void complete() {
    const int nvec = K >> 3;
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      float v[VPT][8];
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const uint4 q = rv[m][i];
        v[i][0] = __uint_as_float(q.x << 16); v[i][1] = __uint_as_float(q.x & 0xffff0000u);
        v[i][2] = __uint_as_float(q.y << 16); v[i][3] = __uint_as_float(q.y & 0xffff0000u);
        v[i][4] = __uint_as_float(q.z << 16); v[i][5] = __uint_as_float(q.z & 0xffff0000u);
        v[i][6] = __uint_as_float(q.w << 16); v[i][7] = __uint_as_float(q.w & 0xffff0000u);
        float s8 = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s8 += v[i][j] * v[i][j];
        ss += ((int)threadIdx.x + 256 * i < nvec) ? s8 : 0.f;
      }
      const float rstd = rsqrtf(block_sum(ss, red) / K + eps);
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int vi = (int)threadIdx.x + 256 * i;
        const uint4 q = wv[i];
        const float w8[8] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                             __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u),
                             __uint_as_float(q.z << 16), __uint_as_float(q.z & 0xffff0000u),
                             __uint_as_float(q.w << 16), __uint_as_float(q.w & 0xffff0000u)};
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = v[i][j] * rstd * w8[j];
        if (vi < nvec) store8(xs + (long)m * K + vi * 8, v[i]);
      }
      if constexpr (MB > 1) __builtin_amdgcn_sched_barrier(0);   // one row's floats live
    }
    __syncthreads();
  }
};

// H16 (SiLU*up only): R = 4 RW rows per workgroup as R/2 gate + the matching R/2 up rows of
// one 32-row gate/up block (waves 0-1 the gate rows, waves 2-3 the up rows; RW 4: 8 + 8,
// RW 1: 2 + 2 — tile 58, 4x the workgroups of tile 29), so the pairing
// runs at the 16-row grid (2x the workgroups of the 32-row tile; profiles/r4/b1/)
template <int MB, int RW, int EPI, int UNROLL, bool H16 = false, bool PRO = false, int PV = 0>
__global__ void __launch_bounds__(256) gemv_kernel(
    const u16* __restrict__ A, int lda, const u16* __restrict__ W, int ldw,
    void* __restrict__ C, int ldc, int M, int N, int K, int k_split_len,
    const u16* __restrict__ bias, float* __restrict__ ws, const u16* __restrict__ nw,
    float eps) {
  constexpr int R = 4 * RW;
  static_assert(!H16 || (EPI == EPI_SILU && RW <= 4), "H16 pairs R/2 gate + R/2 up rows");
  constexpr int HR = R / 2, PARTS = 16 / HR;          // H16: rows per half, parts per block
  __shared__ float res[MB][R];
  __shared__ float red[16];
  extern __shared__ __align__(16) u16 xs_dyn[];
  const int n_base = blockIdx.x * R;
  const int ks = blockIdx.y;
  const int wid = threadIdx.x >> 6;
  const int blk = blockIdx.x / PARTS, half = blockIdx.x % PARTS;
  // weight row of res column j
  auto row_of = [&](int j) {
    return H16 ? blk * 32 + (j < HR ? half * HR + j : 16 + half * HR + (j - HR)) : n_base + j;
  };
  if constexpr (PRO && PV > 0) {
    // several rows (launcher: MB > 1): PV row vectors per thread as a template parameter
    // (2 up to K = 4096, 4 up to 8192) — with a runtime branch the unused 4-vector form's
    // registers set the kernel's count (196 VGPRs, 2 waves per SIMD at MB = 4)
    NormPrologue<MB, PV> pro{A, lda, nw, eps, M, K, xs_dyn, red};
    gemv_core<MB, RW, UNROLL, true>(xs_dyn, K, W, ldw, M, N, K, k_split_len, row_of(wid * RW),
                                    ks, res, pro);
  } else if constexpr (PRO) {
    // one row: the runtime branch. Its allocation (124 VGPRs) streams faster than the
    // template form's (101): batch-1 p50 0.188 vs 0.194 s, same box (profiles/r5/s33)
    if (K <= 4096) {
      NormPrologue<MB, 2> pro{A, lda, nw, eps, M, K, xs_dyn, red};
      gemv_core<MB, RW, UNROLL, true>(xs_dyn, K, W, ldw, M, N, K, k_split_len,
                                      row_of(wid * RW), ks, res, pro);
    } else {
      NormPrologue<MB, 4> pro{A, lda, nw, eps, M, K, xs_dyn, red};
      gemv_core<MB, RW, UNROLL, true>(xs_dyn, K, W, ldw, M, N, K, k_split_len,
                                      row_of(wid * RW), ks, res, pro);
    }
  } else {
    NoPrologue pro;
    gemv_core<MB, RW, UNROLL>(A, lda, W, ldw, M, N, K, k_split_len, row_of(wid * RW), ks, res,
                              pro);
  }
  __syncthreads();
  if constexpr (EPI == EPI_RES) {
    for (int t = threadIdx.x; t < MB * R; t += 256) {
      const int m = t / R, j = t % R, n = n_base + j;
      if (m < M && n < N) {
        u16* p = (u16*)C + (long)m * ldc + n;
        *p = f2bf(bf2f(*p) + bf2f(f2bf(res[m][j])));
      }
    }
    return;
  }
  // epilogue: one thread per (row m, output column)
  if (ws != nullptr && gridDim.y > 1) {             // fp32 partial slab of this K slice
    for (int t = threadIdx.x; t < MB * R; t += 256) {
      const int m = t / R, j = t % R, n = row_of(j);
      if (m < M && n < N) ws[((long)ks * M + m) * N + n] = res[m][j];
    }
    return;
  }
  if (H16) {                                        // res 0..HR-1 gate, HR.. the matching up
    for (int t = threadIdx.x; t < MB * HR; t += 256) {
      const int m = t / HR, j = t % HR;
      const int f = blk * 16 + half * HR + j;
      if (m < M && blk * 32 < N)
        ((u16*)C)[(long)m * ldc + f] = f2bf(silu_f(res[m][j]) * res[m][j + HR]);
    }
    return;
  }
  if (EPI == EPI_SILU) {                            // R = 32: rows 0-15 gate, 16-31 up
    for (int t = threadIdx.x; t < MB * 16; t += 256) {
      const int m = t / 16, j = t % 16;
      const int f = (n_base >> 5) * 16 + j;
      if (m < M && n_base + j < N)
        ((u16*)C)[(long)m * ldc + f] = f2bf(silu_f(res[m][j]) * res[m][j + 16]);
    }
    return;
  }
  for (int t = threadIdx.x; t < MB * R; t += 256) {
    const int m = t / R, j = t % R, n = n_base + j;
    if (m < M && n < N) store_pair_or_one<EPI>(C, ldc, m, n, res[m][j], bias);
  }
}

// nw != null (PRO): A is the raw residual, normalised per row into LDS by the prologue
// (MB * K * 2 bytes of dynamic LDS, <= 64 KB)
template <int MB, int RW, int EPI, int UNROLL = 2, bool H16 = false, bool PRO = false>
static int launch_gemv(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M,
                       int N, int K, int splits, const void* bias, void* ws, hipStream_t st,
                       const void* nw = nullptr, float eps = 0.f) {
  constexpr int R = 4 * RW;
  if (M > MB || (EPI == EPI_SILU && ((R != 32 && !H16) || N % 32)) || K % 8 || lda % 8 ||
      ldw % 8)
    return (int)hipErrorInvalidValue;
  const size_t lds = PRO ? (size_t)MB * K * 2 : 0;
  if (PRO && (nw == nullptr || K > 8192 || lds > 65536)) return (int)hipErrorInvalidValue;
  if (EPI == EPI_RES && (splits != 1 || C == nullptr)) return (int)hipErrorInvalidValue;
  int ksl = K / splits;
  ksl = (ksl / 8) * 8;
  if (ksl * splits != K) return (int)hipErrorInvalidValue;
  dim3 grid((N + R - 1) / R, splits);
  constexpr int PV_SMALL = (PRO && MB > 1) ? 2 : 0, PV_LARGE = (PRO && MB > 1) ? 4 : 0;
  if (PRO && MB > 1 && K > 4096)
    gemv_kernel<MB, RW, EPI, UNROLL, H16, PRO, PV_LARGE><<<grid, 256, lds, st>>>(
        (const u16*)A, lda, (const u16*)W, ldw, C, ldc, M, N, K, ksl, (const u16*)bias,
        splits > 1 ? (float*)ws : nullptr, (const u16*)nw, eps);
  else
    gemv_kernel<MB, RW, EPI, UNROLL, H16, PRO, PV_SMALL><<<grid, 256, lds, st>>>(
        (const u16*)A, lda, (const u16*)W, ldw, C, ldc, M, N, K, ksl, (const u16*)bias,
        splits > 1 ? (float*)ws : nullptr, (const u16*)nw, eps);
  if constexpr (EPI != EPI_RES) {
    if (splits > 1 && C != nullptr) {
      const int outN = (EPI == EPI_SILU) ? N / 2 : N;
      const long total = (long)M * outN;
      splitk_reduce_kernel<EPI><<<(int)((total + 255) / 256), 256, 0, st>>>(
          C, ldc, (const float*)ws, M, N, splits, (const u16*)bias);
    }
  }
  DLI_RETURN_LAUNCH();
}

template <int EPI>
static int dispatch_gemv(int tile_cfg, const void* A, int lda, const void* W, int ldw, void* C,
                         int ldc, int M, int N, int K, int splits, const void* bias, void* ws,
                         hipStream_t st) {
  // 30: 16 rows per workgroup, 31: 32 rows (the SiLU gate/up pairing needs 32), 32: 16 rows
  // with 4 K-steps in flight per lane (M = 1)
  const bool r32 = tile_cfg == 31;
  if (tile_cfg == 32)
    return M <= 1 ? launch_gemv<1, 4, EPI, 4>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : (int)hipErrorInvalidValue;
  // 33: 32 rows (SiLU gate/up pairs) with 4 K-steps in flight per lane (M = 1): 32 weight
  // loads of 16 B outstanding per lane instead of 16 (tile 31)
  if (tile_cfg == 33)
    return M <= 1 ? launch_gemv<1, 8, EPI, 4>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : (int)hipErrorInvalidValue;
  // 29: SiLU*up gate/up on the 16-row grid (8 gate + 8 up rows per workgroup); 4 K-steps
  // in flight per lane at M = 1 (tile 32's depth), 2 at M = 2..4 (tile 30's)
  // 58 / 59: the pairing with 2 + 2 / 4 + 4 rows a workgroup and 8 K-steps in flight per
  // lane (tile 56 / 57's grid for the gate/up projection)
  if (tile_cfg == 58 || tile_cfg == 59) {
    if constexpr (EPI == EPI_SILU) {
      const bool r8 = tile_cfg == 59;
      if (M <= 1)
        return r8 ? launch_gemv<1, 2, EPI, 8, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : launch_gemv<1, 1, EPI, 8, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
      if (M <= 2)
        return r8 ? launch_gemv<2, 2, EPI, 4, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : launch_gemv<2, 1, EPI, 8, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
      if (M <= 4)
        return r8 ? launch_gemv<4, 2, EPI, 4, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : launch_gemv<4, 1, EPI, 8, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    }
    return (int)hipErrorInvalidValue;
  }
  if (tile_cfg == 29) {
    if constexpr (EPI == EPI_SILU) {
      if (M <= 1) return launch_gemv<1, 4, EPI, 4, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
      if (M <= 2) return launch_gemv<2, 4, EPI, 2, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
      if (M <= 4) return launch_gemv<4, 4, EPI, 2, true>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    }
    return (int)hipErrorInvalidValue;
  }
  // 56 / 57: 4 / 8 rows a workgroup with 8 K-steps in flight per lane (4x / 2x the
  // workgroups of tile 30 on one projection: full-K or lightly split skinny projections)
  if (tile_cfg == 56 || tile_cfg == 57) {
    if constexpr (EPI != EPI_SILU) {
      const bool r8 = tile_cfg == 57;
      if (M <= 1)
        return r8 ? launch_gemv<1, 2, EPI, 8>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : launch_gemv<1, 1, EPI, 8>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
      if (M <= 2)
        return r8 ? launch_gemv<2, 2, EPI, 4>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : launch_gemv<2, 1, EPI, 8>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
      if (M <= 4)
        return r8 ? launch_gemv<4, 2, EPI, 4>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
                  : launch_gemv<4, 1, EPI, 8>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    }
    return (int)hipErrorInvalidValue;
  }
  if (M <= 1)
    return r32 ? launch_gemv<1, 8, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
               : launch_gemv<1, 4, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
  if (M <= 2)
    return r32 ? launch_gemv<2, 8, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
               : launch_gemv<2, 4, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
  if (M <= 4)
    return r32 ? launch_gemv<4, 8, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st)
               : launch_gemv<4, 4, EPI>(A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
  return (int)hipErrorInvalidValue;
}

int gemm_gemv_dispatch(int epi, int tile_cfg, DLI_GEMM_ARGS) {
  if ((tile_cfg < 29 || tile_cfg > 33) && (tile_cfg < 56 || tile_cfg > 59)) return DLI_NOT_MINE;
  if (go != nullptr) return (int)hipErrorInvalidValue;     // no grouped mode
  (void)groups;
  switch (epi) {
    case EPI_BF16: return dispatch_gemv<EPI_BF16>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    case EPI_F32: return dispatch_gemv<EPI_F32>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    case EPI_SILU: return dispatch_gemv<EPI_SILU>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    case EPI_BIAS_GELU: return dispatch_gemv<EPI_BIAS_GELU>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    case EPI_BIAS: return dispatch_gemv<EPI_BIAS>(tile_cfg, A, lda, W, ldw, C, ldc, M, N, K, splits, bias, ws, st);
    default: return (int)hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------------------
// Batch-1 decode without the split-K reduce kernels (ops.linear_residual / ops.NormedRows):
//  * epi EPI_RES (16), nw null: residual[M, N] (= C) += A . W^T, full K per workgroup;
//  * nw != null: A is the raw residual [M, K]; the GEMV normalises it in its prologue
//    (x = rmsnorm(A) * nw, into LDS) and runs epi 0 (bf16 C, or fp32 slabs when C is null
//    and splits > 1: the fused QKV consumer) or 2 (SiLU*up).
// The O / down projections then write the residual directly and the next GEMV (gate/up,
// the next layer's QKV) applies the norm: two kernels fewer per layer.
// Tiles: 30 / 32 as dli_gemm (16 rows a workgroup, 2 / 4 K-steps in flight), 29 / 31 / 33
// (SiLU), and for EPI_RES 56 (4 rows a workgroup, 8 K-steps in flight: 1024 workgroups on
// a 4096-wide projection) and 57 (8 rows, 8 K-steps).
extern "C" int dli_gemv_fused(const void* A, int lda, const void* nw, float eps, const void* W,
                              int ldw, void* C, int ldc, int M, int N, int K, int epi,
                              int tile_cfg, int splits, void* ws, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  // split K needs the fp32 slabs: the output itself (C null) or the reduce's input
  if (M > 4 || splits < 1 || (splits > 1 && ws == nullptr) || (C == nullptr && splits < 2))
    return (int)hipErrorInvalidValue;
#define DLI_GF(MB, RW, E, U, H, P) \
  return launch_gemv<MB, RW, E, U, H, P>(A, lda, W, ldw, C, ldc, M, N, K, splits, nullptr, ws, st, nw, eps)
#define DLI_GF_M(RW, E, U1, U, H, P)           \
  if (M <= 1) DLI_GF(1, RW, E, U1, H, P);      \
  if (M <= 2) DLI_GF(2, RW, E, U, H, P);       \
  DLI_GF(4, RW, E, U, H, P)
  if (nw != nullptr) {
    if (epi == EPI_SILU) {
      switch (tile_cfg) {
        case 29: DLI_GF_M(4, EPI_SILU, 4, 2, true, true);
        case 31: DLI_GF_M(8, EPI_SILU, 2, 2, false, true);
        case 33: if (M <= 1) DLI_GF(1, 8, EPI_SILU, 4, false, true); break;
        case 58: DLI_GF_M(1, EPI_SILU, 8, 8, true, true);
        case 59: DLI_GF_M(2, EPI_SILU, 8, 4, true, true);
        default: break;
      }
    } else if (epi == EPI_BF16) {
      switch (tile_cfg) {
        case 30: DLI_GF_M(4, EPI_BF16, 2, 2, false, true);
        case 32: if (M <= 1) DLI_GF(1, 4, EPI_BF16, 4, false, true); break;
        case 56: DLI_GF_M(1, EPI_BF16, 8, 8, false, true);
        case 57: DLI_GF_M(2, EPI_BF16, 8, 4, false, true);
        default: break;
      }
    }
    return (int)hipErrorInvalidValue;
  }
  if (epi != EPI_RES) return (int)hipErrorInvalidValue;
  switch (tile_cfg) {
    case 30: DLI_GF_M(4, EPI_RES, 2, 2, false, false);
    case 32: if (M <= 1) DLI_GF(1, 4, EPI_RES, 4, false, false); break;
    case 56: DLI_GF_M(1, EPI_RES, 8, 8, false, false);
    case 57: DLI_GF_M(2, EPI_RES, 8, 4, false, false);
    default: break;
  }
#undef DLI_GF_M
#undef DLI_GF
  return (int)hipErrorInvalidValue;
}
