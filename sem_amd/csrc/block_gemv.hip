// Batched block GEMV with gathered operands: the level step of the interface sweep of the
// Navier-Stokes velocity solve (block cyclic reduction, sem_amd/solvers/velocity_solve.py), which
// replaces the reference's SuperLU triangular solves (NavierStokes_Solver.py:189-203).
//
//   y[yrow[b]] (+)= sum_{s < S} M[b][:, s m : (s+1) m] . src_s[xrow[s][b]]      b = 0 .. nb-1
//
// M is (nb, m, S m) row-major: one dense m x S m operator per output row block (a level's
// [alpha | gamma] or [B^-1 | -B^-1 A | -B^-1 C]).  The kernel is HBM-bound on M (8 S m^2 bytes per
// block, each read once): every workgroup stages the S gathered operand rows of its block in LDS
// and its four waves stream kRows matrix rows each, 64 lanes over a row (512 B per wave load), four
// rows in flight per wave, then reduce across the wave with DPP/shuffles.  The grid is
// (ceil(m / 16), nb) workgroups; blocks of one output never overlap, and the operands it gathers
// are rows the launch does not write (the caller's level structure guarantees it).
#include <hip/hip_runtime.h>

#include <string>

#include "sem_internal.h"

namespace sem {

constexpr int kGemvWaves = 4;
constexpr int kGemvRowsPerWave = 4;
constexpr int kGemvRows = kGemvWaves * kGemvRowsPerWave;  // matrix rows per workgroup (wide form)
constexpr int kGemvUnroll = 8;                            // loads in flight per wave (narrow form)

struct GemvArgs {
  const double* M;
  const double* src[3];
  const int64_t* xrow;  // (S, nb); -1: no operand (its block is skipped)
  const int64_t* yrow;  // (nb)
  double* y;
  int64_t ld_src[3], ld_y;
  int nb, m, S, accumulate;
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void stage_operands(const GemvArgs& a, double* xs, int b) {
  const int m = a.m;
  for (int s = 0; s < a.S; ++s) {
    const int64_t r = a.xrow[static_cast<int64_t>(s) * a.nb + b];
    const double* src = r >= 0 ? a.src[s] + r * a.ld_src[s] : nullptr;
    for (int j = threadIdx.x; j < m; j += blockDim.x) xs[s * m + j] = src ? src[j] : 0.0;
  }
  __syncthreads();
}

// Wide form (many blocks per level): 16 rows per workgroup, four rows in flight per wave.
__global__ __launch_bounds__(64 * kGemvWaves) void block_gemv_kernel(const GemvArgs a) {
  extern __shared__ double xs[];  // S * m gathered operand values (0 for a skipped operand)
  const int b = blockIdx.y, m = a.m, K = a.S * m;
  stage_operands(a, xs, b);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = blockIdx.x * kGemvRows + wave * kGemvRowsPerWave;
  if (r0 >= m) return;
  const double* Mb = a.M + static_cast<int64_t>(b) * m * K;
  double acc[kGemvRowsPerWave];
  const double* row[kGemvRowsPerWave];
#pragma unroll
  for (int i = 0; i < kGemvRowsPerWave; ++i) {
    acc[i] = 0.0;
    row[i] = Mb + static_cast<int64_t>(min(r0 + i, m - 1)) * K;  // clamped rows are computed, not stored
  }
  for (int j = lane; j < K; j += 64) {
    const double xv = xs[j];
#pragma unroll
    for (int i = 0; i < kGemvRowsPerWave; ++i) acc[i] = fma(row[i][j], xv, acc[i]);
  }
  double* yb = a.y + a.yrow[b] * a.ld_y;
#pragma unroll
  for (int i = 0; i < kGemvRowsPerWave; ++i) {
    const double v = wave_sum(acc[i]);
    if (lane == 0 && r0 + i < m) yb[r0 + i] = a.accumulate ? yb[r0 + i] + v : v;
  }
}

// Narrow form (the last cyclic-reduction levels, one to a few blocks): one row per wave, four rows
// per workgroup, so a level's few blocks still spread over ~4x more CUs, and eight independent
// loads in flight per wave along the row.
__global__ __launch_bounds__(64 * kGemvWaves) void block_gemv_narrow_kernel(const GemvArgs a) {
  extern __shared__ double xs[];
  const int b = blockIdx.y, m = a.m, K = a.S * m;
  stage_operands(a, xs, b);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.x * kGemvWaves + wave;
  if (r >= m) return;
  const double* row = a.M + (static_cast<int64_t>(b) * m + r) * K;
  double acc[kGemvUnroll];
#pragma unroll
  for (int u = 0; u < kGemvUnroll; ++u) acc[u] = 0.0;
  int j = lane;
  for (; j + 64 * (kGemvUnroll - 1) < K; j += 64 * kGemvUnroll) {
#pragma unroll
    for (int u = 0; u < kGemvUnroll; ++u) acc[u] = fma(row[j + 64 * u], xs[j + 64 * u], acc[u]);
  }
  for (int u = 0; j < K; j += 64, ++u) acc[u] = fma(row[j], xs[j], acc[u]);
  double v = 0.0;
#pragma unroll
  for (int u = 0; u < kGemvUnroll; ++u) v += acc[u];
  v = wave_sum(v);
  if (lane == 0) {
    double* yb = a.y + a.yrow[b] * a.ld_y;
    yb[r] = a.accumulate ? yb[r] + v : v;
  }
}

// ---- Streaming row-major GEMV (round 4): y = alpha A x + beta y, A (M x K) row-major, one operator read
// once per call -- the block-Thomas interface sweep of the cfg5 velocity solve (one m x 2m forward operator
// [D^-1 | -D^-1 S_lo] and one m x m back operator per interface line, 29 GB per solve).  rocBLAS's gemvt
// streamed them at 3.6 TB/s there (8.1 ms of a 12.4 ms solve, profiles/r04/cfg5_vsolve/); its 5.7 TB/s in
// tools/gemv_probe.py came from repeating one 151 MB operator out of the 256 MB MALL.
// Workgroup = kRowsWG rows x 4 waves; wave w takes the K-quarter w of all of them, so one 16-byte x load
// (two doubles per lane) feeds kRowsWG 16-byte row loads, and kSweepUnroll iterations of those loads are
// issued before their FMAs (~20 KB in flight per wave).  Lane partials -> wave sum -> the four waves' sums
// in LDS in wave order: deterministic.  VEC = false: an unaligned operand, 8-byte loads.
constexpr int kRowsWG = 4;
constexpr int kSweepUnroll = 4;

struct RowGemvArgs {
  const double* A;
  const double* x;
  double* y;
  int64_t lda;
  double alpha, beta;
  int M, K;
};

// One launch, up to two independent GEMVs of M rows each (the twisted sweep's two chains, round 4): blocks
// [0, nb0) compute p[0], the rest p[1].  A single GEMV has nb0 = the grid size.
struct RowGemv2Args {
  RowGemvArgs p[2];
  int nb0;
};

// A's rows are read once per call: NT = true (the default; SEM_GEMV_CPOL=2 for plain loads) loads them
// non-temporally (gfx950 `nt`), so they do not evict x (read by every workgroup) from L2.  Results are bitwise
// identical; alternated A/B at cfg5 (profiles/r05/gemv_cpol/): the velocity solve 8.045 -> 8.018 ms, the strip
// solve's reduced-rows GEMV 5.6 -> 5.75 TB/s, its back-substitution GEMV 6.0 -> 6.25 TB/s.
using dvec2 = double __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ double2 load_a2(const double* p) {
  if constexpr (NT) {
    const dvec2 v = __builtin_nontemporal_load(reinterpret_cast<const dvec2*>(p));
    return make_double2(v.x, v.y);
  } else {
    return *reinterpret_cast<const double2*>(p);
  }
}

// R rows per workgroup, U iterations of loads in flight: neither changes the order in which a row's products are
// summed (each lane walks its columns in increasing order; the four waves' sums meet in wave order), so every
// (R, U) gives bitwise-identical results (SEM_GEMV_SHAPE selects one for A/B runs).
template <bool VEC, bool NT = false, int R = kRowsWG, int U = kSweepUnroll>
__global__ __launch_bounds__(256) void row_gemv_kernel(const RowGemv2Args g) {
  constexpr int kRowsWG = R, kSweepUnroll = U;
  __shared__ double part[4][kRowsWG];
  const bool second = static_cast<int>(blockIdx.x) >= g.nb0;
  const RowGemvArgs a = second ? g.p[1] : g.p[0];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = (static_cast<int>(blockIdx.x) - (second ? g.nb0 : 0)) * kRowsWG;
  // the wave's K range, in units of 2 doubles (VEC) or 1
  constexpr int W = VEC ? 2 : 1;
  const int KU = (a.K + W - 1) / W;
  const int kb = static_cast<int>(static_cast<int64_t>(KU) * wave / 4), ke = static_cast<int>(static_cast<int64_t>(KU) * (wave + 1) / 4);
  const double* rows[kRowsWG];
#pragma unroll
  for (int i = 0; i < kRowsWG; ++i) rows[i] = a.A + static_cast<int64_t>(min(r0 + i, a.M - 1)) * a.lda;  // clamped rows: not stored
  double acc[kRowsWG][2] = {};
  int u = kb + lane;
  if constexpr (VEC) {  // K even: every pair holds two columns
    // main loop: kSweepUnroll pairs per lane per iteration, every load issued before the FMAs
    for (; u + 64 * (kSweepUnroll - 1) < ke; u += 64 * kSweepUnroll) {
      double2 xv[kSweepUnroll], av[kSweepUnroll][kRowsWG];
#pragma unroll
      for (int t = 0; t < kSweepUnroll; ++t) {
        xv[t] = *reinterpret_cast<const double2*>(a.x + 2 * (u + 64 * t));
#pragma unroll
        for (int i = 0; i < kRowsWG; ++i) av[t][i] = load_a2<NT>(rows[i] + 2 * (u + 64 * t));
      }
#pragma unroll
      for (int t = 0; t < kSweepUnroll; ++t)
#pragma unroll
        for (int i = 0; i < kRowsWG; ++i) {
          acc[i][0] = fma(av[t][i].x, xv[t].x, acc[i][0]);
          acc[i][1] = fma(av[t][i].y, xv[t].y, acc[i][1]);
        }
    }
    for (; u < ke; u += 64) {
      const double2 xv = *reinterpret_cast<const double2*>(a.x + 2 * u);
#pragma unroll
      for (int i = 0; i < kRowsWG; ++i) {
        const double2 av = load_a2<NT>(rows[i] + 2 * u);
        acc[i][0] = fma(av.x, xv.x, acc[i][0]);
        acc[i][1] = fma(av.y, xv.y, acc[i][1]);
      }
    }
  } else {
    for (; u + 64 * (kSweepUnroll - 1) < ke; u += 64 * kSweepUnroll) {
      double xv[kSweepUnroll], av[kSweepUnroll][kRowsWG];
#pragma unroll
      for (int t = 0; t < kSweepUnroll; ++t) {
        xv[t] = a.x[u + 64 * t];
#pragma unroll
        for (int i = 0; i < kRowsWG; ++i) av[t][i] = rows[i][u + 64 * t];
      }
#pragma unroll
      for (int t = 0; t < kSweepUnroll; ++t)
#pragma unroll
        for (int i = 0; i < kRowsWG; ++i) acc[i][t & 1] = fma(av[t][i], xv[t], acc[i][t & 1]);
    }
    for (; u < ke; u += 64) {
      const double xv = a.x[u];
#pragma unroll
      for (int i = 0; i < kRowsWG; ++i) acc[i][0] = fma(rows[i][u], xv, acc[i][0]);
    }
  }
#pragma unroll
  for (int i = 0; i < kRowsWG; ++i) {
    const double v = wave_sum(acc[i][0] + acc[i][1]);
    if (lane == 0) part[wave][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < kRowsWG && r0 + static_cast<int>(threadIdx.x) < a.M) {
    const int i = threadIdx.x;
    const double v = a.alpha * (((part[0][i] + part[1][i]) + part[2][i]) + part[3][i]);
    double* yp = a.y + r0 + i;
    *yp = a.beta == 0.0 ? v : fma(a.beta, *yp, v);
  }
}

// 16-byte loads need 16-byte aligned A rows and x, and an even K
static bool row_vec(const RowGemvArgs& a) {
  return (reinterpret_cast<uintptr_t>(a.A) % 16) == 0 && (reinterpret_cast<uintptr_t>(a.x) % 16) == 0 &&
         (a.lda % 2) == 0 && (a.K % 2) == 0;
}

template <int R, int U>
static void launch_row_gemv_ru(RowGemv2Args& g, int M, int parts, hipStream_t s) {
  const int nb = (M + R - 1) / R;
  g.nb0 = nb;
  // non-temporal operator loads (round 5 A/B, profiles/r05/gemv_cpol/: the plain-load variant was retired in round 6)
  hipLaunchKernelGGL((row_gemv_kernel<true, true, R, U>), dim3(parts * nb), dim3(256), 0, s, g);
}

// parts = 1 (sem_gemv_rows) or 2 (sem_gemv_rows2: blocks [0, nb) the first GEMV, the rest the second)
static void launch_row_gemv(RowGemv2Args& g, int M, int parts, bool vec, hipStream_t s) {
  if (!vec) {
    const int nb = (M + kRowsWG - 1) / kRowsWG;
    g.nb0 = nb;
    hipLaunchKernelGGL((row_gemv_kernel<false>), dim3(parts * nb), dim3(256), 0, s, g);
    return;
  }
  // 2 rows per workgroup x 8 loads in flight (alternated A/B over eight shapes, profiles/r05/gemv_shape/: cfg5 velocity
  // solve 7.90 -> 7.82 ms against round 4's 4 x 4; the other shapes were retired in round 6)
  launch_row_gemv_ru<2, 8>(g, M, parts, s);
}

}  // namespace sem

extern "C" {

int sem_gemv_rows(int M, int K, double alpha, const double* A, int64_t lda, const double* x, double beta, double* y,
                  void* stream) {
  if (M < 0 || K < 0 || lda < K) return sem::set_error(SEM_EINVAL, "gemv_rows: bad sizes");
  if (M == 0) return SEM_OK;
  if (!A || !x || !y) return sem::set_error(SEM_EINVAL, "gemv_rows: null argument");
  sem::RowGemv2Args g{{sem::RowGemvArgs{A, x, y, lda, alpha, beta, M, K}, sem::RowGemvArgs{}}, 0};
  sem::launch_row_gemv(g, M, 1, sem::row_vec(g.p[0]), reinterpret_cast<hipStream_t>(stream));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sem::set_error(SEM_EHIP, std::string("gemv_rows launch: ") + hipGetErrorString(e));
  return SEM_OK;
}

int sem_gemv_rows2(int M, double alpha, double beta, int K0, const double* A0, int64_t lda0, const double* x0,
                   double* y0, int K1, const double* A1, int64_t lda1, const double* x1, double* y1, void* stream) {
  if (M < 0 || K0 < 0 || K1 < 0 || lda0 < K0 || lda1 < K1) return sem::set_error(SEM_EINVAL, "gemv_rows2: bad sizes");
  if (M == 0) return SEM_OK;
  if (!A0 || !x0 || !y0 || !A1 || !x1 || !y1) return sem::set_error(SEM_EINVAL, "gemv_rows2: null argument");
  sem::RowGemv2Args g{{sem::RowGemvArgs{A0, x0, y0, lda0, alpha, beta, M, K0},
                       sem::RowGemvArgs{A1, x1, y1, lda1, alpha, beta, M, K1}}, 0};
  sem::launch_row_gemv(g, M, 2, sem::row_vec(g.p[0]) && sem::row_vec(g.p[1]), reinterpret_cast<hipStream_t>(stream));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sem::set_error(SEM_EHIP, std::string("gemv_rows2 launch: ") + hipGetErrorString(e));
  return SEM_OK;
}

int sem_block_gemv(int nb, int m, int S, const double* M, const double* const* src, const int64_t* ld_src,
                   const int64_t* xrow, double* y, int64_t ld_y, const int64_t* yrow, int accumulate, void* stream) {
  if (nb < 0 || m < 1 || S < 1 || S > 3) return sem::set_error(SEM_EINVAL, "block_gemv: bad sizes");
  if (!M || !src || !ld_src || !xrow || !y || !yrow) return sem::set_error(SEM_EINVAL, "block_gemv: null argument");
  const size_t lds = static_cast<size_t>(S) * m * sizeof(double);
  if (lds > 64 * 1024) return sem::set_error(SEM_EUNSUPPORTED, "block_gemv: S m above 8192 doubles");
  if (nb == 0) return SEM_OK;
  sem::GemvArgs a{};
  a.M = M;
  for (int s = 0; s < S; ++s) {
    if (!src[s]) return sem::set_error(SEM_EINVAL, "block_gemv: null operand");
    a.src[s] = src[s];
    a.ld_src[s] = ld_src[s];
  }
  a.xrow = xrow;
  a.yrow = yrow;
  a.y = y;
  a.ld_y = ld_y;
  a.nb = nb;
  a.m = m;
  a.S = S;
  a.accumulate = accumulate;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int wide_blocks = (m + sem::kGemvRows - 1) / sem::kGemvRows;
  if (static_cast<int64_t>(wide_blocks) * nb >= 1024) {
    hipLaunchKernelGGL(sem::block_gemv_kernel, dim3(wide_blocks, nb), dim3(64 * sem::kGemvWaves), lds, s, a);
  } else {  // a level too small to fill the chip with 16-row workgroups
    hipLaunchKernelGGL(sem::block_gemv_narrow_kernel, dim3((m + sem::kGemvWaves - 1) / sem::kGemvWaves, nb),
                       dim3(64 * sem::kGemvWaves), lds, s, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sem::set_error(SEM_EHIP, std::string("block_gemv launch: ") + hipGetErrorString(e));
  return SEM_OK;
}

}  // extern "C"
