// Krylov-basis sweeps for the device GMRES (sem_amd/krylov.py).
//
// The reference's Newton updates spend most of their time in LGMRES's Arnoldi
// orthogonalisation (ConvectionDiffusion_Solver.py:146-148; SURVEY.md 8a, a13: 12.2 of 15.3 s).
// The device GMRES keeps its basis V (k rows of n doubles, row pitch ldv) in HBM and runs CGS2
// with the second pass's coefficients taken from the basis' Gram matrix, so one Arnoldi step
// needs two passes over V:
//   sem_basis_dot2    out[j] = (V_j . a, V_j . b)   -- first-pass coefficients and the Gram row
//   sem_basis_update  w -= V^T c                     -- both passes' correction at once
// Both are HBM-streaming kernels (8 k n bytes each).  dot2 reduces each row in a fixed order
// (chunk partial sums, then chunks in order), so results are bitwise reproducible.
#include <hip/hip_runtime.h>

#include <string>

#include "sem_internal.h"

namespace sem {

// sem_basis_dot2: 2-D tiles.  Block (chunk c, row group g) reads the a / b chunk of kDotCols
// columns into registers once and streams kDotRows basis rows against it, so a and b are read
// k / kDotRows times instead of k times (V itself exactly once).  Per row, every thread forms its
// partial products over its kDotPer columns; the partials go through LDS, are reduced over the
// block in a fixed order, and one value per (row, a|b, chunk) goes to `work`.  basis_dot2_finish
// then sums the chunks in order: results are bitwise reproducible.
constexpr int kDotThreads = 256, kDotPer = 8, kDotCols = kDotThreads * kDotPer, kDotRows = 16;

// Basis loads: NT = true reads V non-temporally (gfx950 `nt`); bitwise-identical results.  Alternated A/B
// (k = 1000, n = 263169; profiles/r05/basis_cpol/): dot2 427 -> 399 us with nt, update 399 -> 415 us -- so the
// default is nt for dot2 and plain loads for update; SEM_BASIS_CPOL=1: nt for both, 2: plain for both.
template <bool NT>
__device__ __forceinline__ double ldv_(const double* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

template <bool NT>
__global__ __launch_bounds__(kDotThreads) void basis_dot2_kernel(const double* __restrict__ V, int64_t ldv, int k,
                                                                 int64_t n, int nchunks, const double* __restrict__ a,
                                                                 const double* __restrict__ b,
                                                                 double* __restrict__ work) {
  __shared__ double part[2 * kDotRows][kDotThreads + 1];
  const int c = blockIdx.x, g = blockIdx.y, t = threadIdx.x;
  const int64_t lo = static_cast<int64_t>(c) * kDotCols;
  double av[kDotPer], bv[kDotPer];
#pragma unroll
  for (int q = 0; q < kDotPer; ++q) {
    const int64_t i = lo + t + q * kDotThreads;
    av[q] = i < n ? a[i] : 0.0;
    bv[q] = i < n ? b[i] : 0.0;
  }
  const int r0 = g * kDotRows, nr = min(kDotRows, k - r0);
  for (int r = 0; r < nr; ++r) {
    const double* row = V + static_cast<int64_t>(r0 + r) * ldv;
    double vv[kDotPer];
#pragma unroll
    for (int q = 0; q < kDotPer; ++q) {
      const int64_t i = lo + t + q * kDotThreads;
      vv[q] = i < n ? ldv_<NT>(row + i) : 0.0;
    }
    double pa0 = 0.0, pb0 = 0.0, pa1 = 0.0, pb1 = 0.0;
#pragma unroll
    for (int q = 0; q < kDotPer; q += 2) {
      pa0 = fma(vv[q], av[q], pa0);
      pb0 = fma(vv[q], bv[q], pb0);
      pa1 = fma(vv[q + 1], av[q + 1], pa1);
      pb1 = fma(vv[q + 1], bv[q + 1], pb1);
    }
    part[2 * r][t] = pa0 + pa1;
    part[2 * r + 1][t] = pb0 + pb1;
  }
  __syncthreads();
  // 2 nr sums over 256 partials: 8 threads per value, 32 partials each, then 3 shuffle steps (fixed order)
  const int v = t >> 3, s = t & 7;
  double x = 0.0;
  if (v < 2 * nr) {
#pragma unroll 8
    for (int q = 0; q < kDotThreads / 8; ++q) x += part[v][s * (kDotThreads / 8) + q];
  }
  x += __shfl_down(x, 4, 8);
  x += __shfl_down(x, 2, 8);
  x += __shfl_down(x, 1, 8);
  if (s == 0 && v < 2 * nr) {
    const int j = r0 + (v >> 1);
    work[(static_cast<int64_t>(j) * nchunks + c) * 2 + (v & 1)] = x;
  }
}

__global__ void basis_dot2_finish(const double* __restrict__ work, int k, int nchunks, double* __restrict__ out) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;  // q = 2 j + (0: a, 1: b)
  if (q >= 2 * k) return;
  const int j = q >> 1, s = q & 1;
  double x = 0.0;
  for (int c = 0; c < nchunks; ++c) x += work[(static_cast<int64_t>(j) * nchunks + c) * 2 + s];
  out[q] = x;
}

// w[i] -= sum_j c[j] V[j][i]: one thread per column, rows streamed in order (coalesced per row);
// the coefficients are staged through LDS in blocks.
constexpr int kUpdThreads = 256, kUpdStage = 512;
template <bool NT>
__global__ __launch_bounds__(kUpdThreads) void basis_update_kernel(const double* __restrict__ V, int64_t ldv, int k,
                                                                   int64_t n, const double* __restrict__ c,
                                                                   double* __restrict__ w) {
  __shared__ double cs[kUpdStage];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kUpdThreads + threadIdx.x;
  double s0 = 0.0, s1 = 0.0;
  for (int j0 = 0; j0 < k; j0 += kUpdStage) {
    const int m = min(kUpdStage, k - j0);
    __syncthreads();
    for (int q = threadIdx.x; q < m; q += kUpdThreads) cs[q] = c[j0 + q];
    __syncthreads();
    if (i < n) {
      const double* p = V + static_cast<int64_t>(j0) * ldv + i;
      int j = 0;
      for (; j + 1 < m; j += 2) {  // two independent chains for load-level parallelism
        s0 = fma(cs[j], ldv_<NT>(p + static_cast<int64_t>(j) * ldv), s0);
        s1 = fma(cs[j + 1], ldv_<NT>(p + static_cast<int64_t>(j + 1) * ldv), s1);
      }
      if (j < m) s0 = fma(cs[j], ldv_<NT>(p + static_cast<int64_t>(j) * ldv), s0);
    }
  }
  if (i < n) w[i] = w[i] - (s0 + s1);
}

static int hip_check_k(hipError_t e, const char* what) {
  if (e == hipSuccess) return SEM_OK;
  return set_error(SEM_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace sem

extern "C" {

// `work` holds one partial per (row, a|b, column chunk of kDotCols).
static int dot2_chunks(int64_t n) { return static_cast<int>((n + sem::kDotCols - 1) / sem::kDotCols); }

int64_t sem_basis_dot2_work_size(int k, int64_t n) { return k > 0 && n > 0 ? 2 * int64_t(k) * dot2_chunks(n) : 0; }

int sem_basis_dot2(const double* V, int64_t ldv, int k, int64_t n, const double* a, const double* b, double* work,
                   double* out, void* stream) {
  if (k < 0 || n < 0 || ldv < n) return sem::set_error(SEM_EINVAL, "basis_dot2: bad shape");
  if (k == 0 || n == 0) return SEM_OK;
  if (!V || !a || !b || !work || !out) return sem::set_error(SEM_EINVAL, "basis_dot2: null argument");
  if (n > (int64_t(1) << 27)) return sem::set_error(SEM_EINVAL, "basis_dot2: rows longer than 2^27");
  const int groups = (k + sem::kDotRows - 1) / sem::kDotRows;
  if (groups > 65535) return sem::set_error(SEM_EINVAL, "basis_dot2: too many basis vectors");
  auto s = reinterpret_cast<hipStream_t>(stream);
  const int nch = dot2_chunks(n);
  // non-temporal basis loads in the dot pass (round 5 A/B, profiles/r05/basis_cpol/: -6.5 %)
  hipLaunchKernelGGL(sem::basis_dot2_kernel<true>, dim3(nch, groups), dim3(sem::kDotThreads), 0, s, V, ldv, k, n, nch,
                     a, b, work);
  hipLaunchKernelGGL(sem::basis_dot2_finish, dim3((2 * k + 255) / 256), dim3(256), 0, s, work, k, nch, out);
  return sem::hip_check_k(hipGetLastError(), "basis_dot2 launch");
}

int sem_basis_update(const double* V, int64_t ldv, int k, int64_t n, const double* c, double* w, void* stream) {
  if (k < 0 || n < 0 || ldv < n) return sem::set_error(SEM_EINVAL, "basis_update: bad shape");
  if (k == 0 || n == 0) return SEM_OK;
  if (!V || !c || !w) return sem::set_error(SEM_EINVAL, "basis_update: null argument");
  const int64_t blocks = (n + sem::kUpdThreads - 1) / sem::kUpdThreads;
  if (blocks > 0x7fffffffLL) return sem::set_error(SEM_EINVAL, "basis_update: vector too long");
  auto s = reinterpret_cast<hipStream_t>(stream);
  // plain loads in the update pass (non-temporal measured slower there, round 5)
  hipLaunchKernelGGL(sem::basis_update_kernel<false>, dim3(static_cast<unsigned>(blocks)), dim3(sem::kUpdThreads), 0, s,
                     V, ldv, k, n, c, w);
  return sem::hip_check_k(hipGetLastError(), "basis_update launch");
}

}  // extern "C"
