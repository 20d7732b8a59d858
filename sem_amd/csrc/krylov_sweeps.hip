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

constexpr int kDotChunks = 64;   // column chunks per row (grid.x); partial sums per row
constexpr int kDotThreads = 256;

// Block (c, j): partial dot products of row j over column chunk c.
__global__ __launch_bounds__(kDotThreads) void basis_dot2_kernel(const double* __restrict__ V, int64_t ldv, int64_t n,
                                                                 const double* __restrict__ a,
                                                                 const double* __restrict__ b,
                                                                 double* __restrict__ work) {
  const int c = blockIdx.x, j = blockIdx.y, t = threadIdx.x;
  const int64_t len = (n + kDotChunks - 1) / kDotChunks;
  const int64_t lo = c * len, hi = min(n, lo + len);
  const double* row = V + j * ldv;
  // four independent accumulator pairs: four rows-loads in flight per thread
  double sa0 = 0.0, sb0 = 0.0, sa1 = 0.0, sb1 = 0.0, sa2 = 0.0, sb2 = 0.0, sa3 = 0.0, sb3 = 0.0;
  int64_t i = lo + t;
  for (; i + 3 * kDotThreads < hi; i += 4 * kDotThreads) {
    const double v0 = row[i], v1 = row[i + kDotThreads], v2 = row[i + 2 * kDotThreads], v3 = row[i + 3 * kDotThreads];
    sa0 = fma(v0, a[i], sa0);
    sb0 = fma(v0, b[i], sb0);
    sa1 = fma(v1, a[i + kDotThreads], sa1);
    sb1 = fma(v1, b[i + kDotThreads], sb1);
    sa2 = fma(v2, a[i + 2 * kDotThreads], sa2);
    sb2 = fma(v2, b[i + 2 * kDotThreads], sb2);
    sa3 = fma(v3, a[i + 3 * kDotThreads], sa3);
    sb3 = fma(v3, b[i + 3 * kDotThreads], sb3);
  }
  for (; i < hi; i += kDotThreads) {
    const double v = row[i];
    sa0 = fma(v, a[i], sa0);
    sb0 = fma(v, b[i], sb0);
  }
  double sa = (sa0 + sa1) + (sa2 + sa3), sb = (sb0 + sb1) + (sb2 + sb3);
  // wave reduction (fixed order), then the four waves in order
  for (int off = 32; off > 0; off >>= 1) {
    sa += __shfl_down(sa, off, 64);
    sb += __shfl_down(sb, off, 64);
  }
  __shared__ double ra[kDotThreads / 64], rb[kDotThreads / 64];
  if ((t & 63) == 0) {
    ra[t >> 6] = sa;
    rb[t >> 6] = sb;
  }
  __syncthreads();
  if (t == 0) {
    double xa = 0.0, xb = 0.0;
    for (int w = 0; w < kDotThreads / 64; ++w) {
      xa += ra[w];
      xb += rb[w];
    }
    work[(static_cast<int64_t>(j) * kDotChunks + c) * 2 + 0] = xa;
    work[(static_cast<int64_t>(j) * kDotChunks + c) * 2 + 1] = xb;
  }
}

__global__ void basis_dot2_finish(const double* __restrict__ work, int k, double* __restrict__ out) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;  // q = 2 j + (0: a, 1: b)
  if (q >= 2 * k) return;
  const int j = q >> 1, s = q & 1;
  double x = 0.0;
  for (int c = 0; c < kDotChunks; ++c) x += work[(static_cast<int64_t>(j) * kDotChunks + c) * 2 + s];
  out[q] = x;
}

// w[i] -= sum_j c[j] V[j][i]: one thread per column, rows streamed in order (coalesced per row);
// the coefficients are staged through LDS in blocks.
constexpr int kUpdThreads = 256, kUpdStage = 512;
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
        s0 = fma(cs[j], p[static_cast<int64_t>(j) * ldv], s0);
        s1 = fma(cs[j + 1], p[static_cast<int64_t>(j + 1) * ldv], s1);
      }
      if (j < m) s0 = fma(cs[j], p[static_cast<int64_t>(j) * ldv], s0);
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

int sem_basis_dot2_work_size(int k) { return k > 0 ? 2 * k * sem::kDotChunks : 0; }

int sem_basis_dot2(const double* V, int64_t ldv, int k, int64_t n, const double* a, const double* b, double* work,
                   double* out, void* stream) {
  if (k < 0 || n < 0 || ldv < n) return sem::set_error(SEM_EINVAL, "basis_dot2: bad shape");
  if (k == 0 || n == 0) return SEM_OK;
  if (!V || !a || !b || !work || !out) return sem::set_error(SEM_EINVAL, "basis_dot2: null argument");
  if (k > 65535) return sem::set_error(SEM_EINVAL, "basis_dot2: more than 65535 basis vectors");
  auto s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sem::basis_dot2_kernel, dim3(sem::kDotChunks, k), dim3(sem::kDotThreads), 0, s, V, ldv, n, a, b,
                     work);
  hipLaunchKernelGGL(sem::basis_dot2_finish, dim3((2 * k + 255) / 256), dim3(256), 0, s, work, k, out);
  return sem::hip_check_k(hipGetLastError(), "basis_dot2 launch");
}

int sem_basis_update(const double* V, int64_t ldv, int k, int64_t n, const double* c, double* w, void* stream) {
  if (k < 0 || n < 0 || ldv < n) return sem::set_error(SEM_EINVAL, "basis_update: bad shape");
  if (k == 0 || n == 0) return SEM_OK;
  if (!V || !c || !w) return sem::set_error(SEM_EINVAL, "basis_update: null argument");
  const int64_t blocks = (n + sem::kUpdThreads - 1) / sem::kUpdThreads;
  if (blocks > 0x7fffffffLL) return sem::set_error(SEM_EINVAL, "basis_update: vector too long");
  hipLaunchKernelGGL(sem::basis_update_kernel, dim3(static_cast<unsigned>(blocks)), dim3(sem::kUpdThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), V, ldv, k, n, c, w);
  return sem::hip_check_k(hipGetLastError(), "basis_update launch");
}

}  // extern "C"
