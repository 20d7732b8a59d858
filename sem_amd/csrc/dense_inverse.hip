// Inverse of one small dense block (n <= 64) in one workgroup: the leaves of the GEMM-recursive inverse
// of the interface sweep's pivot blocks (sem_amd/linalg.py block_inverse; the sweep replaces the
// reference's SuperLU factorisation of the velocity Jacobian, NavierStokes_Solver.py:176-236).
//
// rocSOLVER inverts such a block in ~20 launches (getf2 panel, permutations, trtri, trsm) and spends
// ~130 us on a 64^2 leaf (tools/pivot_probe.py --profile, profiles/r03/cfg5/); here the whole
// Gauss-Jordan elimination runs in one launch with the block in registers: step k finds the pivot row
// p (largest |a[r][k]| among the rows not yet pivoted; partial pivoting, no row exchange), scales row p
// and eliminates column k from every other row (in-place Gauss-Jordan: column k becomes the
// inverse's).  One barrier per step (layout below).
// With pivot row p_k at step k the result R (rows left in place) satisfies A^-1[k][p_j] = R[p_k][j];
// the store applies that permutation.  A zero pivot gives non-finite entries (the caller's A X - I check
// catches them); padding rows / columns (r, c >= n) are the identity and never pivot.
#include <hip/hip_runtime.h>

#include <string>

#include "sem_internal.h"

namespace sem {

// Wave-wide maximum of a 32-bit unsigned key, result in every lane (DPP row shifts within the 16-lane
// rows, then row broadcasts 15 / 31; a disabled source yields 0, the identity of the maximum).
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
  v = max(v, static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xf, 0xf, false)));
  v = max(v, static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xf, 0xf, false)));
  v = max(v, static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xf, 0xf, false)));
  v = max(v, static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xf, 0xf, false)));
  v = max(v, static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false)));
  v = max(v, static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false)));
  return static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(v), 63));
}

// n <= 64, 256 threads.  Lane l of wave w holds column c = 16 w + (l & 15), rows 16 (l >> 4) .. + 15:
// all 64 rows of a column sit in one wave, so the pivot row's entry of every column is one lane
// permute away and a step needs a single barrier (for the broadcast of column k to all four waves).
// The pivot search runs in every wave on the same LDS copy of column k: one key per row (the high word
// of |a[r][k]| with its low 6 bits replaced by 63 - r, rows already pivoted 0) and one DPP maximum -- the
// largest magnitude to 14 mantissa bits, the lowest row among equals.
__global__ __launch_bounds__(256) void gj_inverse_kernel(const double* __restrict__ A, int64_t lda,
                                                         double* __restrict__ X, int64_t ldx, int n) {
  constexpr int R = 16;
  __shared__ double colk[2][64];
  __shared__ int prow[64], pstep[64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c = w * 16 + (lane & 15), r0 = (lane >> 4) * R;
  double a[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int r = r0 + j;
    a[j] = (r < n && c < n) ? A[r * lda + c] : (r == c ? 1.0 : 0.0);
  }
  if (c == 0) {
#pragma unroll
    for (int j = 0; j < R; ++j) colk[0][r0 + j] = a[j];
  }
  bool used = lane >= n;  // lane l tracks row l in the pivot search
  for (int k = 0; k < n; ++k) {
    const int b = k & 1;
    __syncthreads();
    const double x = colk[b][lane];
    // key from the double's own high word (exponent + 20 mantissa bits): monotone in |x| over the whole
    // double range, subnormals included (a float conversion collapsed everything below ~1e-38)
    const unsigned hi = static_cast<unsigned>(static_cast<unsigned long long>(__double_as_longlong(fabs(x))) >> 32);
    const unsigned kx = max(hi & ~63u, 64u) | static_cast<unsigned>(63 - lane);
    const unsigned key = used ? 0u : kx;
    const int p = 63 - static_cast<int>(wave_max_u32(key) & 63u);
    if (lane == p) used = true;
    const double ipiv = 1.0 / colk[b][p];
    // entry (p, c): held by the lane of the same column in row group p / 16, register p % 16
    const int pl = p & 15;
    double sel = a[0];
#pragma unroll
    for (int j = 1; j < R; ++j) sel = pl == j ? a[j] : sel;
    const double prv = __shfl(sel, ((p >> 4) << 4) | (lane & 15), 64);
    const double rv = (c == k ? 1.0 : prv) * ipiv;
    // multipliers of this thread's rows: all loads issued before any use (one LDS round trip, and no
    // branch around a load -- a predicated load per row costs a round trip each)
    double f[R];
#pragma unroll
    for (int j = 0; j < R; ++j) f[j] = colk[b][r0 + j];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const double upd = fma(-f[j], rv, c == k ? 0.0 : a[j]);
      a[j] = r0 + j == p ? rv : upd;
    }
    if (t == 0) prow[k] = p;
    if (c == k + 1) {  // publish the next column (after this step's update) for the next search
#pragma unroll
      for (int j = 0; j < R; ++j) colk[b ^ 1][r0 + j] = a[j];
    }
  }
  __syncthreads();
  if (t < n) pstep[prow[t]] = t;  // step at which row prow[t] pivoted
  __syncthreads();
  if (c < n) {
    const int col = prow[c];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int r = r0 + j;
      if (r < n) X[pstep[r] * ldx + col] = a[j];
    }
  }
}

}  // namespace sem

extern "C" {

int sem_dense_inverse_small(const double* A, int64_t lda, double* X, int64_t ldx, int n, void* stream) {
  if (n < 1 || n > 64) return sem::set_error(SEM_EINVAL, "dense_inverse_small: n must be 1..64");
  if (!A || !X) return sem::set_error(SEM_EINVAL, "dense_inverse_small: null argument");
  if (lda < n || ldx < n) return sem::set_error(SEM_EINVAL, "dense_inverse_small: leading dimension below n");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sem::gj_inverse_kernel, dim3(1), dim3(256), 0, s, A, lda, X, ldx, n);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sem::set_error(SEM_EHIP, std::string("dense_inverse_small launch: ") + hipGetErrorString(e));
  return SEM_OK;
}

}  // extern "C"
