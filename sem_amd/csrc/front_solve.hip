// Nested-dissection solve of the Navier-Stokes velocity Jacobian (ABI 14; sem_amd/solvers/nested_dissection.py):
// the streaming steps that replace the reference's SuperLU triangular solves (NavierStokes_Solver.py:189-203).
//
// sem_front_gemv: one level of fronts (or the element leaves) in ONE launch.  Front f holds a dense row-major
// operator A_f (R_f x K_f, leading dimension ld_f): forward [S^-1; A_BS S^-1] (or [Xi; A_bi Xi] at a leaf),
// back V = S^-1 A_SB (or Xi A_ib).  A workgroup takes `rows` rows of one front (its tile), gathers the front's
// K operand values W[xidx[.]] into LDS once (-1: a zero operand), streams its rows with non-temporal 16-byte loads
// (each operator is read once per solve), `lanes` lanes per row, and reduces each row across its lanes in a fixed
// order:
//   forward: stage[yoff_f + r] = (A_f x)_r
//   back:    W[yidx[yoff_f + r]] -= (A_f x)_r       (the rows' targets are not operands of the same launch)
// sem_front_sparse_rows: a leaf's boundary update A_bi y_i from its sparse coupling rows (nnz = P - 1 per row).
// sem_front_scatter: the forward step's deterministic write-back -- copy targets W[t] = stage[s] (a front's own
// separator / a leaf's interior) and accumulation targets W[t] -= stage[s_0] .. stage[s_3] (the <= 4 fronts of a
// level that update a node of an ancestor separator), summed in the order the host sorted them.
// sem_leaf_forward (ABI 15): the split element leaves' forward step -- y_i = A_ii^-1 b_i from A_uu^-1 and
// S_v^-1 (the components couple through diagonal Newton terms only), straight into W, and A_bi y_i to the stage.
#include <hip/hip_runtime.h>

#include <string>

#include "sem_internal.h"

namespace sem {

using dvec2f = double __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double2 load_nt2(const double* p) {
  const dvec2f v = __builtin_nontemporal_load(reinterpret_cast<const dvec2f*>(p));
  return make_double2(v.x, v.y);
}

// LPR lanes per row: a wave holds 64 / LPR row groups, each group RW rows in flight, each lane U column pairs per
// row per iteration (short rows -- the deep fronts' |S| = 22, the leaves' |b| = 96 -- would leave most of a
// 64-lane row idle).  Rows per workgroup: 4 (64 / LPR) RW.
template <int LPR, int RW, int U>
__global__ __launch_bounds__(256) void front_gemv_kernel(const sem_front_launch a) {
  constexpr int G = 64 / LPR;
  extern __shared__ double xs[];
  const int f = a.tiles[2 * blockIdx.x], r0 = a.tiles[2 * blockIdx.x + 1];
  const int R = a.dims[4 * f], K = a.dims[4 * f + 1], ld = a.dims[4 * f + 2];
  const int32_t* xi = a.xidx + a.xoff[f];
  for (int k = threadIdx.x; k < K; k += 256) {
    const int p = xi[k];
    xs[k] = p >= 0 ? a.W[p] : 0.0;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (r0 + wave * G * RW >= R) return;  // the whole wave beyond the front (groups inside a wave stay together)
  const int g = lane / LPR, sl = lane % LPR;
  const int rb = r0 + (wave * G + g) * RW;
  const double* A = reinterpret_cast<const double*>(a.op[f]);
  const double* rows[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) rows[i] = A + static_cast<int64_t>(min(rb + i, R - 1)) * ld;  // clamped: not stored
  double acc[RW][2];
#pragma unroll
  for (int i = 0; i < RW; ++i) acc[i][0] = acc[i][1] = 0.0;
  const int KP = K >> 1;  // K is even (the host checks): column pairs
  const double2* x2 = reinterpret_cast<const double2*>(xs);
  int u = sl;
  for (; u + LPR * (U - 1) < KP; u += LPR * U) {
    double2 av[U][RW], xv[U];
#pragma unroll
    for (int t = 0; t < U; ++t) {
      xv[t] = x2[u + LPR * t];
#pragma unroll
      for (int i = 0; i < RW; ++i) av[t][i] = load_nt2(rows[i] + 2 * (u + LPR * t));
    }
#pragma unroll
    for (int t = 0; t < U; ++t)
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        acc[i][0] = fma(av[t][i].x, xv[t].x, acc[i][0]);
        acc[i][1] = fma(av[t][i].y, xv[t].y, acc[i][1]);
      }
  }
  if (u < KP) {  // the last < U column pairs of this lane: one masked batch (the same sums, in the same order)
    double2 av[U][RW], xv[U];
#pragma unroll
    for (int t = 0; t < U; ++t) {
      const bool in = u + LPR * t < KP;
      xv[t] = in ? x2[u + LPR * t] : make_double2(0.0, 0.0);
#pragma unroll
      for (int i = 0; i < RW; ++i) av[t][i] = in ? load_nt2(rows[i] + 2 * (u + LPR * t)) : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int t = 0; t < U; ++t)
      if (u + LPR * t < KP) {
#pragma unroll
        for (int i = 0; i < RW; ++i) {
          acc[i][0] = fma(av[t][i].x, xv[t].x, acc[i][0]);
          acc[i][1] = fma(av[t][i].y, xv[t].y, acc[i][1]);
        }
      }
  }
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    double v = acc[i][0] + acc[i][1];
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int r = rb + i;
    if (sl == 0 && r < R) {
      if (a.back) {
        const int p = a.yidx[a.yoff[f] + r];
        a.W[p] -= v;
      } else {
        a.stage[a.yoff[f] + r] = v;
      }
    }
  }
}

// A leaf's boundary update A_bi y_i, sparse: boundary unknown r of item i couples to nnz interior unknowns of its
// own line or column (the element's y rows on a horizontal edge, x rows on a vertical edge; none at a corner).
__global__ __launch_bounds__(256) void front_sparse_rows_kernel(int nitems, int nrows, int nnz,
                                                                const double* __restrict__ coef,
                                                                const int32_t* __restrict__ pat, double* stage,
                                                                int64_t stride, int64_t out_off) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (t >= static_cast<int64_t>(nitems) * nrows) return;
  const int64_t i = t / nrows;
  const int r = static_cast<int>(t - i * nrows);
  // coefficient q of row r at coef[(i nnz + q) nrows + r], pattern at pat[q nrows + r]: a wave's loads of one q are
  // consecutive rows (the row-major (nrows, nnz) layout strode 8 nnz bytes per lane: 4.6x the bytes from HBM)
  const double* c = coef + i * nnz * nrows + r;
  const int32_t* p = pat + r;
  const double* y = stage + i * stride;
  double v = 0.0;
  for (int q = 0; q < nnz; ++q) v = fma(c[static_cast<int64_t>(q) * nrows], y[p[q * nrows]], v);
  stage[i * stride + out_off + r] = v;
}

// form 1 (columns): the operator stored transposed (A^T: K rows of ld >= R doubles), one thread per output row, so
// the fronts whose rows are a few tens of doubles long (the deepest separators: |S| = 2 (P - 1)) stream whole
// coalesced A^T rows; x in LDS.  Each row sums its K products in order (two accumulators: even and odd k).
template <int UK>
__global__ __launch_bounds__(256) void front_gemv_cols_kernel(const sem_front_launch a) {
  extern __shared__ double xs[];
  const int f = a.tiles[2 * blockIdx.x], r0 = a.tiles[2 * blockIdx.x + 1];
  const int R = a.dims[4 * f], K = a.dims[4 * f + 1], ld = a.dims[4 * f + 2];
  const int32_t* xi = a.xidx + a.xoff[f];
  for (int k = threadIdx.x; k < K; k += 256) {
    const int p = xi[k];
    xs[k] = p >= 0 ? a.W[p] : 0.0;
  }
  __syncthreads();
  const int r = r0 + static_cast<int>(threadIdx.x);
  if (r >= R) return;
  const double* A = reinterpret_cast<const double*>(a.op[f]) + r;
  double acc0 = 0.0, acc1 = 0.0;
  int k = 0;
  for (; k + UK <= K; k += UK) {
    double av[UK];
#pragma unroll
    for (int u = 0; u < UK; ++u) av[u] = __builtin_nontemporal_load(A + static_cast<int64_t>(k + u) * ld);
#pragma unroll
    for (int u = 0; u < UK; u += 2) {
      acc0 = fma(av[u], xs[k + u], acc0);
      if (u + 1 < UK) acc1 = fma(av[u + 1], xs[k + u + 1], acc1);
    }
  }
  if (k < K) {  // the last < UK columns: one masked batch (k is even: same parities, same order)
    double av[UK];
#pragma unroll
    for (int u = 0; u < UK; ++u)
      av[u] = k + u < K ? __builtin_nontemporal_load(A + static_cast<int64_t>(k + u) * ld) : 0.0;
#pragma unroll
    for (int u = 0; u < UK; u += 2) {
      if (k + u < K) acc0 = fma(av[u], xs[k + u], acc0);
      if (u + 1 < UK && k + u + 1 < K) acc1 = fma(av[u + 1], xs[k + u + 1], acc1);
    }
  }
  const double v = acc0 + acc1;
  if (a.back) {
    const int p = a.yidx[a.yoff[f] + r];
    a.W[p] -= v;
  } else {
    a.stage[a.yoff[f] + r] = v;
  }
}

__global__ __launch_bounds__(256) void front_scatter_kernel(int ncopy, const int32_t* __restrict__ ct,
                                                            const int32_t* __restrict__ cs, int nacc,
                                                            const int32_t* __restrict__ at,
                                                            const int32_t* __restrict__ as4,
                                                            const double* __restrict__ stage, double* W) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < ncopy) {
    W[ct[i]] = stage[cs[i]];
  } else if (i < ncopy + nacc) {
    const int j = i - ncopy;
    const int4 s = reinterpret_cast<const int4*>(as4)[j];
    double v = W[at[j]];
    if (s.x >= 0) v -= stage[s.x];
    if (s.y >= 0) v -= stage[s.y];
    if (s.z >= 0) v -= stage[s.z];
    if (s.w >= 0) v -= stage[s.w];
    W[at[j]] = v;
  }
}

// sem_leaf_forward: one workgroup per element.  Thread (wave w, lane l) owns rows w 8 + l / 8 + 32 k (k < RK) and
// column pairs l % 8 + 8 u (u < 2 RK) of the element's two n x n inverses, so a row is summed by 8 lanes (pairs in
// u order, then an xor tree).  A_uu^-1's fragment stays in registers from t = A_uu^-1 b_u to A_uu^-1 (D1 y_v);
// S_v^-1 streams through once.  The operand vectors live in LDS, zero beyond n (the pad column multiplies them).
template <int NR, int NU>
__device__ __forceinline__ void leaf_rows(const double2 (&f)[NR][NU], const double* x, int s, double (&acc)[NR]) {
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    double v0 = 0.0, v1 = 0.0;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int c = 2 * (s + 8 * u);
      v0 = fma(f[k][u].x, x[c], v0);
      v1 = fma(f[k][u].y, x[c + 1], v1);
    }
    double v = v0 + v1;
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    acc[k] = v;
  }
}

template <int NR, int NU>
__device__ __forceinline__ void leaf_load(double2 (&f)[NR][NU], const double* A, int n, int ld, int rs, int s) {
#pragma unroll
  for (int k = 0; k < NR; ++k)
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int r = rs + 32 * k, c = 2 * (s + 8 * u);
      f[k][u] = (r < n && c < n) ? load_nt2(A + static_cast<int64_t>(r) * ld + c) : make_double2(0.0, 0.0);
    }
}

// KH rows of S_v^-1 tiles per load batch: RK = 4 streams it in two halves, so A_uu^-1's 128 registers and the
// batch fit 256 (two workgroups per CU: 2.97 against 3.32 ms per cfg5 solve with the whole S_v^-1 tile in flight
// at one workgroup per CU, profiles/r06/velocity/split/)
template <int RK, int KH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void leaf_forward_kernel(
    const sem_leaf_launch a) {
  constexpr int NX = 32 * RK;   // operand slots: every column pair a lane touches
  __shared__ double bu[NX], bv[NX], tt[NX], yv[NX];
  const int e = blockIdx.x, n = a.n, ld = a.ld;
  const double* Au = a.blob + static_cast<int64_t>(e) * a.stride;
  const double* Sv = Au + static_cast<int64_t>(n) * ld;
  const double* d1 = Sv + static_cast<int64_t>(n) * ld;
  const double* d2 = d1 + ld;
  const double* coef = d2 + ld;
  const int tid = threadIdx.x, s = tid & 7, rs = tid >> 3;   // rs = w 8 + l / 8
  double2 fa[RK][2 * RK], fs[KH][2 * RK];
  leaf_load<RK, 2 * RK>(fa, Au, n, ld, rs, s);             // in flight while the operands are gathered ...
  leaf_load<KH, 2 * RK>(fs, Sv, n, ld, rs, s);             // ... and S_v^-1's first batch with them
  const int32_t* ix = a.iidx + static_cast<int64_t>(e) * 2 * n;
  for (int k = tid; k < NX; k += 256) {
    bu[k] = k < n ? a.W[ix[k]] : 0.0;
    bv[k] = k < n ? a.W[ix[n + k]] : 0.0;
    yv[k] = 0.0;
  }
  __syncthreads();
  double acc[RK];
  leaf_rows<RK, 2 * RK>(fa, bu, s, acc);                   // t = A_uu^-1 b_u
#pragma unroll
  for (int k = 0; k < RK; ++k)
    if (s == 0 && rs + 32 * k < n) tt[rs + 32 * k] = acc[k];
  __syncthreads();
  if (tid < n) bv[tid] -= d2[tid] * tt[tid];               // b_v - D2 t
  __syncthreads();
#pragma unroll
  for (int h = 0; h < RK; h += KH) {                       // y_v = S_v^-1 (b_v - D2 t), KH rows of tiles at a time
    double ah[KH];
    if (h) leaf_load<KH, 2 * RK>(fs, Sv, n, ld, rs + 32 * h, s);
    leaf_rows<KH, 2 * RK>(fs, bv, s, ah);
#pragma unroll
    for (int k = 0; k < KH; ++k) acc[h + k] = ah[k];
  }
#pragma unroll
  for (int k = 0; k < RK; ++k)
    if (s == 0 && rs + 32 * k < n) yv[rs + 32 * k] = acc[k];
  __syncthreads();
  if (tid < n) bu[tid] = d1[tid] * yv[tid];                // D1 y_v
  __syncthreads();
  leaf_rows<RK, 2 * RK>(fa, bu, s, acc);                   // y_u = t - A_uu^-1 (D1 y_v)
#pragma unroll
  for (int k = 0; k < RK; ++k)
    if (s == 0 && rs + 32 * k < n) tt[rs + 32 * k] -= acc[k];
  __syncthreads();
  for (int k = tid; k < n; k += 256) {
    a.W[ix[k]] = tt[k];
    a.W[ix[n + k]] = yv[k];
  }
  double* out = a.stage + static_cast<int64_t>(e) * a.sstride + a.soff;
  for (int r = tid; r < a.nb; r += 256) {                 // A_bi y_i on the boundary rows' patterns
    double g = 0.0;
    for (int q = 0; q < a.nnz; ++q) {
      const int p = a.pat[q * a.nb + r];
      g = fma(coef[static_cast<int64_t>(q) * a.nb + r], p < n ? tt[p] : yv[p - n], g);
    }
    out[r] = g;
  }
}

}  // namespace sem

extern "C" {

int sem_front_gemv(const sem_front_launch* d, void* stream) {
  if (!d) return sem::set_error(SEM_EINVAL, "front_gemv: null descriptor");
  if (d->ntiles < 0 || d->kmax < 0) return sem::set_error(SEM_EINVAL, "front_gemv: bad sizes");
  if (d->ntiles == 0) return SEM_OK;
  if (!d->op || !d->dims || !d->xoff || !d->yoff || !d->tiles || !d->xidx || !d->W || (d->back ? !d->yidx : !d->stage))
    return sem::set_error(SEM_EINVAL, "front_gemv: null argument");
  const size_t lds = static_cast<size_t>(d->kmax) * sizeof(double);
  if (lds > 64 * 1024) return sem::set_error(SEM_EUNSUPPORTED, "front_gemv: more than 8192 operands per front");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(d->ntiles), block(256);
  if (d->form == 1) {   // columns: A^T rows, one thread per output row, 256 rows per workgroup
    if (d->rows != 256) return sem::set_error(SEM_EINVAL, "front_gemv: the column form takes 256 rows per workgroup");
    hipLaunchKernelGGL((sem::front_gemv_cols_kernel<8>), grid, block, lds, s, *d);
  } else if (d->form != 0) {
    return sem::set_error(SEM_EINVAL, "front_gemv: form must be 0 (rows) or 1 (columns)");
  } else
#define SEM_FRONT_CASE(L, ROWS, RW, U)                                                   \
  if (d->lanes == L && d->rows == ROWS) {                                                \
    hipLaunchKernelGGL((sem::front_gemv_kernel<L, RW, U>), grid, block, lds, s, *d);     \
  } else
  SEM_FRONT_CASE(64, 16, 4, 2) SEM_FRONT_CASE(64, 4, 1, 8) SEM_FRONT_CASE(32, 16, 2, 2) SEM_FRONT_CASE(32, 8, 1, 4)
  SEM_FRONT_CASE(16, 32, 2, 2) SEM_FRONT_CASE(16, 16, 1, 4) SEM_FRONT_CASE(8, 64, 2, 2) SEM_FRONT_CASE(8, 32, 1, 2)
  SEM_FRONT_CASE(4, 128, 2, 2) SEM_FRONT_CASE(4, 64, 1, 2) {
    return sem::set_error(SEM_EINVAL, "front_gemv: unsupported (lanes, rows): lanes 64/32/16/8/4 with rows "
                                      "16|4, 16|8, 32|16, 64|32, 128|64");
  }
#undef SEM_FRONT_CASE
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sem::set_error(SEM_EHIP, std::string("front_gemv launch: ") + hipGetErrorString(e));
  return SEM_OK;
}

int sem_front_sparse_rows(int nitems, int nrows, int nnz, const double* coef, const int32_t* pat, double* stage,
                          int64_t stride, int64_t out_off, void* stream) {
  if (nitems < 0 || nrows < 0 || nnz < 0 || stride < 0 || out_off < 0 || out_off + nrows > stride)
    return sem::set_error(SEM_EINVAL, "front_sparse_rows: bad sizes");
  const int64_t n = static_cast<int64_t>(nitems) * nrows;
  if (n == 0) return SEM_OK;
  if (!coef || !pat || !stage) return sem::set_error(SEM_EINVAL, "front_sparse_rows: null argument");
  hipLaunchKernelGGL(sem::front_sparse_rows_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), nitems, nrows, nnz, coef, pat, stage, stride, out_off);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sem::set_error(SEM_EHIP, std::string("front_sparse_rows launch: ") + hipGetErrorString(e));
  return SEM_OK;
}

int sem_front_scatter(int ncopy, const int32_t* copy_tgt, const int32_t* copy_src, int nacc, const int32_t* acc_tgt,
                      const int32_t* acc_src4, const double* stage, double* W, void* stream) {
  if (ncopy < 0 || nacc < 0) return sem::set_error(SEM_EINVAL, "front_scatter: bad sizes");
  const int64_t n = static_cast<int64_t>(ncopy) + nacc;
  if (n == 0) return SEM_OK;
  if (!stage || !W || (ncopy && (!copy_tgt || !copy_src)) || (nacc && (!acc_tgt || !acc_src4)))
    return sem::set_error(SEM_EINVAL, "front_scatter: null argument");
  if ((reinterpret_cast<uintptr_t>(acc_src4) % 16) != 0)
    return sem::set_error(SEM_EINVAL, "front_scatter: acc_src4 must be 16-byte aligned");
  hipLaunchKernelGGL(sem::front_scatter_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), ncopy, copy_tgt, copy_src, nacc, acc_tgt, acc_src4, stage,
                     W);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sem::set_error(SEM_EHIP, std::string("front_scatter launch: ") + hipGetErrorString(e));
  return SEM_OK;
}

int sem_leaf_forward(const sem_leaf_launch* d, void* stream) {
  if (!d) return sem::set_error(SEM_EINVAL, "leaf_forward: null descriptor");
  if (d->nelem < 0 || d->n < 1 || d->n > 121 || d->ld < d->n || d->ld % 2 || d->nb < 0 || d->nnz < 0 ||
      d->stride < 2 * static_cast<int64_t>(d->n) * d->ld + 2 * d->ld + static_cast<int64_t>(d->nnz) * d->nb ||
      d->stride % 2 || d->sstride < 0 || d->soff < 0)
    return sem::set_error(SEM_EINVAL, "leaf_forward: bad sizes (n <= 121, ld even >= n, stride even >= the blob)");
  if (d->nelem == 0) return SEM_OK;
  if (!d->blob || !d->iidx || !d->pat || !d->W || !d->stage)
    return sem::set_error(SEM_EINVAL, "leaf_forward: null argument");
  if (reinterpret_cast<uintptr_t>(d->blob) % 16) return sem::set_error(SEM_EINVAL, "leaf_forward: blob not 16-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(d->nelem), block(256);
  const int rk = (d->n + 32) / 32;   // 32 RK operand slots >= n + 1 (the pad column)
  if (rk == 1)
    hipLaunchKernelGGL((sem::leaf_forward_kernel<1, 1>), grid, block, 0, s, *d);
  else if (rk == 2)
    hipLaunchKernelGGL((sem::leaf_forward_kernel<2, 2>), grid, block, 0, s, *d);
  else if (rk == 3)
    hipLaunchKernelGGL((sem::leaf_forward_kernel<3, 3>), grid, block, 0, s, *d);
  else
    hipLaunchKernelGGL((sem::leaf_forward_kernel<4, 2>), grid, block, 0, s, *d);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return sem::set_error(SEM_EHIP, std::string("leaf_forward launch: ") + hipGetErrorString(e));
  return SEM_OK;
}

}  // extern "C"
