// Nested static condensation of an element column's interior, solved in three fused launches
// (sem_amd/solvers/velocity_solve.py: VelocityJacobianSolver._nested_solve), in place of the
// reference's SuperLU triangular solves of the velocity Jacobian (NavierStokes_Solver.py:189-203)
// and of the ~15 torch gathers, batched GEMMs and scatters that computed the same thing.
//
// Inside element column e the interior unknowns (lines l = 1..P-1, components c, nodes gy; column
// offset o = (l-1) m + c N_y + gy, m = nc N_y) split into element interiors (element n: nodes
// gy = nP + j, j = 1..P-1; ni = nc (P-1)^2 unknowns, offsets pi[n][.]) and the horizontal edges
// (gy = kP, k = 0..N_ey; ne1 = nc (P-1) unknowns per edge, offsets pe[k ne1 + .]).  With the factor
//     Xi  = A_ii^-1 per element        (nex, ney, ni, ni)
//     Aei = A_ei per element           (nex, ney, 2 ne1, ni)   edges n, n+1 <- interior n
//     Yie = Xi A_ie per element        (nex, ney, ni, 2 ne1)
//     Se  = edge Schur complement^-1   (nex, n_e, n_e),  n_e = (N_ey+1) ne1
// the solve of A_II y = r is
//   K1 (one workgroup per element):  T = Xi r_i,  C = Aei T
//   K2 (workgroups over edge rows):  r_e[k] -= C[n=k][0:ne1] + C[n=k-1][ne1:],  y_e = Se r_e
//   K3 (one workgroup per element):  y_i = T - Yie [y_e[n]; y_e[n+1]]
// Every matrix is stored column-major (the transpose of the factor's blocks) and read once: a
// thread owns an output row and walks the columns, so each column is one coalesced vector load
// across the lanes and no cross-lane reduction is needed (rows here are short: 2 (P-1)^2 = 98
// at P=8; a row-per-wave GEMV spent most of its time in shuffle reductions).  Threads beyond the
// row count split the columns; the partial sums meet in LDS in a fixed order, so results are
// bitwise reproducible.  Operands sit in LDS.  The right-hand side is read straight from the
// solve's line array (column e's interior lines are contiguous there), optionally corrected by the
// interface coupling r = b - A_IB x_B (the back substitution, A_IB diagonal per line), and the
// result is written straight into a line array: no gather, copy or scatter launches.
#include <hip/hip_runtime.h>

#include <string>

#include "sem_internal.h"

namespace sem {

constexpr int kCondThreads = 256;
constexpr int kEdgeRows = 64;                         // edge-kernel rows per workgroup (4 column splits)

struct CondArgs {
  const double *Xi, *Aei, *Yie, *Se;
  const double *XiB, *AXB;     // ABI 11: Xi A_iB (ni x 2 ne1) and A_ei Xi A_iB (2 ne1 x 2 ne1) per element
  const double* ABY;           // ABI 11: A_Bi Xi A_ie (2 ne1 x 2 ne1) per element
  double* Pw;                  // ABI 11: per-column interface partial sums (nex, 2, m)
  const double* aBI;           // ABI 11 (sem_nested_iface_rhs): interface <- interior lines, (nex, 2, P-1, m)
  const double *Ed, *El, *Eu;  // block-Thomas factors of the edge Schur complement (Se == nullptr)
  const int64_t *pi, *pe;
  double *T, *C, *Ye;
  const double* R;     // column e interior at R + e ld_r (offset o)
  int64_t ld_r;
  const double* aIB;   // nullable: r -= aIB[e][l-1][0][r'] xB[e][r'] + aIB[e][l-1][1][r'] xB[e+1][r']
  const double* xB;    // (nex+1, m)
  double* Y;           // column e interior result at Y + e ld_y (offset o)
  int64_t ld_y;
  int P, nex, ney, m, ni, ne1, n_e;
};

// right-hand side at column offset o of column e (with the optional interface correction)
__device__ __forceinline__ double rhs(const CondArgs& a, int e, int64_t o) {
  double v = a.R[e * a.ld_r + o];
  if (a.aIB) {
    const int64_t l1 = o / a.m, r = o - l1 * a.m;
    const double* ab = a.aIB + ((static_cast<int64_t>(e) * (a.P - 1) + l1) * 2) * a.m + r;
    v -= ab[0] * a.xB[static_cast<int64_t>(e) * a.m + r] + ab[a.m] * a.xB[static_cast<int64_t>(e + 1) * a.m + r];
  }
  return v;
}

// y = M x for a column-major (rows x cols) block M (column j at M + j rows), x in LDS, computed by
// the whole workgroup.  Up to 128 rows: thread t owns row t % RP (RP = rows rounded up to a
// wavefront multiple) over the column split t / RP, and the splits' partial sums meet in `part`
// (LDS) in split order.  More rows: each thread owns rows t, t + 256, ... over all columns.
// out(row, value) stores.
// NT: the factor block is read once per solve -- load it non-temporally (gfx950 `nt`; SEM_COND_CPOL=1).  The
// load policy only: results are bitwise identical.  Measured slower (cfg5 velocity solve 8.00 -> 8.04 ms,
// alternated, profiles/r05/basis_cpol/condcpol_*.json), so off by default.
template <bool NT>
__device__ __forceinline__ double ldm(const double* p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

template <bool NT = false, typename Out>
__device__ __forceinline__ void colmajor_gemv(const double* __restrict__ M, int rows, int cols, const double* x,
                                              double* part, Out out) {
  auto dot = [&](int i, int cb, int ce) {
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
    int j = cb;
    for (; j + 3 < ce; j += 4) {
      acc0 = fma(ldm<NT>(M + static_cast<int64_t>(j) * rows + i), x[j], acc0);
      acc1 = fma(ldm<NT>(M + static_cast<int64_t>(j + 1) * rows + i), x[j + 1], acc1);
      acc2 = fma(ldm<NT>(M + static_cast<int64_t>(j + 2) * rows + i), x[j + 2], acc2);
      acc3 = fma(ldm<NT>(M + static_cast<int64_t>(j + 3) * rows + i), x[j + 3], acc3);
    }
    for (; j < ce; ++j) acc0 = fma(ldm<NT>(M + static_cast<int64_t>(j) * rows + i), x[j], acc0);
    return (acc0 + acc1) + (acc2 + acc3);
  };
  const int t = threadIdx.x;
  if (rows > kCondThreads / 2) {  // one column range; every thread owns rows t, t + 256, ...
    for (int i = t; i < rows; i += kCondThreads) out(i, dot(i, 0, cols));
    return;
  }
  // rows <= 128: RP = rows rounded up to a wavefront multiple, 256 / RP column splits (2 or 4)
  const int RP = (rows + 63) / 64 * 64, splits = kCondThreads / RP;
  const int i = t % RP, sp = t / RP;
  double v = 0.0;
  if (i < rows)
    v = dot(i, static_cast<int>(static_cast<int64_t>(cols) * sp / splits),
            static_cast<int>(static_cast<int64_t>(cols) * (sp + 1) / splits));
  part[sp * RP + i] = v;  // every thread reaches both barriers
  __syncthreads();
  if (sp == 0 && i < rows) {
    double sum = v;
    for (int q = 1; q < splits; ++q) sum += part[q * RP + i];
    out(i, sum);
  }
  __syncthreads();
}

// LDS doubles colmajor_gemv needs for its split partial sums
__host__ __device__ constexpr int part_size() { return kCondThreads; }

// K1: T = Xi r_i, C = Aei T for element (e, n) = (blockIdx.x / ney, blockIdx.x % ney).
template <bool NT>
__global__ __launch_bounds__(kCondThreads) void cond_fwd_kernel(const CondArgs a) {
  extern __shared__ double lds[];
  double* part = lds;                     // part_size()
  double* x = lds + part_size();          // ni: r_i
  double* t = x + a.ni;                   // ni: T
  const int el = blockIdx.x, e = el / a.ney, n = el - e * a.ney;
  const int64_t* pin = a.pi + static_cast<int64_t>(n) * a.ni;
  for (int i = threadIdx.x; i < a.ni; i += blockDim.x) x[i] = rhs(a, e, pin[i]);
  __syncthreads();
  const double* Xi = a.Xi + static_cast<int64_t>(el) * a.ni * a.ni;
  double* T = a.T + static_cast<int64_t>(el) * a.ni;
  colmajor_gemv<NT>(Xi, a.ni, a.ni, x, part, [&](int r, double v) {
    T[r] = v;
    t[r] = v;
  });
  __syncthreads();
  const double* Aei = a.Aei + static_cast<int64_t>(el) * 2 * a.ne1 * a.ni;
  double* C = a.C + static_cast<int64_t>(el) * 2 * a.ne1;
  colmajor_gemv<NT>(Aei, 2 * a.ne1, a.ni, t, part, [&](int r, double v) { C[r] = v; });
}

static void launch_cond_fwd(const CondArgs& a, unsigned elems, size_t lds, hipStream_t s) {
  // plain factor loads (non-temporal measured slower in the nested element step, round 5)
  hipLaunchKernelGGL(cond_fwd_kernel<false>, dim3(elems), dim3(kCondThreads), lds, s, a);
}

// K1 of the back substitution (ABI 11): r_i = b_i - A_iB x_B, so Xi r_i = Xi b_i - XiB x_B|n and
// A_ei Xi r_i = A_ei Xi b_i - AXB x_B|n, where T and C still hold Xi b_i and A_ei Xi b_i from the forward
// solve of the same b.  x_B|n: the 2 ne1 interface values at element n's interior heights, column order
// (side s, component c, height j) = x_B[e + s][c N_y + n P + 1 + j'].  Reads 2 ne1 (ni + 2 ne1) doubles per
// element instead of the forward step's (ni + 2 ne1) ni.
__global__ __launch_bounds__(kCondThreads) void cond_fwd_coupled_kernel(const CondArgs a) {
  extern __shared__ double lds[];
  double* part = lds;                     // part_size()
  double* x = lds + part_size();          // G = 2 ne1: x_B|n
  const int el = blockIdx.x, e = el / a.ney, n = el - e * a.ney;
  const int G = 2 * a.ne1, pm1 = a.P - 1, nc = a.ne1 / pm1, NY = a.m / nc;
  for (int q = threadIdx.x; q < G; q += blockDim.x) {
    const int s = q / a.ne1, r = q - s * a.ne1, c = r / pm1, j = r - c * pm1;
    x[q] = a.xB[static_cast<int64_t>(e + s) * a.m + static_cast<int64_t>(c) * NY + static_cast<int64_t>(n) * a.P + 1 + j];
  }
  __syncthreads();
  double* T = a.T + static_cast<int64_t>(el) * a.ni;
  colmajor_gemv(a.XiB + static_cast<int64_t>(el) * a.ni * G, a.ni, G, x, part, [&](int r, double v) { T[r] -= v; });
  double* C = a.C + static_cast<int64_t>(el) * G;
  colmajor_gemv(a.AXB + static_cast<int64_t>(el) * G * G, G, G, x, part, [&](int r, double v) { C[r] -= v; });
}

// K2: y_e = Se (r_e - edge contributions of C); grid (ceil(n_e / 64), nex).  Every workgroup
// forms the column's whole reduced edge right-hand side in LDS (n_e values) and computes 64 rows
// of the column-major Se with four column splits.
__global__ __launch_bounds__(kCondThreads) void cond_edge_kernel(const CondArgs a) {
  extern __shared__ double lds[];
  double* part = lds;
  double* re = lds + part_size();
  const int e = blockIdx.y, ne1 = a.ne1;
  const double* C = a.C + static_cast<int64_t>(e) * a.ney * 2 * ne1;
  for (int i = threadIdx.x; i < a.n_e; i += blockDim.x) {
    const int k = i / ne1, q = i - k * ne1;
    double v = rhs(a, e, a.pe[i]);
    if (k < a.ney) v -= C[static_cast<int64_t>(k) * 2 * ne1 + q];
    if (k > 0) v -= C[static_cast<int64_t>(k - 1) * 2 * ne1 + ne1 + q];
    re[i] = v;
  }
  __syncthreads();
  const int r0 = blockIdx.x * kEdgeRows;
  const int rows = min(kEdgeRows, a.n_e - r0);
  constexpr int splits = kCondThreads / kEdgeRows;
  const int i = threadIdx.x % kEdgeRows, sp = threadIdx.x / kEdgeRows;
  const int cb = static_cast<int>(static_cast<int64_t>(a.n_e) * sp / splits);
  const int ce = static_cast<int>(static_cast<int64_t>(a.n_e) * (sp + 1) / splits);
  const double* Se = a.Se + static_cast<int64_t>(e) * a.n_e * a.n_e + r0;
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
  if (i < rows) {
    int j = cb;
    for (; j + 3 < ce; j += 4) {
      acc0 = fma(Se[static_cast<int64_t>(j) * a.n_e + i], re[j], acc0);
      acc1 = fma(Se[static_cast<int64_t>(j + 1) * a.n_e + i], re[j + 1], acc1);
      acc2 = fma(Se[static_cast<int64_t>(j + 2) * a.n_e + i], re[j + 2], acc2);
      acc3 = fma(Se[static_cast<int64_t>(j + 3) * a.n_e + i], re[j + 3], acc3);
    }
    for (; j < ce; ++j) acc0 = fma(Se[static_cast<int64_t>(j) * a.n_e + i], re[j], acc0);
  }
  part[sp * kEdgeRows + i] = (acc0 + acc1) + (acc2 + acc3);
  __syncthreads();
  if (sp == 0 && i < rows) {
    double v = part[i];
    for (int q = 1; q < splits; ++q) v += part[q * kEdgeRows + i];
    a.Ye[static_cast<int64_t>(e) * a.n_e + r0 + i] = v;
    a.Y[e * a.ld_y + a.pe[r0 + i]] = v;
  }
}

// K2, block-Thomas form (ABI 10): one wavefront per column; the ne1 x ne1 edge blocks are row-major.
//   forward  z_k = Ed_k (r_k - El_{k-1} z_{k-1}),   back  y_k = z_k - Eu_k y_{k+1}
// Templated on the block width B = ne1, so every row/column guard is compile-time (the runtime-width kernel
// of ABI 9 spilled 112 SGPRs and held 422 VGPRs: each `j < b` of its 32-wide unrolled rows was an exec-mask
// branch).  Lane (h, i) = half h of row i: it owns the H columns [h H, h H + H) of row i, so one GEMV is H
// dependent FMAs per lane instead of B, and the two halves' partial sums meet in LDS, where every lane reads
// the pair sums of its own columns for the next GEMV (one LDS round trip per GEMV, the halves' combination
// folded into the broadcast).  The operands of the next D steps (the half-rows of El_{k-1}, Ed_k or Eu_k,
// and the step's right-hand side) are loaded D steps ahead into a register ring: the edge offsets are
// arithmetic (no index load in front of the right-hand side's load), so no load waits on another and the
// sweep runs at the latency of its FMA chains and LDS round trips, not of memory.  Columns are independent
// (grid = nex).
constexpr int kThomasB = 32;  // largest ne1 (= nc (P-1)) of the block-Thomas form

template <int B>
struct EdgeThomas {
  static constexpr int H = B <= 1 ? 2 : (((B + 1) / 2 + 1) & ~1);  // columns per half-row (even)
  static constexpr bool VEC = (B % 2) == 0;                         // 16-byte aligned half-rows
  // steps loaded ahead: 3 (5-8, AGPR-backed, measured no faster at cfg5: 10.37 against 10.33 ms per velocity
  // solve, so the ~1.2 us per step is the chain of LDS round trips, barriers and FMAs, not memory latency)
  static constexpr int D = 3;
};

// half-row h of row i (columns [h H, h H + H) below B) of the row-major B x B block M.  Every lane issues the
// same loads, from clamped addresses, and nothing is computed from the loaded values here: the compiler's
// wait-count pass waits for all outstanding loads (vmcnt(0)) wherever a path issues fewer loads (a load under a
// lane-dependent branch) or a loaded value is used before the loop's back edge (a select), which would turn
// the operand ring into one memory round trip per round.  Columns at or past B hold in-block values of the
// clamped column and meet zero partial sums in half_dot (pt / pz are zero past B); rows past B are unused.
template <int B>
__device__ __forceinline__ void load_half_row(const double* __restrict__ M, int i, int h,
                                              double (&r)[EdgeThomas<B>::H]) {
  constexpr int H = EdgeThomas<B>::H;
  const int j0 = h * H, ic = i < B ? i : B - 1;
  if constexpr (EdgeThomas<B>::VEC) {
#pragma unroll
    for (int q = 0; q < H; q += 2) {
      const int j = j0 + q, jc = j < B ? j : B - 2;  // B even: j < B means j <= B - 2
      const double2 v = *reinterpret_cast<const double2*>(M + ic * B + jc);
      r[q] = v.x;
      r[q + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int q = 0; q < H; ++q) {
      const int j = j0 + q, jc = j < B ? j : B - 1;
      r[q] = M[ic * B + jc];
    }
  }
}

// LDS ordering inside a one-wave workgroup (round 4).  __syncthreads() is a workgroup release + acquire on
// every address space: after the sweep's global stores (Ye) it compiled to s_waitcnt vmcnt(0), i.e. it also
// waited for the loads the operand ring had issued steps ahead, so every step paid a full memory round trip
// (1.2 us per step, no faster with a deeper ring).  A wave's LDS operations execute in order; all the sweep
// needs is that the compiler keeps them in program order and that the writes have completed.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// the terms of one edge row's reduced right-hand side, r - (a0 x0 + a1 x1) - c0 - c1 (rhs() and the two
// element couplings of edge k), as loaded; value() selects the present terms, in rhs()'s order of operations
struct EdgeRhs {
  double r, a0, x0, a1, x1, c0, c1;
  __device__ __forceinline__ double value(bool own, bool coupled, int k, int ney) const {
    double v = r;
    if (coupled) v -= a0 * x0 + a1 * x1;
    if (k < ney) v -= c0;
    if (k > 0) v -= c1;
    return own ? v : 0.0;
  }
};

// sum over this lane's columns of M-row * (p[0][j] + p[1][j]): the two halves' partial sums of the vector
template <int H>
__device__ __forceinline__ double half_dot(const double (&r)[H], const double* p0, const double* p1) {
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int q = 0; q < H; q += 2) {
    a0 = fma(r[q], p0[q] + p1[q], a0);
    a1 = fma(r[q + 1], p0[q + 1] + p1[q + 1], a1);
  }
  return a0 + a1;
}

template <int B>
__global__ __launch_bounds__(64) void cond_edge_thomas_kernel(const CondArgs a) {
  constexpr int H = EdgeThomas<B>::H, D = EdgeThomas<B>::D;
  constexpr int64_t bb = static_cast<int64_t>(B) * B;
  __shared__ double pt[2][2 * H], pz[2][2 * H];  // [half][row] partial sums of t (forward) and z / y
  const int e = blockIdx.x, nb = a.ney + 1, lane = threadIdx.x, i = lane & 31, h = lane >> 5, j0 = h * H;
  const bool row = i < B, own = row && h == 0;  // own: the lane that holds row i's value
  const double* C = a.C + static_cast<int64_t>(e) * a.ney * 2 * B;
  const double* Ed = a.Ed + static_cast<int64_t>(e) * nb * bb;
  const double* El = a.El + static_cast<int64_t>(e) * a.ney * bb;
  const double* Eu = a.Eu + static_cast<int64_t>(e) * a.ney * bb;
  double* Ye = a.Ye + static_cast<int64_t>(e) * a.n_e;
  double* Y = a.Y + e * a.ld_y;
  // edge offset of row i of edge k: i = (l-1) nc + c  ->  (l-1) m + c N_y + k P  (VelocityJacobianSolver._pe)
  const int nc = B / (a.P - 1), NY = a.m / nc;
  const int64_t off_i = static_cast<int64_t>(i / nc) * a.m + static_cast<int64_t>(i % nc) * NY;
  auto edge_off = [&](int k) { return off_i + static_cast<int64_t>(k) * a.P; };
  // the terms of the reduced edge right-hand side of row i of edge k, loaded raw into the ring (see
  // load_half_row): clamped row and couplings, loaded from R when there are none; EdgeRhs::value() combines them
  const int ic = i < B ? i : B - 1;
  const int64_t off_c = static_cast<int64_t>(ic / nc) * a.m + static_cast<int64_t>(ic % nc) * NY;
  const bool coupled = a.aIB != nullptr;
  auto redge = [&](int k, EdgeRhs& q) {
    const int64_t o = off_c + static_cast<int64_t>(k) * a.P, l1 = o / a.m, r = o - l1 * a.m;
    const double* rp = a.R + e * a.ld_r + o;
    const double* ab = coupled ? a.aIB + ((static_cast<int64_t>(e) * (a.P - 1) + l1) * 2) * a.m + r : rp;
    const double* xb = coupled ? a.xB + static_cast<int64_t>(e) * a.m + r : rp;
    const int64_t am = coupled ? a.m : 0;
    const int kc0 = k < a.ney ? k : a.ney - 1, kc1 = k > 0 ? k - 1 : 0;
    q.r = *rp;
    q.a0 = ab[0];
    q.x0 = xb[0];
    q.a1 = ab[am];
    q.x1 = xb[am];
    q.c0 = C[static_cast<int64_t>(kc0) * 2 * B + ic];
    q.c1 = C[static_cast<int64_t>(kc1) * 2 * B + B + ic];
  };
  if (i >= 2 * H) return;  // no row and no column of this lane (B <= 2 H - 1 < 32); never reaches a barrier
  // ---- forward sweep, operands of steps k .. k+D-1 in the ring (slot k % D).  Whole rounds of D steps
  // refill unconditionally (past the last step: clamped, unused), so every path through the loop issues the
  // same loads and each step waits only for its own operands; the last nb % D steps run without refills.
  double rl[D][H], rd[D][H];
  EdgeRhs rr[D];
  auto load_fwd = [&](int k, int s) {
    const int kk = k < nb ? k : nb - 1;
    load_half_row<B>(El + (kk > 0 ? kk - 1 : 0) * bb, i, h, rl[s]);
    load_half_row<B>(Ed + kk * bb, i, h, rd[s]);
    redge(kk, rr[s]);
  };
  auto fwd_step = [&](int k, int s) {
    // t_i = r_i - (El_{k-1} z_{k-1})_i, as the two halves' partial sums
    double t = rr[s].value(own, coupled, k, a.ney);
    if (k > 0) t -= half_dot<H>(rl[s], &pz[0][j0], &pz[1][j0]);
    wave_lds_sync();
    pt[h][i] = row ? t : 0.0;
    wave_lds_sync();
    const double z = half_dot<H>(rd[s], &pt[0][j0], &pt[1][j0]);
    wave_lds_sync();
    pz[h][i] = row ? z : 0.0;
    wave_lds_sync();
    if (own) Ye[static_cast<int64_t>(k) * B + i] = pz[0][i] + pz[1][i];
  };
#pragma unroll
  for (int s = 0; s < D; ++s) load_fwd(s, s);
  int k0 = 0;
  for (; k0 + D <= nb; k0 += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      fwd_step(k0 + s, s);
      load_fwd(k0 + s + D, s);
    }
  }
#pragma unroll
  for (int s = 0; s < D - 1; ++s)
    if (k0 + s < nb) fwd_step(k0 + s, s);
  // ---- back sweep: pz holds y_{nb-1} = z_{nb-1} (as partial sums); steps k = nb-2 .. 0, slot (nb-2-k) % D
  if (own) Y[edge_off(nb - 1)] = pz[0][i] + pz[1][i];
  double ru[D][H], rz[D];
  auto load_back = [&](int k, int s) {
    const int kk = k > 0 ? k : 0;
    load_half_row<B>(Eu + kk * bb, i, h, ru[s]);
    rz[s] = Ye[static_cast<int64_t>(kk) * B + ic];
  };
  auto back_step = [&](int k, int s) {
    const double y = (own ? rz[s] : 0.0) - half_dot<H>(ru[s], &pz[0][j0], &pz[1][j0]);
    wave_lds_sync();
    pz[h][i] = row ? y : 0.0;
    wave_lds_sync();
    if (own) {
      const double v = pz[0][i] + pz[1][i];
      Ye[static_cast<int64_t>(k) * B + i] = v;
      Y[edge_off(k)] = v;
    }
  };
  const int nback = nb - 1;
  if (nback > 0) {
#pragma unroll
    for (int s = 0; s < D; ++s) load_back(nb - 2 - s, s);
  }
  int c0 = 0;
  for (; c0 + D <= nback; c0 += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      back_step(nb - 2 - (c0 + s), s);
      load_back(nb - 2 - (c0 + s) - D, s);
    }
  }
#pragma unroll
  for (int s = 0; s < D - 1; ++s)
    if (c0 + s < nback) back_step(nb - 2 - (c0 + s), s);
}

// The ABI-9 sweep (runtime block width, one lane per row, one step loaded ahead), kept for in-process A/B
// against the templated kernel (SEM_EDGE_THOMAS=1); it reads the ABI-10 row-major blocks.
__device__ __forceinline__ void load_block_row(const double* __restrict__ M, int b, int i, double (&r)[kThomasB]) {
#pragma unroll
  for (int j = 0; j < kThomasB; ++j) r[j] = (j < b && i < b) ? M[i * b + j] : 0.0;
}

__global__ __launch_bounds__(64) void cond_edge_thomas_rt_kernel(const CondArgs a) {
  __shared__ double vb[2][kThomasB];
  const int e = blockIdx.x, b = a.ne1, nb = a.ney + 1, i = threadIdx.x;
  const int64_t bb = static_cast<int64_t>(b) * b;
  const double* C = a.C + static_cast<int64_t>(e) * a.ney * 2 * b;
  const double* Ed = a.Ed + static_cast<int64_t>(e) * nb * bb;
  const double* El = a.El + static_cast<int64_t>(e) * a.ney * bb;
  const double* Eu = a.Eu + static_cast<int64_t>(e) * a.ney * bb;
  double* Ye = a.Ye + static_cast<int64_t>(e) * a.n_e;
  auto redge = [&](int k) {
    if (i >= b) return 0.0;
    double v = rhs(a, e, a.pe[k * b + i]);
    if (k < a.ney) v -= C[static_cast<int64_t>(k) * 2 * b + i];
    if (k > 0) v -= C[static_cast<int64_t>(k - 1) * 2 * b + b + i];
    return v;
  };
  double ml[kThomasB], md[kThomasB], nl[kThomasB], nd[kThomasB];
  load_block_row(Ed, b, i, md);
  double rk = redge(0);
  for (int k = 0; k < nb; ++k) {
    if (k + 1 < nb) {
      load_block_row(El + k * bb, b, i, nl);
      load_block_row(Ed + (k + 1) * bb, b, i, nd);
    }
    const double rn = k + 1 < nb ? redge(k + 1) : 0.0;
    double t = rk;
    if (k > 0) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < kThomasB; ++j)
        if (j < b) acc = fma(ml[j], vb[0][j], acc);
      t -= acc;
    }
    __syncthreads();
    if (i < b) vb[1][i] = t;
    __syncthreads();
    double z = 0.0;
#pragma unroll
    for (int j = 0; j < kThomasB; ++j)
      if (j < b) z = fma(md[j], vb[1][j], z);
    if (i < b) {
      vb[0][i] = z;
      Ye[static_cast<int64_t>(k) * b + i] = z;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kThomasB; ++j) {
      ml[j] = nl[j];
      md[j] = nd[j];
    }
    rk = rn;
  }
  if (i < b) a.Y[e * a.ld_y + a.pe[static_cast<int64_t>(nb - 1) * b + i]] = vb[0][i];
  if (nb > 1) load_block_row(Eu + (nb - 2) * bb, b, i, md);
  for (int k = nb - 2; k >= 0; --k) {
    if (k > 0) load_block_row(Eu + (k - 1) * bb, b, i, nd);
    const double zk = i < b ? Ye[static_cast<int64_t>(k) * b + i] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < kThomasB; ++j)
      if (j < b) acc = fma(md[j], vb[0][j], acc);
    const double y = zk - acc;
    __syncthreads();
    if (i < b) {
      vb[0][i] = y;
      Ye[static_cast<int64_t>(k) * b + i] = y;
      a.Y[e * a.ld_y + a.pe[static_cast<int64_t>(k) * b + i]] = y;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kThomasB; ++j) md[j] = nd[j];
  }
}

template <int B>
static void launch_edge_thomas(const CondArgs& a, hipStream_t s) {
  if (a.ne1 == B)
    hipLaunchKernelGGL(cond_edge_thomas_kernel<B>, dim3(a.nex), dim3(64), 0, s, a);
  else if constexpr (B < kThomasB)
    launch_edge_thomas<B + 1>(a, s);
}

// K3: y_i = T - Yie [y_e[n]; y_e[n+1]] for element (e, n), written to the element's interior nodes.
__global__ __launch_bounds__(kCondThreads) void cond_back_kernel(const CondArgs a) {
  extern __shared__ double lds[];
  double* part = lds;
  double* ye = lds + part_size();  // 2 ne1: edges n, n+1 (contiguous in Ye)
  const int el = blockIdx.x, e = el / a.ney, n = el - e * a.ney;
  const double* src = a.Ye + static_cast<int64_t>(e) * a.n_e + static_cast<int64_t>(n) * a.ne1;
  for (int i = threadIdx.x; i < 2 * a.ne1; i += blockDim.x) ye[i] = src[i];
  __syncthreads();
  const double* Yie = a.Yie + static_cast<int64_t>(el) * a.ni * 2 * a.ne1;
  const double* T = a.T + static_cast<int64_t>(el) * a.ni;
  const int64_t* pin = a.pi + static_cast<int64_t>(n) * a.ni;
  double* Y = a.Y + e * a.ld_y;
  colmajor_gemv(Yie, a.ni, 2 * a.ne1, ye, part, [&](int r, double v) { Y[pin[r]] = T[r] - v; });
}

// g[L][r] = B[L P][r] - sum_l aBI[L][0][l][r] yI[L][l][r] - sum_l aBI[L-1][1][l][r] yI[L-1][l][r]
struct IfaceArgs {
  const double *B, *aBI, *yI;
  double* g;
  int64_t ld_b, ld_yI;
  int P, nex, m;
};

__global__ __launch_bounds__(256) void cond_iface_rhs_kernel(const IfaceArgs a) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= static_cast<int64_t>(a.nex + 1) * a.m) return;
  const int L = static_cast<int>(t / a.m), r = static_cast<int>(t - static_cast<int64_t>(L) * a.m);
  double v = a.B[static_cast<int64_t>(L) * a.P * a.ld_b + r];
  if (L < a.nex) {
    double s = 0.0;
    for (int l = 0; l < a.P - 1; ++l)
      s = fma(a.aBI[((static_cast<int64_t>(L) * 2 + 0) * (a.P - 1) + l) * a.m + r],
              a.yI[static_cast<int64_t>(L) * a.ld_yI + static_cast<int64_t>(l) * a.m + r], s);
    v -= s;
  }
  if (L > 0) {
    double s = 0.0;
    for (int l = 0; l < a.P - 1; ++l)
      s = fma(a.aBI[((static_cast<int64_t>(L - 1) * 2 + 1) * (a.P - 1) + l) * a.m + r],
              a.yI[static_cast<int64_t>(L - 1) * a.ld_yI + static_cast<int64_t>(l) * a.m + r], s);
    v -= s;
  }
  a.g[t] = v;
}

// Interface partial sums of column e (ABI 11): p[e][s][r] = sum_l aBI[e][s][l][r] y_I[e][l][r] for side s, from
// the element step's T = Xi b_i and the edge values y_e, without forming y_i = T - Yie [y_e(n); y_e(n+1)]:
// at element n's interior heights  p = sum_l aBI T  -  (A_Bi Yie) [y_e(n); y_e(n+1)]  (ABY, 2 ne1 columns),
// at the edge heights k = n (and k = ney for the last element)  p = sum_l aBI y_e(k).  One workgroup per element.
__global__ __launch_bounds__(kCondThreads) void cond_iface_part_kernel(const CondArgs a) {
  extern __shared__ double lds[];
  double* part = lds;                     // part_size()
  double* ye = lds + part_size();         // 2 ne1: edges n, n+1 (contiguous in Ye)
  const int el = blockIdx.x, e = el / a.ney, n = el - e * a.ney;
  const int G = 2 * a.ne1, pm1 = a.P - 1, nc = a.ne1 / pm1, NY = a.m / nc;
  const double* src = a.Ye + static_cast<int64_t>(e) * a.n_e + static_cast<int64_t>(n) * a.ne1;
  for (int i = threadIdx.x; i < G; i += blockDim.x) ye[i] = src[i];
  __syncthreads();
  const double* T = a.T + static_cast<int64_t>(el) * a.ni;
  double* pw = a.Pw + static_cast<int64_t>(e) * 2 * a.m;
  const double* ab = a.aBI + static_cast<int64_t>(e) * 2 * pm1 * a.m;   // [s][l][r]
  colmajor_gemv(a.ABY + static_cast<int64_t>(el) * G * G, G, G, ye, part, [&](int q, double v) {
    const int s = q / a.ne1, r1 = q - s * a.ne1, c = r1 / pm1, j = r1 - c * pm1;
    const int64_t r = static_cast<int64_t>(c) * NY + static_cast<int64_t>(n) * a.P + 1 + j;
    double acc = 0.0;
    for (int l = 0; l < pm1; ++l) acc = fma(ab[(static_cast<int64_t>(s) * pm1 + l) * a.m + r], T[(l * nc + c) * pm1 + j], acc);
    pw[static_cast<int64_t>(s) * a.m + r] = acc - v;
  });
  // edge heights: edge k = n, and the closing edge k = ney on the last element of the column
  const int ne = n == a.ney - 1 ? 2 : 1;
  for (int t = threadIdx.x; t < ne * 2 * nc; t += blockDim.x) {
    const int k = n + t / (2 * nc), sc = t % (2 * nc), s = sc / nc, c = sc - s * nc;
    const int64_t r = static_cast<int64_t>(c) * NY + static_cast<int64_t>(k) * a.P;
    const double* yk = a.Ye + static_cast<int64_t>(e) * a.n_e + static_cast<int64_t>(k) * a.ne1;
    double acc = 0.0;
    for (int l = 0; l < pm1; ++l) acc = fma(ab[(static_cast<int64_t>(s) * pm1 + l) * a.m + r], yk[l * nc + c], acc);
    pw[static_cast<int64_t>(s) * a.m + r] = acc;
  }
}

// g[L] = B[L P] - p[L][0] - p[L-1][1]
struct IfacePartArgs {
  const double *B, *Pw;
  double* g;
  int64_t ld_b;
  int P, nex, m;
};

__global__ __launch_bounds__(256) void cond_iface_sum_kernel(const IfacePartArgs a) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= static_cast<int64_t>(a.nex + 1) * a.m) return;
  const int L = static_cast<int>(t / a.m), r = static_cast<int>(t - static_cast<int64_t>(L) * a.m);
  double v = a.B[static_cast<int64_t>(L) * a.P * a.ld_b + r];
  if (L < a.nex) v -= a.Pw[static_cast<int64_t>(L) * 2 * a.m + r];
  if (L > 0) v -= a.Pw[(static_cast<int64_t>(L - 1) * 2 + 1) * a.m + r];
  a.g[t] = v;
}

static int launch_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) return SEM_OK;
  return set_error(SEM_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// CondArgs of a nested solve from the descriptor (checks shared by both entry points)
static int nested_args(const sem_nested_desc* d, const double* R, int64_t ld_r, const double* aIB, const double* xB,
                       double* Y, int64_t ld_y, CondArgs& a) {
  if (!d || !R || !Y) return set_error(SEM_EINVAL, "nested_solve: null argument");
  if (d->P < 2 || d->nex < 1 || d->ney < 1 || (d->nc != 1 && d->nc != 2) || d->NY != d->ney * d->P + 1)
    return set_error(SEM_EINVAL, "nested_solve: bad sizes");
  const bool thomas = d->Se == nullptr;
  if (!d->Xi || !d->Aei || !d->Yie || !d->pi || !d->pe || !d->T || !d->C || !d->Ye ||
      (thomas && (!d->Ed || (d->ney > 0 && (!d->El || !d->Eu)))))
    return set_error(SEM_EINVAL, "nested_solve: null factor or work array");
  if ((aIB == nullptr) != (xB == nullptr)) return set_error(SEM_EINVAL, "nested_solve: aIB and xB go together");
  a = CondArgs{};
  a.Xi = d->Xi;
  a.Aei = d->Aei;
  a.Yie = d->Yie;
  a.Se = d->Se;
  a.XiB = d->XiB;
  a.AXB = d->AXB;
  a.ABY = d->ABY;
  a.Pw = d->Pw;
  a.Ed = d->Ed;
  a.El = d->El;
  a.Eu = d->Eu;
  a.pi = d->pi;
  a.pe = d->pe;
  a.T = d->T;
  a.C = d->C;
  a.Ye = d->Ye;
  a.R = R;
  a.ld_r = ld_r;
  a.aIB = aIB;
  a.xB = xB;
  a.Y = Y;
  a.ld_y = ld_y;
  a.P = d->P;
  a.nex = d->nex;
  a.ney = d->ney;
  a.m = d->nc * d->NY;
  a.ne1 = d->nc * (d->P - 1);
  a.ni = a.ne1 * (d->P - 1);
  a.n_e = (d->ney + 1) * a.ne1;
  if (thomas && a.ne1 > kThomasB)
    return set_error(SEM_EUNSUPPORTED, "nested_solve: edge blocks wider than the block-Thomas form's 32");
  if (!thomas && static_cast<size_t>(a.n_e + part_size()) * sizeof(double) > 64 * 1024)
    return set_error(SEM_EUNSUPPORTED, "nested_solve: too many edge unknowns per column");
  return SEM_OK;
}

// K2 (edge solve) of a nested solve
static int nested_edge(const CondArgs& a, hipStream_t s) {
  if (a.Se == nullptr && tune(SEM_TUNE_EDGE_THOMAS) == 1)
    hipLaunchKernelGGL(cond_edge_thomas_rt_kernel, dim3(a.nex), dim3(64), 0, s, a);
  else if (a.Se == nullptr)
    launch_edge_thomas<1>(a, s);
  else
    hipLaunchKernelGGL(cond_edge_kernel, dim3((a.n_e + kEdgeRows - 1) / kEdgeRows, a.nex), dim3(kCondThreads),
                       (part_size() + a.n_e) * sizeof(double), s, a);
  return launch_check("nested_solve edge");
}

// K2 and K3 (element back step) of a nested solve
static int nested_edge_back(const CondArgs& a, hipStream_t s) {
  if (int st = nested_edge(a, s)) return st;
  hipLaunchKernelGGL(cond_back_kernel, dim3(static_cast<unsigned>(a.nex) * a.ney), dim3(kCondThreads),
                     (part_size() + 2 * a.ne1) * sizeof(double), s, a);
  return launch_check("nested_solve back");
}

}  // namespace sem

extern "C" {

int sem_nested_solve(const sem_nested_desc* d, const double* R, int64_t ld_r, const double* aIB, const double* xB,
                     double* Y, int64_t ld_y, void* stream) {
  sem::CondArgs a;
  if (int st = sem::nested_args(d, R, ld_r, aIB, xB, Y, ld_y, a)) return st;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t part = sem::part_size() * sizeof(double);
  sem::launch_cond_fwd(a, static_cast<unsigned>(a.nex) * a.ney, part + 2 * a.ni * sizeof(double), s);
  if (int st = sem::launch_check("nested_solve fwd")) return st;
  return sem::nested_edge_back(a, s);
}

int sem_nested_back_solve(const sem_nested_desc* d, const double* R, int64_t ld_r, const double* aIB,
                          const double* xB, double* Y, int64_t ld_y, void* stream) {
  sem::CondArgs a;
  if (!aIB || !xB) return sem::set_error(SEM_EINVAL, "nested_back_solve: aIB and xB are required");
  if (int st = sem::nested_args(d, R, ld_r, aIB, xB, Y, ld_y, a)) return st;
  if (!d->XiB || !d->AXB) return sem::set_error(SEM_EINVAL, "nested_back_solve: the descriptor has no XiB / AXB");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t part = sem::part_size() * sizeof(double);
  hipLaunchKernelGGL(sem::cond_fwd_coupled_kernel, dim3(static_cast<unsigned>(a.nex) * a.ney), dim3(sem::kCondThreads),
                     part + 2 * a.ne1 * sizeof(double), s, a);
  if (int st = sem::launch_check("nested_back_solve fwd")) return st;
  return sem::nested_edge_back(a, s);
}

int sem_nested_iface_rhs(const sem_nested_desc* d, const double* R, int64_t ld_r, const double* B, int64_t ld_b,
                         const double* aBI, double* Y, int64_t ld_y, double* g, void* stream) {
  sem::CondArgs a;
  if (!B || !aBI || !g) return sem::set_error(SEM_EINVAL, "nested_iface_rhs: null argument");
  if (int st = sem::nested_args(d, R, ld_r, nullptr, nullptr, Y, ld_y, a)) return st;
  if (!d->ABY || !d->Pw) return sem::set_error(SEM_EINVAL, "nested_iface_rhs: the descriptor has no ABY / Pw");
  a.aBI = aBI;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned elems = static_cast<unsigned>(a.nex) * a.ney;
  const size_t part = sem::part_size() * sizeof(double);
  sem::launch_cond_fwd(a, elems, part + 2 * a.ni * sizeof(double), s);
  if (int st = sem::launch_check("nested_iface_rhs fwd")) return st;
  if (int st = sem::nested_edge(a, s)) return st;
  hipLaunchKernelGGL(sem::cond_iface_part_kernel, dim3(elems), dim3(sem::kCondThreads),
                     part + 2 * a.ne1 * sizeof(double), s, a);
  if (int st = sem::launch_check("nested_iface_rhs part")) return st;
  sem::IfacePartArgs b{B, d->Pw, g, ld_b, d->P, d->nex, a.m};
  const int64_t n = static_cast<int64_t>(d->nex + 1) * a.m;
  hipLaunchKernelGGL(sem::cond_iface_sum_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, s, b);
  return sem::launch_check("nested_iface_rhs sum");
}

int sem_interface_rhs(int P, int nex, int m, const double* B, int64_t ld_b, const double* aBI, const double* yI,
                      int64_t ld_yI, double* g, void* stream) {
  if (P < 2 || nex < 1 || m < 1 || !B || !aBI || !yI || !g) return sem::set_error(SEM_EINVAL, "interface_rhs");
  sem::IfaceArgs a{B, aBI, yI, g, ld_b, ld_yI, P, nex, m};
  const int64_t n = static_cast<int64_t>(nex + 1) * m;
  hipLaunchKernelGGL(sem::cond_iface_rhs_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return sem::launch_check("interface_rhs");
}

}  // extern "C"
