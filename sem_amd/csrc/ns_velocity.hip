// Navier-Stokes velocity-Jacobian blocks for the device direct solve (sem_amd/solvers/velocity_solve.py).
//
// The reference factorises the Dirichlet-row-replaced 2N x 2N velocity Jacobian
//     [[J_uu, J_uv], [J_vu, J_vv]],  J_uu = Sys + Re diag(G_x u), J_uv = Re diag(G_y u), ...
// with host SuperLU (NavierStokes_Solver.py:176-184) and solves with it twice per Schur-complement
// matvec (:189-203).  Here the structured mesh is split into node lines (x-major numbering,
// SEM.py:110): the interface lines x = L*P (L = 0..N_ex) and the P-1 interior lines of each element
// column.  Interior lines of column e couple only to each other and to the two interface lines
// L = e, e+1, so the Jacobian condenses statically: one dense block A_II per element column
// (batched LU on the device), then a block-tridiagonal Schur complement over the interface lines.
//
// This kernel writes the pieces, one thread per Jacobian row, from the operator's tensor-product
// form (the same algebra as the apply kernels, SEM.py:170-245):
//   A x [gx,gy] = My[gy] sum_k (cK dy/dx Kx[gx][k] + cX cu dy/2 Gx[gx][k]) x[k][gy]
//               + Mx[gx] sum_l (cK dx/dy Ky[gy][l] + cY cv dx/2 Gy[gy][l]) x[gx][l]
//               + cM dx dy/4 Mx[gx] My[gy] x[gx][gy]
// with Kx, Gx, Ky, Gy the 1-D direct-stiffness sums of the GLL tables (GLL.py:62-81) and Mx, My the
// assembled GLL weights.  Unknowns of one line are ordered (component c, y node gy): m = 2 NY.
//   A_II [e][(l-1) m + c NY + gy][(l'-1) m + c' NY + gy']   interior lines l, l' = 1..P-1 (dense)
//   D    [L][c NY + gy][c' NY + gy']                         interface line L with itself (dense)
//   aIB  [e][l-1][s][c NY + gy]   coefficient of line e P + s P (s = 0, 1) in interior row (l, c, gy)
//   aBI  [e][s][l-1][c NY + gy]   coefficient of interior node (l, c, gy) in row (line eP + sP, c, gy)
//   E    [L][c NY + gy]           row on line L, column on line L+1 (same c, gy)
//   F    [L][c NY + gy]           row on line L+1, column on line L
// Dirichlet rows (the reference's mask_bound) are identity rows: 1 on the diagonal, 0 elsewhere,
// in every piece.  The dense blocks are zero-filled by the caller (hipMemsetAsync); each row is
// written by exactly one thread, so nothing races.  A column range [c0, c1) restricts the A_II
// writes to those element columns (A_II then holds c1 - c0 blocks): the factorisation assembles and
// condenses a large mesh's dense interiors a chunk of columns at a time; every other piece is
// written in full by every call.
#include <hip/hip_runtime.h>

#include <string>

#include "sem_internal.h"

namespace sem {

struct VelocityArgs {
  const double* tab;  // K_s | G_s | w (handle table)
  const double *cu, *cv, *juu, *juv, *jvu, *jvv;
  const uint8_t* mask;
  double fKx, fKy, fM, fX, fY;  // cK dy/dx, cK dx/dy, cM dx dy/4, cX dy/2, cY dx/2
  int P, nex, ney, NY, NX;
  int nc;  // components per node: 2 (NS velocity [u | v]) or 1 (a scalar operator, e.g. the CD Jacobian)
  int c0, c1;  // element columns whose A_II blocks are written (A_II indexed from c0)
  int eb, ee, lb0, lb1;  // element columns / global lines of the handle's strip (whole mesh: 0, nex, 0, NX-1)
  unsigned sides;
  double *AII, *D, *aIB, *aBI, *E, *F;
  // ABI 7, condensed layout of the interior rows of columns [c0, c1) (instead of the dense AII):
  //   Aii [e][n][ni][ni], Aie [e][n][ni][2 ne1], Aei [e][n][2 ne1][ni]        (element n of column e)
  //   Aed [e][k][ne1][ne1] (edge k with itself), Aeu [e][k][ne1][ne1] (row edge k, column edge k+1),
  //   Ael [e][k][ne1][ne1] (row edge k+1, column edge k)
  // element-interior index ((l-1) nc + c)(P-1) + j-1 (node (line l, component c, y node nP + j)),
  // edge index (l-1) nc + c (node (l, c, kP)); e counted from c0.
  double *Aii, *Aie, *Aei, *Aed, *Aeu, *Ael;
};

__device__ __forceinline__ bool is_dirichlet(const VelocityArgs& a, int gx, int gy) {
  if (a.mask) return a.mask[static_cast<int64_t>(gx - a.lb0) * a.NY + gy] != 0;
  return ((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NX - 1) ||
         ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == a.NY - 1);
}

// Interior row (column L, line l, component c, node gy) of a non-Dirichlet node in the condensed layout:
// its x couplings (the other interior lines of the column, same c and gy), y couplings (its line's nodes
// in the element(s) holding gy), the other component at the node, and the diagonal, each written to the
// block that holds the pair; the interface couplings go to aIB as in the dense layout.
__device__ void condensed_row(const VelocityArgs& a, int L, int l, int c, int gy, int r, int64_t node, bool dir,
                              double mx, double my, double cu, double cv, const double* Ks, const double* Gs) {
  const int P = a.P, n = P + 1, nc = a.nc, ne1 = nc * (P - 1), ni = ne1 * (P - 1);
  const int ey = gy / P, j = gy - ey * P;
  const int64_t col = L - a.c0;
  double* ib = a.aIB + (static_cast<int64_t>(L - a.eb) * (P - 1) + l - 1) * 2 * a.nc * a.NY + r;
  const int mm = nc * a.NY;
  const double fx = a.fKx * my, gxc = a.fX * cu * my;
  const double fy = a.fKy * mx, gyc = a.fY * cv * mx;
  auto xk = [&](int i, int k) { return fx * Ks[i * n + k] + gxc * Gs[i * n + k]; };
  auto yk = [&](int i, int k) { return fy * Ks[i * n + k] + gyc * Gs[i * n + k]; };
  const int lc = (l - 1) * nc + c;  // position of (l, c) among a node's interior-line unknowns
  if (j != 0) {  // element interior of element ey
    const int64_t el = col * a.ney + ey;
    const int ri = lc * (P - 1) + j - 1;
    double* Ar = a.Aii + (el * ni + ri) * ni;
    if (dir) {
      Ar[ri] = 1.0;
      ib[0] = 0.0;
      ib[mm] = 0.0;
      return;
    }
    double* Er = a.Aie + (el * ni + ri) * 2 * ne1;
    double dg = a.fM * mx * my + (c == 0 ? (a.juu ? a.juu[node] : 0.0) : (a.jvv ? a.jvv[node] : 0.0)) + xk(l, l);
    for (int k = 1; k < P; ++k)
      if (k != l) Ar[((k - 1) * nc + c) * (P - 1) + j - 1] = xk(l, k);
    ib[0] = xk(l, 0);
    ib[mm] = xk(l, P);
    for (int q = 0; q <= P; ++q) {
      const double v = yk(j, q);
      if (q == j) dg += v;
      else if (q == 0) Er[lc] = v;
      else if (q == P) Er[ne1 + lc] = v;
      else Ar[lc * (P - 1) + q - 1] = v;
    }
    if (nc == 2) {
      const double* jc = c == 0 ? a.juv : a.jvu;
      if (jc) Ar[((l - 1) * nc + 1 - c) * (P - 1) + j - 1] = jc[node];
    }
    Ar[ri] = dg;
    return;
  }
  // edge k = ey (gy = kP): row lc of edge k
  const int k = ey;
  double* Dr = a.Aed + ((col * (a.ney + 1) + k) * ne1 + lc) * ne1;
  if (dir) {
    Dr[lc] = 1.0;
    ib[0] = 0.0;
    ib[mm] = 0.0;
    return;
  }
  double dg = a.fM * mx * my + (c == 0 ? (a.juu ? a.juu[node] : 0.0) : (a.jvv ? a.jvv[node] : 0.0)) + xk(l, l);
  for (int kk = 1; kk < P; ++kk)
    if (kk != l) Dr[(kk - 1) * nc + c] = xk(l, kk);
  ib[0] = xk(l, 0);
  ib[mm] = xk(l, P);
  if (k > 0) {  // element k-1 below: the edge is its top edge (rows ne1.. of its A_ei)
    const int64_t el = col * a.ney + k - 1;
    double* Fr = a.Aei + (el * 2 * ne1 + ne1 + lc) * ni;
    for (int q = 0; q <= P; ++q) {
      const double v = yk(P, q);
      if (q == P) dg += v;
      else if (q == 0) a.Ael[((col * a.ney + k - 1) * ne1 + lc) * ne1 + lc] = v;
      else Fr[lc * (P - 1) + q - 1] = v;
    }
  }
  if (k < a.ney) {  // element k above: the edge is its bottom edge (rows 0.. of its A_ei)
    const int64_t el = col * a.ney + k;
    double* Fr = a.Aei + (el * 2 * ne1 + lc) * ni;
    for (int q = 0; q <= P; ++q) {
      const double v = yk(0, q);
      if (q == 0) dg += v;
      else if (q == P) a.Aeu[((col * a.ney + k) * ne1 + lc) * ne1 + lc] = v;
      else Fr[lc * (P - 1) + q - 1] = v;
    }
  }
  if (nc == 2) {
    const double* jc = c == 0 ? a.juv : a.jvu;
    if (jc) Dr[(l - 1) * nc + 1 - c] = jc[node];
  }
  Dr[lc] = dg;
}

// One thread per Jacobian row: row = line gx (the handle's lines lb0..lb1), component c, node gy.  On an
// element-column strip handle (the partitioned solvers) the x sums run over the strip's own columns
// [eb, ee): the strip's two interface lines get the partial rows of its side (their sums over the two
// strips are the whole-mesh rows), and the pointwise Jacobian terms and Dirichlet identity rows of the
// right interface line are left to the strip on its right (the rule of the apply kernels).
__global__ __launch_bounds__(256) void velocity_blocks_kernel(const VelocityArgs a) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int NY = a.NY, P = a.P, n = P + 1, m = a.nc * NY;
  if (t >= static_cast<int64_t>(a.lb1 - a.lb0 + 1) * m) return;
  const int lx = static_cast<int>(t / m), r = static_cast<int>(t - static_cast<int64_t>(lx) * m);
  const int gx = a.lb0 + lx;
  const int c = r / NY, gy = r - c * NY;
  const double* Ks = a.tab;
  const double* Gs = a.tab + n * n;
  const double* w = a.tab + 2 * n * n;
  const int L = gx / P, l = gx - L * P;  // interface line L (l == 0) or interior line l of column L
  const int Ll = L - a.eb;               // the strip's local line / column index
  const int64_t node = static_cast<int64_t>(lx) * NY + gy;
  const bool dir = is_dirichlet(a, gx, gy);
  const bool own = !(gx == a.lb1 && a.ee < a.nex);  // the strip's right interface line: its right owner's
  const int nI = (P - 1) * m;
  // row pointer into the dense block holding this row, and the column offset of line-local node 0
  double* row;
  int64_t col0;  // column index of (this line, c = 0, gy = 0) within the block
  if (l != 0 && (L < a.c0 || L >= a.c1)) {  // interior row of a column outside the A_II range: aIB only
    double* ib = a.aIB + (static_cast<int64_t>(Ll) * (P - 1) + l - 1) * 2 * m + r;
    if (dir) {
      ib[0] = 0.0;
      ib[m] = 0.0;
      return;
    }
    const int ey = gy / P, j = gy - ey * P;
    const double my = j != 0 ? w[j] : (ey > 0 ? w[P] : 0.0) + (ey < a.ney ? w[0] : 0.0);
    const double cu = a.cu ? a.cu[node] : 1.0;
    const double fx = a.fKx * my, gxc = a.fX * cu * my;
    ib[0] = fx * Ks[l * n] + gxc * Gs[l * n];
    ib[m] = fx * Ks[l * n + P] + gxc * Gs[l * n + P];
    return;
  }
  if (l != 0 && a.Aii) {  // ABI 7: condensed layout
    const int ey = gy / P, j = gy - ey * P;
    const double mx = w[l];
    const double my = j != 0 ? w[j] : (ey > 0 ? w[P] : 0.0) + (ey < a.ney ? w[0] : 0.0);
    condensed_row(a, L, l, c, gy, r, node, dir, mx, my, a.cu ? a.cu[node] : 1.0, a.cv ? a.cv[node] : 1.0, Ks, Gs);
    return;
  }
  if (l == 0) {
    row = a.D + (static_cast<int64_t>(Ll) * m + r) * m;
    col0 = 0;
  } else {
    row = a.AII + (static_cast<int64_t>(L - a.c0) * nI + (l - 1) * m + r) * nI;
    col0 = static_cast<int64_t>(l - 1) * m;
  }
  const int64_t self = col0 + r;
  if (dir) {  // identity row (its owner's): no coupling to anything else
    if (own) row[self] = 1.0;
    if (l == 0) {
      if (L < a.ee) {
        a.E[static_cast<int64_t>(Ll) * m + r] = 0.0;
        for (int k = 1; k < P; ++k) a.aBI[((static_cast<int64_t>(Ll) * 2 + 0) * (P - 1) + k - 1) * m + r] = 0.0;
      }
      if (L > a.eb) {
        a.F[static_cast<int64_t>(Ll - 1) * m + r] = 0.0;
        for (int k = 1; k < P; ++k) a.aBI[((static_cast<int64_t>(Ll - 1) * 2 + 1) * (P - 1) + k - 1) * m + r] = 0.0;
      }
    } else {
      for (int s = 0; s < 2; ++s) a.aIB[((static_cast<int64_t>(Ll) * (P - 1) + l - 1) * 2 + s) * m + r] = 0.0;
    }
    return;
  }
  // assembled weights of this node's line (x, over the strip's columns) and column (y)
  const double mx = l != 0 ? w[l] : (L > a.eb ? w[P] : 0.0) + (L < a.ee ? w[0] : 0.0);
  const int ey = gy / P, j = gy - ey * P;
  const double my = j != 0 ? w[j] : (ey > 0 ? w[P] : 0.0) + (ey < a.ney ? w[0] : 0.0);
  const double cu = a.cu ? a.cu[node] : 1.0, cv = a.cv ? a.cv[node] : 1.0;
  const double fx = a.fKx * my, gxc = a.fX * cu * my;  // x rows: fx Ks[.][.] + gxc Gs[.][.]
  const double fy = a.fKy * mx, gyc = a.fY * cv * mx;  // y rows: fy Ks[.][.] + gyc Gs[.][.]
  auto xk = [&](int i, int k) { return fx * Ks[i * n + k] + gxc * Gs[i * n + k]; };
  auto yk = [&](int i, int k) { return fy * Ks[i * n + k] + gyc * Gs[i * n + k]; };

  // diagonal: x part + y part + mass + the Jacobian's own diagonal term (its owner's)
  double dg = a.fM * mx * my;
  if (own) dg += c == 0 ? (a.juu ? a.juu[node] : 0.0) : (a.jvv ? a.jvv[node] : 0.0);
  if (l != 0) {
    dg += xk(l, l);
  } else {
    if (L > a.eb) dg += xk(P, P);
    if (L < a.ee) dg += xk(0, 0);
  }
  // y coupling along the line (same component): elements ey-1 (row P) and ey (row j)
  const int64_t yb = col0 + static_cast<int64_t>(c) * NY;  // column of (this line, c, gy = 0)
  if (j != 0) {
    for (int k = 0; k <= P; ++k) {
      const double v = yk(j, k);
      if (k == j) dg += v; else row[yb + ey * P + k] += v;
    }
  } else {
    if (ey > 0)
      for (int k = 0; k <= P; ++k) {
        const double v = yk(P, k);
        if (k == P) dg += v; else row[yb + (ey - 1) * P + k] += v;
      }
    if (ey < a.ney)
      for (int k = 0; k <= P; ++k) {
        const double v = yk(0, k);
        if (k == 0) dg += v; else row[yb + ey * P + k] += v;
      }
  }
  row[self] += dg;
  // the other component at the same node: J_uv = diag(juv) (u rows), J_vu = diag(jvu) (v rows)
  if (a.nc == 2 && own) {
    const double* jc = c == 0 ? a.juv : a.jvu;
    if (jc) row[col0 + (1 - c) * NY + gy] = jc[node];
  }

  // x coupling to the other lines of this node's element column(s)
  if (l != 0) {
    double* AIIrow = row;
    for (int k = 1; k < P; ++k)
      if (k != l) AIIrow[static_cast<int64_t>(k - 1) * m + r] = xk(l, k);
    for (int s = 0; s < 2; ++s) a.aIB[((static_cast<int64_t>(Ll) * (P - 1) + l - 1) * 2 + s) * m + r] = xk(l, s * P);
  } else {
    if (L < a.ee) {  // left line of column L
      for (int k = 1; k < P; ++k) a.aBI[((static_cast<int64_t>(Ll) * 2 + 0) * (P - 1) + k - 1) * m + r] = xk(0, k);
      a.E[static_cast<int64_t>(Ll) * m + r] = xk(0, P);
    }
    if (L > a.eb) {  // right line of column L-1
      for (int k = 1; k < P; ++k) a.aBI[((static_cast<int64_t>(Ll - 1) * 2 + 1) * (P - 1) + k - 1) * m + r] = xk(P, k);
      a.F[static_cast<int64_t>(Ll - 1) * m + r] = xk(P, 0);
    }
  }
}

static int hip_check_v(hipError_t e, const char* what) {
  if (e == hipSuccess) return SEM_OK;
  return set_error(SEM_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace sem

extern "C" {

int sem_line_block_sizes(const sem_handle* h, int ncomp, int64_t* sizes) {
  if (!h || !sizes) return sem::set_error(SEM_EINVAL, "null argument");
  if (ncomp != 1 && ncomp != 2) return sem::set_error(SEM_EINVAL, "ncomp must be 1 or 2");
  // ABI 7: a strip handle's pieces cover its own element columns and lines
  const int64_t m = ncomp * h->NY, nI = static_cast<int64_t>(h->P - 1) * m, ne = h->ex_end - h->ex_begin;
  sizes[0] = ne * nI * nI;             // A_II
  sizes[1] = (ne + 1) * m * m;         // D
  sizes[2] = ne * (h->P - 1) * 2 * m;  // aIB
  sizes[3] = ne * 2 * (h->P - 1) * m;  // aBI
  sizes[4] = ne * m;                   // E
  sizes[5] = ne * m;                   // F
  return SEM_OK;
}

int sem_velocity_block_sizes(const sem_handle* h, int64_t* sizes) { return sem_line_block_sizes(h, 2, sizes); }

int sem_condensed_block_sizes(const sem_handle* h, int ncomp, int64_t* sizes) {
  if (!h || !sizes) return sem::set_error(SEM_EINVAL, "null argument");
  if (ncomp != 1 && ncomp != 2) return sem::set_error(SEM_EINVAL, "ncomp must be 1 or 2");
  if (h->P < 2) return sem::set_error(SEM_EINVAL, "the condensed layout needs P >= 2");
  const int64_t ne1 = static_cast<int64_t>(ncomp) * (h->P - 1), ni = ne1 * (h->P - 1), ney = h->ney;
  sizes[0] = ney * ni * ni;         // A_ii
  sizes[1] = ney * ni * 2 * ne1;    // A_ie
  sizes[2] = ney * 2 * ne1 * ni;    // A_ei
  sizes[3] = (ney + 1) * ne1 * ne1; // A_ee diagonal blocks
  sizes[4] = ney * ne1 * ne1;       // A_ee upper (edge k -> k+1)
  sizes[5] = ney * ne1 * ne1;       // A_ee lower (edge k+1 -> k)
  return SEM_OK;
}

static int velocity_blocks_impl(sem_handle* h, const sem_velocity_desc* d, double* AII, double* const* cond, double* D,
                                double* aIB, double* aBI, double* E, double* F, void* stream) {
  if (!h || !d || !D || !E || !F) return sem::set_error(SEM_EINVAL, "null argument");
  if (h->P > 1 && ((!AII && !cond) || !aIB || !aBI)) return sem::set_error(SEM_EINVAL, "null interior block");
  if (cond)
    for (int i = 0; i < 6; ++i)
      if (!cond[i]) return sem::set_error(SEM_EINVAL, "null condensed block");
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != h->device)
    return sem::set_error(SEM_EINVAL, "handle belongs to another device than the current one");
  const int nc = d->ncomp == 0 ? 2 : d->ncomp;
  if (nc != 1 && nc != 2) return sem::set_error(SEM_EINVAL, "ncomp must be 0, 1 or 2");
  if (nc == 1 && (d->juv || d->jvu || d->jvv))
    return sem::set_error(SEM_EINVAL, "a one-component operator has no juv / jvu / jvv term");
  // column range in global element columns, inside the handle's strip (col_end 0: to its end)
  const int c0 = d->col_end == 0 && d->col_begin == 0 ? h->ex_begin : d->col_begin;
  const int c1 = d->col_end == 0 ? h->ex_end : d->col_end;
  if (c0 < h->ex_begin || c1 > h->ex_end || c0 >= c1) return sem::set_error(SEM_EINVAL, "bad A_II column range");
  int64_t sz[6];
  sem_line_block_sizes(h, nc, sz);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int st;
  if (cond) {
    int64_t cs[6];
    sem_condensed_block_sizes(h, nc, cs);
    for (int i = 0; i < 6; ++i)
      if ((st = sem::hip_check_v(hipMemsetAsync(cond[i], 0, cs[i] * (c1 - c0) * sizeof(double), s), "memset blocks")))
        return st;
  } else {
    const int64_t szA = sz[0] / (h->ex_end - h->ex_begin) * (c1 - c0);
    if (h->P > 1 && (st = sem::hip_check_v(hipMemsetAsync(AII, 0, szA * sizeof(double), s), "memset A_II")))
      return st;
  }
  if ((st = sem::hip_check_v(hipMemsetAsync(D, 0, sz[1] * sizeof(double), s), "memset D"))) return st;
  sem::VelocityArgs a{};
  a.tab = h->d_tab;
  a.cu = d->cu;
  a.cv = d->cv;
  a.juu = d->juu;
  a.juv = d->juv;
  a.jvu = d->jvu;
  a.jvv = d->jvv;
  a.mask = d->dir_mask;
  a.sides = d->dir_sides;
  a.fKx = d->c_stiff * (h->dy / h->dx);
  a.fKy = d->c_stiff * (h->dx / h->dy);
  a.fM = d->c_mass * ((h->dx / 2.0) * (h->dy / 2.0));
  a.fX = d->c_gradx * (h->dy / 2.0);
  a.fY = d->c_grady * (h->dx / 2.0);
  a.P = h->P;
  a.nex = h->nex;
  a.ney = h->ney;
  a.NY = static_cast<int>(h->NY);
  a.NX = static_cast<int>(h->NX);
  a.nc = nc;
  a.c0 = c0;
  a.c1 = c1;
  a.eb = h->ex_begin;
  a.ee = h->ex_end;
  a.lb0 = static_cast<int>(h->line_begin);
  a.lb1 = static_cast<int>(h->line_end);
  a.AII = AII;
  a.D = D;
  a.aIB = aIB;
  a.aBI = aBI;
  a.E = E;
  a.F = F;
  if (cond) {
    a.AII = nullptr;
    a.Aii = cond[0];
    a.Aie = cond[1];
    a.Aei = cond[2];
    a.Aed = cond[3];
    a.Aeu = cond[4];
    a.Ael = cond[5];
  }
  const int64_t rows = (h->line_end - h->line_begin + 1) * nc * h->NY;
  hipLaunchKernelGGL(sem::velocity_blocks_kernel, dim3(static_cast<unsigned>((rows + 255) / 256)), dim3(256), 0, s, a);
  return sem::hip_check_v(hipGetLastError(), "velocity blocks launch");
}

int sem_velocity_blocks(sem_handle* h, const sem_velocity_desc* d, double* AII, double* D, double* aIB, double* aBI,
                        double* E, double* F, void* stream) {
  return velocity_blocks_impl(h, d, AII, nullptr, D, aIB, aBI, E, F, stream);
}

int sem_condensed_blocks(sem_handle* h, const sem_velocity_desc* d, double* Aii, double* Aie, double* Aei,
                         double* Aed, double* Aeu, double* Ael, double* D, double* aIB, double* aBI, double* E,
                         double* F, void* stream) {
  if (h && h->P < 2) return sem::set_error(SEM_EINVAL, "the condensed layout needs P >= 2");
  double* cond[6] = {Aii, Aie, Aei, Aed, Aeu, Ael};
  return velocity_blocks_impl(h, d, nullptr, cond, D, aIB, aBI, E, F, stream);
}

}  // extern "C"
