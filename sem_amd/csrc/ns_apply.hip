// Fused Navier-Stokes residual / residual-differential apply: all three outputs of the reference's
// _get_residuals (NavierStokes_Solver.py:93-121) or _get_dresiduals (:138-160) in one launch.
//
//   Sys   = cM M + cK K + cX diag(cu) G_x + cY diag(cv) G_y            (:103-106, Re folded into cX, cY)
//   ru    = Sys u + diag(juu) u + diag(juv) v + G_x p                   (:109 / :150)
//   rv    = diag(jvu) u + Sys v + diag(jvv) v + G_y p + c_T M T         (:110 / :151,154)
//   rc    = c_div (G_x u + G_y v)                                       (:111 / :152)
// with the reference's row replacements: Dirichlet rows ru = u - g_u, rv = v - g_v (:114-115 / :157-158),
// artificial Neumann rows rc = (K p) on the same rows (:120 / :159), and the pinned-pressure row
// rc = p - g_p (:116 / :160) -- written before the Neumann rows in the residual (so a pin on the
// boundary is overwritten, as the reference's statement order does) and after them in the differential.
//
// Tiled (ns_apply_tile): one workgroup per tile of element nodes stages u, v, p of the tile and its halo
// in LDS with coalesced loads, then forms every owned node's three outputs from LDS (x-major numbering,
// SEM.py:110; every operator in its tensor-product form with the 1-D direct-stiffness sums of the GLL
// tables -- the algebra of the apply kernels and of ns_velocity.hip).  On an element-column strip handle
// (multi-GPU partition) the x-direction sums run over the strip's own element columns, so the two
// interface lines carry partial sums that the interface exchange adds up; pointwise terms, Dirichlet rows
// and the pinned-pressure row of the right interface line are left to its right-hand owner (the rule of
// the apply kernels), so the exchanged sum is the whole-mesh row.
#include <hip/hip_runtime.h>

#include <string>

#include "apply_common.h"
#include "gll_consts.h"
#include "sem_internal.h"

namespace sem {

struct NsArgs {
  const double* tab;  // K_s | G_s | w (handle table)
  const double *u, *v, *p, *T;
  const double *cu, *cv, *juu, *juv, *jvu, *jvv, *gu, *gv;
  const uint8_t* mask;
  double *ru, *rv, *rc;
  double fKx, fKy, fM, fX, fY;  // Sys: cK dy/dx, cK dx/dy, cM dx dy/4, cX dy/2, cY dx/2
  double hy, hx, sx, sy;        // plain G_x / G_y / K factors: dy/2, dx/2, dy/dx, dx/dy
  double fT, c_div, pin_val;    // c_T dx dy/4
  int64_t pitch;                // local node (lx, gy) of u, v, ru, rv at lx * pitch + gy
  int64_t pin;                  // pinned node (global index), -1: none
  int64_t n_local;              // nodes held: lines [lb0, lb1] x NY
  int P, nex, ney, NY, NX, pin_first;
  int ex_begin, ex_end, lb0, lb1;  // element columns / global lines of the strip
  unsigned sides;
};

// One 1-D direction of the operators at one node: calls f(row, q, off) for the node's element row(s) of
// the K_s / G_s tables -- row i of its element (interior index i != 0), or at an element boundary (i == 0)
// row P of the element on the left (if held: e > e_lo) and row 0 of the element on the right (if
// e < e_hi) -- where off is the offset of that element's node q from the node in the staged arrays
// (`stride` steps one node along the direction: the LDS pitch across lines, 1 along a line).
template <int P, class F>
__device__ __forceinline__ void dir_rows(int stride, int e, int i, int e_lo, int e_hi, F&& f) {
  if (i != 0) {
#pragma unroll
    for (int q = 0; q <= P; ++q) f(i, q, (q - i) * stride);
    return;
  }
  if (e > e_lo) {
#pragma unroll
    for (int q = 0; q <= P; ++q) f(P, q, (q - P) * stride);
  }
  if (e < e_hi) {
#pragma unroll
    for (int q = 0; q <= P; ++q) f(0, q, q * stride);
  }
}

__device__ __forceinline__ double wsum1(int g, int P, int e_lo, int e_hi, const double* w) {
  const int e = g / P, i = g - e * P;
  return i != 0 ? w[i] : (e > e_lo ? w[P] : 0.0) + (e < e_hi ? w[0] : 0.0);
}

// Tile shape: TXE element columns x TYE element rows of owned nodes (lines [gx0, gx0 + TXE P), columns
// [gy0, gy0 + TYE P); the closing line / column of the strip belongs to a ghost tile one position past the
// last element).  Staged: the owned block plus the P lines / columns before it (the left / lower
// neighbour element of the tile's first line / column) and the one after it (the closing node of its last
// element).
template <int P>
struct NsTile {
  static constexpr int TXE = 1;
  // ~32 owned columns: measured faster than one 64-wide line per wavefront (tools/nsbench.py, r03:
  // 14.7 vs 19.6 us for the 48^2 residual -- twice the workgroups to fill the chip)
  static constexpr int TYE = (32 / P) > 0 ? 32 / P : 1;
  static constexpr int BX = TXE * P, BY = TYE * P;
  static constexpr int SX = BX + P + 1, SY = BY + P + 1;
  static constexpr int PITCH = SY | 1;  // odd: lanes striding across staged lines hit distinct banks
  static constexpr int THREADS = 256;
  static_assert((3 * SX * PITCH + 2 * (P + 1) * (P + 1) + P + 1) * 8 <= 64 * 1024, "LDS staging above 64 KB");
};

// One workgroup per tile (XCD-aware order: the 8 XCDs take contiguous runs of tiles, so neighbouring
// tiles -- which stage each other's halo -- share an L2).  Phase 1 stages u, v, p of the tile and its halo
// in LDS with loads coalesced along the lines; phase 2 forms every owned node's outputs from LDS only.
// The Sys rows use the assembled 1-D coefficients (cK K + Re c G of the node's row combined before the
// dot product, as the reference's CSR row of Sys = K + Re (diag(u) G_x + diag(v) G_y) holds them).
// Form flags: which operands are present and which outputs are written, fixed at compile time for the
// forms the solvers launch so that a form does none of the sums it does not use (the residual: all; the
// Schur gradient: G p into ru, rv; the Schur divergence: G u + G v, and K p on Dirichlet rows, into rc).
enum : int { NS_U = 1, NS_P = 2, NS_UV_OUT = 4, NS_C_OUT = 8, NS_ALL = 15 };

template <int P, int F>
__global__ __launch_bounds__(256) void ns_apply_tile(const NsArgs a, int tiles_y, int ntiles, int per_xcd) {
  using T = NsTile<P>;
  constexpr int n = P + 1, BX = T::BX, BY = T::BY, SX = T::SX, SY = T::SY, PIT = T::PITCH;
  __shared__ double tab[2 * n * n + n];
  __shared__ double su[SX * PIT], sv[SX * PIT], sp[SX * PIT];
  const int b = blockIdx.x;
  const int tile = (b & 7) * per_xcd + (b >> 3);
  if (tile >= ntiles) return;
  const int tx = tile / tiles_y, ty = tile - tx * tiles_y;
  const int eb = a.ex_begin, ee = a.ex_end, lb0 = a.lb0, lb1 = a.lb1, NY = a.NY;
  const int gx0 = (eb + tx * T::TXE) * P, gy0 = ty * T::TYE * P;
  const int sx0 = gx0 - P, sy0 = gy0 - P;  // staged origin
  for (int i = threadIdx.x; i < 2 * n * n + n; i += T::THREADS) tab[i] = a.tab[i];
  // phase 1: staging (nodes outside the strip / mesh stay unset and are never read)
  const int64_t pitch = a.pitch;
  for (int k = threadIdx.x; k < SX * SY; k += T::THREADS) {
    const int r = k / SY, c = k - r * SY;
    const int gx = sx0 + r, gy = sy0 + c;
    if (gx < lb0 || gx > lb1 || gy < 0 || gy >= NY) continue;
    const int64_t lx = gx - lb0;
    if ((F & NS_U) && a.u) su[r * PIT + c] = a.u[lx * pitch + gy];
    if ((F & NS_U) && a.v) sv[r * PIT + c] = a.v[lx * pitch + gy];
    if ((F & NS_P) && a.p) sp[r * PIT + c] = a.p[lx * NY + gy];
  }
  __syncthreads();
  const double* Ks = tab;
  const double* Gs = tab + n * n;
  const double* w = tab + 2 * n * n;
  constexpr bool out_uv = (F & NS_UV_OUT) != 0, out_c = (F & NS_C_OUT) != 0;
  const bool want_uv = out_uv && (a.ru || a.rv);
  const bool want_c = out_c && a.rc;
  for (int k = threadIdx.x; k < BX * BY; k += T::THREADS) {
    const int ox = k / BY, oy = k - ox * BY;
    const int gx = gx0 + ox, gy = gy0 + oy;
    if (gx > lb1 || gy >= NY) continue;
    const int ex = gx / P, ix = gx - ex * P, ey = gy / P, iy = gy - ey * P;
    const double mx = wsum1(gx, P, eb, ee, w), my = wsum1(gy, P, 0, a.ney, w);
    const int64_t q = static_cast<int64_t>(gx - lb0) * NY + gy;   // node in the plain (local) vectors
    const int64_t qv = static_cast<int64_t>(gx - lb0) * pitch + gy;  // node in u, v, ru, rv
    const int sidx = (ox + P) * PIT + (oy + P);                    // node in the staged arrays
    const bool own = !(gx == lb1 && ee < a.nex);  // the right interface line of a strip: its right owner's
    const bool dir = a.mask ? a.mask[q] != 0
                            : (((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NX - 1) ||
                               ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == NY - 1));
    const bool hu = (F & NS_U) && a.u != nullptr, hv = (F & NS_U) && a.v != nullptr;
    const bool hp = (F & NS_P) && a.p != nullptr;
    const double u0 = hu ? su[sidx] : 0.0, v0 = hv ? sv[sidx] : 0.0;
    // one pass per direction over the node's element row(s): every operand value and table entry is read
    // from LDS once and feeds all the sums that use it (Sys u, Sys v; G p; G u, G v; K p)
    const double cu = a.cu ? a.cu[q] : 1.0, cv = a.cv ? a.cv[q] : 1.0;
    const double fx = a.fKx * my, gxc = a.fX * cu * my;  // x rows of Sys: fx K + gxc G
    const double fy = a.fKy * mx, gyc = a.fY * cv * mx;  // y rows of Sys: fy K + gyc G
    double Su = 0.0, Sv = 0.0, gxu = 0.0, gyv = 0.0, gxp = 0.0, gyp = 0.0, kxp = 0.0, kyp = 0.0;
    const bool sys = want_uv && (hu || hv);
    const bool kp = want_c && hp && dir;  // K p: the artificial Neumann rows only
    dir_rows<P>(PIT, ex, ix, eb, ee, [&](int row, int c, int off) {
      const double K = Ks[row * n + c], G = Gs[row * n + c];
      const double co = sys ? fma(gxc, G, fx * K) : 0.0;
      if (hu) {
        const double uq = su[sidx + off];
        if (sys) Su = fma(co, uq, Su);
        if (want_c) gxu = fma(G, uq, gxu);
      }
      if (hv && sys) Sv = fma(co, sv[sidx + off], Sv);
      if (hp && (want_uv || kp)) {
        const double pq = sp[sidx + off];
        if (want_uv) gxp = fma(G, pq, gxp);
        if (kp) kxp = fma(K, pq, kxp);
      }
    });
    dir_rows<P>(1, ey, iy, 0, a.ney, [&](int row, int c, int off) {
      const double K = Ks[row * n + c], G = Gs[row * n + c];
      const double co = sys ? fma(gyc, G, fy * K) : 0.0;
      if (hu && sys) Su = fma(co, su[sidx + off], Su);
      if (hv) {
        const double vq = sv[sidx + off];
        if (sys) Sv = fma(co, vq, Sv);
        if (want_c) gyv = fma(G, vq, gyv);
      }
      if (hp && (want_uv || kp)) {
        const double pq = sp[sidx + off];
        if (want_uv) gyp = fma(G, pq, gyp);
        if (kp) kyp = fma(K, pq, kyp);
      }
    });
    if (want_uv) {
      if (dir) {
        if (a.ru) a.ru[qv] = own ? u0 - (a.gu ? a.gu[q] : 0.0) : 0.0;
        if (a.rv) a.rv[qv] = own ? v0 - (a.gv ? a.gv[q] : 0.0) : 0.0;
      } else {
        const double fm = a.fM * mx * my;
        if (a.ru) {
          double z = fma(fm, u0, Su);
          if (a.juu && own) z = fma(a.juu[q], u0, z);
          if (a.juv && own) z = fma(a.juv[q], v0, z);
          a.ru[qv] = fma(a.hy * my, gxp, z);
        }
        if (a.rv) {
          double z = fma(fm, v0, Sv);
          if (a.jvu && own) z = fma(a.jvu[q], u0, z);
          if (a.jvv && own) z = fma(a.jvv[q], v0, z);
          z = fma(a.hx * mx, gyp, z);
          if (a.T) z = fma(a.fT * mx * my, a.T[q], z);
          a.rv[qv] = z;
        }
      }
    }
    if (want_c) {
      const bool pinned = static_cast<int64_t>(gx) * NY + gy == a.pin;
      const double pinrow = own ? (hp ? sp[sidx] : 0.0) - a.pin_val : 0.0;
      double z;
      if (pinned && !a.pin_first)
        z = pinrow;
      else if (dir)  // the (K p) row
        z = a.sx * my * kxp + a.sy * mx * kyp;
      else if (pinned)
        z = pinrow;
      else
        z = a.c_div * (a.hy * my * gxu + a.hx * mx * gyv);
      a.rc[q] = z;
    }
  }
}

// ---- Band form (round 3, the default): the assembled 1-D rows of the operators with compile-time
// coefficients, every lane on a wave-uniform row (the structure of apply_band.hip's band kernel).
//
// Tile = one element-column position (P lines; the closing line of the strip is a ghost position of one
// line) x TYE element rows (BY = TYE P <= 64 columns; the closing column is a ghost position of one
// column).  Staged in LDS: u, v, p over lines gx0-P .. gx0+P and columns gy0-P .. gy0+BY (absent nodes 0),
// and cv of the owned block when the Sys rows need it and cv is not v itself (CVS).  4 waves; wave w takes
// the element rows w, w+4, ... in both directions:
//   Y   lane = (line r, element b): the y-direction rows of element b on line r (Sys u, Sys v + G_y p, and
//       G_y v or K p for the continuity row) -> registers; wave 3 (the fewest y rows) also forms the x rows
//       of the tile's first line over the LEFT element (the only use of the P halo lines gx0-P .. gx0-1)
//   --- barrier: the halo lines are dead; the Y sums and the left-element sums go to LDS over them
//   X   lane = column c: the x-direction rows of its column onto the Y sums, then the node's pointwise
//       terms, the row replacements and the (coalesced) stores.
// Every coefficient is an immediate; each staged value of the element is read from LDS once per window;
// no lane waits on another lane's row type (row 0 -- the shared node -- is a whole wave's row).  Reusing
// the halo lines for the Y sums keeps the LDS to the staged window, 3 workgroups per CU at P = 12.
template <int P>
struct NsBand {
  static constexpr int n = P + 1;
  static constexpr int NW = 4, THREADS = 64 * NW;
  static constexpr int TYE = 64 / P > 0 ? 64 / P : 1;
  static constexpr int BY = TYE * P;          // owned columns of a full tile
  static constexpr int SX = 2 * P + 1;        // staged lines gx0-P .. gx0+P
  static constexpr int SY = BY + P + 1;       // staged columns gy0-P .. gy0+BY
  static constexpr int PIT = SY | 1;          // odd pitch
  static constexpr int FLD = SX * PIT;        // one staged field
  static constexpr int NST = (SX * SY + THREADS - 1) / THREADS;   // staging loads per thread and field
  static constexpr int NCV = (P * BY + THREADS - 1) / THREADS;    // cv staging loads per thread
  static constexpr int XLW = 3;               // the wave with the fewest y rows (rows 3, 7, ...)
  // Y-phase lane -> (line r, element b): line fastest where that makes the staged-window reads
  // ((P + r) PIT + b P + q, ds_read_b64 in two 32-lane groups) and the Y-sum stores (r PIT + b P + j,
  // ds_write_b64 in four 16-lane groups) bank-conflict free (P = 4, 8, 12, 16 exactly; counted per order
  // with the LDS banking of MI355X_MICROARCH.md); element fastest for the orders where it conflicts less.
  static constexpr bool RF = !(P == 3 || P == 6 || P == 7 || P == 10);
  // pitch of the staged cv lines: the staged fields' PIT, so the Y phase's cv reads r SCP + b P + j have the
  // bank pattern of its window reads (P + r) PIT + b P + q, conflict-free for the RF orders (round 4: BY | 1
  // made them 2-way at P = 12, ~80 k of the 108 k conflict cycles per cfg5 Jacobian launch,
  // profiles/r03/ns_lds/pmc_ns128_kernarg_reload.txt)
  static constexpr int SCP = PIT;
  static __device__ __forceinline__ int yline(int lane) { return RF ? lane % P : lane / TYE; }
  static __device__ __forceinline__ int yelem(int lane) { return RF ? lane / P : lane % TYE; }
  static constexpr int rows(int w) { return w < P ? (P - 1 - w) / NW + 1 : 0; }
};

// GLL weight w_J of order P for a runtime J (compile-time constants, no memory access)
template <int P>
__device__ __forceinline__ double ns_gll_w(int J) {
  double r = 0.0;
  for_rows(std::make_integer_sequence<int, P + 1>{}, [&](auto K) {
    constexpr int k = decltype(K)::value;
    if (J == k) r = GllConst<P>::w[k];
  });
  return r;
}

template <int B, int E, int S, class Fn>
__device__ __forceinline__ void ns_sfor(Fn&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    ns_sfor<B + S, E, S>(f);
  }
}

// Which sums a form needs (compile time): the staged fields and the Y / left-element sum arrays.
template <int F>
struct NsForm {
  static constexpr bool HU = (F & NS_U) != 0, HP = (F & NS_P) != 0;
  static constexpr bool OUV = (F & NS_UV_OUT) != 0, OC = (F & NS_C_OUT) != 0;
  static constexpr bool SYS = HU && OUV;
  static constexpr int NF = (HU ? 2 : 0) + (HP ? 1 : 0);               // staged fields u, v | p
  static constexpr int IU = 0, IV = 1, IP = HU ? 2 : 0;                // their order in the staging
  static constexpr int YU = 0, YV = SYS ? 1 : 0, YC = (SYS ? 1 : 0) + (OUV ? 1 : 0);  // Y sums
  static constexpr int NY = YC + (OC ? 1 : 0);
  static constexpr int NXL = (SYS ? 2 : 0) + (HP && OUV ? 1 : 0) + (HU && OC ? 1 : 0) + (HP && OC ? 1 : 0);
  static constexpr int LU = 0, LV = 1, LGP = SYS ? 2 : 0, LGU = LGP + (HP && OUV ? 1 : 0), LKP = LGU + (HU && OC ? 1 : 0);
  static_assert(NY <= NF, "the Y sums live in the staged fields' halo lines");
};

struct NsTileCtx {
  int gx0, gy0, n0, nlx, ncy;  // first line / column, first element row, lines, columns of the tile
  bool hasLx, hasRx;           // the tile's element column has a left neighbour / is not the ghost
};

__device__ __forceinline__ bool ns_dir(const NsArgs& a, int64_t q, int gx, int gy) {
  return a.mask ? a.mask[q] != 0
                : (((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NX - 1) ||
                   ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == a.NY - 1));
}

// Kernel arguments re-read at the point of use.  Taken from the kernel argument `a` by value, the
// ~50 SGPRs of output / operand pointers and factors the epilogue needs are loaded once at kernel entry
// and stay live through every unrolled row; with the fp64 coefficients' SGPR pairs on top, the residual
// forms spilled 35-52 SGPRs into VGPR lanes and paid one v_readlane_b32 (a VALU instruction) per
// reload: ~3,500 readlanes against ~2,600 fp64 FMAs in the P = 12 residual kernel's code.  Read through
// a laundered kernarg-segment pointer instead, each row's fields are fresh scalar loads (s_load through
// the constant cache) whose SGPRs die with the row.  `a` is the kernel's first argument: offset 0.
using NsKArgs = const __attribute__((address_space(4))) NsArgs;
// LAUNDER = false leaves the loads to the compiler (hoisted, as for a by-value argument): the forms without the
// Sys sums (Schur gradient / divergence) never spilled, and per-row reloads cost them 3-10 %.
template <bool LAUNDER>
__device__ __forceinline__ NsKArgs* ns_kargs() {
  auto p = (NsKArgs*)(__builtin_amdgcn_kernarg_segment_ptr());  // C cast: the builtin returns __constant__ void*
  if constexpr (LAUNDER) asm volatile("" : "+s"(p));
  return p;
}

__device__ __forceinline__ bool ns_dir_k(NsKArgs* a, int64_t q, int gx, int gy) {
  return a->mask ? a->mask[q] != 0
                : (((a->sides & SEM_SIDE_W) && gx == 0) || ((a->sides & SEM_SIDE_E) && gx == a->NX - 1) ||
                   ((a->sides & SEM_SIDE_S) && gy == 0) || ((a->sides & SEM_SIDE_N) && gy == a->NY - 1));
}

// One term of a row: the Sys coefficient of the row formed from the 1-D K and G entries (cK K + Re c G, as
// the reference's CSR row holds it) and every sum that uses the operand values.
template <int F>
struct NsAcc {
  double su = 0.0, sv = 0.0, gp = 0.0, gw = 0.0, kp = 0.0;  // Sys u, Sys v, G p, G (u | v), K p
  // d: the divergence operand of the direction (u along x, v along y)
  __device__ __forceinline__ void term(double K, double Gc, double f, double gc, double u, double v, double p,
                                       double d) {
    using M = NsForm<F>;
    if constexpr (M::SYS) {
      const double co = fma(gc, Gc, f * K);
      su = fma(co, u, su);
      sv = fma(co, v, sv);
    }
    if constexpr (M::HU && M::OC) gw = fma(Gc, d, gw);
    if constexpr (M::HP && M::OUV) gp = fma(Gc, p, gp);
    if constexpr (M::HP && M::OC) kp = fma(K, p, kp);
  }
};

template <int P, int F, bool CVS>
__global__ __launch_bounds__(256) void ns_apply_band(const NsArgs a, int tiles_y, int ntiles, int per_xcd, int ubytes,
                                                    int pbytes) {
  using C = NsBand<P>;
  using M = NsForm<F>;
  // per-row kernel-argument reads (ns_kargs) for the residual form (Sys sums, cv = v: 52 SGPR spills and
  // ~3,500 readlanes without them; VALU instructions per launch 22.7 M -> 13.5 M, 72 -> 63 us at cfg5); the
  // Jacobian form (staged cv) measured 3 % slower with them and the Schur forms never spilled: they keep `a`
  constexpr bool KR = M::SYS && !CVS;
#define NSA(f) (KR ? A->f : a.f)
#define NSDIR(...) (KR ? ns_dir_k(A, __VA_ARGS__) : ns_dir(a, __VA_ARGS__))
  constexpr int n = P + 1, BY = C::BY, SX = C::SX, SY = C::SY, PIT = C::PIT, FLD = C::FLD;
  __shared__ double ws[n];
  __shared__ double stg[M::NF * FLD];
  __shared__ double scv[CVS ? P * C::SCP : 1];
  __shared__ double xl[M::NXL > 0 ? M::NXL * 64 : 1];
  double* const su = stg + M::IU * FLD;
  double* const sv = stg + M::IV * FLD;
  double* const sp = stg + M::IP * FLD;
  const int bid = blockIdx.x;
  const int tile = (bid & 7) * per_xcd + (bid >> 3);
  if (tile >= ntiles) return;
  const int tx = tile / tiles_y, ty = tile - tx * tiles_y;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  NsTileCtx t;
  t.gx0 = (a.ex_begin + tx) * P;
  t.n0 = ty * C::TYE;
  t.gy0 = t.n0 * P;
  t.hasLx = tx > 0;
  t.hasRx = a.ex_begin + tx < a.ex_end;
  t.nlx = t.hasRx ? P : 1;
  t.ncy = min(BY, a.NY - t.gy0);
  const int NY = a.NY;

  // ---- staging: every load issued before the first LDS write (buffer loads outside [0, bytes) read 0;
  // columns outside the mesh would wrap into neighbouring lines and are zeroed explicitly)
  const int64_t pitch = a.pitch;
  const auto ru_ = brsrc(M::HU ? a.u : nullptr, M::HU && a.u ? ubytes : 0);
  const auto rv_ = brsrc(M::HU ? a.v : nullptr, M::HU && a.v ? ubytes : 0);
  const auto rp_ = brsrc(M::HP ? a.p : nullptr, M::HP && a.p ? pbytes : 0);
  double st_u[C::NST], st_v[C::NST], st_p[C::NST];
#pragma unroll
  for (int s = 0; s < C::NST; ++s) {
    const int k = min(tid + s * C::THREADS, SX * SY - 1);
    const int r = k / SY, cc = k - r * SY;
    const int gx = t.gx0 - P + r, gy = t.gy0 - P + cc;
    const bool ok = gx >= a.lb0 && gx <= a.lb1;
    const int64_t lx = gx - a.lb0;
    if constexpr (M::HU) {
      const int off = ok ? static_cast<int>((lx * pitch + gy) * 8) : -8;
      st_u[s] = bload(ru_, off);
      st_v[s] = bload(rv_, off);
    }
    if constexpr (M::HP) st_p[s] = bload(rp_, ok ? static_cast<int>((lx * NY + gy) * 8) : -8);
  }
  double st_c[CVS ? C::NCV : 1];
  if constexpr (CVS) {
#pragma unroll
    for (int s = 0; s < C::NCV; ++s) {
      const int k = tid + s * C::THREADS;
      const int r = k / BY, cc = k - r * BY;
      st_c[s] = (k < P * BY && r < t.nlx && cc < t.ncy)
                    ? a.cv[static_cast<int64_t>(t.gx0 + r - a.lb0) * NY + t.gy0 + cc]
                    : 0.0;
    }
  }
  if (tid < n) ws[tid] = ns_gll_w<P>(tid);
#pragma unroll
  for (int s = 0; s < C::NST; ++s) {
    const int k = tid + s * C::THREADS;
    if (k < SX * SY) {
      const int r = k / SY, cc = k - r * SY;
      const int gy = t.gy0 - P + cc;
      const bool inside = gy >= 0 && gy < NY;
      if constexpr (M::HU) {
        su[r * PIT + cc] = inside ? st_u[s] : 0.0;
        sv[r * PIT + cc] = inside ? st_v[s] : 0.0;
      }
      if constexpr (M::HP) sp[r * PIT + cc] = inside ? st_p[s] : 0.0;
    }
  }
  if constexpr (CVS) {
#pragma unroll
    for (int s = 0; s < C::NCV; ++s) {
      const int k = tid + s * C::THREADS;
      if (k < P * BY) scv[(k / BY) * C::SCP + k % BY] = st_c[s];
    }
  }
  __syncthreads();

  // ---- Y phase (+ the left-element x rows of line gx0 on wave XLW): sums in registers
  double yres[(P + C::NW - 1) / C::NW][M::NY > 0 ? M::NY : 1];
  double xlres[M::NXL > 0 ? M::NXL : 1];
  auto y_phase = [&](auto WW) {
    constexpr int W = decltype(WW)::value;
    if constexpr (C::rows(W) > 0) {
      if (lane >= P * C::TYE) return;
      const int r = C::yline(lane), b = C::yelem(lane);
      const int pos = t.n0 + b;
      if (r >= t.nlx || pos > a.ney) return;
      const bool ghost = pos == a.ney, hasL = pos > 0;
      const int gx = t.gx0 + r;
      const double mx = wsum1(gx, P, a.ex_begin, a.ex_end, ws);
      const int base = (P + r) * PIT + b * P;  // staged column b P + q <-> gy = gy0 + b P - P + q
      double tu[n], tv[n], tp[n];              // the element's own nodes (q = P .. 2P)
#pragma unroll
      for (int k = 0; k < n; ++k) {
        if constexpr (M::HU) {
          tu[k] = su[base + P + k];
          tv[k] = sv[base + P + k];
        }
        if constexpr (M::HP) tp[k] = sp[base + P + k];
      }
      const double fy = a.fKy * mx, hxm = a.hx * mx, sym = a.sy * mx;
      ns_sfor<W, P, C::NW>([&](auto J) {
        constexpr int j = decltype(J)::value, slot = (j - W) / C::NW;
        if (ghost && j != 0) return;  // the ghost position holds its row 0 only
        const int c = b * P + j;      // tile column of the node
        double gyc = 0.0;
        if constexpr (M::SYS) {
          const double cvn = CVS ? scv[r * C::SCP + c] : (a.cv ? tv[j] : 1.0);  // !CVS: cv is v itself or absent
          gyc = a.fY * cvn * mx;
        }
        NsAcc<F> acc;
        if constexpr (j == 0) {
          if (hasL) ns_sfor<0, n, 1>([&](auto Q) {
              constexpr int q = decltype(Q)::value;
              const double uq = M::HU ? (q == P ? tu[0] : su[base + q]) : 0.0;
              const double vq = M::HU ? (q == P ? tv[0] : sv[base + q]) : 0.0;
              const double pq = M::HP ? (q == P ? tp[0] : sp[base + q]) : 0.0;
              acc.term(GllConst<P>::K[P * n + q], GllConst<P>::G[P * n + q], fy, gyc, uq, vq, pq, vq);
            });
          if (!ghost) ns_sfor<0, n, 1>([&](auto Q) {
              constexpr int q = decltype(Q)::value;
              acc.term(GllConst<P>::K[q], GllConst<P>::G[q], fy, gyc, M::HU ? tu[q] : 0.0, M::HU ? tv[q] : 0.0, M::HP ? tp[q] : 0.0,
                       M::HU ? tv[q] : 0.0);
            });
        } else {
          ns_sfor<0, n, 1>([&](auto Q) {
            constexpr int q = decltype(Q)::value;
            acc.term(GllConst<P>::K[j * n + q], GllConst<P>::G[j * n + q], fy, gyc, M::HU ? tu[q] : 0.0, M::HU ? tv[q] : 0.0,
                     M::HP ? tp[q] : 0.0, M::HU ? tv[q] : 0.0);
          });
        }
        if constexpr (M::SYS) yres[slot][M::YU] = acc.su;
        if constexpr (M::OUV) yres[slot][M::YV] = M::SYS ? fma(hxm, acc.gp, acc.sv) : hxm * acc.gp;
        if constexpr (M::OC) {
          const int gy = t.gy0 + c;
          NsKArgs* const A = ns_kargs<KR>();  // unused (no load) unless KR
          const bool dir = NSDIR(static_cast<int64_t>(gx - NSA(lb0)) * NY + gy, gx, gy);
          yres[slot][M::YC] = dir ? (M::HP ? sym * acc.kp : 0.0) : (M::HU ? hxm * acc.gw : 0.0);
        }
      });
    }
  };
  switch (w) {
    case 0: y_phase(std::integral_constant<int, 0>{}); break;
    case 1: y_phase(std::integral_constant<int, 1>{}); break;
    case 2: y_phase(std::integral_constant<int, 2>{}); break;
    default: y_phase(std::integral_constant<int, 3>{}); break;
  }
  if (w == C::XLW && t.hasLx && lane < t.ncy) {
    // left-element x rows of line gx0 (row P of element ex_begin + tx - 1) at column `lane`
    const int c = lane, gy = t.gy0 + c;
    const double my = wsum1(gy, P, 0, a.ney, ws);
    const double fx = a.fKx * my;
    double gxc = 0.0;
    if constexpr (M::SYS) {
      const bool cu_is_u = a.cu == a.u;
      const double cun = a.cu ? (cu_is_u ? su[P * PIT + P + c] : a.cu[static_cast<int64_t>(t.gx0 - a.lb0) * NY + gy])
                              : 1.0;
      gxc = a.fX * cun * my;
    }
    NsAcc<F> acc;
    ns_sfor<0, n, 1>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      const int o = q * PIT + P + c;
      acc.term(GllConst<P>::K[P * n + q], GllConst<P>::G[P * n + q], fx, gxc, M::HU ? su[o] : 0.0, M::HU ? sv[o] : 0.0,
               M::HP ? sp[o] : 0.0, M::HU ? su[o] : 0.0);
    });
    if constexpr (M::SYS) {
      xlres[M::LU] = acc.su;
      xlres[M::LV] = acc.sv;
    }
    if constexpr (M::HP && M::OUV) xlres[M::LGP] = acc.gp;
    if constexpr (M::HU && M::OC) xlres[M::LGU] = acc.gw;
    if constexpr (M::HP && M::OC) xlres[M::LKP] = acc.kp;
  }
  __syncthreads();  // the halo lines are dead from here: they take the Y sums

  // ---- Y sums and left-element sums -> LDS (Y sum k over the halo lines of staged field k)
  auto y_store = [&](auto WW) {
    constexpr int W = decltype(WW)::value;
    if constexpr (C::rows(W) > 0 && M::NY > 0) {
      if (lane >= P * C::TYE) return;
      const int r = C::yline(lane), b = C::yelem(lane);
      const int pos = t.n0 + b;
      if (r >= t.nlx || pos > a.ney) return;
      const bool ghost = pos == a.ney;
      ns_sfor<W, P, C::NW>([&](auto J) {
        constexpr int j = decltype(J)::value, slot = (j - W) / C::NW;
        if (ghost && j != 0) return;
#pragma unroll
        for (int k = 0; k < M::NY; ++k) stg[k * FLD + r * PIT + b * P + j] = yres[slot][k];
      });
    }
  };
  switch (w) {
    case 0: y_store(std::integral_constant<int, 0>{}); break;
    case 1: y_store(std::integral_constant<int, 1>{}); break;
    case 2: y_store(std::integral_constant<int, 2>{}); break;
    default: y_store(std::integral_constant<int, 3>{}); break;
  }
  if constexpr (M::NXL > 0) {
    if (w == C::XLW && t.hasLx && lane < t.ncy) {
#pragma unroll
      for (int k = 0; k < M::NXL; ++k) xl[k * 64 + lane] = xlres[k];
    }
  }
  __syncthreads();

  // ---- X phase: lane = column c, rows (lines) w, w+4, ...
  auto x_phase = [&](auto WW) {
    constexpr int W = decltype(WW)::value;
    if constexpr (C::rows(W) > 0) {
      const int c = lane;
      if (c >= t.ncy) return;
      const int gy = t.gy0 + c;
      const double my = wsum1(gy, P, 0, a.ney, ws);
      double tu[n], tv[n], tp[n];  // lines gx0 .. gx0 + P of column c
#pragma unroll
      for (int k = 0; k < n; ++k) {
        const int o = (P + k) * PIT + P + c;
        if constexpr (M::HU) {
          tu[k] = su[o];
          tv[k] = sv[o];
        }
        if constexpr (M::HP) tp[k] = sp[o];
      }
      const bool want_uv = M::OUV && (a.ru || a.rv), want_c = M::OC && a.rc;
      const bool cu_is_u = a.cu == a.u;
      const double fx = a.fKx * my, hym = a.hy * my, sxm = a.sx * my;
      ns_sfor<W, P, C::NW>([&](auto I) {
        constexpr int i = decltype(I)::value, slot = (i - W) / C::NW;
        if (i >= t.nlx) return;  // the ghost position holds its line 0 only
        NsKArgs* const A = ns_kargs<KR>();  // unused (no load) unless KR
        const int gx = t.gx0 + i;
        const int64_t q = static_cast<int64_t>(gx - NSA(lb0)) * NY + gy;
        const int64_t qv = static_cast<int64_t>(gx - NSA(lb0)) * pitch + gy;
        const double mx = wsum1(gx, P, NSA(ex_begin), NSA(ex_end), ws);
        const int o = i * PIT + c;  // Y sums: line pitch PIT (odd)
        double gxc = 0.0;
        if constexpr (M::SYS) {
          const double cun = NSA(cu) ? (cu_is_u ? tu[i] : NSA(cu)[q]) : 1.0;
          gxc = NSA(fX) * cun * my;
        }
        NsAcc<F> acc;
        if constexpr (i == 0) {
          if (t.hasLx) {
            if constexpr (M::SYS) {
              acc.su = xl[M::LU * 64 + c];
              acc.sv = xl[M::LV * 64 + c];
            }
            if constexpr (M::HP && M::OUV) acc.gp = xl[M::LGP * 64 + c];
            if constexpr (M::HU && M::OC) acc.gw = xl[M::LGU * 64 + c];
            if constexpr (M::HP && M::OC) acc.kp = xl[M::LKP * 64 + c];
          }
          if (t.hasRx) ns_sfor<0, n, 1>([&](auto Q) {
              constexpr int qq = decltype(Q)::value;
              acc.term(GllConst<P>::K[qq], GllConst<P>::G[qq], fx, gxc, M::HU ? tu[qq] : 0.0, M::HU ? tv[qq] : 0.0,
                       M::HP ? tp[qq] : 0.0, M::HU ? tu[qq] : 0.0);
            });
        } else {
          ns_sfor<0, n, 1>([&](auto Q) {
            constexpr int qq = decltype(Q)::value;
            acc.term(GllConst<P>::K[i * n + qq], GllConst<P>::G[i * n + qq], fx, gxc, M::HU ? tu[qq] : 0.0, M::HU ? tv[qq] : 0.0,
                     M::HP ? tp[qq] : 0.0, M::HU ? tu[qq] : 0.0);
          });
        }
        const bool own = !(gx == NSA(lb1) && NSA(ex_end) < NSA(nex));  // a strip's right interface line: its right owner's
        const bool dir = NSDIR(q, gx, gy);
        const double u0 = M::HU ? tu[i] : 0.0, v0 = M::HU ? tv[i] : 0.0;
        if constexpr (M::OUV) {
          if (want_uv) {
            if (dir) {
              if (NSA(ru)) NSA(ru)[qv] = own ? u0 - (NSA(gu) ? NSA(gu)[q] : 0.0) : 0.0;
              if (NSA(rv)) NSA(rv)[qv] = own ? v0 - (NSA(gv) ? NSA(gv)[q] : 0.0) : 0.0;
            } else {
              const double fm = NSA(fM) * mx * my;
              if (NSA(ru)) {
                double z = fma(fm, u0, M::SYS ? stg[M::YU * FLD + o] + acc.su : 0.0);
                if (NSA(juu) && own) z = fma(NSA(juu)[q], u0, z);
                if (NSA(juv) && own) z = fma(NSA(juv)[q], v0, z);
                NSA(ru)[qv] = fma(hym, acc.gp, z);
              }
              if (NSA(rv)) {
                double z = fma(fm, v0, stg[M::YV * FLD + o] + (M::SYS ? acc.sv : 0.0));
                if (NSA(jvu) && own) z = fma(NSA(jvu)[q], u0, z);
                if (NSA(jvv) && own) z = fma(NSA(jvv)[q], v0, z);
                if (NSA(T)) z = fma(NSA(fT) * mx * my, NSA(T)[q], z);
                NSA(rv)[qv] = z;
              }
            }
          }
        }
        if constexpr (M::OC) {
          if (want_c) {
            const bool pinned = static_cast<int64_t>(gx) * NY + gy == NSA(pin);
            const double pinrow = own ? (M::HP ? tp[i] : 0.0) - NSA(pin_val) : 0.0;
            const double yc = stg[M::YC * FLD + o];
            double z;
            if (pinned && !NSA(pin_first))
              z = pinrow;
            else if (dir)  // the (K p) row
              z = M::HP ? fma(sxm, acc.kp, yc) : 0.0;
            else if (pinned)
              z = pinrow;
            else
              z = M::HU ? NSA(c_div) * fma(hym, acc.gw, yc) : 0.0;
            NSA(rc)[q] = z;
          }
        }
      });
    }
  };
  switch (w) {
    case 0: x_phase(std::integral_constant<int, 0>{}); break;
    case 1: x_phase(std::integral_constant<int, 1>{}); break;
    case 2: x_phase(std::integral_constant<int, 2>{}); break;
    default: x_phase(std::integral_constant<int, 3>{}); break;
  }
#undef NSA
#undef NSDIR
}

template <int P, int F>
static bool launch_ns_band(const NsArgs& a, hipStream_t s) {
  using C = NsBand<P>;
  // buffer-resource offsets are 32-bit: the band form covers strips below 2 GB per operand
  const int64_t nl = a.lb1 - a.lb0;
  const int64_t ub = (nl * a.pitch + a.NY) * 8, pb = (nl * a.NY + a.NY) * 8;
  if (ub >= (int64_t{1} << 31) || pb >= (int64_t{1} << 31)) return false;
  const int ncols = a.ex_end - a.ex_begin;
  const int tiles_x = ncols + 1;  // positions 0..ncols (ncols: the closing line)
  const int tiles_y = (a.ney + C::TYE) / C::TYE;
  const int ntiles = tiles_x * tiles_y;
  const int per_xcd = (ntiles + 7) / 8;
  const dim3 grid(static_cast<unsigned>(8 * per_xcd)), block(C::THREADS);
  // cv staged in LDS when the Sys rows use a cv that is not v itself (the Jacobian forms)
  if (NsForm<F>::SYS && a.cv && a.cv != a.v)
    hipLaunchKernelGGL((ns_apply_band<P, F, NsForm<F>::SYS>), grid, block, 0, s, a, tiles_y, ntiles, per_xcd,
                       static_cast<int>(ub), static_cast<int>(pb));
  else
    hipLaunchKernelGGL((ns_apply_band<P, F, false>), grid, block, 0, s, a, tiles_y, ntiles, per_xcd,
                       static_cast<int>(ub), static_cast<int>(pb));
  return true;
}

template <int P, int F>
static void launch_ns_tile(const NsArgs& a, hipStream_t s) {
  using T = NsTile<P>;
  const int ncols = a.ex_end - a.ex_begin;
  const int tiles_x = (ncols + T::TXE) / T::TXE;  // positions 0..ncols (ncols: the closing line)
  const int tiles_y = (a.ney + T::TYE) / T::TYE;
  const int ntiles = tiles_x * tiles_y;
  const int per_xcd = (ntiles + 7) / 8;
  hipLaunchKernelGGL((ns_apply_tile<P, F>), dim3(static_cast<unsigned>(8 * per_xcd)), dim3(T::THREADS), 0, s, a, tiles_y,
                     ntiles, per_xcd);
}

static int hip_check_ns(hipError_t e, const char* what) {
  if (e == hipSuccess) return SEM_OK;
  return set_error(SEM_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace sem

extern "C" {

int sem_ns_apply(sem_handle* h, const sem_ns_desc* d, const double* u, const double* v, const double* p, double* ru,
                 double* rv, double* rc, void* stream) {
  if (!h || !d) return sem::set_error(SEM_EINVAL, "null argument");
  if (d->uv_pitch != 0 && d->uv_pitch < h->NY) return sem::set_error(SEM_EINVAL, "uv_pitch below the line length");
  if (d->pin < -1 || d->pin >= h->NX * h->NY) return sem::set_error(SEM_EINVAL, "pinned node out of range");
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != h->device)
    return sem::set_error(SEM_EINVAL, "handle belongs to device " + std::to_string(h->device) +
                                          ", but the current device is " + std::to_string(cur));
  if (!ru && !rv && !rc) return SEM_OK;
  sem::NsArgs a{};
  a.tab = h->d_tab;
  a.u = u;
  a.v = v;
  a.p = p;
  a.T = d->T;
  a.cu = d->cu;
  a.cv = d->cv;
  a.juu = d->juu;
  a.juv = d->juv;
  a.jvu = d->jvu;
  a.jvv = d->jvv;
  a.gu = d->dval_u;
  a.gv = d->dval_v;
  a.mask = d->dir_mask;
  a.sides = d->dir_sides;
  a.ru = ru;
  a.rv = rv;
  a.rc = rc;
  const double dx = h->dx, dy = h->dy;
  a.fKx = d->c_stiff * (dy / dx);
  a.fKy = d->c_stiff * (dx / dy);
  a.fM = d->c_mass * ((dx / 2.0) * (dy / 2.0));
  a.fX = d->c_gradx * (dy / 2.0);
  a.fY = d->c_grady * (dx / 2.0);
  a.hy = dy / 2.0;
  a.hx = dx / 2.0;
  a.sx = dy / dx;
  a.sy = dx / dy;
  a.fT = d->c_T * ((dx / 2.0) * (dy / 2.0));
  a.c_div = d->c_div;
  a.pin = d->pin;
  a.pin_val = d->pin_val;
  a.pin_first = d->pin_first;
  a.pitch = d->uv_pitch ? d->uv_pitch : h->NY;
  a.P = h->P;
  a.nex = h->nex;
  a.ney = h->ney;
  a.NY = static_cast<int>(h->NY);
  a.NX = static_cast<int>(h->NX);
  a.ex_begin = h->ex_begin;
  a.ex_end = h->ex_end;
  a.lb0 = static_cast<int>(h->line_begin);
  a.lb1 = static_cast<int>(h->line_end);
  a.n_local = h->n_local;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // the Schur gradient (p in; ru, rv out) and divergence (u, v, p in; rc out) run specialised kernels
  const int form = ((u || v) ? sem::NS_U : 0) | (p ? sem::NS_P : 0) | ((ru || rv) ? sem::NS_UV_OUT : 0) |
                   (rc ? sem::NS_C_OUT : 0);
  // the band form by default; the tile form on request (SEM_NS_APPLY=1, in-process A/B: results agree to
  // rounding, not bitwise) and for strips beyond the band form's 32-bit buffer offsets
  const bool tile = sem::tune(SEM_TUNE_NS_APPLY) == 1;
  switch (h->P) {
#define SEM_NSCASE(PP)                                                                              \
  case PP:                                                                                          \
    if (form == (sem::NS_P | sem::NS_UV_OUT)) {                                                     \
      if (tile || !sem::launch_ns_band<PP, sem::NS_P | sem::NS_UV_OUT>(a, s))                       \
        sem::launch_ns_tile<PP, sem::NS_P | sem::NS_UV_OUT>(a, s);                                  \
    } else if (form == (sem::NS_U | sem::NS_P | sem::NS_C_OUT)) {                                   \
      if (tile || !sem::launch_ns_band<PP, sem::NS_U | sem::NS_P | sem::NS_C_OUT>(a, s))            \
        sem::launch_ns_tile<PP, sem::NS_U | sem::NS_P | sem::NS_C_OUT>(a, s);                       \
    } else {                                                                                        \
      if (tile || !sem::launch_ns_band<PP, sem::NS_ALL>(a, s)) sem::launch_ns_tile<PP, sem::NS_ALL>(a, s); \
    }                                                                                               \
    break;
    SEM_NSCASE(1) SEM_NSCASE(2) SEM_NSCASE(3) SEM_NSCASE(4) SEM_NSCASE(5) SEM_NSCASE(6) SEM_NSCASE(7) SEM_NSCASE(8)
    SEM_NSCASE(9) SEM_NSCASE(10) SEM_NSCASE(11) SEM_NSCASE(12) SEM_NSCASE(13) SEM_NSCASE(14) SEM_NSCASE(15)
    SEM_NSCASE(16)
#undef SEM_NSCASE
    default:
      return sem::set_error(SEM_EUNSUPPORTED, "polynomial order outside compiled range");
  }
  return sem::hip_check_ns(hipGetLastError(), "ns apply launch");
}

}  // extern "C"
