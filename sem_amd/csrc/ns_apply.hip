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
  switch (h->P) {
#define SEM_NSCASE(PP)                                                        \
  case PP:                                                                    \
    if (form == (sem::NS_P | sem::NS_UV_OUT))                                 \
      sem::launch_ns_tile<PP, sem::NS_P | sem::NS_UV_OUT>(a, s);              \
    else if (form == (sem::NS_U | sem::NS_P | sem::NS_C_OUT))                 \
      sem::launch_ns_tile<PP, sem::NS_U | sem::NS_P | sem::NS_C_OUT>(a, s);   \
    else                                                                      \
      sem::launch_ns_tile<PP, sem::NS_ALL>(a, s);                             \
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
