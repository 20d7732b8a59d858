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
// One thread per node (x-major numbering, SEM.py:110), every operator in its tensor-product form with the
// 1-D direct-stiffness sums of the GLL tables (the algebra of the apply kernels and of
// ns_velocity.hip).  On an element-column strip handle (multi-GPU partition) the x-direction sums run
// over the strip's own element columns, so the two interface lines carry partial sums that the
// interface exchange adds up; pointwise terms, Dirichlet rows and the pinned-pressure row of the
// right interface line are left to its right-hand owner (the rule of the apply kernels), so the
// exchanged sum is the whole-mesh row.  The operands are read through L1/L2 (each value is reused by the 2P+1 threads whose
// windows cover it); the launch is latency-bound at the Navier-Stokes sizes (N <= 10^6), where replacing
// the 7 sem_apply launches of each output set is the point.
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

// K_s / G_s sums of one 1-D direction: global node g (element e = g / P, local index i) of a direction
// whose held elements are [e_lo, e_hi); x[k * stride] is held 1-D node k + off of the line through the
// thread's node (off = the first held line).
__device__ __forceinline__ void dir_sums(const double* __restrict__ x, int64_t stride, int g, int off, int P,
                                         int e_lo, int e_hi, const double* Ks, const double* Gs, double& k,
                                         double& gr) {
  const int n = P + 1, e = g / P, i = g - e * P;
  k = 0.0;
  gr = 0.0;
  if (i != 0) {
    const double* xb = x + static_cast<int64_t>(e * P - off) * stride;
    for (int q = 0; q <= P; ++q) {
      const double t = xb[q * stride];
      k = fma(Ks[i * n + q], t, k);
      gr = fma(Gs[i * n + q], t, gr);
    }
    return;
  }
  if (e > e_lo) {  // row P of the element on the left
    const double* xb = x + static_cast<int64_t>((e - 1) * P - off) * stride;
    for (int q = 0; q <= P; ++q) {
      const double t = xb[q * stride];
      k = fma(Ks[P * n + q], t, k);
      gr = fma(Gs[P * n + q], t, gr);
    }
  }
  if (e < e_hi) {  // row 0 of the element on the right
    const double* xb = x + static_cast<int64_t>(e * P - off) * stride;
    for (int q = 0; q <= P; ++q) {
      const double t = xb[q * stride];
      k = fma(Ks[q], t, k);
      gr = fma(Gs[q], t, gr);
    }
  }
}

__device__ __forceinline__ double wsum1(int g, int P, int e_lo, int e_hi, const double* w) {
  const int e = g / P, i = g - e * P;
  return i != 0 ? w[i] : (e > e_lo ? w[P] : 0.0) + (e < e_hi ? w[0] : 0.0);
}

__global__ __launch_bounds__(256) void ns_apply_kernel(const NsArgs a) {
  extern __shared__ double tab[];
  const int P = a.P, n = P + 1, ntab = 2 * n * n + n;
  for (int i = threadIdx.x; i < ntab; i += blockDim.x) tab[i] = a.tab[i];
  __syncthreads();
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= a.n_local) return;
  const int lx = static_cast<int>(t / a.NY), gy = static_cast<int>(t - static_cast<int64_t>(lx) * a.NY);
  const int gx = a.lb0 + lx;                              // global line
  const double* Ks = tab;
  const double* Gs = tab + n * n;
  const double* w = tab + 2 * n * n;
  const double mx = wsum1(gx, P, a.ex_begin, a.ex_end, w), my = wsum1(gy, P, 0, a.ney, w);
  const int64_t q = t;                                    // node in the plain (local) vectors
  const int64_t qv = static_cast<int64_t>(lx) * a.pitch + gy;  // node in u, v, ru, rv
  // the right interface line of a strip is owned by the strip on its right
  const bool own = !(gx == a.lb1 && a.ex_end < a.nex);
  const bool dir = a.mask ? a.mask[q] != 0
                          : (((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NX - 1) ||
                             ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == a.NY - 1));
  const bool want_uv = a.ru || a.rv;
  // x-direction lines run across lines (stride pitch / NY), y-direction along a line (stride 1)
  double kxu = 0, gxu = 0, kyu = 0, gyu = 0, kxv = 0, gxv = 0, kyv = 0, gyv = 0, kxp = 0, gxp = 0, kyp = 0, gyp = 0;
  const double u0 = a.u ? a.u[qv] : 0.0, v0 = a.v ? a.v[qv] : 0.0;
  const int eb = a.ex_begin, ee = a.ex_end, lb = a.lb0;
  if (a.u && ((want_uv && !dir) || a.rc)) {
    dir_sums(a.u + gy, a.pitch, gx, lb, P, eb, ee, Ks, Gs, kxu, gxu);
    dir_sums(a.u + static_cast<int64_t>(lx) * a.pitch, 1, gy, 0, P, 0, a.ney, Ks, Gs, kyu, gyu);
  }
  if (a.v && ((want_uv && !dir) || a.rc)) {
    dir_sums(a.v + gy, a.pitch, gx, lb, P, eb, ee, Ks, Gs, kxv, gxv);
    dir_sums(a.v + static_cast<int64_t>(lx) * a.pitch, 1, gy, 0, P, 0, a.ney, Ks, Gs, kyv, gyv);
  }
  if (a.p) {
    dir_sums(a.p + gy, a.NY, gx, lb, P, eb, ee, Ks, Gs, kxp, gxp);
    dir_sums(a.p + static_cast<int64_t>(lx) * a.NY, 1, gy, 0, P, 0, a.ney, Ks, Gs, kyp, gyp);
  }
  if (want_uv) {
    if (dir) {
      if (a.ru) a.ru[qv] = own ? u0 - (a.gu ? a.gu[q] : 0.0) : 0.0;
      if (a.rv) a.rv[qv] = own ? v0 - (a.gv ? a.gv[q] : 0.0) : 0.0;
    } else {
      const double cu = a.cu ? a.cu[q] : 1.0, cv = a.cv ? a.cv[q] : 1.0;
      const double fx = a.fKx * my, fy = a.fKy * mx, fm = a.fM * mx * my;
      const double gxc = a.fX * cu * my, gyc = a.fY * cv * mx;
      if (a.ru) {
        double z = fx * kxu + gxc * gxu + fy * kyu + gyc * gyu + fm * u0;
        if (a.juu && own) z = fma(a.juu[q], u0, z);
        if (a.juv && own) z = fma(a.juv[q], v0, z);
        a.ru[qv] = fma(a.hy * my, gxp, z);
      }
      if (a.rv) {
        double z = fx * kxv + gxc * gxv + fy * kyv + gyc * gyv + fm * v0;
        if (a.jvu && own) z = fma(a.jvu[q], u0, z);
        if (a.jvv && own) z = fma(a.jvv[q], v0, z);
        z = fma(a.hx * mx, gyp, z);
        if (a.T) z = fma(a.fT * mx * my, a.T[q], z);
        a.rv[qv] = z;
      }
    }
  }
  if (a.rc) {
    const bool pinned = static_cast<int64_t>(gx) * a.NY + gy == a.pin;
    const double pinrow = own ? (a.p ? a.p[q] : 0.0) - a.pin_val : 0.0;
    double z;
    if (pinned && !a.pin_first)
      z = pinrow;
    else if (dir)
      z = a.sx * my * kxp + a.sy * mx * kyp;  // (K p) row
    else if (pinned)
      z = pinrow;
    else
      z = a.c_div * (a.hy * my * gxu + a.hx * mx * gyv);
    a.rc[q] = z;
  }
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
  const int n = h->P + 1;
  const size_t lds = (2 * n * n + n) * sizeof(double);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sem::ns_apply_kernel, dim3(static_cast<unsigned>((h->n_local + 255) / 256)), dim3(256), lds, s,
                     a);
  return sem::hip_check_ns(hipGetLastError(), "ns apply launch");
}

}  // extern "C"
