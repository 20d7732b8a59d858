// libsemops: MI355X (gfx950) kernels and C ABI of the SEM operator layer.
//
// Hot path: the assembled global operators of Solvers/SEM.py (mass :170-183,
// stiffness :186-203, gradient :206-223, convection :226-245 contracted as in
// ConvectionDiffusion_Solver.py:82-87,112-119) applied matrix-free.
//
// On a structured N_ex x N_ey mesh every element matrix is a tensor product of
// 1-D reference tables (SEM.py:196-202), so the assembled operator is the
// tensor-product sum
//     K = (dy/dx) Kx (x) My + (dx/dy) Mx (x) Ky,   G_x = (dy/2) Gx (x) My, ...
// where Kx, Gx are the 1-D element tables K_s, G_s summed over the element
// columns holding a line and Mx, My the 1-D assembled GLL weights.  The kernel
// applies exactly that: per line, a K_s / G_s contraction over the (P+1) nodes
// of each element holding it (2P+1 at a shared line), scaled by the summed
// weights of the orthogonal direction.  Direct-stiffness summation is implicit:
// each node is owned by one workgroup, which sums the contributions of every
// element holding it from a halo-extended LDS tile -- one launch, no E-vector,
// no atomics, deterministic.
//
// Work decomposition (one workgroup = one tile of TX x TY elements):
//   stage   : x over lines [gx0-P, gx0+BX] x cols [gy0-P, gy0+BY] -> LDS (coalesced in y)
//   phase B : y-direction contractions, lanes along x-lines, results -> LDS
//   phase A : x-direction contractions, lanes along y (coalesced), + combine,
//             convection / extra / accumulate terms, Dirichlet rows, store.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sem_internal.h"

namespace sem {

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
void clear_error() { g_last_error.clear(); }

static int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return SEM_OK;
  return set_error(SEM_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// --------------------------------------------------------------------------- apply kernel

struct ApplyArgs {
  const double* x;
  double* y;
  const double* cu;
  const double* cv;
  const double* ea;
  const double* eb;
  const double* ec;
  const double* ed;
  const uint8_t* mask;
  const double* dval;
  const double* tab;  // K_s | G_s | w
  double cM, cK, cX, cY, cE, cA;
  double sx, sy, hx, hy, hxy;  // dy/dx, dx/dy, dx/2, dy/2, dx*dy/4
  int64_t NY, NXg, line_begin, line_end;
  int nex, ney, ex_begin, ex_end;
  int tiles_y, dir_mode;
  unsigned sides;
  int has_e1, has_e2;
};

template <int P>
struct TileCfg {
  static constexpr int n = P + 1;
  static constexpr int TX = (16 / P) > 0 ? 16 / P : 1;  // elements per tile in x
  static constexpr int TY = (64 / P) > 0 ? 64 / P : 1;  // elements per tile in y
  static constexpr int BX = TX * P;                    // owned lines (+1 at the last tile)
  static constexpr int BY = TY * P;                    // owned columns (+1 at the last tile)
  static constexpr int RX = BX + P + 1;                // staged lines
  static constexpr int RY = BY + P + 1;                // staged columns
  static constexpr int PT = RY | 1;                    // odd pitch: conflict-free strided reads
  static constexpr int PY = (BY + 1) | 1;
  static constexpr int THREADS = 128;
};

// Sum of GLL weights of the elements in [e_lo, e_hi) that hold 1-D node g.
__device__ __forceinline__ double weight_sum(int64_t g, int P, int e_lo, int e_hi, const double* w) {
  const int64_t e = g / P;
  const int i = static_cast<int>(g - e * P);
  if (i != 0) return w[i];
  double s = 0.0;
  if (e - 1 >= e_lo && e - 1 < e_hi) s += w[P];
  if (e >= e_lo && e < e_hi) s += w[0];
  return s;
}

template <int P>
__global__ __launch_bounds__(TileCfg<P>::THREADS) void apply_tp_valu(const ApplyArgs a) {
  using C = TileCfg<P>;
  constexpr int n = C::n;
  __shared__ double Ts[C::RX * C::PT];
  __shared__ double Yk[(C::BX + 1) * C::PY];
  __shared__ double Yg[(C::BX + 1) * C::PY];
  __shared__ double ws[n];

  // XCD-aware bijective remap: blocks b and b+8 share an XCD, so give each XCD a
  // contiguous run of logical tiles (neighbouring tiles share halo lines in L2).
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q = nb >> 3, rem = nb & 7;
  const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int tx = L / a.tiles_y, ty = L - tx * a.tiles_y;

  const int m0 = a.ex_begin + tx * C::TX;
  const int m1 = min(m0 + C::TX, a.ex_end);
  const int n0 = ty * C::TY;
  const int n1 = min(n0 + C::TY, a.ney);
  const int64_t gx0 = static_cast<int64_t>(m0) * P;
  const int64_t gy0 = static_cast<int64_t>(n0) * P;
  const int BXo = (m1 - m0) * P + (m1 == a.ex_end ? 1 : 0);  // owned lines
  const int BYo = (n1 - n0) * P + (n1 == a.ney ? 1 : 0);     // owned columns
  const int tid = threadIdx.x;

  const double* Ks = a.tab;
  const double* Gs = a.tab + n * n;
  if (tid < n) ws[tid] = a.tab[2 * n * n + tid];

  // ---- stage x tile (zero outside the locally held lines / the domain)
  for (int idx = tid; idx < C::RX * C::RY; idx += C::THREADS) {
    const int rr = idx / C::RY, cc = idx - rr * C::RY;
    const int64_t gx = gx0 - P + rr, gy = gy0 - P + cc;
    double v = 0.0;
    if (gx >= a.line_begin && gx <= a.line_end && gy >= 0 && gy < a.NY) v = a.x[(gx - a.line_begin) * a.NY + gy];
    Ts[rr * C::PT + cc] = v;
  }
  __syncthreads();

  // ---- phase B: y-direction (K_s / G_s along each x-line), lanes along lines
  const int itemsB = (n1 - n0) * BXo;
  for (int it = tid; it < itemsB; it += C::THREADS) {
    const int ae = it / BXo, r = it - ae * BXo;
    const int ne = n0 + ae;
    const int64_t gx = gx0 + r;
    double t[2 * P + 1];
#pragma unroll
    for (int qq = 0; qq <= 2 * P; ++qq) t[qq] = Ts[(r + P) * C::PT + ae * P + qq];
    const double mx = weight_sum(gx, P, a.ex_begin, a.ex_end, ws);
    const double fk = a.sy * mx, fg = a.hx * mx;
    const bool hasL = ne > 0;
    const bool last = ne == a.ney - 1;
#pragma unroll
    for (int j = 0; j <= P; ++j) {
      if (j == P && !last) continue;  // the closing column exists only in the last element row
      double k = 0.0, g = 0.0;
      if (j == 0 && hasL) {
#pragma unroll
        for (int l = 0; l <= P; ++l) {
          k = fma(Ks[P * n + l], t[l], k);
          g = fma(Gs[P * n + l], t[l], g);
        }
      }
#pragma unroll
      for (int l = 0; l <= P; ++l) {
        k = fma(Ks[j * n + l], t[P + l], k);
        g = fma(Gs[j * n + l], t[P + l], g);
      }
      Yk[r * C::PY + ae * P + j] = fk * k;
      Yg[r * C::PY + ae * P + j] = fg * g;
    }
  }
  __syncthreads();

  // ---- phase A: x-direction + combine + epilogue, lanes along columns (coalesced)
  const int itemsA = (m1 - m0) * BYo;
  for (int it = tid; it < itemsA; it += C::THREADS) {
    const int be = it / BYo, c = it - be * BYo;
    const int me = m0 + be;
    const int64_t gy = gy0 + c;
    double t[2 * P + 1];
#pragma unroll
    for (int qq = 0; qq <= 2 * P; ++qq) t[qq] = Ts[(be * P + qq) * C::PT + c + P];
    const double my = weight_sum(gy, P, 0, a.ney, ws);
    const bool hasL = me - 1 >= a.ex_begin;
    const bool last = me == a.ex_end - 1;
#pragma unroll
    for (int i = 0; i <= P; ++i) {
      if (i == P && !last) continue;  // the closing line exists only in the last element column
      double k = 0.0, g = 0.0;
      if (i == 0 && hasL) {
#pragma unroll
        for (int l = 0; l <= P; ++l) {
          k = fma(Ks[P * n + l], t[l], k);
          g = fma(Gs[P * n + l], t[l], g);
        }
      }
#pragma unroll
      for (int l = 0; l <= P; ++l) {
        k = fma(Ks[i * n + l], t[P + l], k);
        g = fma(Gs[i * n + l], t[P + l], g);
      }
      const int rl = be * P + i;  // owned-line index within the tile
      const int64_t gx = gx0 + rl;
      const int64_t p = (gx - a.line_begin) * a.NY + gy;
      const double xv = t[P + i];
      double z = 0.0;
      if (a.cK != 0.0) z = a.cK * fma(a.sx * my, k, Yk[rl * C::PY + c]);
      if (a.cM != 0.0) z = fma(a.cM * a.hxy * weight_sum(gx, P, a.ex_begin, a.ex_end, ws) * my, xv, z);
      if (a.cX != 0.0) z = fma(a.cX * (a.cu ? a.cu[p] : 1.0), a.hy * my * g, z);
      if (a.cY != 0.0) z = fma(a.cY * (a.cv ? a.cv[p] : 1.0), Yg[rl * C::PY + c], z);
      if (a.has_e1) z = fma(a.cE * a.ea[p], a.eb[p], z);
      if (a.has_e2) z = fma(a.cE * a.ec[p], a.ed[p], z);
      if (a.cA != 0.0) z = fma(a.cA, a.y[p], z);
      if (a.dir_mode != SEM_DIR_NONE) {
        const bool isd = a.mask ? (a.mask[p] != 0)
                                : (((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NXg - 1) ||
                                   ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == a.NY - 1));
        if (isd) {
          // an interface line's Dirichlet row is written by its owner (the right strip) only
          const bool owner = !(gx == a.line_end && a.ex_end < a.nex);
          if (!owner)
            z = 0.0;
          else if (a.dir_mode == SEM_DIR_IDENTITY)
            z = xv - (a.dval ? a.dval[p] : 0.0);
          else
            z = a.dval[p];
        }
      }
      a.y[p] = z;
    }
  }
}

template <int P>
static int launch_apply(const ApplyArgs& args_in, const sem_handle* h, hipStream_t s) {
  using C = TileCfg<P>;
  ApplyArgs args = args_in;
  const int ncols = h->ex_end - h->ex_begin;
  const int tiles_x = (ncols + C::TX - 1) / C::TX;
  const int tiles_y = (h->ney + C::TY - 1) / C::TY;
  args.tiles_y = tiles_y;
  const long long nblk = static_cast<long long>(tiles_x) * tiles_y;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return set_error(SEM_EINVAL, "mesh too large for one launch");
  hipLaunchKernelGGL(apply_tp_valu<P>, dim3(static_cast<unsigned>(nblk)), dim3(C::THREADS), 0, s, args);
  return hip_check(hipGetLastError(), "apply launch");
}

// --------------------------------------------------------------------------- gather / DSS

__global__ void gather_kernel(const double* __restrict__ u, double* __restrict__ ue, int P, int ney, int ex_begin,
                              int64_t line_begin, int64_t NY, int64_t total) {
  const int n = P + 1;
  for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int j = static_cast<int>(t % n);
    int64_t r = t / n;
    const int i = static_cast<int>(r % n);
    r /= n;
    const int ne = static_cast<int>(r % ney);
    const int64_t me = r / ney + ex_begin;
    const int64_t gx = me * P + i, gy = static_cast<int64_t>(ne) * P + j;
    ue[t] = u[(gx - line_begin) * NY + gy];
  }
}

__global__ void dss_kernel(const double* __restrict__ ae, double* __restrict__ out, int P, int ney, int ex_begin,
                           int ex_end, int64_t line_begin, int64_t NY, int64_t total) {
  const int n = P + 1;
  for (int64_t p = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; p < total;
       p += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t gx = line_begin + p / NY, gy = p % NY;
    // candidate (element, local index) pairs, in increasing element order
    int64_t mc[2], ic[2], nc[2], jc[2];
    int nm = 0, nn = 0;
    const int64_t mx = gx / P, ix = gx - mx * P;
    if (ix == 0 && mx - 1 >= ex_begin && mx - 1 < ex_end) { mc[nm] = mx - 1; ic[nm++] = P; }
    if (mx >= ex_begin && mx < ex_end) { mc[nm] = mx; ic[nm++] = ix; }
    const int64_t my = gy / P, jy = gy - my * P;
    if (jy == 0 && my - 1 >= 0) { nc[nn] = my - 1; jc[nn++] = P; }
    if (my < ney) { nc[nn] = my; jc[nn++] = jy; }
    double s = 0.0;
    for (int a = 0; a < nm; ++a)
      for (int b = 0; b < nn; ++b)
        s += ae[(((mc[a] - ex_begin) * ney + nc[b]) * n + ic[a]) * n + jc[b]];
    out[p] = s;
  }
}

__global__ void iface_pack_kernel(const double* __restrict__ y, double* __restrict__ buf, int64_t NY, int nslots,
                                  int left_slot, int64_t left_off, int right_slot, int64_t right_off) {
  const int64_t total = static_cast<int64_t>(nslots) * NY;
  for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int s = static_cast<int>(t / NY);
    const int64_t c = t - s * NY;
    double v = 0.0;
    if (s == left_slot) v = y[left_off + c];
    if (s == right_slot) v = y[right_off + c];
    buf[t] = v;
  }
}

__global__ void iface_unpack_kernel(const double* __restrict__ buf, double* __restrict__ y, int64_t NY, int left_slot,
                                    int64_t left_off, int right_slot, int64_t right_off) {
  for (int64_t c = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; c < NY;
       c += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    if (left_slot >= 0) y[left_off + c] = buf[left_slot * NY + c];
    if (right_slot >= 0) y[right_off + c] = buf[right_slot * NY + c];
  }
}

// SEM.eval_interpolation (SEM.py:248-273): out[a][b] = sum_kl Sx[a][k] u_e[m_a][n_b][k][l] Sy[b][l]
// for plot rows a (element m_a, evaluation row Sx[a]) and plot columns b; points whose element
// index is negative (outside the mesh) are left untouched, like the reference's np.place.
__global__ void interp_kernel(const double* __restrict__ ue, int P, int ney, int ex_begin, int ex_end,
                              const int* __restrict__ mi, const double* __restrict__ Sx, int na,
                              const int* __restrict__ ni, const double* __restrict__ Sy, int nb,
                              double* __restrict__ out) {
  const int n = P + 1;
  const int64_t total = static_cast<int64_t>(na) * nb;
  for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int a = static_cast<int>(t / nb), b = static_cast<int>(t - static_cast<int64_t>(a) * nb);
    const int m = mi[a], e = ni[b];
    if (m < ex_begin || m >= ex_end || e < 0 || e >= ney) continue;
    const double* u = ue + (static_cast<int64_t>(m - ex_begin) * ney + e) * n * n;
    double s = 0.0;
    for (int k = 0; k < n; ++k) {
      double r = 0.0;
      for (int l = 0; l < n; ++l) r = fma(u[k * n + l], Sy[static_cast<int64_t>(b) * n + l], r);
      s = fma(Sx[static_cast<int64_t>(a) * n + k], r, s);
    }
    out[t] = s;
  }
}

static unsigned grid_for(int64_t total, int threads) {
  int64_t g = (total + threads - 1) / threads;
  return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(g, 65536)));
}

}  // namespace sem

// =========================================================================== C ABI
using namespace sem;

extern "C" {

int sem_abi_version(void) { return SEM_ABI_VERSION; }
const char* sem_last_error(void) { return g_last_error.c_str(); }
int sem_max_order(void) { return kMaxOrder; }

int sem_gll_nodes(int P, double* xi, double* w, double* V) { return gll_nodes(P, xi, w, V); }
int sem_gll_differentiation(int P, double* D) {
  if (!D) return set_error(SEM_EINVAL, "null output");
  return gll_differentiation(P, D);
}
int sem_gll_gradient(int P, double* G) {
  if (!G) return set_error(SEM_EINVAL, "null output");
  return gll_gradient(P, G);
}
int sem_gll_stiffness(int P, double* K) {
  if (!K) return set_error(SEM_EINVAL, "null output");
  return gll_stiffness(P, K);
}
int sem_gll_evaluation(int P, const double* xe, int64_t count, double* S) {
  if (count < 0 || (count > 0 && (!xe || !S))) return set_error(SEM_EINVAL, "bad evaluation arguments");
  return gll_evaluation(P, xe, count, S);
}
int sem_global_index(int P, int nex, int ney, const int64_t* m, const int64_t* n, const int64_t* i, const int64_t* j,
                     int64_t count, int64_t* out) {
  if (count < 0 || (count > 0 && (!m || !n || !i || !j || !out))) return set_error(SEM_EINVAL, "bad index arguments");
  return global_index(P, nex, ney, m, n, i, j, count, out);
}

int sem_create(int P, int nex, int ney, double dx, double dy, int ex_begin, int ex_end, int device, sem_handle** out) {
  if (!out) return set_error(SEM_EINVAL, "null handle output");
  *out = nullptr;
  if (P < 1 || P > kMaxOrder) return set_error(SEM_EUNSUPPORTED, "polynomial order outside compiled range [1, 16]");
  if (nex < 1 || ney < 1) return set_error(SEM_EINVAL, "N_ex and N_ey must be positive");
  if (!(dx > 0.0) || !(dy > 0.0)) return set_error(SEM_EINVAL, "element widths must be positive");
  if (ex_begin < 0 || ex_end > nex || ex_begin >= ex_end) return set_error(SEM_EINVAL, "bad element-column range");
  const int n = P + 1;
  std::vector<double> tab(2 * n * n + n);
  int st = gll_stiffness(P, tab.data());
  if (!st) st = gll_gradient(P, tab.data() + n * n);
  if (!st) st = gll_nodes(P, nullptr, tab.data() + 2 * n * n, nullptr);
  if (st) return st;
  int prev = 0;
  if ((st = hip_check(hipGetDevice(&prev), "hipGetDevice"))) return st;
  if ((st = hip_check(hipSetDevice(device), "hipSetDevice"))) return st;
  double* d_tab = nullptr;
  hipError_t e = hipMalloc(&d_tab, tab.size() * sizeof(double));
  if (e != hipSuccess) {
    (void)hipSetDevice(prev);
    return set_error(SEM_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  }
  e = hipMemcpy(d_tab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    (void)hipFree(d_tab);
    return set_error(SEM_EHIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
  }
  sem_handle* h = new sem_handle;
  h->P = P;
  h->nex = nex;
  h->ney = ney;
  h->ex_begin = ex_begin;
  h->ex_end = ex_end;
  h->device = device;
  h->dx = dx;
  h->dy = dy;
  h->NX = static_cast<int64_t>(nex) * P + 1;
  h->NY = static_cast<int64_t>(ney) * P + 1;
  h->N = h->NX * h->NY;
  h->line_begin = static_cast<int64_t>(ex_begin) * P;
  h->line_end = static_cast<int64_t>(ex_end) * P;
  h->n_local = (h->line_end - h->line_begin + 1) * h->NY;
  h->d_tab = d_tab;
  *out = h;
  return SEM_OK;
}

int sem_destroy(sem_handle* h) {
  if (!h) return SEM_OK;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(h->device);
  (void)hipFree(h->d_tab);
  (void)hipSetDevice(prev);
  delete h;
  return SEM_OK;
}

int sem_get_info(const sem_handle* h, sem_info* o) {
  if (!h || !o) return set_error(SEM_EINVAL, "null argument");
  o->P = h->P;
  o->nex = h->nex;
  o->ney = h->ney;
  o->ex_begin = h->ex_begin;
  o->ex_end = h->ex_end;
  o->device = h->device;
  o->dx = h->dx;
  o->dy = h->dy;
  o->NX = h->NX;
  o->NY = h->NY;
  o->N = h->N;
  o->line_begin = h->line_begin;
  o->line_end = h->line_end;
  o->n_local = h->n_local;
  o->dof_begin = h->line_begin * h->NY;
  return SEM_OK;
}

int sem_apply(sem_handle* h, const sem_apply_desc* d, const double* x, double* y, void* stream) {
  if (!h || !d) return set_error(SEM_EINVAL, "null handle or descriptor");
  if (!x || !y) return set_error(SEM_EINVAL, "null x or y");
  if (x == y) return set_error(SEM_EINVAL, "x and y must not alias");
  if (d->dir_mode < SEM_DIR_NONE || d->dir_mode > SEM_DIR_REPLACE) return set_error(SEM_EINVAL, "bad dir_mode");
  if (d->dir_mode == SEM_DIR_REPLACE && !d->dir_val) return set_error(SEM_EINVAL, "SEM_DIR_REPLACE needs dir_val");
  if (d->algo == SEM_ALGO_MFMA) return set_error(SEM_EUNSUPPORTED, "MFMA algorithm not built in this version");
  ApplyArgs a{};
  a.x = x;
  a.y = y;
  a.cu = d->cu;
  a.cv = d->cv;
  a.ea = d->ea;
  a.eb = d->eb;
  a.ec = d->ec;
  a.ed = d->ed;
  a.has_e1 = (d->c_extra != 0.0 && d->ea && d->eb) ? 1 : 0;
  a.has_e2 = (d->c_extra != 0.0 && d->ec && d->ed) ? 1 : 0;
  a.mask = d->dir_mask;
  a.dval = d->dir_val;
  a.tab = h->d_tab;
  a.cM = d->c_mass;
  a.cK = d->c_stiff;
  a.cX = d->c_gradx;
  a.cY = d->c_grady;
  a.cE = d->c_extra;
  a.cA = d->c_acc;
  a.sx = h->dy / h->dx;
  a.sy = h->dx / h->dy;
  a.hx = h->dx / 2.0;
  a.hy = h->dy / 2.0;
  a.hxy = (h->dx / 2.0) * (h->dy / 2.0);
  a.NY = h->NY;
  a.NXg = h->NX;
  a.line_begin = h->line_begin;
  a.line_end = h->line_end;
  a.nex = h->nex;
  a.ney = h->ney;
  a.ex_begin = h->ex_begin;
  a.ex_end = h->ex_end;
  a.dir_mode = d->dir_mode;
  a.sides = d->dir_sides;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (h->P) {
#define SEM_CASE(PP) \
  case PP:           \
    return launch_apply<PP>(a, h, s);
    SEM_CASE(1) SEM_CASE(2) SEM_CASE(3) SEM_CASE(4) SEM_CASE(5) SEM_CASE(6) SEM_CASE(7) SEM_CASE(8)
    SEM_CASE(9) SEM_CASE(10) SEM_CASE(11) SEM_CASE(12) SEM_CASE(13) SEM_CASE(14) SEM_CASE(15) SEM_CASE(16)
#undef SEM_CASE
    default:
      return set_error(SEM_EUNSUPPORTED, "polynomial order outside compiled range");
  }
}

int sem_gather_elements(sem_handle* h, const double* u, double* ue, void* stream) {
  if (!h || !u || !ue) return set_error(SEM_EINVAL, "null argument");
  const int n = h->P + 1;
  const int64_t total = static_cast<int64_t>(h->ex_end - h->ex_begin) * h->ney * n * n;
  hipLaunchKernelGGL(gather_kernel, dim3(grid_for(total, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), u,
                     ue, h->P, h->ney, h->ex_begin, h->line_begin, h->NY, total);
  return hip_check(hipGetLastError(), "gather launch");
}

int sem_dss(sem_handle* h, const double* ae, double* out, void* stream) {
  if (!h || !ae || !out) return set_error(SEM_EINVAL, "null argument");
  if (static_cast<const void*>(ae) == static_cast<const void*>(out)) return set_error(SEM_EINVAL, "in/out alias");
  hipLaunchKernelGGL(dss_kernel, dim3(grid_for(h->n_local, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     ae, out, h->P, h->ney, h->ex_begin, h->ex_end, h->line_begin, h->NY, h->n_local);
  return hip_check(hipGetLastError(), "dss launch");
}

int sem_eval_interpolation(sem_handle* h, const double* ue, int na, const int* m_idx, const double* Sx, int nb,
                           const int* n_idx, const double* Sy, double* out, void* stream) {
  if (!h || !ue || !out || na < 0 || nb < 0) return set_error(SEM_EINVAL, "bad interpolation arguments");
  if (na == 0 || nb == 0) return SEM_OK;
  if (!m_idx || !Sx || !n_idx || !Sy) return set_error(SEM_EINVAL, "null interpolation table");
  hipLaunchKernelGGL(interp_kernel, dim3(grid_for(static_cast<int64_t>(na) * nb, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), ue, h->P, h->ney, h->ex_begin, h->ex_end, m_idx, Sx, na,
                     n_idx, Sy, nb, out);
  return hip_check(hipGetLastError(), "interpolation launch");
}

static int iface_slots(const sem_handle* h, const int* bounds, int G, int* left, int* right) {
  if (!bounds || G < 1) return set_error(SEM_EINVAL, "bad partition");
  if (bounds[0] != 0 || bounds[G] != h->nex) return set_error(SEM_EINVAL, "partition must cover [0, N_ex]");
  int r = -1;
  for (int k = 0; k < G; ++k) {
    if (bounds[k] >= bounds[k + 1]) return set_error(SEM_EINVAL, "partition bounds must increase");
    if (bounds[k] == h->ex_begin && bounds[k + 1] == h->ex_end) r = k;
  }
  if (r < 0) return set_error(SEM_EINVAL, "handle's element range is not a part of the partition");
  *left = r > 0 ? r - 1 : -1;
  *right = r < G - 1 ? r : -1;
  return SEM_OK;
}

int sem_interface_pack(sem_handle* h, const double* y, const int* bounds, int G, double* buf, void* stream) {
  if (!h || !y || !buf) return set_error(SEM_EINVAL, "null argument");
  int L, R, st;
  if ((st = iface_slots(h, bounds, G, &L, &R))) return st;
  if (G < 2) return SEM_OK;
  const int64_t total = static_cast<int64_t>(G - 1) * h->NY;
  hipLaunchKernelGGL(iface_pack_kernel, dim3(grid_for(total, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     y, buf, h->NY, G - 1, L, static_cast<int64_t>(0), R, h->n_local - h->NY);
  return hip_check(hipGetLastError(), "interface pack launch");
}

int sem_interface_unpack(sem_handle* h, const double* buf, const int* bounds, int G, double* y, void* stream) {
  if (!h || !y || !buf) return set_error(SEM_EINVAL, "null argument");
  int L, R, st;
  if ((st = iface_slots(h, bounds, G, &L, &R))) return st;
  if (G < 2) return SEM_OK;
  hipLaunchKernelGGL(iface_unpack_kernel, dim3(grid_for(h->NY, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), buf, y, h->NY, L, static_cast<int64_t>(0), R,
                     h->n_local - h->NY);
  return hip_check(hipGetLastError(), "interface unpack launch");
}

}  // extern "C"
