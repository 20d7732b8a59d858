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
#include <type_traits>
#include <utility>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "apply_common.h"

namespace sem {

int launch_apply_band(const ApplyArgs& a, const sem_handle* h, hipStream_t s);  // apply_band.hip
static bool band_fits(const sem_handle* h) { return h->n_local + (h->P + 1) * h->NY < (int64_t(1) << 28); }
std::string band_kernel_name(int P, long long n_local);
int launch_apply_bmfma(const ApplyArgs& a, const sem_handle* h, hipStream_t s);  // apply_band.hip
std::string bmfma_kernel_name(int P);

static int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return SEM_OK;
  return set_error(SEM_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// --------------------------------------------------------------------------- apply kernel

template <int P>
struct TileCfg {
  static constexpr int n = P + 1;
  static constexpr int THREADS = 128;
  static constexpr int TX = (16 / P) > 0 ? 16 / P : 1;                       // elements per tile in x
  static constexpr int TY = (THREADS / (TX * P)) > 0 ? THREADS / (TX * P) : 1; // elements per tile in y
  static constexpr int BX = TX * P;      // owned lines (+1 closing line at the last tile)
  static constexpr int BY = TY * P;      // owned columns (+1 closing column at the last tile)
  static constexpr int RX = BX + P + 1;  // staged lines   [gx0-P, gx0+BX]
  static constexpr int RY = BY + P + 1;  // staged columns [gy0-P, gy0+BY]
  static constexpr int PT = RY | 1;      // odd pitch: conflict-free strided LDS reads
  static constexpr int PY = (BY + 1) | 1;
  static constexpr int NSTAGE = (RX * RY + THREADS - 1) / THREADS;  // staging loads per thread
  static_assert(TX * BY <= THREADS && TY * BX <= THREADS, "one phase item per thread");
};

// Phase B item: y-direction contractions of element row `ae` on owned line r (lanes along lines).
template <int P>
__device__ __forceinline__ void phase_b(const ApplyArgs& a, const double* Ts, double* Yk, double* Yg, const double* ws,
                                       int ae, int r, int n0, int64_t gx0) {
  using C = TileCfg<P>;
  const int ne = n0 + ae;
  double t[2 * P + 1];
#pragma unroll
  for (int q = 0; q <= 2 * P; ++q) t[q] = Ts[(r + P) * C::PT + ae * P + q];
  const double mx = weight_sum(gx0 + r, P, a.ex_begin, a.ex_end, ws);
  const double fk = a.sy * mx, fg = a.hx * mx;
  const bool hasL = ne > 0, last = ne == a.ney - 1;
  for_rows(std::make_integer_sequence<int, P + 1>{}, [&](auto J) {
    constexpr int j = decltype(J)::value;
    if (j == P && !last) return;  // the closing column exists only in the last element row
    double k, g;
    contract_row<P, j>(t, hasL, k, g);
    Yk[r * C::PY + ae * P + j] = fk * k;
    Yg[r * C::PY + ae * P + j] = fg * g;
  });
}

// Phase A item: x-direction contractions of element column `be` at owned column c, combined
// with phase B's results and the pointwise terms; writes P (or P+1) outputs of column c.
template <int P>
__device__ __forceinline__ void phase_a(const ApplyArgs& a, const double* Ts, const double* Yk, const double* Yg,
                                        const double* ws, int be, int c, int m0, int64_t gx0, int64_t gy0,
                                        const double (&pu)[P + 1], const double (&pv)[P + 1]) {
  using C = TileCfg<P>;
  const int me = m0 + be;
  const int64_t gy = gy0 + c;
  double t[2 * P + 1];
#pragma unroll
  for (int q = 0; q <= 2 * P; ++q) t[q] = Ts[(be * P + q) * C::PT + c + P];
  const double my = weight_sum(gy, P, 0, a.ney, ws);
  const bool hasL = me - 1 >= a.ex_begin, last = me == a.ex_end - 1;
  for_rows(std::make_integer_sequence<int, P + 1>{}, [&](auto I) {
    constexpr int i = decltype(I)::value;
    if (i == P && !last) return;  // the closing line exists only in the last element column
    double k, g;
    contract_row<P, i>(t, hasL, k, g);
    const int rl = be * P + i;
    const int64_t gx = gx0 + rl;
    const int64_t p = (gx - a.line_begin) * a.NY + gy;
    const double xv = t[P + i];
    double z = 0.0;
    if (a.cK != 0.0) z = a.cK * fma(a.sx * my, k, Yk[rl * C::PY + c]);
    if (a.cM != 0.0) z = fma(a.cM * a.hxy * weight_sum(gx, P, a.ex_begin, a.ex_end, ws) * my, xv, z);
    if (a.cX != 0.0) z = fma(a.cX * pu[i], a.hy * my * g, z);
    if (a.cY != 0.0) z = fma(a.cY * pv[i], Yg[rl * C::PY + c], z);
    // pointwise terms are node values, not partial sums: on a strip's right interface line they
    // are left to the right-hand owner (the exchange sums the two strips' values)
    const bool own = !(gx == a.line_end && a.ex_end < a.nex);
    if (a.has_e1 && own) z = fma(a.cE * a.ea[p], a.eb[p], z);
    if (a.has_e2 && own) z = fma(a.cE * a.ec[p], a.ed[p], z);
    if (a.cA != 0.0 && own) z = fma(a.cA, a.y[p], z);
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
  });
}

// Pointwise coefficients u, v of the P (+1) outputs of a phase-A item, loaded up front so
// their latency hides under the staging loads (and no load has to wait behind a y store).
template <int P>
__device__ __forceinline__ void prefetch_uv(const ApplyArgs& a, int be, int c, int m0, int64_t gx0, int64_t gy0,
                                            double (&pu)[P + 1], double (&pv)[P + 1]) {
  const bool last = m0 + be == a.ex_end - 1;
  // row P of a non-last element column is the next element's row 0: still a valid address,
  // so every load is unconditional (see the staging loop); its value is simply unused.
  (void)last;
  const int64_t p0 = (gx0 + be * P - a.line_begin) * a.NY + gy0 + c;
  if (a.cu) {
#pragma unroll
    for (int i = 0; i <= P; ++i) pu[i] = a.cu[p0 + i * a.NY];
  } else {
#pragma unroll
    for (int i = 0; i <= P; ++i) pu[i] = 1.0;
  }
  if (a.cv) {
#pragma unroll
    for (int i = 0; i <= P; ++i) pv[i] = a.cv[p0 + i * a.NY];
  } else {
#pragma unroll
    for (int i = 0; i <= P; ++i) pv[i] = 1.0;
  }
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
  const int tid = threadIdx.x;
  const bool lastx = m1 == a.ex_end, lasty = n1 == a.ney;

  // ---- issue every global load of this thread first: the staged tile and u, v
  // GLL weights for weight_sum: issued first so the LDS store below waits for this load only
  const double wreg = a.tab[2 * n * n + min(tid, n - 1)];

  // Loads are unconditional from clamped (always in-bounds) addresses: a per-element
  // "load or zero" select makes hipcc branch around, and wait for, each load in turn.
  // Staged entries outside the domain / the local lines hold clamped copies; they are
  // never consumed (they only feed left windows gated by hasL, or non-owned rows).
  double stage[C::NSTAGE];
#pragma unroll
  for (int s = 0; s < C::NSTAGE; ++s) {
    const int idx = min(tid + s * C::THREADS, C::RX * C::RY - 1);
    const int rr = idx / C::RY, cc = idx - rr * C::RY;
    const int64_t gx = min(max(gx0 - P + rr, a.line_begin), a.line_end);
    const int64_t gy = min(max(gy0 - P + cc, int64_t(0)), a.NY - 1);
    stage[s] = a.x[(gx - a.line_begin) * a.NY + gy];
  }
  // phase-A item of this thread: (element column be, owned column c)
  const int be = tid / C::BY, cA = tid - be * C::BY;
  const bool hasA = be < m1 - m0 && cA < (n1 - n0) * P;
  double pu[P + 1], pv[P + 1];
  if (hasA) prefetch_uv<P>(a, be, cA, m0, gx0, gy0, pu, pv);

  if (tid < n) ws[tid] = wreg;
#pragma unroll
  for (int s = 0; s < C::NSTAGE; ++s) {
    const int idx = tid + s * C::THREADS;
    if (idx < C::RX * C::RY) {
      const int rr = idx / C::RY, cc = idx - rr * C::RY;
      Ts[rr * C::PT + cc] = stage[s];
    }
  }
  __syncthreads();

  // ---- phase B: (element row ae, owned line r), lanes along lines
  {
    const int ae = tid / C::BX, r = tid - ae * C::BX;
    if (ae < n1 - n0 && r < (m1 - m0) * P) phase_b<P>(a, Ts, Yk, Yg, ws, ae, r, n0, gx0);
    if (lastx && tid < n1 - n0) phase_b<P>(a, Ts, Yk, Yg, ws, tid, (m1 - m0) * P, n0, gx0);  // closing line
  }
  __syncthreads();

  // ---- phase A: (element column be, owned column c), lanes along columns (coalesced I/O)
  if (hasA) phase_a<P>(a, Ts, Yk, Yg, ws, be, cA, m0, gx0, gy0, pu, pv);
  if (lasty && tid < m1 - m0) {  // closing column
    const int cz = (n1 - n0) * P;
    double qu[P + 1], qv[P + 1];
    prefetch_uv<P>(a, tid, cz, m0, gx0, gy0, qu, qv);
    phase_a<P>(a, Ts, Yk, Yg, ws, tid, cz, m0, gx0, gy0, qu, qv);
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

// =========================================================================== MFMA path
//
// Same operator, same tile ownership; the per-element contractions run on the fp64
// matrix cores (v_mfma_f64_16x16x4_f64) instead of the VALU:
//   phase A (x): for each element column e of the tile (plus the left halo element) and
//                each 16-column block,  D[i][c] = sum_k K_s[i][k] T[eP+k][c]  (and G_s),
//                A = K_s (rows i <= P, zero-padded to 16 x 4*KS), B = staged x.
//   phase B (y): for each element row e and each 16-line block,
//                D[line][j] = sum_l T[line][eP+l] K_s[j][l]                    (and G_s),
//                A = staged x, B = K_s^T -- the SAME per-lane registers as phase A's A.
// Results go to LDS per element (all P+1 rows), and the epilogue sums the one or two
// element contributions of every owned node in a fixed order (deterministic DSS).
// The VALU is left with staging, the epilogue and the pointwise terms.
typedef double dbl4 __attribute__((ext_vector_type(4)));

constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <int P, int TX_, int TY_, int NW_, bool SPLIT_, bool SWZ_ = true>
struct MCfg {
  static constexpr int n = P + 1, TX = TX_, TY = TY_, NW = NW_, THREADS = 64 * NW_;
  static constexpr bool SPLIT = SPLIT_;                   // K and G chains as separate wave tasks
  static constexpr int BX = TX * P, BY = TY * P;          // owned lines / columns (w/o closing ones)
  static constexpr int NLB = (BX + 15) / 16, NCB = (BY + 15) / 16;  // 16-wide MFMA blocks
  static constexpr int KS = (n + 3) / 4;                  // k-steps of 4
  static constexpr int RX = cmax(TX * P + 4 * KS, P + 16 * NLB);    // staged lines from gx0-P
  static constexpr int RY = cmax(TY * P + 4 * KS, P + 16 * NCB);    // staged columns from gy0-P
  // Staged tile layout (round 4, bank-conflict-free; tools/lds_banks_mfma.py): rows of R16 = RY rounded up to
  // 16 slots, pitch PT == 16 (mod 32) doubles, column c of row r at c ^ 2 ((r >> 1) & 7) (a permutation inside
  // each aligned 16-column block).  Phase A reads two rows x 16 columns per 32-lane group: PT puts the rows in
  // opposite bank halves.  Phase B reads 16 rows x 2 columns: the swizzle spreads the rows of each parity over
  // 8 distinct 2-double bank slots.  Staging stores one aligned 16-column run per 16-lane group.  (pitch18 with
  // row-major staging had 2-way conflicts in phase A, staging and the epilogue: 95,488 conflict cycles per cfg2
  // dispatch, profiles/r03/mfma64/.)
  // SWZ = false (the persistent large-tile variants, where the swizzle's address arithmetic spilled VGPRs):
  // the round-3 layout, row-major staging at pitch == 18 (mod 32).
  static constexpr bool SWZ = SWZ_;
  static constexpr int R16 = (RY + 15) / 16 * 16;
  static constexpr int PT = SWZ ? R16 + ((16 - R16 % 32) + 32) % 32 : RY + ((18 - (RY % 32)) + 32) % 32;
  __host__ __device__ static constexpr int ts(int r, int c) { return r * PT + (SWZ ? c ^ (((r >> 1) & 7) << 1) : c); }
  static constexpr int EC = 16 * NCB;   // E (x-results) column pitch
  static constexpr int FL = 16 * NLB;   // F (y-results) lines per element row
  static constexpr int TA = (TX + 1) * NCB, TB = (TY + 1) * NLB;
  static constexpr int NWA = NW > 1 ? NW / 2 : 1;         // waves running phase A (the rest: phase B)
  static_assert(NW >= 2, "phase A and B run on separate waves");
  static constexpr int MAXG = 4;                          // tasks batched per wave (register bound)
  // staging slots per row: R16 when that costs no extra staging register, else the unpadded RY (the
  // large-tile persistent variants, whose prefetched next tile would spill)
  static constexpr int SR =
      SWZ && (RX * R16 + THREADS - 1) / THREADS == (RX * RY + THREADS - 1) / THREADS ? R16 : RY;
  static constexpr int NSTAGE = (RX * SR + THREADS - 1) / THREADS;
  static constexpr int NMAIN = (BX * BY + THREADS - 1) / THREADS;  // epilogue nodes per thread
  static_assert(n <= 16, "MFMA path needs P+1 <= 16");
};

template <class C>
struct MSmem {
  double Ts[C::RX * C::PT];
  double EK[(C::TX + 1) * C::n * C::EC];
  double EG[(C::TX + 1) * C::n * C::EC];
  double FK[(C::TY + 1) * C::FL * C::n];
  double FG[(C::TY + 1) * C::FL * C::n];
  double ws[C::n];
};

template <int P, int TX, int TY, int NW, bool PERSIST, bool SPLIT>
__global__ __launch_bounds__(64 * NW, PERSIST ? 2 : (NW >= 4 ? 4 : 2)) void apply_tp_mfma(const ApplyArgs a) {
  using C = MCfg<P, TX, TY, NW, SPLIT, !PERSIST>;
  constexpr int n = C::n;
  __shared__ MSmem<C> sm;

  // Workgroups walk contiguous runs of tiles (y fastest); the XCD-aware remap gives the
  // workgroups of one XCD neighbouring runs (halo lines shared through that XCD's L2).
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q = nb >> 3, rem = nb & 7;
  const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int ntiles = a.tiles_x * a.tiles_y;
  const int t_begin = PERSIST ? static_cast<int>((static_cast<long long>(L) * ntiles) / nb) : L;
  const int t_end = PERSIST ? static_cast<int>((static_cast<long long>(L + 1) * ntiles) / nb) : L + 1;

  const int lb0 = static_cast<int>(a.line_begin), lb1 = static_cast<int>(a.line_end), NY = static_cast<int>(a.NY);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lk = lane >> 4;
  SEM_STAMP(0);
  SEM_STAMP_HWID();

  const int nbytes = a.n_local32 * 8;
  const auto rx = brsrc(a.x, nbytes), ru = brsrc(a.cu, a.cu ? nbytes : 0), rv = brsrc(a.cv, a.cv ? nbytes : 0);

  // Tile-invariant per-thread byte offsets of the staged window entries and epilogue nodes.
  int soff[C::NSTAGE], noff[C::NMAIN];
#pragma unroll
  for (int s = 0; s < C::NSTAGE; ++s) {
    const int idx = tid + s * C::THREADS;
    const int rr = idx / C::SR, cc = idx - rr * C::SR;
    soff[s] = rr < C::RX && cc < C::RY ? (rr * NY + cc) * 8 : -(1 << 30);  // padding slots: no memory touched
  }
#pragma unroll
  for (int qn = 0; qn < C::NMAIN; ++qn) {
    const int idx = tid + qn * C::THREADS;
    const int rl = idx / C::BY, c = idx - rl * C::BY;
    noff[qn] = (rl * NY + c) * 8;
  }

  // Issue every global load of tile t (staged x window, u and v of this thread's epilogue nodes).
  // Entries outside the local lines read 0 (buffer bounds check); entries past the domain's
  // y-ends wrap into neighbouring lines.  Neither is ever consumed.
  double st[C::NSTAGE], pu[C::NMAIN], pv[C::NMAIN];
  auto issue = [&](int t) {
    const int tx = t / a.tiles_y, ty = t - tx * a.tiles_y;
    const int gx0 = (a.ex_begin + tx * TX) * P, gy0 = ty * TY * P;
    const int sbase = ((gx0 - P - lb0) * NY + gy0 - P) * 8, nbase = ((gx0 - lb0) * NY + gy0) * 8;
#pragma unroll
    for (int s = 0; s < C::NSTAGE; ++s) st[s] = bload(rx, sbase + soff[s]);
#pragma unroll
    for (int qn = 0; qn < C::NMAIN; ++qn) {
      pu[qn] = bload(ru, nbase + noff[qn]);
      pv[qn] = bload(rv, nbase + noff[qn]);
    }
  };
  if (t_begin < t_end) issue(t_begin);

  // Per-lane MFMA coefficient operands A[i=lr][k=4s+lk] = K_s[lr][k] (0 outside n x n) and the
  // GLL weights, loaded AFTER the tile's loads so nothing waits for them before staging starts.
  double aK[C::KS], aG[C::KS];
#pragma unroll
  for (int s = 0; s < C::KS; ++s) {
    const int k = 4 * s + lk;
    const bool ok = lr <= P && k <= P;
    const int idx = ok ? lr * n + k : 0;
    const double kv = a.tab[idx], gv = a.tab[n * n + idx];
    aK[s] = ok ? kv : 0.0;
    aG[s] = ok ? gv : 0.0;
  }
  const double wreg = a.tab[2 * n * n + min(tid, n - 1)];
  bool ws_done = false;
  // Uniform epilogue factors (absent terms have coefficient 0 and contribute exact zeros).
  const double fKx = a.cK * a.sx, fKy = a.cK * a.sy, fM = a.cM * a.hxy, fX = a.cX * a.hy, fY = a.cY * a.hx;
  const bool has_u = a.cu != nullptr, has_v = a.cv != nullptr;
  SEM_STAMP(1);

  for (int t = t_begin; t < t_end; ++t) {
    const int tx = t / a.tiles_y, ty = t - tx * a.tiles_y;
    const int m0 = a.ex_begin + tx * TX, m1 = min(m0 + TX, a.ex_end);
    const int n0 = ty * TY, n1 = min(n0 + TY, a.ney);
    const int gx0 = m0 * P, gy0 = n0 * P;

    if (PERSIST) __syncthreads();  // the previous tile's epilogue has finished reading Ts
#pragma unroll
    for (int s = 0; s < C::NSTAGE; ++s) {
      const int idx = tid + s * C::THREADS;
      const int rr = idx / C::SR, cc = idx - rr * C::SR;
      if (rr < C::RX && cc < C::RY) sm.Ts[C::ts(rr, cc)] = st[s];
    }
    if (!ws_done) {
      if (tid < n) sm.ws[tid] = wreg;
      ws_done = true;
    }
    double cu_[C::NMAIN], cv_[C::NMAIN];
#pragma unroll
    for (int qn = 0; qn < C::NMAIN; ++qn) {
      cu_[qn] = has_u ? pu[qn] : 1.0;
      cv_[qn] = has_v ? pv[qn] : 1.0;
    }
    SEM_STAMP(2);
    __syncthreads();
    SEM_STAMP(3);
    if (PERSIST && t + 1 < t_end) issue(t + 1);  // next tile's loads fly while this tile computes

    // ---- phases A and B: each wave owns a homogeneous list of tasks (the first half of the
    // waves phase A, the rest phase B); it issues every operand read of its tasks first, then
    // all MFMAs with one independent K and one G accumulator chain per task, then the writes.
    if (!(kDiag && (a.diag & 1))) {
      constexpr int NWA = C::NWA, NWB = NW - C::NWA;
      if (wave < NWA) {
        constexpr int TW = (C::TA + NWA - 1) / NWA, TG = TW < C::MAXG ? TW : C::MAXG;
#pragma unroll
        for (int g0 = 0; g0 < TW; g0 += TG) {
          double bv[TG][C::KS];
#pragma unroll
          for (int tt = 0; tt < TG; ++tt) {
            const int task = min(wave + (g0 + tt) * NWA, C::TA - 1);
            const int e = task / C::NCB, cb = task - e * C::NCB;  // element line e (0 = halo), column block
#pragma unroll
            for (int s = 0; s < C::KS; ++s) {
              const int k = 4 * s + lk;
              const double v = sm.Ts[C::ts(e * P + k, P + cb * 16 + lr)];
              bv[tt][s] = (4 * s + 3 > P && k > P) ? 0.0 : v;  // next element's nodes: keep NaN/Inf out
            }
          }
          dbl4 accK[TG], accG[TG];
#pragma unroll
          for (int tt = 0; tt < TG; ++tt) accK[tt] = accG[tt] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int s = 0; s < C::KS; ++s)
#pragma unroll
            for (int tt = 0; tt < TG; ++tt) {
              accK[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(aK[s], bv[tt][s], accK[tt], 0, 0, 0);
              accG[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(aG[s], bv[tt][s], accG[tt], 0, 0, 0);
            }
#pragma unroll
          for (int tt = 0; tt < TG; ++tt) {
            const int task = wave + (g0 + tt) * NWA;
            if (g0 + tt < TW && task < C::TA) {
              const int e = task / C::NCB, cb = task - e * C::NCB;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int i = lk + 4 * r;  // C/D row of an f64 16x16x4 MFMA: (lane>>4) + 4*reg
                if (i <= P) {
                  sm.EK[(e * n + i) * C::EC + cb * 16 + lr] = accK[tt][r];
                  sm.EG[(e * n + i) * C::EC + cb * 16 + lr] = accG[tt][r];
                }
              }
            }
          }
        }
      } else {
        constexpr int TW = (C::TB + NWB - 1) / NWB, TG = TW < C::MAXG ? TW : C::MAXG;
        const int wb = wave - NWA;
#pragma unroll
        for (int g0 = 0; g0 < TW; g0 += TG) {
          double av[TG][C::KS];
#pragma unroll
          for (int tt = 0; tt < TG; ++tt) {
            const int task = min(wb + (g0 + tt) * NWB, C::TB - 1);
            const int e = task / C::NLB, lbk = task - e * C::NLB;  // element column e (0 = halo), line block
#pragma unroll
            for (int s = 0; s < C::KS; ++s) {
              const int k = 4 * s + lk;
              const double v = sm.Ts[C::ts(P + lbk * 16 + lr, e * P + k)];
              av[tt][s] = (4 * s + 3 > P && k > P) ? 0.0 : v;
            }
          }
          dbl4 accK[TG], accG[TG];
#pragma unroll
          for (int tt = 0; tt < TG; ++tt) accK[tt] = accG[tt] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int s = 0; s < C::KS; ++s)
#pragma unroll
            for (int tt = 0; tt < TG; ++tt) {
              accK[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tt][s], aK[s], accK[tt], 0, 0, 0);
              accG[tt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tt][s], aG[s], accG[tt], 0, 0, 0);
            }
#pragma unroll
          for (int tt = 0; tt < TG; ++tt) {
            const int task = wb + (g0 + tt) * NWB;
            if (g0 + tt < TW && task < C::TB && lr <= P) {
              const int e = task / C::NLB, lbk = task - e * C::NLB;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int line = lbk * 16 + lk + 4 * r;
                sm.FK[(e * C::FL + line) * n + lr] = accK[tt][r];
                sm.FG[(e * C::FL + line) * n + lr] = accG[tt][r];
              }
            }
          }
        }
      }
    }
    SEM_STAMP(4);
    __syncthreads();
    SEM_STAMP(5);

    // ---- epilogue, interior nodes: one node per item, lanes along columns.  For these the
    // right/upper element always exists and the line is never the partition's closing line.
    const int BXo = (m1 - m0) * P, BYo = (n1 - n0) * P;  // owned without closing line / column
    const int nbase = ((gx0 - lb0) * NY + gy0) * 8;
    const auto ry = brsrc(a.y, nbytes);
    const bool leftx = m0 > a.ex_begin, lefty = n0 > 0;
    const double wP = sm.ws[P];
#pragma unroll
    for (int qn = 0; qn < C::NMAIN; ++qn) {
      const int idx = tid + qn * C::THREADS;
      const int rl = idx / C::BY, c = idx - rl * C::BY;
      if (!((qn + 1) * C::THREADS <= C::BX * C::BY || idx < C::BX * C::BY) || rl >= BXo || c >= BYo) continue;
      const int off = nbase + noff[qn];
      const int i = rl % P, ex = rl / P, j = c % P, ey = c / P;
      const bool hasLx = i == 0 && (ex > 0 || leftx), hasLy = j == 0 && (ey > 0 || lefty);
      const double xv = sm.Ts[C::ts(P + rl, P + c)];
      const double kl = sm.EK[(ex * n + P) * C::EC + c], gl = sm.EG[(ex * n + P) * C::EC + c];
      const double kr = sm.EK[((ex + 1) * n + i) * C::EC + c], gr = sm.EG[((ex + 1) * n + i) * C::EC + c];
      const double fkl = sm.FK[(ey * C::FL + rl) * n + P], fgl = sm.FG[(ey * C::FL + rl) * n + P];
      const double fkr = sm.FK[((ey + 1) * C::FL + rl) * n + j], fgr = sm.FG[((ey + 1) * C::FL + rl) * n + j];
      const double wi = sm.ws[i], wj = sm.ws[j];
      if (kDiag && (a.diag & 2)) {
        bstore(ry, off, xv * cu_[qn] + cv_[qn]);
        continue;
      }
      const double XK = hasLx ? kl + kr : kr, XG = hasLx ? gl + gr : gr;
      const double YK = hasLy ? fkl + fkr : fkr, YG = hasLy ? fgl + fgr : fgr;
      const double mx = hasLx ? wP + wi : wi, my = hasLy ? wP + wj : wj;
      double z = fma(fKx * my, XK, fKy * mx * YK);
      z = fma(fM * mx * my, xv, z);
      z = fma(fX * cu_[qn], my * XG, z);
      z = fma(fY * cv_[qn], mx * YG, z);
      if (a.has_e1) z = fma(a.cE * a.ea[off >> 3], a.eb[off >> 3], z);
      if (a.has_e2) z = fma(a.cE * a.ec[off >> 3], a.ed[off >> 3], z);
      if (a.cA != 0.0) z = fma(a.cA, bload(ry, off), z);
      if (a.dir_mode != SEM_DIR_NONE) {
        const int gx = gx0 + rl, gy = gy0 + c;
        const bool isd = a.mask ? (a.mask[off >> 3] != 0)
                                : (((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NXg - 1) ||
                                   ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == NY - 1));
        if (isd) z = a.dir_mode == SEM_DIR_IDENTITY ? xv - (a.dval ? a.dval[off >> 3] : 0.0) : a.dval[off >> 3];
      }
      bstore(ry, off, z);
    }

    // ---- epilogue, closing line / column of the local domain (edge tiles only): general path
    const bool lastx = m1 == a.ex_end, lasty = n1 == a.ney;
    if (lastx || lasty) {
      auto edge = [&](int rl, int c) {
        const int gx = gx0 + rl, gy = gy0 + c;
        const int p = (gx - lb0) * NY + gy;
        const double uu = a.cu ? a.cu[p] : 1.0, vv = a.cv ? a.cv[p] : 1.0;
        const double xv = sm.Ts[C::ts(P + rl, P + c)];
        if (kDiag && (a.diag & 2)) {
          a.y[p] = xv * uu + vv;
          return;
        }
        const int i = rl % P, ex = rl / P;
        const int mR = m0 + ex;
        const bool hasR = mR < a.ex_end, hasLx = i == 0 && mR - 1 >= a.ex_begin;
        double XK = 0.0, XG = 0.0;
        if (c < C::EC) {
          if (hasLx) {
            XK = sm.EK[(ex * n + P) * C::EC + c];
            XG = sm.EG[(ex * n + P) * C::EC + c];
          }
          if (hasR) {
            XK += sm.EK[((ex + 1) * n + i) * C::EC + c];
            XG += sm.EG[((ex + 1) * n + i) * C::EC + c];
          }
        } else {
          contract_generic_f<P>(a.tab, a.tab + n * n, [&](int l) { return sm.Ts[C::ts(P + rl - i + l, P + c)]; }, i,
                                hasR, hasLx, XK, XG);
        }
        const int j = c % P, ey = c / P;
        const int nR = n0 + ey;
        const bool hasRy = nR < a.ney, hasLy = j == 0 && nR - 1 >= 0;
        double YK = 0.0, YG = 0.0;
        if (rl < C::FL) {
          if (hasLy) {
            YK = sm.FK[(ey * C::FL + rl) * n + P];
            YG = sm.FG[(ey * C::FL + rl) * n + P];
          }
          if (hasRy) {
            YK += sm.FK[((ey + 1) * C::FL + rl) * n + j];
            YG += sm.FG[((ey + 1) * C::FL + rl) * n + j];
          }
        } else {
          contract_generic_f<P>(a.tab, a.tab + n * n, [&](int l) { return sm.Ts[C::ts(P + rl, P + c - j + l)]; }, j,
                                hasRy, hasLy, YK, YG);
        }
        const double mx = wsum<P>(gx, a.ex_begin, a.ex_end, sm.ws);
        const double my = wsum<P>(gy, 0, a.ney, sm.ws);
        double z = fma(fKx * my, XK, fKy * mx * YK);
        z = fma(fM * mx * my, xv, z);
        z = fma(fX * uu, my * XG, z);
        z = fma(fY * vv, mx * YG, z);
        const bool own = !(gx == lb1 && a.ex_end < a.nex);  // pointwise terms: right-hand owner only
        if (a.has_e1 && own) z = fma(a.cE * a.ea[p], a.eb[p], z);
        if (a.has_e2 && own) z = fma(a.cE * a.ec[p], a.ed[p], z);
        if (a.cA != 0.0 && own) z = fma(a.cA, a.y[p], z);
        if (a.dir_mode != SEM_DIR_NONE) {
          const bool isd = a.mask ? (a.mask[p] != 0)
                                  : (((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NXg - 1) ||
                                     ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == NY - 1));
          if (isd) {
            // an interface line's Dirichlet row is written by its owner (the right strip) only
            const bool owner = !(gx == lb1 && a.ex_end < a.nex);
            if (!owner)
              z = 0.0;
            else if (a.dir_mode == SEM_DIR_IDENTITY)
              z = xv - (a.dval ? a.dval[p] : 0.0);
            else
              z = a.dval[p];
          }
        }
        a.y[p] = z;
      };
      if (lastx)  // closing line of the local lines
        for (int c = tid; c < BYo + (lasty ? 1 : 0); c += C::THREADS) edge(BXo, c);
      if (lasty)  // closing column of the domain
        for (int rl = tid; rl < BXo; rl += C::THREADS) edge(rl, BYo);
    }
  }
  SEM_STAMP(6);
}

template <int P, int TX, int TY, int NW, bool PERSIST, bool SPLIT>
static int launch_apply_mfma(const ApplyArgs& args_in, const sem_handle* h, hipStream_t s) {
  using C = MCfg<P, TX, TY, NW, SPLIT, !PERSIST>;
  ApplyArgs args = args_in;
  const int ncols = h->ex_end - h->ex_begin;
  args.tiles_x = (ncols + TX - 1) / TX;
  args.tiles_y = (h->ney + TY - 1) / TY;
  const long long ntiles = static_cast<long long>(args.tiles_x) * args.tiles_y;
  if (ntiles <= 0 || ntiles > 0x7fffffffLL) return set_error(SEM_EINVAL, "mesh too large for one launch");
  long long grid = ntiles;
  if (PERSIST) {  // persistent grid: the resident workgroups of every CU, never more than the tiles
    static int resident = [] {
      int per_cu = 0, dev = 0, cus = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, apply_tp_mfma<P, TX, TY, NW, PERSIST, SPLIT>,
                                                       C::THREADS, 0) != hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
      return per_cu * cus;
    }();
    grid = std::min<long long>(ntiles, resident);
  }
  hipLaunchKernelGGL((apply_tp_mfma<P, TX, TY, NW, PERSIST, SPLIT>), dim3(static_cast<unsigned>(grid)),
                     dim3(C::THREADS), 0, s, args);
  return hip_check(hipGetLastError(), "apply (mfma) launch");
}

// Tile shapes: element tiles of ~32 x 32 nodes (4 waves, persistent) for large meshes; ~16 x 16
// nodes for meshes too small to give every CU several workgroups (4 waves with the K and G
// chains as separate tasks; SEM_MFMA_TILE=1 selects the earlier 2-wave variant).
template <int P>
static int launch_apply_mfma_auto(const ApplyArgs& args, const sem_handle* h, hipStream_t s) {
  constexpr int TL = (32 / P) > 0 ? 32 / P : 1;
  constexpr int TS = (16 / P) > 0 ? 16 / P : 1;
  const long long big_tiles = static_cast<long long>((h->ex_end - h->ex_begin + TL - 1) / TL) * ((h->ney + TL - 1) / TL);
  if (big_tiles >= 4 * 256) return launch_apply_mfma<P, TL, TL, 4, true, false>(args, h, s);
  return launch_apply_mfma<P, TS, TS, 4, false, true>(args, h, s);   // the round-4 default
}

// =========================================================================== column kernel
//
// Single-phase VALU kernel.  Thread = (element column e of the tile, row split s, column c);
// lanes run along columns (coalesced global I/O), so within a wave the element-local row i
// is uniform: the x-direction coefficients K_s[i][.] / G_s[i][.] are instruction immediates
// and the x-window T[eP-P .. eP+P][c] is loaded once into registers and reused by every row.
// The y-direction needs the coefficient row of the column's local index j = gy mod P, which
// differs per lane but is fixed for the thread: it is loaded once into registers.  No
// intermediate buffers, one barrier per tile.
template <int P, int TX, int BY, int RS>
struct CCfg {
  static constexpr int n = P + 1;
  static constexpr int RP = P / RS;                   // rows per thread
  static constexpr int THREADS = TX * RS * BY;
  static constexpr int BX = TX * P;
  static constexpr int RX = BX + P + 1;               // staged lines   [gx0-P, gx0+BX]
  static constexpr int RY = BY + 2 * P + 1;           // staged columns [gy0-P, gy0+BY+P]
  static constexpr int PT = RY;                       // lanes read along a row: any pitch is conflict-free
  static constexpr int NSTAGE = (RX * RY + THREADS - 1) / THREADS;
  static_assert(P % RS == 0, "row splits must divide P");
  static_assert((BY * RS) % 64 == 0, "a wave must hold one (element column, split)");
  static_assert(THREADS <= 1024, "workgroup too large");
};

template <int P, int TX, int BY, int RS>
__global__ __launch_bounds__((CCfg<P, TX, BY, RS>::THREADS)) void apply_tp_col(const ApplyArgs a) {
  using C = CCfg<P, TX, BY, RS>;
  constexpr int n = C::n, RP = C::RP;
  __shared__ double Ts[C::RX * C::PT];
  __shared__ double ws[n];

  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q = nb >> 3, rem = nb & 7;
  const int L = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  const int tx = L / a.tiles_y, ty = L - tx * a.tiles_y;
  const int lb0 = static_cast<int>(a.line_begin), lb1 = static_cast<int>(a.line_end), NY = static_cast<int>(a.NY);
  const int m0 = a.ex_begin + tx * TX, m1 = min(m0 + TX, a.ex_end);
  const int gx0 = m0 * P, gy0 = ty * BY;
  const int BYo = min(BY, NY - 1 - gy0);     // owned columns without the domain's closing one
  const bool lasty = gy0 + BY >= NY - 1;
  const int tid = threadIdx.x;
  const int c = tid % BY;
  // (element column, split) are wave-uniform by construction (BY*RS is a multiple of 64):
  // readfirstlane puts them and everything derived per row (line, weights, flags) in SGPRs
  const int s = __builtin_amdgcn_readfirstlane((tid / BY) % RS);
  const int e = __builtin_amdgcn_readfirstlane(tid / (BY * RS));
  const int me = m0 + e;                      // this thread's element column
  const bool hasE = me < m1;

  const double wreg = a.tab[2 * n * n + min(tid, n - 1)];
  // ---- stage x (clamped, unconditional loads)
  double st[C::NSTAGE];
#pragma unroll
  for (int k = 0; k < C::NSTAGE; ++k) {
    const int idx = min(tid + k * C::THREADS, C::RX * C::RY - 1);
    const int rr = idx / C::RY, cc = idx - rr * C::RY;
    const int gx = min(max(gx0 - P + rr, lb0), lb1);
    const int gy = min(max(gy0 - P + cc, 0), NY - 1);
    st[k] = a.x[(gx - lb0) * NY + gy];
  }
  // ---- this thread's rows: u, v prefetch (clamped addresses)
  const int nmax = a.n_local32 - 1;
  double pu[RP + 1], pv[RP + 1];
#pragma unroll
  for (int ii = 0; ii <= RP; ++ii) {
    const int p = min((me * P + s * RP + ii - lb0) * NY + gy0 + c, nmax);
    pu[ii] = a.cu ? a.cu[p] : 1.0;
    pv[ii] = a.cv ? a.cv[p] : 1.0;
  }
  // the y coefficient rows of this thread's column, loaded with the tile (no wait before staging)
  double rK0[n], rG0[n];
  auto coef_rows = [&](int cc, double (&rK)[n], double (&rG)[n]) {
    const int gy = gy0 + cc;
    const int j = gy % P;
    const bool hasRy = gy / P < a.ney;
#pragma unroll
    for (int l = 0; l <= P; ++l) {
      const int idx = (hasRy ? j : 0) * n + l;
      const double kv = a.tab[idx], gv = a.tab[n * n + idx];
      rK[l] = hasRy ? kv : 0.0;
      rG[l] = hasRy ? gv : 0.0;
    }
  };
  coef_rows(c, rK0, rG0);
  if (tid < n) ws[tid] = wreg;
#pragma unroll
  for (int k = 0; k < C::NSTAGE; ++k) {
    const int idx = tid + k * C::THREADS;
    if (idx < C::RX * C::RY) {
      const int rr = idx / C::RY, cc = idx - rr * C::RY;
      Ts[rr * C::PT + cc] = st[k];
    }
  }
  __syncthreads();

  // per-column (per-lane) y data: local index j, right/left element flags, coefficient rows
  auto column = [&](int cc, double (&uu)[RP + 1], double (&vv)[RP + 1], const double (&rK)[n], const double (&rG)[n]) {
    const int gy = gy0 + cc;
    const int j = gy % P, ne = gy / P;
    const bool hasLy = j == 0 && ne > 0;
    const double my = wsum<P>(gy, 0, a.ney, ws);
    // x-window of this element column along column cc: T[meP-P+k][gy], k = 0..2P
    double xt[2 * P + 1];
#pragma unroll
    for (int k = 0; k <= 2 * P; ++k) xt[k] = Ts[(e * P + k) * C::PT + P + cc];
    const bool hasLx = me - 1 >= a.ex_begin, lastE = me == a.ex_end - 1;
    const double* trow0 = &Ts[P + cc - j];  // y-window base of the right element (row offset added below)
    auto row = [&](auto I, double uval, double vval) {
      constexpr int i = decltype(I)::value;
      const int rl = e * P + i;  // line index within the tile
      const int gx = gx0 + rl;
      double kx, gxv;
      contract_row<P, i>(xt, hasLx, kx, gxv);
      // y-direction for line gx
      const double* tr = trow0 + (P + rl) * C::PT;
      double ky = 0.0, gyv = 0.0;
      if (hasLy) row_dot<P, P>(tr - P, ky, gyv, std::make_integer_sequence<int, P + 1>{});  // left element, row P
#pragma unroll
      for (int l = 0; l <= P; ++l) {
        const double t = tr[l];
        ky = fma(rK[l], t, ky);
        gyv = fma(rG[l], t, gyv);
      }
      const int p = (gx - lb0) * NY + gy;
      const double xv = xt[P + i];
      const double mx = wsum<P>(gx, a.ex_begin, a.ex_end, ws);
      double z = 0.0;
      if (a.cK != 0.0) z = a.cK * fma(a.sx * my, kx, a.sy * mx * ky);
      if (a.cM != 0.0) z = fma(a.cM * a.hxy * mx * my, xv, z);
      if (a.cX != 0.0) z = fma(a.cX * uval, a.hy * my * gxv, z);
      if (a.cY != 0.0) z = fma(a.cY * vval, a.hx * mx * gyv, z);
      const bool own = !(gx == lb1 && a.ex_end < a.nex);  // pointwise terms: right-hand owner only
      if (a.has_e1 && own) z = fma(a.cE * a.ea[p], a.eb[p], z);
      if (a.has_e2 && own) z = fma(a.cE * a.ec[p], a.ed[p], z);
      if (a.cA != 0.0 && own) z = fma(a.cA, a.y[p], z);
      if (a.dir_mode != SEM_DIR_NONE) {
        const bool isd = a.mask ? (a.mask[p] != 0)
                                : (((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NXg - 1) ||
                                   ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == NY - 1));
        if (isd) {
          const bool owner = !(gx == lb1 && a.ex_end < a.nex);
          if (!owner)
            z = 0.0;
          else if (a.dir_mode == SEM_DIR_IDENTITY)
            z = xv - (a.dval ? a.dval[p] : 0.0);
          else
            z = a.dval[p];
        }
      }
      a.y[p] = z;
    };
    // rows of this split (wave-uniform split -> compile-time rows), plus the closing line
    auto rows = [&](auto S) {
      constexpr int s0 = decltype(S)::value * RP;
      for_rows(std::make_integer_sequence<int, RP>{}, [&](auto II) {
        constexpr int ii = decltype(II)::value;
        row(std::integral_constant<int, s0 + ii>{}, uu[ii], vv[ii]);
      });
      if constexpr (decltype(S)::value == RS - 1) {
        if (lastE) row(std::integral_constant<int, P>{}, uu[RP], vv[RP]);
      }
    };
    for_rows(std::make_integer_sequence<int, RS>{}, [&](auto S) {
      if (s == decltype(S)::value) rows(S);
    });
  };
  if (hasE && c < BYo) column(c, pu, pv, rK0, rG0);
  if (hasE && lasty && c == 0) {  // the domain's closing column
    double qu[RP + 1], qv[RP + 1], rK1[n], rG1[n];
    coef_rows(BYo, rK1, rG1);
#pragma unroll
    for (int ii = 0; ii <= RP; ++ii) {
      const int p = min((me * P + s * RP + ii - lb0) * NY + gy0 + BYo, nmax);
      qu[ii] = a.cu ? a.cu[p] : 1.0;
      qv[ii] = a.cv ? a.cv[p] : 1.0;
    }
    column(BYo, qu, qv, rK1, rG1);
  }
}

template <int P, int TX, int BY, int RS>
static int launch_apply_col(const ApplyArgs& args_in, const sem_handle* h, hipStream_t s) {
  using C = CCfg<P, TX, BY, RS>;
  ApplyArgs args = args_in;
  const int ncols = h->ex_end - h->ex_begin;
  args.tiles_x = (ncols + TX - 1) / TX;
  args.tiles_y = static_cast<int>((h->NY - 1 + BY - 1) / BY);
  const long long nblk = static_cast<long long>(args.tiles_x) * args.tiles_y;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return set_error(SEM_EINVAL, "mesh too large for one launch");
  hipLaunchKernelGGL((apply_tp_col<P, TX, BY, RS>), dim3(static_cast<unsigned>(nblk)), dim3(C::THREADS), 0, s, args);
  return hip_check(hipGetLastError(), "apply (column) launch");
}

template <int P>
static int launch_apply_col_auto(const ApplyArgs& args, const sem_handle* h, hipStream_t s) {
  // 2 element columns x 64 lines, no row split (the other tiles of rounds 1-2 lost their A/B; retired in round 6)
  return launch_apply_col<P, 2, 64, 1>(args, h, s);
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

// Every launcher runs on the handle's device: a handle used while another device is current
// would launch there against this device's pointers, so it is an error (SEM_EINVAL).
static int on_device(const sem_handle* h) {
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess) return sem::set_error(SEM_EHIP, "hipGetDevice failed");
  if (cur != h->device)
    return sem::set_error(SEM_EINVAL, "handle belongs to device " + std::to_string(h->device) + " but device " +
                                          std::to_string(cur) + " is current");
  return SEM_OK;
}

extern "C" {

int sem_abi_version(void) { return SEM_ABI_VERSION; }

static bool retired_knob(int knob) {
  return knob == SEM_TUNE_RETIRED_1 || knob == SEM_TUNE_RETIRED_3 || knob == SEM_TUNE_RETIRED_5 ||
         (knob >= SEM_TUNE_RETIRED_8 && knob <= SEM_TUNE_RETIRED_12);
}

int sem_set_tuning(int knob, int value) {
  if (knob < 0 || knob >= SEM_TUNE_COUNT) return set_error(SEM_EINVAL, "unknown tuning knob");
  if (retired_knob(knob)) return set_error(SEM_EINVAL, "retired tuning knob (round 6)");
  tuning().v[knob] = value;
  return SEM_OK;
}

int sem_get_tuning(int knob, int* value) {
  if (knob < 0 || knob >= SEM_TUNE_COUNT || !value) return set_error(SEM_EINVAL, "unknown tuning knob");
  *value = tuning().v[knob];
  return SEM_OK;
}
const char* sem_last_error(void) { return last_error(); }
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
  if (d->algo < SEM_ALGO_AUTO || d->algo > SEM_ALGO_BAND) return set_error(SEM_EINVAL, "bad algo");
  // SEM_ALGO_MFMA: the band-form MFMA kernel (apply_bmfma, P <= 16; round 5); SEM_MFMA_TILE = 1, 2, 3 select the
  // element-block MFMA kernel of rounds 1-4 (apply_tp_mfma, P <= 15) for A/B
  const bool legacy_mfma = tune(SEM_TUNE_MFMA_TILE) != 0;
  if (d->algo == SEM_ALGO_MFMA && legacy_mfma && h->P > 15)
    return set_error(SEM_EUNSUPPORTED, "the element-block MFMA path needs P <= 15");
  const bool ranged = d->pos_end > 0;
  if (ranged && (d->pos_begin < 0 || d->pos_begin >= d->pos_end || d->pos_end > h->ex_end - h->ex_begin + 1))
    return set_error(SEM_EINVAL, "element-position range outside [0, ex_end - ex_begin + 1)");
  if (ranged && d->algo != SEM_ALGO_AUTO && d->algo != SEM_ALGO_BAND)
    return set_error(SEM_EUNSUPPORTED, "element-position ranges are implemented by the band kernel only");
  if (int st = on_device(h)) return st;
  ApplyArgs a{};
  a.pos0 = ranged ? d->pos_begin : 0;
  a.pos1 = ranged ? d->pos_end : 0;
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
  a.n_local32 = static_cast<int>(std::min<int64_t>(h->n_local, 0x7fffffff));
  a.diag = kDiag ? diag_bits() : 0;
  a.stamps = (kDiag && (a.diag & 8)) ? diag_stamps() : nullptr;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // Buffer-resource kernels (MFMA, band) address the local vector with 32-bit byte offsets.
  // AUTO, measured on MI355X (tools/kbench.py): the band kernel on every mesh whose local vector
  // fits its 32-bit buffer offsets (it beats the other kernels from 64^2 to 1024^2 elements);
  // the single-phase column kernel above that.
  const bool fits32 = h->n_local < (int64_t(1) << 28);
  // the band kernel's staging offsets (an absent column at 2^31 + a line offset) stay outside the buffer when
  // n_local + (P + 1) N_y <= 2^28 (apply_band.hip, band_body)
  const bool band_auto = band_fits(h);
  if (ranged && !band_auto) return set_error(SEM_EUNSUPPORTED, "element-position ranges need n_local + (P+1) N_y < 2^28");
  if (d->algo == SEM_ALGO_BAND || (d->algo == SEM_ALGO_AUTO && band_auto)) {
    if (!band_auto) return set_error(SEM_EUNSUPPORTED, "band path needs n_local + (P+1) N_y < 2^28");
    return launch_apply_band(a, h, s);
  }
  const bool use_col = d->algo == SEM_ALGO_COLUMN || d->algo == SEM_ALGO_AUTO;
  if (use_col) {
    switch (h->P) {
#define SEM_CCASE(PP) \
  case PP:            \
    return launch_apply_col_auto<PP>(a, h, s);
      SEM_CCASE(1) SEM_CCASE(2) SEM_CCASE(3) SEM_CCASE(4) SEM_CCASE(5) SEM_CCASE(6) SEM_CCASE(7) SEM_CCASE(8)
      SEM_CCASE(9) SEM_CCASE(10) SEM_CCASE(11) SEM_CCASE(12) SEM_CCASE(13) SEM_CCASE(14) SEM_CCASE(15) SEM_CCASE(16)
#undef SEM_CCASE
      default:
        break;
    }
  }
  const bool mfma = d->algo == SEM_ALGO_MFMA || d->algo == SEM_ALGO_AUTO;
  if (mfma && !fits32) return set_error(SEM_EUNSUPPORTED, "MFMA path needs n_local < 2^28");
  if (d->algo == SEM_ALGO_MFMA && !legacy_mfma) return launch_apply_bmfma(a, h, s);
  if (mfma) {
    switch (h->P) {
#define SEM_MCASE(PP) \
  case PP:            \
    return launch_apply_mfma_auto<PP>(a, h, s);
      SEM_MCASE(1) SEM_MCASE(2) SEM_MCASE(3) SEM_MCASE(4) SEM_MCASE(5) SEM_MCASE(6) SEM_MCASE(7) SEM_MCASE(8)
      SEM_MCASE(9) SEM_MCASE(10) SEM_MCASE(11) SEM_MCASE(12) SEM_MCASE(13) SEM_MCASE(14) SEM_MCASE(15)
#undef SEM_MCASE
      default:
        break;
    }
  }
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

int sem_kernel_name(const sem_handle* h, int algo, char* buf, int len) {
  if (!h || !buf || len < 1) return set_error(SEM_EINVAL, "bad arguments");
  std::string name;
  const int P = h->P;
  if (algo == SEM_ALGO_BAND || (algo == SEM_ALGO_AUTO && band_fits(h))) {
    name = band_kernel_name(P, h->n_local);
  } else if (algo == SEM_ALGO_COLUMN || algo == SEM_ALGO_AUTO) {
    name = "sem::apply_tp_col<" + std::to_string(P) + ", 2, 64, 1>";
  } else if (algo == SEM_ALGO_MFMA && tune(SEM_TUNE_MFMA_TILE) == 0) {
    name = bmfma_kernel_name(P);
  } else if ((algo == SEM_ALGO_MFMA || algo == SEM_ALGO_AUTO) && P <= 15) {
    const int TL = std::max(1, 32 / P), TS = std::max(1, 16 / P);
    const long long big = static_cast<long long>((h->ex_end - h->ex_begin + TL - 1) / TL) * ((h->ney + TL - 1) / TL);
    name = big >= 4 * 256 ? "sem::apply_tp_mfma<" + std::to_string(P) + ", " + std::to_string(TL) + ", " +
                                std::to_string(TL) + ", 4, true, false>"
                          : "sem::apply_tp_mfma<" + std::to_string(P) + ", " + std::to_string(TS) + ", " +
                                std::to_string(TS) + ", 4, false, true>";
  } else {
    name = "sem::apply_tp_valu<" + std::to_string(P) + ">";
  }
  std::snprintf(buf, static_cast<size_t>(len), "%s", name.c_str());
  return SEM_OK;
}

int sem_gather_elements(sem_handle* h, const double* u, double* ue, void* stream) {
  if (!h || !u || !ue) return set_error(SEM_EINVAL, "null argument");
  if (int st = on_device(h)) return st;
  const int n = h->P + 1;
  const int64_t total = static_cast<int64_t>(h->ex_end - h->ex_begin) * h->ney * n * n;
  hipLaunchKernelGGL(gather_kernel, dim3(grid_for(total, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), u,
                     ue, h->P, h->ney, h->ex_begin, h->line_begin, h->NY, total);
  return hip_check(hipGetLastError(), "gather launch");
}

int sem_dss(sem_handle* h, const double* ae, double* out, void* stream) {
  if (!h || !ae || !out) return set_error(SEM_EINVAL, "null argument");
  if (static_cast<const void*>(ae) == static_cast<const void*>(out)) return set_error(SEM_EINVAL, "in/out alias");
  if (int st = on_device(h)) return st;
  hipLaunchKernelGGL(dss_kernel, dim3(grid_for(h->n_local, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     ae, out, h->P, h->ney, h->ex_begin, h->ex_end, h->line_begin, h->NY, h->n_local);
  return hip_check(hipGetLastError(), "dss launch");
}

int sem_eval_interpolation(sem_handle* h, const double* ue, int na, const int* m_idx, const double* Sx, int nb,
                           const int* n_idx, const double* Sy, double* out, void* stream) {
  if (!h || !ue || !out || na < 0 || nb < 0) return set_error(SEM_EINVAL, "bad interpolation arguments");
  if (na == 0 || nb == 0) return SEM_OK;
  if (!m_idx || !Sx || !n_idx || !Sy) return set_error(SEM_EINVAL, "null interpolation table");
  if (int st = on_device(h)) return st;
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
  if ((st = on_device(h))) return st;
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
  if ((st = on_device(h))) return st;
  hipLaunchKernelGGL(iface_unpack_kernel, dim3(grid_for(h->NY, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), buf, y, h->NY, L, static_cast<int64_t>(0), R,
                     h->n_local - h->NY);
  return hip_check(hipGetLastError(), "interface unpack launch");
}

}  // extern "C"
