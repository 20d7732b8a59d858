// Banded-assembly apply kernel for gfx950 (SEM_ALGO_BAND).
//
// Same operator as the other apply kernels -- the assembled global operators of
// Solvers/SEM.py (mass :170-183, stiffness :186-203, gradient :206-223, convection
// :226-245 as contracted at ConvectionDiffusion_Solver.py:82-87,112-119) -- but written
// against the *assembled* 1-D operators instead of per-element blocks:
//
//     (K x)[gx,gy] = (dy/dx) My[gy] sum_k Kx[gx][k] x[k][gy] + (dx/dy) Mx[gx] sum_l Ky[gy][l] x[gx][l]
//
// where Kx (resp. Gx) is the 1-D direct-stiffness sum of K_s (G_s) over the element
// columns holding a line (SEM.py:196-202): row gx of an element-interior node is one row
// of K_s over that element's P+1 nodes; the row of a node shared by two elements is
// K_s[P][.] over the left element plus K_s[0][.] over the right one.  Every owned node's
// result is therefore one banded dot product per direction -- no element halo is
// recomputed and no element-local results are summed afterwards.
//
// One workgroup = one tile of TXE x TYE elements (BX = TXE*P lines, BY = TYE*P columns).
// Waves have fixed roles, chosen so that every coefficient is wave-uniform (compile-time
// constants, gll_consts.h) and every global access is coalesced along y:
//   X waves    lane = column c, wave = (element column a, row split s): the x-direction
//              rows of element a at column c from a (2P+1)-node window held in registers;
//              afterwards the epilogue of those nodes (coalesced loads / stores).
//   Y waves    lane = (line r, element b), wave = column split h: the y-direction rows of
//              element b on line r from a (2P+1)-node window; results (scaled) -> LDS.
// The local domain's closing line (x = line_end) and column (y = NY-1) are row / column 0 of a
// *ghost* element past the last one: tiles run over ncols+1 x ney+1 element positions, and a
// ghost element contributes only its row / column 0 (left element only).  Every node therefore
// goes through the same wave-uniform fast path, and the ghost tiles are light.
// Barriers: staged tile in LDS -> X and Y contractions run concurrently -> X epilogue.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "apply_common.h"

namespace sem {


// ---- Even-odd (centro-symmetric) form of one element's rows.
// G_s is exactly centro-antisymmetric (G[P-i][P-l] = -G[i][l], GLL.py:62-70); K_s is
// centro-symmetric to rounding (|K[i][l] - K[P-i][P-l]| <= 1.5 ulp), and is used in its symmetrised
// form Ks = (K + centro(K))/2, a change far below the 1e-13 parity tolerance.  With e_m =
// t_m + t_{P-m}, o_m = t_m - t_{P-m} (m < (P+1)/2) the rows i and P-i of an element share
//     E_i = sum_m S_i[m] e_m (+ A[i][P/2] t_{P/2}),  O_i = sum_m D_i[m] o_m,
//     S_i[m] = (A[i][m] + A[i][P-m])/2,  D_i[m] = (A[i][m] - A[i][P-m])/2,
// and y_i = E_i + O_i, y_{P-i} = E_i - O_i (K), O_i - E_i (G): about half the multiply-adds and
// half the coefficient constants of the direct rows.  The shared-node row 0 folds the left
// element's row P onto row 0 the same way: Ks[0][m] (t_{P+m} + t_{P-m}), G[0][m] (t_{P+m} - t_{P-m}).
template <int P>
struct EOC {
  static constexpr int n = P + 1, H = (P + 1) / 2, c = P / 2, NP = (P - 1) / 2;
  static constexpr bool EVEN = P % 2 == 0;
  static constexpr double K(int i, int l) { return GllConst<P>::K[i * n + l]; }
  static constexpr double G(int i, int l) { return GllConst<P>::G[i * n + l]; }
  static constexpr double Ks(int i, int l) { return 0.5 * (K(i, l) + K(P - i, P - l)); }
  static constexpr double SK(int i, int m) { return 0.5 * (Ks(i, m) + Ks(i, P - m)); }
  static constexpr double DK(int i, int m) { return 0.5 * (Ks(i, m) - Ks(i, P - m)); }
  static constexpr double SG(int i, int m) { return 0.5 * (G(i, m) + G(i, P - m)); }
  static constexpr double DG(int i, int m) { return 0.5 * (G(i, m) - G(i, P - m)); }
};

// Work items of an element's rows: item 0 = row 0 (the shared node; it also folds in the left
// element's row P), items 1..NP = the mirror pairs (k, P-k), item NP+1 = the centre row P/2 (even
// P).  They are dealt to NS splits (one thread each) longest-first by VALU cost.
template <int P, int NS>
struct EPlan {
  static constexpr int NP = EOC<P>::NP, H = EOC<P>::H;
  static constexpr bool EVEN = EOC<P>::EVEN;
  static constexpr int NITEMS = 1 + NP + (EVEN ? 1 : 0);
  static constexpr int code(int k) { return k == 0 ? 0 : (k <= NP ? k : -1); }
  static constexpr int size(int k) { return code(k) > 0 ? 2 : 1; }
  static constexpr int cost(int k) { return code(k) == 0 ? 4 * P + 2 : (code(k) > 0 ? 4 * H + 8 : 2 * H + 2); }
  struct Deal {
    int of[24];
  };
  static constexpr Deal deal() {
    Deal d{};
    int load[NS] = {};
    bool done[24] = {};
    for (int step = 0; step < NITEMS; ++step) {
      int best = -1;
      for (int k = 0; k < NITEMS; ++k)
        if (!done[k] && (best < 0 || cost(k) > cost(best))) best = k;
      int sp = 0;
      for (int q = 1; q < NS; ++q)
        if (load[q] < load[sp]) sp = q;
      d.of[best] = sp;
      load[sp] += cost(best);
      done[best] = true;
    }
    return d;
  }
  static constexpr Deal DEAL = deal();
  static constexpr bool in_split(int k, int sp) { return DEAL.of[k] == sp; }
  static constexpr int nrows(int sp) {
    int r = 0;
    for (int k = 0; k < NITEMS; ++k)
      if (in_split(k, sp)) r += size(k);
    return r;
  }
  static constexpr int slot(int sp, int k) {  // first slot of item k within split sp
    int r = 0;
    for (int q = 0; q < k; ++q)
      if (in_split(q, sp)) r += size(q);
    return r;
  }
  static constexpr int row(int sp, int sl) {  // element-local row of slot sl of split sp (-1: none)
    for (int k = 0; k < NITEMS; ++k) {
      if (!in_split(k, sp)) continue;
      const int f = slot(sp, k), it = code(k);
      if (sl == f) return it == 0 ? 0 : (it < 0 ? P / 2 : it);
      if (it > 0 && sl == f + 1) return P - it;
    }
    return -1;
  }
  static constexpr int nrmax() {
    int m = 0;
    for (int sp = 0; sp < NS; ++sp)
      if (nrows(sp) > m) m = nrows(sp);
    return m;
  }
  static constexpr bool needs_left(int sp) { return in_split(0, sp); }
  static constexpr bool needs_eo(int sp) {
    for (int k = 1; k < NITEMS; ++k)
      if (in_split(k, sp)) return true;
    return false;
  }
};

// Coefficient list of split S, in the order eo_rows consumes them (the DPP variant keeps them 16
// per VGPR, lane l of every 16-lane row holding entry l, and broadcasts entry k with
// v_fmac_f64_dpp row_newbcast:k -- one VALU operand instead of two s_mov_b32 per coefficient).
// Per item: row 0 -> Ks(0,m), G(0,m) for m = 1..P; a pair -> SK, DK, SG, DG for m < H (+ Ks(it,c),
// G(it,c) for even P); the centre row -> SK(c,m), DG(c,m) for m < H, then Ks(c,c), G(c,c).
template <int P, int NS>
struct CList {
  using E = EOC<P>;
  using L = EPlan<P, NS>;
  static constexpr int H = E::H;
  static constexpr int count(int kk) {
    const int it = L::code(kk);
    return it == 0 ? 2 * P : (it > 0 ? 4 * H + (E::EVEN ? 2 : 0) : 2 * H + 2);
  }
  static constexpr int base(int S, int kk) {
    int b = 0;
    for (int q = 0; q < kk; ++q)
      if (L::in_split(q, S)) b += count(q);
    return b;
  }
  static constexpr int size(int S) { return base(S, L::NITEMS); }
  static constexpr int nmax() {
    int m = 0;
    for (int S = 0; S < NS; ++S) m = size(S) > m ? size(S) : m;
    return m;
  }
  static constexpr int NCV = (nmax() + 15) / 16;  // VGPR pairs per lane
  static constexpr int NPAD = 16 * (NCV > 0 ? NCV : 1);
  static constexpr double value(int S, int j) {  // entry j of split S
    for (int kk = 0; kk < L::NITEMS; ++kk) {
      if (!L::in_split(kk, S)) continue;
      const int b = base(S, kk);
      if (j < b || j >= b + count(kk)) continue;
      const int o = j - b, it = L::code(kk);
      if (it == 0) return (o & 1) ? E::G(0, o / 2 + 1) : E::Ks(0, o / 2 + 1);
      if (it > 0) {
        if (o < 4 * H) {
          const int m = o / 4, wh = o % 4;
          return wh == 0 ? E::SK(it, m) : wh == 1 ? E::DK(it, m) : wh == 2 ? E::SG(it, m) : E::DG(it, m);
        }
        return o == 4 * H ? E::Ks(it, E::c) : E::G(it, E::c);
      }
      if (o < 2 * H) return (o & 1) ? E::DG(E::c, o / 2) : E::SK(E::c, o / 2);
      return o == 2 * H ? E::Ks(E::c, E::c) : E::G(E::c, E::c);
    }
    return 0.0;
  }
  struct Tab {
    double v[NS * NPAD];
  };
  static constexpr Tab make() {
    Tab t{};
    for (int S = 0; S < NS; ++S)
      for (int j = 0; j < NPAD; ++j) t.v[S * NPAD + j] = value(S, j);
    return t;
  }
};

template <int P, int NS>
__device__ const typename CList<P, NS>::Tab kBandCoef = CList<P, NS>::make();

// acc + c * x with the coefficient of entry IDX of split S's list: CM = 0 an fp64 immediate (two
// s_mov_b32 into an SGPR pair), CM = 1 a DPP broadcast from the split's VGPR-resident list (only valid
// with every lane of the wave active: a DPP read of a disabled lane does not return its value).  (Round 2's
// CM = 2, scalar loads from a constant-memory copy, measured no faster and was retired in round 6.)
template <int CM, int P, int NS, int S, int IDX, int NCV>
__device__ __forceinline__ double cfma(const double (&cv)[NCV], double c, double x, double acc) {
  if constexpr (CM == 1) {
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc)
        : "v"(cv[IDX / 16]), "v"(x), "n"(IDX % 16));
    return acc;
  } else {
    return fma(c, x, acc);
  }
}

// Rows of split S of one element from a (2P+1)-node window t (t[P..2P] = the element, t[0..P] = the
// left neighbour; absent elements are zero in the staged tile).  fk = hasL + hasR and
// fg = hasR - hasL weight the shared node t[P] in row 0.  Results go to slots (EPlan order).
template <int P, int NS, int S, int CM, int NR, int NCV>
__device__ __forceinline__ void eo_rows(const double (&t)[2 * P + 1], double fk, double fg, double (&k)[NR],
                                        double (&g)[NR], const double (&cv)[NCV]) {
  using E = EOC<P>;
  using L = EPlan<P, NS>;
  using CL = CList<P, NS>;
  constexpr int H = E::H;
  double e[H], o[H];
  // row 0 (which reads the whole window) before the even / odd sums (which read t[P..2P] only): the left half of
  // the window dies before e, o are formed (round 6: 8 fewer live VGPRs at P = 8)
  auto form_eo = [&]() {
    if constexpr (L::needs_eo(S)) {
#pragma unroll
      for (int m = 0; m < H; ++m) {
        e[m] = t[P + m] + t[2 * P - m];
        o[m] = t[P + m] - t[2 * P - m];
      }
    }
  };
  if constexpr (!L::in_split(0, S)) form_eo();
  for_rows(std::make_integer_sequence<int, L::NITEMS>{}, [&](auto KI) {
    constexpr int kk = decltype(KI)::value;
    constexpr int it = L::code(kk);
    if constexpr (kk == 1 && L::in_split(0, S)) form_eo();
    if constexpr (L::in_split(kk, S)) {
      constexpr int sl = L::slot(S, kk);
      constexpr int cb = CL::base(S, kk);
      if constexpr (it == 0) {  // shared-node row 0 (+ the left element's row P)
        constexpr double k00 = E::Ks(0, 0), g00 = E::G(0, 0);
        double kv = (k00 * fk) * t[P], gv = (g00 * fg) * t[P];
        for_rows(std::make_integer_sequence<int, P>{}, [&](auto MI) {
          constexpr int m = decltype(MI)::value + 1;
          constexpr double km = E::Ks(0, m), gm = E::G(0, m);
          kv = cfma<CM, P, NS, S, cb + 2 * (m - 1)>(cv, km, t[P + m] + t[P - m], kv);
          gv = cfma<CM, P, NS, S, cb + 2 * (m - 1) + 1>(cv, gm, t[P + m] - t[P - m], gv);
        });
        k[sl] = kv;
        g[sl] = gv;
      } else if constexpr (it > 0) {  // mirror pair (it, P-it)
        double Ek = 0.0, Ok = 0.0, Eg = 0.0, Og = 0.0;
        for_rows(std::make_integer_sequence<int, H>{}, [&](auto MI) {
          constexpr int m = decltype(MI)::value;
          constexpr double sk = E::SK(it, m), dk = E::DK(it, m), sg = E::SG(it, m), dg = E::DG(it, m);
          Ek = cfma<CM, P, NS, S, cb + 4 * m>(cv, sk, e[m], Ek);
          Ok = cfma<CM, P, NS, S, cb + 4 * m + 1>(cv, dk, o[m], Ok);
          Eg = cfma<CM, P, NS, S, cb + 4 * m + 2>(cv, sg, e[m], Eg);
          Og = cfma<CM, P, NS, S, cb + 4 * m + 3>(cv, dg, o[m], Og);
        });
        if constexpr (E::EVEN) {
          constexpr double kc_ = E::Ks(it, E::c), gc_ = E::G(it, E::c);
          Ek = cfma<CM, P, NS, S, cb + 4 * H>(cv, kc_, t[P + E::c], Ek);
          Eg = cfma<CM, P, NS, S, cb + 4 * H + 1>(cv, gc_, t[P + E::c], Eg);
        }
        k[sl] = Ek + Ok;
        k[sl + 1] = Ek - Ok;
        g[sl] = Eg + Og;
        g[sl + 1] = Og - Eg;
      } else {  // centre row P/2: Ks symmetric, G antisymmetric about it
        double kv = 0.0, gv = 0.0;
        for_rows(std::make_integer_sequence<int, H>{}, [&](auto MI) {
          constexpr int m = decltype(MI)::value;
          constexpr double sk = E::SK(E::c, m), dg = E::DG(E::c, m);
          kv = cfma<CM, P, NS, S, cb + 2 * m>(cv, sk, e[m], kv);
          gv = cfma<CM, P, NS, S, cb + 2 * m + 1>(cv, dg, o[m], gv);
        });
        constexpr double kcc = E::Ks(E::c, E::c), gcc = E::G(E::c, E::c);
        kv = cfma<CM, P, NS, S, cb + 2 * H>(cv, kcc, t[P + E::c], kv);
        if constexpr (gcc != 0.0) gv = cfma<CM, P, NS, S, cb + 2 * H + 1>(cv, gcc, t[P + E::c], gv);
        k[sl] = kv;
        g[sl] = gv;
      }
    }
  });
}

template <int P, int TXE, int TYE, int NS>
struct BCfg {
  static constexpr int n = P + 1;
  static constexpr int BX = TXE * P, BY = TYE * P;      // lines / columns of the tile's element positions
  static constexpr int XW = (BY + 63) / 64;             // waves per (element position, split) X group
  static constexpr int LW = 64 * XW;                    // lanes per tile line (X role and epilogue)
  static constexpr int NXW = TXE * NS * XW;             // X waves
  static constexpr int YL = BX * TYE;                   // Y lanes per split: (line, element position)
  static constexpr int YW = (YL + 63) / 64;
  static constexpr int NYW = NS * YW;                   // Y waves
  static constexpr int NW = NXW + NYW;
  static constexpr int THREADS = 64 * NW;
  static constexpr int RP = EPlan<P, NS>::nrmax();      // rows (columns) per X (Y) thread
  static constexpr int RX = BX + P + 1, RY = BY + P + 1;  // staged lines [gx0-P, gx0+BX] x cols [gy0-P, gy0+BY]
  static constexpr int PT = RY | 1;                     // odd pitch
  static constexpr int PY = LW + 1;                     // result tiles: BX lines x LW columns
  static constexpr int NSTAGE = (RX * RY + THREADS - 1) / THREADS;
  static constexpr int NE = (BX * LW + THREADS - 1) / THREADS;  // epilogue nodes per thread
  // staging (round 6): wave w stages window lines w + NW k, k < NSL (lanes = columns 0..63), and the columns
  // 64..RY-1 of its lines (RYX per line) in NXL further loads
  static constexpr int NSL = (RX + NW - 1) / NW;
  static constexpr int RYX = RY - 64;
  static constexpr int NXL = (NSL * RYX + 63) / 64;
  static_assert(RY > 64 && RY <= 128, "staging assumes 64 < RY <= 128 window columns");
  static_assert(NS >= 1 && NS <= 4, "1 to 4 splits");
  static_assert(THREADS <= 1024, "workgroup too large");
};

// Kernel arguments of the band kernel: compact, the fields every wave needs first at the
// front (two s_load_dwordx16 fetch them), all epilogue factors fused on the host.  Every field
// is read once at kernel entry; a kernarg load sunk into a later phase is a full memory round
// trip on that phase's critical path.
struct BandArgs {
  const double* x;
  double* y;
  const double* cu;
  const double* cv;
  double fKx, fKy, fM, fX, fY;  // cK*dy/dx, cK*dx/dy, cM*dx*dy/4, cX*dy/2, cY*dx/2
  int NY, lb0, lb1, ex_begin, ex_end, ney, nex, NXg, tiles_y, nbytes, dir_mode, diag;
  unsigned sides, flags;  // flags: 1 = cu given, 2 = cv given
  int nblk;               // grid size (gridDim would be a second, dependent kernarg fetch)
  int cpol;               // cache policy of the y stores / u,v loads (SEM_BAND_CPOL; see bstore_any)
  int mchunk;             // apply_march: element positions marched by one workgroup
  int pos0, pos1;         // element-position range of the launch (struct-argument kernel only; the
                          // preloaded-argument kernel always covers [0, ncols + 1))
  // FULL kernels only
  const double* ea;
  const double* eb;
  const double* ec;
  const double* ed;
  const double* dval;
  const uint8_t* mask;
  double cE, cA;
  int has_e1, has_e2;
  unsigned long long* stamps;  // SEM_DIAG bit 8
};

// Pin a kernel argument to kernel entry (an empty asm use keeps the compiler from sinking
// or rematerialising its s_load into a later phase).
#define BPIN(v) asm volatile("" ::"s"(v))

// Per-node operands of the optional terms (extra pairs, accumulate, Dirichlet mask / values).
// FULL kernels load them in the prologue with the tile, so the epilogue issues no load: on
// gfx950 vmcnt counts stores too, and a load-dependent wait between the epilogue's stores would
// serialise them behind the stores' completion.
struct NodeOps {
  double ea, eb, ec, ed, ya, dv;
  unsigned mk;
};

__device__ __forceinline__ NodeOps load_node_ops(const BandArgs& a, int p) {
  const int nb = a.nbytes;
  NodeOps o;
  o.ea = bload(brsrc(a.ea, a.has_e1 ? nb : 0), p * 8);
  o.eb = bload(brsrc(a.eb, a.has_e1 ? nb : 0), p * 8);
  o.ec = bload(brsrc(a.ec, a.has_e2 ? nb : 0), p * 8);
  o.ed = bload(brsrc(a.ed, a.has_e2 ? nb : 0), p * 8);
  o.ya = bload(brsrc(a.y, a.cA != 0.0 ? nb : 0), p * 8);
  o.dv = bload(brsrc(a.dval, a.dval ? nb : 0), p * 8);
  o.mk = __builtin_amdgcn_raw_buffer_load_b8(brsrc(a.mask, a.mask ? nb / 8 : 0), p, 0, 0);
  return o;
}

// Operator value z of one node -> + extra / accumulate terms, Dirichlet rows (no memory access).
template <bool FULL>
__device__ __forceinline__ double finish_node(const BandArgs& a, const NodeOps& o, int gx, int gy, double xv,
                                              double z) {
  if constexpr (FULL) {
    // pointwise terms are node values, not partial sums: on a strip's right interface line they
    // are left to the right-hand owner (the exchange sums the two strips' values)
    const bool own = !(gx == a.lb1 && a.ex_end < a.nex);
    if (a.has_e1 && own) z = fma(a.cE * o.ea, o.eb, z);
    if (a.has_e2 && own) z = fma(a.cE * o.ec, o.ed, z);
    if (a.cA != 0.0 && own) z = fma(a.cA, o.ya, z);
  }
  if (a.dir_mode != SEM_DIR_NONE) {
    const bool side = ((a.sides & SEM_SIDE_W) && gx == 0) || ((a.sides & SEM_SIDE_E) && gx == a.NXg - 1) ||
                      ((a.sides & SEM_SIDE_S) && gy == 0) || ((a.sides & SEM_SIDE_N) && gy == a.NY - 1);
    bool isd = side;
    if constexpr (FULL) isd = a.mask ? (o.mk & 0xff) != 0 : side;
    if (isd) {
      // an interface line's Dirichlet row is written by its owner (the right strip) only
      const bool owner = !(gx == a.lb1 && a.ex_end < a.nex);
      const double dv = FULL ? o.dv : 0.0;
      if (!owner)
        z = 0.0;
      else if (a.dir_mode == SEM_DIR_IDENTITY)
        z = xv - dv;
      else
        z = dv;
    }
  }
  return z;
}

// y store with the launch's cache policy (wave-uniform switch; the policy must be an immediate).
__device__ __forceinline__ void bstore_any(int cpol, __amdgpu_buffer_rsrc_t r, int off, double v) {
  switch (cpol & 255) {
    case 1: bstore_c<2>(r, off, v); break;     // non-temporal
    case 2: bstore_c<16>(r, off, v); break;    // sc1
    case 3: bstore_c<17>(r, off, v); break;    // sc0 sc1 (system scope: write through L2)
    case 4: bstore_c<19>(r, off, v); break;    // nt + sc0 sc1
    default: bstore(r, off, v);
  }
}

// GLL weight w_J of order P for a runtime J (compile-time constants, no memory access).
template <int P>
__device__ __forceinline__ double gll_w(int J) {
  double r = 0.0;
  for_rows(std::make_integer_sequence<int, P + 1>{}, [&](auto K) {
    constexpr int k = decltype(K)::value;
    if (J == k) r = GllConst<P>::w[k];
  });
  return r;
}

// GLL weights of order P as a device table (the band kernel's LDS weight array ws[] is filled from it)
template <int P>
struct GllWTab {
  double v[P + 1];
  static constexpr GllWTab make() {
    GllWTab t{};
    for (int k = 0; k <= P; ++k) t.v[k] = GllConst<P>::w[k];
    return t;
  }
};
template <int P>
__device__ const GllWTab<P> kGllW = GllWTab<P>::make();

// FULL = false: no extra / accumulate terms, no Dirichlet mask or values (side bits only).
// DPP = true: row coefficients from the split's DPP-broadcast list (CList) instead of immediates.
// GRAD = false: no gradient / convection terms (mass + stiffness only: the Laplacian K x, the
// Helmholtz operators of Solvers/README.md, the NS pressure rows K[mask,:] p); the G rows are
// then dead code and are not computed.
// Kernel body.  The fields the prologue needs before its first global load (x, cu, cv pointers and
// the tile-mapping integers) arrive as separate values: from the struct (apply_band) or as leading
// scalar kernel arguments that the command processor preloads into SGPRs (apply_band_kp, KP =
// true), so the first staging load does not wait for a kernarg memory fetch.
template <int P, int TXE, int TYE, int NS, bool FULL, int CM, bool GRAD, bool KP>
__device__ __forceinline__ void band_body(const double* __restrict__ px, const double* __restrict__ pcu,
                                          const double* __restrict__ pcv, int pNY, int plb0, int pex_begin,
                                          int pex_end, int pney, int pnblk, int ptiles_y, int pnbytes,
                                          const BandArgs& a) {
  using C = BCfg<P, TXE, TYE, NS>;
  using PL = EPlan<P, NS>;
  using CL = CList<P, NS>;
  constexpr bool DPP = CM == 1;
  constexpr int n = C::n, BX = C::BX, PT = C::PT, PY = C::PY, LW = C::LW, NW = C::NW;
  __shared__ double Ts[C::RX * PT];
  __shared__ double XK[BX * PY];
  // XG, YG are allocated for the Laplacian-only form (GRAD = false) too although it never touches them: the
  // smaller footprint let 8 workgroups share a CU instead of 6 and ran 3 % slower at 1024^2 (round-6 A/B,
  // profiles/r06/band_ab/ab_tile_and_lds_variants.jsonl) -- more tiles in flight contend for the same L2 halos
  __shared__ double XG[BX * PY];
  __shared__ double YK[BX * PY];
  __shared__ double YG[BX * PY];
  __shared__ double ws[n];

  // XCD-aware remap: blocks b and b+8 share an XCD, so each XCD gets a contiguous run of tiles (y fastest) and
  // neighbouring tiles share their halo lines through that XCD's L2.
  const int nb = pnblk, bid = blockIdx.x, tyn = ptiles_y;
  const int xcd = bid & 7, rk = bid >> 3, q8 = nb >> 3, rem = nb & 7;
  const int L = (xcd < rem ? xcd * (q8 + 1) : rem * (q8 + 1) + (xcd - rem) * q8) + rk;
  const int tx = L / tyn, ty = L - tx * tyn;

  const int lb0 = plb0, NY = pNY;
  // element positions [m0, m1) x [n0, n1); position ex_end (ney) is the ghost holding the closing line (column).
  // KP kernels cover every position; the struct kernel may be restricted to [pos0, pos1) (the multi-GPU overlap
  // applies the interface positions first, then the interior)
  const int m0 = pex_begin + (KP ? 0 : a.pos0) + tx * TXE;
  const int m1 = min(m0 + TXE, KP ? pex_end + 1 : pex_begin + a.pos1);
  const int n0 = ty * TYE, n1 = min(n0 + TYE, pney + 1);
  const int gx0 = m0 * P, gy0 = n0 * P;
  const int rows_ok = (min(m1, pex_end) - m0) * P + (m1 > pex_end ? 1 : 0);  // valid lines of the tile
  const int cols_ok = (min(n1, pney) - n0) * P + (n1 > pney ? 1 : 0);       // valid columns
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int nbytes = pnbytes;
  const bool has_u = pcu != nullptr, has_v = pcv != nullptr;
  const auto rx = brsrc(px, nbytes), ru = brsrc(pcu, has_u ? nbytes : 0), rv = brsrc(pcv, has_v ? nbytes : 0);
  const auto ry = brsrc(a.y, nbytes);
  const int nodeb = (gx0 - lb0) * NY + gy0;  // local DOF index of the tile's first node

  // ---- staging, one window line per wave step (round 6: per-lane index math once, not per staged value).
  // Wave w stages lines rr = w + NW k of the window [gx0 - P, gx0 + BX] x [gy0 - P, gy0 + BY]: lanes = columns
  // 0..63 (one load each), and the columns 64..RY-1 of all its lines together in NXL more loads.  A column outside
  // [0, NY) carries the offset 2^31 + line offset, a line outside the local range a negative offset: both are
  // outside the buffer (the launcher keeps nbytes + (P + 1) NY 8 <= 2^31), so every absent node loads 0 -- no
  // select per value.  Loads are issued in the order they are consumed (vmcnt retires in order).
  // the GLL weights for ws[]: loaded from a device table FIRST, so the load returns under the staging loads behind it
  // (issued after them it put one more memory round trip on wave 0's way to the barrier: +2-6 % on HBM-sized meshes)
  const double wsv = tid < n ? kGllW<P>.v[tid] : 0.0;
  // DPP variant: this wave's coefficient list (split of its role), entry 16 j + (lane & 15) in cv[j] -- also before
  // the staging loads (the contractions wait for it)
  double cv[DPP ? CL::NCV : 1];
  if constexpr (DPP) {
    const int wsplit = w < C::NXW ? (w / C::XW) % NS : (w - C::NXW) / C::YW;
    const double* tb = kBandCoef<P, NS>.v + wsplit * CL::NPAD + (lane & 15);
#pragma unroll
    for (int j = 0; j < CL::NCV; ++j) cv[j] = tb[16 * j];
  } else {
    cv[0] = 0.0;
  }
  const int lstep = NW * NY * 8;
  const int line0 = (gx0 - P - lb0 + w) * NY * 8;  // byte offset of this wave's first staged line
  const int gyA = gy0 - P + lane;
  const unsigned vA = (gyA >= 0 && gyA < NY) ? static_cast<unsigned>(gyA) * 8u : 0x80000000u;
  double sA[C::NSL];
#pragma unroll
  for (int k = 0; k < C::NSL; ++k)
    if (k < C::NSL - 1 || w + NW * k < C::RX)  // only the last step can pass the window's end
      sA[k] = bload(rx, static_cast<int>(vA + static_cast<unsigned>(line0 + k * lstep)));
  double sX[C::NXL];
  int xts[C::NXL];
#pragma unroll
  for (int j = 0; j < C::NXL; ++j) {
    const int lp = lane + 64 * j, k = lp / C::RYX, cc = 64 + lp - k * C::RYX, rr = w + NW * k;
    const int gy = gy0 - P + cc;
    const bool ok = k < C::NSL && rr < C::RX;
    const unsigned vx = (ok && gy >= 0 && gy < NY) ? static_cast<unsigned>(gy) * 8u : 0x80000000u;
    xts[j] = ok ? rr * PT + cc : -1;
    sX[j] = bload(rx, static_cast<int>(vx + static_cast<unsigned>(line0 + k * lstep)));
  }
  // epilogue nodes of this thread: q = tid + e*THREADS -> tile line r = q / LW, column c = q % LW
  double pu[C::NE], pv[C::NE];
  int eoff[C::NE];
  NodeOps ops[C::NE] = {};
#pragma unroll
  for (int e = 0; e < C::NE; ++e) {
    const int q = tid + e * C::THREADS;
    const int r = q / LW, c = q - r * LW;
    const bool ok = q < BX * LW && r < rows_ok && c < cols_ok;
    eoff[e] = ok ? nodeb + r * NY + c : -(1 << 26);  // out of bounds: touches no memory
  }
  const bool nt_uv = (a.cpol & 256) != 0;   // u, v are read once per launch: non-temporal (HBM-sized meshes)
  if constexpr (KP) {  // the struct's fields: fetched now, while the staging loads are in flight
    BPIN(a.y);
    BPIN(a.fKx);
    BPIN(a.fKy);
    BPIN(a.fM);
    BPIN(a.fX);
    BPIN(a.fY);
    BPIN(a.NXg);
    BPIN(a.dir_mode);
    BPIN(a.sides);
    BPIN(a.cpol);
    BPIN(a.lb1);
    BPIN(a.nex);
  }

  // ---- LDS: staged window, weights
#pragma unroll
  for (int k = 0; k < C::NSL; ++k)
    if (k < C::NSL - 1 || w + NW * k < C::RX) Ts[(w + NW * k) * PT + lane] = sA[k];
#pragma unroll
  for (int j = 0; j < C::NXL; ++j)
    if (xts[j] >= 0) Ts[xts[j]] = sX[j];
  if (tid < n) ws[tid] = wsv;
  // the epilogue's pointwise operands: issued after the staged window has gone to LDS, so they land during the
  // contractions (round 4)
  if (nt_uv) {
#pragma unroll
    for (int e = 0; e < C::NE; ++e) {
      pu[e] = bload_c<2>(ru, eoff[e] * 8);
      pv[e] = bload_c<2>(rv, eoff[e] * 8);
    }
  } else {
#pragma unroll
    for (int e = 0; e < C::NE; ++e) {
      pu[e] = bload(ru, eoff[e] * 8);
      pv[e] = bload(rv, eoff[e] * 8);
    }
  }
  if constexpr (FULL) {
#pragma unroll
    for (int e = 0; e < C::NE; ++e) ops[e] = load_node_ops(a, eoff[e]);
  }
  __syncthreads();

  constexpr double w0 = GllConst<P>::w[0], wP = GllConst<P>::w[P];
  if (w < C::NXW) {
    // ---- X role: wave = (element position xa, split xs), lane = column xc: the x-direction rows of the split
    // from a (2P+1)-node window along x -> LDS, scaled by the column's fKx My and fX My (round 6: the epilogue's
    // column factors moved here, once per lane).  Lines outside the local range are staged as 0, so absent
    // elements contribute nothing.
    const int xg = w / C::XW;
    const int xa = xg / NS, xs = xg - xa * NS;
    const int xc = (w - xg * C::XW) * 64 + lane;
    if (xa < m1 - m0) {
      const bool xghost = m0 + xa == pex_end, hasLx = m0 + xa - 1 >= pex_begin;  // wave-uniform
      const double fk = (hasLx ? 1.0 : 0.0) + (xghost ? 0.0 : 1.0);
      const double fg = (xghost ? 0.0 : 1.0) - (hasLx ? 1.0 : 0.0);
      for_rows(std::make_integer_sequence<int, NS>{}, [&](auto S) {
        constexpr int s = decltype(S)::value;
        if (xs != s) return;
        double t[2 * P + 1];
        constexpr int q0 = PL::needs_left(s) ? 0 : P;  // only row 0 reads the left element
#pragma unroll
        for (int qq = q0; qq <= 2 * P; ++qq) t[qq] = Ts[(xa * P + qq) * PT + P + xc];
#pragma unroll
        for (int qq = 0; qq < q0; ++qq) t[qq] = 0.0;
        double k[C::RP], g[C::RP];
        eo_rows<P, NS, s, CM>(t, fk, fg, k, g, cv);
        const int jc = xc % P, nc = n0 + xc / P;
        const double myc = jc != 0 ? ws[jc] : (nc - 1 >= 0 ? wP : 0.0) + (nc < pney ? w0 : 0.0);
        const double sxk = a.fKx * myc, sxg = a.fX * myc;
#pragma unroll
        for (int sl = 0; sl < PL::nrows(s); ++sl) {
          const int i = PL::row(s, sl);
          if (xghost && i != 0) continue;  // a ghost position holds its row 0 only
          XK[(xa * P + i) * PY + xc] = sxk * k[sl];
          if constexpr (GRAD) XG[(xa * P + i) * PY + xc] = sxg * g[sl];
        }
      });
    }
  } else {
    // ---- Y role: wave = split h, lane = (line r, element position b): the y-direction columns of the split from
    // a (2P+1)-node window along the line -> LDS, scaled by Mx of the line.
    const int wy = w - C::NXW;
    const int h = wy / C::YW;
    const int t2 = (wy - h * C::YW) * 64 + lane;
    const bool yok = t2 < C::YL && t2 % BX < rows_ok && t2 / BX < n1 - n0;
    // the DPP variant computes on every lane (a DPP read of a disabled lane is not its value) from clamped,
    // in-bounds positions; only the LDS stores are predicated
    const int r = DPP ? min(t2 % BX, BX - 1) : t2 % BX, b = DPP ? min(t2 / BX, C::YL / BX - 1) : t2 / BX;
    if (DPP || yok) {
      const bool hasLy = n0 + b - 1 >= 0, hasRy = n0 + b < pney;
      const double fk = (hasLy ? 1.0 : 0.0) + (hasRy ? 1.0 : 0.0), fg = (hasRy ? 1.0 : 0.0) - (hasLy ? 1.0 : 0.0);
      const int i = r % P, ex = m0 + r / P;
      const double mx = i != 0 ? ws[i] : (ex - 1 >= pex_begin ? wP : 0.0) + (ex < pex_end ? w0 : 0.0);
      const double sk = a.fKy * mx, sg = a.fY * mx;
      for_rows(std::make_integer_sequence<int, NS>{}, [&](auto H) {
        constexpr int hh = decltype(H)::value;
        if (h != hh) return;
        double t[2 * P + 1];
        constexpr int q0 = PL::needs_left(hh) ? 0 : P;
#pragma unroll
        for (int qq = q0; qq <= 2 * P; ++qq) t[qq] = Ts[(P + r) * PT + b * P + qq];
#pragma unroll
        for (int qq = 0; qq < q0; ++qq) t[qq] = 0.0;
        double k[C::RP], g[C::RP];
        eo_rows<P, NS, hh, CM>(t, fk, fg, k, g, cv);
        if (yok) {
#pragma unroll
          for (int sl = 0; sl < PL::nrows(hh); ++sl) {
            const int j = PL::row(hh, sl);
            YK[r * PY + b * P + j] = sk * k[sl];
            if constexpr (GRAD) YG[r * PY + b * P + j] = sg * g[sl];
          }
        }
      });
    }
  }
  __syncthreads();

  // ---- epilogue, every wave: node (r, c) = X + Y rows (+ mass) + the pointwise convection terms; Dirichlet rows, the extra /
  // accumulate terms and the strip-ownership rules only in a tile that can hold one (tile-uniform test)
  const int NXg = a.NXg;
  bool special = FULL;
  if (a.dir_mode != SEM_DIR_NONE) {
    const int gxl = gx0 + rows_ok - 1, gyl = gy0 + cols_ok - 1;
    const unsigned sd = a.sides;
    special = special || ((sd & SEM_SIDE_W) && gx0 == 0) || ((sd & SEM_SIDE_E) && gxl >= NXg - 1) ||
              ((sd & SEM_SIDE_S) && gy0 == 0) || ((sd & SEM_SIDE_N) && gyl >= NY - 1);
  }
  double zz[C::NE];
#pragma unroll
  for (int e = 0; e < C::NE; ++e) {
    const int q = tid + e * C::THREADS;
    const int r = q / LW, c = q - r * LW;
    const int o = r * PY + c;
    double z = XK[o] + YK[o];
    if (a.fM != 0.0) {   // the mass term (not on the CD / NS hot paths: a uniform branch, its weights from LDS)
      const int i = r % P, me = m0 + r / P, j = c % P, ne = n0 + c / P;
      const double mx = i != 0 ? ws[i] : (me - 1 >= pex_begin ? wP : 0.0) + (me < pex_end ? w0 : 0.0);
      const double my = j != 0 ? ws[j] : (ne - 1 >= 0 ? wP : 0.0) + (ne < pney ? w0 : 0.0);
      z = fma(a.fM * mx * my, Ts[(P + r) * PT + P + c], z);
    }
    if constexpr (GRAD) {
      z = fma(has_u ? pu[e] : 1.0, XG[o], z);
      z = fma(has_v ? pv[e] : 1.0, YG[o], z);
    }
    if (special && eoff[e] >= 0) z = finish_node<FULL>(a, ops[e], gx0 + r, gy0 + c, Ts[(P + r) * PT + P + c], z);
    zz[e] = z;
  }
  if ((a.cpol & 255) == 3) {   // system-scope stores (a mesh whose working set stays in the MALL)
#pragma unroll
    for (int e = 0; e < C::NE; ++e)
      if (eoff[e] >= 0) bstore_c<17>(ry, eoff[e] * 8, zz[e]);
  } else {
#pragma unroll
    for (int e = 0; e < C::NE; ++e)
      if (eoff[e] >= 0) bstore(ry, eoff[e] * 8, zz[e]);
  }
}

template <int P, int TXE, int TYE, int NS, bool FULL, int CM, bool GRAD = true>
__global__ __launch_bounds__((BCfg<P, TXE, TYE, NS>::THREADS)) void apply_band(const BandArgs a) {
  BPIN(a.x);
  BPIN(a.y);
  BPIN(a.cu);
  BPIN(a.cv);
  BPIN(a.fKx);
  BPIN(a.fKy);
  BPIN(a.fM);
  BPIN(a.fX);
  BPIN(a.fY);
  BPIN(a.NY);
  BPIN(a.lb0);
  BPIN(a.lb1);
  BPIN(a.ex_begin);
  BPIN(a.ex_end);
  BPIN(a.ney);
  BPIN(a.nex);
  BPIN(a.NXg);
  BPIN(a.tiles_y);
  BPIN(a.nbytes);
  BPIN(a.dir_mode);
  if constexpr (kDiag) BPIN(a.diag);
  BPIN(a.sides);
  BPIN(a.flags);
  if constexpr (kDiag) BPIN(a.stamps);
  BPIN(a.nblk);
  BPIN(a.cpol);
  band_body<P, TXE, TYE, NS, FULL, CM, GRAD, false>(a.x, (a.flags & 1) ? a.cu : nullptr, (a.flags & 2) ? a.cv : nullptr,
                                                     a.NY, a.lb0, a.ex_begin, a.ex_end, a.ney, a.nblk, a.tiles_y,
                                                     a.nbytes, a);
}

// Same kernel with the prologue's fields as leading scalar arguments (14 SGPRs, preloaded by the
// command processor when the code object asks for it: -amdgpu-kernarg-preload-count in build.py).
template <int P, int TXE, int TYE, int NS, bool FULL, int CM, bool GRAD = true>
__global__ __launch_bounds__((BCfg<P, TXE, TYE, NS>::THREADS)) void apply_band_kp(
    const double* px, const double* pcu, const double* pcv, int pNY, int plb0, int pex_begin, int pex_end, int pney,
    int pnblk, int ptiles_y, int pnbytes, const BandArgs a) {
  band_body<P, TXE, TYE, NS, FULL, CM, GRAD, true>(px, pcu, pcv, pNY, plb0, pex_begin, pex_end, pney, pnblk, ptiles_y,
                                                    pnbytes, a);
}

static int hip_check_b(hipError_t e, const char* what) {
  if (e == hipSuccess) return SEM_OK;
  return set_error(SEM_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Default cache policy (measured in-process, tools/ab_env.py, profiles/r01/band/cpol_ab.txt): on a mesh
// whose working set stays in the MALL, system-scope y stores (sc0 sc1: written through L2 as they
// are issued) save the end-of-kernel L2 writeback, 4.66 -> 4.38 us at cfg2; on HBM-sized meshes
// that costs ~1 %, and non-temporal u, v loads (read once) are neutral to slightly better.
static int band_cpol(long long n_local) { return 32LL * n_local < (128LL << 20) ? 3 : 256; }

// The kernel arguments every band-family launch shares (apply_band, apply_bmfma): pointers, fused factors,
// the strip and the Dirichlet fields; the launch sets its grid fields.
static BandArgs band_args(const ApplyArgs& g) {
  BandArgs b{};
  b.x = g.x;
  b.y = g.y;
  b.cu = g.cu;
  b.cv = g.cv;
  b.fKx = g.cK * g.sx;
  b.fKy = g.cK * g.sy;
  b.fM = g.cM * g.hxy;
  b.fX = g.cX * g.hy;
  b.fY = g.cY * g.hx;
  b.NY = static_cast<int>(g.NY);
  b.lb0 = static_cast<int>(g.line_begin);
  b.lb1 = static_cast<int>(g.line_end);
  b.ex_begin = g.ex_begin;
  b.ex_end = g.ex_end;
  b.ney = g.ney;
  b.nex = g.nex;
  b.NXg = static_cast<int>(g.NXg);
  b.nbytes = g.n_local32 * 8;
  b.dir_mode = g.dir_mode;
  b.diag = g.diag;
  b.sides = g.sides;
  b.flags = (g.cu ? 1u : 0u) | (g.cv ? 2u : 0u);
  b.ea = g.ea;
  b.eb = g.eb;
  b.ec = g.ec;
  b.ed = g.ed;
  b.dval = g.dval;
  b.mask = g.mask;
  b.cE = g.cE;
  b.cA = g.cA;
  b.has_e1 = g.has_e1;
  b.has_e2 = g.has_e2;
  b.stamps = g.stamps;
  b.cpol = band_cpol(g.n_local32);
  return b;
}

template <int P, int TXE, int TYE, int NS, int CM = 0>
static int launch_band(const ApplyArgs& g, const sem_handle* h, hipStream_t s) {
  using C = BCfg<P, TXE, TYE, NS>;
  const int ncols = h->ex_end - h->ex_begin;
  // element positions [pos0, pos1) of 0..ncols (ncols = the ghost position of the closing line)
  const bool ranged = g.pos1 > 0;
  const int pos0 = ranged ? g.pos0 : 0, pos1 = ranged ? g.pos1 : ncols + 1;
  const int tiles_x = (pos1 - pos0 + TXE - 1) / TXE;
  const int tiles_y = (h->ney + 1 + TYE - 1) / TYE;
  const long long nblk = static_cast<long long>(tiles_x) * tiles_y;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return set_error(SEM_EINVAL, "mesh too large for one launch");
  BandArgs b = band_args(g);
  b.pos0 = pos0;
  b.pos1 = pos1;
  b.tiles_y = tiles_y;
  b.nblk = static_cast<int>(nblk);
  const bool full = g.has_e1 || g.has_e2 || g.cA != 0.0 || g.mask || g.dval;
  const bool grad = g.cX != 0.0 || g.cY != 0.0;
  const dim3 grid(static_cast<unsigned>(nblk)), block(C::THREADS);
  if (tune(SEM_TUNE_BAND_KP) >= 0 && !ranged) {  // -1 (SEM_BAND_KP=0): struct-only arguments (A/B)
#define SEM_KP_ARGS b.x, b.cu, b.cv, b.NY, b.lb0, b.ex_begin, b.ex_end, b.ney, b.nblk, b.tiles_y, b.nbytes, b
    if (full && grad)
      hipLaunchKernelGGL((apply_band_kp<P, TXE, TYE, NS, true, CM, true>), grid, block, 0, s, SEM_KP_ARGS);
    else if (full)
      hipLaunchKernelGGL((apply_band_kp<P, TXE, TYE, NS, true, CM, false>), grid, block, 0, s, SEM_KP_ARGS);
    else if (grad)
      hipLaunchKernelGGL((apply_band_kp<P, TXE, TYE, NS, false, CM, true>), grid, block, 0, s, SEM_KP_ARGS);
    else
      hipLaunchKernelGGL((apply_band_kp<P, TXE, TYE, NS, false, CM, false>), grid, block, 0, s, SEM_KP_ARGS);
#undef SEM_KP_ARGS
    return hip_check_b(hipGetLastError(), "apply (band) launch");
  }
  if (full && grad)
    hipLaunchKernelGGL((apply_band<P, TXE, TYE, NS, true, CM, true>), grid, block, 0, s, b);
  else if (full)
    hipLaunchKernelGGL((apply_band<P, TXE, TYE, NS, true, CM, false>), grid, block, 0, s, b);
  else if (grad)
    hipLaunchKernelGGL((apply_band<P, TXE, TYE, NS, false, CM, true>), grid, block, 0, s, b);
  else
    hipLaunchKernelGGL((apply_band<P, TXE, TYE, NS, false, CM, false>), grid, block, 0, s, b);
  return hip_check_b(hipGetLastError(), "apply (band) launch");
}

// =========================================================================== band-form MFMA kernel
//
// The assembled 1-D operators of the band kernel (Kx, Gx along x; Ky, Gy along y; SEM.py:186-223) applied as
// small dense matmuls on the fp64 matrix cores (v_mfma_f64_16x16x4_f64) -- north_star's MFMA form without the
// element-block form's waste (round 5, VERDICT r4 item 8: apply_tp_mfma computes every element's rows, the halo
// element's included, stores them all to LDS and sums the one or two contributions of each node in the epilogue:
// 940 K VALU instructions per cfg2 launch against the band kernel's 630 K).  Here every output row is formed
// exactly once, the x and y results of a node land in the SAME lane (the f64 16x16x4 D layout is
// row = (lane >> 4) + 4 reg, column = lane & 15 for both products), and the epilogue combines them in
// registers: no result round trip through LDS, no DSS sums.
//   tile   RX = TXE P lines (TXE = 16 / P whole element columns, RX <= 16) x NB column blocks of CB = RX columns;
//          one wave per column block.
//   x      D[i][n] = sum_k Ab[i][k] T[gx0 - P + k][col n],  Ab = the tile's RX rows of Kx (Gx) over the window
//          of KW = 4 KS lines from gx0 - P: row i of element e = i / P is K_s[i % P][.] over that element's lines,
//          a shared row (i % P == 0) K_s[P][.] over the left element plus K_s[0][.] over the right one.  Ab is the
//          same for every tile (tiles are element aligned), a per-lane constant (kBMTab).
//   y      D[m][n] = sum_k T[gx0 + m][gy0b - P + k] Ab[n][k]: the SAME per-lane registers as the x product's A
//          operand, now as B.
// Lines / columns outside the local domain are staged as 0 (buffer bounds, explicit zero past the y ends), so an
// absent element contributes nothing except the diagonal term of the shared row's folded coefficient, which the
// epilogue removes (K_s[P][P] x without a left element, K_s[0][0] x without a right one).
typedef double dbl4v __attribute__((ext_vector_type(4)));

template <int P>
struct BMCfg {
  static constexpr int TXE = 16 / P > 0 ? 16 / P : 1;
  static constexpr int RX = TXE * P;                       // output lines per tile (<= 16)
  static constexpr int CB = RX;                            // output columns per block (element aligned)
  static constexpr int KS = (RX + P + 1 + 3) / 4;          // k-steps of the (RX + P + 1)-wide window
  static constexpr int KW = 4 * KS;
  static constexpr int NB = 4;                             // column blocks (= waves) per tile
  static constexpr int THREADS = 64 * NB;
  static constexpr int SL = KW > P + 16 ? KW : P + 16;     // staged lines from gx0 - P (y product reads P .. P + 15)
  static constexpr int SC0 = (NB - 1) * CB + KW, SC1 = P + (NB - 1) * CB + 16;
  static constexpr int SC = SC0 > SC1 ? SC0 : SC1;         // staged columns from gy0 - P
  static constexpr int R16 = (SC + 15) / 16 * 16;
  static constexpr int PT = R16 + ((16 - R16 % 32) + 32) % 32;   // pitch == 16 (mod 32) doubles
  static constexpr int NSTAGE = (SL * SC + THREADS - 1) / THREADS;
  // column c of staged row r at c ^ 2 ((r >> 1) & 7), a permutation inside each aligned 16-column run: the x
  // product's 4 rows x 16 columns and the y product's 16 rows x 4 columns both spread over the banks
  __host__ __device__ static constexpr int ts(int r, int c) { return r * PT + (c ^ (((r >> 1) & 7) << 1)); }
  static_assert(P >= 1 && P <= 16, "P in 1..16");
};

template <int P>
struct BMTab {
  using C = BMCfg<P>;
  static constexpr double coef(const double* T, int i, int k) {   // Ab[i][k] of table T (K_s or G_s)
    if (i >= C::RX) return 0.0;
    const int e = i / P, li = i % P, n = P + 1;
    double v = 0.0;
    if (li != 0) {
      const int kk = k - P - e * P;
      if (kk >= 0 && kk <= P) v = T[li * n + kk];
    } else {
      const int kl = k - e * P, kr = k - P - e * P;
      if (kl >= 0 && kl <= P) v += T[P * n + kl];
      if (kr >= 0 && kr <= P) v += T[kr];
    }
    return v;
  }
  struct Tab {
    double v[2 * 16 * C::KW];   // [K | G][i][k]
  };
  static constexpr Tab make() {
    Tab t{};
    for (int i = 0; i < 16; ++i)
      for (int k = 0; k < C::KW; ++k) {
        t.v[i * C::KW + k] = coef(GllConst<P>::K, i, k);
        t.v[16 * C::KW + i * C::KW + k] = coef(GllConst<P>::G, i, k);
      }
    return t;
  }
};
template <int P>
__device__ const typename BMTab<P>::Tab kBMTab = BMTab<P>::make();

template <int P, bool FULL, bool GRAD>
__global__ __launch_bounds__(BMCfg<P>::THREADS) void apply_bmfma(const BandArgs a) {
  using C = BMCfg<P>;
  constexpr int NW = C::NB, PT = C::PT;
  constexpr int NTAB = (GRAD ? 2 : 1) * 16 * C::KW;                 // operand table [K | G][i][k] (global, dense)
  // its LDS copy: row pitch AP = 2 (mod 32) doubles, so a half-wave's reads (rows lr = 0..15, entries lk = 0, 1)
  // fall on 32 distinct 2-bank slots -- the dense pitch KW = 28 put rows lr and lr + 8 on one bank (2-way conflicts:
  // 45.5 M conflict cycles per 1024^2 launch, profiles/r06/mfma)
  constexpr int AP = (C::KW + 29) / 32 * 32 + 2 >= C::KW ? (C::KW + 29) / 32 * 32 + 2 : (C::KW + 29) / 32 * 32 + 34;
  constexpr int NAP = (GRAD ? 2 : 1) * 16 * AP;
  constexpr int NAB = (NTAB + C::THREADS - 1) / C::THREADS;
  // staging (round 6, as the band kernel): wave w stages window lines w + NW k (lanes = columns 0..63) and the
  // columns 64..SC-1 of its lines in NXL more loads; absent columns / lines load 0 through out-of-range offsets
  constexpr int NSL = (C::SL + NW - 1) / NW, SCX = C::SC - 64, NXL = SCX > 0 ? (NSL * SCX + 63) / 64 : 0;
  static_assert(C::SC <= 128, "staged columns");
  __shared__ double Ts[C::SL * PT];
  __shared__ double ws[P + 1];   // GLL weights: one LDS read per weight instead of a compare-select chain
  // the Ab operands live in LDS, read per k-step (round 6): as per-lane registers they held 2 KS doubles per lane through
  // the whole kernel and, with the accumulators, capped the kernel at 4 waves per SIMD
  __shared__ double Ab[NAP];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lk = lane >> 4;
  // XCD-aware remap (as apply_band): each XCD a contiguous run of tiles, y fastest
  const int nb = a.nblk, bid = blockIdx.x, xcd = bid & 7, rk = bid >> 3, q8 = nb >> 3, rem = nb & 7;
  const int L = (xcd < rem ? xcd * (q8 + 1) : rem * (q8 + 1) + (xcd - rem) * q8) + rk;
  const int tx = L / a.tiles_y, ty = L - tx * a.tiles_y;
  const int lb0 = a.lb0, NY = a.NY;
  const int gx0 = lb0 + tx * C::RX, gy0 = ty * (C::NB * C::CB);
  const int rows_ok = min(C::RX, a.lb1 + 1 - gx0);
  const int nbytes = a.nbytes;
  const auto rx = brsrc(a.x, nbytes), ry = brsrc(a.y, nbytes);
  const bool has_u = (a.flags & 1) != 0, has_v = (a.flags & 2) != 0;
  const auto ru = brsrc(a.cu, has_u ? nbytes : 0), rv = brsrc(a.cv, has_v ? nbytes : 0);

  // ---- tables first (their loads return under the staging loads), then the staged window
  const double wsv = tid <= P ? kGllW<P>.v[tid] : 0.0;
  double abv[NAB];
#pragma unroll
  for (int q = 0; q < NAB; ++q) {
    const int idx = tid + q * C::THREADS;
    abv[q] = idx < NTAB ? kBMTab<P>.v[idx] : 0.0;
  }
  const int lstep = NW * NY * 8;
  const int line0 = (gx0 - P - lb0 + w) * NY * 8;
  const int gyA = gy0 - P + lane;
  const unsigned vA = (gyA >= 0 && gyA < NY) ? static_cast<unsigned>(gyA) * 8u : 0x80000000u;
  double sA[NSL];
#pragma unroll
  for (int k = 0; k < NSL; ++k)
    if (k < NSL - 1 || w + NW * k < C::SL) sA[k] = bload(rx, static_cast<int>(vA + static_cast<unsigned>(line0 + k * lstep)));
  double sX[NXL > 0 ? NXL : 1];
  int xts[NXL > 0 ? NXL : 1];
#pragma unroll
  for (int j = 0; j < NXL; ++j) {
    const int lp = lane + 64 * j, k = lp / SCX, cc = 64 + lp - k * SCX, rr = w + NW * k;
    const int gy = gy0 - P + cc;
    const bool ok = k < NSL && rr < C::SL;
    const unsigned vx = (ok && gy >= 0 && gy < NY) ? static_cast<unsigned>(gy) * 8u : 0x80000000u;
    xts[j] = ok ? C::ts(rr, cc) : -1;
    sX[j] = bload(rx, static_cast<int>(vx + static_cast<unsigned>(line0 + k * lstep)));
  }
  // this lane's epilogue nodes: tile row i = lk + 4 r, column gy0 + w CB + lr
  const int gyn = gy0 + w * C::CB + lr;
  const bool col_ok = lr < C::CB && gyn < NY;
  int eoff[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = lk + 4 * r;
    eoff[r] = (col_ok && i < rows_ok) ? ((gx0 + i - lb0) * NY + gyn) : -(1 << 26);
  }
#pragma unroll
  for (int k = 0; k < NSL; ++k)
    if (k < NSL - 1 || w + NW * k < C::SL) Ts[C::ts(w + NW * k, lane)] = sA[k];
#pragma unroll
  for (int j = 0; j < NXL; ++j)
    if (xts[j] >= 0) Ts[xts[j]] = sX[j];
  if (tid <= P) ws[tid] = wsv;
#pragma unroll
  for (int q = 0; q < NAB; ++q) {
    const int idx = tid + q * C::THREADS;
    if (idx < NTAB) Ab[(idx / C::KW) * AP + idx % C::KW] = abv[q];
  }
  // pointwise operands, issued after the staging stores (they land during the products)
  double pu[4], pv[4];
  NodeOps ops[4] = {};
  if (a.cpol & 256) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pu[r] = bload_c<2>(ru, eoff[r] * 8);
      pv[r] = bload_c<2>(rv, eoff[r] * 8);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pu[r] = bload(ru, eoff[r] * 8);
      pv[r] = bload(rv, eoff[r] * 8);
    }
  }
  if constexpr (FULL) {
#pragma unroll
    for (int r = 0; r < 4; ++r) ops[r] = load_node_ops(a, eoff[r]);
  }
  __syncthreads();

  // ---- the two products of this wave's 16 x 16 output block (independent accumulator chains)
  dbl4v xk = {0.0, 0.0, 0.0, 0.0}, xg = xk, yk = xk, yg = xk;
  const int cb0 = w * C::CB;
  // operands of step q + 1 are read while step q's MFMAs run; the scheduling barrier keeps the compiler from
  // hoisting every step's reads to the top (which held all 4 KS operands live and cost a wave per SIMD)
  double aK = Ab[lr * AP + lk], aG = GRAD ? Ab[16 * AP + lr * AP + lk] : 0.0;
  double bx = Ts[C::ts(lk, P + cb0 + lr)], ay = Ts[C::ts(P + lr, cb0 + lk)];
#pragma unroll
  for (int q = 0; q < C::KS; ++q) {
    double aK1 = 0.0, aG1 = 0.0, bx1 = 0.0, ay1 = 0.0;
    if (q + 1 < C::KS) {
      aK1 = Ab[lr * AP + 4 * (q + 1) + lk];
      if constexpr (GRAD) aG1 = Ab[16 * AP + lr * AP + 4 * (q + 1) + lk];
      bx1 = Ts[C::ts(4 * (q + 1) + lk, P + cb0 + lr)];     // T[gx0 - P + 4q + lk][gy0 + cb0 + lr]
      ay1 = Ts[C::ts(P + lr, cb0 + 4 * (q + 1) + lk)];     // T[gx0 + lr][gy0 + cb0 - P + 4q + lk]
    }
    xk = __builtin_amdgcn_mfma_f64_16x16x4f64(aK, bx, xk, 0, 0, 0);
    yk = __builtin_amdgcn_mfma_f64_16x16x4f64(ay, aK, yk, 0, 0, 0);
    if constexpr (GRAD) {
      xg = __builtin_amdgcn_mfma_f64_16x16x4f64(aG, bx, xg, 0, 0, 0);
      yg = __builtin_amdgcn_mfma_f64_16x16x4f64(ay, aG, yg, 0, 0, 0);
    }
    aK = aK1, aG = aG1, bx = bx1, ay = ay1;
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue in registers: node (tile row lk + 4 r, column gyn)
  constexpr double w0 = GllConst<P>::w[0], wP = GllConst<P>::w[P];
  constexpr double K00 = GllConst<P>::K[0], KPP = GllConst<P>::K[P * (P + 1) + P];
  constexpr double G00 = GllConst<P>::G[0], GPP = GllConst<P>::G[P * (P + 1) + P];
  const int lj = gyn % P, ne = gyn / P;
  const bool hasLy = lj == 0 && ne - 1 >= 0, hasRy = lj != 0 || ne < a.ney;
  const double my = lj != 0 ? ws[lj] : (hasLy ? wP : 0.0) + (hasRy ? w0 : 0.0);
  const double sxk = a.fKx * my, sxg = a.fX * my;
  // tile-uniform: can a node of this tile lack a neighbour element (strip / domain edge) or be a Dirichlet row?
  const int gxl = gx0 + rows_ok - 1, gyl = gy0 + C::NB * C::CB - 1;
  const bool xedge = gx0 <= a.ex_begin * P || gxl >= a.ex_end * P, yedge = gy0 == 0 || gyl >= NY - 1;
  bool special = FULL;
  if (a.dir_mode != SEM_DIR_NONE) {
    const unsigned sd = a.sides;
    special = special || ((sd & SEM_SIDE_W) && gx0 == 0) || ((sd & SEM_SIDE_E) && gxl >= a.NXg - 1) ||
              ((sd & SEM_SIDE_S) && gy0 == 0) || ((sd & SEM_SIDE_N) && gyl >= NY - 1);
  }
  // a shared row / column without its left / right element drops that element's folded diagonal term: the y
  // corrections are per lane (its column), the x corrections per row; both zero away from strip / domain edges
  const double dyk = lj == 0 ? (hasLy ? 0.0 : -KPP) + (hasRy ? 0.0 : -K00) : 0.0;
  const double dyg = lj == 0 ? (hasLy ? 0.0 : -GPP) + (hasRy ? 0.0 : -G00) : 0.0;
  const bool full_path = xedge || yedge || a.fM != 0.0 || special;   // tile-uniform
  double zz[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = lk + 4 * r, gx = gx0 + i;
    const int li = gx % P, me = gx / P;
    const bool hasLx = li == 0 && me - 1 >= a.ex_begin, hasRx = li != 0 || me < a.ex_end;
    const double mx = li != 0 ? ws[li] : (hasLx ? wP : 0.0) + (hasRx ? w0 : 0.0);
    double XK = xk[r], XG = xg[r], YK = yk[r], YG = yg[r];
    double z;
    if (full_path) {
      const double xv = Ts[C::ts(P + i, P + cb0 + lr)];
      const double dxk = li == 0 ? (hasLx ? 0.0 : -KPP) + (hasRx ? 0.0 : -K00) : 0.0;
      const double dxg = li == 0 ? (hasLx ? 0.0 : -GPP) + (hasRx ? 0.0 : -G00) : 0.0;
      XK = fma(dxk, xv, XK);
      XG = fma(dxg, xv, XG);
      YK = fma(dyk, xv, YK);
      YG = fma(dyg, xv, YG);
      z = fma(sxk, XK, a.fKy * mx * YK);
      z = fma(a.fM * mx * my, xv, z);
      if constexpr (GRAD) {
        z = fma(has_u ? pu[r] : 1.0, sxg * XG, z);
        z = fma(a.fY * (has_v ? pv[r] : 1.0), mx * YG, z);
      }
      if (special) z = finish_node<FULL>(a, ops[r], gx, gyn, xv, z);
    } else {
      z = fma(sxk, XK, a.fKy * mx * YK);
      if constexpr (GRAD) {
        z = fma(has_u ? pu[r] : 1.0, sxg * XG, z);
        z = fma(a.fY * (has_v ? pv[r] : 1.0), mx * YG, z);
      }
    }
    zz[r] = z;
  }
  if ((a.cpol & 255) == 3) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (eoff[r] >= 0) bstore_c<17>(ry, eoff[r] * 8, zz[r]);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (eoff[r] >= 0) bstore(ry, eoff[r] * 8, zz[r]);
  }
}

template <int P>
static int launch_bmfma(const ApplyArgs& g, const sem_handle* h, hipStream_t s) {
  using C = BMCfg<P>;
  if (g.pos1 > 0) return set_error(SEM_EUNSUPPORTED, "element-position ranges are implemented by the band kernel only");
  const long long nlines = static_cast<long long>(h->ex_end - h->ex_begin) * P + 1;
  const long long tiles_x = (nlines + C::RX - 1) / C::RX;
  const long long tiles_y = (h->NY + C::NB * C::CB - 1) / (C::NB * C::CB);
  const long long nblk = tiles_x * tiles_y;
  if (nblk <= 0 || nblk > 0x7fffffffLL) return set_error(SEM_EINVAL, "mesh too large for one launch");
  BandArgs b = band_args(g);
  b.tiles_y = static_cast<int>(tiles_y);
  b.nblk = static_cast<int>(nblk);
  const bool full = g.has_e1 || g.has_e2 || g.cA != 0.0 || g.mask || g.dval;
  const bool grad = g.cX != 0.0 || g.cY != 0.0;
  const dim3 grid(static_cast<unsigned>(nblk)), block(C::THREADS);
  if (full && grad)
    hipLaunchKernelGGL((apply_bmfma<P, true, true>), grid, block, 0, s, b);
  else if (full)
    hipLaunchKernelGGL((apply_bmfma<P, true, false>), grid, block, 0, s, b);
  else if (grad)
    hipLaunchKernelGGL((apply_bmfma<P, false, true>), grid, block, 0, s, b);
  else
    hipLaunchKernelGGL((apply_bmfma<P, false, false>), grid, block, 0, s, b);
  return hip_check_b(hipGetLastError(), "apply (band MFMA) launch");
}

// Tile shape per order: ~64 columns (TYE = 64/P element positions) so a wave spans one tile line;
// TXE element columns for ~512-node tiles; rows of an element split over NS threads.
template <int P>
struct BandShape {
  static constexpr int TYE = (64 / P) > 0 ? 64 / P : 1;
  static constexpr int TXE = (8 / P) > 4 ? 4 : ((8 / P) > 0 ? 8 / P : 1);
  static constexpr int NS = P >= 2 ? 2 : 1;
};

template <int P>
static int launch_band_auto(const ApplyArgs& args, const sem_handle* h, hipStream_t s) {
  using S = BandShape<P>;
  // coefficient mode: DPP-broadcast lists from ~1M DOFs up (the issue-bound regime), fp64 immediates below (the
  // launch-latency-bound meshes, whose extra coefficient loads sit on the critical path: profiles/r01/band/dpp_ab.txt);
  // SEM_BAND_TILE = 3 / 4 forces DPP / immediates (the bitwise-variant tests)
  const int force = tune(SEM_TUNE_BAND_TILE);
  const bool dpp = force == 3 || (force != 4 && args.n_local32 >= (1 << 20));
  if (dpp) return launch_band<P, S::TXE, S::TYE, S::NS, 1>(args, h, s);
  return launch_band<P, S::TXE, S::TYE, S::NS, 0>(args, h, s);
}

std::string band_kernel_name(int P, long long n_local) {
  const int TYE = std::max(1, 64 / P), TXE = std::min(4, std::max(1, 8 / P));
  const int NS = P >= 2 ? 2 : 1;
  const int force = tune(SEM_TUNE_BAND_TILE);
  const bool dpp = force == 3 || (force != 4 && n_local >= (1 << 20));
  const bool kp = tune(SEM_TUNE_BAND_KP) >= 0;
  return std::string(kp ? "sem::apply_band_kp<" : "sem::apply_band<") + std::to_string(P) + ", " + std::to_string(TXE) +
         ", " + std::to_string(TYE) + ", " + std::to_string(NS) + (dpp ? ", dpp" : "") + ">";
}

int launch_apply_bmfma(const ApplyArgs& a, const sem_handle* h, hipStream_t s) {
  switch (h->P) {
#define SEM_BMCASE(PP) \
  case PP:             \
    return launch_bmfma<PP>(a, h, s);
    SEM_BMCASE(1) SEM_BMCASE(2) SEM_BMCASE(3) SEM_BMCASE(4) SEM_BMCASE(5) SEM_BMCASE(6) SEM_BMCASE(7) SEM_BMCASE(8)
    SEM_BMCASE(9) SEM_BMCASE(10) SEM_BMCASE(11) SEM_BMCASE(12) SEM_BMCASE(13) SEM_BMCASE(14) SEM_BMCASE(15)
    SEM_BMCASE(16)
#undef SEM_BMCASE
    default:
      return set_error(SEM_EUNSUPPORTED, "polynomial order outside compiled range");
  }
}

std::string bmfma_kernel_name(int P) {
  const int TXE = std::max(1, 16 / P);
  return "sem::apply_bmfma<" + std::to_string(P) + ", " + std::to_string(TXE * P) + " x " +
         std::to_string(4 * TXE * P) + ">";
}

int launch_apply_band(const ApplyArgs& a, const sem_handle* h, hipStream_t s) {
  switch (h->P) {
#define SEM_BCASE(PP) \
  case PP:            \
    return launch_band_auto<PP>(a, h, s);
    SEM_BCASE(1) SEM_BCASE(2) SEM_BCASE(3) SEM_BCASE(4) SEM_BCASE(5) SEM_BCASE(6) SEM_BCASE(7) SEM_BCASE(8)
    SEM_BCASE(9) SEM_BCASE(10) SEM_BCASE(11) SEM_BCASE(12) SEM_BCASE(13) SEM_BCASE(14) SEM_BCASE(15) SEM_BCASE(16)
#undef SEM_BCASE
    default:
      return set_error(SEM_EUNSUPPORTED, "polynomial order outside compiled range");
  }
}

}  // namespace sem
