// Host-side GLL reference-element tables and connectivity for libsemops.
//
// Restates the published GLL construction used by Solvers/GLL.py: Newton
// iteration on the Chebyshev-Gauss-Lobatto guess with the Legendre three-term
// recurrence (GLL.py:13-28), weights 2/(P(P+1)L_P^2) (GLL.py:31), the
// barycentric-style differentiation matrix (GLL.py:51-58), and the derived
// G = W D, K = D^T W D tables (GLL.py:62-81).  Operation order follows the
// reference element-wise NumPy expressions so the fp64 bits agree with it
// (FP contraction is disabled for this translation unit by the build).
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "sem_internal.h"

#pragma clang fp contract(off)

namespace sem {

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
void clear_error() { g_last_error.clear(); }
const char* last_error() { return g_last_error.c_str(); }

static int env_int(const char* name) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : 0;
}

Tuning& tuning() {
  static Tuning t = [] {  // the environment is read once, at the first use
    Tuning r{};
    r.v[SEM_TUNE_BAND_TILE] = env_int("SEM_BAND_TILE");
    const char* kp = std::getenv("SEM_BAND_KP");  // SEM_BAND_KP=0: struct-only kernel arguments
    r.v[SEM_TUNE_BAND_KP] = (kp && std::atoi(kp) == 0) ? -1 : 0;
    r.v[SEM_TUNE_MFMA_TILE] = env_int("SEM_MFMA_TILE");
    r.v[SEM_TUNE_NS_APPLY] = env_int("SEM_NS_APPLY");
    r.v[SEM_TUNE_EDGE_THOMAS] = env_int("SEM_EDGE_THOMAS");
    return r;
  }();
  return t;
}

#if SEM_DIAGNOSTICS
int diag_bits() {
  static const int d = env_int("SEM_DIAG");  // ablation bits: results are wrong when set (diagnostic builds only)
  return d;
}
unsigned long long* diag_stamps() {
  static unsigned long long* p = [] {
    const char* e = std::getenv("SEM_DIAG_BUF");  // device address of a stamp buffer
    return e ? reinterpret_cast<unsigned long long*>(std::strtoull(e, nullptr, 0)) : nullptr;
  }();
  return p;
}
#else
int diag_bits() { return 0; }
unsigned long long* diag_stamps() { return nullptr; }
#endif

int gll_nodes(int P, double* xi, double* w, double* V) {
  if (P < 1 || P > 64) return set_error(SEM_EINVAL, "polynomial order must be in [1, 64]");
  const int n = P + 1;
  std::vector<double> x(n), vd(static_cast<size_t>(n) * n, 0.0), upd(n, 1.0);
  const double pi = 3.141592653589793;
  for (int k = 0; k < n; ++k) x[k] = -std::cos(pi * static_cast<double>(k) / static_cast<double>(P));
  const double eps = std::numeric_limits<double>::epsilon();
  for (int iter = 0; iter < 1000; ++iter) {
    double maxu = 0.0;
    for (int k = 0; k < n; ++k) maxu = std::fmax(maxu, std::fabs(upd[k]));
    if (!(maxu > eps)) break;
    for (int r = 0; r < n; ++r) {
      double* row = &vd[static_cast<size_t>(r) * n];
      row[0] = 1.0;
      row[1] = x[r];
      for (int k = 2; k <= P; ++k)
        row[k] = ((2.0 * k - 1.0) * x[r] * row[k - 1] - (k - 1.0) * row[k - 2]) / static_cast<double>(k);
    }
    for (int r = 0; r < n; ++r) {
      const double* row = &vd[static_cast<size_t>(r) * n];
      upd[r] = -(x[r] * row[P] - row[P - 1]) / ((P + 1.0) * row[P]);
    }
    for (int r = 0; r < n; ++r) x[r] = x[r] + upd[r];
  }
  for (int r = 0; r < n; ++r) {
    if (xi) xi[r] = x[r];
    const double lp = vd[static_cast<size_t>(r) * n + P];
    if (w) w[r] = 2.0 / (static_cast<double>(P * (P + 1)) * (lp * lp));
  }
  if (V) std::memcpy(V, vd.data(), sizeof(double) * vd.size());
  return SEM_OK;
}

int gll_differentiation(int P, double* D) {
  const int n = P + 1;
  std::vector<double> x(n), V(static_cast<size_t>(n) * n);
  int st = gll_nodes(P, x.data(), nullptr, V.data());
  if (st) return st;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double d = 0.0;
      // (V_iP / V_jP * 1) / (x_i - x_j), the reference's left-to-right order (GLL.py:56)
      if (i != j) d = V[static_cast<size_t>(i) * n + P] / V[static_cast<size_t>(j) * n + P] / (x[i] - x[j]);
      D[static_cast<size_t>(i) * n + j] = d;
    }
  D[0] = -P * (P + 1) / 4.0;
  D[static_cast<size_t>(n) * n - 1] = P * (P + 1) / 4.0;
  return SEM_OK;
}

int gll_gradient(int P, double* G) {
  const int n = P + 1;
  std::vector<double> w(n);
  int st = gll_nodes(P, nullptr, w.data(), nullptr);
  if (st) return st;
  st = gll_differentiation(P, G);
  if (st) return st;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) G[static_cast<size_t>(i) * n + j] = w[i] * G[static_cast<size_t>(i) * n + j];
  return SEM_OK;
}

int gll_stiffness(int P, double* K) {
  const int n = P + 1;
  std::vector<double> w(n), D(static_cast<size_t>(n) * n);
  int st = gll_nodes(P, nullptr, w.data(), nullptr);
  if (st) return st;
  st = gll_differentiation(P, D.data());
  if (st) return st;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int k = 0; k < n; ++k) s += w[k] * D[static_cast<size_t>(k) * n + i] * D[static_cast<size_t>(k) * n + j];
      K[static_cast<size_t>(i) * n + j] = s;
    }
  return SEM_OK;
}

int gll_evaluation(int P, const double* xe, int64_t count, double* S) {
  const int n = P + 1;
  std::vector<double> x(n);
  int st = gll_nodes(P, x.data(), nullptr, nullptr);
  if (st) return st;
  for (int64_t q = 0; q < count; ++q)
    for (int j = 0; j < n; ++j) {
      double prod = 1.0;
      bool first = true;
      for (int k = 0; k < n; ++k) {
        if (k == j) continue;
        const double f = (xe[q] - x[k]) / (x[j] - x[k]);
        prod = first ? f : prod * f;
        first = false;
      }
      S[q * n + j] = prod;
    }
  return SEM_OK;
}

int global_index(int P, int nex, int ney, const int64_t* m, const int64_t* n, const int64_t* i, const int64_t* j,
                 int64_t count, int64_t* out) {
  if (P < 1 || nex < 1 || ney < 1) return set_error(SEM_EINVAL, "P, N_ex, N_ey must be positive");
  // Same range test as the reference (SEM.py:108-109): upper bounds only.
  for (int64_t q = 0; q < count; ++q)
    if (m[q] >= nex || n[q] >= ney || i[q] > P || j[q] > P) return set_error(SEM_EINVAL, "Indices out of range");
  const int64_t NY = static_cast<int64_t>(ney) * P + 1;
  for (int64_t q = 0; q < count; ++q) out[q] = n[q] * P + j[q] + NY * (m[q] * P + i[q]);
  return SEM_OK;
}

}  // namespace sem

// One column of the GMRES least-squares update, on the host (sem_amd/krylov.py): the k earlier Givens rotations
// applied to col[0..k+1] in order, rotation k formed from (col[k], col[k+1]) and applied to col and to the rotated
// right-hand side g[k], g[k+1].  The same operations, in the same order and without contraction, as the Python
// loop it replaces (bitwise equal results); that loop cost ~0.6 us per earlier rotation in the interpreter,
// i.e. ~1 ms per Arnoldi step at the 1,600-2,600-step NS Schur solves of cfg4 at Ra = 1e6, with the GPU idle.
extern "C" int sem_givens_column(double* col, double* cs, double* sn, double* g, int k) {
#pragma clang fp contract(off)
  if (!col || !cs || !sn || !g || k < 0) return sem::set_error(SEM_EINVAL, "givens_column: bad argument");
  for (int i = 0; i < k; ++i) {
    const double c = cs[i], s = sn[i], a = col[i], b = col[i + 1];
    col[i] = c * a + s * b;
    col[i + 1] = -s * a + c * b;
  }
  const double den = std::hypot(col[k], col[k + 1]);
  if (den == 0.0) {
    cs[k] = 1.0;
    sn[k] = 0.0;
  } else {
    cs[k] = col[k] / den;
    sn[k] = col[k + 1] / den;
  }
  col[k] = cs[k] * col[k] + sn[k] * col[k + 1];
  col[k + 1] = 0.0;
  g[k + 1] = -sn[k] * g[k];
  g[k] = cs[k] * g[k];
  return SEM_OK;
}

#ifndef SEM_BUILD_ID
#define SEM_BUILD_ID "unknown"
#endif
extern "C" const char* sem_build_id(void) { return sem::kDiag ? SEM_BUILD_ID "+diag" : SEM_BUILD_ID; }
