// Internal declarations shared by the libsemops translation units.
#pragma once

#include <cstdint>
#include <string>

#include "../../include/sem_ops.h"

namespace sem {

// Thread-local last-error text (sem_last_error); returns `code` for chaining.
int set_error(int code, const std::string& msg);
void clear_error();
const char* last_error();

int gll_nodes(int P, double* xi, double* w, double* V);
int gll_differentiation(int P, double* D);
int gll_gradient(int P, double* G);
int gll_stiffness(int P, double* K);
int gll_evaluation(int P, const double* xe, int64_t count, double* S);
int global_index(int P, int nex, int ney, const int64_t* m, const int64_t* n, const int64_t* i, const int64_t* j,
                 int64_t count, int64_t* out);

constexpr int kMaxOrder = 16;  // largest P with a compiled device kernel

// Diagnostic builds only (python -m sem_amd.build --diag): ablation bits and per-wave phase
// stamps for performance analysis.  The shipped library is built with SEM_DIAGNOSTICS=0: the
// ablation paths are compiled out and no environment variable can reach them.
#ifndef SEM_DIAGNOSTICS
#define SEM_DIAGNOSTICS 0
#endif
constexpr bool kDiag = SEM_DIAGNOSTICS != 0;

// Kernel-selection knobs (enum sem_tune).  They pick among variants that compute bitwise-identical
// results (tile shapes, cache policies, argument passing), so they never change an answer.  They
// are read from the environment once, at the first use, and changed afterwards only through
// sem_set_tuning (in-process A/B tools).  0 = library default.
struct Tuning {
  int v[SEM_TUNE_COUNT];
};
Tuning& tuning();
inline int tune(int knob) { return tuning().v[knob]; }

// Diagnostic state (SEM_DIAGNOSTICS builds only): SEM_DIAG bits and the SEM_DIAG_BUF stamp buffer.
int diag_bits();
unsigned long long* diag_stamps();

}  // namespace sem

// Immutable per-(device, partition) state.  Device table layout (doubles):
//   [0, n*n)        K_s  (GLL.py:73-81)
//   [n*n, 2n*n)     G_s  (GLL.py:62-70)
//   [2n*n, 2n*n+n)  w    (GLL.py:31)
struct sem_handle {
  int P, nex, ney, ex_begin, ex_end, device;
  double dx, dy;
  int64_t NX, NY, N, line_begin, line_end, n_local;
  double* d_tab;
};
