/*
 * sem_ops.h -- C ABI of the MI355X-native SEM operator layer (libsemops.so).
 *
 * Drop-in boundary for the hot path of Tangxiaotian11/SEM: the GLL reference
 * tables of Solvers/GLL.py and the global operator / assembly API of
 * Solvers/SEM.py, applied matrix-free on gfx950.  Every entry point names the
 * reference interface it replaces.  The reference is pure Python, so the
 * "binding a maintainer would add" is the ctypes layer in sem_amd/_lib.py
 * (shown in INTEGRATION.md); no torch types cross this boundary.
 *
 * Conventions
 *   - All arithmetic is IEEE fp64.  Vectors are global-DOF vectors in the
 *     reference's x-major numbering p = (N_ey*P+1)*(m*P+i) + n*P+j
 *     (SEM.py:97-110), restricted to the handle's local line range.
 *   - Device pointers are plain device (HBM) pointers; `stream` is a
 *     hipStream_t passed as void* (NULL = default stream).  Every device call
 *     is asynchronous and stream-ordered; nothing is allocated or synchronised
 *     inside an apply, so applies may be captured into a hipGraph.
 *   - Status codes: 0 = ok, otherwise SEM_E*.  No exceptions cross the ABI;
 *     sem_last_error() returns a thread-local message for the last failure.
 *     The Python wrapper maps SEM_EINVAL -> ValueError (the reference raises
 *     ValueError for bad indices / vector lengths, SEM.py:18-19,108-109,158-159)
 *     and everything else -> RuntimeError.
 *   - Handles are immutable after sem_create: concurrent applies on distinct
 *     streams are safe.
 */
#ifndef SEM_OPS_H
#define SEM_OPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SEM_ABI_VERSION 15

enum sem_status {
  SEM_OK = 0,
  SEM_EINVAL = 1,       /* bad argument (maps to ValueError) */
  SEM_EHIP = 2,         /* HIP runtime error */
  SEM_ENOMEM = 3,       /* device allocation failed */
  SEM_EUNSUPPORTED = 4  /* e.g. polynomial order outside the compiled range */
};

/* Dirichlet side bits (used when no explicit mask is given). */
enum sem_side { SEM_SIDE_W = 1u, SEM_SIDE_E = 2u, SEM_SIDE_S = 4u, SEM_SIDE_N = 8u };

/* Dirichlet row modes applied after the operator (and after any accumulate). */
enum sem_dir_mode {
  SEM_DIR_NONE = 0,     /* plain operator rows                                        */
  SEM_DIR_IDENTITY = 1, /* y[p] = x[p] - g[p] (g = dir_val, NULL -> 0):
                           ConvectionDiffusion_Solver.py:90 (res) and :119 (dres)      */
  SEM_DIR_REPLACE = 2   /* y[p] = dir_val[p]                                            */
};

/* Kernel selection.  All compute the same operator (parity-tested against each other and the
 * oracle); AUTO picks by mesh size from MI355X measurements. */
enum sem_algo {
  SEM_ALGO_AUTO = 0,
  SEM_ALGO_VALU = 1,   /* two-phase VALU tile kernel (x and y contractions in separate passes)   */
  SEM_ALGO_MFMA = 2,   /* fp64 MFMA (v_mfma_f64_16x16x4_f64) element-block contractions, P <= 15 */
  SEM_ALGO_COLUMN = 3, /* single-phase VALU column kernel                                         */
  SEM_ALGO_BAND = 4    /* assembled-band VALU kernel: one banded dot product per node and direction,
                          x / y roles on separate waves, wave-uniform compile-time coefficients   */
};

typedef struct sem_handle sem_handle;

/* Static description of a handle (all sizes in DOFs / lines). */
typedef struct sem_info {
  int P, nex, ney, ex_begin, ex_end, device;
  double dx, dy;
  int64_t NX, NY;       /* global node lines in x / nodes per line (N_ex*P+1, N_ey*P+1) */
  int64_t N;            /* global DOFs = NX*NY  (ConvectionDiffusion_Solver.py:50)       */
  int64_t line_begin;   /* first global line held locally = ex_begin*P                   */
  int64_t line_end;     /* last global line held locally  = ex_end*P   (inclusive)       */
  int64_t n_local;      /* local vector length = (line_end-line_begin+1)*NY              */
  int64_t dof_begin;    /* global DOF index of local element 0 = line_begin*NY           */
} sem_info;

/*
 * Fused operator descriptor.  One launch computes
 *     z = c_mass*M x + c_stiff*K x + c_gradx*cu.(G_x x) + c_grady*cv.(G_y x)
 *         + c_extra*(ea.eb + ec.ed) + c_acc*y_in
 * then applies the Dirichlet rows, and writes y.
 *   M, K, G_x, G_y : SEM.global_{mass,stiffness,gradient}_matrices (SEM.py:170-223)
 *   cu.(G_x x)     : Pe * tensordot(C_x, u, (1,0)) @ x  == diag(u) G_x x
 *                    (SEM.py:226-245 contracted at ConvectionDiffusion_Solver.py:82-83)
 *   ea.eb          : Jacobian terms Pe*tensordot(C_x, T, (2,0)) @ du == (G_x T).du
 *                    (ConvectionDiffusion_Solver.py:101-102,114-116)
 * NULL cu/cv mean "all ones"; an extra pair (ea,eb) or (ec,ed) is skipped when
 * either of its pointers is NULL.  c_acc != 0 reads y before overwriting it.
 * x must not alias y.
 * On a strip handle (ex_end < N_ex) the rows of the right interface line x = ex_end*P are partial
 * sums of the local elements; the pointwise terms (c_extra, c_acc) and Dirichlet rows of that line
 * are left to the right-hand owner, so that the interface exchange (sum of the two strips'
 * values) gives the assembled row.
 */
typedef struct sem_apply_desc {
  double c_mass, c_stiff, c_gradx, c_grady;
  const double* cu;
  const double* cv;
  double c_extra;
  const double* ea;
  const double* eb;
  const double* ec;
  const double* ed;
  double c_acc;
  int dir_mode;              /* enum sem_dir_mode */
  const uint8_t* dir_mask;   /* nullable: per-DOF mask (np.isclose-derived masks) */
  const double* dir_val;     /* nullable */
  unsigned dir_sides;        /* SEM_SIDE_* bits used when dir_mask == NULL */
  int algo;                  /* enum sem_algo */
  /* Element-position range [pos_begin, pos_end) of the handle's strip whose output lines are
   * written (position p < ncols = ex_end - ex_begin covers lines (ex_begin+p)*P ..+P-1, position
   * ncols the closing line ex_end*P); every other entry of y is left untouched.  pos_end = 0:
   * all positions.  Each written node is the full (local) operator row, so applying the
   * interface positions and the interior positions in separate launches gives the same y as one
   * launch: the multi-GPU step overlaps the interface exchange with the interior launch.
   * Band kernel only (AUTO / BAND). */
  int pos_begin, pos_end;
} sem_apply_desc;

/* Kernel-selection knobs (test / A-B use only).  Defaults come from the environment variable named
 * beside each knob, read ONCE at the first use; 0 = library default.  The values are PROCESS-GLOBAL
 * and unsynchronised: sem_set_tuning is not thread-safe, and a knob changed while launches are in
 * flight on other threads or streams affects whichever launches read it afterwards.  Set knobs from
 * one thread before launching; the handles themselves stay immutable (include note in sem_create).
 * Round 6 retired the knobs whose A/B lost (their enum values stay reserved; sem_set_tuning returns
 * SEM_EINVAL for them): band cache policy, marching kernel, tile order, GEMV / basis / condensed-solve
 * load policies, GEMV shapes, the band kernel's other tiles and scalar-load coefficients, the column
 * kernel's other tiles, the two-ended edge sweep. */
enum sem_tune {
  SEM_TUNE_BAND_TILE = 0, /* SEM_BAND_TILE: 3 = DPP-broadcast coefficients, 4 = fp64 immediates (the
                           * band kernel picks by mesh size; bitwise-identical results)              */
  SEM_TUNE_RETIRED_1 = 1,
  SEM_TUNE_BAND_KP = 2,   /* SEM_BAND_KP: -1 = struct-only kernel arguments, else preloaded (bitwise) */
  SEM_TUNE_RETIRED_3 = 3,
  SEM_TUNE_MFMA_TILE = 4, /* SEM_MFMA_TILE: 0 = band-form MFMA kernel; 3 = element-block MFMA (round 4) */
  SEM_TUNE_RETIRED_5 = 5,
  SEM_TUNE_NS_APPLY = 6,  /* SEM_NS_APPLY: 1 = sem_ns_apply's LDS-tile form instead of the band form
                           * (agree to rounding, not bitwise)                                         */
  SEM_TUNE_EDGE_THOMAS = 7, /* SEM_EDGE_THOMAS: 1 = the ABI-9 runtime-width edge sweep of sem_nested_solve
                             * instead of the templated one (agree to rounding)                     */
  SEM_TUNE_RETIRED_8 = 8,
  SEM_TUNE_RETIRED_9 = 9,
  SEM_TUNE_RETIRED_10 = 10,
  SEM_TUNE_RETIRED_11 = 11,
  SEM_TUNE_RETIRED_12 = 12,
  SEM_TUNE_COUNT = 13
};

/* ---- library ------------------------------------------------------------ */
int sem_abi_version(void);
const char* sem_last_error(void);
/* Largest polynomial order with a compiled device kernel. */
int sem_max_order(void);
/* Hash of the sources and headers the library was built from (sem_amd/build.py embeds it); the
 * Python loader refuses a library whose hash differs from the in-tree sources.  A "+diag" suffix
 * marks a diagnostic build. */
const char* sem_build_id(void);
/* Set / read a kernel-selection knob (enum sem_tune); SEM_EINVAL for an unknown or retired knob.
 * Not thread-safe (process-global state, see enum sem_tune). */
int sem_set_tuning(int knob, int value);
int sem_get_tuning(int knob, int* value);

/* ---- GLL reference element (host), Solvers/GLL.py ------------------------ */
/* GLL.standard_nodes (GLL.py:7-33): xi[P+1], w[P+1], V[(P+1)^2] row-major (V nullable). */
int sem_gll_nodes(int P, double* xi, double* w, double* V);
/* GLL.standard_differentiation_matrix (GLL.py:45-59): D[i*(P+1)+j] = l'_j(xi_i). */
int sem_gll_differentiation(int P, double* D);
/* GLL.standard_gradient_matrix (GLL.py:62-70): G[i][j] = w_i D_ij. */
int sem_gll_gradient(int P, double* G);
/* GLL.standard_stiffness_matrix (GLL.py:73-81): K[i][j] = sum_k w_k D_ki D_kj. */
int sem_gll_stiffness(int P, double* K);
/* GLL.standard_evaluation_matrix (GLL.py:105-116): S[q*(P+1)+j] = l_j(xi_eval[q]). */
int sem_gll_evaluation(int P, const double* xi_eval, int64_t count, double* S);

/* ---- connectivity (host), Solvers/SEM.py ------------------------------- */
/* SEM.global_index (SEM.py:97-110), vectorised; SEM_EINVAL if any index is out of range. */
int sem_global_index(int P, int nex, int ney, const int64_t* m, const int64_t* n, const int64_t* i,
                     const int64_t* j, int64_t count, int64_t* out);

/* ---- handles ------------------------------------------------------------ */
/* Mesh of nex x ney elements of order P, widths dx, dy; this handle holds the
 * element columns [ex_begin, ex_end) (ex_begin=0, ex_end=nex for one GPU).
 * Uploads the reference-element tables to `device`. */
int sem_create(int P, int nex, int ney, double dx, double dy, int ex_begin, int ex_end, int device,
               sem_handle** out);
int sem_destroy(sem_handle* h);
int sem_get_info(const sem_handle* h, sem_info* out);

/* ---- device operators ------------------------------------------------- */
/* Fused matrix-free operator apply (see sem_apply_desc).  x, y: n_local doubles. */
int sem_apply(sem_handle* h, const sem_apply_desc* d, const double* x, double* y, void* stream);

/* Name of the kernel sem_apply launches for this handle and algorithm (for profiles / reports). */
int sem_kernel_name(const sem_handle* h, int algo, char* buf, int len);

/* SEM.scatter (SEM.py:149-167): u_e[m][n][i][j] = u[global_index(m,n,i,j)] for the
 * local elements; u_e has (ex_end-ex_begin)*ney*(P+1)^2 doubles. */
int sem_gather_elements(sem_handle* h, const double* u, double* u_e, void* stream);

/* SEM.assemble for a 4-D element array (SEM.py:113-127,146): direct-stiffness
 * summation a[p] = sum over elements holding p of a_e[m][n][i][j], summed in the
 * reference's (m,n) lexicographic order starting from +0.0 (bit-exact). */
int sem_dss(sem_handle* h, const double* a_e, double* a, void* stream);

/* SEM.eval_interpolation (SEM.py:248-273) for an ij-meshgrid of plot points:
 * out[a*nb+b] = sum_kl Sx[a][k] u_e[m_idx[a]][n_idx[b]][k][l] Sy[b][l], where m_idx / Sx are
 * the element index and Lagrange evaluation row (GLL.standard_evaluation_matrix) of plot
 * row a (SEM.x2xi, SEM.py:23-36) and n_idx / Sy those of plot column b.  Entries whose
 * element is not held locally are left untouched.  All pointers are device pointers. */
int sem_eval_interpolation(sem_handle* h, const double* u_e, int na, const int* m_idx, const double* Sx, int nb,
                           const int* n_idx, const double* Sy, double* out, void* stream);

/* ---- multi-GPU interface lines (element-strip partition) --------------- */
/* Pack the local partial sums on the two interface lines into buf[(G-1)*NY]
 * (slot s = global line (s+1)*... of partition boundary s), zeros elsewhere;
 * `bounds` = the G+1 element-column boundaries of the partition.  After a sum
 * all-reduce of buf over all ranks, sem_interface_unpack writes the assembled
 * values back into y. */
int sem_interface_pack(sem_handle* h, const double* y, const int* bounds, int G, double* buf,
                       void* stream);
int sem_interface_unpack(sem_handle* h, const double* buf, const int* bounds, int G, double* y,
                         void* stream);

/* ---- Krylov-basis sweeps (device GMRES, sem_amd/krylov.py) ------------- */
/* Replace the Arnoldi orthogonalisation of the reference's LGMRES
 * (ConvectionDiffusion_Solver.py:146-148, NavierStokes_Solver.py:222-224; SciPy's
 * lgmres inner loop) on a basis V of k rows of n doubles, row pitch ldv, in device memory.
 * sem_basis_dot2:   out[2j] = V_j . a, out[2j+1] = V_j . b (one pass over V; fixed summation
 *                   order, bitwise reproducible); work: sem_basis_dot2_work_size(k, n) doubles.
 * sem_basis_update: w -= V^T c (one pass over V).
 * Stream-ordered; all pointers are device pointers. */
int64_t sem_basis_dot2_work_size(int k, int64_t n);
int sem_basis_dot2(const double* V, int64_t ldv, int k, int64_t n, const double* a, const double* b, double* work,
                   double* out, void* stream);
int sem_basis_update(const double* V, int64_t ldv, int k, int64_t n, const double* c, double* w, void* stream);

/* ---- Navier-Stokes velocity Jacobian (device direct solve) --------------- */
/* Replaces the host-side materialisation of the 2N x 2N velocity Jacobian for SuperLU
 * (NavierStokes_Solver.py:176-184: sp_sparse.bmat of the four Jacobian blocks, Dirichlet rows
 * set to identity, splu).  The Jacobian
 *     J_uu = A + diag(juu), J_uv = diag(juv), J_vu = diag(jvu), J_vv = A + diag(jvv),
 *     A = c_mass M + c_stiff K + c_gradx diag(cu) G_x + c_grady diag(cv) G_y
 * (Sys = K + Re(u@C_x + v@C_y), :106; Jacobians :131-136) is written as the pieces of its static
 * condensation over node lines (see sem_amd/csrc/ns_velocity.hip for the layout): dense
 * interior blocks A_II per element column, dense interface-line blocks D, and the diagonal
 * line-to-line couplings aIB, aBI, E, F.  Rows in the Dirichlet set (dir_mask, or dir_sides when
 * dir_mask is NULL) are identity rows.  Whole-mesh handles only.  Sizes (doubles) from
 * sem_velocity_block_sizes: sizes[0..5] = A_II, D, aIB, aBI, E, F. */
typedef struct sem_velocity_desc {
  double c_mass, c_stiff, c_gradx, c_grady;
  const double* cu;   /* nullable = ones */
  const double* cv;
  const double* juu;  /* nullable = zeros */
  const double* juv;
  const double* jvu;
  const double* jvv;
  const uint8_t* dir_mask;
  unsigned dir_sides;
  int ncomp;          /* 0 or 2: the velocity pair; 1: the scalar operator A + diag(juu) alone (the
                       * convection-diffusion Jacobian, ConvectionDiffusion_Solver.py:104-121) */
  int col_begin;      /* ABI 6: A_II holds element columns [col_begin, col_end) only (col_end 0 = all), */
  int col_end;        /* so a large mesh's dense interiors are assembled a chunk of columns at a time */
} sem_velocity_desc;
/* Sizes for ncomp components per node (m = ncomp N_y unknowns per line); the velocity form is
 * sem_line_block_sizes(h, 2, sizes). */
int sem_line_block_sizes(const sem_handle* h, int ncomp, int64_t* sizes);
int sem_velocity_block_sizes(const sem_handle* h, int64_t* sizes);
int sem_velocity_blocks(sem_handle* h, const sem_velocity_desc* d, double* A_II, double* D, double* aIB, double* aBI,
                        double* E, double* F, void* stream);
/* ABI 7: the same Jacobian with the interior rows of element columns [col_begin, col_end) written straight
 * into the layout of the nested condensation (VelocityJacobianSolver.factor_condensed) instead of a dense
 * A_II per column: per element n of a column the interior block A_ii (ni x ni), its couplings to the
 * column's horizontal edges n, n+1 A_ie (ni x 2 ne1) and A_ei (2 ne1 x ni); per column the block-tridiagonal
 * edge operator A_ee as diagonal blocks Aed (N_ey+1 of ne1 x ne1), upper blocks Aeu (edge k -> k+1) and
 * lower blocks Ael (edge k+1 -> k), N_ey each.  Row-major blocks; element-interior unknown
 * ((l-1) nc + c)(P-1) + j-1 = line l, component c, y node nP + j; edge unknown (l-1) nc + c.  The interface
 * pieces D, aIB, aBI, E, F are as sem_velocity_blocks writes them.  P >= 2.  Per-column sizes (doubles)
 * from sem_condensed_block_sizes: sizes[0..5] = A_ii, A_ie, A_ei, Aed, Aeu, Ael (times col_end - col_begin
 * columns).  Replaces the 9 GB dense column interiors the ABI-6 path assembled per cfg5 column. */
int sem_condensed_block_sizes(const sem_handle* h, int ncomp, int64_t* sizes);
int sem_condensed_blocks(sem_handle* h, const sem_velocity_desc* d, double* Aii, double* Aie, double* Aei,
                         double* Aed, double* Aeu, double* Ael, double* D, double* aIB, double* aBI, double* E,
                         double* F, void* stream);

/* ---- nested interior solve of the condensation (velocity / CD Jacobian) ---- */
/* y = A_II^-1 r for every element column at once, from the factor VelocityJacobianSolver keeps
 * (sem_amd/solvers/velocity_solve.py; layouts in sem_amd/csrc/ns_condense.hip): per element the
 * interior inverse Xi (ni x ni), A_ei (2 ne1 x ni) and Xi A_ie (ni x 2 ne1), per column the inverse
 * edge Schur block Se (n_e x n_e), every block stored column-major; pi (N_ey, ni) and pe (n_e) are the column-interior offsets of
 * the element interiors and edges; T, C, Ye are work arrays of nex N_ey ni, nex N_ey 2 ne1 and
 * nex n_e doubles.  ni = nc (P-1)^2, ne1 = nc (P-1), n_e = (N_ey+1) ne1, m = nc N_y.  Replaces the
 * reference's SuperLU triangular solves (NavierStokes_Solver.py:189-203). */
typedef struct sem_nested_desc {
  int P, nex, ney, nc;
  int64_t NY;
  const double* Xi;
  const double* Aei;
  const double* Yie;
  const double* Se;
  const int64_t* pi;
  const int64_t* pe;
  double* T;
  double* C;
  double* Ye;
  /* ABI 9: the edge Schur complement as its block-Thomas factors instead of the dense inverse Se (Se = NULL):
   * per column Ed[k] = inverse pivot block k (N_ey+1 of ne1 x ne1), El[k] = lower block (edge k+1 <- k) and
   * Eu[k] = Ed[k] A_up[k] (edge k <- k+1), N_ey each; the edge solve is then a forward and a
   * back sweep over the column's N_ey+1 edges (one wavefront per column) reading O(N_ey ne1^2) doubles
   * instead of the n_e^2 of the dense inverse (cfg5: 1.5 MB instead of 64 MB per column).  ne1 <= 32.
   * ABI 10: these three are stored ROW-major (half-rows are 16-byte vector loads in the templated sweep), and
   * the sweep computes the edge offsets as pe[k ne1 + (l-1) nc + c] = (l-1) m + c N_y + k P instead of
   * loading pe (the layout VelocityJacobianSolver._nested_index builds). */
  const double* Ed;
  const double* El;
  const double* Eu;
  /* ABI 11 (nullable): per element XiB = Xi A_iB (ni x 2 ne1) and AXB = A_ei Xi A_iB (2 ne1 x 2 ne1), column-major,
   * where A_iB couples element n's interior to the interface nodes at its interior heights (columns ordered
   * (side s, component c, height j = 1..P-1): x_B[e+s][c N_y + n P + j]).  Used by sem_nested_back_solve. */
  const double* XiB;
  const double* AXB;
  /* (nullable) per element ABY = A_Bi Xi A_ie (2 ne1 x 2 ne1, column-major; rows (s, c, j) as XiB's columns,
   * columns edges n, n+1), and a work array Pw of nex * 2 * m doubles.  Used by sem_nested_iface_rhs. */
  const double* ABY;
  double* Pw;
  /* (ABI 12's two-ended edge sweep -- Es, Edb, Eub, edge_mid -- was removed in ABI 13: without pivoting across
   * its meeting block it lost accuracy on some meshes and made cfg5's coupled solve diverge) */
} sem_nested_desc;
/* Column e's right-hand side at R + e ld_r (interior offsets o = (l-1) m + c N_y + gy), minus
 * aIB[e][l-1][s][.] xB[e+s][.] when aIB and xB are given (the back substitution r = b - A_IB x_B);
 * the solution goes to Y + e ld_y at the same offsets.  Three launches, stream-ordered. */
int sem_nested_solve(const sem_nested_desc* d, const double* R, int64_t ld_r, const double* aIB, const double* xB,
                     double* Y, int64_t ld_y, void* stream);
/* ABI 11: the back substitution x_I = A_II^-1 (b_I - A_IB x_B) of the condensed solve, called right after
 * sem_nested_solve(d, R, ld_r, NULL, NULL, ...) with the SAME R and descriptor (whose work arrays T and C still
 * hold that solve's Xi b_i and A_ei Xi b_i): the element step becomes T -= XiB x_B|n, C -= AXB x_B|n, reading
 * 2 ne1 columns per element instead of Xi's ni (cfg5: 1.65 GB instead of 9.09 GB).  The edge and back steps
 * are sem_nested_solve's with the interface correction (aIB, xB).  Needs d->XiB and d->AXB. */
int sem_nested_back_solve(const sem_nested_desc* d, const double* R, int64_t ld_r, const double* aIB,
                          const double* xB, double* Y, int64_t ld_y, void* stream);
/* ABI 11: the forward half of the condensed solve in one call -- y_I = A_II^-1 b_I (sem_nested_solve's element
 * and edge steps; the element values are NOT formed) and the interface right-hand side
 * g[L] = B[L P] - A_BI y_I of sem_interface_rhs, taken from the element step's T = Xi b_i and the edge values:
 * A_Bi y_i = A_Bi T - ABY [y_e(n); y_e(n+1)] per element, aBI on the edge nodes.  Reads ABY (2 ne1 columns per
 * element) instead of Xi A_ie (ni rows) and writes no y_I.  R: column e's interior at R + e ld_r; B: lines ld_b
 * apart (interface line L at B + L P ld_b); Y receives the edge values at the interior offsets (work, ld_y);
 * g: (nex + 1) x m.  Needs d->ABY and d->Pw.  Follow with sem_nested_back_solve on the same R. */
int sem_nested_iface_rhs(const sem_nested_desc* d, const double* R, int64_t ld_r, const double* B, int64_t ld_b,
                         const double* aBI, double* Y, int64_t ld_y, double* g, void* stream);
/* g[L] = B[L P] - sum_l aBI[L][0][l] yI[L][l] - sum_l aBI[L-1][1][l] yI[L-1][l] (L = 0..nex, rows
 * of m doubles; B rows ld_b apart, yI columns ld_yI apart): the interface right-hand side of the
 * condensed solve. */
int sem_interface_rhs(int P, int nex, int m, const double* B, int64_t ld_b, const double* aBI, const double* yI,
                      int64_t ld_yI, double* g, void* stream);

/* ---- batched block GEMV (interface sweep of the velocity solve) ----------- */
/* y[yrow[b]] (+)= sum_{s<S} M[b][:, s m:(s+1) m] . src[s][xrow[s nb + b]]  for b < nb (S <= 3):
 * one level of the block cyclic reduction that solves the interface system of the condensed
 * velocity Jacobian (sem_amd/solvers/velocity_solve.py), in place of the reference's SuperLU
 * triangular solves (NavierStokes_Solver.py:189-203).  M: (nb, m, S m) row-major; operand row r of
 * src[s] at src[s] + r ld_src[s]; xrow = -1: that operand is absent (its block is skipped); output row
 * yrow[b] at y + yrow[b] ld_y, accumulated when `accumulate`.  Output rows must be distinct and not
 * read by the same call.  S m <= 8192.  src and ld_src are host arrays of S entries; M, the operand
 * rows, y, xrow and yrow are device memory.  Stream-ordered. */
int sem_block_gemv(int nb, int m, int S, const double* M, const double* const* src, const int64_t* ld_src,
                   const int64_t* xrow, double* y, int64_t ld_y, const int64_t* yrow, int accumulate, void* stream);

/* ---- streaming row-major GEMV (the block-Thomas interface sweep) -------- */
/* y = alpha A x + beta y (beta = 0: y is not read) for a row-major M x K operator (row i at A + i lda):
 * one forward ([D^-1 | -D^-1 S_lo], m x 2m) or back (D^-1 S_up, m x m) step of the block-Thomas sweep of
 * the condensed velocity solve (sem_amd/solvers/velocity_solve.py fused_thomas_solve), which replaces the
 * reference's SuperLU triangular solves (NavierStokes_Solver.py:189-203).  Deterministic (fixed summation
 * order).  Device pointers; y must not overlap A or x.  Stream-ordered.  (ABI 10) */
int sem_gemv_rows(int M, int K, double alpha, const double* A, int64_t lda, const double* x, double beta, double* y,
                  void* stream);
/* ABI 11: two independent GEMVs of M rows each in ONE launch, y_j = alpha A_j x_j + beta y_j (j = 0, 1; K_j,
 * lda_j per operator): the two chains of the twisted (two-ended) block-Thomas sweep step together, so the sweep
 * is ~N_ex + 1 dependent launches instead of 2 N_ex (velocity_solve.py twisted_thomas_solve). */
int sem_gemv_rows2(int M, double alpha, double beta, int K0, const double* A0, int64_t lda0, const double* x0,
                   double* y0, int K1, const double* A1, int64_t lda1, const double* x1, double* y1, void* stream);

/* ---- nested-dissection solve of the velocity Jacobian (ABI 14) ---------- */
/* The streaming steps of sem_amd/solvers/nested_dissection.py, which orders the Dirichlet-row-replaced velocity
 * Jacobian by nested dissection of the element grid (the analogue of the fill-reducing column order of the
 * reference's `splu`, NavierStokes_Solver.py:184) and replaces its triangular solves (:189-203).
 * One launch = one level of fronts (or the element leaves): front f has a row-major operator at op[f] (device
 * address; R_f x K_f, leading dimension ld_f: dims[4 f .. 4 f + 2] = R_f, K_f, ld_f; K_f and ld_f even, rows
 * 16-byte aligned), its K_f operand positions in W at xidx[xoff[f] ..] (-1: a zero operand), and
 *   back = 0: stage[yoff[f] + r] = (A_f x)_r
 *   back = 1: W[yidx[yoff[f] + r]] -= (A_f x)_r   (targets distinct and not operands of the same launch).
 * tiles[2 b], tiles[2 b + 1] = (front, first row) of workgroup b; `lanes` lanes per operator row and `rows` rows
 * per workgroup, one of (64, 16 | 4), (32, 16 | 8), (16, 32 | 16), (8, 64 | 32), (4, 128 | 64) (short rows take
 * fewer lanes); kmax >= every K_f of the launch (<= 8192).  All arrays are device memory; deterministic (fixed
 * summation order for a given `lanes`). */
typedef struct sem_front_launch {
  int ntiles, rows, lanes, kmax, back;
  /* form 0: row-major operators, `lanes` lanes per row (above); form 1: each operator stored TRANSPOSED (A^T: K
   * rows of ld_f >= R_f doubles, 8-byte aligned), one thread per output row, rows = 256 (short rows: the deepest
   * separators' |S| = 2 (P - 1) columns). */
  int form;
  const int64_t* op;
  const int32_t* dims;
  const int64_t* xoff;
  const int64_t* yoff;
  const int32_t* tiles;
  const int32_t* xidx;
  const int32_t* yidx;
  double* W;
  double* stage;
} sem_front_launch;
int sem_front_gemv(const sem_front_launch* d, void* stream);
/* stage[i stride + out_off + r] = sum_q coef[(i nnz + q) nrows + r] stage[i stride + pat[q nrows + r]] for items
 * i < nitems, rows r < nrows (pattern shared by the items; entries pat[.] < stride and out_off + nrows <= stride,
 * the operand and output ranges of an item disjoint): the leaves' boundary update A_bi y_i of the nested-dissection
 * forward solve, from the P - 1 couplings of each element-boundary unknown to its line or column.  Device memory. */
int sem_front_sparse_rows(int nitems, int nrows, int nnz, const double* coef, const int32_t* pat, double* stage,
                          int64_t stride, int64_t out_off, void* stream);
/* The write-back of a forward step: W[copy_tgt[i]] = stage[copy_src[i]] (i < ncopy) and
 * W[acc_tgt[j]] -= stage[s] for s = acc_src4[4 j + k], k = 0..3 in order, skipping s = -1 (j < nacc; acc_src4
 * 16-byte aligned).  Targets distinct.  Device memory; stream-ordered. */
int sem_front_scatter(int ncopy, const int32_t* copy_tgt, const int32_t* copy_src, int nacc, const int32_t* acc_tgt,
                      const int32_t* acc_src4, const double* stage, double* W, void* stream);
/* ABI 15: the element leaves' forward step of the two-component (u, v) velocity Jacobian in ONE launch, one
 * workgroup per element.  The element's interior block A_ii = [A_uu D1; D2 A_vv] couples the components only
 * through the diagonal Newton terms D1, D2 (mass-lumped: NavierStokes_Solver.py:123-136), so y_i = A_ii^-1 b_i is
 *   t = A_uu^-1 b_u;  y_v = S_v^-1 (b_v - D2 t);  y_u = t - A_uu^-1 (D1 y_v)      (S_v = A_vv - D2 A_uu^-1 D1)
 * with A_uu^-1 held in registers between its two products: two n x n operators read per element instead of the
 * (2n)^2 of A_ii^-1.  Then y_i is written to W (its interior entries: read by no other element), and the boundary
 * rows g_r = sum_q coef[q nb + r] y[pat[q nb + r]] (A_bi y_i on its line / column pattern) go to
 * stage[e sstride + soff + r] for the scatter.
 * Per element e, at blob + e stride (16-byte aligned, stride even): A_uu^-1 (n x ld), S_v^-1 (n x ld), D1 (ld),
 * D2 (ld), coef (nnz x nb); ld = n rounded up to even, pad entries zero; n = (P - 1)^2 <= 121.
 * iidx[e 2n + k]: W index of interior u node k (k < n), v node k - n (k >= n); pat (nnz x nb): positions in
 * [y_u; y_v].  Deterministic; device memory; stream-ordered. */
typedef struct sem_leaf_launch {
  int nelem, n, ld, nb, nnz;
  int64_t stride;
  const double* blob;
  const int32_t* iidx;
  const int32_t* pat;
  double* W;
  double* stage;
  int64_t sstride, soff;
} sem_leaf_launch;
int sem_leaf_forward(const sem_leaf_launch* d, void* stream);

/* ---- GMRES least-squares column (host) ------------------------------------ */
/* Host memory, no device work (ABI 11): applies the Givens rotations 0..k-1 (cs, sn) to col[0..k+1], forms
 * rotation k from (col[k], col[k+1]) into cs[k], sn[k], applies it to col and to the rotated right-hand side
 * g[k], g[k+1] -- one Arnoldi step's update of the device GMRES (sem_amd/krylov.py), the host half of the
 * Krylov solves that replace the reference's LGMRES (NavierStokes_Solver.py:197-229). */
int sem_givens_column(double* col, double* cs, double* sn, double* g, int k);

/* ---- small dense inverse (leaves of the sweep's pivot inverses) --------- */
/* X = A^-1 for one n x n row-major block, n <= 64 (row r of A at A + r lda, of X at X + r ldx; device
 * memory; X must not overlap A): Gauss-Jordan elimination with partial pivoting in one workgroup (ABI 8).
 * The leaves of the GEMM-recursive inverse of the interface sweep's pivot blocks
 * (sem_amd/linalg.py block_inverse), which replace the reference's SuperLU factorisation of the
 * velocity Jacobian (NavierStokes_Solver.py:176-236).  A singular block yields non-finite entries, not
 * an error: callers check A X - I.  Stream-ordered. */
int sem_dense_inverse_small(const double* A, int64_t lda, double* X, int64_t ldx, int n, void* stream);

/* ---- Navier-Stokes residuals (fused) ------------------------------------ */
/* All three outputs of NavierStokes_Solver._get_residuals (NavierStokes_Solver.py:93-121) or
 * _get_dresiduals (:138-160) in one launch, instead of one sem_apply per operand:
 *     Sys = c_mass M + c_stiff K + c_gradx diag(cu) G_x + c_grady diag(cv) G_y
 *     ru  = Sys u + diag(juu) u + diag(juv) v + G_x p
 *     rv  = diag(jvu) u + Sys v + diag(jvv) v + G_y p + c_T M T
 *     rc  = c_div (G_x u + G_y v)
 * Rows in the Dirichlet set (dir_mask, or dir_sides when dir_mask is NULL): ru = u - dval_u,
 * rv = v - dval_v, rc = (K p).  Row `pin` (-1: none): rc = p - pin_val, written before the Dirichlet
 * rows when pin_first (the residual's statement order, :116-120) and after them otherwise (:159-160).
 * u, v, p, T, cu, cv, j**, dval_* are nullable (NULL = zeros; cu, cv: ones); a NULL output is not
 * computed.  u, v, ru, rv hold node (gx, gy) at gx * uv_pitch + gy (0 = NY: plain vectors; 2 NY: the
 * line-interleaved [u | v] layout of the velocity solve).  `pin` is a global node index.  On an
 * element-column strip handle (ABI 5) every vector holds the strip's lines; the two interface lines
 * get partial sums over the strip's elements, and pointwise terms, Dirichlet rows and the pinned row of
 * the right interface line are written by its right-hand owner only (0 here), so summing the interface
 * lines across strips (sem_interface_pack/unpack + an all-reduce) gives the whole-mesh rows. */
typedef struct sem_ns_desc {
  double c_mass, c_stiff, c_gradx, c_grady;
  const double* cu;
  const double* cv;
  const double* juu;
  const double* juv;
  const double* jvu;
  const double* jvv;
  double c_T;
  const double* T;
  double c_div;
  const double* dval_u;
  const double* dval_v;
  const uint8_t* dir_mask;
  unsigned dir_sides;
  int pin_first;
  int64_t pin;
  double pin_val;
  int64_t uv_pitch;
} sem_ns_desc;
int sem_ns_apply(sem_handle* h, const sem_ns_desc* d, const double* u, const double* v, const double* p, double* ru,
                 double* rv, double* rc, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SEM_OPS_H */
