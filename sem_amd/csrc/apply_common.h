// Shared device-side definitions of the apply kernels (sem_ops.hip, apply_band.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "gll_consts.h"
#include "sem_internal.h"

namespace sem {

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
  int tiles_x, tiles_y, dir_mode;
  unsigned sides;
  int has_e1, has_e2;
  int n_local32;  // local vector length (MFMA path: < 2^31)
  int pos0, pos1; // element-position range (band kernel; pos1 == 0: all positions)
  int diag;       // ablation bits for performance diagnosis (SEM_DIAG env); 0 in production
  unsigned long long* stamps;  // SEM_DIAG bit 8: per-wave s_memtime phase stamps (diagnostic builds only)
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

// One element's K_s / G_s contraction for output row `row` from a (2P+1)-window t
// (t[P..2P] = this element's nodes, t[0..P] = the left neighbour's, used at row 0).
// The K_s / G_s coefficients are compile-time constants (gll_consts.h, generated from the same
// host code that builds each handle's tables).  They are read through template indices into
// constexpr locals, so every coefficient is folded into the instruction stream: the
// contraction issues no table loads (a constexpr *array* indexed in a loop is emitted as a
// global and re-fetched with serialised scalar loads).
template <int P, int I>
__device__ __forceinline__ constexpr double kc() {
  constexpr double v = GllConst<P>::K[I];
  return v;
}
template <int P, int I>
__device__ __forceinline__ constexpr double gc() {
  constexpr double v = GllConst<P>::G[I];
  return v;
}

template <int P, int ROW, int... L>
__device__ __forceinline__ void row_dot(const double* t, double& k, double& g, std::integer_sequence<int, L...>) {
  ((k = fma(kc<P, ROW * (P + 1) + L>(), t[L], k), g = fma(gc<P, ROW * (P + 1) + L>(), t[L], g)), ...);
}

// One element's K_s / G_s contraction for output row ROW from a (2P+1)-window t
// (t[P..2P] = this element's nodes, t[0..P] = the left neighbour's, used at row 0).
template <int P, int ROW>
__device__ __forceinline__ void contract_row(const double (&t)[2 * P + 1], bool hasL, double& k, double& g) {
  using Seq = std::make_integer_sequence<int, P + 1>;
  k = 0.0;
  g = 0.0;
  if (ROW == 0 && hasL) row_dot<P, P>(t, k, g, Seq{});
  row_dot<P, ROW>(t + P, k, g, Seq{});
}

// Compile-time loop over output rows 0..P: f(std::integral_constant<int, ROW>).
template <int... R, class F>
__device__ __forceinline__ void for_rows(std::integer_sequence<int, R...>, F&& f) {
  (f(std::integral_constant<int, R>{}), ...);
}

// Diagnostic phase stamp (SEM_DIAG bit 8): lane 0 of each wave records s_memtime.
#define SEM_STAMP(k)                                                                      \
  do {                                                                                    \
    if (kDiag && a.stamps) {                                                              \
      unsigned long long t_;                                                              \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if ((threadIdx.x & 63) == 0) a.stamps[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (k)] = t_; \
    }                                                                                     \
  } while (0)

// Diagnostic slot 7: the XCD and hardware id this wave runs on (stamps are per-XCD clocks).
#define SEM_STAMP_HWID()                                                                                     \
  do {                                                                                                       \
    if (kDiag && a.stamps && (threadIdx.x & 63) == 0) {                                                      \
      unsigned xcc_, hw_;                                                                                    \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_HW_ID)"           \
                   : "=s"(xcc_), "=s"(hw_));                                                                 \
      a.stamps[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + 7] =                              \
          (static_cast<unsigned long long>(hw_) << 8) | (xcc_ & 0xf);                                        \
    }                                                                                                        \
  } while (0)

// Sum of GLL weights of the elements in [e_lo, e_hi) that hold 1-D node g (32-bit, P compile-time).
template <int P>
__device__ __forceinline__ double wsum(int g, int e_lo, int e_hi, const double* w) {
  const int e = g / P, i = g - e * P;
  const double wi = w[i], wP = w[P], w0 = w[0];  // unconditional reads: no per-lane branch
  return i != 0 ? wi : (e - 1 >= e_lo && e - 1 < e_hi ? wP : 0.0) + (e >= e_lo && e < e_hi ? w0 : 0.0);
}

// Generic (VALU) contraction along one staged direction for nodes the MFMA blocks do not
// cover (the domain's closing line / column): `base` points at the element's node 0 in the
// staged tile, `stride` is the distance between consecutive nodes of the direction.
template <int P>
__device__ __forceinline__ void contract_generic(const double* Kt, const double* Gt, const double* base, int stride,
                                                 int row, bool hasR, bool hasL, double& k, double& g) {
  constexpr int n = P + 1;
  k = 0.0;
  g = 0.0;
  if (row == 0 && hasL) {
    for (int l = 0; l <= P; ++l) {
      const double t = base[(l - P) * stride];
      k = fma(Kt[P * n + l], t, k);
      g = fma(Gt[P * n + l], t, g);
    }
  }
  if (hasR) {
    for (int l = 0; l <= P; ++l) {
      const double t = base[l * stride];
      k = fma(Kt[row * n + l], t, k);
      g = fma(Gt[row * n + l], t, g);
    }
  }
}

// The same with the staged nodes read through get(l), l = -P..P relative to the element's node 0 (a
// swizzled LDS tile, apply_tp_mfma).
template <int P, typename Get>
__device__ __forceinline__ void contract_generic_f(const double* Kt, const double* Gt, Get get, int row, bool hasR,
                                                   bool hasL, double& k, double& g) {
  constexpr int n = P + 1;
  k = 0.0;
  g = 0.0;
  if (row == 0 && hasL) {
    for (int l = 0; l <= P; ++l) {
      const double t = get(l - P);
      k = fma(Kt[P * n + l], t, k);
      g = fma(Gt[P * n + l], t, g);
    }
  }
  if (hasR) {
    for (int l = 0; l <= P; ++l) {
      const double t = get(l);
      k = fma(Kt[row * n + l], t, k);
      g = fma(Gt[row * n + l], t, g);
    }
  }
}

// Buffer resource over `bytes` bytes at p (wave-uniform inputs only).  Loads at offsets outside
// [0, bytes) -- including "negative" offsets, which wrap to huge unsigned values -- return 0
// without touching memory, so halo staging needs no clamps.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ double bload(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v),
                                        r, off, 0, 0);
}
// Store / load with a compile-time cache policy (gfx950 CPol bits: 1 = sc0, 2 = nt, 16 = sc1).
template <int CPOL>
__device__ __forceinline__ void bstore_c(__amdgpu_buffer_rsrc_t r, int off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), v),
                                        r, off, 0, CPOL);
}
template <int CPOL>
__device__ __forceinline__ double bload_c(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, CPOL));
}


}  // namespace sem
