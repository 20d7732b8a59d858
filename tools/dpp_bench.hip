// Micro-benchmark: fp64 FMA chains with 64-bit coefficient immediates (materialised in SGPRs by
// s_mov_b32 pairs) vs the same coefficients held 16 per VGPR and broadcast with DPP row_newbcast
// (v_fmac_f64_dpp).  Also checks the DPP results bit for bit.  Build:
//   hipcc -O3 --offload-arch=gfx950 -o tools/dpp_bench tools/dpp_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

constexpr int NC = 64;
__host__ __device__ constexpr double coef(int k) { return 1.0 / (k + 3.0) + k * 1e-3; }

template <int L>
__device__ __forceinline__ double fma_bc(double cvec, double x, double acc) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(cvec), "v"(x), "n"(L));
  return acc;
}

template <int... K, class F>
__device__ __forceinline__ void unroll(std::integer_sequence<int, K...>, F&& f) {
  (f(std::integral_constant<int, K>{}), ...);
}

__global__ __launch_bounds__(256) void k_imm(const double* x, double* y, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  double xv[8];
  for (int i = 0; i < 8; ++i) xv[i] = x[(t + i) & 4095];
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  for (int it = 0; it < iters; ++it) {
    unroll(std::make_integer_sequence<int, NC / 4>{}, [&](auto KI) {
      constexpr int k = decltype(KI)::value * 4;
      a0 = fma(coef(k), xv[k % 8], a0);
      a1 = fma(coef(k + 1), xv[(k + 1) % 8], a1);
      a2 = fma(coef(k + 2), xv[(k + 2) % 8], a2);
      a3 = fma(coef(k + 3), xv[(k + 3) % 8], a3);
    });
    xv[it & 7] += a0 * 1e-9;
  }
  y[t] = a0 + a1 + a2 + a3;
}

__global__ __launch_bounds__(256) void k_dpp(const double* x, const double* ctab, double* y, int iters) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int ln = threadIdx.x & 15;
  double c[NC / 16];
  for (int j = 0; j < NC / 16; ++j) c[j] = ctab[j * 16 + ln];
  double xv[8];
  for (int i = 0; i < 8; ++i) xv[i] = x[(t + i) & 4095];
  double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  for (int it = 0; it < iters; ++it) {
    unroll(std::make_integer_sequence<int, NC / 4>{}, [&](auto KI) {
      constexpr int k = decltype(KI)::value * 4;
      a0 = fma_bc<k % 16>(c[k / 16], xv[k % 8], a0);
      a1 = fma_bc<(k + 1) % 16>(c[(k + 1) / 16], xv[(k + 1) % 8], a1);
      a2 = fma_bc<(k + 2) % 16>(c[(k + 2) / 16], xv[(k + 2) % 8], a2);
      a3 = fma_bc<(k + 3) % 16>(c[(k + 3) / 16], xv[(k + 3) % 8], a3);
    });
    xv[it & 7] += a0 * 1e-9;
  }
  y[t] = a0 + a1 + a2 + a3;
}

int main(int argc, char** argv) {
  const int nblk = argc > 1 ? atoi(argv[1]) : 585, iters = argc > 2 ? atoi(argv[2]) : 4;
  const int n = nblk * 256;
  std::vector<double> hx(4096), hc(NC);
  for (int i = 0; i < 4096; ++i) hx[i] = 0.5 + (i % 97) * 0.01;
  for (int k = 0; k < NC; ++k) hc[k] = coef(k);
  double *x, *c, *y1, *y2;
  hipMalloc(&x, 4096 * 8);
  hipMalloc(&c, NC * 8);
  hipMalloc(&y1, n * 8);
  hipMalloc(&y2, n * 8);
  hipMemcpy(x, hx.data(), 4096 * 8, hipMemcpyHostToDevice);
  hipMemcpy(c, hc.data(), NC * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int pass = 0; pass < 2; ++pass) {
    for (int v = 0; v < 2; ++v) {
      for (int w = 0; w < 20; ++w) {
        if (v == 0) k_imm<<<nblk, 256>>>(x, y1, iters);
        else k_dpp<<<nblk, 256>>>(x, c, y2, iters);
      }
      hipEventRecord(e0);
      const int R = 200;
      for (int r = 0; r < R; ++r) {
        if (v == 0) k_imm<<<nblk, 256>>>(x, y1, iters);
        else k_dpp<<<nblk, 256>>>(x, c, y2, iters);
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (pass) printf("%s nblk=%d iters=%d: %.3f us/launch\n", v ? "dpp" : "imm", nblk, iters, ms * 1e3 / R);
    }
  }
  std::vector<double> h1(n), h2(n);
  hipMemcpy(h1.data(), y1, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(h2.data(), y2, n * 8, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) bad += h1[i] != h2[i];
  printf("mismatches: %d of %d\n", bad, n);
  return bad != 0;
}
