// Workgroup-dispatch cost on MI355X: time per launch of a trivial kernel (one store per
// workgroup) for several grid sizes, workgroup sizes and LDS footprints, 100 launches per
// hipGraph.  Used to size the apply kernels' grids (tools/kbench.py).
//   hipcc -O3 --offload-arch=gfx950 -o tools/dispatch_bench tools/dispatch_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

template <int LDS>
__global__ void touch(double* out) {
  __shared__ double s[LDS > 0 ? LDS / 8 : 1];
  if (LDS > 0) s[threadIdx.x % (LDS > 0 ? LDS / 8 : 1)] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = LDS > 0 ? s[1] : 1.0;
}

template <int LDS>
static int run(double* out, int grid, int threads, hipStream_t st) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(touch<LDS>, dim3(grid), dim3(threads), 0, st, out);
  CHECK(hipStreamEndCapture(st, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CHECK(hipGraphLaunch(ge, st));
  CHECK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(a, st));
    CHECK(hipGraphLaunch(ge, st));
    CHECK(hipEventRecord(b, st));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  std::printf("grid %5d threads %4d lds %6d: %7.2f us/launch\n", grid, threads, LDS, best * 10.0f);
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return 0;
}

int main() {
  double* out;
  CHECK(hipMalloc(&out, 1 << 20));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  const int grids[] = {1, 256, 512, 1024, 2048, 4096};
  const int threads[] = {64, 256, 576, 1024};
  for (int t : threads)
    for (int g : grids) {
      if (run<0>(out, g, t, st)) return 1;
      if (run<32768>(out, g, t, st)) return 1;
    }
  return 0;
}
