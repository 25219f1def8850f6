// Microbenchmark (tooling, not product): cycles per fp64 (and fp32) instruction on gfx950, dependent chain vs 4/8
// independent chains, one wave and 2 waves per SIMD.  hipcc --offload-arch=gfx950 -O3 fp64_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T, int CH, int OP>
__global__ void k(T* out, long long* cyc, T a, T b, int n) {
  // cyc[0]: s_memtime ticks, cyc[1]: s_memrealtime ticks (100 MHz) over the same loop
  T x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = a + threadIdx.x + c;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; i += 32) {  // 32 steps per loop trip: the loop's branch is amortised
#pragma unroll
    for (int u = 0; u < 32; ++u)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (OP == 0) x[c] = x[c] * b;
      else if (OP == 1) x[c] = x[c] + b;
      else if (OP == 2) x[c] = __builtin_fma(x[c], b, a);
      else if (OP == 3) x[c] = floor(x[c]) + b;
      else if (OP == 4) x[c] = x[c] / b;
      else if (OP == 5) x[c] = sqrt(x[c]) + b;
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  T s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = r1 - r0; }
}

template <int CH, int OP, typename T = double>
void run(const char* name, int threads) {
  T* out; long long* cyc;
  hipMalloc(&out, 4096 * sizeof(T)); hipMalloc(&cyc, 64 * sizeof(long long));
  const int n = 4096;
  hipLaunchKernelGGL((k<T, CH, OP>), dim3(1), dim3(threads), 0, 0, out, cyc, (T)1.0000001, (T)0.9999999, n);
  hipDeviceSynchronize();
  long long cc[2] = {0, 0};
  hipMemcpy(cc, cyc, sizeof(cc), hipMemcpyDeviceToHost);
  const double c = (double)cc[0], ns = (double)cc[1] * 10.0;
  printf("%-3s %-8s chains %d threads %4d: %.2f s_memtime ticks per instruction per wave (per chain step %.2f; %.2f ns, "
         "s_memtime at %.0f MHz)\n", sizeof(T) == 8 ? "f64" : "f32", name, CH, threads, c / (n * CH), c / n, ns / n,
         c / ns * 1e3);
  hipFree(out); hipFree(cyc);
}

int main() {
  for (int th : {64, 512}) {
    run<1, 0>("mul", th); run<4, 0>("mul", th); run<8, 0>("mul", th);
    run<1, 1>("add", th); run<8, 1>("add", th);
    run<1, 2>("fma", th); run<8, 2>("fma", th);
    run<1, 3>("floor", th); run<8, 3>("floor", th);
    run<1, 4>("div", th); run<8, 4>("div", th);
    run<1, 5>("sqrt", th); run<8, 5>("sqrt", th);
    run<1, 0, float>("mul", th); run<8, 0, float>("mul", th);
    run<1, 1, float>("add", th); run<8, 1, float>("add", th);
    run<1, 2, float>("fma", th); run<8, 2, float>("fma", th);
    run<1, 4, float>("div", th); run<1, 5, float>("sqrt", th);
  }
  return 0;
}
