// Microbenchmark (tooling, not product): cost of a non-inlined device call on gfx950 in a 512-thread workgroup
// when the callee keeps values live across a call of its own (so it saves callee-saved VGPRs to scratch on entry and
// reloads them on return), against the same body with the inner call inlined (no callee-saved registers), with and
// without an agent-scope acquire before each call (the planner's polling invalidates L1 that way).
//   hipcc --offload-arch=gfx950 -O3 call_overhead.hip -o /tmp/call_overhead && /tmp/call_overhead
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NV = 48;  // doubles live across the inner call: 96 VGPRs

__device__ __noinline__ void leaf_call(double* lds, int i) {
  lds[threadIdx.x] += (double)i;
  __syncthreads();
}
__device__ __forceinline__ void leaf_inl(double* lds, int i) {
  lds[threadIdx.x] += (double)i;
  __syncthreads();
}

template <bool INNER_CALL>
__device__ __noinline__ double body(double* lds, const double* __restrict__ g, int n, int it) {
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = g[(threadIdx.x * NV + k + it) % n];
  if (INNER_CALL) {
    leaf_call(lds, it);
    // clobbers 56 callee-saved VGPRs (v40-47, v56-63, ..., v136-143): the prologue / epilogue saves and reloads them,
    // as the planner's nearest / near_set / edge_validity do
    asm volatile("" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143");
  } else {
    leaf_inl(lds, it);
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < NV; ++k) s += v[k] * v[(k + 7) % NV];
  return s;
}

template <bool INNER_CALL>
__device__ __forceinline__ double body_inl(double* lds, const double* __restrict__ g, int n, int it) {
  double v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = g[(threadIdx.x * NV + k + it) % n];
  leaf_inl(lds, it);
  double s = 0;
#pragma unroll
  for (int k = 0; k < NV; ++k) s += v[k] * v[(k + 7) % NV];
  return s;
}

// MODE 0: body with an inner call (callee-saved spills), 1: body non-inlined but leaf inlined, 2: all inlined
template <int MODE, bool ACQ>
__global__ void __launch_bounds__(512) k(const double* g, int n, double* out, long long* cyc, int reps) {
  __shared__ double lds[512];
  lds[threadIdx.x] = 0;
  __syncthreads();
  double acc = 0;
  long long t0 = wall_clock64();
  for (int it = 0; it < reps; ++it) {
    if (ACQ) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (MODE == 0) acc += body<true>(lds, g, n, it);
    else if (MODE == 1) acc += body<false>(lds, g, n, it);
    else acc += body_inl<false>(lds, g, n, it);
  }
  __syncthreads();
  long long t1 = wall_clock64();
  out[blockIdx.x * 512 + threadIdx.x] = acc + lds[threadIdx.x];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, bool ACQ>
void run(const char* name, const double* g, int n, double* out, long long* cyc) {
  const int reps = 2000;
  hipLaunchKernelGGL((k<MODE, ACQ>), dim3(1), dim3(512), 0, 0, g, n, out, cyc, 10);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((k<MODE, ACQ>), dim3(1), dim3(512), 0, 0, g, n, out, cyc, reps);
  hipDeviceSynchronize();
  long long c = 0;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-34s acquire %d: %.3f us per call (wall clock 100 MHz)\n", name, (int)ACQ, c * 1e-2 / reps);
}

int main() {
  const int n = 1 << 16;
  double *g, *out;
  long long* cyc;
  hipMalloc(&g, n * sizeof(double));
  hipMemset(g, 0, n * sizeof(double));
  hipMalloc(&out, 512 * sizeof(double));
  hipMalloc(&cyc, sizeof(long long));
  run<0, false>("call, callee saves 56 VGPRs", g, n, out, cyc);
  run<0, true>("call, callee saves 56 VGPRs", g, n, out, cyc);
  run<1, false>("call, no inner call", g, n, out, cyc);
  run<1, true>("call, no inner call", g, n, out, cyc);
  run<2, false>("inlined", g, n, out, cyc);
  run<2, true>("inlined", g, n, out, cyc);
  return 0;
}
