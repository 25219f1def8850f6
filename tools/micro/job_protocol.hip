// Standalone check (tooling) of the leader/helper job hand-off used by plan_kernel: agent-scope payload
// stores + flag, CAS tile claims tagged with the job number, done counter, stop flag.  Every loop is bounded.
// hipcc --offload-arch=gfx950 -O3 job_protocol.hip -o job_protocol && ./job_protocol
#include <hip/hip_runtime.h>
#include <cstdio>

struct Board {
  int seq, stop, pad0[30];
  unsigned long long claim;
  int pad1[30];
  int done, pad2[31];
  int first[32];
  int ntiles, pad3[31];
  int payload[1024];
};

__device__ __forceinline__ void st_agent(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int ld_agent(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ int claim(Board* b, int seq, int ntiles, int* fails) {
  unsigned long long v = ld_agent(&b->claim);
  for (int a = 0; a < 100000; ++a) {
    if ((int)(v >> 32) != seq || (int)(v & 0xffffffffu) >= ntiles) return -1;
    unsigned long long e = v;
    if (__hip_atomic_compare_exchange_strong(&b->claim, &e, v + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return (int)(v & 0xffffffffu);
    v = e;
    atomicAdd(fails, 1);
  }
  return -2;
}

__shared__ int s_tile, s_go, s_seq, s_ntiles;
__shared__ int s_payload[1024];

__device__ void work(Board* b, int* stats) {
  for (;;) {
    if (threadIdx.x == 0) s_tile = claim(b, s_seq, s_ntiles, &stats[2]);
    __syncthreads();
    int t = s_tile;
    if (t < 0) { if (t == -2 && threadIdx.x == 0) atomicAdd(&stats[3], 1); break; }
    // dummy tile: 8 slots; slot value = payload; "collides" if payload % 7 == 3 -> atomicMin first[slot % 32]
    if (threadIdx.x < 8) {
      int sl = t * 8 + threadIdx.x;
      int v = s_payload[sl];
      if (v % 7 == 3) atomicMin(&b->first[sl % 32], sl);
    }
    drain();
    __syncthreads();
    if (threadIdx.x == 0) { atomicAdd(&b->done, 1); atomicAdd(&stats[4], 1); }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(512) k(Board* b, int njobs, int* stats, int* results) {
  if (blockIdx.x > 0) {  // helper
    int last = 0;
    unsigned long long t0 = wall_clock64();
    for (;;) {
      if (threadIdx.x == 0) {
        int go = -1;
        for (;;) {
          int s = ld_agent(&b->seq);
          if (s != last) { go = s; break; }
          if (ld_agent(&b->stop)) break;
          if (wall_clock64() - t0 > 200000000ull) break;
          __builtin_amdgcn_s_sleep(2);
        }
        s_go = go;
      }
      __syncthreads();
      int go = s_go;
      if (go < 0) break;
      last = go;
      int nt = ld_agent(&b->ntiles);
      for (int i = threadIdx.x; i < nt * 8 && i < 1024; i += blockDim.x) s_payload[i] = ld_agent(&b->payload[i]);
      if (threadIdx.x == 0) { s_seq = go; s_ntiles = nt; atomicAdd(&stats[1], 1); }
      __syncthreads();
      work(b, stats);
      t0 = wall_clock64();
    }
    return;
  }
  for (int j = 1; j <= njobs; ++j) {
    int nt = 1 + (j * 37) % 63;
    for (int i = threadIdx.x; i < nt * 8; i += blockDim.x) { s_payload[i] = i * 13 + j; st_agent(&b->payload[i], i * 13 + j); }
    if (threadIdx.x < 32) st_agent(&b->first[threadIdx.x], 1 << 30);
    if (threadIdx.x == 0) {
      st_agent(&b->ntiles, nt);
      st_agent(&b->done, 0);
      st_agent(&b->claim, (unsigned long long)j << 32);
      s_seq = j; s_ntiles = nt;
    }
    drain();
    __syncthreads();
    if (threadIdx.x == 0) { drain(); st_agent(&b->seq, j); atomicAdd(&stats[0], 1); }
    work(b, stats);
    if (threadIdx.x == 0) {
      unsigned long long t0 = wall_clock64();
      while (ld_agent(&b->done) < nt) {
        if (wall_clock64() - t0 > 200000000ull) { atomicAdd(&stats[5], 1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    // check: expected first[g] = min slot sl with sl % 32 == g and payload % 7 == 3
    if (threadIdx.x < 32) {
      int exp = 1 << 30;
      for (int sl = threadIdx.x; sl < nt * 8; sl += 32) if ((sl * 13 + j) % 7 == 3) { exp = sl; break; }
      if (ld_agent(&b->first[threadIdx.x]) != exp) atomicAdd(&results[0], 1);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) st_agent(&b->stop, 1);
}

int main() {
  Board* b; int* stats; int* res;
  (void)hipMalloc(&b, sizeof(Board)); (void)hipMalloc(&stats, 8 * sizeof(int)); (void)hipMalloc(&res, 4 * sizeof(int));
  for (int nh : {0, 1, 3, 63}) {
    (void)hipMemset(b, 0, sizeof(Board)); (void)hipMemset(stats, 0, 8 * sizeof(int)); (void)hipMemset(res, 0, 4 * sizeof(int));
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(1 + nh), dim3(512), 0, 0, b, 2000, stats, res);
    (void)hipEventRecord(e1);
    hipError_t err = hipDeviceSynchronize();
    float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
    int s[8], r[4];
    (void)hipMemcpy(s, stats, sizeof(s), hipMemcpyDeviceToHost); (void)hipMemcpy(r, res, sizeof(r), hipMemcpyDeviceToHost);
    printf("helpers %2d: %s  %.2f ms (%.2f us/job)  published %d joined %d casfail %d giveup %d tiles %d timeouts %d wrong %d\n",
           nh, hipGetErrorString(err), ms, ms * 1e3 / 2000, s[0], s[1], s[2], s[3], s[4], s[5], r[0]);
    if (err != hipSuccess) return 1;
  }
  return 0;
}
