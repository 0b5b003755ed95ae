// alloc_gap: the GPU-side cost of a stream-ordered allocation per call (hipMallocAsync +
// hipFreeAsync around a call's kernels) on back-to-back calls of one stream.  A call = a
// ~400-us streaming kernel + a tiny tail kernel; variants: no allocation, a per-call
// hipMallocAsync/hipFreeAsync buffer, the same with a memset of the buffer, a buffer reused
// across calls.  Prints microseconds per call for each.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_stream(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = a[i];
    v.x += 1;
    b[i] = v;
  }
}
__global__ void k_tail(uint32_t* p, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n && p && p[i] == 0xFFFFFFFFu) p[i] = 0;
}

int main() {
  const size_t n = (size_t)1 << 23;  // 128 MB read + 128 MB write: ~40 us
  uint4 *a, *b;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMemset(a, 0, n * 16));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipMemPool_t pool;
  CK(hipDeviceGetDefaultMemPool(&pool, 0));
  uint64_t thr = ~0ull;
  CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
  const size_t lb = 50u << 20;
  void* keep;
  CK(hipMalloc(&keep, lb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"none", "malloc_async", "malloc_async+memset", "reused", "tail_only"};
  for (int round = 0; round < 3; ++round)
    for (int v = 0; v < 5; ++v) {
      const int K = 200;
      CK(hipEventRecord(e0, st));
      for (int k = 0; k < K; ++k) {
        void* p = nullptr;
        if (v == 1 || v == 2) CK(hipMallocAsync(&p, lb, st));
        if (v == 3) p = keep;
        if (v == 2) CK(hipMemsetAsync(p, 0, 400000, st));
        k_stream<<<8192, 256, 0, st>>>(a, b, n);
        if (v != 0) k_tail<<<2560, 256, 0, st>>>(static_cast<uint32_t*>(p), 655360);
        if (v == 1 || v == 2) CK(hipFreeAsync(p, st));
      }
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("round %d %-22s %8.2f us per call\n", round, names[v], ms * 1e3 / K);
    }
  return 0;
}
