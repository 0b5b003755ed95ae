// sorted_gather_bench.hip — does address order among concurrently issued random
// line reads change the rate?  12.5 M 32-B reads (one C4 count step: one line per
// pattern) from a 2 GB table of lines (C4's occurrence lines), issued
//   random : lane t reads line idx[t], idx uniform random
//   sorted : the same indices sorted ascending across lanes
// plus the cost of one stable 4-way partition pass over 12.5 M 16-B query records
// (the per-step reorder a sorted engine would pay), as a streaming read+write.
//
//   hipcc -O3 --offload-arch=gfx950 sorted_gather_bench.hip -o sorted_gather_bench
//   ./sorted_gather_bench [table_GB=2] [reads_M=12.5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__global__ void k_read(const uint4* __restrict__ tab, const uint32_t* __restrict__ idx, uint64_t nr,
                       uint32_t* __restrict__ out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= nr) return;
  const uint4* p = tab + (uint64_t)idx[t] * 2;
  const uint4 a = p[0], b = p[1];
  out[t] = a.x ^ a.y ^ b.z ^ b.w;
}

__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t < n) out[t] = in[t];
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += nt)
    p[i] = i * 0x9E3779B97F4A7C15ull;
}

static float time_read(const uint4* tab, const uint32_t* idx, uint64_t nr, uint32_t* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned grid = (unsigned)((nr + 255) / 256);
  k_read<<<grid, 256>>>(tab, idx, nr, out);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(a));
    k_read<<<grid, 256>>>(tab, idx, nr, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
  }
  return best;
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 2.0;
  const uint64_t nr = (uint64_t)((argc > 2 ? std::atof(argv[2]) : 12.5) * 1e6);
  const uint64_t bytes = (uint64_t)(gb * 1e9) & ~(uint64_t)31;
  const uint64_t nlines = bytes / 32;
  uint4* tab;
  CK(hipMalloc(&tab, bytes));
  k_fill<<<8192, 256>>>(reinterpret_cast<uint64_t*>(tab), bytes / 8);
  std::vector<uint32_t> h(nr);
  std::mt19937_64 rng(7);
  for (auto& x : h) x = (uint32_t)(rng() % nlines);
  uint32_t *d_idx, *d_out;
  CK(hipMalloc(&d_idx, nr * 4));
  CK(hipMalloc(&d_out, nr * 4));
  CK(hipMemcpy(d_idx, h.data(), nr * 4, hipMemcpyHostToDevice));
  const float ms_rand = time_read(tab, d_idx, nr, d_out);
  std::sort(h.begin(), h.end());
  CK(hipMemcpy(d_idx, h.data(), nr * 4, hipMemcpyHostToDevice));
  const float ms_sort = time_read(tab, d_idx, nr, d_out);
  std::printf("table %.2f GB (%llu lines), %llu reads\n", bytes / 1e9, (unsigned long long)nlines,
              (unsigned long long)nr);
  std::printf("random : %8.3f ms  %7.2f Greads/s\n", ms_rand, nr / ms_rand / 1e6);
  std::printf("sorted : %8.3f ms  %7.2f Greads/s\n", ms_sort, nr / ms_sort / 1e6);
  for (int shift : {4, 8, 12}) {  // sort by the top bits only: coarse buckets
    std::vector<uint32_t> g(nr);
    for (uint64_t i = 0; i < nr; ++i) g[i] = (uint32_t)(rng() % nlines);
    const uint32_t top = 32 - __builtin_clz((uint32_t)nlines);
    const uint32_t drop = top > (uint32_t)shift ? top - shift : 0;
    std::stable_sort(g.begin(), g.end(), [&](uint32_t x, uint32_t y) { return (x >> drop) < (y >> drop); });
    CK(hipMemcpy(d_idx, g.data(), nr * 4, hipMemcpyHostToDevice));
    const float ms = time_read(tab, d_idx, nr, d_out);
    std::printf("bucketed by top %2d bits (%6u buckets): %8.3f ms  %7.2f Greads/s\n", shift, 1u << shift,
                ms, nr / ms / 1e6);
  }
  {
    uint4 *a, *b;
    CK(hipMalloc(&a, nr * 16));
    CK(hipMalloc(&b, nr * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned grid = (unsigned)((nr + 255) / 256);
    k_copy<<<grid, 256>>>(a, b, nr);
    CK(hipEventRecord(e0));
    k_copy<<<grid, 256>>>(a, b, nr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("copy 16-B records: %8.3f ms  (%.0f GB/s r+w)\n", ms, 2.0 * nr * 16 / ms / 1e6);
  }
  return 0;
}
