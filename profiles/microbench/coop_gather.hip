// coop_gather.hip — random W-byte reads (W = 16, 32, 64) over a large table, each read
// either by ONE lane (W / 16 loads of 16 B: as gather_bench's `indep`) or by W / 16
// consecutive lanes cooperatively (one 16-B load each, the group's loads falling in one
// W-byte block: one coalesced request).  Question: does a 64-B record cost one random
// request when a quad of lanes reads it (so a record 4x wider is as cheap as a 16-B one)?
//
//   hipcc -O3 --offload-arch=gfx950 coop_gather.hip -o coop_gather
//   ./coop_gather [table_GB=17] [reads_M=256]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// one lane per read
template <int W>
__global__ void k_lane(const uint4* __restrict__ tab, uint64_t ngran, uint64_t reads, uint32_t* sink) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t r = t; r < reads; r += nt) {
    const uint4* p = tab + (mix(r * 0x9E3779B97F4A7C15ull + 17) % ngran) * (W / 16);
#pragma unroll
    for (int k = 0; k < W / 16; ++k) {
      const uint4 v = p[k];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) sink[t & 1023] = acc;
}

// W / 16 lanes per read, one 16-B chunk each
template <int W>
__global__ void k_coop(const uint4* __restrict__ tab, uint64_t ngran, uint64_t reads, uint32_t* sink) {
  constexpr int G = W / 16;
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t s = t; s < reads * G; s += nt) {
    const uint64_t r = s / G;
    const uint4 v = tab[(mix(r * 0x9E3779B97F4A7C15ull + 17) % ngran) * G + (s % G)];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[t & 1023] = acc;
}

template <class F>
static void timeit(const char* name, int W, uint64_t reads, F&& f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("%-5s W=%3d: %8.3f ms  %7.2f G reads/s\n", name, W, ms, reads / ms / 1e6);
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 17.0;
  const uint64_t reads = (uint64_t)((argc > 2 ? std::atof(argv[2]) : 256.0) * 1e6);
  const uint64_t bytes = (uint64_t)(gb * 1e9) & ~63ull;
  uint4* tab;
  uint32_t* sink;
  CK(hipMalloc(&tab, bytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(tab, 1, bytes));
  std::printf("table %.2f GB, %llu reads per run\n", bytes / 1e9, (unsigned long long)reads);
  const int grid = 8192;
  for (int round = 0; round < 2; ++round) {
    timeit("lane", 16, reads, [&] { k_lane<16><<<grid, 256>>>(tab, bytes / 16, reads, sink); });
    timeit("lane", 32, reads, [&] { k_lane<32><<<grid, 256>>>(tab, bytes / 32, reads, sink); });
    timeit("lane", 64, reads, [&] { k_lane<64><<<grid, 256>>>(tab, bytes / 64, reads, sink); });
    timeit("coop", 32, reads, [&] { k_coop<32><<<grid, 256>>>(tab, bytes / 32, reads, sink); });
    timeit("coop", 64, reads, [&] { k_coop<64><<<grid, 256>>>(tab, bytes / 64, reads, sink); });
  }
  return 0;
}
