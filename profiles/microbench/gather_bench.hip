// gather_bench.hip — the practical roofline for the count kernel's access
// pattern: random, independent W-byte reads (W = 16, 32, 64, 128) from a table far
// beyond the 256 MB Infinity Cache, and dependent chains of such reads.  Also the
// FETCH_SIZE calibration workload for this access width (MI355X_MICROARCH.md §HBM:
// "Other access widths are uncalibrated: calibrate on a known byte count").
//
//   hipcc -O3 --offload-arch=gfx950 gather_bench.hip -o gather_bench
//   ./gather_bench [table_GB=4] [reads_M=256] [contiguous=0] [mixed=0]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// independent reads: thread t reads `per` random W-byte granules
template <int W>
__global__ void k_indep(const uint4* __restrict__ tab, uint64_t ngran, uint64_t reads,
                        uint32_t* __restrict__ sink) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t r = t; r < reads; r += nt) {
    const uint64_t g = mix(r * 0x9E3779B97F4A7C15ull + 17) % ngran;
    const uint4* p = tab + g * (W / 16);
#pragma unroll
    for (int k = 0; k < W / 16; ++k) {
      const uint4 v = p[k];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) sink[t & 1023] = acc;
}

// independent 32-B reads with the non-temporal hint (no L2/MALL allocation)
__global__ void k_indep_nt(const uint4* __restrict__ tab, uint64_t ngran, uint64_t reads,
                           uint32_t* __restrict__ sink) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t r = t; r < reads; r += nt) {
    const uint64_t g = mix(r * 0x9E3779B97F4A7C15ull + 17) % ngran;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* p = reinterpret_cast<const u32x4*>(tab + g * 2);
    const u32x4 v0 = __builtin_nontemporal_load(p);
    const u32x4 v1 = __builtin_nontemporal_load(p + 1);
    acc ^= v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
  }
  if (acc == 0x12345678u) sink[t & 1023] = acc;
}

// independent 8-B reads
__global__ void k_indep8(const uint2* __restrict__ tab, uint64_t ngran, uint64_t reads,
                         uint32_t* __restrict__ sink) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t r = t; r < reads; r += nt) {
    const uint2 v = tab[mix(r * 0x9E3779B97F4A7C15ull + 17) % ngran];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x12345678u) sink[t & 1023] = acc;
}

// the count kernel's memory mix: per query a random W-byte read plus a coalesced
// stream (32 B read: pattern + offset; 8 B written: the count) — does the stream slow
// the random reads down?
template <int W>
__global__ void k_mixed(const uint4* __restrict__ tab, uint64_t ngran, uint64_t reads,
                        const uint4* __restrict__ stream, uint64_t* __restrict__ out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r = t; r < reads; r += nt) {
    const uint4 a = stream[2 * r], b = stream[2 * r + 1];
    const uint64_t g = mix(r * 0x9E3779B97F4A7C15ull + 17 + (a.x & b.w & 1)) % ngran;
    const uint4* p = tab + g * (W / 16);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < W / 16; ++k) {
      const uint4 v = p[k];
      x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[r] = x;
  }
}

// dependent chains: each lane does `depth` reads, next address from the data
template <int W>
__global__ void k_chain(const uint4* __restrict__ tab, uint64_t ngran, uint64_t lanes, int depth,
                        uint32_t* __restrict__ sink) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= lanes) return;
  uint64_t g = mix(t + 99) % ngran;
  uint32_t acc = 0;
  for (int d = 0; d < depth; ++d) {
    const uint4* p = tab + g * (W / 16);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < W / 16; ++k) {
      const uint4 v = p[k];
      x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    acc += x;
    g = mix(g + x + d) % ngran;
  }
  if (acc == 0x12345678u) sink[t & 1023] = acc;
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += nt) p[i] = mix(i);
}

template <int W>
void run(const uint4* tab, uint64_t bytes, uint64_t reads, uint32_t* sink) {
  const uint64_t ng = bytes / W;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int grid : {2048, 8192, 32768}) {
    k_indep<W><<<grid, 256>>>(tab, ng, reads / 4, sink);
    CK(hipEventRecord(a));
    k_indep<W><<<grid, 256>>>(tab, ng, reads, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("indep W=%3d grid=%6d: %8.3f ms  %7.2f Greads/s  %7.1f GB/s (useful)\n", W, grid, ms,
                reads / ms / 1e6, reads * (double)W / ms / 1e6);
  }
  for (uint64_t lanes : {262144ull, 1048576ull, 4194304ull}) {
    const int depth = 64;
    k_chain<W><<<(lanes + 255) / 256, 256>>>(tab, ng, lanes, depth / 4, sink);
    CK(hipEventRecord(a));
    k_chain<W><<<(lanes + 255) / 256, 256>>>(tab, ng, lanes, depth, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double r = (double)lanes * depth;
    std::printf("chain W=%3d lanes=%8llu depth=%d: %8.3f ms  %7.2f Greads/s  %7.1f GB/s  lat/read %.0f ns\n",
                W, (unsigned long long)lanes, depth, ms, r / ms / 1e6, r * W / ms / 1e6,
                ms * 1e6 / depth);
  }
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 4.0;
  const uint64_t reads = (uint64_t)((argc > 2 ? std::atof(argv[2]) : 256.0) * 1e6);
  const uint64_t bytes = (uint64_t)(gb * 1e9) & ~(uint64_t)127;
  const int contiguous = argc > 3 ? std::atoi(argv[3]) : 0;  // hipDeviceMallocContiguous
  uint4* tab;
  uint32_t* sink;
  if (contiguous)
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&tab), bytes, hipDeviceMallocContiguous));
  else
    CK(hipMalloc(&tab, bytes));
  std::printf("allocation: %s\n", contiguous ? "hipDeviceMallocContiguous" : "hipMalloc");
  CK(hipMalloc(&sink, 4096));
  k_fill<<<8192, 256>>>(reinterpret_cast<uint64_t*>(tab), bytes / 8);
  CK(hipDeviceSynchronize());
  std::printf("table %.2f GB, %llu reads per run\n", bytes / 1e9, (unsigned long long)reads);
  {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int grid : {8192, 32768}) {
      float ms = 0;
      k_indep_nt<<<grid, 256>>>(tab, bytes / 32, reads / 4, sink);
      CK(hipEventRecord(a));
      k_indep_nt<<<grid, 256>>>(tab, bytes / 32, reads, sink);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("indep-nt W= 32 grid=%6d: %8.3f ms  %7.2f Greads/s\n", grid, ms, reads / ms / 1e6);
      k_indep8<<<grid, 256>>>(reinterpret_cast<const uint2*>(tab), bytes / 8, reads / 4, sink);
      CK(hipEventRecord(a));
      k_indep8<<<grid, 256>>>(reinterpret_cast<const uint2*>(tab), bytes / 8, reads, sink);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("indep    W=  8 grid=%6d: %8.3f ms  %7.2f Greads/s\n", grid, ms, reads / ms / 1e6);
    }
  }
  if (argc > 4 && std::atoi(argv[4]) == 1) {  // the count kernel's mix (k_mixed)
    uint4* stream;
    uint64_t* out;
    CK(hipMalloc(&stream, reads * 32));
    CK(hipMalloc(&out, reads * 8));
    CK(hipMemset(stream, 0x5A, reads * 32));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int grid : {8192, 32768, 131072}) {
      float ms = 0;
      k_mixed<16><<<grid, 256>>>(tab, bytes / 16, reads / 4, stream, out);
      CK(hipEventRecord(a));
      k_mixed<16><<<grid, 256>>>(tab, bytes / 16, reads, stream, out);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("mixed W= 16 + 32 B read + 8 B written per read, grid=%6d: %8.3f ms  %7.2f Greads/s\n",
                  grid, ms, reads / ms / 1e6);
      k_indep<16><<<grid, 256>>>(tab, bytes / 16, reads / 4, sink);
      CK(hipEventRecord(a));
      k_indep<16><<<grid, 256>>>(tab, bytes / 16, reads, sink);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("indep W= 16 (same grid)                             grid=%6d: %8.3f ms  %7.2f Greads/s\n",
                  grid, ms, reads / ms / 1e6);
    }
    CK(hipFree(stream));
    CK(hipFree(out));
    CK(hipFree(tab));
    return 0;
  }
  run<16>(tab, bytes, reads, sink);
  run<32>(tab, bytes, reads, sink);
  run<64>(tab, bytes, reads, sink);
  run<128>(tab, bytes, reads, sink);
  CK(hipFree(tab));
  return 0;
}
