// pipe_bench.hip — is the count kernel's access-mix ceiling (gather_bench k_mixed:
// 33.5 G/s against 49 G/s for bare random reads) a bandwidth limit of the mix, or the
// latency of the chain stream read -> random read inside each lane?
//   mixed      per item: a 32-B stream read, a random 16-B read whose address depends
//              on it, an 8-B write (gather_bench's k_mixed)
//   indep+io   the same traffic, the random address independent of the stream read
//   pipe       as mixed, the next item's stream read issued before this item's random
//              read is waited on (one item of look-ahead per lane)
//   pipe2      as pipe with two items per lane per iteration
//
//   hipcc -O3 --offload-arch=gfx950 pipe_bench.hip -o pipe_bench
//   ./pipe_bench [table_GB=17] [reads_M=256]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

__device__ __forceinline__ uint64_t gran(uint64_t r, uint4 a, uint4 b, uint64_t ng) {
  return mix(r * 0x9E3779B97F4A7C15ull + 17 + (a.x & b.w & 1)) % ng;
}

__global__ void k_mixed(const uint4* __restrict__ tab, uint64_t ng, uint64_t reads,
                        const uint4* __restrict__ s, uint64_t* __restrict__ out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r = t; r < reads; r += nt) {
    const uint4 a = s[2 * r], b = s[2 * r + 1];
    const uint4 v = tab[gran(r, a, b, ng)];
    out[r] = v.x ^ v.y ^ v.z ^ v.w;
  }
}

__global__ void k_indep_io(const uint4* __restrict__ tab, uint64_t ng, uint64_t reads,
                           const uint4* __restrict__ s, uint64_t* __restrict__ out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r = t; r < reads; r += nt) {
    const uint4 v = tab[gran(r, make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), ng)];
    const uint4 a = s[2 * r], b = s[2 * r + 1];
    out[r] = v.x ^ v.y ^ v.z ^ v.w ^ a.y ^ b.z;
  }
}

__global__ void k_pipe(const uint4* __restrict__ tab, uint64_t ng, uint64_t reads,
                       const uint4* __restrict__ s, uint64_t* __restrict__ out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint64_t r = t;
  if (r >= reads) return;
  uint4 a = s[2 * r], b = s[2 * r + 1];
  for (; r < reads; r += nt) {
    const uint4* p = tab + gran(r, a, b, ng);
    const uint4 v = *p;
    const uint64_t rn = r + nt;
    if (rn < reads) {
      a = s[2 * rn];
      b = s[2 * rn + 1];
    }
    out[r] = v.x ^ v.y ^ v.z ^ v.w;
  }
}

__global__ void k_pipe2(const uint4* __restrict__ tab, uint64_t ng, uint64_t reads,
                        const uint4* __restrict__ s, uint64_t* __restrict__ out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint64_t r = t;  // items r and r + nt per iteration
  uint4 a0 = make_uint4(0, 0, 0, 0), b0 = a0, a1 = a0, b1 = a0;
  if (r < reads) { a0 = s[2 * r]; b0 = s[2 * r + 1]; }
  if (r + nt < reads) { a1 = s[2 * (r + nt)]; b1 = s[2 * (r + nt) + 1]; }
  for (; r < reads; r += 2 * nt) {
    const uint64_t r1 = r + nt;
    const uint4 v0 = tab[gran(r, a0, b0, ng)];
    uint4 v1 = make_uint4(0, 0, 0, 0);
    if (r1 < reads) v1 = tab[gran(r1, a1, b1, ng)];
    const uint64_t n0 = r + 2 * nt, n1 = r1 + 2 * nt;
    if (n0 < reads) { a0 = s[2 * n0]; b0 = s[2 * n0 + 1]; }
    if (n1 < reads) { a1 = s[2 * n1]; b1 = s[2 * n1 + 1]; }
    out[r] = v0.x ^ v0.y ^ v0.z ^ v0.w;
    if (r1 < reads) out[r1] = v1.x ^ v1.y ^ v1.z ^ v1.w;
  }
}

// one item per thread, no loop (the count kernel's launch shape: a lane per pattern)
__global__ void k_mixed_flat(const uint4* __restrict__ tab, uint64_t ng, uint64_t reads,
                             const uint4* __restrict__ s, uint64_t* __restrict__ out) {
  const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (r >= reads) return;
  const uint4 a = s[2 * r], b = s[2 * r + 1];
  const uint4 v = tab[gran(r, a, b, ng)];
  out[r] = v.x ^ v.y ^ v.z ^ v.w;
}

__global__ void k_fill(uint64_t* p, uint64_t n) {
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += nt) p[i] = mix(i);
}

typedef void (*Kern)(const uint4*, uint64_t, uint64_t, const uint4*, uint64_t*);

static void timeit(const char* name, Kern k, unsigned grid, const uint4* tab, uint64_t ng,
                   uint64_t reads, const uint4* s, uint64_t* out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k<<<grid, 256>>>(tab, ng, reads / 4, s, out);
  CK(hipEventRecord(a));
  k<<<grid, 256>>>(tab, ng, reads, s, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("%-10s grid=%7u: %8.3f ms  %7.2f Gitems/s\n", name, grid, ms, reads / ms / 1e6);
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 17.0;
  const uint64_t reads = (uint64_t)((argc > 2 ? std::atof(argv[2]) : 256.0) * 1e6);
  const uint64_t bytes = (uint64_t)(gb * 1e9) & ~(uint64_t)127;
  uint4 *tab, *s;
  uint64_t* out;
  CK(hipMalloc(&tab, bytes));
  CK(hipMalloc(&s, reads * 32));
  CK(hipMalloc(&out, reads * 8));
  k_fill<<<8192, 256>>>(reinterpret_cast<uint64_t*>(tab), bytes / 8);
  k_fill<<<8192, 256>>>(reinterpret_cast<uint64_t*>(s), reads * 4);
  CK(hipDeviceSynchronize());
  const uint64_t ng = bytes / 16;
  std::printf("table %.2f GB, %llu items per run\n", bytes / 1e9, (unsigned long long)reads);
  for (unsigned grid : {8192u, 32768u}) {
    timeit("mixed", k_mixed, grid, tab, ng, reads, s, out);
    timeit("indep+io", k_indep_io, grid, tab, ng, reads, s, out);
    timeit("pipe", k_pipe, grid, tab, ng, reads, s, out);
    timeit("pipe2", k_pipe2, grid, tab, ng, reads, s, out);
  }
  timeit("flat", k_mixed_flat, (unsigned)((reads + 255) / 256), tab, ng, reads, s, out);
  CK(hipFree(tab));
  CK(hipFree(s));
  CK(hipFree(out));
  return 0;
}
