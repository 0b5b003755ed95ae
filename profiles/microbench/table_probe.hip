// table_probe.hip — gather_bench's independent random 16-B reads (k_indep<16>) over a
// caller's device buffer, as a shared library, so that profiles/scripts/table_probe.py
// can time them over an index's own prefix table and over a fresh buffer in one process.
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC table_probe.hip -o libtable_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_probe16(const uint4* __restrict__ tab, uint64_t ngran, uint64_t reads,
                          uint32_t* __restrict__ sink) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t r = t; r < reads; r += nt) {
    const uint4 v = tab[mix(r * 0x9E3779B97F4A7C15ull + 17) % ngran];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[t & 1023] = acc;
}

// -> mean ms of `reps` launches of `reads` random 16-B reads over [tab, tab + bytes)
extern "C" float table_probe16(const void* tab, uint64_t bytes, uint64_t reads, int grid, int reps) {
  uint32_t* sink = nullptr;
  if (hipMalloc(&sink, 4096) != hipSuccess) return -1.f;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const uint64_t ng = bytes / 16;
  k_probe16<<<grid, 256>>>(static_cast<const uint4*>(tab), ng, reads / 4, sink);
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) k_probe16<<<grid, 256>>>(static_cast<const uint4*>(tab), ng, reads, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFree(sink);
  return ms / reps;
}

__global__ void k_iota(uint64_t* p, uint64_t n) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = i * 0x9E3779B97F4A7C15ull + 17;
}

// The count kernels' shape without their logic: one lane per U patterns, each lane reads
// its patterns' 8-B stream words (coalesced), hashes each to a random 16-B table entry,
// reads the U entries together and writes U 8-B results (coalesced).  grid_stride = 1:
// a fixed grid whose lanes loop over the batch instead of one-shot lanes.
template <int U>
__global__ void k_shape(const uint4* __restrict__ tab, uint64_t ngran, const uint64_t* __restrict__ in,
                        uint64_t npat, uint64_t* __restrict__ out, int grid_stride) {
  const uint64_t step = grid_stride ? (uint64_t)gridDim.x * blockDim.x * U : npat;
  for (uint64_t q0 = blockIdx.x * (uint64_t)(blockDim.x * U) + threadIdx.x; q0 < npat; q0 += step) {
    uint64_t a[U];
    uint4 v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t q = q0 + (uint64_t)j * blockDim.x;
      a[j] = q < npat ? mix(in[q]) % ngran : 0;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = tab[a[j]];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t q = q0 + (uint64_t)j * blockDim.x;
      if (q < npat) out[q] = v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    if (!grid_stride) break;
  }
}

// -> mean ms of `reps` launches of k_shape<u> over npat patterns (grid 0: one-shot lanes)
extern "C" float table_probe_shape(const void* tab, uint64_t bytes, uint64_t npat, int u, int grid,
                                   int reps) {
  uint64_t *in = nullptr, *out = nullptr;
  if (hipMalloc(&in, npat * 8) != hipSuccess || hipMalloc(&out, npat * 8) != hipSuccess) return -1.f;
  k_iota<<<(unsigned)((npat + 255) / 256), 256>>>(in, npat);
  const uint64_t ng = bytes / 16;
  const int gs = grid > 0;
  const unsigned g = gs ? (unsigned)grid : (unsigned)((npat + 256 * u - 1) / (256 * u));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&] {
    if (u == 1) k_shape<1><<<g, 256>>>(static_cast<const uint4*>(tab), ng, in, npat, out, gs);
    else if (u == 2) k_shape<2><<<g, 256>>>(static_cast<const uint4*>(tab), ng, in, npat, out, gs);
    else k_shape<4><<<g, 256>>>(static_cast<const uint4*>(tab), ng, in, npat, out, gs);
  };
  launch();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(in);
  (void)hipFree(out);
  return ms / reps;
}
