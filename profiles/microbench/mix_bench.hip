// mix_bench.hip — the ceiling of the C4 headline count's access mix (VERDICT r05 "next" 1).
//
// Per query the production count (k_count_ctx, routed, uint64 counts) reads its two offsets
// (8 B streamed: offs[q + 1] is the next query's offs[q]), its 20 pattern bytes (streamed),
// ONE random 16-B context record out of a 4^15 x 16 B = 17.2 GB table, and writes one 8-B
// count (streamed, non-temporal).  This program reproduces exactly that mix over
// synthetic DNA 20-mers (12.5 M by default) and times it in several kernel shapes, next to
// the two halves alone:
//
//   rand      the 12.5 M random 16-B record reads alone (indices from a hash; no stream)
//   stream    the stream alone (offsets + pattern bytes in, counts out; no record read)
//   oneshot   the production shape: grid = npat / (256 U), each lane U queries, stages
//             (offsets+pattern) -> U record reads -> counts; U = 1, 2, 4; waves/EU 6 or 8
//   persist   a grid of G blocks looping over the batch, software-pipelined: the next
//             iteration's offsets and pattern bytes are loaded while this iteration's
//             record reads are in flight; U = 1, 2, 4
//   split     two passes: pass 1 streams the patterns and writes each query's 4-B record
//             index, pass 2 reads the indices (4 B, coalesced) and gathers the records
//
// Reported per shape: the median of `reps` launches (HIP events around each launch) in ms,
// the queries/s and the random-read rate.
//
//   hipcc -O3 --offload-arch=gfx950 mix_bench.hip -o mix_bench
//   ./mix_bench [npat_M=12.5] [reps=21]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

constexpr int kK = 15;                 // table characters (C4: k = 15)
constexpr int kM = 20;                 // pattern length
constexpr uint64_t kRecs = 1ull << 30;  // 4^15 records of 16 B

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint4 ld_nt16(const uint4* p) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(r.x, r.y, r.z, r.w);
}

// the 20 pattern bytes at o (4-aligned here, as every offset of a 20-mer batch is): 5 dwords
__device__ __forceinline__ void load_pat(const uint8_t* pats, uint64_t o, uint32_t u[5]) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(pats + o);
#pragma unroll
  for (int i = 0; i < 5; ++i) u[i] = w[i];
}

// 2-bit code of an ACGT byte (A=0x41 C=0x43 G=0x47 T=0x54): ((b >> 1) ^ (b >> 2)) & 3
__device__ __forceinline__ uint32_t code(uint32_t b) { return ((b >> 1) ^ (b >> 2)) & 3u; }

// table index of the last 15 characters, context key of the first 5
__device__ __forceinline__ void key(const uint32_t u[5], uint32_t& t, uint32_t& want) {
  t = 0;
  want = 0;
#pragma unroll
  for (int i = 0; i < kM; ++i) {
    const uint32_t c = code((u[i >> 2] >> (8 * (i & 3))) & 0xFFu);
    if (i >= kM - kK) t = t * 4 + c;
    else want |= c << (2 * (kM - kK - 1 - i));
  }
}

// a count from a record: the rows whose 10-bit context equals `want` (shape of kRec16)
__device__ __forceinline__ uint64_t rec_count(uint4 a, uint32_t want) {
  const uint32_t wc = a.y & 15u;
  uint32_t n = 0;
  const uint32_t d[3] = {a.z, a.w, a.y >> 4};
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t e = (d[i / 3] >> (10 * (i % 3))) & 0x3FFu;
    n += (uint32_t)(i < (int)(wc % 10) && e == want);
  }
  return n;
}

// ---- the two halves alone ------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rand(const uint4* __restrict__ tab, uint64_t npat,
                                              uint64_t* __restrict__ sink) {
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < npat; q += nt) {
    const uint4 a = ld_nt16(tab + (mix(q * 0x9E3779B97F4A7C15ull + 7) & (kRecs - 1)));
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_stream(const uint8_t* __restrict__ pats,
                                                const uint64_t* __restrict__ offs, uint64_t npat,
                                                uint64_t* __restrict__ out) {
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < npat; q += nt) {
    const uint64_t o = offs[q], m = offs[q + 1] - o;
    uint32_t u[5];
    load_pat(pats, o, u);
    uint32_t t, w;
    key(u, t, w);
    __builtin_nontemporal_store((uint64_t)(t ^ w) + m, out + q);
  }
}

// ---- the production shape --------------------------------------------------------------
template <int U, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_oneshot(
    const uint4* __restrict__ tab, const uint8_t* __restrict__ pats, const uint64_t* __restrict__ offs,
    uint64_t npat, uint64_t* __restrict__ out) {
  const uint64_t q0 = blockIdx.x * (uint64_t)(256 * U) + threadIdx.x;
  uint32_t t[U], w[U];
  bool live[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * 256;
    live[j] = q < npat;
    t[j] = w[j] = 0;
    if (!live[j]) continue;
    const uint64_t o = offs[q], m = offs[q + 1] - o;
    if (m != kM) continue;
    uint32_t u[5];
    load_pat(pats, o, u);
    key(u, t[j], w[j]);
  }
  uint4 a[U];
#pragma unroll
  for (int j = 0; j < U; ++j) a[j] = live[j] ? ld_nt16(tab + t[j]) : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < U; ++j)
    if (live[j]) __builtin_nontemporal_store(rec_count(a[j], w[j]), out + q0 + (uint64_t)j * 256);
}

// ---- the production shape plus the production kernel's extras, one at a time (round 6) -----
// NALU: a dependent chain of NALU / 2 multiply-shift-add rounds (≈ 3 vector ops each) per
// pattern, half on the key before the record read, half on the record after it (the
// production count issues ~1,056 VALU per wave against the one-shot's 326: NALU = 122 at U = 2
// adds ≈ 730 per wave);
// kSecond: one lane in 50 makes a second, dependent random 64-B read after its record (the
// production's context sectors, ~2 % of the 20-mers)
template <int U, int WPE, int NALU, bool kSecond>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_oneshot_x(
    const uint4* __restrict__ tab, const uint8_t* __restrict__ pats, const uint64_t* __restrict__ offs,
    uint64_t npat, uint64_t* __restrict__ out) {
  const uint64_t q0 = blockIdx.x * (uint64_t)(256 * U) + threadIdx.x;
  uint32_t t[U], w[U];
  bool live[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * 256;
    live[j] = q < npat;
    t[j] = w[j] = 0;
    if (!live[j]) continue;
    const uint64_t o = offs[q], m = offs[q + 1] - o;
    if (m != kM) continue;
    uint32_t u[5];
    load_pat(pats, o, u);
    key(u, t[j], w[j]);
    uint32_t x = w[j];
#pragma unroll 1
    for (int i = 0; i < NALU / 2; ++i) x = x * 0x9E3779B1u + (x >> 7);
    w[j] ^= (x & 0x80000000u);  // (bit 31 of a 10-bit want: no effect on the match, kept live)
  }
  uint4 a[U];
#pragma unroll
  for (int j = 0; j < U; ++j) a[j] = live[j] ? ld_nt16(tab + t[j]) : make_uint4(0, 0, 0, 0);
  if constexpr (kSecond) {
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (live[j] && (mix(q0 + j * 256) % 50) == 0) {
        const uint4 b = ld_nt16(tab + ((t[j] ^ a[j].x) & (kRecs - 1)));
        a[j].x ^= b.x & 0x80000000u;
      }
  }
#pragma unroll
  for (int j = 0; j < U; ++j) {
    uint32_t x = a[j].x;
#pragma unroll 1
    for (int i = 0; i < NALU / 2; ++i) x = x * 0x9E3779B1u + (x >> 7);
    a[j].y ^= (x & 0x80000000u) >> 31 << 30;  // (bit 30 of y: outside the width and contexts)
  }
#pragma unroll
  for (int j = 0; j < U; ++j)
    if (live[j]) __builtin_nontemporal_store(rec_count(a[j], w[j]), out + q0 + (uint64_t)j * 256);
}

// ---- the production shape's prologue: a symbol map staged in LDS from global memory --------
// kOverlap false: map load -> LDS -> barrier, then offsets and patterns (k_count_ctx, round 5);
// true: the map load issued first, its LDS store and the barrier after the pattern loads are
// in flight.  kP32: the pattern through load_pattern32's nine predicated dword loads.
__device__ __forceinline__ void load_pattern32(const uint8_t* __restrict__ pats, uint64_t o0, uint32_t m,
                                               uint32_t u[8]) {
  const uint32_t* w0 = reinterpret_cast<const uint32_t*>(pats + (o0 & ~3ull));
  const uint32_t a = (uint32_t)(o0 & 3) * 8;
  const uint32_t nw = ((uint32_t)(o0 & 3) + m + 3) >> 2;
  uint32_t w[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) w[j] = (uint32_t)j < nw ? w0[j] : 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j) u[j] = (uint32_t)((((uint64_t)w[j + 1] << 32) | w[j]) >> a);
}
template <int U, bool kOverlap, bool kP32>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_oneshot_lds(
    const uint4* __restrict__ tab, const uint8_t* __restrict__ pats, const uint64_t* __restrict__ offs,
    uint64_t npat, uint64_t* __restrict__ out, const uint16_t* __restrict__ gmap) {
  __shared__ uint16_t cmap[256];
  uint16_t mv = 0;
  if (!kOverlap) {
    cmap[threadIdx.x] = gmap[threadIdx.x];
    __syncthreads();
  } else {
    mv = gmap[threadIdx.x];
  }
  const uint64_t q0 = blockIdx.x * (uint64_t)(256 * U) + threadIdx.x;
  uint32_t u[U][8];
  bool live[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * 256;
    live[j] = q < npat;
    if (!live[j]) continue;
    const uint64_t o = offs[q], m = offs[q + 1] - o;
    if (m != kM) {
      live[j] = false;
      continue;
    }
    if (kP32) load_pattern32(pats, o, (uint32_t)m, u[j]);
    else load_pat(pats, o, u[j]);
  }
  if (kOverlap) {
    cmap[threadIdx.x] = mv;
    __syncthreads();
  }
  uint32_t t[U], w[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    t[j] = w[j] = 0;
    if (!live[j]) continue;
#pragma unroll
    for (int i = 0; i < kM; ++i) {
      const uint32_t c = cmap[(u[j][i >> 2] >> (8 * (i & 3))) & 0xFFu] & 3u;
      if (i >= kM - kK) t[j] = t[j] * 4 + c;
      else w[j] |= c << (2 * (kM - kK - 1 - i));
    }
  }
  uint4 a[U];
#pragma unroll
  for (int j = 0; j < U; ++j) a[j] = live[j] ? ld_nt16(tab + t[j]) : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < U; ++j)
    if (live[j]) __builtin_nontemporal_store(rec_count(a[j], w[j]), out + q0 + (uint64_t)j * 256);
}

// ---- persistent, software-pipelined -------------------------------------------------------
// lane l of the grid takes queries l + i * S (S = lanes of the grid) in groups of U: while the
// records of group i are in flight, the pattern bytes of group i + 1 (whose offsets came with
// group i) and the offsets of group i + 2 load
template <int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_persist(
    const uint4* __restrict__ tab, const uint8_t* __restrict__ pats, const uint64_t* __restrict__ offs,
    uint64_t npat, uint64_t* __restrict__ out) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t step = S * U;
  // prologue: offsets of groups 0 and 1, pattern bytes of group 0
  uint64_t oc[U], mc[U], on[U], mn[U];
  uint32_t uc[U][5];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = l + (uint64_t)j * S, q1 = q + step;
    oc[j] = q < npat ? offs[q] : 0;
    mc[j] = q < npat ? offs[q + 1] - oc[j] : 0;
    on[j] = q1 < npat ? offs[q1] : 0;
    mn[j] = q1 < npat ? offs[q1 + 1] - on[j] : 0;
  }
#pragma unroll
  for (int j = 0; j < U; ++j)
    if (mc[j] == kM) load_pat(pats, oc[j], uc[j]);
  for (uint64_t b = l; b < npat; b += step) {
    uint32_t t[U], w[U];
    uint4 a[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      t[j] = w[j] = 0;
      if (mc[j] == kM) key(uc[j], t[j], w[j]);
      a[j] = mc[j] == kM ? ld_nt16(tab + t[j]) : make_uint4(0, 0, 0, 0);
    }
    // next group's pattern bytes, the one after's offsets (in flight with the records)
    uint32_t un[U][5];
    uint64_t o2[U], m2[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (mn[j] == kM) load_pat(pats, on[j], un[j]);
      const uint64_t q2 = b + 2 * step + (uint64_t)j * S;
      o2[j] = q2 < npat ? offs[q2] : 0;
      m2[j] = q2 < npat ? offs[q2 + 1] - o2[j] : 0;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t q = b + (uint64_t)j * S;
      if (q < npat) __builtin_nontemporal_store(mc[j] == kM ? rec_count(a[j], w[j]) : 0ull, out + q);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      oc[j] = on[j];
      mc[j] = mn[j];
      on[j] = o2[j];
      mn[j] = m2[j];
#pragma unroll
      for (int i = 0; i < 5; ++i) uc[j][i] = un[j][i];
    }
  }
}

// ---- two passes ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_split1(const uint8_t* __restrict__ pats,
                                                const uint64_t* __restrict__ offs, uint64_t npat,
                                                uint2* __restrict__ key_out) {
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= npat) return;
  const uint64_t o = offs[q], m = offs[q + 1] - o;
  uint32_t t = ~0u, w = 0;
  if (m == kM) {
    uint32_t u[5];
    load_pat(pats, o, u);
    key(u, t, w);
  }
  key_out[q] = make_uint2(t, w);
}
template <int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_split2(
    const uint4* __restrict__ tab, const uint2* __restrict__ keys, uint64_t npat, uint64_t* __restrict__ out) {
  const uint64_t q0 = blockIdx.x * (uint64_t)(256 * U) + threadIdx.x;
  uint2 k[U];
  uint4 a[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * 256;
    k[j] = q < npat ? keys[q] : make_uint2(~0u, 0);
  }
#pragma unroll
  for (int j = 0; j < U; ++j) a[j] = k[j].x != ~0u ? ld_nt16(tab + k[j].x) : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * 256;
    if (q < npat) __builtin_nontemporal_store(rec_count(a[j], k[j].y), out + q);
  }
}

// ---- setup --------------------------------------------------------------------------------
__global__ void k_fill_tab(uint64_t* p, uint64_t n) {
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += nt) p[i] = mix(i);
}
__global__ void k_fill_pats(uint8_t* pats, uint64_t* offs, uint64_t npat) {
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < npat; q += nt) {
    const uint64_t h = mix(q + 12345);
    for (int i = 0; i < kM; ++i) pats[q * kM + i] = "ACGT"[(h >> (2 * i)) & 3];
    offs[q] = q * kM;
    if (q == npat - 1) offs[npat] = npat * kM;
  }
}

template <class F>
double median_ms(int reps, F launch) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();  // warm
  CK(hipDeviceSynchronize());
  std::vector<float> v;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    v.push_back(ms);
  }
  CK(hipGetLastError());
  std::sort(v.begin(), v.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const uint64_t npat = (uint64_t)((argc > 1 ? std::atof(argv[1]) : 12.5) * 1e6);
  const int reps = argc > 2 ? std::atoi(argv[2]) : 21;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  uint4* tab;
  uint8_t* pats;
  uint64_t *offs, *out, *sink;
  uint2* keys;
  uint16_t* gmap;
  // argv[3]: the table's allocation — 0 hipMalloc, 1 hipExtMallocWithFlags(hipDeviceMallocContiguous)
  // (physically contiguous: address-translation reach); argv[4] = 1: the random and one-shot
  // shapes only
  const int alloc = argc > 3 ? std::atoi(argv[3]) : 0;
  const bool quick = argc > 4 && std::atoi(argv[4]) != 0;
  if (alloc == 1) CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&tab), kRecs * 16, hipDeviceMallocContiguous));
  else CK(hipMalloc(&tab, kRecs * 16));
  CK(hipMalloc(&pats, npat * kM + 64));
  CK(hipMalloc(&offs, (npat + 1) * 8));
  CK(hipMalloc(&out, npat * 8));
  CK(hipMalloc(&keys, npat * 8));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&gmap, 512));
  {
    std::vector<uint16_t> hm(256, 0xFF);
    hm['A'] = 0; hm['C'] = 1; hm['G'] = 2; hm['T'] = 3;
    CK(hipMemcpy(gmap, hm.data(), 512, hipMemcpyHostToDevice));
  }
  k_fill_tab<<<8192, 256>>>(reinterpret_cast<uint64_t*>(tab), kRecs * 2);
  k_fill_pats<<<4096, 256>>>(pats, offs, npat);
  CK(hipDeviceSynchronize());
  const double alg = npat * (8.0 + kM + 16 + 8);  // bytes per query the count reads / writes
  std::printf("{\"npat\": %llu, \"table_gb\": %.2f, \"cus\": %d, \"alg_bytes\": %.0f, \"alloc\": %d}\n",
              (unsigned long long)npat, kRecs * 16 / 1e9, ncu, alg, alloc);
  auto report = [&](const char* name, double ms, bool rand_reads) {
    std::printf("{\"shape\": \"%s\", \"ms\": %.4f, \"queries_per_s\": %.4g, \"rand_reads_per_s\": %.4g, "
                "\"alg_GBps\": %.1f}\n",
                name, ms, npat / ms * 1e3, rand_reads ? npat / ms * 1e3 : 0.0, alg / ms / 1e6);
    std::fflush(stdout);
  };
  const unsigned g1 = (unsigned)((npat + 255) / 256);
  for (unsigned g : {g1, 8u * ncu, 32u * ncu}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "rand grid=%u", g);
    report(nm, median_ms(reps, [&] { k_rand<<<g, 256>>>(tab, npat, sink); }), true);
  }
  for (unsigned g : {g1, 8u * ncu}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "stream grid=%u", g);
    report(nm, median_ms(reps, [&] { k_stream<<<g, 256>>>(pats, offs, npat, out); }), false);
  }
#define ONESHOT(U, WPE)                                                                        \
  report("oneshot U=" #U " wpe=" #WPE, median_ms(reps, [&] {                                 \
           k_oneshot<U, WPE><<<(unsigned)((npat + 256 * U - 1) / (256 * U)), 256>>>(tab, pats, offs, \
                                                                                 npat, out);    \
         }),                                                                                   \
         true)
  ONESHOT(1, 8);
  ONESHOT(2, 6);
#define ONESHOT_X(NALU, SEC)                                                                   \
  report("oneshot_x U=2 wpe=6 alu=" #NALU " second=" #SEC, median_ms(reps, [&] {              \
           k_oneshot_x<2, 6, NALU, SEC><<<(unsigned)((npat + 511) / 512), 256>>>(tab, pats, offs, npat, out); \
         }),                                                                                   \
         true)
  ONESHOT_X(0, false);
  ONESHOT_X(0, true);
  ONESHOT_X(122, false);
  ONESHOT_X(122, true);
  ONESHOT_X(244, false);
  if (quick) return 0;
  ONESHOT(2, 8);
  ONESHOT(4, 6);
#define ONESHOT_LDS(U, OV, P32)                                                                  \
  report("oneshot_lds U=" #U " overlap=" #OV " p32=" #P32, median_ms(reps, [&] {              \
           k_oneshot_lds<U, OV, P32><<<(unsigned)((npat + 256 * U - 1) / (256 * U)), 256>>>(      \
               tab, pats, offs, npat, out, gmap);                                                \
         }),                                                                                     \
         true)
  ONESHOT_LDS(1, false, false);
  ONESHOT_LDS(1, true, false);
  ONESHOT_LDS(2, false, false);
  ONESHOT_LDS(2, true, false);
  ONESHOT_LDS(2, false, true);
  ONESHOT_LDS(2, true, true);
  ONESHOT_LDS(1, true, true);
#define PERSIST(U, BPC)                                                                             \
  {                                                                                                 \
    char nm[64];                                                                                    \
    std::snprintf(nm, sizeof nm, "persist U=%d blocks/CU=%d", U, BPC);                              \
    report(nm, median_ms(reps, [&] { k_persist<U><<<(unsigned)(BPC * ncu), 256>>>(tab, pats, offs, npat, out); }), \
           true);                                                                                   \
  }
  PERSIST(1, 4);
  PERSIST(1, 8);
  PERSIST(2, 4);
  PERSIST(2, 8);
  PERSIST(4, 4);
  report("split pass1", median_ms(reps, [&] { k_split1<<<g1, 256>>>(pats, offs, npat, keys); }), false);
  report("split pass2 U=2", median_ms(reps, [&] {
           k_split2<2><<<(unsigned)((npat + 511) / 512), 256>>>(tab, keys, npat, out);
         }),
         true);
  report("split both U=2", median_ms(reps, [&] {
           k_split1<<<g1, 256>>>(pats, offs, npat, keys);
           k_split2<2><<<(unsigned)((npat + 511) / 512), 256>>>(tab, keys, npat, out);
         }),
         true);
  CK(hipFree(tab));
  CK(hipFree(pats));
  CK(hipFree(offs));
  CK(hipFree(out));
  CK(hipFree(keys));
  CK(hipFree(sink));
  return 0;
}
