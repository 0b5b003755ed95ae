// fm_build.hip — index construction on the device (replaces, with identical
// output, FMIndex::build_from_text, src/api/fm_index.cpp:16-69):
//
//   1. suffix array in plain suffix order (src/core/sais.hpp:8-16: a proper prefix
//      sorts first) by prefix doubling over device radix sorts (rocPRIM) —
//      O(n log L) instead of the reference's O(n^2 log n) string sort;
//   2. cyclic BWT (src/core/bwt.hpp:7-15) and row-sampled SSA (fm_index.cpp:57-66);
//   3. C[] (fm_index.cpp:36-47) from the symbol histogram (the BWT is a permutation
//      of the text);
//   4. the rank structure (fm_build_rank.hip): occurrence lines when at most four
//      symbols carry all but a few rows (DNA), else the quaternary wavelet matrix,
//      or the reference's 8-level binary wavelet matrix (src/core/wavelet.cpp:14-53)
//      as rank lines; the locate walk lines;
//   5. the node table (starts, ranks, purity) for the query kernels.
// Index construction is not the timed hot path; it is HBM-streaming work.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fm_internal.hpp"

namespace fmx {
namespace {

constexpr unsigned kBlk = 256;

__global__ void k_hist(const uint8_t* __restrict__ t, uint64_t n,
                       unsigned long long* __restrict__ hist) {
  __shared__ unsigned int h[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t n16 = n / 16;
  const uint4* t16 = reinterpret_cast<const uint4*>(t);
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint4 v = t16[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int b = 0; b < 4; ++b) atomicAdd(&h[(w[k] >> (8 * b)) & 0xFFu], 1u);
    }
  }
  for (uint64_t i = n16 * 16 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    atomicAdd(&h[t[i]], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

// Initial key: the first K symbols, dense codes 1..sigma (0 past the end, so a
// proper prefix sorts first), b bits each.
__global__ void k_init_keys(const uint8_t* __restrict__ t, uint64_t n,
                            const uint16_t* __restrict__ code_g, int b, int K,
                            uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
  __shared__ uint16_t code[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) code[i] = code_g[i];
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t k = 0;
    for (int j = 0; j < K; ++j) {
      const uint64_t c = (i + j < n) ? code[t[i + j]] : 0u;
      k = (k << b) | c;
    }
    key[i] = k;
    val[i] = (uint32_t)i;
  }
}

// Group heads of the sorted keys: hp[j] = j at a head, else 0; counts heads.
__global__ void k_heads(const uint64_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ hp,
                        unsigned long long* __restrict__ ngroups) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long local = 0;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += stride) {
    const bool head = (j == 0) || key[j] != key[j - 1];
    hp[j] = head ? (uint32_t)j : 0u;
    local += head;
  }
  // wave reduce then one atomic per wave
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(ngroups, local);
}

__global__ void k_scatter_rank(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ hp,
                               uint64_t n, uint32_t* __restrict__ rank) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n; j += stride)
    rank[sa[j]] = hp[j] + 1u;
}

__global__ void k_double_keys(const uint32_t* __restrict__ rank, uint64_t n, uint64_t h, int B,
                              uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t r2 = (i + h < n) ? rank[i + h] : 0u;
    key[i] = ((uint64_t)rank[i] << B) | r2;
    val[i] = (uint32_t)i;
  }
}

// bwt.hpp:7-15 and fm_index.cpp:57-66 in one pass, plus the inverse-SA samples
// (row of every pstride-th text position) for extract and the walk-line marks.
template <class SampleT>
__global__ void k_bwt_ssa(const uint8_t* __restrict__ t, const uint32_t* __restrict__ sa,
                          uint32_t n, uint32_t stride, uint32_t pstride, uint8_t* __restrict__ bwt,
                          SampleT* __restrict__ ssa, SampleT* __restrict__ isa) {
  const uint32_t gs = gridDim.x * blockDim.x;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gs) {
    const uint32_t s = sa[j];
    bwt[j] = t[s == 0 ? n - 1 : s - 1];
    if (j % stride == 0) ssa[j / stride] = s;
    if (s % pstride == 0) isa[s / pstride] = j;
  }
}

// CS_FM_VERBOSE=1: phase timings of the build on stderr.
struct PhaseLog {
  bool on;
  hipStream_t st;
  std::chrono::steady_clock::time_point t0;
  explicit PhaseLog(hipStream_t s) : on(build_opt("CS_FM_VERBOSE") != nullptr), st(s),
                                     t0(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (!on) return;
    (void)hipStreamSynchronize(st);
    const auto t = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[cs_fm build] %-28s %9.1f ms\n", what,
                 std::chrono::duration<double, std::milli>(t - t0).count());
    t0 = t;
  }
};

uint32_t bitrev(uint32_t x, int bits) {
  uint32_t r = 0;
  for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
  return r;
}

struct SortTemp {
  DevBuf buf;
  size_t bytes = 0;
};

}  // namespace

cs_status build_sa_device(const uint8_t* d_text, uint64_t n, uint32_t* d_sa, hipStream_t st) {
  if (n == 0) return CS_OK;
  if (n >= (1ull << 32)) {
    set_error("text length must be < 2^32 (uint32 suffix array, src/core/sais.hpp:9)");
    return CS_ERR_INVALID;
  }
  // symbol histogram -> dense codes
  DevBuf d_hist;
  FMX_HIP(d_hist.alloc(256 * sizeof(unsigned long long)));
  FMX_HIP(hipMemsetAsync(d_hist.p, 0, 256 * sizeof(unsigned long long), st));
  k_hist<<<grid_for(n / 16 + 1, kBlk, 8192), kBlk, 0, st>>>(d_text, n, d_hist.as<unsigned long long>());
  unsigned long long hist[256];
  FMX_HIP(hipMemcpyAsync(hist, d_hist.p, sizeof hist, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  uint16_t code[256];  // 1..sigma, sigma <= 256 needs 9 bits
  int sigma = 0;
  for (int c = 0; c < 256; ++c) code[c] = hist[c] ? (uint16_t)(++sigma) : 0;
  int b = 1;
  while ((1 << b) <= sigma) ++b;  // codes 0..sigma need b bits
  const int K = 64 / b;
  DevBuf d_code;
  FMX_HIP(d_code.alloc(sizeof code));
  FMX_HIP(hipMemcpyAsync(d_code.p, code, sizeof code, hipMemcpyHostToDevice, st));

  DevBuf k0, k1, v1, hp, hp2, rank, d_ng;
  FMX_HIP(k0.alloc(n * 8));
  FMX_HIP(k1.alloc(n * 8));
  FMX_HIP(v1.alloc(n * 4));
  FMX_HIP(hp.alloc(n * 4));
  FMX_HIP(hp2.alloc(n * 4));
  FMX_HIP(rank.alloc(n * 4));
  FMX_HIP(d_ng.alloc(8));
  uint32_t* v0 = d_sa;  // sorted values end up in either buffer; copied to d_sa at the end

  PhaseLog plog(st);
  plog.mark("sa: histogram+alloc");
  const unsigned G = grid_for(n, kBlk, 16384);
  k_init_keys<<<G, kBlk, 0, st>>>(d_text, n, d_code.as<uint16_t>(), b, K, k0.as<uint64_t>(), v0);
  FMX_HIP(hipGetLastError());

  int B = 1;
  while (B < 64 && (1ull << B) <= n) ++B;  // ranks 1..n need B bits
  SortTemp tmp;
  uint64_t h = (uint64_t)K;
  int end_bit = b * K;
  for (int iter = 0;; ++iter) {
    rocprim::double_buffer<uint64_t> kb(k0.as<uint64_t>(), k1.as<uint64_t>());
    rocprim::double_buffer<uint32_t> vb(v0, v1.as<uint32_t>());
    size_t need = 0;
    FMX_HIP(rocprim::radix_sort_pairs(nullptr, need, kb, vb, n, 0, end_bit, st));
    if (need > tmp.bytes) {
      FMX_HIP(tmp.buf.alloc(need));
      tmp.bytes = need;
    }
    FMX_HIP(rocprim::radix_sort_pairs(tmp.buf.p, need, kb, vb, n, 0, end_bit, st));
    plog.mark("sa: radix sort");
    const uint64_t* skey = kb.current();
    const uint32_t* sval = vb.current();
    FMX_HIP(hipMemsetAsync(d_ng.p, 0, 8, st));
    k_heads<<<G, kBlk, 0, st>>>(skey, n, hp.as<uint32_t>(), d_ng.as<unsigned long long>());
    size_t sneed = 0;
    FMX_HIP(rocprim::inclusive_scan(nullptr, sneed, hp.as<uint32_t>(), hp2.as<uint32_t>(), n,
                                    rocprim::maximum<uint32_t>(), st));
    if (sneed > tmp.bytes) {
      FMX_HIP(tmp.buf.alloc(sneed));
      tmp.bytes = sneed;
    }
    FMX_HIP(rocprim::inclusive_scan(tmp.buf.p, sneed, hp.as<uint32_t>(), hp2.as<uint32_t>(), n,
                                    rocprim::maximum<uint32_t>(), st));
    unsigned long long ng = 0;
    FMX_HIP(hipMemcpyAsync(&ng, d_ng.p, 8, hipMemcpyDeviceToHost, st));
    FMX_HIP(hipStreamSynchronize(st));
    plog.mark("sa: heads+scan");
    if (plog.on) std::fprintf(stderr, "[cs_fm build] sa round %d: h=%llu groups=%llu of %llu\n",
                              iter, (unsigned long long)h, ng, (unsigned long long)n);
    if (ng == n) {  // every suffix has a distinct h-prefix: sval is the SA
      if (sval != d_sa) FMX_HIP(hipMemcpyAsync(d_sa, sval, n * 4, hipMemcpyDeviceToDevice, st));
      FMX_HIP(hipStreamSynchronize(st));
      return CS_OK;
    }
    k_scatter_rank<<<G, kBlk, 0, st>>>(sval, hp2.as<uint32_t>(), n, rank.as<uint32_t>());
    // next round sorts (rank[i], rank[i+h]) = the 2h-prefix
    k_double_keys<<<G, kBlk, 0, st>>>(rank.as<uint32_t>(), n, h, B, k0.as<uint64_t>(), v0);
    FMX_HIP(hipGetLastError());
    end_bit = 2 * B;
    h *= 2;
    if (iter > 64) {
      set_error("suffix sorting did not converge");
      return CS_ERR_INVALID;
    }
  }
}

static cs_status finish_index(DevBuf& bwt, const unsigned long long* hist, cs_fm_index* h,
                              hipStream_t st, PhaseLog& plog, DevBuf* sa_pending = nullptr);

// Text-position sample stride (inverse-SA samples for extract; walk-line marks and
// their position samples for locate): an eighth of the SSA stride, at least 1.  A locate
// walk then averages about pstride / 2 steps instead of stride / 2, an extract
// (stride - pstride) / 2 fewer; the reference's row-sampled SSA (fm_index.cpp:57-66) is
// kept as is.  The walk's position samples cost 4 B (narrow) or 5 B (wide: 40-bit
// entries) x n / pstride (C4: 4 GB, C5: 40 GB); a wide index's inverse-SA samples (u64) are
// thinned to every eighth once the walk lines are built (thin_isa: C5 8 GB), so its HBM
// still goes to the left contexts and context records first (round 2 kept C5 at pstride
// 8 with u64 samples, 3.2 walk steps per position).  C4 walk of 12.5 M positions: 1.8 ms
// at pstride 8, 1.3 ms at 4 (profiles/r01/locate_phases_c4_p*.json).  CS_FM_PSTRIDE
// overrides.
static uint32_t position_stride(uint32_t stride, bool wide) {
  (void)wide;
  uint32_t p = stride / 8u;
  if (const char* e = build_opt("CS_FM_PSTRIDE")) p = (uint32_t)std::atoi(e);
  return p ? p : 1u;
}

template <class S>
__global__ void k_thin(const S* __restrict__ in, uint64_t nout, uint32_t f, S* __restrict__ out) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < nout; k += gs) out[k] = in[k * f];
}

// Keep every f-th inverse-SA sample (stride xstride = f pstride): extract then starts
// at most f pstride positions past its end instead of pstride; the walk marks and their
// position samples (built from the full set) stay at pstride.
static cs_status thin_isa(cs_fm_index* h, uint32_t f, hipStream_t st) {
  const uint64_t xs = (uint64_t)h->pstride * f;
  const uint64_t nout = (h->n + xs - 1) / xs;
  void* out = nullptr;
  FMX_HIP(hipMalloc(&out, (nout ? nout : 1) * h->sample_bytes()));
  if (h->wide)
    k_thin<uint64_t><<<grid_for(nout, kBlk, 16384), kBlk, 0, st>>>(
        static_cast<const uint64_t*>(h->d_isa), nout, f, static_cast<uint64_t*>(out));
  else
    k_thin<uint32_t><<<grid_for(nout, kBlk, 16384), kBlk, 0, st>>>(
        static_cast<const uint32_t*>(h->d_isa), nout, f, static_cast<uint32_t*>(out));
  FMX_HIP(hipGetLastError());
  FMX_HIP(hipStreamSynchronize(st));
  FMX_HIP(hipFree(h->d_isa));
  h->d_isa = out;
  h->nisa = nout;
  h->xstride = (uint32_t)xs;
  return CS_OK;
}

cs_status build_index_device(const uint8_t* d_text, uint64_t n, uint32_t stride, cs_fm_index* h,
                             hipStream_t st) {
  if (stride == 0) {
    set_error("ssa_stride must be > 0");
    return CS_ERR_INVALID;
  }
  if (n >= (1ull << 38)) {
    set_error("text length must be < 2^38");
    return CS_ERR_INVALID;
  }
  h->n = n;
  h->stride = stride;
  // wide index: u64 samples / table entries and 64-B lines (n >= 2^32, or forced
  // by the CS_FM_WIDE test hook)
  h->wide = n >= (1ull << 32);
  if (const char* e = build_opt("CS_FM_WIDE"))
    if (std::atoi(e) == 1) h->wide = true;
  h->nsamples = (n + stride - 1) / stride;
  NodeTable& T = h->h_table;
  std::memset(&T, 0, sizeof T);

  // --- histogram (BWT is a permutation of the text) ---
  unsigned long long hist[256] = {0};
  if (n) {
    DevBuf d_hist;
    FMX_HIP(d_hist.alloc(256 * sizeof(unsigned long long)));
    FMX_HIP(hipMemsetAsync(d_hist.p, 0, 256 * sizeof(unsigned long long), st));
    k_hist<<<grid_for(n / 16 + 1, kBlk, 8192), kBlk, 0, st>>>(d_text, n,
                                                              d_hist.as<unsigned long long>());
    FMX_HIP(hipMemcpyAsync(hist, d_hist.p, sizeof hist, hipMemcpyDeviceToHost, st));
    FMX_HIP(hipStreamSynchronize(st));
  }

  if (n) {  // unique smallest last symbol: LF is one n-cycle, suffix order = rotation order
    uint8_t last = 0;
    FMX_HIP(hipMemcpy(&last, d_text + n - 1, 1, hipMemcpyDeviceToHost));
    int smallest = 0;
    while (smallest < 256 && hist[smallest] == 0) ++smallest;
    h->lf_exact = hist[last] == 1 && last == smallest;
  }
  PhaseLog plog(st);
  plog.mark("histogram");
  // --- SA, BWT, SSA ---
  DevBuf bwt;
  FMX_HIP(bwt.alloc(n));
  FMX_HIP(hipMalloc(&h->d_ssa, (h->nsamples ? h->nsamples : 1) * h->sample_bytes()));
  h->pstride = position_stride(stride, h->wide);
  h->nisa = (n + h->pstride - 1) / h->pstride;  // text positions 0, pstride, ... < n
  h->xstride = h->pstride;
  FMX_HIP(hipMalloc(&h->d_isa, (h->nisa ? h->nisa : 1) * h->sample_bytes()));
  DevBuf sa_pending;  // with an HBM budget: the full SA, kept at the end if it still fits
  bool bucketed = n >= (1ull << 32);
  if (const char* e = build_opt("CS_FM_SA_BUILDER"))
    if (std::string(e) == "bucketed") bucketed = true;
  if (n && bucketed) {  // BWT + samples pass by pass, no full SA (fm_bwt_bucketed.hip)
    cs_status s = build_bwt_bucketed(d_text, n, stride, h->pstride, h->wide, bwt.as<uint8_t>(), h->d_ssa,
                                     h->d_isa, st);
    if (s != CS_OK) return s;
  } else if (n) {  // prefix doubling over the full u32 SA
    DevBuf sa;
    FMX_HIP(sa.alloc(n * 4));
    cs_status s = build_sa_device(d_text, n, sa.as<uint32_t>(), st);
    if (s != CS_OK) return s;
    if (h->wide)
      k_bwt_ssa<uint64_t><<<grid_for(n, kBlk, 16384), kBlk, 0, st>>>(
          d_text, sa.as<uint32_t>(), (uint32_t)n, stride, h->pstride, bwt.as<uint8_t>(),
          static_cast<uint64_t*>(h->d_ssa), static_cast<uint64_t*>(h->d_isa));
    else
      k_bwt_ssa<uint32_t><<<grid_for(n, kBlk, 16384), kBlk, 0, st>>>(
          d_text, sa.as<uint32_t>(), (uint32_t)n, stride, h->pstride, bwt.as<uint8_t>(),
          static_cast<uint32_t*>(h->d_ssa), static_cast<uint32_t*>(h->d_isa));
    FMX_HIP(hipGetLastError());
    FMX_HIP(hipStreamSynchronize(st));
    // Keep the full suffix array (as the reference keeps sa_, fm_index.hpp:43) when LF is
    // one n-cycle: a located row's position is then SA[row] (what the reference's SSA
    // walk computes, fm_index.cpp:125-153), one read instead of a walk.  4n bytes (C4:
    // 16 GB), an eighth of the device left free; CS_FM_FULL_SA=0 keeps only the samples.
    bool keep = h->lf_exact;
    if (const char* e = build_opt("CS_FM_FULL_SA")) keep = keep && std::atoi(e) != 0;
    size_t free_b = 0, total_b = 0;
    if (keep && h->hbm_budget) {
      // an HBM budget: the full SA ranks after the count structures, so it is decided
      // last (finish_index), replacing the walk lines when it fits
      std::swap(sa_pending.p, sa.p);
    } else if (keep && hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > total_b / 8 + n * 8) {
      h->d_sa = sa.p;  // the handle owns it from here
      sa.p = nullptr;
    }
  }
  plog.mark("suffix array + bwt + ssa");

  return finish_index(bwt, hist, h, st, plog, &sa_pending);
}

// Everything after the BWT and the samples: rank structure, C[], node table, prefix
// table, walk lines.  Shared by the text builder and cs_fm_create.
static cs_status finish_index(DevBuf& bwt, const unsigned long long* hist, cs_fm_index* h,
                              hipStream_t st, PhaseLog& plog, DevBuf* sa_pending) {
  const uint64_t n = h->n;
  NodeTable& T = h->h_table;
  // --- rank structure: occurrence lines (<= 4 frequent symbols) or the wavelet
  //     matrix levels as rank lines ---
  CodeMap occ_map;
  uint8_t occ_sym[4] = {0, 0, 0, 0};
  bool occ = occ_feasible(hist, n, occ_map, occ_sym);
  bool qwm = !occ && n > 0 && n < (1ull << 40);
  bool learned = false;  // learned occurrence lines instead of occurrence lines
  if (const char* e = build_opt("CS_FM_ENGINE")) {  // test hooks: force an engine
    const std::string want(e);
    if (want == "learned") learned = occ;
    if (want == "wavelet") occ = qwm = false;
    if (want == "qwm" && n > 0 && n < (1ull << 40)) {
      occ = false;
      qwm = true;
    }
  }
  if (qwm) {
    h->line_fmt = kFmtQwm;
    h->line_bytes = OccLine::kBytes;
    h->line_bits = OccLine::kRows;
    h->nlines = (n >> 6) + 1;
    cs_status qs = build_qwm(bwt.as<uint8_t>(), n, hist, h, st);
    if (qs != CS_OK) return qs;
    bool walk = true;
    if (const char* e = build_opt("CS_FM_WALK"))  // "0": walk over the matrix levels
      walk = std::atoi(e) != 0;
    if (walk) {  // walk lines carry level 0: each symbol's first base-4 digit
      CodeMap d0;
      std::memset(d0.c, 0, sizeof d0.c);
      const int L = (int)T.qlevels;
      for (int c = 0; c < 256; ++c)
        if (hist[c]) d0.c[c] = (uint8_t)((T.occ_code[c] >> (2 * (L - 1))) & 3u);
      qs = build_walk(bwt.as<uint8_t>(), n, d0, h, st);
      if (qs != CS_OK) return qs;
    }
  } else if (occ) {
    h->line_fmt = learned ? kFmtLOcc : kFmtOcc;
    h->line_bytes = OccLine::kBytes;
    h->line_bits = learned ? LOccLine::kRows : OccLine::kRows;
    h->nlevels = 1;
    // + the line holding row n, so occ(c, n) is a line read
    h->nlines = learned ? n / LOccLine::kRows + 1 : (n >> 6) + 1;
    std::memcpy(T.occ_code, occ_map.c, sizeof T.occ_code);
    std::memcpy(T.occ_sym, occ_sym, sizeof T.occ_sym);
    cs_status os = learned ? build_locc(bwt.as<uint8_t>(), n, occ_map, h, st)
                           : build_occ(bwt.as<uint8_t>(), n, occ_map, h, st);
    if (os != CS_OK) return os;
    bool walk = true;
    if (const char* e = build_opt("CS_FM_WALK"))  // "0": walk over the occurrence lines
      walk = std::atoi(e) != 0;
    if (walk) {
      os = build_walk(bwt.as<uint8_t>(), n, occ_map, h, st);
      if (os != CS_OK) return os;
    }
  } else {
    std::memset(T.occ_code, kNoCode, sizeof T.occ_code);
    h->line_fmt = h->wide ? kFmtLine32W : kFmtLine32;  // Line32 bases are u32
    if (const char* e = build_opt("CS_FM_LINE_BYTES"))  // test hook: force 64-B lines
      if (std::atoi(e) == 64) h->line_fmt = kFmtLine64;
    h->line_bytes = h->line_fmt == kFmtLine64 ? 64 : 32;
    h->line_bits = h->line_fmt == kFmtLine32 ? Line32::kBits
                   : h->line_fmt == kFmtLine32W ? Line32W::kBits : Line64::kBits;
    h->nlevels = kLevels;
    h->nlines = n / h->line_bits + 1;  // + sentinel so rank1(n) is a line read
    cs_status ws = build_wm_levels(bwt.as<uint8_t>(), n, h, st);
    if (ws != CS_OK) return ws;
  }
  FMX_HIP(hipStreamSynchronize(st));
  bwt.release();
  if (h->wide && h->nisa) {  // the walk marks are built: extract keeps every eighth sample
    cs_status ts = thin_isa(h, 8, st);
    if (ts != CS_OK) return ts;
  }
  plog.mark("wavelet levels");

  // --- node table from the histogram ---
  uint64_t cum = 0;
  for (int c = 0; c < 256; ++c) {
    T.C[c] = cum;
    cum += hist[c];
  }
  T.C[256] = cum;
  for (int l = 0; l <= kLevels && !qwm; ++l) {  // binary wavelet nodes (QWM set its own)
    const int np = 1 << l;
    std::vector<uint64_t> cnt(np, 0);
    for (int c = 0; c < 256; ++c) cnt[l ? (c >> (8 - l)) : 0] += hist[c];
    // level-l order: by the bit-reversed l-bit prefix (stable partitions, MSB first)
    std::vector<uint32_t> order(np);
    for (int x = 0; x < np; ++x) order[bitrev(x, l)] = x;
    uint64_t s = 0;
    for (int r = 0; r < np; ++r) {
      const int x = order[r];
      if (l < kLevels) T.S[node_id(l, x)] = s;
      else T.S8[x] = s;
      s += cnt[x];
    }
    if (l == kLevels) break;
    for (int x = 0; x < np; ++x) {
      int seen = 0, b0 = -1;
      bool pure = true;
      for (int c = 0; c < 256; ++c) {
        if (!hist[c] || (l ? (c >> (8 - l)) : 0) != x) continue;
        const int b = (c >> (7 - l)) & 1;
        if (!seen) b0 = b;
        else if (b != b0) pure = false;
        seen = 1;
      }
      uint8_t f = 0;
      if (pure) f = kPure | (b0 == 1 ? kPureBit : 0);
      T.flags[node_id(l, x)] = f;
    }
  }
  for (int c = 0; c < 256; ++c) {
    uint32_t m = 0;
    for (int l = 0; l < kLevels && !qwm; ++l)
      if (!(T.flags[node_id(l, l ? (c >> (8 - l)) : 0)] & kPure)) m |= 1u << l;
    if (occ) m = T.occ_code[c] != kNoCode ? 1u : 0u;  // one line per occ, none for rare symbols
    if (qwm) {
      m = 0;
      const int L = (int)T.qlevels;
      const uint32_t x = T.occ_code[c];
      for (int l = 0; l < L; ++l)
        if (!(T.flags[qnode_id(l, x >> (2 * (L - l)))] & kPure)) m |= 1u << l;
    }
    h->active_levels[c] = hist[c] ? m : 0;
  }
  FMX_HIP(hipMalloc(&h->d_table, sizeof(NodeTable)));
  FMX_HIP(hipMemcpyAsync(h->d_table, &T, sizeof T, hipMemcpyHostToDevice, st));
  {
    DevBuf dR;
    FMX_HIP(dR.alloc(kNodes * 8));
    cs_status rs = launch_node_ranks(h, dR.as<uint64_t>(), st);
    if (rs != CS_OK) return rs;
    FMX_HIP(hipMemcpyAsync(T.R, dR.p, kNodes * 8, hipMemcpyDeviceToHost, st));
    FMX_HIP(hipStreamSynchronize(st));
  }
  FMX_HIP(hipMemcpyAsync(h->d_table, &T, sizeof T, hipMemcpyHostToDevice, st));
  {
    cs_status ps = build_prefix_table(h, st);
    if (ps != CS_OK) return ps;
    FMX_HIP(hipMemcpyAsync(h->d_table, &T, sizeof T, hipMemcpyHostToDevice, st));
  }
  plog.mark("prefix table");
  {
    cs_status cs = build_left_contexts(h, st);
    if (cs != CS_OK) return cs;
  }
  plog.mark("left contexts");
  {
    cs_status cs = build_context_records(h, st);
    if (cs != CS_OK) return cs;
  }
  plog.mark("context records");
  if (sa_pending && sa_pending->p) {
    // budget builds: the full suffix array replaces the walk lines and their position
    // samples when the index still fits its budget with it
    const uint64_t walk_b = (h->d_walk ? h->nwalk * 32 : 0) + (h->d_wssa ? h->nwssa * h->wssa_bytes() : 0);
    if (index_hbm_bytes(h) + n * 4 <= h->hbm_budget + walk_b) {
      if (h->d_walk) FMX_HIP(hipFree(h->d_walk));
      if (h->d_wssa) FMX_HIP(hipFree(h->d_wssa));
      h->d_walk = h->d_wssa = nullptr;
      h->nwalk = 0;
      h->walk_marks = 0;
      h->d_sa = sa_pending->p;  // the handle owns it from here
      sa_pending->p = nullptr;
    }
    sa_pending->release();
  }
  FMX_HIP(hipMalloc(&h->d_err, 8));
  FMX_HIP(hipMemsetAsync(h->d_err, 0xFF, 8, st));
  FMX_HIP(hipStreamSynchronize(st));
  plog.mark("node table");
  return CS_OK;
}

// cs_fm_create: the index from a BWT and the reference's row-sampled SSA built
// elsewhere (the members FMIndex::build_from_text leaves in bwt_ and ssa_,
// src/api/fm_index.cpp:49-66).  No suffix sorting; no inverse-SA samples, so the
// walk uses the given row samples and extract needs the caller's text.
cs_status build_index_from_bwt(const uint8_t* bwt_host, uint64_t n, const uint32_t* ssa_host,
                               uint64_t nsamples, uint32_t stride, cs_fm_index* h, hipStream_t st) {
  if (stride == 0) {
    set_error("ssa_stride must be > 0");
    return CS_ERR_INVALID;
  }
  if (n >= (1ull << 32)) {
    set_error("cs_fm_create: u32 samples need n < 2^32");
    return CS_ERR_INVALID;
  }
  if (nsamples != (n + stride - 1) / stride) {
    set_error("cs_fm_create: ssa must hold ceil(n / stride) samples");
    return CS_ERR_INVALID;
  }
  h->n = n;
  h->stride = stride;
  h->pstride = h->xstride = stride;
  h->wide = false;
  h->nsamples = nsamples;
  h->nisa = 0;
  NodeTable& T = h->h_table;
  std::memset(&T, 0, sizeof T);
  PhaseLog plog(st);
  DevBuf bwt;
  FMX_HIP(bwt.alloc(n));
  FMX_HIP(hipMalloc(&h->d_ssa, (nsamples ? nsamples : 1) * 4));
  if (n) {
    FMX_HIP(hipMemcpyAsync(bwt.p, bwt_host, n, hipMemcpyHostToDevice, st));
    FMX_HIP(hipMemcpyAsync(h->d_ssa, ssa_host, nsamples * 4, hipMemcpyHostToDevice, st));
  }
  unsigned long long hist[256] = {0};
  if (n) {
    DevBuf d_hist;
    FMX_HIP(d_hist.alloc(256 * sizeof(unsigned long long)));
    FMX_HIP(hipMemsetAsync(d_hist.p, 0, 256 * sizeof(unsigned long long), st));
    k_hist<<<grid_for(n / 16 + 1, kBlk, 8192), kBlk, 0, st>>>(bwt.as<uint8_t>(), n,
                                                              d_hist.as<unsigned long long>());
    FMX_HIP(hipMemcpyAsync(hist, d_hist.p, sizeof hist, hipMemcpyDeviceToHost, st));
    FMX_HIP(hipStreamSynchronize(st));
    // LF is one n-cycle when the unique smallest symbol ends the text: then the
    // smallest suffix is the last one, SA[0] = n - 1
    int smallest = 0;
    while (smallest < 256 && hist[smallest] == 0) ++smallest;
    h->lf_exact = hist[smallest] == 1 && ssa_host[0] == n - 1;
  }
  return finish_index(bwt, hist, h, st, plog);
}

}  // namespace fmx
