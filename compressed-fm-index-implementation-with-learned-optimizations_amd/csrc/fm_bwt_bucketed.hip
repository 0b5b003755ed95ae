// fm_bwt_bucketed.hip — suffix sorting for texts the prefix-doubling builder cannot
// hold (n >= 2^32, BASELINE.json configs[4]: 32 GB): the BWT (src/core/bwt.hpp:7-15),
// the row-sampled SA (fm_index.cpp:57-66) and the inverse-SA samples are emitted
// pass by pass, without ever materialising the n-entry suffix array (256 GB at
// n = 3.2e10).  Same order as src/core/sais.hpp:8-16 (a proper prefix sorts first).
//
//   * symbols -> dense codes 1..sigma (0 = past the end), b bits; a 64-bit key
//     chunk holds K = 64/b consecutive codes, first symbol most significant;
//   * bins = the first L codes (b*L <= 12 bits); passes = runs of consecutive bins
//     whose suffix count fits the memory budget (rows of a pass are contiguous);
//   * per pass: select its positions (rocPRIM select over a counting iterator with
//     the bin predicate), sort (key chunk 0, position) by radix sort, then resolve
//     groups of equal keys with the next chunks (stable sorts by chunk then group)
//     over the compacted set of still-tied suffixes only, until every suffix is
//     alone — for random DNA one or two extra chunks, for an exact repeat of length
//     R about R/K rounds of a few launches over the repeat's suffixes;
//   * emit BWT bytes, SSA samples (row % stride == 0) and ISA samples
//     (position % pstride == 0) for the pass's rows.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "fm_internal.hpp"

namespace fmx {
namespace {

constexpr unsigned kBlk = 256;

struct Codes {
  uint16_t code[256];
  int b;  // bits per code
  int K;  // codes per 64-bit chunk
};

__device__ __forceinline__ uint64_t key_chunk(const uint8_t* __restrict__ t, uint64_t n,
                                              const uint16_t* __restrict__ code, int b, int K,
                                              uint64_t pos, uint64_t chunk) {
  uint64_t k = 0;
  const uint64_t s = pos + chunk * (uint64_t)K;
  for (int j = 0; j < K; ++j) {
    const uint64_t c = (s + j < n) ? code[t[s + j]] : 0u;
    k = (k << b) | c;
  }
  return k;
}

struct BinPred {
  const uint8_t* t;
  uint64_t n;
  const uint16_t* code;
  int b, L;
  uint32_t lo, hi;
  __device__ bool operator()(uint64_t i) const {
    uint32_t bin = 0;
    for (int j = 0; j < L; ++j) bin = (bin << b) | (i + j < n ? code[t[i + j]] : 0u);
    return bin >= lo && bin < hi;
  }
};

__global__ void k_bin_hist(const uint8_t* __restrict__ t, uint64_t n,
                           const uint16_t* __restrict__ code_g, int b, int L, uint32_t nbins,
                           unsigned long long* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* h = reinterpret_cast<uint32_t*>(smem);
  uint16_t* code = reinterpret_cast<uint16_t*>(smem + nbins * 4);
  for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x) h[i] = 0;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) code[i] = code_g[i];
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t bin = 0;
    for (int j = 0; j < L; ++j) bin = (bin << b) | (i + j < n ? code[t[i + j]] : 0u);
    atomicAdd(&h[bin], 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nbins; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

__global__ void k_hist256(const uint8_t* __restrict__ t, uint64_t n,
                          unsigned long long* __restrict__ hist) {
  __shared__ unsigned int h[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    atomicAdd(&h[t[i]], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x)
    if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

__global__ void k_keys(const uint8_t* __restrict__ t, uint64_t n, const uint16_t* __restrict__ code,
                       int b, int K, const uint64_t* __restrict__ pos, uint64_t P, uint64_t chunk,
                       uint64_t* __restrict__ key) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < P; j += stride)
    key[j] = key_chunk(t, n, code, b, K, pos[j], chunk);
}

// Group boundaries after the first sort: bound[j] = (j==0 || key[j] != key[j-1]).
__global__ void k_bounds(const uint64_t* __restrict__ key, uint64_t P, uint8_t* __restrict__ bound) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < P; j += stride)
    bound[j] = (j == 0 || key[j] != key[j - 1]) ? 1 : 0;
}

// tied[j]: slot j shares its group with another slot; gid_in = bound ? j : 0.
__global__ void k_tied(const uint8_t* __restrict__ bound, uint64_t P, uint32_t* __restrict__ gid_in,
                       uint8_t* __restrict__ tied, unsigned long long* __restrict__ ntied) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long local = 0;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < P; j += stride) {
    const bool single = bound[j] && (j + 1 == P || bound[j + 1]);
    tied[j] = single ? 0 : 1;
    gid_in[j] = bound[j] ? (uint32_t)j : 0u;
    local += !single;
  }
  for (int off = 32; off > 0; off >>= 1) local += __shfl_down(local, off, 64);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(ntied, local);
}

// Entering the compacted refinement: tied slot S[i] -> its group (slot of the group's
// first member) and its text position.
__global__ void k_init_compact(const uint64_t* __restrict__ S, uint64_t T,
                               const uint32_t* __restrict__ gid_scan, const uint64_t* __restrict__ pos,
                               uint32_t* __restrict__ cg, uint64_t* __restrict__ cpos) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < T; i += stride) {
    const uint64_t j = S[i];
    cg[i] = gid_scan[j];
    cpos[i] = pos[j];
  }
}

// Next key chunk of every still-tied suffix, plus iota for the permutation.
__global__ void k_ckeys(const uint8_t* __restrict__ t, uint64_t n, const uint16_t* __restrict__ code,
                        int b, int K, const uint64_t* __restrict__ cpos, uint64_t T, uint64_t chunk,
                        uint64_t* __restrict__ ckey, uint32_t* __restrict__ iota) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < T; i += stride) {
    ckey[i] = key_chunk(t, n, code, b, K, cpos[i], chunk);
    iota[i] = (uint32_t)i;
  }
}

__global__ void k_gather_gid(const uint32_t* __restrict__ tg, const uint32_t* __restrict__ idx,
                             uint64_t T, uint32_t* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < T; i += stride)
    out[i] = tg[idx[i]];
}

// Sorted tied element i (source idx[i]) goes to slot S[i]: groups keep their slot
// ranges, ordered inside by the new key.  A new group starts where the group or the
// key changes (startv = i there, for the max-scan).
__global__ void k_round_writeback(const uint64_t* __restrict__ S, const uint32_t* __restrict__ idx,
                                  const uint32_t* __restrict__ cg, const uint64_t* __restrict__ ckey,
                                  const uint64_t* __restrict__ cpos, uint64_t T,
                                  uint64_t* __restrict__ pos, uint32_t* __restrict__ startv,
                                  uint8_t* __restrict__ nbf) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < T; i += stride) {
    const uint32_t src = idx[i];
    pos[S[i]] = cpos[src];
    bool nb = i == 0;
    if (!nb) {
      const uint32_t prv = idx[i - 1];
      nb = cg[src] != cg[prv] || ckey[src] != ckey[prv];
    }
    startv[i] = nb ? (uint32_t)i : 0u;
    nbf[i] = nb ? 1 : 0;
  }
}

// still tied = not alone in its new group
__global__ void k_round_flags(const uint8_t* __restrict__ nbf, uint64_t T, uint8_t* __restrict__ tf) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < T; i += stride)
    tf[i] = (nbf[i] && (i + 1 == T || nbf[i + 1])) ? 0 : 1;
}

// Keep the still-tied elements (sel: their sorted indices, increasing), so the slot
// list stays increasing and the group id is the slot of the group's first member.
__global__ void k_round_compact(const uint32_t* __restrict__ sel, uint64_t T2,
                                const uint64_t* __restrict__ S, const uint32_t* __restrict__ start,
                                const uint32_t* __restrict__ idx, const uint64_t* __restrict__ cpos,
                                uint64_t* __restrict__ S2, uint32_t* __restrict__ cg2,
                                uint64_t* __restrict__ cpos2) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < T2; j += stride) {
    const uint32_t i = sel[j];
    S2[j] = S[i];
    cg2[j] = (uint32_t)S[start[i]];
    cpos2[j] = cpos[idx[i]];
  }
}

template <class SampleT>
__global__ void k_emit(const uint8_t* __restrict__ t, uint64_t n, uint32_t stride, uint32_t pstride,
                       const uint64_t* __restrict__ pos, uint64_t P, uint64_t row0,
                       uint8_t* __restrict__ bwt, SampleT* __restrict__ ssa, SampleT* __restrict__ isa) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < P; j += gs) {
    const uint64_t row = row0 + j, s = pos[j];
    bwt[row] = t[s == 0 ? n - 1 : s - 1];
    if (row % stride == 0) ssa[row / stride] = (SampleT)s;
    if (s % pstride == 0) isa[s / pstride] = (SampleT)row;
  }
}

template <class F, class... A>
cs_status tmp_call(DevBuf& tmp, size_t& tmp_bytes, F f) {
  size_t need = 0;
  FMX_HIP(f(nullptr, need));
  if (need > tmp_bytes) {
    FMX_HIP(tmp.alloc(need));
    tmp_bytes = need;
  }
  FMX_HIP(f(tmp.p, need));
  return CS_OK;
}

}  // namespace

cs_status build_bwt_bucketed(const uint8_t* d_text, uint64_t n, uint32_t stride, uint32_t pstride,
                             bool wide,
                             uint8_t* d_bwt, void* d_ssa, void* d_isa, hipStream_t st) {
  if (n == 0) return CS_OK;
  const bool verbose = build_opt("CS_FM_VERBOSE") != nullptr;
  // ---- codes ----
  DevBuf d_h;
  FMX_HIP(d_h.alloc(256 * 8));
  FMX_HIP(hipMemsetAsync(d_h.p, 0, 256 * 8, st));
  k_hist256<<<grid_for(n, kBlk, 8192), kBlk, 0, st>>>(d_text, n, d_h.as<unsigned long long>());
  unsigned long long hist[256];
  FMX_HIP(hipMemcpyAsync(hist, d_h.p, sizeof hist, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  Codes cd;
  int sigma = 0;
  for (int c = 0; c < 256; ++c) cd.code[c] = hist[c] ? (uint16_t)(++sigma) : 0;
  cd.b = 1;
  while ((1 << cd.b) <= sigma) ++cd.b;
  cd.K = 64 / cd.b;
  const int L = (12 / cd.b) > 0 ? (12 / cd.b) : 1;
  const uint32_t nbins = 1u << (cd.b * L);
  DevBuf d_code;
  FMX_HIP(d_code.alloc(sizeof cd.code));
  FMX_HIP(hipMemcpyAsync(d_code.p, cd.code, sizeof cd.code, hipMemcpyHostToDevice, st));
  const uint16_t* code = d_code.as<uint16_t>();

  // ---- bins and passes ----
  DevBuf d_bins;
  FMX_HIP(d_bins.alloc((size_t)nbins * 8));
  FMX_HIP(hipMemsetAsync(d_bins.p, 0, (size_t)nbins * 8, st));
  const size_t lds = (size_t)nbins * 4 + 512;
  k_bin_hist<<<grid_for(n, kBlk, 2048), kBlk, lds, st>>>(d_text, n, code, cd.b, L, nbins,
                                                          d_bins.as<unsigned long long>());
  FMX_HIP(hipGetLastError());
  std::vector<unsigned long long> bins(nbins);
  FMX_HIP(hipMemcpyAsync(bins.data(), d_bins.p, (size_t)nbins * 8, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  size_t free_b = 0, total_b = 0;
  FMX_HIP(hipMemGetInfo(&free_b, &total_b));
  uint64_t pmax = free_b / 64;  // ~40 B per element in flight + sort scratch
  if (pmax > (1ull << 31)) pmax = 1ull << 31;
  if (const char* e = build_opt("CS_FM_PASS_MAX")) pmax = std::strtoull(e, nullptr, 10);
  struct Pass { uint32_t lo, hi; uint64_t count, row0; };
  std::vector<Pass> passes;
  {
    uint64_t row = 0;
    uint32_t b0 = 0;
    uint64_t acc = 0;
    for (uint32_t bi = 0; bi < nbins; ++bi) {
      if (bins[bi] > pmax) {
        set_error("bucketed suffix sort: a bin exceeds the pass budget (text too repetitive)");
        return CS_ERR_INVALID;
      }
      if (acc + bins[bi] > pmax && acc) {
        passes.push_back({b0, bi, acc, row});
        row += acc;
        acc = 0;
        b0 = bi;
      }
      acc += bins[bi];
    }
    if (acc) passes.push_back({b0, nbins, acc, row});
  }
  uint64_t pbig = 0;
  for (auto& p : passes) pbig = p.count > pbig ? p.count : pbig;
  if (verbose)
    std::fprintf(stderr, "[cs_fm bucketed] sigma=%d b=%d K=%d L=%d passes=%zu max_pass=%llu\n", sigma,
                 cd.b, cd.K, L, passes.size(), (unsigned long long)pbig);

  DevBuf pos0, pos1, key0, key1, bound, gid_in, gid_scan, tied, d_cnt, tmp;
  size_t tmp_bytes = 0;
  FMX_HIP(pos0.alloc(pbig * 8));
  FMX_HIP(pos1.alloc(pbig * 8));
  FMX_HIP(key0.alloc(pbig * 8));
  FMX_HIP(key1.alloc(pbig * 8));
  FMX_HIP(bound.alloc(pbig));
  FMX_HIP(gid_in.alloc(pbig * 4));
  FMX_HIP(gid_scan.alloc(pbig * 4));
  FMX_HIP(tied.alloc(pbig));
  FMX_HIP(d_cnt.alloc(16));
  const unsigned G = grid_for(pbig, kBlk, 16384);

  for (const Pass& ps : passes) {
    const uint64_t P = ps.count;
    // 1. positions of the pass (increasing), by predicate over all text positions
    BinPred pred{d_text, n, code, cd.b, L, ps.lo, ps.hi};
    rocprim::counting_iterator<uint64_t> it(0);
    cs_status s = tmp_call(tmp, tmp_bytes, [&](void* p, size_t& b) {
      return rocprim::select(p, b, it, pos0.as<uint64_t>(), d_cnt.as<uint64_t>(), (size_t)n, pred, st);
    });
    if (s != CS_OK) return s;
    // 2. chunk-0 keys, sort (key, pos)
    k_keys<<<G, kBlk, 0, st>>>(d_text, n, code, cd.b, cd.K, pos0.as<uint64_t>(), P, 0,
                               key0.as<uint64_t>());
    rocprim::double_buffer<uint64_t> kb(key0.as<uint64_t>(), key1.as<uint64_t>());
    rocprim::double_buffer<uint64_t> vb(pos0.as<uint64_t>(), pos1.as<uint64_t>());
    s = tmp_call(tmp, tmp_bytes, [&](void* p, size_t& b) {
      return rocprim::radix_sort_pairs(p, b, kb, vb, P, 0, cd.b * cd.K, st);
    });
    if (s != CS_OK) return s;
    uint64_t* pos = vb.current();
    uint64_t* pos_alt = vb.alternate();
    k_bounds<<<G, kBlk, 0, st>>>(kb.current(), P, bound.as<uint8_t>());
    // 3. refine groups of equal keys with further chunks.  One full-pass sweep finds
    // the tied slots; from then on every round works on the compacted tied set only
    // (cost O(tied), not O(P)), so a long exact repeat costs rounds of a few small
    // launches each.  Suffixes of one group differ at the latest where the shorter
    // one ends (past-the-end code 0), so at most n/K + 1 rounds are needed.
    FMX_HIP(hipMemsetAsync(d_cnt.p, 0, 16, st));
    k_tied<<<G, kBlk, 0, st>>>(bound.as<uint8_t>(), P, gid_in.as<uint32_t>(), tied.as<uint8_t>(),
                               d_cnt.as<unsigned long long>() + 1);
    unsigned long long ntied = 0;
    FMX_HIP(hipMemcpyAsync(&ntied, d_cnt.as<unsigned long long>() + 1, 8, hipMemcpyDeviceToHost, st));
    FMX_HIP(hipStreamSynchronize(st));
    if (verbose)
      std::fprintf(stderr, "[cs_fm bucketed] pass bins [%u,%u) P=%llu: %llu tied after chunk 0\n",
                   ps.lo, ps.hi, (unsigned long long)P, ntied);
    if (ntied) {
      uint64_t T = ntied;
      s = tmp_call(tmp, tmp_bytes, [&](void* p, size_t& b) {
        return rocprim::inclusive_scan(p, b, gid_in.as<uint32_t>(), gid_scan.as<uint32_t>(), (size_t)P,
                                       rocprim::maximum<uint32_t>(), st);
      });
      if (s != CS_OK) return s;
      // compact arrays, sized once for the first tied set (it only shrinks); the
      // pass-sized key/pos/flag buffers are free from here on and are reused
      DevBuf S0, S1, cpos1, cg1, cgs, gscr, iota, idx1, start, sel;
      FMX_HIP(S0.alloc(T * 8));
      FMX_HIP(S1.alloc(T * 8));
      FMX_HIP(cpos1.alloc(T * 8));
      FMX_HIP(cg1.alloc(T * 4));
      FMX_HIP(cgs.alloc(T * 4));
      FMX_HIP(gscr.alloc(T * 4));
      FMX_HIP(iota.alloc(T * 4));
      FMX_HIP(idx1.alloc(T * 4));
      FMX_HIP(start.alloc(T * 4));
      FMX_HIP(sel.alloc(T * 4));
      uint64_t* cS = S0.as<uint64_t>();
      uint64_t* nS = S1.as<uint64_t>();
      uint64_t* cpos = pos_alt;
      uint64_t* npos = cpos1.as<uint64_t>();
      uint32_t* cg = gid_in.as<uint32_t>();
      uint32_t* ncg = cg1.as<uint32_t>();
      uint64_t* ckey = key0.as<uint64_t>();
      uint64_t* ckey2 = key1.as<uint64_t>();
      uint32_t* startv = gid_scan.as<uint32_t>();
      uint8_t* nbf = bound.as<uint8_t>();
      uint8_t* tf = tied.as<uint8_t>();
      const uint8_t* tied_all = tied.as<uint8_t>();
      s = tmp_call(tmp, tmp_bytes, [&](void* p, size_t& b) {
        return rocprim::select(p, b, rocprim::counting_iterator<uint64_t>(0), tied_all, cS,
                               d_cnt.as<uint64_t>(), (size_t)P, st);
      });
      if (s != CS_OK) return s;
      // gid_scan is read here before its buffer becomes startv
      k_init_compact<<<grid_for(T, kBlk, 16384), kBlk, 0, st>>>(cS, T, gid_scan.as<uint32_t>(), pos,
                                                                 cg, cpos);
      FMX_HIP(hipGetLastError());
      int gbits = 1;
      while (gbits < 32 && (1ull << gbits) < P) ++gbits;
      const uint64_t max_chunk = n / (uint64_t)cd.K + 2;
      uint64_t chunk = 1;
      for (;; ++chunk) {
        if (chunk > max_chunk) {
          set_error("bucketed suffix sort: refinement did not converge (internal error)");
          return CS_ERR_INVALID;
        }
        const unsigned GT = grid_for(T, kBlk, 16384);
        k_ckeys<<<GT, kBlk, 0, st>>>(d_text, n, code, cd.b, cd.K, cpos, T, chunk, ckey,
                                     iota.as<uint32_t>());
        // stable by key, then stable by group -> (group, key) order in iota
        s = tmp_call(tmp, tmp_bytes, [&](void* p, size_t& b) {
          return rocprim::radix_sort_pairs(p, b, ckey, ckey2, iota.as<uint32_t>(), idx1.as<uint32_t>(),
                                           T, 0, cd.b * cd.K, st);
        });
        if (s != CS_OK) return s;
        k_gather_gid<<<GT, kBlk, 0, st>>>(cg, idx1.as<uint32_t>(), T, cgs.as<uint32_t>());
        s = tmp_call(tmp, tmp_bytes, [&](void* p, size_t& b) {
          return rocprim::radix_sort_pairs(p, b, cgs.as<uint32_t>(), gscr.as<uint32_t>(),
                                           idx1.as<uint32_t>(), iota.as<uint32_t>(), T, 0, gbits, st);
        });
        if (s != CS_OK) return s;
        const uint32_t* idx = iota.as<uint32_t>();
        k_round_writeback<<<GT, kBlk, 0, st>>>(cS, idx, cg, ckey, cpos, T, pos, startv, nbf);
        k_round_flags<<<GT, kBlk, 0, st>>>(nbf, T, tf);
        FMX_HIP(hipGetLastError());
        s = tmp_call(tmp, tmp_bytes, [&](void* p, size_t& b) {
          return rocprim::inclusive_scan(p, b, startv, start.as<uint32_t>(), (size_t)T,
                                         rocprim::maximum<uint32_t>(), st);
        });
        if (s != CS_OK) return s;
        s = tmp_call(tmp, tmp_bytes, [&](void* p, size_t& b) {
          return rocprim::select(p, b, rocprim::counting_iterator<uint32_t>(0), (const uint8_t*)tf,
                                 sel.as<uint32_t>(), d_cnt.as<uint64_t>(), (size_t)T, st);
        });
        if (s != CS_OK) return s;
        uint64_t T2 = 0;
        FMX_HIP(hipMemcpyAsync(&T2, d_cnt.p, 8, hipMemcpyDeviceToHost, st));
        FMX_HIP(hipStreamSynchronize(st));
        if (verbose && (chunk <= 3 || (chunk & (chunk - 1)) == 0))
          std::fprintf(stderr, "[cs_fm bucketed]   chunk %llu: %llu tied\n", (unsigned long long)chunk,
                       (unsigned long long)T2);
        if (!T2) break;
        k_round_compact<<<grid_for(T2, kBlk, 16384), kBlk, 0, st>>>(
            sel.as<uint32_t>(), T2, cS, start.as<uint32_t>(), idx, cpos, nS, ncg, npos);
        FMX_HIP(hipGetLastError());
        std::swap(cS, nS);
        std::swap(cg, ncg);
        std::swap(cpos, npos);
        T = T2;
      }
    }
    // 4. emit the pass's rows
    if (wide)
      k_emit<uint64_t><<<G, kBlk, 0, st>>>(d_text, n, stride, pstride, pos, P, ps.row0, d_bwt,
                                           static_cast<uint64_t*>(d_ssa), static_cast<uint64_t*>(d_isa));
    else
      k_emit<uint32_t><<<G, kBlk, 0, st>>>(d_text, n, stride, pstride, pos, P, ps.row0, d_bwt,
                                           static_cast<uint32_t*>(d_ssa), static_cast<uint32_t*>(d_isa));
    FMX_HIP(hipGetLastError());
    FMX_HIP(hipStreamSynchronize(st));
  }
  return CS_OK;
}

}  // namespace fmx
