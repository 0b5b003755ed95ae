// fm_build_rank.hip — the rank structures, built on the device from a BWT in HBM
// (the second half of FMIndex::build_from_text, src/api/fm_index.cpp:49-55, and
// WaveletTree::build, src/core/wavelet.cpp:14-53):
//   * the reference's binary wavelet matrix as rank lines (fm_device.hpp Line*):
//     ballot bit-packing per level, line popcounts + exclusive scan for the bases,
//     stable zeros-then-ones partition through the level's own rank lines;
//   * occurrence lines (OccLine) for <= 4 frequent symbols, rare rows listed;
//   * the quaternary wavelet matrix: occurrence lines per base-4 digit, stable
//     4-way partitions;
//   * the locate walk lines (WalkLine / WalkLineW) with their sample marks.
// All streaming HBM work; index construction is not the timed hot path.
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fm_internal.hpp"

namespace fmx {
namespace {

constexpr unsigned kBlk = 256;

// Payload word w of a level (global word index) lives in line w/7, slot w%7.
template <class F>
__device__ __forceinline__ void store_word(void* L, uint64_t w, uint64_t v) {
  const uint64_t line = w / F::kWords, slot = w % F::kWords;
  if (F::kWordBits == 32)  // 32-B lines: 8 dwords
    reinterpret_cast<uint32_t*>(L)[line * 8 + F::kBaseWords + slot] = (uint32_t)v;
  else
    reinterpret_cast<uint64_t*>(L)[line * 8 + F::kBaseWords + slot] = v;
}

// One wave per 64 positions: ballot of the level bit (= 1 or 2 payload words).
template <class F>
__global__ void k_pack_level(const uint8_t* __restrict__ cur, uint64_t n, int bit,
                             void* __restrict__ L, uint64_t ngroups, uint64_t nwords) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t g = wave; g < ngroups; g += nwaves) {
    const uint64_t p = g * 64 + lane;
    const int b = p < n ? (cur[p] >> bit) & 1 : 0;
    const uint64_t w = __ballot(b);
    if (F::kWordBits == 64) {
      if (lane == 0) store_word<F>(L, g, w);
    } else {  // a line holds 7 dwords, so the last group may straddle the end
      if (lane == 0) store_word<F>(L, 2 * g, w & 0xFFFFFFFFull);
      if (lane == 1 && 2 * g + 1 < nwords) store_word<F>(L, 2 * g + 1, w >> 32);
    }
  }
}

template <class F>
__global__ void k_line_counts(const void* __restrict__ L, uint64_t nlines,
                              uint64_t* __restrict__ cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; l < nlines; l += stride) {
    typename F::Raw v;
    F::load(L, l, v);
    cnt[l] = F::prefix(v, F::kBits);
  }
}

template <class F>
__global__ void k_set_base(void* __restrict__ L, const uint64_t* __restrict__ base,
                           uint64_t nlines) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; l < nlines; l += stride) {
    if (F::kBaseWords == 1 && F::kWordBits == 32)  // Line32: u32 base
      reinterpret_cast<uint32_t*>(L)[l * 8] = (uint32_t)base[l];
    else  // u64 base at the line start (Line32W: 4 qwords per line, Line64: 8)
      reinterpret_cast<uint64_t*>(L)[l * (F::kBytes / 8)] = base[l];
  }
}

// Stable zeros-then-ones partition (wavelet.cpp:27-30, :47-50) using the level's
// own rank lines: dst = b ? Z + rank1(p) : p - rank1(p).
template <class F>
__global__ void k_partition(const uint8_t* __restrict__ cur, uint64_t n, int bit,
                            const void* __restrict__ L, uint64_t Z, uint8_t* __restrict__ nxt) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p < n; p += stride) {
    const uint8_t s = cur[p];
    const uint64_t r = rank1_at<F>(L, p);
    const uint64_t dst = ((s >> bit) & 1) ? Z + r : p - r;
    nxt[dst] = s;
  }
}

template <class F>
__global__ void k_node_rank(const void* __restrict__ lines, uint64_t nlines,
                            const NodeTable* __restrict__ T, uint64_t* __restrict__ R) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kNodes) return;
  int level = 0;
  while ((1 << (level + 1)) - 1 <= t) ++level;
  const void* lv = reinterpret_cast<const uint8_t*>(lines) + (uint64_t)level * nlines * F::kBytes;
  R[t] = rank1_at<F>(lv, T->S[t]);
}

}  // namespace

// 8 wavelet-matrix levels (wavelet.cpp:14-53) from the BWT in `cur` (consumed).
template <class F>
static cs_status build_levels(uint8_t* cur, uint64_t n, cs_fm_index* h, hipStream_t st) {
  const uint64_t nl = h->nlines;
  const size_t lbytes = (size_t)kLevels * nl * F::kBytes;
  FMX_HIP(hipMalloc(&h->d_lines, lbytes));
  FMX_HIP(hipMemsetAsync(h->d_lines, 0, lbytes, st));
  NodeTable& T = h->h_table;  // Z[] filled here, the rest by the caller
  DevBuf nxt, cnt, base, tmp;
  FMX_HIP(nxt.alloc(n));
  FMX_HIP(cnt.alloc(nl * 8));
  FMX_HIP(base.alloc(nl * 8));
  size_t tmp_bytes = 0;
  FMX_HIP(rocprim::exclusive_scan(nullptr, tmp_bytes, cnt.as<uint64_t>(), base.as<uint64_t>(),
                                  (uint64_t)0, nl, rocprim::plus<uint64_t>(), st));
  FMX_HIP(tmp.alloc(tmp_bytes));
  uint8_t* nx = nxt.as<uint8_t>();
  const uint64_t nwords = nl * F::kWords;
  const uint64_t ngroups = (nwords * F::kWordBits + 63) / 64;  // 64 positions per wave
  for (int l = 0; l < kLevels; ++l) {
    const int bit = 7 - l;
    void* L = reinterpret_cast<uint8_t*>(h->d_lines) + (uint64_t)l * nl * F::kBytes;
    k_pack_level<F><<<grid_for(ngroups * 64, kBlk, 16384), kBlk, 0, st>>>(cur, n, bit, L, ngroups, nwords);
    k_line_counts<F><<<grid_for(nl, kBlk, 16384), kBlk, 0, st>>>(L, nl, cnt.as<uint64_t>());
    size_t tb = tmp_bytes;
    FMX_HIP(rocprim::exclusive_scan(tmp.p, tb, cnt.as<uint64_t>(), base.as<uint64_t>(), (uint64_t)0,
                                    nl, rocprim::plus<uint64_t>(), st));
    k_set_base<F><<<grid_for(nl, kBlk, 16384), kBlk, 0, st>>>(L, base.as<uint64_t>(), nl);
    uint64_t last[2];
    FMX_HIP(hipMemcpyAsync(&last[0], base.as<uint64_t>() + nl - 1, 8, hipMemcpyDeviceToHost, st));
    FMX_HIP(hipMemcpyAsync(&last[1], cnt.as<uint64_t>() + nl - 1, 8, hipMemcpyDeviceToHost, st));
    FMX_HIP(hipStreamSynchronize(st));
    T.Z[l] = n - (last[0] + last[1]);
    if (l + 1 < kLevels && n) {
      k_partition<F><<<grid_for(n, kBlk, 16384), kBlk, 0, st>>>(cur, n, bit, L, T.Z[l], nx);
      FMX_HIP(hipGetLastError());
      std::swap(cur, nx);
    }
  }
  FMX_HIP(hipStreamSynchronize(st));
  return CS_OK;
}

cs_status build_wm_levels(uint8_t* bwt, uint64_t n, cs_fm_index* h, hipStream_t st) {
  return h->line_fmt == kFmtLine32    ? build_levels<Line32>(bwt, n, h, st)
         : h->line_fmt == kFmtLine32W ? build_levels<Line32W>(bwt, n, h, st)
                                      : build_levels<Line64>(bwt, n, h, st);
}

// ---- occurrence lines (fm_device.hpp OccLine) ----

// One thread per line q: pack the 64 rows' codes (rare symbols as code 0, rows past
// n as code 0), count codes 0..2 among the rows < n, and list the rare rows.
__global__ void k_occ_pack(const uint8_t* __restrict__ bwt, uint64_t n, CodeMap map, uint64_t nl,
                           uint32_t* __restrict__ lines, uint32_t* __restrict__ cnt,
                           unsigned long long* __restrict__ exc_rows, uint8_t* __restrict__ exc_sym,
                           unsigned int* __restrict__ exc_n) {
  __shared__ uint8_t code[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) code[i] = map.c[i];
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < nl; q += stride) {
    const uint64_t a = q << 6;
    uint32_t w[4] = {0, 0, 0, 0};
    uint32_t c0 = 0, c1 = 0, c2 = 0;
    for (int r = 0; r < 64; ++r) {
      if (a + r >= n) break;
      const uint32_t sym = bwt[a + r];
      uint32_t k = code[sym];
      if (k == kNoCode) {
        const unsigned int e = atomicAdd(exc_n, 1u);
        if (e < (unsigned)kMaxExc) {
          exc_rows[e] = a + r;
          exc_sym[e] = (uint8_t)sym;
        }
        k = 0;
      }
      w[r >> 4] |= k << (2 * (r & 15));
      c0 += k == 0;
      c1 += k == 1;
      c2 += k == 2;
    }
    uint4* L = reinterpret_cast<uint4*>(lines) + q * 2;
    L[1] = make_uint4(w[0], w[1], w[2], w[3]);
    cnt[q] = c0;
    cnt[nl + q] = c1;
    cnt[2 * nl + q] = c2;
  }
}

// dword j and byte 12+j of each line = scanned occ(code j) (n < 2^40)
__global__ void k_occ_base(uint32_t* __restrict__ lines, const uint64_t* __restrict__ base,
                           uint64_t nl, int j) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < nl; q += stride) {
    const uint64_t b = base[q];
    lines[q * 8 + j] = (uint32_t)b;
    reinterpret_cast<uint8_t*>(lines)[q * 32 + 12 + j] = (uint8_t)(b >> 32);
  }
}

// ---- learned occurrence lines (fm_device.hpp LOccLine) ----
// One thread per line: the 104 rows' codes (rare symbols as code 0, listed), and the
// line's count of codes 0..2.
__global__ void k_locc_pack(const uint8_t* __restrict__ bwt, uint64_t n, CodeMap map, uint64_t nl,
                            uint32_t* __restrict__ lines, uint32_t* __restrict__ cnt,
                            unsigned long long* __restrict__ exc_rows, uint8_t* __restrict__ exc_sym,
                            unsigned int* __restrict__ exc_n) {
  __shared__ uint8_t code[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) code[i] = map.c[i];
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < nl; q += stride) {
    const uint64_t a = q * LOccLine::kRows;
    uint32_t w[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t c0 = 0, c1 = 0, c2 = 0;
    for (uint32_t r = 0; r < LOccLine::kRows; ++r) {
      if (a + r >= n) break;
      const uint32_t sym = bwt[a + r];
      uint32_t k = code[sym];
      if (k == kNoCode) {
        const unsigned int e = atomicAdd(exc_n, 1u);
        if (e < (unsigned)kMaxExc) {
          exc_rows[e] = a + r;
          exc_sym[e] = (uint8_t)sym;
        }
        k = 0;
      }
      w[r >> 4] |= k << (2 * (r & 15));
      c0 += k == 0;
      c1 += k == 1;
      c2 += k == 2;
    }
    uint4* L = reinterpret_cast<uint4*>(lines) + q * 2;
    L[0] = make_uint4(w[0], w[1], w[2], w[3]);
    L[1] = make_uint4(w[4], w[5], w[6], 0u);  // residuals are filled in per code
    cnt[q] = c0;
    cnt[nl + q] = c1;
    cnt[2 * nl + q] = c2;
  }
}

// One thread per superblock: the model of code j through the occ values at the
// superblock's first and last line starts (base[] = exclusive scan of the counts).
__global__ void k_locc_model(const uint64_t* __restrict__ base, uint64_t nl, uint32_t shift,
                             uint64_t nsb, int j, LOccModel* __restrict__ models) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < nsb; b += gs) {
    const uint64_t q0 = b << shift;
    uint64_t q1 = q0 + (1ull << shift) - 1;
    if (q1 >= nl) q1 = nl - 1;
    const uint64_t b0 = base[q0], b1 = base[q1];
    const uint64_t rows = 104ull * (q1 - q0);
    models[b].base[j] = b0;
    models[b].slope[j] = rows ? ((b1 - b0) << 32) / rows : 0;
  }
}

// One thread per line: residual of code j against its superblock's model; flags any
// residual outside int16.
__global__ void k_locc_resid(uint32_t* __restrict__ lines, const uint64_t* __restrict__ base,
                             uint64_t nl, uint32_t shift, const LOccModel* __restrict__ models,
                             int j, unsigned int* __restrict__ bad) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < nl; q += gs) {
    const LOccModel m = models[q >> shift];
    const int64_t r = (int64_t)base[q] - (int64_t)locc_pred(m, (uint32_t)j, q - ((q >> shift) << shift));
    if (r < -32768 || r > 32767) atomicOr(bad, 1u);
    uint16_t* h16 = reinterpret_cast<uint16_t*>(lines + q * 8 + 6);  // w3 bits 16.. (dwords 6, 7)
    h16[1 + j] = (uint16_t)(int16_t)r;
  }
}

// ---- quaternary wavelet matrix (fm_query.hip QWM) ----
__global__ void k_qcodes(const uint8_t* __restrict__ bwt, uint64_t n, CodeMap map,
                         uint8_t* __restrict__ out) {
  __shared__ uint8_t code[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) code[i] = map.c[i];
  __syncthreads();
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += gs)
    out[i] = code[bwt[i]];
}

// One thread per occurrence line of a level: digit (cur >> shift) & 3 of 64 rows,
// per-line counts of digits 0..2.
__global__ void k_qwm_pack(const uint8_t* __restrict__ cur, uint64_t n, int shift, uint64_t nl,
                           uint32_t* __restrict__ lines, uint8_t* __restrict__ cnt) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < nl; q += gs) {
    const uint64_t a = q << 6;
    uint32_t w[4] = {0, 0, 0, 0};
    uint32_t c0 = 0, c1 = 0, c2 = 0;
    for (int r = 0; r < 64 && a + r < n; ++r) {
      const uint32_t d = (cur[a + r] >> shift) & 3u;
      w[r >> 4] |= d << (2 * (r & 15));
      c0 += d == 0;
      c1 += d == 1;
      c2 += d == 2;
    }
    reinterpret_cast<uint4*>(lines)[q * 2 + 1] = make_uint4(w[0], w[1], w[2], w[3]);
    cnt[q] = (uint8_t)c0;
    cnt[nl + q] = (uint8_t)c1;
    cnt[2 * nl + q] = (uint8_t)c2;
  }
}

struct QZ {
  uint64_t z[4];
};

// stable 4-way partition by the level's digit: nxt[Z[d] + occ(d, i)] = cur[i]
__global__ void k_qwm_partition(const uint8_t* __restrict__ cur, uint64_t n, int shift,
                                const void* __restrict__ lines, QZ Z, uint8_t* __restrict__ nxt) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += gs) {
    const uint8_t v = cur[i];
    const uint32_t d = (v >> shift) & 3u;
    OccLine::Raw L;
    const uint64_t q = i >> 6;
    OccLine::load(lines, q, L);
    nxt[Z.z[d] + OccLine::base(L, d, q) + OccLine::prefix(L, d, (uint32_t)(i & 63))] = v;
  }
}

// R of every pure node: occ_l(d, S) at its start
__global__ void k_qnode_rank(const void* __restrict__ lines, uint64_t nl,
                             const NodeTable* __restrict__ T, uint64_t* __restrict__ R) {
  for (int l = 0; l < (int)T->qlevels; ++l) {
    const int np = 1 << (2 * l);
    for (int x = threadIdx.x; x < np; x += blockDim.x) {
      const int nid = qnode_id(l, (uint32_t)x);
      uint64_t r = 0;
      if (T->flags[nid] & kPure) {
        const uint32_t d = (T->flags[nid] >> 2) & 3u;
        const uint64_t S = T->S[nid], q = S >> 6;
        OccLine::Raw v;
        OccLine::load(static_cast<const uint8_t*>(lines) + (uint64_t)l * nl * OccLine::kBytes, q, v);
        r = OccLine::base(v, d, q) + OccLine::prefix(v, d, (uint32_t)(S & 63));
      }
      R[nid] = r;
    }
  }
}

cs_status build_qwm(const uint8_t* bwt, uint64_t n, const unsigned long long* hist, cs_fm_index* h,
                    hipStream_t st) {
  NodeTable& T = h->h_table;
  CodeMap map;
  std::memset(map.c, 0, sizeof map.c);
  uint32_t sigma = 0;
  std::vector<uint64_t> hc;
  for (int c = 0; c < 256; ++c)
    if (hist[c]) {
      map.c[c] = (uint8_t)sigma;
      T.qsym[sigma] = (uint8_t)c;
      hc.push_back(hist[c]);
      ++sigma;
    }
  std::memcpy(T.occ_code, map.c, sizeof T.occ_code);
  int L = 1;
  while ((1u << (2 * L)) < sigma) ++L;
  T.qlevels = (uint32_t)L;
  h->nlevels = (uint32_t)L;
  const uint64_t nl = h->nlines;
  FMX_HIP(hipMalloc(&h->d_lines, (uint64_t)L * nl * OccLine::kBytes));
  FMX_HIP(hipMemsetAsync(h->d_lines, 0, (uint64_t)L * nl * OccLine::kBytes, st));
  DevBuf cur, nxt, cnt, base, tmp;
  FMX_HIP(cur.alloc(n));
  FMX_HIP(nxt.alloc(n));
  FMX_HIP(cnt.alloc(3 * nl));
  FMX_HIP(base.alloc(nl * 8));
  k_qcodes<<<grid_for(n, kBlk, 16384), kBlk, 0, st>>>(bwt, n, map, cur.as<uint8_t>());
  FMX_HIP(hipGetLastError());
  size_t tb = 0;
  FMX_HIP(rocprim::exclusive_scan(nullptr, tb, cnt.as<uint8_t>(), base.as<uint64_t>(), (uint64_t)0,
                                  nl, rocprim::plus<uint64_t>(), st));
  FMX_HIP(tmp.alloc(tb));
  for (int l = 0; l < L; ++l) {
    const int shift = 2 * (L - 1 - l);
    uint32_t* lv = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(h->d_lines) +
                                               (uint64_t)l * nl * OccLine::kBytes);
    k_qwm_pack<<<grid_for(nl, kBlk, 16384), kBlk, 0, st>>>(cur.as<uint8_t>(), n, shift, nl, lv,
                                                          cnt.as<uint8_t>());
    FMX_HIP(hipGetLastError());
    uint64_t tot[3];
    for (int j = 0; j < 3; ++j) {
      size_t t2 = tb;
      FMX_HIP(rocprim::exclusive_scan(tmp.p, t2, cnt.as<uint8_t>() + (uint64_t)j * nl,
                                      base.as<uint64_t>(), (uint64_t)0, nl,
                                      rocprim::plus<uint64_t>(), st));
      k_occ_base<<<grid_for(nl, kBlk, 16384), kBlk, 0, st>>>(lv, base.as<uint64_t>(), nl, j);
      FMX_HIP(hipGetLastError());
      uint64_t last = 0;
      uint8_t lc = 0;
      FMX_HIP(hipMemcpyAsync(&last, base.as<uint64_t>() + nl - 1, 8, hipMemcpyDeviceToHost, st));
      FMX_HIP(hipMemcpyAsync(&lc, cnt.as<uint8_t>() + (uint64_t)j * nl + nl - 1, 1,
                             hipMemcpyDeviceToHost, st));
      FMX_HIP(hipStreamSynchronize(st));
      tot[j] = last + lc;
    }
    QZ Z;
    Z.z[0] = 0;
    Z.z[1] = tot[0];
    Z.z[2] = tot[0] + tot[1];
    Z.z[3] = tot[0] + tot[1] + tot[2];
    for (int d = 0; d < 4; ++d) T.qZ[l][d] = Z.z[d];
    if (l + 1 < L) {
      k_qwm_partition<<<grid_for(n, kBlk, 16384), kBlk, 0, st>>>(cur.as<uint8_t>(), n, shift, lv, Z,
                                                                nxt.as<uint8_t>());
      FMX_HIP(hipGetLastError());
      std::swap(cur.p, nxt.p);
    }
  }
  // node starts (digit-reversed prefix order, as the stable partitions leave them),
  // purity and leaf starts from the code histogram
  for (int l = 0; l <= L; ++l) {
    const int np = 1 << (2 * l);
    std::vector<uint64_t> cntx(np, 0);
    for (uint32_t y = 0; y < sigma; ++y) cntx[l ? (y >> (2 * (L - l))) : 0] += hc[y];
    std::vector<std::pair<uint32_t, int>> ord;
    for (int x = 0; x < np; ++x) {
      uint32_t rev = 0;
      for (int k = 0; k < l; ++k) rev |= ((x >> (2 * k)) & 3u) << (2 * (l - 1 - k));
      ord.push_back({rev, x});
    }
    std::sort(ord.begin(), ord.end());
    uint64_t sacc = 0;
    for (auto& e : ord) {
      const int x = e.second;
      if (l < L) T.S[qnode_id(l, (uint32_t)x)] = sacc;
      else T.S8[x] = sacc;
      sacc += cntx[x];
    }
    if (l == L) break;
    for (int x = 0; x < np; ++x) {
      int d0 = -1;
      bool pure = true;
      for (uint32_t y = 0; y < sigma; ++y) {
        if ((l ? (y >> (2 * (L - l))) : 0u) != (uint32_t)x) continue;
        const int d = (int)((y >> (2 * (L - 1 - l))) & 3u);
        if (d0 < 0) d0 = d;
        else if (d != d0) pure = false;
      }
      T.flags[qnode_id(l, (uint32_t)x)] = pure ? (uint8_t)(kPure | ((d0 < 0 ? 0 : d0) << 2)) : 0;
    }
  }
  FMX_HIP(hipStreamSynchronize(st));
  return CS_OK;
}

// Occurrence-line engine choice: the (at most) four most frequent symbols get
// 2-bit codes in symbol order; the rest must hold at most kMaxExc rows.
bool occ_feasible(const unsigned long long* hist, uint64_t n, CodeMap& map, uint8_t occ_sym[4]) {
  if (n == 0 || n >= (1ull << 40)) return false;
  int order[256], np = 0;
  for (int c = 0; c < 256; ++c)
    if (hist[c]) order[np++] = c;
  std::stable_sort(order, order + np, [&](int x, int y) { return hist[x] > hist[y]; });
  const int nc = np < 4 ? np : 4;
  uint64_t rare = 0;
  for (int i = nc; i < np; ++i) rare += hist[order[i]];
  if (rare > (uint64_t)kMaxExc) return false;
  std::sort(order, order + nc);
  std::memset(map.c, kNoCode, sizeof map.c);
  for (int k = 0; k < 4; ++k) occ_sym[k] = k < nc ? (uint8_t)order[k] : 0;
  for (int k = 0; k < nc; ++k) map.c[order[k]] = (uint8_t)k;
  return true;
}

// Learned occurrence lines (LOccLine): codes and residuals per line, models per
// superblock of 2^14 lines (2^8 when a residual of the first try overflows int16:
// then every residual fits, fm_device.hpp).  Rare rows as build_occ.
cs_status build_locc(const uint8_t* bwt, uint64_t n, const CodeMap& map, cs_fm_index* h,
                     hipStream_t st) {
  const uint64_t nl = h->nlines;
  FMX_HIP(hipMalloc(&h->d_lines, nl * LOccLine::kBytes));
  DevBuf cnt, base, tmp, erow, esym, en, bad;
  FMX_HIP(cnt.alloc(3 * nl * 4));
  FMX_HIP(base.alloc(3 * nl * 8));
  FMX_HIP(erow.alloc(kMaxExc * 8));
  FMX_HIP(esym.alloc(kMaxExc));
  FMX_HIP(en.alloc(4));
  FMX_HIP(bad.alloc(4));
  FMX_HIP(hipMemsetAsync(en.p, 0, 4, st));
  k_locc_pack<<<grid_for(nl, kBlk, 16384), kBlk, 0, st>>>(
      bwt, n, map, nl, static_cast<uint32_t*>(h->d_lines), cnt.as<uint32_t>(),
      erow.as<unsigned long long>(), esym.as<uint8_t>(), en.as<unsigned int>());
  FMX_HIP(hipGetLastError());
  size_t tb = 0;
  FMX_HIP(rocprim::exclusive_scan(nullptr, tb, cnt.as<uint32_t>(), base.as<uint64_t>(), (uint64_t)0,
                                  nl, rocprim::plus<uint64_t>(), st));
  FMX_HIP(tmp.alloc(tb));
  for (int j = 0; j < 3; ++j) {
    size_t t2 = tb;
    FMX_HIP(rocprim::exclusive_scan(tmp.p, t2, cnt.as<uint32_t>() + (uint64_t)j * nl,
                                    base.as<uint64_t>() + (uint64_t)j * nl, (uint64_t)0, nl,
                                    rocprim::plus<uint64_t>(), st));
  }
  uint32_t shift = 14;
  if (const char* e = build_opt("CS_FM_LEARNED_SHIFT")) shift = (uint32_t)std::atoi(e);
  for (;;) {
    const uint64_t nsb = ((nl - 1) >> shift) + 1;
    if (h->d_lmodel) (void)hipFree(h->d_lmodel);
    FMX_HIP(hipMalloc(&h->d_lmodel, nsb * sizeof(LOccModel)));
    FMX_HIP(hipMemsetAsync(bad.p, 0, 4, st));
    for (int j = 0; j < 3; ++j) {
      const uint64_t* bj = base.as<uint64_t>() + (uint64_t)j * nl;
      k_locc_model<<<grid_for(nsb, kBlk, 16384), kBlk, 0, st>>>(
          bj, nl, shift, nsb, j, static_cast<LOccModel*>(h->d_lmodel));
      k_locc_resid<<<grid_for(nl, kBlk, 16384), kBlk, 0, st>>>(
          static_cast<uint32_t*>(h->d_lines), bj, nl, shift,
          static_cast<const LOccModel*>(h->d_lmodel), j, bad.as<unsigned int>());
      FMX_HIP(hipGetLastError());
    }
    unsigned int b = 0;
    FMX_HIP(hipMemcpyAsync(&b, bad.p, 4, hipMemcpyDeviceToHost, st));
    FMX_HIP(hipStreamSynchronize(st));
    h->nlmodel = nsb;
    h->lmodel_shift = shift;
    if (!b) break;
    if (shift <= 8) {
      set_error("learned occurrence lines: residual overflow");
      return CS_ERR_INVALID;
    }
    shift = 8;
  }
  unsigned int ne = 0;
  uint64_t rows[kMaxExc];
  uint8_t syms[kMaxExc];
  FMX_HIP(hipMemcpyAsync(&ne, en.p, 4, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipMemcpyAsync(rows, erow.p, sizeof rows, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipMemcpyAsync(syms, esym.p, sizeof syms, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  if (ne > (unsigned)kMaxExc) {
    set_error("occurrence lines: rare-symbol rows exceed the table");
    return CS_ERR_INVALID;
  }
  std::vector<int> idx(ne);
  for (unsigned i = 0; i < ne; ++i) idx[i] = (int)i;
  std::sort(idx.begin(), idx.end(), [&](int x, int y) { return rows[x] < rows[y]; });
  NodeTable& T = h->h_table;
  T.exc_n = ne;
  for (unsigned i = 0; i < ne; ++i) {
    T.exc_row[i] = rows[idx[i]];
    T.exc_sym[i] = syms[idx[i]];
  }
  return CS_OK;
}

cs_status build_occ(const uint8_t* bwt, uint64_t n, const CodeMap& map, cs_fm_index* h,
                    hipStream_t st) {
  const uint64_t nl = h->nlines;
  FMX_HIP(hipMalloc(&h->d_lines, nl * OccLine::kBytes));
  DevBuf cnt, base, tmp, erow, esym, en;
  FMX_HIP(cnt.alloc(3 * nl * 4));
  FMX_HIP(base.alloc(nl * 8));
  FMX_HIP(erow.alloc(kMaxExc * 8));
  FMX_HIP(esym.alloc(kMaxExc));
  FMX_HIP(en.alloc(4));
  FMX_HIP(hipMemsetAsync(en.p, 0, 4, st));
  k_occ_pack<<<grid_for(nl, kBlk, 16384), kBlk, 0, st>>>(
      bwt, n, map, nl, static_cast<uint32_t*>(h->d_lines), cnt.as<uint32_t>(),
      erow.as<unsigned long long>(), esym.as<uint8_t>(), en.as<unsigned int>());
  FMX_HIP(hipGetLastError());
  size_t tb = 0;
  FMX_HIP(rocprim::exclusive_scan(nullptr, tb, cnt.as<uint32_t>(), base.as<uint64_t>(), (uint64_t)0,
                                  nl, rocprim::plus<uint64_t>(), st));
  FMX_HIP(tmp.alloc(tb));
  for (int j = 0; j < 3; ++j) {
    size_t t2 = tb;
    FMX_HIP(rocprim::exclusive_scan(tmp.p, t2, cnt.as<uint32_t>() + (uint64_t)j * nl,
                                    base.as<uint64_t>(), (uint64_t)0, nl,
                                    rocprim::plus<uint64_t>(), st));
    k_occ_base<<<grid_for(nl, kBlk, 16384), kBlk, 0, st>>>(static_cast<uint32_t*>(h->d_lines),
                                                          base.as<uint64_t>(), nl, j);
    FMX_HIP(hipGetLastError());
  }
  unsigned int ne = 0;
  uint64_t rows[kMaxExc];
  uint8_t syms[kMaxExc];
  FMX_HIP(hipMemcpyAsync(&ne, en.p, 4, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipMemcpyAsync(rows, erow.p, sizeof rows, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipMemcpyAsync(syms, esym.p, sizeof syms, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  if (ne > (unsigned)kMaxExc) {
    set_error("occurrence lines: rare-symbol rows exceed the table");
    return CS_ERR_INVALID;
  }
  std::vector<int> idx(ne);
  for (unsigned i = 0; i < ne; ++i) idx[i] = (int)i;
  std::sort(idx.begin(), idx.end(), [&](int x, int y) { return rows[x] < rows[y]; });
  NodeTable& T = h->h_table;
  T.exc_n = ne;
  for (unsigned i = 0; i < ne; ++i) {
    T.exc_row[i] = rows[idx[i]];
    T.exc_sym[i] = syms[idx[i]];
  }
  return CS_OK;
}

// ---- walk lines (fm_device.hpp WalkLine / WalkLineW) ----
// position marks: bit isa[k] for every sampled text position k*pstride
__global__ void k_mark_positions(const void* __restrict__ isa, uint64_t nisa, uint32_t wide,
                                 unsigned int* __restrict__ bits) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < nisa; k += stride) {
    const uint64_t r = wide ? static_cast<const uint64_t*>(isa)[k] : static_cast<const uint32_t*>(isa)[k];
    atomicOr(&bits[r >> 5], 1u << (r & 31));
  }
}

// One thread per walk line: codes (rare symbols as code 0), marks (from the bitmap,
// or row % stride == 0 when bits == null), per-line counts of codes 0..2 and marks.
template <class W>
__global__ void k_walk_pack(const uint8_t* __restrict__ bwt, uint64_t n, CodeMap map, uint64_t nw,
                            const unsigned int* __restrict__ bits, uint32_t stride,
                            uint32_t* __restrict__ lines, uint8_t* __restrict__ cnt) {
  __shared__ uint8_t code[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) code[i] = map.c[i];
  __syncthreads();
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < nw; q += gs) {
    const uint64_t a = q * W::kRows;
    uint64_t codes0 = 0, codes1 = 0, marks = 0;
    uint32_t c0 = 0, c1 = 0, c2 = 0, cm = 0;
    for (uint32_t r = 0; r < W::kRows && a + r < n; ++r) {
      const uint64_t row = a + r;
      uint32_t k = code[bwt[row]];
      if (k == kNoCode) k = 0;
      const bool mk = bits ? ((bits[row >> 5] >> (row & 31)) & 1u) : (row % stride == 0);
      if (r < 32) codes0 |= (uint64_t)k << (2 * r);
      else codes1 |= (uint64_t)k << (2 * (r - 32));
      marks |= (uint64_t)mk << r;
      c0 += k == 0;
      c1 += k == 1;
      c2 += k == 2;
      cm += mk;
    }
    uint32_t* L = lines + q * 8;
    if (W::kRows == 42) {  // WalkLine
      const uint64_t hi = codes1 | (marks << 20);
      L[4] = (uint32_t)codes0;
      L[5] = (uint32_t)(codes0 >> 32);
      L[6] = (uint32_t)hi;
      L[7] = (uint32_t)(hi >> 32);
    } else {  // WalkLineW
      L[4] = 0;
      L[5] = (uint32_t)codes0;
      L[6] = (uint32_t)(codes0 >> 32);
      L[7] = (uint32_t)marks;
    }
    cnt[q] = (uint8_t)c0;
    cnt[nw + q] = (uint8_t)c1;
    cnt[2 * nw + q] = (uint8_t)c2;
    cnt[3 * nw + q] = (uint8_t)cm;
  }
}

// field j (occ of code 0..2, 3 = marks) of every walk line = base[q]
template <class W>
__global__ void k_walk_base(uint32_t* __restrict__ lines, const uint64_t* __restrict__ base,
                            uint64_t nw, int j) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < nw; q += gs) {
    const uint64_t b = base[q];
    lines[q * 8 + j] = (uint32_t)b;
    if (W::kRows != 42) reinterpret_cast<uint8_t*>(lines)[q * 32 + 16 + j] = (uint8_t)(b >> 32);
  }
}

// position samples in mark order: wssa[mark_rank(isa[k])] = k * pstride; EB = bytes per
// entry (4, or 5: 40-bit little-endian entries, written byte by byte — entries are disjoint)
template <class W, class SampleT, int EB>
__global__ void k_walk_samples(const SampleT* __restrict__ isa, uint64_t nisa, uint32_t pstride,
                               const void* __restrict__ lines, void* __restrict__ wssa) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < nisa; k += gs) {
    uint64_t q;
    uint32_t o;
    W::locate((uint64_t)isa[k], q, o);
    typename W::Raw v;
    W::load(lines, q, v);
    const uint64_t i = W::mark_rank(v, o), val = k * pstride;
    if constexpr (EB == 5) {
      uint8_t* b = static_cast<uint8_t*>(wssa) + 5 * i;
#pragma unroll
      for (int j = 0; j < 5; ++j) b[j] = (uint8_t)(val >> (8 * j));
    } else {
      static_cast<uint32_t*>(wssa)[i] = (uint32_t)val;
    }
  }
}

template <class W>
cs_status build_walk_t(const uint8_t* bwt, uint64_t n, const CodeMap& map, bool pos_marks,
                       cs_fm_index* h, hipStream_t st) {
  const uint64_t nw = n / W::kRows + 1;
  h->nwalk = nw;
  FMX_HIP(hipMalloc(&h->d_walk, nw * W::kBytes));
  FMX_HIP(hipMemsetAsync(h->d_walk, 0, nw * W::kBytes, st));
  DevBuf bits, cnt, base, tmp;
  if (pos_marks) {
    const uint64_t words = (n >> 5) + 1;
    FMX_HIP(bits.alloc(words * 4));
    FMX_HIP(hipMemsetAsync(bits.p, 0, words * 4, st));
    k_mark_positions<<<grid_for(h->nisa, kBlk, 16384), kBlk, 0, st>>>(
        h->d_isa, h->nisa, h->wide ? 1u : 0u, bits.as<unsigned int>());
    FMX_HIP(hipGetLastError());
  }
  FMX_HIP(cnt.alloc(4 * nw));
  FMX_HIP(base.alloc(nw * 8));
  k_walk_pack<W><<<grid_for(nw, kBlk, 16384), kBlk, 0, st>>>(
      bwt, n, map, nw, pos_marks ? bits.as<unsigned int>() : nullptr, h->stride,
      static_cast<uint32_t*>(h->d_walk), cnt.as<uint8_t>());
  FMX_HIP(hipGetLastError());
  size_t tb = 0;
  FMX_HIP(rocprim::exclusive_scan(nullptr, tb, cnt.as<uint8_t>(), base.as<uint64_t>(), (uint64_t)0,
                                  nw, rocprim::plus<uint64_t>(), st));
  FMX_HIP(tmp.alloc(tb));
  for (int j = 0; j < 4; ++j) {
    size_t t2 = tb;
    FMX_HIP(rocprim::exclusive_scan(tmp.p, t2, cnt.as<uint8_t>() + (uint64_t)j * nw,
                                    base.as<uint64_t>(), (uint64_t)0, nw,
                                    rocprim::plus<uint64_t>(), st));
    k_walk_base<W><<<grid_for(nw, kBlk, 16384), kBlk, 0, st>>>(static_cast<uint32_t*>(h->d_walk),
                                                              base.as<uint64_t>(), nw, j);
    FMX_HIP(hipGetLastError());
  }
  if (pos_marks) {
    h->nwssa = h->nisa;
    h->wssa_eb = h->wide ? 5u : 4u;  // positions < 2^40 (n < 2^38)
    FMX_HIP(hipMalloc(&h->d_wssa, h->nisa * h->wssa_eb + kPartPad));  // + the dword past the last entry
    if (h->wide)
      k_walk_samples<W, uint64_t, 5><<<grid_for(h->nisa, kBlk, 16384), kBlk, 0, st>>>(
          static_cast<const uint64_t*>(h->d_isa), h->nisa, h->pstride, h->d_walk, h->d_wssa);
    else
      k_walk_samples<W, uint32_t, 4><<<grid_for(h->nisa, kBlk, 16384), kBlk, 0, st>>>(
          static_cast<const uint32_t*>(h->d_isa), h->nisa, h->pstride, h->d_walk, h->d_wssa);
    FMX_HIP(hipGetLastError());
  }
  FMX_HIP(hipStreamSynchronize(st));
  return CS_OK;
}

// Walk lines for the occurrence engine (codes) or the quaternary matrix (level-0
// digits; `map` gives each symbol's 2-bit value).  Position marks need LF to be one n-cycle
// (lf_exact) so that every walk ends at a sampled text position; otherwise the
// reference's row marks (row % stride == 0) keep its overrun behaviour.
cs_status build_walk(const uint8_t* bwt, uint64_t n, const CodeMap& map, cs_fm_index* h,
                     hipStream_t st) {
  // with the full suffix array kept (lf_exact), locate reads SA[row] and never walks:
  // no walk lines (C4: 3 GB + 4 GB of position samples saved)
  if (h->d_sa && h->lf_exact && !build_opt("CS_FM_WALK_MARKS")) {
    h->walk_marks = 0;
    return CS_OK;
  }
  bool pos_marks = h->lf_exact && h->d_isa && h->nisa == (n + h->pstride - 1) / h->pstride;
  if (const char* e = build_opt("CS_FM_WALK_MARKS"))  // test hook: "row" forces row marks
    if (std::string(e) == "row") pos_marks = false;
  const uint64_t rows = h->wide ? WalkLineW::kRows : WalkLine::kRows;
  if (!hbm_room(h, (n / rows + 1) * 32 + (pos_marks ? h->nisa * (h->wide ? 5u : 4u) : 0))) {
    h->walk_marks = 0;  // locate walks over the rank structure instead
    return CS_OK;
  }
  h->walk_marks = pos_marks ? 2u : 1u;
  return h->wide ? build_walk_t<WalkLineW>(bwt, n, map, pos_marks, h, st)
                 : build_walk_t<WalkLine>(bwt, n, map, pos_marks, h, st);
}

// R[] of the node table: rank1 at every binary wavelet node's start, or the
// quaternary matrix's occ of the pure digit at its pure nodes' starts.
cs_status launch_node_ranks(const cs_fm_index* h, uint64_t* d_R, hipStream_t st) {
  FMX_HIP(hipMemsetAsync(d_R, 0, kNodes * 8, st));
  if (h->line_fmt == kFmtOcc || h->line_fmt == kFmtLOcc) return CS_OK;  // no wavelet nodes
  if (h->line_fmt == kFmtQwm)
    k_qnode_rank<<<1, 128, 0, st>>>(h->d_lines, h->nlines, h->d_table, d_R);
  else if (h->line_fmt == kFmtLine32)
    k_node_rank<Line32><<<1, kBlk, 0, st>>>(h->d_lines, h->nlines, h->d_table, d_R);
  else if (h->line_fmt == kFmtLine32W)
    k_node_rank<Line32W><<<1, kBlk, 0, st>>>(h->d_lines, h->nlines, h->d_table, d_R);
  else
    k_node_rank<Line64><<<1, kBlk, 0, st>>>(h->d_lines, h->nlines, h->d_table, d_R);
  FMX_HIP(hipGetLastError());
  return CS_OK;
}

}  // namespace fmx
