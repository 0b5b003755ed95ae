// fm_structs.hip — the index structures the staged searches read, built on the GPU from
// the rank lines: the k-mer prefix table, left contexts, k-mer context records, locate
// records and the 2-bit / byte text kept in HBM.  Split out of fm_query.hip
// in round 6; the search helpers they share are in fm_search.hpp.
#include "fm_search.hpp"

namespace fmx {
namespace {

// Prefix table entry t: backward search of the k-mer whose j-th character from
// the end is sym[digit_j(t)] (same steps as above, from C[]).
template <class E>
__global__ __launch_bounds__(kBlk) void k_build_ptab(DevIndex ix, uint64_t entries,
                                                     void* __restrict__ tab, uint64_t wmax) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < entries; t += stride) {
    uint64_t rest = t;
    uint32_t c = T.sym[rest % ix.ptab_sigma];
    rest /= ix.ptab_sigma;
    uint64_t sp = T.C[c], ep = T.C[c + 1];
    bool live = sp < ep;
    for (uint32_t j = 1; j < ix.ptab_k && live; ++j) {
      c = T.sym[rest % ix.ptab_sigma];
      rest /= ix.ptab_sigma;
      live = E::step(ix, T, c, sp, ep);
    }
    if (!live) sp = ep = 0;
    if (ix.wide)  // packed (sp, width), widths >= wmax escaped (fm_device.hpp ptab_at)
      static_cast<uint64_t*>(tab)[t] = ep - sp >= wmax ? kPtabEsc << 38 : sp | ((ep - sp) << 38);
    else
      static_cast<uint2*>(tab)[t] = make_uint2((uint32_t)sp, (uint32_t)ep);
  }
}

// Left contexts (fm_device.hpp kCtxQ): row r follows its LF chain q steps (the
// first line read is shared by neighbouring lanes, the rest are random).
template <class E>
__global__ __launch_bounds__(kBlk) void k_build_lctx(DevIndex ix,
                                                     typename E::CtxEnt* __restrict__ out) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  constexpr bool kEsc = sizeof(typename E::CtxEnt) == 2;
  const uint32_t q = ix.lctx_q, sb = ix.lctx_sb;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < ix.n; r += stride) {
    uint64_t p = r;
    uint32_t v = 0;
    for (uint32_t t = 0; t < q; ++t) {
      uint32_t c;
      p = E::lf(ix, T, p, &c);
      const uint32_t d = T.occ_code[c];
      v |= (kEsc && d == kNoCode) ? kCtxEsc : d << (sb * t);
    }
    out[r] = (typename E::CtxEnt)v;
  }
}

}  // namespace

// Prefix table over the frequent alphabet: symbols with at least n/2^20
// occurrences (all present symbols for small texts), k = largest with
// sigma^k <= min(2^32, max(4096, n/2)) entries of 8 B (at most 4n bytes, capped at
// 32 GiB); none when k < 2.  Each character in the table saves one dependent random
// line read per query, and HBM (288 GB) is not the constraint: C4 k = 14 -> 15 is
// +14 % count rate; C5 k = 15 -> 16 leaves a range of ~7 rows instead of ~30 for the
// left contexts.  DNA: k = 12 at 100 MB, 15 at 4 GB, 16 at 32 GB.  Entries are (sp, ep)
// as 2 x u32, or packed (sp, width) in wide indexes (fm_device.hpp ptab_at).
// CS_FM_PREFIX_K overrides k (0 = off); CS_FM_PTAB_WMAX lowers the escape width (test
// hook).
cs_status build_prefix_table(cs_fm_index* h, hipStream_t st) {
  NodeTable& T = h->h_table;
  std::memset(T.code, kNoCode, sizeof T.code);
  std::memset(T.sym, 0, sizeof T.sym);
  h->ptab_k = 0;
  h->ptab_sigma = 0;
  const uint64_t n = h->n;
  if (n == 0) return CS_OK;
  uint32_t sigma = 0;
  for (int c = 0; c < 256; ++c) {
    const uint64_t f = T.C[c + 1] - T.C[c];
    if (f && f * (1ull << 20) >= n) {
      T.code[c] = (uint8_t)sigma;
      T.sym[sigma++] = (uint8_t)c;
    }
  }
  if (sigma == 0) return CS_OK;
  // Entries: at most n for DNA-like alphabets (sigma <= 4; C2 k = 13, C4 k = 15), 8n for
  // larger ones, where a table character saves a multi-level step (C3, sigma = 256:
  // k = 4, 2^32 entries, 34 GB: 2x the count rate of k = 3); at most 2^32, and the
  // table leaves an eighth of HBM free.
  uint64_t cap = sigma <= 4 ? n : 8 * n;
  if (cap < 4096) cap = 4096;
  if (cap > (1ull << 32)) cap = 1ull << 32;
  size_t free_b = 0, total_b = 0;
  FMX_HIP(hipMemGetInfo(&free_b, &total_b));
  uint64_t budget = free_b > total_b / 8 ? (free_b - total_b / 8) / 8 : 0;
  if (h->hbm_budget) {  // the index's HBM budget: the largest table that still fits it
    const uint64_t have = index_hbm_bytes(h);
    const uint64_t left = h->hbm_budget > have ? (h->hbm_budget - have) / h->ptab_entry_bytes() : 0;
    if (left < budget) budget = left;
    if (cap > budget) cap = budget;
  }
  if (cap > budget && budget >= 4096) cap = budget;
  uint32_t k = 0;
  uint64_t entries = 1;
  while (k < 32 && entries * sigma <= cap) {
    entries *= sigma;
    ++k;
  }
  if (const char* e = build_opt("CS_FM_PREFIX_K")) {
    const int want = std::atoi(e);
    k = 0;
    entries = 1;
    while ((int)k < want && entries * sigma <= (1ull << 32)) {
      entries *= sigma;
      ++k;
    }
  }
  if (k < 2 || sigma < 2) {
    std::memset(T.code, kNoCode, sizeof T.code);
    return CS_OK;
  }
  FMX_HIP(hipMemcpyAsync(h->d_table, &T, sizeof T, hipMemcpyHostToDevice, st));
  FMX_HIP(hipMalloc(&h->d_ptab, entries * h->ptab_entry_bytes()));
  h->ptab_sigma = sigma;
  h->ptab_k = k;
  DevIndex ix = h->dev();
  ix.ptab = nullptr;  // the builder itself searches from C[]
  uint64_t wmax = kPtabEsc;
  if (const char* e = build_opt("CS_FM_PTAB_WMAX")) wmax = std::strtoull(e, nullptr, 10);
  FMX_DISPATCH(h, k_build_ptab, grid_for(entries, kBlk, 65536), ix, entries, h->d_ptab, wmax);
  FMX_HIP(hipStreamSynchronize(st));
  return CS_OK;
}

// Left contexts: u16 per row over occurrence lines (2n bytes; C4 8 GB), u32 over the
// quaternary matrix (4n bytes; C3 4 GB); rows rounded up to whole 32-B sectors plus
// one pad sector.  Skipped (count steps through the rank structure instead) for the
// binary wavelet matrix, when CS_FM_LCTX=0, or when HBM is short: the index must
// leave an eighth of the device free (36 GB on MI355X) for the query buffers.
cs_status build_left_contexts(cs_fm_index* h, hipStream_t st) {
  h->d_lctx = nullptr;
  h->nlctx = 0;
  h->lctx_q = h->lctx_sb = h->lctx_eb = 0;
  const bool occ = h->line_fmt == kFmtOcc || h->line_fmt == kFmtLOcc, qwm = h->line_fmt == kFmtQwm;
  if (!(occ || qwm) || h->n == 0) return CS_OK;
  if (const char* e = build_opt("CS_FM_LCTX"))
    if (std::atoi(e) == 0) return CS_OK;
  const uint32_t eb = occ ? 2 : 4, R = 32 / eb;
  const uint32_t sb = occ ? 2 : 2 * h->h_table.qlevels;
  const uint32_t q = occ ? kCtxQ : (32 / sb < 16 ? 32 / sb : 16);
  const uint64_t rows = ((h->n + R - 1) & ~(uint64_t)(R - 1)) + R;
  if (!hbm_room(h, rows * eb)) return CS_OK;
  FMX_HIP(hipMalloc(&h->d_lctx, rows * eb));
  h->nlctx = rows;
  h->lctx_q = q;
  h->lctx_sb = sb;
  h->lctx_eb = eb;
  FMX_HIP(hipMemsetAsync(static_cast<uint8_t*>(h->d_lctx) + h->n * eb, 0, (rows - h->n) * eb, st));
  const DevIndex ix = h->dev();
  if (h->line_fmt == kFmtLOcc)
    k_build_lctx<LOccE><<<grid_for(h->n, kBlk, 65536), kBlk, 0, st>>>(
        ix, static_cast<uint16_t*>(h->d_lctx));
  else if (occ)
    k_build_lctx<OccE><<<grid_for(h->n, kBlk, 65536), kBlk, 0, st>>>(
        ix, static_cast<uint16_t*>(h->d_lctx));
  else
    k_build_lctx<QWM><<<grid_for(h->n, kBlk, 65536), kBlk, 0, st>>>(
        ix, static_cast<uint32_t*>(h->d_lctx));
  FMX_HIP(hipGetLastError());
  FMX_HIP(hipStreamSynchronize(st));
  return CS_OK;
}

// Context records (fm_device.hpp kRecCtx) from the 8-B table and the left contexts:
// one lane per k-mer.
__global__ __launch_bounds__(kBlk) void k_fill_records(const uint2* __restrict__ tab,
                                                       uint64_t entries,
                                                       const uint16_t* __restrict__ lctx,
                                                       uint32_t* __restrict__ rec) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < entries; t += gs) {
    const uint2 e = tab[t];
    const uint32_t w = e.y - e.x;
    uint32_t d[6] = {0, 0, 0, 0, 0, 0};
    for (uint32_t i = 0; i < kRecCtx && i < w; ++i) d[i >> 1] |= (uint32_t)lctx[e.x + i] << (16 * (i & 1));
    uint4* r = reinterpret_cast<uint4*>(rec) + t * 2;
    r[0] = make_uint4(e.x, w, d[0], d[1]);
    r[1] = make_uint4(d[2], d[3], d[4], d[5]);
  }
}

// Compact 16-B records (fm_device.hpp kRec16Ctx): the width inline when at most
// kRec16Ctx rows and no row's context is escaped, else kRec16Wide and the width.
__global__ __launch_bounds__(kBlk) void k_fill_records16(const uint2* __restrict__ tab,
                                                         uint64_t entries,
                                                         const uint16_t* __restrict__ lctx,
                                                         uint4* __restrict__ rec) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < entries; t += gs) {
    const uint2 e = tab[t];
    const uint32_t w = e.y - e.x;
    bool esc = false;
    uint64_t lo = 0;
    uint32_t hi = 0;
    for (uint32_t i = 0; i < kRec16Ctx && i < w; ++i) {
      const uint32_t c = lctx[e.x + i];
      esc |= (c & kCtxEsc) != 0;
      if (i < 6)
        lo |= (uint64_t)(c & 0x3FFu) << (4 + 10 * i);
      else
        hi |= (c & 0x3FFu) << (10 * (i - 6));
    }
    if (w <= kRec16Ctx && !esc) {
      rec[t] = make_uint4(e.x, (uint32_t)lo | w, (uint32_t)(lo >> 32), hi);
      continue;
    }
    // a wide range: its two most frequent contexts (Misra-Gries with two counters finds every
    // context above a third of the rows; a second pass counts the candidates exactly)
    uint32_t y = kRec16Wide, w3 = 0;
    if (!esc && w > kRec16Ctx && w <= kRec16MajScan) {
      uint32_t ca = 0, cb = 0, na = 0, nb = 0;
      for (uint32_t i = 0; i < w && !esc; ++i) {
        const uint32_t c = lctx[e.x + i];
        esc |= (c & kCtxEsc) != 0;
        const uint32_t v = c & 0x3FFu;
        if (na && v == ca) ++na;
        else if (nb && v == cb) ++nb;
        else if (!na) ca = v, na = 1;
        else if (!nb) cb = v, nb = 1;
        else --na, --nb;
      }
      uint32_t xa = 0, xb = 0;
      for (uint32_t i = 0; i < w && !esc; ++i) {
        const uint32_t v = lctx[e.x + i] & 0x3FFu;
        xa += na && v == ca;
        xb += nb && v == cb;
      }
      if (!esc && na && xb > xa) {  // A the more frequent
        const uint32_t tc = ca; ca = cb; cb = tc;
        const uint32_t tx = xa; xa = xb; xb = tx;
      }
      if (!esc && xa && xa <= 0xFFFFu && xb <= 0xFFFFu) {
        y |= kRec16Maj | (ca << 6) | (xb ? cb << 16 : 0u);
        if (xa + xb == w) y |= kRec16MajAll;
        w3 = xa | (xb << 16);
      }
    }
    rec[t] = make_uint4(e.x, y, w, w3);
  }
}

// Compact records of a wide index from its packed 8-B table (fm_device.hpp kRec16CtxW):
// 4-character contexts of rows 0-9, bits 32-37 of sp in dword 3.
__global__ __launch_bounds__(kBlk) void k_fill_records16_wide(const uint64_t* __restrict__ tab,
                                                              uint64_t entries,
                                                              const uint16_t* __restrict__ lctx,
                                                              uint4* __restrict__ rec) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < entries; t += gs) {
    const uint64_t e = tab[t], w = e >> 38, sp = e & ((1ull << 38) - 1);
    const uint32_t sph = (uint32_t)(sp >> 32) << 24;
    if (w == kPtabEsc) {  // the 8-B table escaped this range: the search starts from C[]
      rec[t] = make_uint4(0u, kRec16Wide, kRec16NoRange, 0u);
      continue;
    }
    bool esc = false;
    uint32_t y = 0, z = 0, x3 = 0;
    for (uint32_t i = 0; i < kRec16CtxW && i < w; ++i) {
      const uint32_t c = lctx[sp + i];
      esc |= (c & kCtxEsc) != 0;
      const uint32_t b = c & 0xFFu;
      if (i < 3)
        y |= b << (4 + 8 * i);
      else if (i < 7)
        z |= b << (8 * (i - 3));
      else
        x3 |= b << (8 * (i - 7));
    }
    if (w > kRec16CtxW || esc)
      rec[t] = make_uint4((uint32_t)sp, kRec16Wide, (uint32_t)w, sph);
    else
      rec[t] = make_uint4((uint32_t)sp, y | (uint32_t)w, z, x3 | sph);
  }
}

// Quaternary-matrix records (fm_device.hpp kRecQCtx): sp, width, contexts of rows 0-1.
__global__ __launch_bounds__(kBlk) void k_fill_records_q(const uint2* __restrict__ tab,
                                                         uint64_t entries,
                                                         const uint32_t* __restrict__ lctx,
                                                         uint4* __restrict__ rec) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < entries; t += gs) {
    const uint2 e = tab[t];
    const uint32_t w = e.y - e.x;
    rec[t] = make_uint4(e.x, w, w > 0 && w <= kRecQCtx ? lctx[e.x] : 0u,
                        w > 1 && w <= kRecQCtx ? lctx[e.x + 1] : 0u);
  }
}

// Replace the 8-B prefix table by 32-B context records (narrow occurrence-engine
// indexes with left contexts; C4: 34 GB for k = 15) when HBM allows (an eighth of the
// device stays free) and the table spans at least 13 characters: records pay for
// patterns of k+1 .. k+7 characters (the 20-mers of the DNA configs from k = 13 on:
// C2, k = 13: 2.35e10 patterns/s with records, 1.64e10 without) and cost 4x the plain
// table's reads in bytes otherwise (C2, k = 12: 7.9e9 with records, 9.1e9 without).  CS_FM_CTX_RECORDS=0 keeps the plain table, =1 forces
// records for any k (test hook), =16 forces the compact 16-B records, which replace the
// 32-B ones by default from k = 15 when the table's mean range is at most 4 rows (C4:
// n / 4^15 = 3.7; a range wider than kRec16Ctx rows or a pattern with 6-7 characters
// left after the table then reads its context sector).
cs_status build_context_records(cs_fm_index* h, hipStream_t st) {
  h->ptab_rec = 0;
  if (!h->d_ptab || !h->ptab_k || !h->d_lctx) return CS_OK;
  if (h->wide && h->lctx_eb != 2) return CS_OK;  // wide records: occurrence lines only
  const uint64_t entries = h->ptab_entries();
  if (h->lctx_eb == 4) {  // quaternary matrix: 16-B records when ranges average <= 2 rows
    if (const char* e = build_opt("CS_FM_CTX_RECORDS"))
      if (std::atoi(e) == 0) return CS_OK;
    if (h->n > kRecQCtx * entries) return CS_OK;
    // the records replace the 8-B table
    if (!hbm_room(h, entries * 16, entries * h->ptab_entry_bytes())) return CS_OK;
    void* rq = nullptr;
    FMX_HIP(hipMalloc(&rq, entries * 16));
    k_fill_records_q<<<grid_for(entries, kBlk, 65536), kBlk, 0, st>>>(
        static_cast<const uint2*>(h->d_ptab), entries, static_cast<const uint32_t*>(h->d_lctx),
        static_cast<uint4*>(rq));
    hipError_t eq = hipGetLastError();
    if (eq == hipSuccess) eq = hipStreamSynchronize(st);
    if (eq != hipSuccess) {
      (void)hipFree(rq);
      return hip_fail(eq, "context records");
    }
    FMX_HIP(hipFree(h->d_ptab));
    h->d_ptab = rq;
    h->ptab_rec = 3;
    return CS_OK;
  }
  if (h->lctx_eb != 2) return CS_OK;
  // a record answers patterns of up to k + q characters: q = 7 (32 B) from k = 13 covers
  // the 20-mers of the DNA workloads; the compact q = 5 still does from k = 15
  bool want = h->ptab_k >= 13;
  uint32_t fmt = h->ptab_k >= 15 && h->n <= 4 * entries ? 2 : 1;
  if (h->wide) {  // compact only (sp needs more than 32 bits); ranges averaging <= 8 rows
    want = h->ptab_k >= 15 && h->n <= 8 * entries;
    fmt = 2;
  }
  if (const char* e = build_opt("CS_FM_CTX_RECORDS")) {
    want = std::atoi(e) != 0;
    fmt = h->wide || std::atoi(e) == 16 ? 2 : 1;
  }
  if (!want) return CS_OK;
  const uint64_t bytes = entries * (fmt == 2 ? 16 : 32);
  // the records replace the 8-B table
  if (!hbm_room(h, bytes, entries * h->ptab_entry_bytes())) return CS_OK;
  void* rec = nullptr;
  FMX_HIP(hipMalloc(&rec, bytes));
  if (h->wide)
    k_fill_records16_wide<<<grid_for(entries, kBlk, 65536), kBlk, 0, st>>>(
        static_cast<const uint64_t*>(h->d_ptab), entries, static_cast<const uint16_t*>(h->d_lctx),
        static_cast<uint4*>(rec));
  else if (fmt == 2)
    k_fill_records16<<<grid_for(entries, kBlk, 65536), kBlk, 0, st>>>(
        static_cast<const uint2*>(h->d_ptab), entries, static_cast<const uint16_t*>(h->d_lctx),
        static_cast<uint4*>(rec));
  else
    k_fill_records<<<grid_for(entries, kBlk, 65536), kBlk, 0, st>>>(
        static_cast<const uint2*>(h->d_ptab), entries, static_cast<const uint16_t*>(h->d_lctx),
        static_cast<uint32_t*>(rec));
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    (void)hipFree(rec);
    return hip_fail(e, "context records");
  }
  FMX_HIP(hipFree(h->d_ptab));
  h->d_ptab = rec;
  h->ptab_rec = fmt;
  return CS_OK;
}

// The text in HBM for extract (the reference keeps text_, fm_index.hpp:41): n bytes
// (C4: 4 GB, C5: 32 GB), kept when an eighth of the device stays free;
// CS_FM_DEVICE_TEXT=0 leaves extract to LF inversion from the inverse-SA samples.
cs_status keep_device_text(cs_fm_index* h, const uint8_t* src, bool src_on_device, hipStream_t st) {
  if (!src || !h->n || h->d_dtext) return CS_OK;
  // (round 6: without the byte text, a walk_verify() index still takes the 2-bit text of the
  // build's device text — C5: 8 GB where the 32-GB text does not fit the eighth)
  const uint8_t* dsrc = src_on_device ? src : nullptr;
  if (const char* e = build_opt("CS_FM_DEVICE_TEXT"))
    if (std::atoi(e) == 0) return derive_packed_text(h, st, dsrc);
  if (!hbm_room(h, h->n)) return derive_packed_text(h, st, dsrc);
  FMX_HIP(hipMalloc(&h->d_dtext, h->n + kPartPad));
  FMX_HIP(hipMemsetAsync(static_cast<uint8_t*>(h->d_dtext) + h->n, 0, kPartPad, st));
  FMX_HIP(hipMemcpyAsync(h->d_dtext, src, h->n,
                         src_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
  FMX_HIP(hipStreamSynchronize(st));
  return derive_packed_text(h, st);
}

// The 2-bit text (cs_fm_index::d_ptext): word w holds the occurrence codes of text[32 w,
// 32 w + 32), rare symbols as code 0, their positions appended to `rare` (at most cap, the
// counter counts them all).  A thread per word.
__global__ __launch_bounds__(kBlk) void k_pack_text(const uint8_t* __restrict__ text, uint64_t n,
                                                    const NodeTable* __restrict__ table,
                                                    uint64_t* __restrict__ out, uint64_t nw,
                                                    uint64_t* __restrict__ rare, uint32_t cap,
                                                    unsigned int* __restrict__ nrare) {
  __shared__ uint8_t code[256];
  if (threadIdx.x < 256) code[threadIdx.x] = table->occ_code[threadIdx.x];
  __syncthreads();
  const uint64_t w = blockIdx.x * (uint64_t)kBlk + threadIdx.x;
  if (w >= nw) return;
  const uint64_t* tw = reinterpret_cast<const uint64_t*>(text) + 4 * w;  // the text has kPartPad slack
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint64_t x = tw[c];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t i = 32 * w + 8 * c + b;
      if (i >= n) break;
      const uint32_t d = code[(uint32_t)(x >> (8 * b)) & 0xFFu];
      if (d == kNoCode) {
        const unsigned int e = atomicAdd(nrare, 1u);
        if (e < cap) rare[e] = i;
      } else {
        acc |= (uint64_t)d << (2 * (8 * c + b));
      }
    }
  }
  out[w] = acc;
}

// the last, partial word of the 2-bit text (`len` < 32 characters at text position `at`,
// from a zero-padded copy): one lane
__global__ void k_pack_text_tail(const uint8_t* __restrict__ text, uint64_t len, uint64_t at,
                                 const NodeTable* __restrict__ table, uint64_t* __restrict__ out,
                                 uint64_t* __restrict__ rare, uint32_t cap, unsigned int* __restrict__ nrare) {
  if (threadIdx.x != 0) return;
  uint64_t acc = 0;
  for (uint64_t i = 0; i < len; ++i) {
    const uint32_t d = table->occ_code[text[i]];
    if (d == kNoCode) {
      const unsigned int e = atomicAdd(nrare, 1u);
      if (e < cap) rare[e] = at + i;
    } else {
      acc |= (uint64_t)d << (2 * i);
    }
  }
  *out = acc;
}

// Long patterns are verified against 32 text characters per 8-B word instead of 8
// (k_count_long): n / 4 bytes (C4: 1 GB), for narrow lf_exact occurrence-line indexes that
// keep the full suffix array and the text in HBM (the verification's preconditions), and
// (round 6) for walk_verify() indexes — no full SA, walk lines with text-position marks (C5:
// 8 GB), whose long patterns are verified at their walks' positions — HBM allowing.  Derived
// from the text kept in HBM or, for walk_verify() indexes, from the build's device text
// `src`; rebuilt on open / import rather than saved.  The rare-symbol positions go to d_prare
// (u32, narrow) or d_prare64 (u64, walk_verify()).  CS_FM_PACKED_TEXT=0 (read at build /
// open) leaves it out.
cs_status derive_packed_text(cs_fm_index* h, hipStream_t st, const uint8_t* src) {
  if (h->d_ptext || h->line_fmt != kFmtOcc || !h->lf_exact || !h->n) return CS_OK;
  const bool narrow_sa = h->d_sa && !h->wide && h->n < (1ull << 32);
  const bool walk = h->walk_verify();
  const uint8_t* text = h->d_dtext ? static_cast<const uint8_t*>(h->d_dtext) : src;
  if (!text || !(narrow_sa || walk)) return CS_OK;
  if (narrow_sa && !h->d_dtext) return CS_OK;  // (its verification reads the byte text too)
  if (const char* e = build_opt("CS_FM_PACKED_TEXT"))
    if (std::atoi(e) == 0) return CS_OK;
  const uint64_t nw = (h->n + 31) / 32;
  if (!hbm_room(h, nw * 8, 0, h->d_dtext ? 0 : h->n)) return CS_OK;
  void* pt = nullptr;
  FMX_HIP(hipMalloc(&pt, nw * 8 + kPartPad));
  DevBuf rb;
  if (rb.alloc(kMaxExc * 8 + 8) != hipSuccess) {
    (void)hipFree(pt);
    return hip_fail(hipGetLastError(), "hipMalloc (packed text)");
  }
  unsigned int* d_n = reinterpret_cast<unsigned int*>(rb.as<uint8_t>() + kMaxExc * 8);
  hipError_t e = hipMemsetAsync(d_n, 0, 4, st);
  if (e == hipSuccess && !h->d_dtext) {
    // (the caller's text has no kPartPad slack: the last word is packed from a padded copy)
    const uint64_t full = h->n / 32;
    if (full)
      k_pack_text<<<grid_for(full, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(text, full * 32, h->d_table,
                                                                        static_cast<uint64_t*>(pt), full,
                                                                        rb.as<uint64_t>(), kMaxExc, d_n);
    e = hipGetLastError();
    if (e == hipSuccess && full < nw) {
      DevBuf tail;
      e = tail.alloc(64);
      if (e == hipSuccess) e = hipMemsetAsync(tail.p, 0, 64, st);
      if (e == hipSuccess) e = hipMemcpyAsync(tail.p, text + full * 32, h->n - full * 32, hipMemcpyDeviceToDevice, st);
      if (e == hipSuccess)
        k_pack_text_tail<<<1, 64, 0, st>>>(tail.as<uint8_t>(), h->n - full * 32, full * 32, h->d_table,
                                           static_cast<uint64_t*>(pt) + full, rb.as<uint64_t>(), kMaxExc, d_n);
      if (e == hipSuccess) e = hipGetLastError();
      if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
  } else if (e == hipSuccess) {
    k_pack_text<<<grid_for(nw, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(
        text, h->n, h->d_table, static_cast<uint64_t*>(pt), nw, rb.as<uint64_t>(), kMaxExc, d_n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemsetAsync(static_cast<uint8_t*>(pt) + nw * 8, 0, kPartPad, st);
  unsigned int nr = 0;
  std::vector<uint64_t> pos(kMaxExc);
  if (e == hipSuccess) e = hipMemcpyAsync(&nr, d_n, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(pos.data(), rb.p, kMaxExc * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess || nr > (unsigned)kMaxExc) {  // more rare positions than the list holds
    (void)hipFree(pt);
    return e == hipSuccess ? CS_OK : hip_fail(e, "packed text");
  }
  pos.resize(nr);
  std::sort(pos.begin(), pos.end());
  void* pr = nullptr;
  if (walk) {
    if (hipMalloc(&pr, kMaxExc * 8) != hipSuccess ||
        (nr && hipMemcpy(pr, pos.data(), nr * 8, hipMemcpyHostToDevice) != hipSuccess)) {
      (void)hipFree(pt);
      if (pr) (void)hipFree(pr);
      return hip_fail(hipGetLastError(), "hipMalloc (packed text)");
    }
    h->d_prare64 = pr;
    h->nrare64 = nr;
  } else {
    std::vector<uint32_t> p32(pos.begin(), pos.end());
    if (hipMalloc(&pr, kMaxExc * 4) != hipSuccess ||
        (nr && hipMemcpy(pr, p32.data(), nr * 4, hipMemcpyHostToDevice) != hipSuccess)) {
      (void)hipFree(pt);
      if (pr) (void)hipFree(pr);
      return hip_fail(hipGetLastError(), "hipMalloc (packed text)");
    }
    h->d_prare = pr;
    h->nrare = nr;
  }
  h->d_ptext = pt;
  return CS_OK;
}

// Locate records (fm_device.hpp kLocRec*) of the (k+1)-mers c.x, from the k-mer x's context
// record and left contexts: a lane per k-mer x.  The rows of c.x are the rows r of x whose
// chain starts with c (BWT[r] = c), in order (LF keeps the order of equal symbols); each
// gives SA[r] - 1 (mod n) and its chain shifted by one symbol.  o2d: the table digit of
// occurrence code o in byte o.  A range wider than kLocRecScan rows, or one holding an
// escaped context, makes all four children kLocRecNone (their locates read the context
// record instead); a child with more than kLocRecRows rows is kLocRecNone too.
constexpr uint32_t kLocRecScan = 64;
__global__ __launch_bounds__(kBlk) void k_fill_locrec(const uint4* __restrict__ rec, uint32_t ptab_rec,
                                                      uint64_t entries,
                                                      const uint16_t* __restrict__ lctx,
                                                      const uint32_t* __restrict__ sa, uint64_t n,
                                                      uint32_t o2d, uint4* __restrict__ out) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < entries; t += gs) {
    // a 32-B record (ptab_rec 1): sp and the width, the rows' contexts from lctx (as for a
    // compact record too wide for its inline contexts)
    const uint4 a = ptab_rec == 1 ? make_uint4(rec[2 * t].x, kRec16Wide, rec[2 * t].y, 0u) : rec[t];
    const uint32_t wc = a.y & 15u;
    const bool wide = wc == kRec16Wide;
    const uint64_t sp = a.x;
    const uint32_t w = wide ? a.z : wc;
    bool none = wide && (a.z == kRec16NoRange || a.z > kLocRecScan);
    uint32_t ctx10[kRec16Ctx];  // inline record: the rows' 5-symbol chains
    if (!wide) {
      uint32_t dw[5];
      rec16_contexts(a.y, a.z, a.w, dw);
#pragma unroll
      for (uint32_t i = 0; i < kRec16Ctx; ++i) ctx10[i] = (dw[i >> 1] >> (16 * (i & 1))) & 0x3FFu;
    }
    if (wide && !none)
      for (uint32_t i = 0; i < w; ++i) none |= (lctx[sp + i] & kCtxEsc) != 0;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
      uint32_t c = 0, cx = 0, sv[kLocRecRows] = {0u, 0u, 0u};
      for (uint32_t i = 0; i < w && !none; ++i) {
        const uint32_t e = wide ? lctx[sp + i] : ctx10[i < kRec16Ctx ? i : 0];
        if (((o2d >> (8 * (e & 3u))) & 0xFFu) != d) continue;
        if (c < kLocRecRows) {
          const uint32_t v = sa[sp + i];
          const uint32_t v1 = v ? v - 1u : (uint32_t)(n - 1);
#pragma unroll
          for (uint32_t r = 0; r < kLocRecRows; ++r)
            if (r == c) sv[r] = v1;
          cx |= ((e >> 2) & 0xFFu) << (8 * c);
        }
        ++c;
      }
      out[(uint64_t)d * entries + t] = none || c > kLocRecRows
                                           ? make_uint4(0u, 0u, 0u, kLocRecNone << 24)
                                           : make_uint4(sv[0], sv[1], sv[2], cx | (c << 24));
    }
  }
}

// 64-B locate records (fm_device.hpp kLocRec64*): the record of k-mer t from its context
// record (sp, width, inline contexts) or lctx, and the rows' SA entries
__global__ __launch_bounds__(kBlk) void k_fill_locrec64(const uint4* __restrict__ rec, uint32_t ptab_rec,
                                                        uint64_t entries,
                                                        const uint16_t* __restrict__ lctx,
                                                        const uint32_t* __restrict__ sa,
                                                        uint4* __restrict__ out) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < entries; t += gs) {
    const uint4 a = ptab_rec == 1 ? make_uint4(rec[2 * t].x, kRec16Wide, rec[2 * t].y, 0u) : rec[t];
    const uint32_t wc = a.y & 15u;
    const bool wide = wc == kRec16Wide;
    const uint64_t sp = a.x;
    const uint32_t w = wide ? a.z : wc;
    bool none = w > kLocRec64Rows || (wide && a.z == kRec16NoRange);
    uint32_t ctx10[kRec16Ctx];  // inline record: the rows' 5-symbol chains
    if (!wide) {
      uint32_t dw[5];
      rec16_contexts(a.y, a.z, a.w, dw);
#pragma unroll
      for (uint32_t i = 0; i < kRec16Ctx; ++i) ctx10[i] = (dw[i >> 1] >> (16 * (i & 1))) & 0x3FFu;
    }
    if (wide && !none)
      for (uint32_t i = 0; i < w; ++i) none |= (lctx[sp + i] & kCtxEsc) != 0;
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) {
      uint4 o = make_uint4(~0u, 0u, 0u, 0u);
      if (!none) {
        const uint32_t vc = w > 3 * c ? (w - 3 * c < 3 ? w - 3 * c : 3u) : 0u;
        uint32_t sv[3] = {0u, 0u, 0u}, cx = vc << 30;
        for (uint32_t i = 0; i < vc; ++i) {
          const uint32_t r = 3 * c + i;
          sv[i] = sa[sp + r];
          cx |= (wide ? (uint32_t)lctx[sp + r] & 0x3FFu : ctx10[r < kRec16Ctx ? r : 0]) << (10 * i);
        }
        o = make_uint4(sv[0], sv[1], sv[2], cx);
      }
      out[4 * t + c] = o;
    }
  }
}

// Build the locate records when the index can use them: narrow lf_exact occurrence-line
// indexes with context records (16 B, or 32 B: C2) over a 4-symbol table of k <= 15, the
// left contexts and the full suffix array (C4: k = 15 -> 4^16 records, 69 GB; C2: k = 13 ->
// 4^14, 4.3 GB), HBM allowing (an eighth of the
// device stays free; within CS_FM_HBM_BUDGET).  CS_FM_LOC_RECORDS=0 (read at build / open /
// import) leaves them out.  Derived from the other parts, not saved.
cs_status derive_locate_records(cs_fm_index* h, hipStream_t st) {
  if (h->d_lrec || (h->ptab_rec != 1 && h->ptab_rec != 2) || !h->d_ptab || !h->d_sa || !h->lf_exact || h->wide ||
      !h->d_lctx || h->lctx_eb != 2 || h->line_fmt != kFmtOcc || h->ptab_sigma != 4 ||
      h->ptab_k < 1 || h->ptab_k + 1 > 16 || h->n >= (1ull << 32))
    return CS_OK;
  if (const char* e = build_opt("CS_FM_LOC_RECORDS"))
    if (std::atoi(e) == 0) return CS_OK;
  // the table digit of each occurrence code; every code must have one
  uint32_t o2d = 0xFFFFFFFFu;
  for (int c = 0; c < 256; ++c) {
    const uint32_t oc = h->h_table.occ_code[c], d = h->h_table.code[c];
    if (oc < 4 && d < 4) o2d = (o2d & ~(0xFFu << (8 * oc))) | (d << (8 * oc));
  }
  for (int oc = 0; oc < 4; ++oc)
    if (((o2d >> (8 * oc)) & 0xFFu) >= 4) return CS_OK;
  const uint64_t entries = h->ptab_entries(), bytes = entries * 4 * 16;  // either layout
  if (!hbm_room(h, bytes)) return CS_OK;
  // CS_FM_LOC_REC64=0 (read at build / open / import): the 16-B (k+1)-mer records of early
  // round 4 instead of the 64-B k-mer ones
  bool w64 = true;
  if (const char* e = build_opt("CS_FM_LOC_REC64"))
    w64 = std::atoi(e) != 0;
  void* p = nullptr;
  FMX_HIP(hipMalloc(&p, bytes));
  if (w64)
    k_fill_locrec64<<<grid_for(entries, kBlk, 1u << 20), kBlk, 0, st>>>(
        static_cast<const uint4*>(h->d_ptab), h->ptab_rec, entries, static_cast<const uint16_t*>(h->d_lctx),
        static_cast<const uint32_t*>(h->d_sa), static_cast<uint4*>(p));
  else
    k_fill_locrec<<<grid_for(entries, kBlk, 1u << 20), kBlk, 0, st>>>(
        static_cast<const uint4*>(h->d_ptab), h->ptab_rec, entries, static_cast<const uint16_t*>(h->d_lctx),
        static_cast<const uint32_t*>(h->d_sa), h->n, o2d, static_cast<uint4*>(p));
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    (void)hipFree(p);
    return hip_fail(e, "locate records");
  }
  h->d_lrec = p;
  h->lrec_w = w64 ? 64 : 16;
  return CS_OK;
}

}  // namespace fmx
