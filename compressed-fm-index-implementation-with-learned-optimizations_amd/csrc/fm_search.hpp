// fm_search.hpp — device-side search helpers shared by the query kernels (fm_query.hip)
// and the index-structure builders (fm_structs.hip): the node table in LDS, one
// backward-search step per rank engine, the prefix-table / left-context / record
// lookups and the search loops the kernels are built from, plus the engine dispatch
// macros.  Everything sits in an anonymous namespace: each translation unit
// instantiates the templates it launches.
#pragma once
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>
#include <cstring>
#include <mutex>

#include "fm_internal.hpp"

namespace fmx {
namespace {

constexpr unsigned kBlk = 256;

__device__ __forceinline__ void load_table(NodeTable& T, const NodeTable* __restrict__ g) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&T);
  constexpr int nw = sizeof(NodeTable) / 4;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) dst[i] = src[i];
}

// A 2-bit packed DNA pattern (cs_fm_count_packed_device): character i is code
// (x >> 2i) & 3 of "ACGT".  Indexes like the byte pointer of a byte-string pattern,
// so every search helper takes either (template parameter PT).
constexpr uint32_t kDnaSyms = 0x54474341u;  // 'A' 'C' 'G' 'T', little-endian
struct PackedDna {
  uint64_t x;
  __device__ __forceinline__ uint32_t operator[](uint64_t i) const {
    return (kDnaSyms >> (8u * (uint32_t)((x >> (2 * i)) & 3u))) & 0xFFu;
  }
};


// One backward-search step (fm_index.cpp:90-96) for a symbol c present in the
// text: [sp, ep) -> [C[c] + occ(c, sp), C[c] + occ(c, ep)).  Returns false when
// the range empties (the reference's `return 0`).
template <class F>
__device__ __forceinline__ bool search_step(const DevIndex& ix, const NodeTable& T, uint32_t c,
                                            uint64_t& sp, uint64_t& ep,
                                            uint64_t* bytes = nullptr) {
  const uint64_t Cc = T.C[c];
  if (Cc == T.C[c + 1]) return false;  // symbol absent: occ == 0 on both ends
  uint64_t ds = sp, de = ep;
#pragma unroll
  for (int l = 0; l < kLevels; ++l) {
    const int nid = (1 << l) - 1 + (int)(l ? (c >> (8 - l)) : 0u);
    if (!(T.flags[nid] & kPure)) {
      const uint64_t S = T.S[nid], R = T.R[nid];
      const void* lv = level_ptr<F>(ix, l);
      uint32_t qa, oa, qe, oe;
      F::locate(S + ds, qa, oa);
      F::locate(S + de, qe, oe);
      if (bytes) *bytes += (qa == qe ? 1u : 2u) * F::kBytes;  // distinct lines (measurement)
      typename F::Raw va, ve;
      F::load(lv, qa, va);
#pragma unroll
      for (int k = 0; k < (int)(sizeof(va) / sizeof(va[0])); ++k) ve[k] = va[k];
      if (qe != qa) F::load(lv, qe, ve);  // sp and ep in one line: one read
      const uint64_t rs = F::base(va) + F::prefix(va, oa) - R;
      const uint64_t re = F::base(ve) + F::prefix(ve, oe) - R;
      const bool b = (c >> (7 - l)) & 1u;
      ds = b ? rs : ds - rs;
      de = b ? re : de - re;
    }
  }
  sp = Cc + ds;
  ep = Cc + de;
  return sp < ep;
}

// One LF step (fm_index.hpp:62-66): descend the wavelet matrix from row i reading
// the BWT symbol bit by bit (WaveletTree::access, wavelet.cpp:102-128) while
// mapping i; the leaf offset is rank(c, i).  Pure nodes cost no load.
template <class F>
__device__ __forceinline__ uint64_t lf_step(const DevIndex& ix, const NodeTable& T, uint64_t pos,
                                            uint32_t* sym_out = nullptr) {
  uint32_t x = 0;
#pragma unroll
  for (int l = 0; l < kLevels; ++l) {
    const int nid = (1 << l) - 1 + (int)x;
    const uint8_t f = T.flags[nid];
    uint32_t b;
    uint64_t r;
    if (f & kPure) {
      b = (f & kPureBit) ? 1u : 0u;
      r = T.R[nid] + (b ? pos - T.S[nid] : 0);
    } else {
      uint32_t q, o;
      F::locate(pos, q, o);
      typename F::Raw v;
      F::load(level_ptr<F>(ix, l), q, v);
      b = F::bit(v, o);
      r = F::base(v) + F::prefix(v, o);
    }
    pos = b ? T.Z[l] + r : pos - r;
    x = (x << 1) | b;
  }
  if (sym_out) *sym_out = x;
  return T.C[x] + (pos - T.S8[x]);
}

// ---- rare-symbol rows of the occurrence-line engine (NodeTable::exc_*) ----
// number of exception rows < i (lower bound in the ascending list)
__device__ __forceinline__ uint32_t exc_before(const NodeTable& T, uint64_t i) {
  uint32_t lo = 0, hi = T.exc_n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (T.exc_row[mid] < i) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// occ(c, i) of a rare symbol c
__device__ __forceinline__ uint64_t exc_rank(const NodeTable& T, uint32_t c, uint64_t i) {
  uint64_t r = 0;
  for (uint32_t j = 0; j < T.exc_n && T.exc_row[j] < i; ++j) r += T.exc_sym[j] == c;
  return r;
}

// ---- engines: what the kernels call per backward-search step / LF step / rank ----
// WM<F>: the 8-level wavelet matrix (the reference's WaveletTree) in rank lines F.
template <class F>
struct WM {
  static constexpr bool kCtx = false;  // no left contexts
  using CtxEnt = uint32_t;
  __device__ static __forceinline__ bool step(const DevIndex& ix, const NodeTable& T, uint32_t c,
                                              uint64_t& sp, uint64_t& ep,
                                              uint64_t* bytes = nullptr) {
    return search_step<F>(ix, T, c, sp, ep, bytes);
  }
  __device__ static __forceinline__ uint64_t lf(const DevIndex& ix, const NodeTable& T,
                                                uint64_t pos, uint32_t* sym = nullptr) {
    return lf_step<F>(ix, T, pos, sym);
  }
  // WaveletTree::rank(c, i) (wavelet.cpp:59-96) for 0 < i <= n, c present
  __device__ static __forceinline__ uint64_t rank(const DevIndex& ix, const NodeTable& T,
                                                  uint32_t c, uint64_t i) {
    uint64_t d = i;
    for (int l = 0; l < kLevels; ++l) {
      const int nid = (1 << l) - 1 + (int)(l ? (c >> (8 - l)) : 0u);
      if (!(T.flags[nid] & kPure)) {
        const uint64_t r = rank1_at<F>(level_ptr<F>(ix, l), T.S[nid] + d) - T.R[nid];
        d = ((c >> (7 - l)) & 1u) ? r : d - r;
      }
    }
    return d;
  }
};

// OccE: occurrence lines (fm_device.hpp OccLine).  occ(c, i) = one line read:
// base(code) + rows of that code before i in the line, minus the rare-symbol rows
// below i when c has code 0 (they are stored as code 0); rare symbols are counted
// from the LDS list.  sp and ep in the same line share one read.
struct OccE {
  static constexpr bool kCtx = true;  // left contexts (DevIndex::lctx) when built
  using CtxEnt = uint16_t;
  __device__ static __forceinline__ uint64_t occ_line(const OccLine::Raw& v, uint32_t code,
                                                      uint64_t i) {
    return OccLine::base(v, code, i >> 6) + OccLine::prefix(v, code, (uint32_t)(i & 63));
  }
  __device__ static __forceinline__ bool step(const DevIndex& ix, const NodeTable& T, uint32_t c,
                                              uint64_t& sp, uint64_t& ep,
                                              uint64_t* bytes = nullptr) {
    const uint64_t Cc = T.C[c];
    if (Cc == T.C[c + 1]) return false;  // symbol absent: occ == 0 on both ends
    const uint32_t code = T.occ_code[c];
    uint64_t rs, re;
    if (code == kNoCode) {
      rs = exc_rank(T, c, sp);
      re = exc_rank(T, c, ep);
    } else {
      const uint64_t qa = sp >> 6, qe = ep >> 6;
      if (bytes) *bytes += (qa == qe ? 1u : 2u) * OccLine::kBytes;
      OccLine::Raw va;
      OccLine::load(ix.lines, qa, va);
      OccLine::Raw ve = {va[0], va[1]};
      if (qe != qa) OccLine::load(ix.lines, qe, ve);
      rs = occ_line(va, code, sp);
      re = occ_line(ve, code, ep);
      if (code == 0 && T.exc_n) {
        rs -= exc_before(T, sp);
        re -= exc_before(T, ep);
      }
    }
    sp = Cc + rs;
    ep = Cc + re;
    return sp < ep;
  }
  // LF(i) = C[BWT[i]] + occ(BWT[i], i), symbol and occ from the same line
  __device__ static __forceinline__ uint64_t lf(const DevIndex& ix, const NodeTable& T,
                                                uint64_t pos, uint32_t* sym_out = nullptr) {
    OccLine::Raw v;
    OccLine::load(ix.lines, pos >> 6, v);
    const uint32_t code = OccLine::code(v, (uint32_t)(pos & 63));
    uint32_t c = T.occ_sym[code];
    uint64_t r = occ_line(v, code, pos);
    if (code == 0 && T.exc_n) {
      const uint32_t e = exc_before(T, pos);
      if (e < T.exc_n && T.exc_row[e] == pos) {
        c = T.exc_sym[e];
        r = exc_rank(T, c, pos);
      } else {
        r -= e;
      }
    }
    if (sym_out) *sym_out = c;
    return T.C[c] + r;
  }
  __device__ static __forceinline__ uint64_t rank(const DevIndex& ix, const NodeTable& T,
                                                  uint32_t c, uint64_t i) {
    const uint32_t code = T.occ_code[c];
    if (code == kNoCode) return exc_rank(T, c, i);
    OccLine::Raw v;
    OccLine::load(ix.lines, i >> 6, v);
    uint64_t r = occ_line(v, code, i);
    if (code == 0) r -= exc_before(T, i);
    return r;
  }
};

// LOccE: learned occurrence lines (fm_device.hpp LOccLine), the occurrence engine
// with 104 rows per line.  occ(c, i) = the model's prediction at the line start + the
// line's residual + rows of code c before i in the line (bitvector_learned.cpp:152-203:
// coarse prediction + micro correction + tail popcount); the superblock model is an
// L2-resident read beside the line.  Rare rows as OccE.
struct LOccE {
  static constexpr bool kCtx = true;
  using CtxEnt = uint16_t;
  __device__ static __forceinline__ uint64_t line_of(uint64_t i) { return i / LOccLine::kRows; }
  // occ(code, i) with i in line q
  __device__ static __forceinline__ uint64_t occ_line(const DevIndex& ix, const LOccLine::Raw& v,
                                                      uint32_t code, uint64_t q, uint64_t i) {
    const uint64_t b = q >> ix.lmodel_shift, dq = q - (b << ix.lmodel_shift);
    const LOccModel* m = static_cast<const LOccModel*>(ix.lmodel) + b;
    uint64_t start;
    if (code < 3) {
      start = m->base[code] + ((m->slope[code] * (104ull * dq)) >> 32) + (int64_t)LOccLine::resid(v, code);
    } else {
      start = 104ull * q;
#pragma unroll
      for (uint32_t c = 0; c < 3; ++c)
        start -= m->base[c] + ((m->slope[c] * (104ull * dq)) >> 32) + (int64_t)LOccLine::resid(v, c);
    }
    return start + LOccLine::prefix(v, code, (uint32_t)(i - q * LOccLine::kRows));
  }
  __device__ static __forceinline__ bool step(const DevIndex& ix, const NodeTable& T, uint32_t c,
                                              uint64_t& sp, uint64_t& ep,
                                              uint64_t* bytes = nullptr) {
    const uint64_t Cc = T.C[c];
    if (Cc == T.C[c + 1]) return false;  // symbol absent: occ == 0 on both ends
    const uint32_t code = T.occ_code[c];
    uint64_t rs, re;
    if (code == kNoCode) {
      rs = exc_rank(T, c, sp);
      re = exc_rank(T, c, ep);
    } else {
      const uint64_t qa = line_of(sp), qe = line_of(ep);
      if (bytes) *bytes += (qa == qe ? 1u : 2u) * LOccLine::kBytes;
      LOccLine::Raw va;
      LOccLine::load(ix.lines, qa, va);
      LOccLine::Raw ve = {va[0], va[1]};
      if (qe != qa) LOccLine::load(ix.lines, qe, ve);
      rs = occ_line(ix, va, code, qa, sp);
      re = occ_line(ix, ve, code, qe, ep);
      if (code == 0 && T.exc_n) {
        rs -= exc_before(T, sp);
        re -= exc_before(T, ep);
      }
    }
    sp = Cc + rs;
    ep = Cc + re;
    return sp < ep;
  }
  __device__ static __forceinline__ uint64_t lf(const DevIndex& ix, const NodeTable& T,
                                                uint64_t pos, uint32_t* sym_out = nullptr) {
    const uint64_t q = line_of(pos);
    LOccLine::Raw v;
    LOccLine::load(ix.lines, q, v);
    const uint32_t code = LOccLine::code(v, (uint32_t)(pos - q * LOccLine::kRows));
    uint32_t c = T.occ_sym[code];
    uint64_t r = occ_line(ix, v, code, q, pos);
    if (code == 0 && T.exc_n) {
      const uint32_t e = exc_before(T, pos);
      if (e < T.exc_n && T.exc_row[e] == pos) {
        c = T.exc_sym[e];
        r = exc_rank(T, c, pos);
      } else {
        r -= e;
      }
    }
    if (sym_out) *sym_out = c;
    return T.C[c] + r;
  }
  __device__ static __forceinline__ uint64_t rank(const DevIndex& ix, const NodeTable& T,
                                                  uint32_t c, uint64_t i) {
    const uint32_t code = T.occ_code[c];
    if (code == kNoCode) return exc_rank(T, c, i);
    const uint64_t q = line_of(i);
    LOccLine::Raw v;
    LOccLine::load(ix.lines, q, v);
    uint64_t r = occ_line(ix, v, code, q, i);
    if (code == 0) r -= exc_before(T, i);
    return r;
  }
};

// QWM: quaternary wavelet matrix over dense symbol codes, for alphabets beyond the
// occurrence engine (e.g. sigma = 256: 4 levels instead of 8).  Level l holds digit
// l (2 bits, most significant first) of the level-l sequence as occurrence lines
// (OccLine, 64 rows per 32-B line); the next sequence is the stable 4-way
// partition by that digit.  A position p maps to the next level as
// p' = qZ[l][d] + occ_l(d, p) — one line read — or affinely inside a pure node
// (all its symbols share digit d): p' = qZ[l][d] + R + (p - S).  After the last
// level, occ(c, i) = p_L(i) - S8[code(c)] (the WaveletTree::rank identity,
// wavelet.cpp:59-96, in base 4).
struct QWM {
  static constexpr bool kCtx = true;
  using CtxEnt = uint32_t;
  __device__ static __forceinline__ const void* level(const DevIndex& ix, int l) {
    return static_cast<const uint8_t*>(ix.lines) + (uint64_t)l * ix.nlines * OccLine::kBytes;
  }
  __device__ static __forceinline__ bool step(const DevIndex& ix, const NodeTable& T, uint32_t c,
                                              uint64_t& sp, uint64_t& ep,
                                              uint64_t* bytes = nullptr) {
    const uint64_t Cc = T.C[c];
    if (Cc == T.C[c + 1]) return false;  // symbol absent: occ == 0 on both ends
    const uint32_t x = T.occ_code[c];
    const int L = (int)T.qlevels;
    uint64_t ps = sp, pe = ep;
    for (int l = 0; l < L; ++l) {
      const int nid = qnode_id(l, x >> (2 * (L - l)));
      const uint32_t d = (x >> (2 * (L - 1 - l))) & 3u;
      const uint8_t f = T.flags[nid];
      if (f & kPure) {
        const uint64_t off = T.qZ[l][d] + T.R[nid] - T.S[nid];
        ps += off;
        pe += off;
      } else {
        const void* lv = level(ix, l);
        const uint64_t qa = ps >> 6, qe = pe >> 6;
        if (bytes) *bytes += (qa == qe ? 1u : 2u) * OccLine::kBytes;
        OccLine::Raw va;
        OccLine::load(lv, qa, va);
        OccLine::Raw ve = {va[0], va[1]};
        if (qe != qa) OccLine::load(lv, qe, ve);
        ps = T.qZ[l][d] + OccLine::base(va, d, qa) + OccLine::prefix(va, d, (uint32_t)(ps & 63));
        pe = T.qZ[l][d] + OccLine::base(ve, d, qe) + OccLine::prefix(ve, d, (uint32_t)(pe & 63));
      }
    }
    sp = Cc + (ps - T.S8[x]);
    ep = Cc + (pe - T.S8[x]);
    return sp < ep;
  }
  // LF(i): the digits of BWT[i] and its mapped position, one line per level
  __device__ static __forceinline__ uint64_t lf(const DevIndex& ix, const NodeTable& T,
                                                uint64_t pos, uint32_t* sym_out = nullptr) {
    const int L = (int)T.qlevels;
    uint32_t x = 0;
    uint64_t p = pos;
    for (int l = 0; l < L; ++l) {
      const int nid = qnode_id(l, x);
      const uint8_t f = T.flags[nid];
      uint32_t d;
      if (f & kPure) {
        d = (f >> 2) & 3u;
        p = T.qZ[l][d] + T.R[nid] + (p - T.S[nid]);
      } else {
        OccLine::Raw v;
        const uint64_t q = p >> 6;
        OccLine::load(level(ix, l), q, v);
        const uint32_t o = (uint32_t)(p & 63);
        d = OccLine::code(v, o);
        p = T.qZ[l][d] + OccLine::base(v, d, q) + OccLine::prefix(v, d, o);
      }
      x = (x << 2) | d;
    }
    const uint32_t c = T.qsym[x];
    if (sym_out) *sym_out = c;
    return T.C[c] + (p - T.S8[x]);
  }
  __device__ static __forceinline__ uint64_t rank(const DevIndex& ix, const NodeTable& T,
                                                  uint32_t c, uint64_t i) {
    uint64_t sp = 0, ep = i;
    (void)step(ix, T, c, sp, ep);
    return ep - sp;
  }
};

// Start of a backward search (fm_index.cpp:84-89): the first step from C[]
// (sp = C[c], ep = C[c+1]), or the first k steps from the prefix table when the
// pattern's last k characters are all in its alphabet.  k receives the characters
// still to process (P[k-1] .. P[0]).  Requires m >= 1.
// With context records, *inl receives the entry's contexts (kRecCtx u16 in 6 dwords),
// or the compact record itself (fm_device.hpp kRec16Ctx) when it holds contexts.
// maj: a wide compact record's majority contexts (kRec16Maj), when it holds them.
template <class PT>
__device__ __forceinline__ void search_start(const DevIndex& ix, const NodeTable& T,
                                             PT P, uint64_t m,
                                             uint64_t& sp, uint64_t& ep, uint64_t& k,
                                             uint64_t* bytes, const uint32_t** inl = nullptr,
                                             const uint32_t** maj = nullptr) {
  if (inl) *inl = nullptr;
  if (maj) *maj = nullptr;
  if (ix.ptab_k && m >= ix.ptab_k) {
    uint32_t t = 0;
    bool ok = true;
    for (uint32_t i = (uint32_t)(m - ix.ptab_k); i < m; ++i) {
      const uint32_t d = T.code[P[i]];
      ok &= d != kNoCode;
      t = t * ix.ptab_sigma + d;
    }
    if (ok && ptab_at(ix, t, sp, ep)) {
      if (bytes) *bytes += ix.ptab_rec == 1 ? 32u : ix.ptab_rec >= 2 ? 16u : 8u;
      if (inl && ix.ptab_rec == 3 && ep - sp <= kRecQCtx)
        *inl = static_cast<const uint32_t*>(ix.ptab) + (uint64_t)t * 4 + 2;
      if (inl && ix.ptab_rec == 1) *inl = static_cast<const uint32_t*>(ix.ptab) + (uint64_t)t * 8 + 2;
      if ((inl || maj) && ix.ptab_rec == 2) {
        const uint32_t* r = static_cast<const uint32_t*>(ix.ptab) + (uint64_t)t * 4;
        if ((r[1] & 15u) != kRec16Wide) {
          if (inl) *inl = r;
        } else if (maj && !ix.wide && (r[1] & kRec16Maj)) {
          *maj = r;
        }
      }
      k = m - ix.ptab_k;
      return;
    }
  }
  const uint32_t c = P[m - 1];
  sp = T.C[c];  // occ(c,0)=0, occ(c,n)=freq(c)
  ep = T.C[c + 1];
  k = m - 1;
}

// Backward search of one pattern (fm_index.cpp:84-98).  Returns false when the
// range empties.  Requires m >= 1, n >= 1.
template <class E, class PT>
__device__ __forceinline__ bool backward_search(const DevIndex& ix, const NodeTable& T,
                                                PT P, uint64_t m,
                                                uint64_t& sp_out, uint64_t& ep_out,
                                                uint64_t* bytes = nullptr) {
  uint64_t sp, ep, k;
  search_start(ix, T, P, m, sp, ep, k, bytes);
  if (sp >= ep) return false;
  uint32_t cn = k ? P[k - 1] : 0u;
  while (k-- > 0) {
    const uint32_t c = cn;
    if (k > 0) cn = P[k - 1];  // prefetch the next character
    if (!E::step(ix, T, c, sp, ep, bytes)) return false;
  }
  sp_out = sp;
  ep_out = ep;
  return true;
}

// The last k <= lctx_q characters P[0..k) over the left contexts of the rows
// [sp, ep) (fm_device.hpp kCtxQ): the rows whose chain spells P[k-1], ..., P[0].
// Needs ep - (sp & ~(R-1)) <= 2R, R = rows per 32-B sector (16 for u16 entries, 8
// for u32).  Returns kCtxNone — the caller keeps stepping — when a character has no
// code (a rare symbol) or a row in the range has an escaped context; kCtxAbsent when
// a character does not occur in the text (count 0, as the reference's step);
// otherwise kCtxOk with bit i of `mm` set when row base + i matches.
enum : uint32_t { kCtxNone = 0, kCtxAbsent = 1, kCtxOk = 2 };
// whether a record's inline contexts answer k characters over a w-row range
__device__ __forceinline__ bool rec_inline(const DevIndex& ix, uint64_t k, uint64_t w) {
  return ix.ptab_rec == 2 ? k <= (ix.wide ? kRec16QW : kRec16Q)
                          : ix.ptab_rec == 3 ? w <= kRecQCtx : w <= kRecCtx;
}
// inl: the contexts of a context record whose range [sp, ep) is at most kRecCtx rows
// (already read with the record: no further access), else null.
template <class Ent, class PT>
__device__ __forceinline__ uint32_t ctx_match(const DevIndex& ix, const NodeTable& T,
                                              PT P, uint32_t k,
                                              uint64_t sp, uint64_t ep, uint32_t& mm,
                                              uint64_t& base, uint64_t* bytes,
                                              const uint32_t* inl = nullptr) {
  constexpr uint32_t R = 32 / sizeof(Ent);
  constexpr bool kEsc = sizeof(Ent) == 2;
  const uint32_t sb = kEsc ? 2u : ix.lctx_sb;
  uint32_t want = 0;
  for (uint32_t t = 0; t < k; ++t) {  // chain symbol t = P[k-1-t]
    const uint32_t c = P[k - 1 - t];
    if (T.C[c] == T.C[c + 1]) return kCtxAbsent;
    const uint32_t d = T.occ_code[c];
    // a rare symbol of the occurrence engine; the quaternary matrix codes every present
    // symbol densely (with 256 symbols one of them is code 0xFF == kNoCode)
    if (kEsc && d == kNoCode) return kCtxNone;
    want |= d << (sb * t);
  }
  const uint32_t kb = sb * k;
  const uint32_t mask = (kb >= 32 ? ~0u : ((1u << kb) - 1u)) | (kEsc ? kCtxEsc : 0u);
  uint4 w[4];
  uint32_t lo, hi;  // rows [lo, hi) of the 2R from base
  if (!kEsc && inl) {  // quaternary-matrix record: rows sp, sp+1 (u32 entries)
    base = sp;
    lo = 0;
    hi = (uint32_t)(ep - sp);
    w[0] = make_uint4(inl[0], inl[1], 0, 0);
    w[1] = w[2] = w[3] = make_uint4(0, 0, 0, 0);
  } else if (kEsc && inl) {
    base = sp;
    lo = 0;
    hi = (uint32_t)(ep - sp);
    if (ix.ptab_rec == 2) {
      uint32_t d[5];
      if (ix.wide)
        rec16w_contexts(inl[1], inl[2], inl[3], d);
      else
        rec16_contexts(inl[1], inl[2], inl[3], d);
      w[0] = make_uint4(d[0], d[1], d[2], d[3]);
      w[1] = make_uint4(d[4], 0, 0, 0);
    } else {
      w[0] = make_uint4(inl[0], inl[1], inl[2], inl[3]);
      w[1] = make_uint4(inl[4], inl[5], 0, 0);
    }
    w[2] = w[3] = make_uint4(0, 0, 0, 0);
  } else {
    base = sp & ~(uint64_t)(R - 1);
    lo = (uint32_t)(sp - base);
    hi = (uint32_t)(ep - base);
    const uint4* p = reinterpret_cast<const uint4*>(static_cast<const Ent*>(ix.lctx) + base);
    const bool two = hi > R;
    if (bytes) *bytes += two ? 64u : 32u;
    w[0] = p[0];
    w[1] = p[1];
    if (two) {
      w[2] = p[2];
      w[3] = p[3];
    } else {
      w[2] = w[3] = make_uint4(0, 0, 0, 0);
    }
  }
  const uint32_t* dw = reinterpret_cast<const uint32_t*>(w);
  uint32_t match = 0, esc = 0;  // bit i: row base + i
#pragma unroll
  for (int i = 0; i < (int)(2 * R); ++i) {
    const uint32_t e = kEsc ? (dw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu : dw[i];
    match |= (uint32_t)((e & mask) == want) << i;
    if (kEsc) esc |= (uint32_t)((e & kCtxEsc) != 0) << i;
  }
  const uint32_t in = (hi >= 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
  if (esc & in) return kCtxNone;
  mm = match & in;
  return kCtxOk;
}

template <class Ent, class PT>
__device__ __forceinline__ bool ctx_count(const DevIndex& ix, const NodeTable& T,
                                          PT P, uint32_t k,
                                          uint64_t sp, uint64_t ep, uint64_t& cnt,
                                          uint64_t* bytes, const uint32_t* inl = nullptr) {
  uint32_t mm = 0;
  uint64_t base;
  const uint32_t r = ctx_match<Ent>(ix, T, P, k, sp, ep, mm, base, bytes, inl);
  if (r == kCtxNone) return false;
  cnt = r == kCtxOk ? (uint64_t)__popc(mm) : 0;
  return true;
}

template <class E, class PT, bool kLA = false>
__device__ __forceinline__ uint64_t count_rest(const DevIndex& ix, const NodeTable& T, PT P,
                                               uint64_t k, uint64_t sp, uint64_t ep,
                                               uint64_t* bytes, const uint32_t* inl);

// count() of one pattern (fm_index.cpp:84-100), m >= 1, n >= 1: the backward
// search, finished over the left contexts once at most kCtxQ characters remain and
// the range is narrow (engines with contexts, when built).
template <class E, class PT, bool kLA = false>
__device__ __forceinline__ uint64_t count_pattern(const DevIndex& ix, const NodeTable& T,
                                                  PT P, uint64_t m,
                                                  uint64_t* bytes = nullptr) {
  uint64_t sp, ep, k;
  const uint32_t *inl, *maj;
  search_start(ix, T, P, m, sp, ep, k, bytes, &inl, &maj);
  if (sp >= ep) return 0;
  if (maj && k == kRec16Q) {  // a wide record's majority contexts (kRec16Maj)
    uint32_t want = 0;
    bool ok = true;
    for (uint32_t t = 0; t < kRec16Q; ++t) {  // chain symbol t = P[k-1-t]
      const uint32_t d = T.occ_code[P[kRec16Q - 1 - t]];
      ok &= d != kNoCode;
      want |= (d & 3u) << (2 * t);
    }
    uint64_t c;
    if (ok && rec16_majority(maj[1], maj[3], want, c)) return c;
  }
  return count_rest<E, PT, kLA>(ix, T, P, k, sp, ep, bytes, inl);
}

// One suffix-array entry: a random read nothing re-reads, non-temporal as the records are
// (C4 one-call locate 0.835 -> 0.815 ms, 64-mer count 1.268 -> 1.256 ms, three A/B rounds:
// profiles/r03/ab_nt_sa_load.jsonl)
__device__ __forceinline__ uint32_t load_sa(const uint32_t* sa, uint64_t r) {
  return __builtin_nontemporal_load(sa + r);
}

// Verification against the text (lf_exact indexes that keep the full suffix array and the
// text in HBM: DevIndex::vsa / vtext).  Row r of [sp, ep) survives the k remaining steps
// iff its chain spells P[k-1], ..., P[0]; LF^t(r) is the row of the rotation SA[r] - t, so
// that chain is text[SA[r] - k .. SA[r]) (cyclically, as the rotations).  A narrow range
// with many characters left is therefore finished by reading its rows' SA entries (one
// sector: the rows are consecutive) and comparing k text bytes before each — two
// dependent rounds of reads instead of k rank steps (a 64-mer: 49 steps).  The result is
// the count the steps would give, exactly.
constexpr uint32_t kVerifyRows = 8;
constexpr uint32_t kVerifyWords = 8;  // text words compared per round (64 characters)

// bytes P[j, j + 8) as a little-endian uint64, from realigned dword loads that touch only
// dwords holding bytes of P[0, k) (bytes at or past k: unspecified)
__device__ __forceinline__ uint64_t pat8(const uint8_t* P, uint64_t j, uint64_t k) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(P) + j;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t off = (uint32_t)(a & 3);
  const uint64_t left = k - j;
  const uint32_t nb = off + (uint32_t)(left < 8 ? left : 8);  // bytes spanned from w
  const uint32_t w0 = w[0];
  const uint32_t w1 = nb > 4 ? w[1] : 0u;
  const uint32_t w2 = nb > 8 ? w[2] : 0u;
  const uint64_t lo = ((uint64_t)w1 << 32) | w0;
  return off ? (lo >> (8 * off)) | ((uint64_t)w2 << (64 - 8 * off)) : lo;
}
__device__ __forceinline__ uint64_t pat8(PackedDna P, uint64_t j, uint64_t) {
  uint64_t x = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) x |= (uint64_t)P[j + i] << (8 * i);
  return x;
}
// A pattern read byte by byte: copies in kernel arguments or LDS (k_count_one, the
// resident server), where realigned word loads would force the copy to scratch.
struct BytePat {
  const uint8_t* b;
  __device__ __forceinline__ uint32_t operator[](uint64_t i) const { return b[i]; }
};
__device__ __forceinline__ uint64_t pat8(BytePat P, uint64_t j, uint64_t k) {
  uint64_t x = 0;
  for (uint32_t i = 0; i < 8 && j + i < k; ++i) x |= (uint64_t)P[j + i] << (8 * i);
  return x;
}
// the mask of the bytes of a chunk at j that lie inside P[0, k)
__device__ __forceinline__ uint64_t chunk_mask(uint64_t j, uint64_t k) {
  return k - j >= 8 ? ~0ull : (1ull << (8 * (k - j))) - 1;
}
// text[t, t + 8) from the aligned words w0 (holding t) and w1 (the next one)
__device__ __forceinline__ uint64_t text8(uint64_t w0, uint64_t w1, uint64_t t) {
  const uint32_t sh = (uint32_t)(t & 7) * 8;
  return sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
}

// text[q, q + k) == P[0, k), cyclically (positions mod n).  Windows inside [0, n) compare
// 8 kVerifyWords bytes per round of aligned 8-B loads; a window through the end of the text (a row
// whose suffix starts fewer than k positions into the text) byte by byte.
// kLA (long patterns, CS_Q_LONG): rounds of kVerifyWordsLA words, the next round's words loaded before
// this round compares, so a window of R rounds waits for one HBM round trip plus R - 1
// overlapped ones instead of R.  The extra registers are why it is a separate kernel.
constexpr uint32_t kVerifyWordsLA = 16;  // 8 and 12 measured: 150-mers 2.47 / 2.56 vs 2.56·10⁹/s
template <class PT, bool kLA = false>
__device__ __forceinline__ bool window_eq(const DevIndex& ix, PT P, uint64_t q, uint64_t k,
                                          uint64_t* bytes) {
  const uint64_t n = ix.n;
  if (q + k > n) {
    for (uint64_t j = 0; j < k; ++j) {
      uint64_t t = q + j;
      if (t >= n) t -= n;
      if (ix.vtext[t] != (uint8_t)P[j]) return false;
    }
    if (bytes) *bytes += 64;
    return true;
  }
  const uint64_t* tw = reinterpret_cast<const uint64_t*>(ix.vtext);
  const uint64_t last = (q + k - 1) >> 3;  // the last word holding a byte of the window
  if constexpr (kLA) {
    constexpr uint32_t V = kVerifyWordsLA;
    uint64_t w[V + 1];
    uint64_t a = q >> 3;
#pragma unroll
    for (uint32_t i = 0; i <= V; ++i) w[i] = a + i <= last ? tw[a + i] : 0ull;
    for (uint64_t j0 = 0; j0 < k; j0 += 8 * V) {
      const bool more = j0 + 8 * V < k;
      uint64_t x[V];  // the next round's words past w[V] (which it starts with)
#pragma unroll
      for (uint32_t i = 0; i < V; ++i) {
        const uint64_t b = a + V + 1 + i;
        x[i] = more && b <= last ? tw[b] : 0ull;
      }
      if (bytes) *bytes += 8 * V;
      uint64_t diff = 0;
#pragma unroll
      for (uint32_t i = 0; i < V; ++i) {
        const uint64_t j = j0 + 8 * i;
        if (j < k) diff |= (text8(w[i], w[i + 1], q + j) ^ pat8(P, j, k)) & chunk_mask(j, k);
      }
      if (diff) return false;
      w[0] = w[V];
#pragma unroll
      for (uint32_t i = 0; i < V; ++i) w[i + 1] = x[i];
      a += V;
    }
    return true;
  }
  for (uint64_t j0 = 0; j0 < k; j0 += 8 * kVerifyWords) {
    const uint64_t a = (q + j0) >> 3;
    uint64_t w[kVerifyWords + 1];
#pragma unroll
    for (uint32_t i = 0; i <= kVerifyWords; ++i) w[i] = a + i <= last ? tw[a + i] : 0ull;
    if (bytes) *bytes += 8 * kVerifyWords;
    uint64_t diff = 0;
#pragma unroll
    for (uint32_t i = 0; i < kVerifyWords; ++i) {
      const uint64_t j = j0 + 8 * i;
      if (j < k) diff |= (text8(w[i], w[i + 1], q + j) ^ pat8(P, j, k)) & chunk_mask(j, k);
    }
    if (diff) return false;
  }
  return true;
}

// The rows of [sp, ep) (at most kVerifyRows) worth a full comparison: for two rows or more,
// their SA entries (consecutive rows: one sector) in one round, then one aligned 8-B word
// at the start of every row's window in one round (1-8 of its first characters against
// the same pattern chunk).  Bit i: row sp + i.
template <class PT>
__device__ __forceinline__ uint32_t verify_filter(const DevIndex& ix, PT P, uint64_t k,
                                                  uint64_t sp, uint64_t ep, uint64_t* bytes) {
  const uint32_t w = (uint32_t)(ep - sp);
  if (w == 1) return 1u;
  const uint64_t n = ix.n;
  const uint64_t* tw = reinterpret_cast<const uint64_t*>(ix.vtext);
  uint32_t pos[kVerifyRows];
#pragma unroll
  for (uint32_t i = 0; i < kVerifyRows; ++i) pos[i] = i < w ? ix.vsa[sp + i] : 0u;
  if (bytes) *bytes += 32 + 32ull * w;
  const uint64_t p0 = pat8(P, 0, k) & chunk_mask(0, k);
  uint32_t pass = 0;
#pragma unroll
  for (uint32_t i = 0; i < kVerifyRows; ++i) {
    if (i >= w) break;
    const uint64_t p = pos[i];
    const uint64_t q = p >= k ? p - k : p + n - k;  // P[0] sits at text[q]
    const uint32_t sh = (uint32_t)(q & 7) * 8;
    const uint64_t x = tw[q >> 3] >> sh;  // text[q, q + 8 - (q & 7)): inside the word
    const uint64_t msk = chunk_mask(0, k) & (~0ull >> sh) & (q + 8 <= n ? ~0ull : (1ull << (8 * (n - q))) - 1);
    if (((x ^ p0) & msk) == 0) pass |= 1u << i;
  }
  return pass;
}

// P[s, ...) as a pattern of its own
__device__ __forceinline__ const uint8_t* pat_shift(const uint8_t* P, uint64_t s) { return P + s; }
__device__ __forceinline__ BytePat pat_shift(BytePat P, uint64_t s) { return BytePat{P.b + s}; }
__device__ __forceinline__ PackedDna pat_shift(PackedDna P, uint64_t s) {
  return PackedDna{s < 32 ? P.x >> (2 * s) : 0ull};
}

// The candidate rows base + i (bit i of mm) — their contexts matched P[k - qf, k), or they
// passed verify_filter (qf = 0): each one's SA entry, then P[0, k - qf) against the text
// before its suffix's last qf characters.
template <class PT, bool kLA = false>
__device__ __forceinline__ uint64_t verify_rows(const DevIndex& ix, PT P, uint64_t k, uint32_t qf,
                                                uint64_t base, uint32_t mm, uint64_t* bytes) {
  const uint64_t n = ix.n;
  uint64_t cnt = 0;
  while (mm) {
    const uint32_t i = (uint32_t)__ffs(mm) - 1u;
    mm &= mm - 1;
    const uint64_t p = load_sa(ix.vsa, base + i);
    if (bytes) *bytes += 32;
    cnt += window_eq<PT, kLA>(ix, P, p >= k ? p - k : p + n - k, k - qf, bytes) ? 1u : 0u;
  }
  return cnt;
}

// The rest of a count() from the range [sp, ep) (non-empty) with P[0..k) still to
// process (fm_index.cpp:90-98); inl as search_start's.
template <class E, class PT, bool kLA>
__device__ __forceinline__ uint64_t count_rest(const DevIndex& ix, const NodeTable& T, PT P,
                                               uint64_t k, uint64_t sp, uint64_t ep,
                                               uint64_t* bytes, const uint32_t* inl) {
  constexpr uint32_t R = 32 / sizeof(typename E::CtxEnt);  // context rows per sector
  bool ctx = E::kCtx && ix.lctx != nullptr;
  // context characters a record holds inline
  const uint32_t qi = ix.ptab_rec == 2 ? (ix.wide ? kRec16QW : kRec16Q) : ix.lctx_q;
  while (k > 0) {
    // verification against the text pays once it saves more than the one step + context
    // read it replaces; the contexts (of the record: no read, or of a sector) filter the
    // rows first, on P's last qf characters
    const bool ver = ix.vsa && k > (ctx ? ix.lctx_q + 1u : 2u) && k < ix.n;
    uint32_t qf = 0;
    if (ctx && k <= ix.lctx_q) qf = (uint32_t)k;
    else if (ctx && ver) qf = inl && rec_inline(ix, qi, ep - sp) ? qi : ix.lctx_q;
    if (inl && !(qf && rec_inline(ix, qf, ep - sp))) inl = nullptr;
    uint32_t mm = 0;
    uint64_t base = sp;
    bool cand = false;
    if (qf && (inl || ep - (sp & ~(uint64_t)(R - 1)) <= 2 * R)) {
      const uint32_t r = ctx_match<typename E::CtxEnt>(ix, T, pat_shift(P, k - qf), qf, sp, ep, mm,
                                                       base, bytes, inl);
      if (r == kCtxAbsent) return 0;
      if (r == kCtxOk) {
        if (qf == k) return (uint64_t)__popc(mm);
        cand = true;
      } else {
        ctx = false;  // an escaped context or a rare symbol
      }
    }
    if (!cand && ver && ep - sp <= kVerifyRows) {
      mm = verify_filter(ix, P, k, sp, ep, bytes);
      base = sp;
      qf = 0;
      cand = true;
    }
    if (cand) return verify_rows<PT, kLA>(ix, P, k, qf, base, mm, bytes);
    inl = nullptr;
    --k;
    if (!E::step(ix, T, P[k], sp, ep, bytes)) return 0;
  }
  return ep - sp;
}

// Locate records (phase 1 -> phase 2, cs_fm_locate_ranges_device's d_sp): the
// first row of the range [sp, ep), or — for a search finished over the left
// contexts (lf_exact indexes only) — the window of matching rows r at k characters
// before the end: bit 63 set, bits 60-62 k, bits 38-59 the matches relative to the
// first one (bit i: row r0 + i), bits 0-37 r0.  The final rows are LF^k(r), in the
// same order (LF keeps the order of rows with equal chains), and with LF one n-cycle
// SA[LF^k(r)] = SA[r] - k (mod n), so phase 2 walks from r and subtracts k.
constexpr uint64_t kLocCtx = 1ull << 63;
constexpr uint64_t kLocRowMask = (1ull << 38) - 1;
constexpr uint32_t kLocSpanBits = 22;
// locate phase 2 kernels fused with the records: a lane takes a pattern of at most this
// many rows (every context window: <= kLocSpanBits); wider ranges go a block per range
constexpr uint64_t kLocSmall = 32;
// rows handed to the walk: row | k << kWalkAdjShift (k = positions to subtract)
constexpr int kWalkAdjShift = 56;
constexpr uint64_t kWalkRowMask = (1ull << kWalkAdjShift) - 1;

// A window of rows verified against the text (locate_search, indexes with DevIndex::vsa):
// bits 60-62 zero (a context window has k >= 1 there), bits 38-49 the matches relative to
// the first one, bits 50-59 k.  Its positions are SA[row] - k as for a context window.
constexpr uint32_t kLocVerRelBits = 12;
constexpr uint64_t kLocVerMaxK = (1u << 10) - 1;

// rows, adjustment and match bits of a window record (s & kLocCtx)
__device__ __forceinline__ void loc_window(uint64_t s, uint64_t& r0, uint64_t& adj, uint32_t& rel) {
  r0 = s & kLocRowMask;
  adj = (s >> 60) & 7u;
  if (adj) {
    rel = (uint32_t)(s >> 38) & ((1u << kLocSpanBits) - 1u);
  } else {
    rel = (uint32_t)(s >> 38) & ((1u << kLocVerRelBits) - 1u);
    adj = (s >> 50) & kLocVerMaxK;
  }
}

// The rows base + i (bit i of mm) whose window text[SA - k, SA - qf) spells P[0, k - qf)
// (verify_rows' test, as a mask).
template <class PT>
__device__ __forceinline__ uint32_t verify_mask(const DevIndex& ix, PT P, uint64_t k, uint32_t qf,
                                                uint64_t base, uint32_t mm) {
  const uint64_t n = ix.n;
  uint32_t out = 0;
  while (mm) {
    const uint32_t i = (uint32_t)__ffs(mm) - 1u;
    mm &= mm - 1;
    const uint64_t p = load_sa(ix.vsa, base + i);
    if (window_eq(ix, P, p >= k ? p - k : p + n - k, k - qf, nullptr)) out |= 1u << i;
  }
  return out;
}

// locate()'s search (fm_index.cpp:107-124): the count and the pattern's record — its
// range's first row, a context window (the last <= 7 characters over the left contexts),
// or a verified window (long patterns over lf_exact indexes with the full suffix array and
// the text: the rows of a narrow range whose text before their suffix spells the rest of
// the pattern, count_rest's verification; SA[r] - k is then the position, so phase 2 reads
// the same SA entries the verification read).
template <class E, class PT>
__device__ __forceinline__ uint64_t locate_search(const DevIndex& ix, const NodeTable& T,
                                                  PT P, uint64_t m,
                                                  uint64_t& rec) {
  uint64_t sp, ep, k;
  const uint32_t* inl;
  rec = 0;
  search_start(ix, T, P, m, sp, ep, k, nullptr, &inl);
  if (sp >= ep) return 0;
  constexpr uint32_t R = 32 / sizeof(typename E::CtxEnt);
  bool ctx = E::kCtx && ix.lctx != nullptr && ix.lf_exact;
  bool ver = ix.vsa != nullptr;  // implies lf_exact
  const uint32_t qi = ix.ptab_rec == 2 ? kRec16Q : ix.lctx_q;  // vsa: narrow indexes only
  while (k > 0) {
    const uint64_t w = ep - sp;
    const bool fits = ep - (sp & ~(uint64_t)(R - 1)) <= 2 * R;
    if (ctx && k <= ix.lctx_q && k <= 7) {
      const uint32_t* in = inl && rec_inline(ix, k, w) ? inl : nullptr;
      if (in || fits) {
        uint32_t mm = 0;
        uint64_t base;
        const uint32_t r = ctx_match<typename E::CtxEnt>(ix, T, P, (uint32_t)k, sp, ep, mm, base,
                                                         nullptr, in);
        if (r == kCtxAbsent || (r == kCtxOk && mm == 0)) return 0;
        if (r == kCtxOk) {
          const uint32_t f = (uint32_t)__ffs(mm) - 1u;
          const uint32_t rel = mm >> f;
          if ((rel >> kLocSpanBits) == 0) {
            rec = kLocCtx | (k << 60) | ((uint64_t)rel << 38) | (base + f);
            return (uint64_t)__popc(mm);
          }
        }
        ctx = false;
      }
    }
    if (ver && k > (ctx ? ix.lctx_q + 1u : 2u) && k < ix.n && k <= kLocVerMaxK) {
      uint32_t qf = 0, mm = 0;
      uint64_t base = sp;
      bool cand = false;
      if (ctx) {  // filter on P's last qf characters first (count_rest)
        qf = inl && rec_inline(ix, qi, w) ? qi : ix.lctx_q;
        const uint32_t* in = inl && rec_inline(ix, qf, w) ? inl : nullptr;
        if (in || fits) {
          const uint32_t r = ctx_match<typename E::CtxEnt>(ix, T, pat_shift(P, k - qf), qf, sp, ep,
                                                           mm, base, nullptr, in);
          if (r == kCtxAbsent) return 0;
          if (r == kCtxOk) cand = true;
          else ctx = false;
        }
      }
      if (!cand && w <= kVerifyRows) {
        mm = verify_filter(ix, P, k, sp, ep, nullptr);
        base = sp;
        qf = 0;
        cand = true;
      }
      if (cand) {
        mm = verify_mask(ix, P, k, qf, base, mm);
        if (!mm) return 0;
        const uint32_t f = (uint32_t)__ffs(mm) - 1u;
        const uint32_t rel = mm >> f;
        if ((rel >> kLocVerRelBits) == 0) {
          rec = kLocCtx | (k << 50) | ((uint64_t)rel << 38) | (base + f);
          return (uint64_t)__popc(mm);
        }
        ver = false;  // matches too far apart for the record: step on
      }
    }
    inl = nullptr;
    --k;
    if (!E::step(ix, T, P[k], sp, ep, nullptr)) return 0;
  }
  rec = sp;
  return ep - sp;
}

}  // namespace

// Dispatch on the handle's engine / rank-line format.
#define FMX_DISPATCH(h, KERNEL, GRID, ...)                                      \
  do {                                                                          \
    if ((h)->line_fmt == kFmtOcc)                                               \
      KERNEL<OccE><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                       \
    else if ((h)->line_fmt == kFmtLOcc)                                         \
      KERNEL<LOccE><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                      \
    else if ((h)->line_fmt == kFmtQwm)                                          \
      KERNEL<QWM><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                        \
    else if ((h)->line_fmt == kFmtLine32)                                       \
      KERNEL<WM<Line32>><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                 \
    else if ((h)->line_fmt == kFmtLine32W)                                      \
      KERNEL<WM<Line32W>><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                \
    else                                                                        \
      KERNEL<WM<Line64>><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                 \
    FMX_HIP(hipGetLastError());                                                 \
  } while (0)

// Same, with a second template argument after the engine.
#define FMX_DISPATCH2(h, KERNEL, TARG, GRID, ...)                               \
  do {                                                                          \
    if ((h)->line_fmt == kFmtOcc)                                               \
      KERNEL<OccE, TARG><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                 \
    else if ((h)->line_fmt == kFmtLOcc)                                         \
      KERNEL<LOccE, TARG><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                \
    else if ((h)->line_fmt == kFmtQwm)                                          \
      KERNEL<QWM, TARG><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);                  \
    else if ((h)->line_fmt == kFmtLine32)                                       \
      KERNEL<WM<Line32>, TARG><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);           \
    else if ((h)->line_fmt == kFmtLine32W)                                      \
      KERNEL<WM<Line32W>, TARG><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);          \
    else                                                                        \
      KERNEL<WM<Line64>, TARG><<<(GRID), kBlk, 0, st>>>(__VA_ARGS__);           \
    FMX_HIP(hipGetLastError());                                                 \
  } while (0)

// Same, one 64-lane block.
#define FMX_DISPATCH1(h, KERNEL, ...)                                           \
  do {                                                                          \
    if ((h)->line_fmt == kFmtOcc)                                               \
      KERNEL<OccE><<<1, 64, 0, st>>>(__VA_ARGS__);                              \
    else if ((h)->line_fmt == kFmtLOcc)                                         \
      KERNEL<LOccE><<<1, 64, 0, st>>>(__VA_ARGS__);                             \
    else if ((h)->line_fmt == kFmtQwm)                                          \
      KERNEL<QWM><<<1, 64, 0, st>>>(__VA_ARGS__);                               \
    else if ((h)->line_fmt == kFmtLine32)                                       \
      KERNEL<WM<Line32>><<<1, 64, 0, st>>>(__VA_ARGS__);                        \
    else if ((h)->line_fmt == kFmtLine32W)                                      \
      KERNEL<WM<Line32W>><<<1, 64, 0, st>>>(__VA_ARGS__);                       \
    else                                                                        \
      KERNEL<WM<Line64>><<<1, 64, 0, st>>>(__VA_ARGS__);                        \
    FMX_HIP(hipGetLastError());                                                 \
  } while (0)

}  // namespace fmx
