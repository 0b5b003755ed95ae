// fm_device.hpp — HBM layout of the index and the device-side rank primitives:
// the binary wavelet matrix's rank lines (Line32 / Line32W / Line64, below), the
// occurrence lines shared by the occurrence engine and the quaternary wavelet
// matrix (OccLine), and the locate walk lines (WalkLine / WalkLineW).
//
// Wavelet matrix (the reference's "WaveletTree", src/core/wavelet.cpp:14-53): 8
// levels, level l holds bit (7-l) of the level-l sequence; the next sequence is the
// stable zeros-then-ones partition.  Each level's BitVector (src/core/bitvector.hpp:
// 95-98: bits_ + super_ u32 every 2048 bits + blocks_ u16 every 256 bits) is stored
// re-laid-out as RANK LINES, one HBM access per rank1:
//
//   Line32  { u32 base; u32 w[7]; }   32 B, 224 payload bits   (n < 2^32, default)
//   Line32W { u64 base; u32 w[6]; }   32 B, 192 payload bits   (wide: n >= 2^32)
//   Line64  { u64 base; u64 w[7]; }   64 B, 448 payload bits   (any n < 2^38)
//
// base = rank1 at the line's first bit (absolute), w[] = the bits LSB-first.
// rank1(i) = base + popcount of the line's bits below i.  MI355X serves random
// 16/32-B reads at ~50 G/s and 64-B reads at ~26 G/s (profiles/microbench:
// DRAM access granularity is 32 B), so the 32-B line halves the DRAM cost of a
// rank; it is used whenever the text fits u32 ranks (the reference's own limit,
// SURVEY.md §0.6).  rank1(i) equals BitVector::rank1(i) for every 0 <= i <= n
// (tests/test_gpu_parity.py checks every position against the oracle).  A
// sentinel line past n makes rank1(n) (the reference's count_ones() special case,
// bitvector.cpp:168-170) a plain line read.
//
// Node table: the wavelet-matrix node of prefix x (top l bits of a symbol) at level
// l is a contiguous block [S, S+size) of level l.  R = rank1_l(S).  A node is PURE
// when all its bits are equal (every symbol under it has the same bit 7-l); then
// rank1 inside it is affine (R, or R + (i - S)) and needs no memory access.  This
// is exact: it removes only loads whose result is determined by the symbol
// histogram.  For ACGT+'$' text 2-4 of the 8 levels need a load per rank.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fmx {

constexpr int kLevels = 8;
constexpr int kNodes = 255;  // internal nodes, levels 0..7
constexpr uint8_t kPure = 1, kPureBit = 2;
constexpr int kMaxExc = 128;  // occurrence-line engine: rare-symbol rows kept in LDS

// Everything the query kernels read besides the lines; copied into LDS by every
// block (10.3 KB).
struct NodeTable {
  uint64_t S[kNodes];   // node start in its level
  uint64_t R[kNodes];   // rank1_l(S)
  uint64_t Z[kLevels];  // zeros per level (size - ones)
  uint64_t C[257];      // fm_index.cpp:36-47 (u64)
  uint64_t S8[256];     // start of each symbol's run after the last level
  uint8_t flags[256];   // kPure | kPureBit per node
  uint8_t code[256];    // prefix-table digit of each symbol, kNoCode if not in its alphabet
  uint8_t sym[256];     // digit -> symbol
  // occurrence-line engine (OccLine below): 2-bit code of each coded symbol
  // (kNoCode: rare or absent), code -> symbol, and the BWT rows holding a rare
  // symbol (ascending; stored as code 0 in the lines and corrected here)
  uint8_t occ_code[256];
  uint8_t occ_sym[4];
  uint32_t exc_n;
  uint64_t exc_row[kMaxExc];
  uint8_t exc_sym[kMaxExc];
  // quaternary wavelet matrix engine (QWM below): occ_code holds each present
  // symbol's dense code, qsym the inverse; levels; per level the start of each
  // digit's block in the next level; the node arrays S / R / flags (kPure |
  // digit << 2) are indexed by qnode_id, S8 by code (leaf starts).
  uint32_t qlevels;
  uint64_t qZ[4][4];
  uint8_t qsym[256];
};
constexpr uint8_t kNoCode = 0xFF;

// rank-line formats (cs_fm_index::line_fmt)
enum LineFmt : uint32_t {
  kFmtLine32 = 0, kFmtLine32W = 1, kFmtLine64 = 2, kFmtOcc = 3, kFmtQwm = 4, kFmtLOcc = 5
};

// Quaternary wavelet matrix: node of the l-digit code prefix x at level l.
__host__ __device__ inline int qnode_id(int level, uint32_t prefix) {
  return ((1 << (2 * level)) - 1) / 3 + (int)prefix;
}

struct DevIndex {
  const void* lines;     // kLevels * nlines rank lines of the handle's format
  uint64_t nlines;       // per level = n / line_bits + 1
  uint64_t n;
  // Row-sampled SA (fm_index.cpp:57-66): u32 as the reference when the index is not
  // wide, u64 for wide indexes (n >= 2^32).  Same widths for isa and the prefix
  // table entries (2 x u32 / 2 x u64).
  uint32_t wide;
  const void* ssa;
  uint64_t nsamples;
  uint32_t stride;
  uint32_t stride_shift; // log2(stride) when stride is a power of two, else 0xFFFFFFFF
  const NodeTable* table;
  // Prefix table: (sp, ep) of every k-mer over the frequent alphabet (sigma_t
  // symbols), index = sum_j digit(P[m-1-j]) * sigma_t^j.  The generalisation of
  // C[] (the k = 1 table, fm_index.cpp:36-47): a count() whose last k characters
  // are all in the alphabet starts at step k+1.  Empty when ptab_k == 0.
  const void* ptab;
  uint32_t ptab_k;
  uint32_t ptab_sigma;
  uint32_t ptab_rec;     // 1: entries are 32-B context records, 2: 16-B ones (kRecCtx below)
  // Inverse-SA samples: isa[k] = row of the suffix at text position k*stride, for
  // extract by LF inversion (needs suffix order == rotation order, i.e. a unique
  // smallest last symbol: lf_exact).
  const void* isa;
  uint64_t nisa;
  uint32_t pstride;      // their text-position stride (finer than the SSA's; cs_fm_index::xstride)
  uint32_t lf_exact;
  // Walk lines and the samples they index (WalkLine above); null when absent.
  const void* walk;
  const void* wssa;      // sample of each mark, in row order (u32; wide: 40-bit entries)
  uint32_t wssa_eb;      // bytes per wssa entry: 4, 5 (40 bits, little-endian) or 8
  // Left contexts (null when absent): per BWT row the codes of the lctx_q symbols
  // its LF chain meets, lctx_sb bits each (see kCtxQ below).
  const void* lctx;
  uint32_t lctx_q;
  uint32_t lctx_sb;
  // Learned occurrence lines (LOccLine below): one LOccModel per superblock of
  // 2^lmodel_shift lines.
  const void* lmodel;
  uint32_t lmodel_shift;
  // Full suffix array (u32) and text (n bytes) of an lf_exact index that keeps both in
  // HBM, for verifying narrow ranges against the text (fm_query.hip verify_count); null
  // otherwise or under CS_Q_NO_CONTEXTS / CS_Q_NO_VERIFY.
  const uint32_t* vsa;
  const uint8_t* vtext;
  // Round 6: the byte text of an lf_exact occurrence-line index WITHOUT the full suffix array
  // but with walk lines and text-position marks (C5): long patterns' candidate rows are
  // verified against it at the position their short walk gives (k_count_long kWalk) instead
  // of stepping every character.  Null otherwise or under CS_Q_NO_CONTEXTS / CS_Q_NO_VERIFY.
  const uint8_t* wtext;
  // ... and its rare-symbol positions (u64, sorted; the packed text stores them as code 0) when
  // the walk-verified long patterns compare against the 2-bit text (ptext, no full SA)
  const uint64_t* wrare;
  uint32_t nwrare;
  // The same text 2-bit packed (occurrence codes, character i at bits 2 (i % 32) of word
  // i / 32, rare symbols as code 0) and the sorted positions of the rare symbols: long
  // patterns are verified against 32 characters per 8-B word (k_count_long).  Null
  // unless vtext is set and the index has occurrence lines.
  const uint64_t* ptext;
  const uint32_t* prare;
  uint32_t nrare;
  // Locate records (null when absent; see kLocRec below): lrec64 = 1: one 64-B record per
  // ptab_k-mer (kLocRec64*), index = its prefix-table index; else one 16-B record per
  // (ptab_k + 1)-mer, index = the prefix-table index of its last ptab_k characters plus
  // digit(first character) * 4^ptab_k.
  const void* lrec;
  uint32_t lrec64;
  // Round 6: the prefix table's digits and the occurrence codes are both the standard DNA code
  // (A C G T = 0 1 2 3, every other byte in neither alphabet): the staged count maps a
  // pattern's characters four at a time in registers instead of one LDS lookup each
  uint32_t dna_std;
};

// Locate records (narrow lf_exact occurrence-line indexes with 16-B context records, the
// left contexts and the full SA; C4: k + 1 = 16, 69 GB).  A Q_text locate through the
// context record reads the record, then the matching row's SA entry — two dependent random
// reads where count needs one.  The locate record of a (k+1)-mer holds the SA values
// themselves: for a (k+1)-mer with at most kLocRecRows rows, dwords 0-2 = SA[row i] for its
// rows i < w, dword 3 = the rows' kLocRecQ-character left contexts (8 bits each, the low bits
// of their lctx entries) at bits 8i, and w at bits 24-26 (kLocRecNone: more rows, or an
// escaped context — read the context record instead).  A pattern of k+1+j characters, j <=
// kLocRecQ, matches row i iff the low 2j bits of its context spell the j characters before
// the (k+1)-mer (the backward-search invariant, fm_device.hpp kCtxQ), and a single matching
// row's position is SA[row i] - j (SA[LF^j(r)] = SA[r] - j, lf_exact).  C4 (n / 4^16 = 0.93
// rows per 16-mer): a text 20-mer's 16-mer has at most 3 rows 93 % of the time.  Built from
// the k-mer's context record and lctx: the rows of c.x are the rows r of x with BWT[r] = c
// (the first symbol of r's chain), in order, with SA[r] - 1 and r's chain shifted by one.
constexpr uint32_t kLocRecRows = 3;
constexpr uint32_t kLocRecQ = 4;
constexpr uint32_t kLocRecNone = 7;

// 64-B locate records (round 4, the default): a random 64-B block read by four consecutive
// lanes, 16 B each, costs one DRAM request and runs at the 16-B read rate (49 G/s over 17
// and 69 GB, profiles/r04/coop_gather_*.txt; one lane reading 64 B: 19 G/s).  So a record
// per k-mer x (the context record's index) holds up to kLocRec64Rows rows: chunk c (16 B,
// lane c of the quad) = SA[row 3c + i] in dwords 0-2 and, in dword 3, the rows' 5-character
// left contexts (10 bits each, the low bits of their lctx entries) at bits 10 i and the
// number of valid rows in the chunk at bits 30-31.  A pattern of k + j characters, j <=
// kLocRec64Q, matches row r iff the low 2j bits of r's context spell its first j characters
// (the backward-search invariant), and a single match's position is SA[r] - j.  More rows
// than kLocRec64Rows, or an escaped context: every chunk is (~0, 0, 0, 0) — read the
// context record instead.  C4 (n / 4^15 = 3.7 rows per 15-mer): 99.6 % of the Q_text
// 20-mers are answered by the one read (bench.py locate_record_hit_frac).
constexpr uint32_t kLocRec64Rows = 12;
constexpr uint32_t kLocRec64Q = 5;

// Left context of BWT row r: the codes of BWT[LF^t(r)], t = 0..q-1 — the q
// characters preceding the row's rotation — symbol t in bits [sb t, sb (t+1)).
// Occurrence engine: u16 entries, 2-bit codes, q = kCtxQ = 7, and bit 15 (kCtxEsc)
// when one of the symbols is a rare one.  Quaternary matrix: u32 entries, the dense
// symbol code (sb = 2 x levels bits: 8 for sigma = 256), q = 32 / sb (4 for sigma =
// 256), no escapes (every present symbol has a code).  A backward search with
// k <= q characters left and its range [sp, ep) inside two 32-B sectors of lctx
// counts the rows whose context matches those characters in one read: the rows
// surviving the remaining steps are exactly the rows whose chain spells them (each
// step keeps {LF(r) : BWT[r] = c}, fm_index.cpp:90-96, monotone in r).
constexpr uint32_t kCtxQ = 7;
constexpr uint32_t kCtxEsc = 0x8000u;

// Where a batch count writes (cs_count_out): uint64 counts (the reference's type), uint32
// (exact when n < 2^32, checked by the caller), or uint8 with counts >= 255 stored as 255
// and listed as (pattern, count) pairs behind an atomic counter (pairs past exc_cap are
// dropped; the counter still counts them).
struct CountOut {
  void* out;
  uint64_t* exc;
  unsigned long long* exc_n;
  uint64_t exc_cap;
  uint32_t width;
};
// W: the width when known at compile time (8, 4, 1), 0 = o.width
template <int W>
__device__ __forceinline__ void store_count(const CountOut& o, uint64_t q, uint64_t v) {
  const uint32_t w = W ? (uint32_t)W : o.width;
  if (w == 8) {
    // non-temporal: the counts stream out past the caches that the random record reads
    // use (C4 headline 0.396 -> 0.388 ms in one box session; non-temporal pattern loads
    // were measured too, 0.408 ms: profiles/r03/ab_nt_store.jsonl)
    __builtin_nontemporal_store(v, static_cast<uint64_t*>(o.out) + q);
  } else if (w == 4) {  // (non-temporal as the uint64 counts: packed 0.357 -> 0.350 ms, u32 0.430
    // -> 0.425, profiles/r04/ab_lib_r04ad_*.jsonl)
    __builtin_nontemporal_store((uint32_t)v, static_cast<uint32_t*>(o.out) + q);
  } else {
    __builtin_nontemporal_store((uint8_t)(v < 255 ? v : 255), static_cast<uint8_t*>(o.out) + q);
    if (v >= 255) {
      const unsigned long long e = atomicAdd(o.exc_n, 1ull);
      if (e < o.exc_cap) {
        o.exc[2 * e] = q;
        o.exc[2 * e + 1] = v;
      }
    }
  }
}

// Long-pattern routing inside one call (fm_query.hip launch_count_staged / the one-call
// locate): the staged kernel leaves the patterns its one read cannot answer (m >= kFastM and
// m > k + kCtxQ) to the long-pattern kernel launched behind it on the same stream.  Lists
// are per wave of the staged kernel, so no block barrier orders them: wave w of block b
// (its 128 patterns b kLongRegion + {64 w + l, kBlk + 64 w + l : l < 64}) owns slot
// 4 b + w and lists its long patterns there — each pattern's offset inside the block's
// region (u16) at list[slot kLongSlot + i], the number in cnt[slot] (a ballot orders them) —
// and zeroes cnt2[slot]; the list kernels read every slot's length on the device and take
// the entries of their slots flattened (all lanes busy), and what they cannot finish goes
// to the slot lists `list2` / `cnt2` of the pattern for the general-search kernel after
// them.  No host synchronisation and no state in the handle: every list is the call's own
// buffer (the caller's workspace, or one allocated for the call), so concurrent calls on other
// streams cannot interfere.  All null: no routing.
// Round 5: the routed count also lists the patterns its one read cannot finish (the general
// search: wide ranges, escaped contexts, symbols off the table) in the wave's slot of list2
// (gen_list), so no lane of the staged kernel runs a dependent chain while 63 others idle,
// and the waves that list anything add their number to `listed` (kListedLanes counters, one
// per 256-B line, blockIdx.x % kListedLanes): a list kernel whose counters sum to 0 leaves at
// its first load — no slot scan.  The counters are zero between calls: the list kernel's last
// block to retire (the `retire` counter) zeroes them and itself.  A workspace is therefore
// zero-filled once before its first use (cs_fm_workspace_bytes, cs_fmindex.h).
constexpr uint32_t kLongRegion = 512;  // = 2 kBlk: the staged kernels' patterns per block (U = 2)
constexpr uint32_t kLongSlot = 128;    // a wave's patterns (64 lanes x U = 2): one slot
constexpr uint32_t kSlotsPerRegion = kLongRegion / kLongSlot;
constexpr uint32_t kListedLanes = 16;
constexpr uint32_t kListedStride = 64;  // uint32 words between the counters (256 B)
constexpr uint64_t kListHdrBytes = (uint64_t)(kListedLanes + 1) * kListedStride * 4;  // + retire
struct LongList {
  uint16_t* list = nullptr;
  uint32_t* cnt = nullptr;
  uint32_t* list2 = nullptr;  // (u32: the offset in bits 0-8, the routed count's chain above)
  uint32_t* cnt2 = nullptr;
  uint32_t* hdr = nullptr;  // listed[kListedLanes] (kListedStride apart), then retire
  uint32_t gen_list = 0;    // the routed count: general-search patterns to list2
  // the routed count: per list2 entry the range the staged kernel's table read left (sp in
  // bits 0-31, its width in 32-63; narrow indexes) or kNoRange (the search starts over)
  // (and in the list2 entry's bits 9-26, beside a range, the 2-bit occurrence codes of the
  // characters still to step — list_chain — or kChainNone: a symbol without a code, the
  // pattern is read again)
  uint64_t* rng2 = nullptr;
  uint32_t grid = 0;  // (host side: the list kernel's grid, cs_fm_index::list_grid; 0 = default)
};
constexpr uint64_t kNoRange = ~0ull;
// A listed pattern's chain (18 bits, a list2 entry's bits 9-26): its first k <= 7 characters'
// occurrence codes, character i at bits 2 (k - 1 - i) (the staged kernel's context key: the
// next character to step at bits 0-1), k at bits 14-16, bit 17 set.
constexpr uint32_t kChainNone = 0;
constexpr uint32_t kChainShift = 9;  // log2(kLongRegion): the entry's offset below it
__host__ __device__ inline uint32_t list_chain(uint32_t codes, uint32_t k) {
  return codes | (k << 14) | (1u << 17);
}
// the staged kernel's wave adds its listed patterns (lane 0; n uniform over the wave)
__device__ __forceinline__ void list_listed_add(const LongList& ll, uint32_t n) {
  if (n && (threadIdx.x & 63) == 0)
    atomicAdd(ll.hdr + (blockIdx.x % kListedLanes) * kListedStride, n);
}
// whether any pattern was listed (every thread of a block; uniform)
__device__ __forceinline__ bool list_any(const LongList& ll) {
  uint32_t v = 0;
  if (threadIdx.x < kListedLanes)
    v = __hip_atomic_load(ll.hdr + threadIdx.x * kListedStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __syncthreads_or(v != 0) != 0;
}
// a list kernel's block is done (every thread; after list_any was true): the last block of
// the grid zeroes the counters for the next call on this workspace
__device__ __forceinline__ void list_retire(const LongList& ll) {
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* retire = ll.hdr + kListedLanes * kListedStride;
    __threadfence();
    if (atomicAdd(retire, 1u) == gridDim.x - 1) {
      for (uint32_t i = 0; i < kListedLanes; ++i) ll.hdr[i * kListedStride] = 0;
      *retire = 0;
    }
  }
}
// the slot of pattern q: its block's region, the wave of the lane that holds it
__host__ __device__ inline uint64_t long_slot(uint64_t q) {
  return (q / kLongRegion) * kSlotsPerRegion + ((q % kLongRegion) % 256) / 64;
}

// A single pattern passed by value in kernel arguments (k_count_one).
struct OnePattern {
  static constexpr uint32_t kMax = 128;
  uint8_t b[kMax];
  uint32_t m;
};

// Resident single-pattern server (cs_fm_serve_start): the request mailbox is
// kServeWords 8-byte words in fine-grained pinned host memory, each (tag << 32 |
// payload) — word 0 carries the pattern length (kServeStop = shut down), words 1..
// four pattern bytes each.  Aligned 8-byte stores and loads are single-copy atomic on
// both sides, so a request is complete when every word it uses carries its tag.
constexpr uint32_t kServeWords = 32;
constexpr uint32_t kServeMax = (kServeWords - 1) * 4;  // 124 bytes
constexpr uint32_t kServeStop = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t ssa_at(const DevIndex& ix, uint64_t k) {
  return ix.wide ? static_cast<const uint64_t*>(ix.ssa)[k] : static_cast<const uint32_t*>(ix.ssa)[k];
}
__device__ __forceinline__ uint64_t isa_at(const DevIndex& ix, uint64_t k) {
  return ix.wide ? static_cast<const uint64_t*>(ix.isa)[k] : static_cast<const uint32_t*>(ix.isa)[k];
}
// Prefix-table entries: 2 x u32 (sp, ep); in wide indexes (n >= 2^32) one u64 packing
// sp (38 bits, n < 2^38) and the range width (26 bits), so the table keeps 8 B per
// k-mer.  A width >= kPtabEsc is stored as kPtabEsc: that k-mer's search starts from
// C[] instead (ptab_at returns false).
constexpr uint64_t kPtabEsc = (1ull << 26) - 1;
// Context records (narrow occurrence-engine indexes with left contexts): each entry
// is 32 B — sp (u32), width (u32) and the left contexts (u16) of the range's first
// kRecCtx rows — so a search whose range after the table is at most kRecCtx rows
// wide and has at most kCtxQ characters left is answered by the ONE random read of its
// table entry (the contexts are the rows' lctx entries, fm_device.hpp kCtxQ).
// Compact records (ptab_rec 2, tables whose mean range is at most 4 rows) are 16 B —
// half the table, and 16-B random reads run faster than 32-B ones over a multi-GB table
// (DESIGN.md §2): dword 0 sp; dword 1 bits 0-3 the width w when w <= kRec16Ctx, else
// kRec16Wide (the width is then dword 2, no contexts: also used when a row of the range
// has an escaped context); contexts of kRec16Q characters (10 bits, the low bits of the
// rows' lctx entries) of rows 0-5 at bits 4 + 10i of dwords 1-2, rows 6-8 at bits
// 10(i-6) of dword 3.
// Quaternary-matrix records (ptab_rec 3, tables with at most 2 rows per k-mer on
// average; C3: k = 4, 0.23): 16 B — sp, width, and the u32 contexts of rows 0-1.
constexpr uint32_t kRecQCtx = 2;
constexpr uint32_t kRecCtx = 12;
constexpr uint32_t kRec16Ctx = 9;
constexpr uint32_t kRec16Q = 5;
constexpr uint32_t kRec16Wide = 15;
// Compact records of a wide index (n >= 2^32; C5, k = 16: 7.5 rows per k-mer): 4-character
// contexts (8 bits, the low bits of the rows' lctx entries) of rows 0-9 — dword 1 bits 4-27
// rows 0-2, dword 2 rows 3-6, dword 3 bits 0-23 rows 7-9 — and bits 32-37 of sp in dword 3
// bits 24-29.  Enough for a 20-mer at k = 16.  A k-mer whose range the 8-B wide table
// escaped (wider than kPtabEsc) has width kRec16Wide and dword 2 = ~0: its search starts
// from C[].
// Majority contexts of a wide compact record (narrow indexes, round 4): a range wider than
// kRec16Ctx rows whose rows' contexts repeat — repetitive text, where a k-mer's rows are
// copies of one locus — keeps the two most frequent kRec16Q-character contexts with their
// exact counts: dword 1 bit 4 (kRec16Maj) set, bit 5 (kRec16MajAll) when every row's context
// is one of the two, bits 6-15 context A, bits 16-25 context B; dword 3 count A (bits 0-15)
// and count B (bits 16-31, 0 = no B).  A count of a pattern with kRec16Q characters before
// the table part is then the count of its context (0 when absent from a complete list) — the
// rows surviving the reference's remaining steps are the rows whose chain spells them
// (kCtxQ), exactly.  Built only for ranges without escaped contexts, of at most kRec16MajScan
// rows, whose counts fit 16 bits.
constexpr uint32_t kRec16Maj = 1u << 4;
constexpr uint32_t kRec16MajAll = 1u << 5;
constexpr uint32_t kRec16MajScan = 1u << 20;
// the count of the kRec16Q-character context want10 from a majority record, when it answers
__device__ __forceinline__ bool rec16_majority(uint32_t y, uint32_t w3, uint32_t want10, uint64_t& cnt) {
  if (!(y & kRec16Maj)) return false;
  if (want10 == ((y >> 6) & 0x3FFu)) {
    cnt = w3 & 0xFFFFu;
    return true;
  }
  if ((w3 >> 16) && want10 == ((y >> 16) & 0x3FFu)) {
    cnt = w3 >> 16;
    return true;
  }
  if (y & kRec16MajAll) {
    cnt = 0;
    return true;
  }
  return false;
}
constexpr uint32_t kRec16CtxW = 10;
constexpr uint32_t kRec16QW = 4;
constexpr uint32_t kRec16NoRange = 0xFFFFFFFFu;
__device__ __forceinline__ uint64_t rec16_sp(uint32_t x, uint32_t w, uint32_t wide) {
  return (uint64_t)x | (wide ? (uint64_t)((w >> 24) & 0x3Fu) << 32 : 0ull);
}
// the rows' contexts of a wide compact record, as u16 entries in dw[0..4]
__device__ __forceinline__ void rec16w_contexts(uint32_t y, uint32_t z, uint32_t w, uint32_t dw[5]) {
  uint32_t e[10];
#pragma unroll
  for (int i = 0; i < 3; ++i) e[i] = (y >> (4 + 8 * i)) & 0xFFu;
#pragma unroll
  for (int i = 0; i < 4; ++i) e[3 + i] = (z >> (8 * i)) & 0xFFu;
#pragma unroll
  for (int i = 0; i < 3; ++i) e[7 + i] = (w >> (8 * i)) & 0xFFu;
#pragma unroll
  for (int i = 0; i < 5; ++i) dw[i] = e[2 * i] | (e[2 * i + 1] << 16);
}
// the rows' contexts of a compact record, as u16 entries in dw[0..4] (dw[4] bits 0-15)
__device__ __forceinline__ void rec16_contexts(uint32_t y, uint32_t z, uint32_t w, uint32_t dw[5]) {
  const uint64_t lo = (uint64_t)y | ((uint64_t)z << 32);
  uint32_t e[10];
#pragma unroll
  for (int i = 0; i < 6; ++i) e[i] = (uint32_t)(lo >> (4 + 10 * i)) & 0x3FFu;
#pragma unroll
  for (int i = 6; i < 9; ++i) e[i] = (w >> (10 * (i - 6))) & 0x3FFu;
  e[9] = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) dw[i] = e[2 * i] | (e[2 * i + 1] << 16);
}
// the rows of a compact record (rec16_contexts' entries) whose context matches the k <= 5
// chain codes `want` (k = 0: every row): bit i for row i, rows 0..8
__device__ __forceinline__ uint32_t rec16_match(uint32_t y, uint32_t z, uint32_t w, uint32_t want, uint32_t k) {
  const uint64_t lo = (uint64_t)y | ((uint64_t)z << 32);
  const uint32_t mask = (1u << (2 * k)) - 1u;
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 6; ++i) m |= (uint32_t)((((uint32_t)(lo >> (4 + 10 * i)) ^ want) & mask) == 0) << i;
#pragma unroll
  for (int i = 6; i < 9; ++i) m |= (uint32_t)((((w >> (10 * (i - 6))) ^ want) & mask) == 0) << i;
  return m;
}
__device__ __forceinline__ bool ptab_at(const DevIndex& ix, uint64_t t, uint64_t& sp, uint64_t& ep) {
  if (ix.ptab_rec == 1) {
    const uint2 r = static_cast<const uint2*>(ix.ptab)[t * 4];
    sp = r.x;
    ep = (uint64_t)r.x + r.y;
    return true;
  }
  if (ix.ptab_rec == 3) {
    const uint2 r = static_cast<const uint2*>(ix.ptab)[t * 2];
    sp = r.x;
    ep = (uint64_t)r.x + r.y;
    return true;
  }
  if (ix.ptab_rec == 2) {
    const uint4 r = static_cast<const uint4*>(ix.ptab)[t];
    const uint32_t wc = r.y & 15u;
    sp = rec16_sp(r.x, r.w, ix.wide);
    ep = sp + (wc == kRec16Wide ? r.z : wc);
    return !(wc == kRec16Wide && r.z == kRec16NoRange);
  }
  if (ix.wide) {
    const uint64_t e = static_cast<const uint64_t*>(ix.ptab)[t];
    const uint64_t w = e >> 38;
    sp = e & ((1ull << 38) - 1);
    ep = sp + w;
    return w != kPtabEsc;
  }
  const uint2 r = static_cast<const uint2*>(ix.ptab)[t];
  sp = r.x;
  ep = r.y;
  return true;
}

__host__ __device__ inline int node_id(int level, uint32_t prefix) {
  return (1 << level) - 1 + (int)prefix;
}

__device__ __forceinline__ uint64_t u64_of(uint32_t lo, uint32_t hi) {
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// ---------------------------------------------------------------------------
// 32-byte line: dword 0 = base, dwords 1..7 = payload (224 bits)
struct Line32 {
  static constexpr uint32_t kBytes = 32;
  static constexpr uint32_t kWordBits = 32;
  static constexpr int kWords = 7;
  static constexpr int kBaseWords = 1;  // payload starts at dword 1
  static constexpr uint32_t kBits = kWords * kWordBits;  // 224
  using Raw = uint4[2];

  // p < 2^32 * 32: q = (p/32)/7 in 32-bit arithmetic
  __device__ static __forceinline__ void locate(uint64_t p, uint32_t& q, uint32_t& o) {
    const uint32_t g = (uint32_t)(p >> 5);
    q = g / 7u;
    o = (uint32_t)(p - (uint64_t)q * kBits);
  }
  __device__ static __forceinline__ void load(const void* lines, uint64_t idx, Raw& v) {
    const uint4* p = reinterpret_cast<const uint4*>(lines) + idx * 2;
    v[0] = p[0];
    v[1] = p[1];
  }
  __device__ static __forceinline__ uint64_t base(const Raw& v) { return v[0].x; }
  // popcount of the first o payload bits, o in [0, 224]
  __device__ static __forceinline__ uint32_t prefix(const Raw& v, uint32_t o) {
    const uint32_t w[7] = {v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int sh = (int)o - 32 * k;
      const uint32_t m = sh >= 32 ? ~0u : (sh <= 0 ? 0u : ((1u << sh) - 1u));
      r += (uint32_t)__popc(w[k] & m);
    }
    return r;
  }
  __device__ static __forceinline__ uint32_t bit(const Raw& v, uint32_t o) {
    const uint32_t w[7] = {v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    const uint32_t k = o >> 5;
    uint32_t d = w[0];
#pragma unroll
    for (int j = 1; j < 7; ++j) d = (k == (uint32_t)j) ? w[j] : d;
    return (d >> (o & 31)) & 1u;
  }
};

// 32-byte wide line: dwords 0-1 = u64 base, dwords 2..7 = payload (192 bits);
// the 32-B DRAM granule for indexes whose ranks exceed u32 (n >= 2^32).
struct Line32W {
  static constexpr uint32_t kBytes = 32;
  static constexpr uint32_t kWordBits = 32;
  static constexpr int kWords = 6;
  static constexpr int kBaseWords = 2;  // payload starts at dword 2
  static constexpr uint32_t kBits = kWords * kWordBits;  // 192 = 3 x 64
  using Raw = uint4[2];

  __device__ static __forceinline__ void locate(uint64_t p, uint32_t& q, uint32_t& o) {
    const uint32_t g = (uint32_t)(p >> 6);  // p < 2^38
    q = g / 3u;
    o = (uint32_t)(p - (uint64_t)q * kBits);
  }
  __device__ static __forceinline__ void load(const void* lines, uint64_t idx, Raw& v) {
    const uint4* p = reinterpret_cast<const uint4*>(lines) + idx * 2;
    v[0] = p[0];
    v[1] = p[1];
  }
  __device__ static __forceinline__ uint64_t base(const Raw& v) { return u64_of(v[0].x, v[0].y); }
  __device__ static __forceinline__ uint32_t prefix(const Raw& v, uint32_t o) {
    const uint32_t w[6] = {v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int sh = (int)o - 32 * k;
      const uint32_t m = sh >= 32 ? ~0u : (sh <= 0 ? 0u : ((1u << sh) - 1u));
      r += (uint32_t)__popc(w[k] & m);
    }
    return r;
  }
  __device__ static __forceinline__ uint32_t bit(const Raw& v, uint32_t o) {
    const uint32_t w[6] = {v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
    const uint32_t k = o >> 5;
    uint32_t d = w[0];
#pragma unroll
    for (int j = 1; j < 6; ++j) d = (k == (uint32_t)j) ? w[j] : d;
    return (d >> (o & 31)) & 1u;
  }
};

// 64-byte line: qword 0 = base, qwords 1..7 = payload (448 bits)
struct Line64 {
  static constexpr uint32_t kBytes = 64;
  static constexpr uint32_t kWordBits = 64;
  static constexpr int kWords = 7;
  static constexpr int kBaseWords = 1;  // payload starts at qword 1
  static constexpr uint32_t kBits = kWords * kWordBits;  // 448
  using Raw = uint4[4];

  __device__ static __forceinline__ void locate(uint64_t p, uint32_t& q, uint32_t& o) {
    const uint32_t g = (uint32_t)(p >> 6);
    q = g / 7u;
    o = (uint32_t)(p - (uint64_t)q * kBits);
  }
  __device__ static __forceinline__ void load(const void* lines, uint64_t idx, Raw& v) {
    const uint4* p = reinterpret_cast<const uint4*>(lines) + idx * 4;
    v[0] = p[0];
    v[1] = p[1];
    v[2] = p[2];
    v[3] = p[3];
  }
  __device__ static __forceinline__ uint64_t base(const Raw& v) { return u64_of(v[0].x, v[0].y); }
  __device__ static __forceinline__ uint32_t prefix(const Raw& v, uint32_t o) {
    const uint64_t w[7] = {u64_of(v[0].z, v[0].w), u64_of(v[1].x, v[1].y), u64_of(v[1].z, v[1].w),
                           u64_of(v[2].x, v[2].y), u64_of(v[2].z, v[2].w), u64_of(v[3].x, v[3].y),
                           u64_of(v[3].z, v[3].w)};
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int sh = (int)o - 64 * k;
      const uint64_t m = sh >= 64 ? ~0ull : (sh <= 0 ? 0ull : ((1ull << sh) - 1));
      r += (uint32_t)__popcll(w[k] & m);
    }
    return r;
  }
  __device__ static __forceinline__ uint32_t bit(const Raw& v, uint32_t o) {
    const uint32_t dw[14] = {v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w, v[2].x,
                             v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
    const uint32_t k = o >> 5;
    uint32_t d = dw[0];
#pragma unroll
    for (int j = 1; j < 14; ++j) d = (k == (uint32_t)j) ? dw[j] : d;
    return (d >> (o & 31)) & 1u;
  }
};

// ---------------------------------------------------------------------------
// Occurrence line (small-alphabet engine): the whole BWT in one sequence of 32-B
// lines, 64 rows each, one HBM access per rank of ANY symbol:
//   dwords 0-2  low 32 bits of occ(code 0..2) at the line's first row
//   dword 3     bits 8j..8j+7 = bits 32..39 of occ(code j)        (n < 2^40)
//   dwords 4-7  the 64 rows' 2-bit codes, row r at bits 2r of the 128-bit payload
// occ(code 3) = 64 q - occ0 - occ1 - occ2.  Used when at most four symbols carry
// all but kMaxExc rows (DNA + terminator): a wavelet matrix then needs 2-4 line
// reads per rank (one per non-pure level), this needs one.  Rows of the remaining
// (rare) symbols are stored as code 0 and listed in NodeTable::exc_row.
struct OccLine {
  static constexpr uint32_t kBytes = 32;
  static constexpr uint32_t kRows = 64;
  using Raw = uint4[2];
  __device__ static __forceinline__ void load(const void* lines, uint64_t q, Raw& v) {
    const uint4* p = reinterpret_cast<const uint4*>(lines) + q * 2;
    v[0] = p[0];
    v[1] = p[1];
  }
  // occ(code c) at the first row of line q
  __device__ static __forceinline__ uint64_t base(const Raw& v, uint32_t c, uint64_t q) {
    const uint64_t o0 = u64_of(v[0].x, v[0].w & 0xFFu);
    const uint64_t o1 = u64_of(v[0].y, (v[0].w >> 8) & 0xFFu);
    const uint64_t o2 = u64_of(v[0].z, (v[0].w >> 16) & 0xFFu);
    return c == 0 ? o0 : c == 1 ? o1 : c == 2 ? o2 : (q << 6) - o0 - o1 - o2;
  }
  // rows among the first o (0..64) of the line whose code is c
  __device__ static __forceinline__ uint32_t prefix(const Raw& v, uint32_t c, uint32_t o) {
    constexpr uint64_t k55 = 0x5555555555555555ull;
    const uint64_t pat = k55 * c;
    const uint64_t x0 = u64_of(v[1].x, v[1].y) ^ pat, x1 = u64_of(v[1].z, v[1].w) ^ pat;
    const uint64_t e0 = ~(x0 | (x0 >> 1)) & k55, e1 = ~(x1 | (x1 >> 1)) & k55;
    const uint64_t m0 = o >= 32 ? ~0ull : ((1ull << (2 * o)) - 1);
    const uint64_t m1 = o <= 32 ? 0ull : (o >= 64 ? ~0ull : ((1ull << (2 * (o - 32))) - 1));
    return (uint32_t)(__popcll(e0 & m0) + __popcll(e1 & m1));
  }
  // code of row o (0..63)
  __device__ static __forceinline__ uint32_t code(const Raw& v, uint32_t o) {
    const uint64_t lo = u64_of(v[1].x, v[1].y), hi = u64_of(v[1].z, v[1].w);
    return (uint32_t)(((o < 32 ? lo : hi) >> (2 * (o & 31))) & 3u);
  }
};

// ---------------------------------------------------------------------------
// Learned occurrence lines (LOccE; SURVEY.md §8(f) item 4 — the reference's learned
// occ, src/core/bitvector_learned.cpp:114-203: rank = coarse model prediction + micro
// residual + tail popcount, with the model of src/learned/pgm.hpp:31-79).  The
// occurrence line's three absolute 40-bit counts become three int16 residuals against a
// linear model of occ(c, .) per superblock of 2^sb lines, fitted through the
// superblock's end points, so a 32-B line holds 104 rows instead of 64:
//   occ(c, 104 q) = pred_c(q) + r_c(q),
//   pred_c(q) = base_c + (slope_c * 104 (q - q0)) >> 32,  q0 = first line of q's superblock
// (integers only: the builder and the queries evaluate the same expression).  A rank is
// still one line read; the 48-B models of all superblocks (C4: 28 KB) stay in L2 and
// are read beside the line.  Residuals are bounded by the superblock's rows, so a
// superblock of 2^8 lines (26,624 rows) always fits int16; the builder tries 2^14 first.
//   words (u64): w0 rows 0-31, w1 rows 32-63, w2 rows 64-95 (2-bit codes), w3 bits 0-15
//   rows 96-103, bits 16-31 r_0, 32-47 r_1, 48-63 r_2.
struct LOccModel {
  uint64_t base[3];   // occ(c, 104 q0)
  uint64_t slope[3];  // 2^32 x (occ(c) at the superblock's last line start - base) / rows
};
struct LOccLine {
  static constexpr uint32_t kBytes = 32, kRows = 104;
  using Raw = uint4[2];
  __device__ static __forceinline__ void load(const void* lines, uint64_t q, Raw& v) {
    const uint4* p = reinterpret_cast<const uint4*>(lines) + q * 2;
    v[0] = p[0];
    v[1] = p[1];
  }
  // rows among the first o (0..104) of the line whose code is c
  __device__ static __forceinline__ uint32_t prefix(const Raw& v, uint32_t c, uint32_t o) {
    constexpr uint64_t k55 = 0x5555555555555555ull;
    const uint64_t pat = k55 * c;
    const uint64_t w[4] = {u64_of(v[0].x, v[0].y), u64_of(v[0].z, v[0].w), u64_of(v[1].x, v[1].y),
                           (uint64_t)(v[1].z & 0xFFFFu)};
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t x = w[k] ^ pat;
      const uint64_t e = ~(x | (x >> 1)) & k55;
      const int rows = (int)o - 32 * k;
      const uint64_t m = rows >= 32 ? ~0ull : (rows <= 0 ? 0ull : ((1ull << (2 * rows)) - 1));
      r += (uint32_t)__popcll(e & m);
    }
    return r;
  }
  __device__ static __forceinline__ uint32_t code(const Raw& v, uint32_t o) {
    const uint32_t k = o >> 4;  // dword holding row o
    const uint32_t d[7] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z};
    uint32_t x = d[0];
#pragma unroll
    for (int j = 1; j < 7; ++j) x = k == (uint32_t)j ? d[j] : x;
    return (x >> (2 * (o & 15))) & 3u;
  }
  __device__ static __forceinline__ int32_t resid(const Raw& v, uint32_t c) {
    const uint32_t h = c == 0 ? (v[1].z >> 16) : c == 1 ? (v[1].w & 0xFFFFu) : (v[1].w >> 16);
    return (int32_t)(int16_t)(uint16_t)h;
  }
};

__host__ __device__ inline uint64_t locc_pred(const LOccModel& m, uint32_t c, uint64_t dq) {
  return m.base[c] + ((m.slope[c] * (104ull * dq)) >> 32);
}

// ---------------------------------------------------------------------------
// Walk lines (locate's LF walk, occurrence engine): one 32-B line gives, for a
// row, its BWT code, occ(code) at the row (so LF), whether the row holds an SA
// sample ("mark") and the sample's index (marks before it).  The walk reads one
// line per step and stops at a mark.  Marks are the rows whose suffix starts at a
// text position that is a multiple of the stride when LF is one n-cycle
// (lf_exact: the walk then takes SA[row] mod stride < stride steps, mean
// (stride-1)/2), else the rows i with i % stride == 0, as the reference's SSA
// (fm_index.cpp:57-66, 125-153).  Positions are SA values either way, so results
// are identical.
//   WalkLine  (n < 2^32): 42 rows.  dwords 0-3 occ(code 0..2), marks before the
//     line (u32); dwords 4-5 codes of rows 0-31; dwords 6-7 bits 0-19 codes of
//     rows 32-41, bits 20-61 the 42 marks.
//   WalkLineW (wide): 32 rows.  dwords 0-3 low 32 bits of occ(code 0..2), marks;
//     dword 4 their bits 32-39 (byte j); dwords 5-6 codes; dword 7 marks.
__device__ __forceinline__ uint64_t eq2(uint64_t x, uint32_t c) {  // rows whose code == c
  constexpr uint64_t k55 = 0x5555555555555555ull;
  const uint64_t y = x ^ (k55 * c);
  return ~(y | (y >> 1)) & k55;
}
__device__ __forceinline__ uint64_t low_mask(uint32_t bits) {  // bits in [0, 64]
  return bits >= 64 ? ~0ull : ((1ull << bits) - 1);
}

struct WalkLine {
  static constexpr uint32_t kBytes = 32, kRows = 42;
  using Raw = uint4[2];
  __device__ static __forceinline__ void locate(uint64_t r, uint64_t& q, uint32_t& o) {
    const uint32_t r32 = (uint32_t)r;  // r < 2^32
    const uint32_t qq = r32 / kRows;
    q = qq;
    o = r32 - qq * kRows;
  }
  __device__ static __forceinline__ void load(const void* lines, uint64_t q, Raw& v) {
    const uint4* p = reinterpret_cast<const uint4*>(lines) + q * 2;
    v[0] = p[0];
    v[1] = p[1];
  }
  __device__ static __forceinline__ uint32_t code(const Raw& v, uint32_t o) {
    const uint64_t lo = u64_of(v[1].x, v[1].y), hi = u64_of(v[1].z, v[1].w);
    return (uint32_t)(((o < 32 ? lo : hi) >> (2 * (o & 31))) & 3u);
  }
  // occ(code c) at row q*42 + o
  __device__ static __forceinline__ uint64_t occ(const Raw& v, uint32_t c, uint64_t q, uint32_t o) {
    const uint64_t lo = u64_of(v[1].x, v[1].y), hi = u64_of(v[1].z, v[1].w) & 0xFFFFFull;
    const uint32_t in = (uint32_t)(__popcll(eq2(lo, c) & low_mask(2 * (o < 32 ? o : 32))) +
                                   __popcll(eq2(hi, c) & 0x55555ull & low_mask(o > 32 ? 2 * (o - 32) : 0)));
    const uint64_t b0 = v[0].x, b1 = v[0].y, b2 = v[0].z;
    const uint64_t base = c == 0 ? b0 : c == 1 ? b1 : c == 2 ? b2 : q * kRows - b0 - b1 - b2;
    return base + in;
  }
  __device__ static __forceinline__ bool mark(const Raw& v, uint32_t o) {
    return (u64_of(v[1].z, v[1].w) >> (20 + o)) & 1u;
  }
  __device__ static __forceinline__ uint64_t mark_rank(const Raw& v, uint32_t o) {
    return (uint64_t)v[0].w + __popcll((u64_of(v[1].z, v[1].w) >> 20) & low_mask(o));
  }
};

struct WalkLineW {
  static constexpr uint32_t kBytes = 32, kRows = 32;
  using Raw = uint4[2];
  __device__ static __forceinline__ void locate(uint64_t r, uint64_t& q, uint32_t& o) {
    q = r >> 5;
    o = (uint32_t)(r & 31);
  }
  __device__ static __forceinline__ void load(const void* lines, uint64_t q, Raw& v) {
    const uint4* p = reinterpret_cast<const uint4*>(lines) + q * 2;
    v[0] = p[0];
    v[1] = p[1];
  }
  __device__ static __forceinline__ uint32_t code(const Raw& v, uint32_t o) {
    return (uint32_t)((u64_of(v[1].y, v[1].z) >> (2 * o)) & 3u);
  }
  __device__ static __forceinline__ uint64_t occ(const Raw& v, uint32_t c, uint64_t q, uint32_t o) {
    const uint32_t in = (uint32_t)__popcll(eq2(u64_of(v[1].y, v[1].z), c) & low_mask(2 * o));
    const uint32_t hb = v[1].x;
    const uint64_t b0 = u64_of(v[0].x, hb & 0xFFu), b1 = u64_of(v[0].y, (hb >> 8) & 0xFFu),
                   b2 = u64_of(v[0].z, (hb >> 16) & 0xFFu);
    const uint64_t base = c == 0 ? b0 : c == 1 ? b1 : c == 2 ? b2 : q * kRows - b0 - b1 - b2;
    return base + in;
  }
  __device__ static __forceinline__ bool mark(const Raw& v, uint32_t o) { return (v[1].w >> o) & 1u; }
  __device__ static __forceinline__ uint64_t mark_rank(const Raw& v, uint32_t o) {
    return u64_of(v[0].w, v[1].x >> 24) + __popc(v[1].w & (uint32_t)low_mask(o));
  }
};

// rank1 of level `lv` (pointer to that level's first line) at position p.
template <class F>
__device__ __forceinline__ uint64_t rank1_at(const void* lv, uint64_t p) {
  uint32_t q, o;
  F::locate(p, q, o);
  typename F::Raw v;
  F::load(lv, q, v);
  return F::base(v) + F::prefix(v, o);
}

template <class F>
__device__ __forceinline__ const void* level_ptr(const DevIndex& ix, int level) {
  return reinterpret_cast<const uint8_t*>(ix.lines) + (uint64_t)level * ix.nlines * F::kBytes;
}

}  // namespace fmx
