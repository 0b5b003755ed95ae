// fm_query.hip — the hot path: batched backward search (FMIndex::count,
// src/api/fm_index.cpp:79-101) and the LF/SSA walk of FMIndex::locate
// (src/api/fm_index.cpp:107-157), as hand-written CDNA4 kernels.
//
// Every kernel is a template over a rank ENGINE (occ(c, i) for a search step, and
// LF with the BWT symbol), dispatched on the index's format (FMX_DISPATCH):
//   OccE        occurrence lines: one 32-B line per rank of any symbol (<= 4
//               frequent symbols, rare rows listed in the node table);
//   QWM         quaternary wavelet matrix of occurrence lines: one line per base-4
//               level (any alphabet; 4 levels for sigma = 256);
//   WM<F>       the reference's binary wavelet matrix (WaveletTree::rank,
//               src/core/wavelet.cpp:59-96) in rank lines F, in the "relative"
//               form: per level l with c's node not pure
//                   r = rank1_l(S + d) - R;  d = bit ? r : d - r.
// The node table (C[], node starts/ranks, code maps, rare rows) is staged in LDS per
// block.  The first k characters come from the prefix table (a k-mer -> (sp, ep)
// generalisation of C[]); absent symbols and empty ranges exit early exactly where
// the reference returns 0.
//
// locate: (1) the same search writes sp and min(count, limit); (2) exclusive scan ->
// CSR offsets; (3) rows expanded in row order (fm_index.cpp:125); (4) a persistent
// walk kernel: each block owns a contiguous slice of rows, its lanes pull rows from
// an LDS counter and cycle fetch -> walk -> sample with one dependent load per loop
// iteration.  With walk lines (fm_device.hpp WalkLine) one 32-B read per step gives
// the symbol, its occ and the sample mark; no separate BWT array is kept.
#include "fm_search.hpp"

namespace fmx {
namespace {

// offs == nullptr: patterns of one length fixed_m at stride fixed_m (cs_fm_count_fixed_device);
// kPacked: pats holds one uint64 per pattern, fixed_m <= 32 2-bit DNA characters (PackedDna);
// kLA: long patterns (launch_count_ex, CS_Q_LONG), the text comparison with look-ahead
template <class E, bool kPacked, bool kLA = false>
__global__ __launch_bounds__(kBlk) void k_count(DevIndex ix, const uint8_t* __restrict__ pats,
                                                const uint64_t* __restrict__ offs, uint64_t npat,
                                                CountOut co, uint64_t fixed_m) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= npat) return;
  uint64_t res;
  if constexpr (kPacked) {
    const uint64_t x = reinterpret_cast<const uint64_t*>(pats)[q];
    if (fixed_m == 0) res = ix.n;  // fm_index.cpp:80
    else if (ix.n == 0) res = 0;   // :81
    else res = count_pattern<E>(ix, T, PackedDna{x}, fixed_m);
  } else {
    const uint64_t o0 = offs ? offs[q] : q * fixed_m, m = offs ? offs[q + 1] - o0 : fixed_m;
    if (m == 0) res = ix.n;       // fm_index.cpp:80
    else if (ix.n == 0) res = 0;  // :81
    else res = count_pattern<E, const uint8_t*, kLA>(ix, T, pats + o0, m);
  }
  store_count<0>(co, q, res);
}

// The batch count over occurrence lines with left contexts, the C4/C5 shape: a
// pattern whose last k = ptab_k characters are in the prefix table and whose other
// m - k <= kCtxQ characters are coded needs two dependent reads — its table entry,
// then the context sector(s) of its range (one, when the entry is a context record
// holding the range).  Each lane takes U patterns (q0 + j * kBlk) and runs them in
// stages so their reads are in flight together: (A) offsets and pattern bytes
// (realigned dword loads, not byte loads), table index and context key; (B) the U
// table entries; (C) the U context sectors; (D) counts.  Anything else — patterns
// over 32 characters, symbols outside the table alphabet, wide ranges, escaped
// contexts — takes count_pattern, the general search (which reads the table entry
// again: carrying the range across would cost the kernel a wave per SIMD).
// kLoc: the same stages for locate's phase 1 (k_locate_ranges): co.out = min(count,
// limit) as uint64, rec = the pattern's locate record (locate_search), context windows
// only when LF is one n-cycle (lf_exact).
// kPacked: one uint64 of 2-bit DNA per pattern (PackedDna), fixed_m characters.
constexpr uint32_t kFastM = 32;

// bytes [0, m) of a pattern at byte offset o0, m <= 32, realigned: byte i is
// (u[i >> 2] >> 8 (i & 3)) & 0xFF.  Reads only the dwords holding pattern bytes.
// 64-bit value lo | hi << 32 of 2-bit digits (digit i at bits 2i, 2i + 1) with the digits'
// order reversed: digit i at bits 62 - 2i, 63 - 2i (low bit first)
__device__ __forceinline__ uint64_t rev_pairs64(uint32_t lo, uint32_t hi) {
  const uint64_t r = ((uint64_t)__builtin_bitreverse32(lo) << 32) | __builtin_bitreverse32(hi);
  return ((r >> 1) & 0x5555555555555555ull) | ((r & 0x5555555555555555ull) << 1);
}
// (the same in two halves, so that several patterns' loads can be in flight before the
// first is realigned: the dwords, then the realignment)
// Branch-free: all nine loads are issued, those past the pattern (m = 0: all of them) from
// `dummy` (any readable 36 B) and zeroed after.
__device__ __forceinline__ void load_pattern32_raw(const uint8_t* __restrict__ pats, uint64_t o0, uint32_t m,
                                                   uint32_t w[9], const uint32_t* __restrict__ dummy) {
  const uint32_t* w0 = reinterpret_cast<const uint32_t*>(pats + (o0 & ~3ull));
  const uint32_t nw = m ? ((uint32_t)(o0 & 3) + m + 3) >> 2 : 0u;
#pragma unroll
  for (int j = 0; j < 9; ++j) w[j] = ((uint32_t)j < nw ? w0 : dummy)[j];
#pragma unroll
  for (int j = 0; j < 9; ++j) w[j] = (uint32_t)j < nw ? w[j] : 0u;
}
__device__ __forceinline__ void realign_pattern32(uint64_t o0, const uint32_t w[9], uint32_t u[8]) {
  const uint32_t a = (uint32_t)(o0 & 3) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) u[j] = (uint32_t)((((uint64_t)w[j + 1] << 32) | w[j]) >> a);
}
__device__ __forceinline__ void load_pattern32(const uint8_t* __restrict__ pats, uint64_t o0,
                                               uint32_t m, uint32_t u[8]) {
  const uint32_t* w0 = reinterpret_cast<const uint32_t*>(pats + (o0 & ~3ull));
  const uint32_t a = (uint32_t)(o0 & 3) * 8;
  const uint32_t nw = ((uint32_t)(o0 & 3) + m + 3) >> 2;
  uint32_t w[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) w[j] = (uint32_t)j < nw ? w0[j] : 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j) u[j] = (uint32_t)((((uint64_t)w[j + 1] << 32) | w[j]) >> a);
}

// the patterns of a k_count_ctx lane that need the general search (st == 3); kOne: the
// locate results stay in the lane's registers (kc, kr)
// rng: k_count_ctx's s_rng ([U][kBlk][2]): the range after the table of a pattern with st 5
template <class E, int U, bool kLoc, bool kPacked, int W, bool kOne = false>
__device__ __forceinline__ void general_rest(const DevIndex& ix, const NodeTable& T,
                                             const uint8_t* __restrict__ pats, const uint8_t* st,
                                             const uint64_t* o0, const uint32_t* m, uint64_t q0,
                                             const CountOut& co, uint64_t limit,
                                             uint64_t* __restrict__ rec, uint64_t* kc = nullptr,
                                             uint64_t* kr = nullptr, const uint64_t* rng = nullptr) {
  uint64_t* const cnt_out = static_cast<uint64_t*>(co.out);  // kLoc
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if constexpr (!kLoc) {
      if (st[j] == 5) {  // from the range the table entry gave, m - ptab_k characters left
        const uint64_t q = q0 + (uint64_t)j * kBlk;
        const uint64_t* r = rng + 2 * ((uint64_t)j * kBlk + threadIdx.x);
        const uint64_t k = m[j] - ix.ptab_k;
        if constexpr (kPacked) {
          store_count<W>(co, q, count_rest<E>(ix, T, PackedDna{o0[j]}, k, r[0], r[1], nullptr, nullptr));
        } else {
          store_count<W>(co, q, count_rest<E>(ix, T, pats + o0[j], k, r[0], r[1], nullptr, nullptr));
        }
        continue;
      }
    }
    if (st[j] != 3) continue;
    const uint64_t q = q0 + (uint64_t)j * kBlk;
    if constexpr (kLoc) {
      uint64_t r;
      const uint64_t c = locate_search<E>(ix, T, pats + o0[j], m[j], r);
      if constexpr (kOne) {
        kc[j] = c < limit ? c : limit;
        kr[j] = r;
      } else {
        cnt_out[q] = c < limit ? c : limit;
        rec[q] = r;
      }
    } else if constexpr (kPacked) {
      const PackedDna P{o0[j]};
      store_count<W>(co, q, count_pattern<E>(ix, T, P, m[j]));
    } else {
      const uint8_t* P = pats + o0[j];
      store_count<W>(co, q, count_pattern<E>(ix, T, P, m[j]));
    }
  }
}

// Batch locate in one call (cs_fm_locate_device) over an index that keeps the full suffix
// array: three launches and one host synchronisation —
//   (1) k_count_ctx with kOne: the staged search; per pattern its record and, unless the
//       record is the pattern's only position (kLocStash below: count 1, 99.6 % of C4
//       Q_text), min(count, limit) — 8 B written per pattern instead of 12;
//       Per tile (a search block's 2 x 256 patterns) the total, added by each wave.
//   (2) k_scan_tiles: the exclusive scan of the tile totals (one block; C4: 24 k tiles);
//   (3) k_locate_emit: per tile, the block's scan of its counts plus the tile's prefix
//       give the output offsets, then the positions straight from the records through SA.
// (A look-back inside the search kernel, measured in round 3, made every block wait for the
// slowest search among its predecessors: 3.2 ms against 1.1 ms; the other forms round 5
// tried are listed at k_locate_emit.)  Against the two phases this drops the scan of a
// 100-MB count array and the host round trip between the phases.
// Indexes without the full suffix array but with walk lines and text-position marks (C5;
// C4 under CS_FM_FULL_SA=0) take the same launches (round 3): a position is the
// short walk from its row (walk_position: at most pstride - 1 LF steps, one 32-B walk line
// each, then the mark's sample) instead of SA[row], in (1) for a pattern's only position
// and in (3) / k_locate_emit_wide for the rest (kPos: 0 the full SA, 1 WalkLine, 2
// WalkLineW).  Counts are u64 (cnt64) when the index is wide.
// The one-call locate's outputs (offsets and positions) leave through non-temporal stores:
// nothing on the device reads them again (C4 one call 0.853 -> 0.818 ms in an A/B on one
// box; the search kernel's records and counts, which the emit kernel reads back, measured
// the same either way: profiles/r03/ab_nt_locate.jsonl)
template <class T>
__device__ __forceinline__ void st_out(T* p, T v) {
  __builtin_nontemporal_store(v, p);
}

struct OnePass {
  uint32_t* cnt = nullptr;               // (1) -> (3): min(count, limit) per pattern (narrow),
                                         // unless its record is a stashed position (count 1)
  uint64_t* cnt64 = nullptr;             // the same, wide indexes
  uint64_t* rec = nullptr;               // (1) -> (3): the pattern's record
  uint64_t* tiles = nullptr;             // per tile (a search block's patterns): its total, then
                                         // its exclusive prefix (k_scan_tiles)
  const uint32_t* sa = nullptr;          // full suffix array
  uint64_t* out_offs = nullptr;          // npat + 1 exclusive offsets
  uint64_t* out_pos = nullptr;           // positions, `cap` of them
  uint64_t cap = 0;
  uint64_t* wide = nullptr;              // (q, first row) of ranges over kLocSmall rows
  unsigned long long* nwide = nullptr;
  uint64_t wide_cap = 0;
  uint32_t defer = 0;  // locate records: a pattern its record does not answer -> k_locate_list
  // walk-line indexes (kPos 1 / 2): the positions of patterns with 2..kLocSmall rows, as
  // (output index, row | adj << 56) pairs for k_locate_walks — one lane per position, so no
  // emit wave waits on a lane's chain of walks — kLocTile slots per tile (tile t's at
  // t kLocTile, their number in wcnt[t]: no global counter); past them the emit walks them
  uint64_t* walks = nullptr;
  uint32_t* wcnt = nullptr;
  // k_scan_chained: per scan block its published total (bit 63: ready), zeroed by the search
  // kernel's block 0 (or a memset where no search kernel runs)
  unsigned long long* sflags = nullptr;
};
constexpr uint32_t kScanBlock = 1024;     // tiles per block of k_scan_chained
constexpr uint32_t kScanMaxBlocks = 1024; // (its look-back: one predecessor per thread)
constexpr uint32_t kWalkAdjShift56 = 56;
__device__ __forceinline__ void onepass_zero(const OnePass& op) {
  // the call's wide-range counter and the chained scan's flags and ticket (no memset launch;
  // stream order makes the stores visible to the kernels after this one)
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) *op.nwide = 0;
    if (op.sflags && blockIdx.x < kScanMaxBlocks) op.sflags[blockIdx.x] = 0;
    if (op.sflags && blockIdx.x == 0) op.sflags[kScanMaxBlocks] = 0;
  }
}
// Tiles of the one-call locate's scan (k_count_ctx kOne with U = 2 patterns per lane)
constexpr uint64_t kLocTile = 2 * kBlk;
static_assert(kLocTile == kLongRegion, "a tile is a region: one block's patterns");

// the text position of BWT row `row` by the short walk, and the same for U rows walked in
// lockstep (their line reads in flight together) — defined with the walks below
template <class W>
__device__ __forceinline__ uint64_t walk_position(const DevIndex& ix, const NodeTable& T, uint64_t row);
template <class W>
__device__ __forceinline__ uint64_t walk_position_steps(const DevIndex& ix, const NodeTable& T, uint64_t row,
                                                        uint64_t& steps);
template <class W, int U>
__device__ __forceinline__ void walk_positions(const DevIndex& ix, const NodeTable& T, uint64_t* pos,
                                               bool* act);
// the constants an LF step of a walk reads from the node table, held in registers by a
// barrier-free kernel whose table is the global one (a walk step through the caches waits on
// two more dependent loads: round 5, C5's one-call search 1.56 -> 1.70 ms that way)
struct WalkK {
  uint64_t C[4];     // C[] of each occurrence code's symbol
  uint32_t nexc;     // rare rows
  uint64_t exc_row0; // the rare row when there is one (C5's terminator), and C[] of its symbol
  uint64_t exc_c0;
};
__device__ __forceinline__ WalkK walk_consts(const NodeTable& T) {
  WalkK k;
#pragma unroll
  for (int c = 0; c < 4; ++c) k.C[c] = T.C[T.occ_sym[c]];
  k.nexc = T.exc_n;
  k.exc_row0 = k.nexc ? T.exc_row[0] : 0;
  k.exc_c0 = k.nexc ? T.C[T.exc_sym[0]] : 0;
  return k;
}
template <class W, int U>
__device__ __forceinline__ void walk_positions_k(const DevIndex& ix, const NodeTable& T, const WalkK& K,
                                                 uint64_t* pos, bool* act);

// position of BWT row `row` for the one-call locate: SA[row] (kPos 0) or the short walk
template <int kPos>
__device__ __forceinline__ uint64_t onepass_pos(const DevIndex& ix, const NodeTable& T, const OnePass& op,
                                                uint64_t row) {
  if constexpr (kPos == 0) return load_sa(op.sa, row);
  else if constexpr (kPos == 1) return walk_position<WalkLine>(ix, T, row);
  else return walk_position<WalkLineW>(ix, T, row);
}

// Exclusive scan over the block's U x kBlk values in pattern order (segment j holds the
// patterns q0 + j kBlk, j < U): mine[j] = the offset of the lane's j-th value inside the
// block, agg = the block's total.  Every thread of the block.
template <int U>
__device__ __forceinline__ void block_scan(const uint64_t* kc, uint64_t* mine, uint64_t& agg) {
  constexpr int NW = kBlk / 64;
  __shared__ uint64_t s_wsum[U][NW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t x[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    x[j] = kc[j];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(x[j], d, 64);
      if (lane >= d) x[j] += y;
    }
    if (lane == 63) s_wsum[j][wv] = x[j];
  }
  __syncthreads();
  agg = 0;
#pragma unroll
  for (int j = 0; j < U; ++j) {
    uint64_t before = agg;
    for (int w2 = 0; w2 < NW; ++w2) {
      if (w2 < wv) before += s_wsum[j][w2];
      agg += s_wsum[j][w2];
    }
    mine[j] = before + x[j] - kc[j];
  }
}

__device__ __forceinline__ void tile_total_add(const OnePass& op, uint64_t tile, uint64_t v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(op.tiles + tile), v);
}

// (1)'s tail: the lane's results.
// A pattern reporting exactly one position gets it here, from the record already in the
// lane (its first row: SA[row] - k for a context window), so its SA read overlaps the
// other blocks' record reads instead of waiting for k_locate_emit; the record then holds
// kLocStash | position and stands for the count 1 (no count is stored: 8 B per pattern).
// (C4 Q_text: 99.6 % of the patterns.)
constexpr uint64_t kLocStash = 1ull << 62;  // with bit 63 clear: not a window, not a row
__device__ __forceinline__ bool loc_stashed(uint64_t r) { return (r >> 62) == 1; }
// skip: bit j set = the lane's j-th pattern is k_locate_long's (routing): its count and record
// are left for that kernel to write
// kWaveTile (the barrier-free search, kPos 0): each wave adds its patterns' total to the tile
// (zeroed at the block's start) instead of a block scan storing it, so no wave waits for the
// block's others
template <int U, int kPos = 0, bool kWaveTile = false>
__device__ __forceinline__ void locate_split_store(const DevIndex& ix, const NodeTable& T, uint64_t npat,
                                                   uint64_t tile, uint64_t q0, const uint64_t* kc,
                                                   const uint64_t* kr, const OnePass& op, uint32_t skip = 0) {
  const uint64_t n = ix.n;
  uint64_t rs[U];
  if constexpr (kWaveTile) {
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < U; ++j) sum += kc[j];
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) sum += __shfl_xor(sum, dd, 64);
    if ((threadIdx.x & 63) == 0 && sum) tile_total_add(op, tile, sum);
  } else {
    uint64_t mine[U], agg;
    block_scan<U>(kc, mine, agg);
    if (threadIdx.x == 0) op.tiles[tile] = agg;
  }
  uint64_t row[U], adj[U];
  bool one[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk, s = kr[j];
    rs[j] = s;
    row[j] = s;
    adj[j] = 0;
    one[j] = q < npat && kc[j] == 1 && !loc_stashed(s);  // (not stashed by a locate record)
    uint32_t rel;
    if (one[j] && (s & kLocCtx)) loc_window(s, row[j], adj[j], rel);  // a window's only match: its first row
  }
  if constexpr (kPos == 0) {
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (one[j]) row[j] = load_sa(op.sa, row[j]);
  } else {  // the lane's walks in lockstep: row[j] becomes the position
    bool act[U];
#pragma unroll
    for (int j = 0; j < U; ++j) act[j] = one[j];
    if constexpr (kWaveTile)  // (T is the global table: the walks' constants in registers)
      walk_positions_k<std::conditional_t<kPos == 1, WalkLine, WalkLineW>, U>(ix, T, walk_consts(T), row, act);
    else
      walk_positions<std::conditional_t<kPos == 1, WalkLine, WalkLineW>, U>(ix, T, row, act);
  }
#pragma unroll
  for (int j = 0; j < U; ++j)
    if (one[j]) rs[j] = kLocStash | (row[j] >= adj[j] ? row[j] - adj[j] : row[j] + n - adj[j]);
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk;
    if (q >= npat || ((skip >> j) & 1u)) continue;
    if (!(kc[j] == 1 && loc_stashed(rs[j]))) {  // the count, and no stash standing for 1
      if (op.cnt64) op.cnt64[q] = kc[j];
      else op.cnt[q] = (uint32_t)kc[j];
      if (loc_stashed(rs[j])) rs[j] = 0;  // (a limit of 0)
    }
    op.rec[q] = rs[j];
  }
}

// (2): exclusive scan of the tile totals in place, one block; total -> *total_out.  The
// tiles pass through LDS 16 k at a time (128 KB + padding: a workgroup may hold 160 KB), so
// the global loads and stores are coalesced — the round-3 form gave each thread 32
// consecutive tiles straight from memory (strided loads and stores: 28 us for C4's 24 k
// tiles) — then each thread scans a contiguous run of 16 in registers and the block scans
// the run totals.
__device__ __forceinline__ uint32_t scan_pad(uint32_t i) { return i + (i >> 4); }  // LDS bank spread
__global__ __launch_bounds__(1024) void k_scan_tiles(uint64_t* __restrict__ tiles, uint64_t ntiles,
                                                     uint64_t* __restrict__ total_out) {
  constexpr int kRun = 16;                     // tiles per thread per round
  constexpr uint32_t kChunk = 1024u * kRun;    // tiles per round
  __shared__ uint64_t s_v[kChunk + kChunk / kRun];
  __shared__ uint64_t s_w[16];
  __shared__ uint64_t s_carry;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) s_carry = 0;
  for (uint64_t b = 0; b < ntiles; b += kChunk) {
#pragma unroll
    for (int r = 0; r < kRun; ++r) {  // coalesced: tile b + r 1024 + t
      const uint64_t i = b + (uint64_t)r * 1024 + t;
      s_v[scan_pad(r * 1024u + t)] = i < ntiles ? tiles[i] : 0ull;
    }
    __syncthreads();
    uint64_t v[kRun], run = 0;
#pragma unroll
    for (int r = 0; r < kRun; ++r) {  // the thread's run: tiles b + t kRun + r
      v[r] = s_v[scan_pad(t * kRun + r)];
      run += v[r];
    }
    uint64_t x = run;  // inclusive scan of the run totals over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(x, d, 64);
      if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int w2 = 0; w2 < 16; ++w2) {
      if (w2 < (int)wv) pre += s_w[w2];
      tot += s_w[w2];
    }
    uint64_t acc = s_carry + pre + x - run;
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
      s_v[scan_pad(t * kRun + r)] = acc;
      acc += v[r];
    }
    __syncthreads();  // (every thread has read s_carry and s_w of this round)
    if (t == 0) s_carry += tot;
#pragma unroll
    for (int r = 0; r < kRun; ++r) {
      const uint64_t i = b + (uint64_t)r * 1024 + t;
      if (i < ntiles) tiles[i] = s_v[scan_pad(r * 1024u + t)];
    }
    __syncthreads();  // before the next round's loads overwrite s_v and its scan reads s_carry
  }
  if (t == 0) *total_out = s_carry;
}

// the positions of c <= kLocSmall rows — rows r0 + i, or r0 + the set bits of rel (a context
// window) — minus adj (mod n), to out: SA reads kEmitRows at a time, in flight together
// (the walk-line forms list their rows instead: emit_walk_lines)
constexpr int kEmitRows = 4;
template <int kPos>
__device__ __forceinline__ void emit_rows(const DevIndex& ix, const NodeTable& T, const OnePass& op,
                                          uint64_t* __restrict__ out, uint64_t c, uint64_t r0, uint32_t rel,
                                          uint64_t adj) {
  const uint64_t n = ix.n;
  for (uint64_t i = 0; i < c; i += kEmitRows) {
    uint64_t row[kEmitRows];
    bool act[kEmitRows];
#pragma unroll
    for (int u = 0; u < kEmitRows; ++u) {
      act[u] = i + u < c;
      row[u] = 0;
      if (!act[u]) continue;
      if (rel) {
        row[u] = r0 + (uint32_t)__ffs(rel) - 1u;
        rel &= rel - 1u;
      } else {
        row[u] = r0 + i + u;
      }
    }
    static_assert(kPos == 0, "walk-line indexes list their rows (emit_walk_lines)");
#pragma unroll
    for (int u = 0; u < kEmitRows; ++u)
      if (act[u]) row[u] = load_sa(op.sa, row[u]);
#pragma unroll
    for (int u = 0; u < kEmitRows; ++u)
      if (act[u]) st_out(out + i + u, row[u] >= adj ? row[u] - adj : row[u] + n - adj);
  }
}

// (2'): the same scan over ceil(ntiles / 1024) blocks of 1024 tiles (one per thread): each
// block publishes its total (one flag word), sums its predecessors' — every thread polls one
// of them — and writes its tiles' exclusive prefixes; the last block writes the total.  The
// blocks wait only on lower ones.  (Round 5: the one-block scan took 18 us of C4's 0.53-ms
// one-call locate, its 24 k tiles passing through one CU.)  A block's place in the chain is
// the order in which it STARTS (an atomic ticket, sflags[kScanMaxBlocks], zeroed by the
// search kernel with the flags), not its blockIdx: a block only ever waits on blocks that
// are already running, whatever order the dispatcher picks (with other streams'
// kernels sharing the CUs, blockIdx order is not guaranteed).
__global__ __launch_bounds__(kScanBlock) void k_scan_chained(uint64_t* __restrict__ tiles, uint64_t ntiles,
                                                             uint64_t* __restrict__ total_out,
                                                             unsigned long long* __restrict__ sflags) {
  __shared__ uint64_t s_w[kScanBlock / 64];
  __shared__ uint64_t s_p[kScanBlock / 64];
  __shared__ uint32_t s_id;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) s_id = (uint32_t)atomicAdd(sflags + kScanMaxBlocks, 1ull);
  __syncthreads();
  const uint32_t bid = s_id;
  const uint64_t i = (uint64_t)bid * kScanBlock + t;
  const uint64_t v = i < ntiles ? tiles[i] : 0ull;
  uint64_t x = v;  // inclusive scan over the wave, then the block
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  uint64_t pre = 0, agg = 0;
#pragma unroll
  for (int w2 = 0; w2 < (int)(kScanBlock / 64); ++w2) {
    if (w2 < (int)wv) pre += s_w[w2];
    agg += s_w[w2];
  }
  if (t == 0)
    __hip_atomic_store(sflags + bid, (1ull << 63) | agg, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t p = 0;  // predecessor t's total
  if (t < bid) {
    unsigned long long f;
    do {
      f = __hip_atomic_load(sflags + t, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    } while (!(f >> 63));
    p = f & ~(1ull << 63);
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) p += __shfl_xor(p, d, 64);
  if (lane == 0) s_p[wv] = p;
  __syncthreads();
  uint64_t base = 0;
#pragma unroll
  for (int w2 = 0; w2 < (int)(kScanBlock / 64); ++w2) base += s_p[w2];
  if (i < ntiles) tiles[i] = base + pre + x - v;
  if (bid == gridDim.x - 1 && t == 0) *total_out = base + agg;
}

// (3) on walk-line indexes: offsets, the stashed positions, and the rows of every pattern
// with 2..kLocSmall positions listed for k_locate_walks in the tile's slots (a block scan
// places them: no atomic) instead of walked here — a lane walking its pattern's positions
// one after another kept its wave, and the emit, waiting (C5: the emit 360 us per 12.5 M
// 20-mers; 617 with four walks of a lane in lockstep; 1,156 with one global list counter,
// 98 k same-address atomics, profiles/r05/r05x, r05y).  A pattern past the tile's kLocTile
// slots is walked here (its slots below the limit marked void).
template <int U, int kPos>
__device__ __forceinline__ void emit_walk_lines(const DevIndex& ix, NodeTable& T, uint64_t npat, uint64_t tile,
                                                uint64_t q0, const uint64_t* kc, const uint64_t* kr,
                                                const uint64_t* mine, uint64_t base, const OnePass& op) {
  using W = std::conditional_t<kPos == 1, WalkLine, WalkLineW>;
  const uint64_t n = ix.n;
  uint64_t nl[U], tot = 0;
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk, a = base + mine[j], c = kc[j], s = kr[j];
    nl[j] = 0;
    if (q >= npat) continue;
    st_out(op.out_offs + q, a);
    if (!c || a + c > op.cap) continue;  // capacity short: the caller sees the total
    if (loc_stashed(s)) {
      st_out(op.out_pos + a, s & (kLocStash - 1));
    } else if ((s & kLocCtx) || c <= kLocSmall) {
      nl[j] = c;
    } else {
      const unsigned long long e = atomicAdd(op.nwide, 1ull);
      if (e < op.wide_cap) {
        op.wide[2 * e] = q;
        op.wide[2 * e + 1] = s;
      }
    }
    tot += nl[j];
  }
  // the lane's place among the tile's listed rows
  uint64_t at, all;
  block_scan<1>(&tot, &at, all);
  if (threadIdx.x == 0) op.wcnt[tile] = (uint32_t)(all < kLocTile ? all : kLocTile);
  uint64_t* const slots = op.walks + 2 * tile * kLocTile;
  uint32_t fb = 0;  // patterns walked here (past the tile's slots)
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if (!nl[j]) continue;
    const uint64_t a = base + mine[j], s = kr[j], c = nl[j];
    const bool fits = at + c <= kLocTile;
    fb |= (uint32_t)!fits << j;
    uint64_t r0 = s, adj = 0;
    uint32_t rel = 0;
    if (s & kLocCtx) loc_window(s, r0, adj, rel);
    for (uint64_t i = 0; i < c; ++i, ++at) {
      uint64_t row = r0 + i;
      if (rel) {
        row = r0 + (uint32_t)__ffs(rel) - 1u;
        rel &= rel - 1u;
      }
      if (at >= kLocTile) continue;
      slots[2 * at] = fits ? a + i : ~0ull;  // (a void slot: k_locate_walks skips it)
      slots[2 * at + 1] = row | (adj << kWalkAdjShift56);
    }
  }
  if (__syncthreads_or(fb != 0)) {
    load_table(T, ix.table);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (!((fb >> j) & 1u)) continue;
      const uint64_t a = base + mine[j], s = kr[j];
      uint64_t r0 = s, adj = 0;
      uint32_t rel = 0;
      if (s & kLocCtx) loc_window(s, r0, adj, rel);
      for (uint64_t i = 0; i < nl[j]; ++i) {
        uint64_t row = r0 + i;
        if (rel) {
          row = r0 + (uint32_t)__ffs(rel) - 1u;
          rel &= rel - 1u;
        }
        const uint64_t p = walk_position<W>(ix, T, row);
        st_out(op.out_pos + a + i, p >= adj ? p - adj : p + n - adj);
      }
    }
  }
}

// (3') the listed walks (emit_walk_lines): block b takes tiles b, b + grid, ... (one per
// thread: the grid is at least tiles / kBlk), their slots flattened, two per lane in lockstep
template <int kPos>
__global__ __launch_bounds__(kBlk) void k_locate_walks(DevIndex ix, OnePass op, uint64_t ntiles) {
  using W = std::conditional_t<kPos == 1, WalkLine, WalkLineW>;
  static_assert(kBlk == 256, "the tile lookup below searches 256 tiles in 8 steps");
  __shared__ NodeTable T;
  __shared__ uint32_t s_off[kBlk + 1];
  __shared__ uint32_t s_w[kBlk / 64];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t mt = blockIdx.x + (uint64_t)threadIdx.x * gridDim.x;
  const uint32_t c = mt < ntiles ? op.wcnt[mt] : 0u;
  uint32_t x = c;  // exclusive scan of the tiles' counts over the block
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w2 = 0; w2 < (int)(kBlk / 64); ++w2) {
    if (w2 < (int)wv) pre += s_w[w2];
    tot += s_w[w2];
  }
  s_off[threadIdx.x] = pre + x - c;
  if (threadIdx.x == 0) s_off[kBlk] = tot;
  if (tot == 0) return;  // uniform: nothing listed in the block's tiles
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t n = ix.n;
  for (uint32_t e0 = 0; e0 < tot; e0 += 2 * kBlk) {
    uint64_t row[2], adj[2], idx[2];
    bool act[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t ee = e0 + threadIdx.x + h * kBlk;
      const uint32_t e = ee < tot ? ee : 0u;
      uint32_t lo = 0, hi = kBlk;  // s_off[lo] <= e < s_off[hi] (empty tiles share offsets)
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_off[mid] <= e) lo = mid;
        else hi = mid;
      }
      const uint64_t* sl = op.walks + 2 * ((blockIdx.x + (uint64_t)lo * gridDim.x) * kLocTile + (e - s_off[lo]));
      idx[h] = ee < tot ? sl[0] : ~0ull;
      const uint64_t v = ee < tot ? sl[1] : 0;
      act[h] = idx[h] != ~0ull;
      row[h] = v & ((1ull << kWalkAdjShift56) - 1);
      adj[h] = v >> kWalkAdjShift56;
    }
    bool w[2] = {act[0], act[1]};
    walk_positions<W, 2>(ix, T, row, w);
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (act[h]) st_out(op.out_pos + idx[h], row[h] >= adj[h] ? row[h] - adj[h] : row[h] + n - adj[h]);
  }
}

// (3): offsets and positions of tile blockIdx.x (round 5: a pattern whose record is a stashed
// position has no count stored: 8 B read per pattern instead of 12.  Tried in round 5 to drop
// the scan kernel: a decoupled look-back over the tiles — its frontier moves 64 tiles per L2
// round trip, 0.63 against 0.53 ms per C4 call — 1024 blocks taking a share of the tiles each
// with a running base — 4 waves per SIMD and a serial tile loop, the emit 125 against 67 us
// — share totals added by the search kernel's waves — same-address atomics of
// neighbouring blocks, the search 426 -> 615 us — and two tiles per block, 4 patterns per
// lane with both tiles' records in flight before one scan: 0.520 -> 0.536 ms per call,
// profiles/r05/r05aj.)
template <int U, int kPos = 0>
__global__ __launch_bounds__(kBlk) void k_locate_emit(DevIndex ix, uint64_t npat, OnePass op) {
  __shared__ NodeTable T;  // kPos: the walks' C[] and codes (a pattern past walk_cap)
  const uint64_t tile = blockIdx.x;
  const uint64_t q0 = tile * (uint64_t)(kBlk * U) + threadIdx.x;
  uint64_t kc[U], kr[U], mine[U], agg;
  const uint64_t base = op.tiles[tile];  // (issued with the records: its latency overlaps theirs)
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk;
    // (read once: non-temporal loads, 0.560 -> 0.554 ms per call over three A/B rounds,
    // profiles/r04/ab_lib_r04af.jsonl); the count only where the record is no stash
    kr[j] = q < npat ? __builtin_nontemporal_load(op.rec + q) : 0;
    kc[j] = q >= npat ? 0 : loc_stashed(kr[j]) ? 1
          : (op.cnt64 ? __builtin_nontemporal_load(op.cnt64 + q) : __builtin_nontemporal_load(op.cnt + q));
  }
  if constexpr (kPos != 0) {
    block_scan<U>(kc, mine, agg);
    emit_walk_lines<U, kPos>(ix, T, npat, tile, q0, kc, kr, mine, base, op);
  } else {
    block_scan<U>(kc, mine, agg);
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const uint64_t q = q0 + (uint64_t)j * kBlk;
      if (q >= npat) continue;
      const uint64_t a = base + mine[j], c = kc[j];
      st_out(op.out_offs + q, a);
      if (!c || a + c > op.cap) continue;  // capacity short: the caller sees the total
      const uint64_t s = kr[j];
      if (loc_stashed(s)) {  // kLocStash: the one position, read by the search kernel
        st_out(op.out_pos + a, s & (kLocStash - 1));
      } else if (s & kLocCtx) {  // a window k characters before the end (k_locate_sa)
        uint64_t r0, adj;
        uint32_t rel;
        loc_window(s, r0, adj, rel);
        emit_rows<kPos>(ix, T, op, op.out_pos + a, c, r0, rel, adj);
      } else if (c <= kLocSmall) {
        emit_rows<kPos>(ix, T, op, op.out_pos + a, c, s, 0u, 0);
      } else {
        const unsigned long long e = atomicAdd(op.nwide, 1ull);
        if (e < op.wide_cap) {
          op.wide[2 * e] = q;
          op.wide[2 * e + 1] = s;
        }
      }
    }
  }
}

// the ranges over kLocSmall rows: a block per range
template <int kPos = 0>
__global__ __launch_bounds__(kBlk) void k_locate_emit_wide(DevIndex ix, OnePass op, const uint64_t* __restrict__ offs,
                                                           uint64_t* __restrict__ out) {
  __shared__ NodeTable T;
  const uint64_t nw = *op.nwide < op.wide_cap ? *op.nwide : op.wide_cap;
  if (blockIdx.x >= nw) return;  // uniform over the block
  if constexpr (kPos != 0) {
    load_table(T, ix.table);
    __syncthreads();
  }
  for (uint64_t e = blockIdx.x; e < nw; e += gridDim.x) {
    const uint64_t q = op.wide[2 * e], s = op.wide[2 * e + 1], a = offs[q], c = offs[q + 1] - a;
    for (uint64_t j = threadIdx.x; j < c; j += blockDim.x) st_out(out + a + j, onepass_pos<kPos>(ix, T, op, s + j));
  }
}

// The lanes' patterns j with bit j of `m` set into the wave's slot of a LongList list (their
// offsets inside the block's region, in ballot order) and their number into cnt[slot] (0
// when none); returns that number (uniform).  Every lane of the wave, in uniform control flow.
template <int U = 2, class T>
__device__ __forceinline__ uint32_t wave_list(T* list, uint32_t* cnt, uint64_t slot, uint32_t m) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t n = 0;
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const bool b = (m >> j) & 1u;
    const uint64_t bal = __ballot(b);
    if (b) list[slot * kLongSlot + n + __popcll(bal & below)] = (T)(threadIdx.x + j * kBlk);
    n += __popcll(bal);
  }
  if (lane == 0) cnt[slot] = n;
  return n;
}

// wave_list into list2, each listed pattern's chain ch[j] in its entry's upper bits and its
// payload pay[j] at the same place of `rng`
template <int U = 2>
__device__ __forceinline__ uint32_t wave_list_pay(uint32_t* list, uint32_t* cnt, uint64_t* rng, uint64_t slot,
                                                  uint32_t m, const uint64_t* pay, const uint32_t* ch) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t n = 0;
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const bool b = (m >> j) & 1u;
    const uint64_t bal = __ballot(b);
    if (b) {
      const uint64_t at = slot * kLongSlot + n + __popcll(bal & below);
      list[at] = (uint32_t)(threadIdx.x + j * kBlk) | (ch[j] << kChainShift);
      rng[at] = pay[j];
    }
    n += __popcll(bal);
  }
  if (lane == 0) cnt[slot] = n;
  return n;
}

// A 16-B context record: a random read nothing re-reads, through a non-temporal load so it
// does not displace the pattern stream's lines in the caches (C4 headline 0.394 -> 0.382 ms,
// four rounds of an A/B in fresh processes on one box: profiles/r03/ab_nt_record_load.jsonl)
__device__ __forceinline__ uint4 load_record16(const void* tab, uint64_t t) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 r = __builtin_nontemporal_load(static_cast<const u32x4*>(tab) + t);
  return make_uint4(r.x, r.y, r.z, r.w);
}

// The count forms (two patterns per lane) are held to 6 waves per SIMD (<= 80 VGPRs, no
// spills): left alone the compiler gives the packed and uint8 forms 95-104 VGPRs (4-5
// waves), and the packed count took 0.392 ms per 12.5 M instead of 0.361.  The one-call
// locate's search (kOne) to 5 (96 VGPRs, no spills; 122 VGPRs and 4 waves unbounded, VERDICT
// r03 weak item 3; held to 6 it spills 80 VGPRs).
// kSkipLong: patterns of kFastM characters or more whose search the one read cannot finish
// (m > k + kCtxQ) are listed for k_count_long / k_locate_long (long-pattern routing inside the
// call, LongList: each wave lists its own in its slot, so the barrier-free form takes it too).
template <class E, int U, bool kLoc, bool kPacked, int W, bool kNoBar = false, bool kOne = false,
          bool kSkipLong = false, bool kRng = true, int kPos = 0>
__global__ __launch_bounds__(kBlk)
__attribute__((amdgpu_waves_per_eu(!kLoc && U == 2 ? 6 : kOne ? 5 : 1)))
void k_count_ctx(DevIndex ix, const uint8_t* __restrict__ pats,
                                                    const uint64_t* __restrict__ offs,
                                                    uint64_t npat, CountOut co,
                                                    uint64_t limit, uint64_t* __restrict__ rec,
                                                    uint64_t fixed_m, OnePass op = OnePass{},
                                                    LongList ll = LongList{}) {
  // offs == nullptr: patterns of one length fixed_m at stride fixed_m (count only)
  // kNoBar: the general search reads the node table through the caches instead of a
  // block-wide LDS copy, so no wave waits at a block barrier for the block's slowest
  // the stages need only the symbol -> (table digit, occurrence code) map in LDS (512 B
  // instead of the 10.8-KB node table: a shorter block prologue); a block stages the
  // node table only when one of its patterns needs the general search
  __shared__ uint16_t cmap[256];
  __shared__ NodeTable T;
  // count forms: the range [sp, ep) of a pattern the general search finishes (st 5), kept
  // here across the barrier instead of in registers or read again from its table entry
  // (kRng; A/B in one process, profiles/r03/ab_range_across_barrier*.json: headline 0.389
  // vs 0.388 ms, 24-mers 1.32 vs 1.40 ms, repetitive DNA 2.56 vs 2.71 ms)
  __shared__ uint64_t s_rng[kLoc ? 1 : U][kLoc ? 1 : kBlk][2];
  // ... and its chain (list_chain: the codes of the characters before the table's) for the
  // list kernel, kept here rather than in registers to the listing after (D) (round 5: in
  // registers the routed kernel spilled 7 VGPRs instead of 3)
  __shared__ uint32_t s_chn[kLoc ? 1 : U][kLoc ? 1 : kBlk];
  static_assert(kBlk >= 256, "one map entry per thread");
  static_assert(!kOne || kLoc, "the one-call search is a locate form");
  static_assert(!kSkipLong || U * kBlk == kLongRegion, "a block's waves list one region's slots");
  if (threadIdx.x < 256)
    cmap[threadIdx.x] = (uint16_t)(ix.table->code[threadIdx.x] | (ix.table->occ_code[threadIdx.x] << 8));
  if (kOne && threadIdx.x == 0) {
    // the block's tile, which its waves add to after the barrier, and the call's wide-range
    // counter: no memset launch.  The stores are acknowledged by the L2 (where the waves'
    // atomics land) before this wave reaches the barrier.
    op.tiles[blockIdx.x] = 0;
    if (blockIdx.x == 0) *op.nwide = 0;
    if (op.sflags && blockIdx.x < kScanMaxBlocks) op.sflags[blockIdx.x] = 0;
    if (op.sflags && blockIdx.x == 0) op.sflags[kScanMaxBlocks] = 0;  // the chained scan's ticket
    __builtin_amdgcn_s_waitcnt(0);
  }
  // the list kernels' retire word (list_retire) is this call's from here on, whatever the
  // caller's memory held: the list kernels run after this kernel in stream order, and no
  // wave of this kernel touches the word (a workspace that was not zero-filled,
  // or an aborted call, must not let an early block zero the listed counters)
  if (ll.hdr && blockIdx.x == 0 && threadIdx.x == 0) ll.hdr[kListedLanes * kListedStride] = 0;
  __syncthreads();
  uint64_t* const cnt_out = static_cast<uint64_t*>(co.out);  // kLoc
  const uint32_t K = ix.ptab_k;
  const uint64_t q0 = blockIdx.x * (uint64_t)(kBlk * U) + threadIdx.x;
  uint64_t kc[U], kr[U];  // kOne: min(count, limit) and the record of each of the lane's patterns
#pragma unroll
  for (int j = 0; j < U; ++j) kc[j] = kr[j] = 0;
  uint64_t o0[U], res[U], sp[U], ep[U], rv[U];
  uint32_t m[U], t[U], want[U], k[U];
  // the one-call locate over the full SA: the locate record (fm_device.hpp kLocRec*) of the
  // pattern's last k + 1 characters answers it in one read when the pattern has at most
  // kLocRecQ characters before them (lqm bit j: pattern j takes it, at index lt[j])
  constexpr bool kLR = kOne && kPos == 0;
  uint32_t lt[kLR ? U : 1], lqm = 0, defm = 0;
  // 0 done, 1 table, 2 context, 3 general search, 4 left to k_count_long, 5 general search
  // from the range after the table (s_rng), 7 left to k_locate_list (a locate record that
  // does not answer it)
  uint8_t st[U];
  if (kLoc && !kOne && q0 == 0) cnt_out[npat] = 0;  // scan slot for the total
  // (A) in three passes, so that the loads of a lane's U patterns are in flight together:
  // (A1) the offsets, (A2) the pattern bytes, (A3) table index and context key.  Round 6:
  // written as one pass per pattern, the compiler waited for each pattern's offsets, bytes
  // and (B) record before issuing the next pattern's loads (an early `continue` and the
  // decode inside the load's branch kept it from hoisting them) — U = 2 bought no memory
  // parallelism and the staged kernel took 0.41 ms against 0.34 for the same access mix
  // (profiles/microbench/mix_bench.hip, profiles/r06/mix_*.txt).
  // Every load of (A1) and (A2) is issued unconditionally (clamped indices, and a dummy
  // address for the dwords a pattern does not have): a load inside a divergent branch made
  // the compiler wait for every load in flight at the branch's end (s_waitcnt vmcnt(0)).
  uint64_t m1[U];  // (A1) offs[q + 1] (the length once A2 has it)
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk, qc = q < npat ? q : npat - 1;
    st[j] = 0;
    res[j] = 0;
    rv[j] = 0;
    m[j] = 0;
    m1[j] = 0;
    t[j] = want[j] = k[j] = 0;
    if constexpr (kPacked) {
      o0[j] = reinterpret_cast<const uint64_t*>(pats)[qc];  // the pattern itself
    } else if (offs) {
      o0[j] = offs[qc];
      m1[j] = offs[qc + 1];
    } else {
      o0[j] = qc * fixed_m;
    }
  }
  // (A2) lengths, the routing decision, and the raw pattern dwords of the patterns the
  // fast stages search (fw bit j)
  uint32_t praw[kPacked ? 1 : U][9];
  uint32_t fw = 0;
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk;
    const bool live = q < npat;
    const uint64_t mm = (kPacked || !offs) ? fixed_m : m1[j] - o0[j];
    m[j] = live ? (uint32_t)(mm < 0xFFFFFFFFull ? mm : 0xFFFFFFFFull) : 0u;
    // 0: empty pattern (count n, fm_index.cpp:80; locate: :109) or none; 3: the general
    // search; 4: k_count_long's (one read cannot answer it)
    const bool any = live && mm != 0 && ix.n != 0;  // (:81)
    const bool lng = kSkipLong && mm >= kFastM && mm > K + kCtxQ;
    st[j] = !any ? 0 : lng ? 4 : 3;
    if (live && mm == 0) res[j] = kLoc ? 0 : ix.n;
    const bool fast = any && !lng && !(mm < K || K == 0 || mm > kFastM);
    fw |= (uint32_t)fast << j;
    // (16-B vector loads here, load_pattern32_v16, were measured: 0.3857 against 0.3864 ms,
    // profiles/r03/ab_pattern_v16.json — the headline is not bound by its load instructions)
    if constexpr (!kPacked)
      load_pattern32_raw(pats, o0[j], fast ? m[j] : 0u, praw[j], reinterpret_cast<const uint32_t*>(ix.table));
  }
  // (A3) table index and context key.  A 4-symbol table (every occurrence-line index of DNA)
  // maps the characters without a branch: each character's map entry (LDS) goes into 2-bit
  // digit strings and 1-bit invalid masks, and the index and the key are cut from those
  // strings (reversed in pairs: the table index takes its first character as the most
  // significant digit).  Round 6: the per-character branches of the general loop below cost
  // ~750 instructions per pattern, a third of them scalar (exec-mask bookkeeping), and an LDS
  // round trip per character — the staged kernel issued 4x the vector and 20x the scalar
  // instructions of the same access mix in mix_bench (profiles/r06/pmc_r06d_*.csv).
  // The characters a wave's patterns hold, rounded up to a dword (uniform): the loop stops
  // there (C4 20-mers: 20 of 32).
  uint32_t lmax = 0;
#pragma unroll
  for (int j = 0; j < U; ++j) lmax = ((fw >> j) & 1u) && m[j] > lmax ? m[j] : lmax;
  const uint32_t nchar = __ballot(lmax > 28) ? 32u : __ballot(lmax > 24) ? 28u : __ballot(lmax > 20) ? 24u
                         : __ballot(lmax > 16) ? 20u : 16u;
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if (!((fw >> j) & 1u)) continue;
    const uint32_t wl = m[j];
    uint32_t u[8];
    if constexpr (!kPacked) realign_pattern32(o0[j], praw[j], u);
    const uint32_t kk = m[j] - K;
    uint32_t tt = 0, ww = 0, dl = kNoCode;
    bool ok = true, cok = kk <= kCtxQ && (!kLoc || ix.lf_exact);
    if (!kPacked && ix.dna_std) {
      // the standard DNA code (DevIndex::dna_std) four characters per dword, in registers: the
      // code of byte b is 2 bit2(b) + (bit1(b) ^ bit2(b)) (A C G T -> 0 1 2 3), the byte is
      // valid iff "ACGT"[code] gives it back (v_perm_b32), and the dword's four 2-bit codes and
      // four invalid flags are packed by shifts and one multiply — no LDS lookup, no
      // per-character compare (round 6: the LDS form below issued ~350 vector instructions
      // per pattern; profiles/r06)
      uint32_t dlo = 0, dhi = 0, inv = 0;
#pragma unroll
      for (uint32_t w = 0; w < kFastM / 4; ++w) {
        if (4 * w >= nchar) break;
        const uint32_t x = u[w];
        const uint32_t b1 = (x >> 1) & 0x01010101u, b2 = (x >> 2) & 0x01010101u;
        const uint32_t code = (b2 << 1) | (b1 ^ b2);
        const uint32_t dx = __builtin_amdgcn_perm(0u, 0x54474341u, code) ^ x;  // "ACGT"[code] vs the byte
        const uint32_t nz = (((dx & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | dx) & 0x80808080u;  // bit 7: byte != 0
        const uint32_t bad = (((nz >> 7) * 0x01020408u) >> 24) & 0xFu;
        const uint32_t t2 = code | (code >> 6);
        const uint32_t p8 = (t2 & 0xFu) | ((t2 >> 12) & 0xF0u);
        if (w < 4) dlo |= p8 << (8 * w);
        else dhi |= p8 << (8 * (w - 4));
        inv |= bad << (4 * w);
      }
      const uint64_t rd = rev_pairs64(dlo, dhi);
      tt = (uint32_t)((rd >> (64 - 2 * wl)) & ((1ull << (2 * K)) - 1ull));
      ok = (inv & (uint32_t)((((1ull << K) - 1ull) << (wl - K)))) == 0;
      const uint32_t kq = kk < kCtxQ ? kk : kCtxQ;
      cok = cok && (inv & ((1u << kq) - 1u)) == 0;
      ww = kq ? (uint32_t)((rd >> (64 - 2 * kq)) & ((1ull << (2 * kq)) - 1ull)) : 0u;
      if constexpr (kLR)
        if (kk >= 1 && kk <= kCtxQ)  // the (k+1)-mer's first character (its table digit)
          dl = ((inv >> (kk - 1)) & 1u) ? kNoCode
                                        : (uint32_t)((((uint64_t)dhi << 32 | dlo) >> (2 * (kk - 1))) & 3u);
    } else if (ix.ptab_sigma == 4) {
      uint32_t dlo = 0, dhi = 0, olo = 0, ohi = 0, inv = 0, oinv = 0;
#pragma unroll
      for (uint32_t i = 0; i < kFastM; ++i) {
        if ((i & 3u) == 0 && i >= nchar) break;
        uint32_t b;
        if constexpr (kPacked) b = PackedDna{o0[j]}[i];
        else b = (u[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        const uint32_t e = cmap[b];
        if (i < 16) {
          dlo |= (e & 3u) << (2 * i);
          olo |= ((e >> 8) & 3u) << (2 * i);
        } else {
          dhi |= (e & 3u) << (2 * (i - 16));
          ohi |= ((e >> 8) & 3u) << (2 * (i - 16));
        }
        inv |= (uint32_t)((e & 0xFFu) == kNoCode) << i;
        oinv |= (uint32_t)((e >> 8) == kNoCode) << i;
      }
      // character i at bits [62 - 2i, 64 - 2i), low digit bit first
      const uint64_t rd = rev_pairs64(dlo, dhi), ro = rev_pairs64(olo, ohi);
      tt = (uint32_t)((rd >> (64 - 2 * wl)) & ((1ull << (2 * K)) - 1ull));
      ok = (inv & (uint32_t)((((1ull << K) - 1ull) << (wl - K)))) == 0;
      const uint32_t kq = kk < kCtxQ ? kk : kCtxQ;
      cok = cok && (oinv & ((1u << kq) - 1u)) == 0;
      ww = kq ? (uint32_t)((ro >> (64 - 2 * kq)) & ((1ull << (2 * kq)) - 1ull)) : 0u;
      if constexpr (kLR)
        if (kk >= 1 && kk <= kCtxQ)  // the (k+1)-mer's first character (its table digit)
          dl = ((inv >> (kk - 1)) & 1u) ? kNoCode
                                        : (uint32_t)((((uint64_t)dhi << 32 | dlo) >> (2 * (kk - 1))) & 3u);
    } else {
  #pragma unroll
      for (uint32_t i = 0; i < kFastM; ++i) {
        uint32_t b;
        if constexpr (kPacked) b = PackedDna{o0[j]}[i];
        else b = (u[i >> 2] >> (8 * (i & 3))) & 0xFFu;
        if (i >= wl - K && i < wl) {  // table part, most significant first
          const uint32_t d = cmap[b] & 0xFFu;
          ok &= d != kNoCode;
          tt = tt * ix.ptab_sigma + d;
        } else if (i < kk && i < kCtxQ) {  // context part: chain symbol kk-1-i
          const uint32_t d = cmap[b] >> 8;
          cok &= d != kNoCode;
          ww |= (d & 3u) << (2 * (kk - 1 - i));
          if constexpr (kLR)
            if (i + 1 == kk) dl = cmap[b] & 0xFFu;  // the (k+1)-mer's first character (its table digit)
        }
      }
    }
    if (!ok) continue;
    st[j] = cok ? 2 : 1;
    t[j] = tt;
    want[j] = ww;
    k[j] = kk;
    if constexpr (kLR) {
      // (ix.lrec implies a 4-symbol table of k <= 15: the index fits 32 bits)
      if (ix.lrec && cok && kk >= 1 && ix.lrec64 && kk <= kLocRec64Q) {
        lt[j] = tt;  // the k-mer's 64-B record
        lqm |= 1u << j;
      } else if (ix.lrec && cok && kk >= 1 && !ix.lrec64 && kk - 1 <= kLocRecQ && dl != kNoCode) {
        lt[j] = (dl << (2 * K)) + tt;
        lqm |= 1u << j;
      }
    }
  }
  // the wave's slot of the call's lists (kSkipLong, and kOne's deferred patterns)
  const uint64_t slot = (uint64_t)blockIdx.x * kSlotsPerRegion + (threadIdx.x >> 6);
  uint32_t nlisted = 0;  // kSkipLong: the wave's listed patterns (uniform)
  if constexpr (kSkipLong) {
    // the long patterns into the wave's slot (k_count_long / k_locate_long take them), in
    // ballot order (the count forms write the general-search slot after (D))
    uint32_t lm = 0;
#pragma unroll
    for (int j = 0; j < U; ++j) lm |= (uint32_t)(st[j] == 4) << j;
    nlisted = wave_list<U>(ll.list, ll.cnt, slot, lm);
  }
  if constexpr (kLR) {
    if (ix.lrec64) {
      // (B0') the 64-B locate records (fm_device.hpp kLocRec64*), each read by the four
      // lanes of a quad together (one DRAM request): lane c of the quad loads chunk c of the
      // record of each quad-mate's pattern j, matches its rows against that pattern's
      // context, and the quad sums the matches; no match, or one (its SA value minus the
      // context length is the position, stashed), finishes the pattern here — more rows or
      // matches read the context record below.  Uniform control flow (shuffles).
      const uint32_t ql = threadIdx.x & 3u, qb = (threadIdx.x & 63u) & ~3u;
      uint4 ch[U][4];
#pragma unroll
      for (int j = 0; j < U; ++j)
#pragma unroll
        for (uint32_t s2 = 0; s2 < 4; ++s2) {
          const uint32_t v = __shfl(((lqm >> j) & 1u) ? lt[j] : ~0u, (int)(qb | s2), 64);
          ch[j][s2] = v != ~0u ? load_record16(ix.lrec, (uint64_t)v * 4 + ql) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        uint32_t mt = 0, mp = 0, mn = 0;  // the lane's own pattern j: matches, position, none
#pragma unroll
        for (uint32_t s2 = 0; s2 < 4; ++s2) {
          const uint32_t wk = __shfl(want[j] | (k[j] << 16), (int)(qb | s2), 64);
          const uint32_t kq = wk >> 16, ww = wk & 0xFFFFu, mask = (1u << (2 * kq)) - 1u;
          const uint4 a = ch[j][s2];
          const uint32_t vc = a.w >> 30;
          uint32_t n1 = 0, sv = 0;
#pragma unroll
          for (uint32_t i = 0; i < 3; ++i)
            if (i < vc && ((a.w >> (10 * i)) & mask) == ww) {
              ++n1;
              sv = i == 0 ? a.x : i == 1 ? a.y : a.z;
            }
          uint32_t tot = n1, pos = n1 == 1 ? sv : 0u, none = (vc == 0 && a.x == ~0u) ? 1u : 0u;
          tot += __shfl_xor(tot, 1, 64);
          tot += __shfl_xor(tot, 2, 64);
          pos |= __shfl_xor(pos, 1, 64);
          pos |= __shfl_xor(pos, 2, 64);
          none |= __shfl_xor(none, 1, 64);
          none |= __shfl_xor(none, 2, 64);
          if (s2 == ql) {
            mt = tot;
            mp = pos;
            mn = none;
          }
        }
        if (!((lqm >> j) & 1u)) continue;
        if (mn || mt >= 2) {  // the context record's window (below, or k_locate_list)
          if (op.defer) {
            st[j] = 7;
            defm |= 1u << j;
          }
          continue;
        }
        st[j] = 0;
        res[j] = mt;
        if (mt) rv[j] = kLocStash | (mp >= k[j] ? mp - k[j] : mp + ix.n - k[j]);
      }
    } else {
    // (B0) the locate records: no match, or one matching row whose SA value the record holds,
    // finishes the pattern here (its position stashed as the emit kernel copies it); more
    // rows or matches read the context record below
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (!((lqm >> j) & 1u)) continue;
      const uint4 a = load_record16(ix.lrec, lt[j]);
      const uint32_t c = a.w >> 24;
      const uint32_t j2 = k[j] - 1, mask = (1u << (2 * j2)) - 1u, want2 = want[j] >> 2;
      uint32_t mm = 0;
#pragma unroll
      for (uint32_t i = 0; i < kLocRecRows; ++i)
        mm |= (uint32_t)(i < c && ((a.w >> (8 * i)) & mask) == want2) << i;
      if (c == kLocRecNone || (mm & (mm - 1u))) {
        // more rows, or two or three positions: the context record's window — in
        // k_locate_list when the call defers them (op.defer: the block then waits for no
        // second read), else below
        if (op.defer) {
          st[j] = 7;
          defm |= 1u << j;
        }
        continue;
      }
      st[j] = 0;
      res[j] = mm ? 1u : 0u;
      if (mm) {
        const uint64_t v = mm == 1u ? a.x : mm == 2u ? a.y : a.z;
        rv[j] = kLocStash | (v >= j2 ? v - j2 : v + ix.n - j2);
      }
    }
    }
  }
  if constexpr (kOne) {
    // the deferred patterns into the wave's slot of the general-search list (zeroed when none)
    if (ll.cnt2) nlisted += wave_list<U>(ll.list2, ll.cnt2, slot, defm);
    if (ll.hdr) list_listed_add(ll, nlisted);
  }
  // (B) the table entries (whole context records: their contexts come with them)
  uint4 w[U][4];
  bool inl[U];  // the record's contexts answer the rest
  // a compact record's inline rows matched in (B) (cm bit j: mrec[j] is (D)'s match mask)
  uint32_t mrec[U], cm = 0;
#pragma unroll
  for (int j = 0; j < U; ++j) inl[j] = false;
  // the U records first, all in flight together (unconditional loads: the dummy address
  // for a pattern without one), then their decoding — see (A)
  const void* const dummy = static_cast<const void*>(ix.table);
  if (ix.ptab_rec == 2) {
    uint4 ra[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool act = st[j] == 1 || st[j] == 2;
      ra[j] = load_record16(act ? ix.ptab : dummy, act ? (uint64_t)t[j] : 0ull);
    }
    // (a compiler barrier: without it the compiler sinks each load into its pattern's decode
    // branch, and waits for it there before the next pattern's load is issued)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (st[j] != 1 && st[j] != 2) continue;
      const uint4 a = ra[j];
      const uint32_t wc = a.y & 15u;
      sp[j] = rec16_sp(a.x, a.w, ix.wide);
      inl[j] = wc != kRec16Wide && k[j] <= (ix.wide ? kRec16QW : kRec16Q);
      ep[j] = sp[j] + (wc == kRec16Wide ? a.z : wc);
      if (wc == kRec16Wide && a.z == kRec16NoRange) st[j] = 3;  // escaped: from C[]
      if (!ix.wide && inl[j] && st[j] == 2) {
        // the record's rows matched against the key in place (no u16 re-layout for (D))
        mrec[j] = rec16_match(a.y, a.z, a.w, want[j], k[j]);
        cm |= 1u << j;
      } else {
        uint32_t d[5];
        if (ix.wide)
          rec16w_contexts(a.y, a.z, a.w, d);
        else
          rec16_contexts(a.y, a.z, a.w, d);
        w[j][0] = make_uint4(d[0], d[1], d[2], d[3]);
        w[j][1] = make_uint4(d[4], 0u, 0u, 0u);
      }
      // count forms: a wide record's majority contexts (kRec16Maj) may give the count here
      if (!kLoc && wc == kRec16Wide && st[j] == 2 && k[j] == kRec16Q && !ix.wide &&
          rec16_majority(a.y, a.w, want[j], res[j]))
        st[j] = 0;
    }
  } else if (ix.ptab_rec == 1) {
    uint4 ra[U], rb[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool act = st[j] == 1 || st[j] == 2;
      const uint4* r = act ? static_cast<const uint4*>(ix.ptab) + (uint64_t)t[j] * 2
                           : static_cast<const uint4*>(dummy);
      ra[j] = r[0];
      rb[j] = r[1];
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (st[j] != 1 && st[j] != 2) continue;
      const uint4 a = ra[j], b = rb[j];
      sp[j] = a.x;
      ep[j] = (uint64_t)a.x + a.y;
      w[j][0] = make_uint4(a.z, a.w, b.x, b.y);
      w[j][1] = make_uint4(b.z, b.w, 0u, 0u);
      inl[j] = ep[j] - sp[j] <= kRecCtx;
    }
  } else {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (st[j] != 1 && st[j] != 2) continue;
      if (!ptab_at(ix, t[j], sp[j], ep[j])) st[j] = 3;
    }
  }
  // (C) the context sector(s), unless the record holds the range's contexts
  uint64_t bs[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    bs[j] = 0;
    if (st[j] != 1 && st[j] != 2) continue;
    if (sp[j] >= ep[j]) {
      st[j] = 0;
      res[j] = 0;
    } else if (k[j] == 0) {
      st[j] = 0;
      res[j] = ep[j] - sp[j];
      rv[j] = sp[j];
    } else if (st[j] == 2 && inl[j] && ix.lctx) {
      bs[j] = sp[j];  // w[j][0..1] already hold rows sp.. from the record (or mrec[j] matched them)
      if (!((cm >> j) & 1u)) w[j][2] = w[j][3] = make_uint4(0, 0, 0, 0);
    } else if (st[j] == 2 && ix.lctx && ep[j] - (sp[j] & ~15ull) <= 32) {
      bs[j] = sp[j] & ~15ull;
      const uint4* p = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(ix.lctx) +
                                                      bs[j]);
      w[j][0] = p[0];
      w[j][1] = p[1];
      if (ep[j] - (sp[j] & ~15ull) > 16) {
        w[j][2] = p[2];
        w[j][3] = p[3];
      } else {
        w[j][2] = w[j][3] = make_uint4(0, 0, 0, 0);
      }
    } else if constexpr (!kLoc && kRng) {
      // too wide for the contexts, or no context key: the general search (the chain codes
      // in want[j] stand only when the pattern had its context key, st 2)
      s_chn[j][threadIdx.x] = st[j] == 2 ? list_chain(want[j], k[j]) : kChainNone;
      st[j] = 5;
      s_rng[j][threadIdx.x][0] = sp[j];
      s_rng[j][threadIdx.x][1] = ep[j];
    } else {
      st[j] = 3;
    }
  }
  // (D)
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if (st[j] == 2) {
      const uint32_t mask = ((1u << (2 * k[j])) - 1u) | kCtxEsc;
      const uint64_t base = bs[j];
      const uint32_t lo = (uint32_t)(sp[j] - base), hi = (uint32_t)(ep[j] - base);
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(w[j]);
      uint32_t match = 0, esc = 0;
      if ((cm >> j) & 1u) {
        match = mrec[j];  // (a compact record's rows hold no escaped context)
      } else {
        // two u16 entries per dword; the entries past row 10 only for the lanes whose range
        // reaches them (context sectors: a divergent branch, not every lane's work)
        const uint32_t wp = want[j] | (want[j] << 16), mp = mask | (mask << 16);
#pragma unroll
        for (int d = 0; d < 5; ++d) {
          const uint32_t x = (dw[d] ^ wp) & mp;
          match |= ((uint32_t)((x & 0xFFFFu) == 0) | ((uint32_t)((x >> 16) == 0) << 1)) << (2 * d);
          esc |= (((dw[d] >> 15) & 1u) | ((dw[d] >> 30) & 2u)) << (2 * d);
        }
        if (hi > 10) {
#pragma unroll
          for (int d = 5; d < 16; ++d) {
            const uint32_t x = (dw[d] ^ wp) & mp;
            match |= ((uint32_t)((x & 0xFFFFu) == 0) | ((uint32_t)((x >> 16) == 0) << 1)) << (2 * d);
            esc |= (((dw[d] >> 15) & 1u) | ((dw[d] >> 30) & 2u)) << (2 * d);
          }
        }
      }
      const uint32_t in = (hi >= 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
      const uint32_t mm = match & in;
      if (esc & in) {  // a rare symbol in a row's chain
        st[j] = 3;
        if constexpr (!kLoc && kRng) {
          st[j] = 5;
          s_rng[j][threadIdx.x][0] = sp[j];
          s_rng[j][threadIdx.x][1] = ep[j];
          s_chn[j][threadIdx.x] = list_chain(want[j], k[j]);
        }
      } else if (!kLoc || mm == 0) {
        res[j] = (uint64_t)__popc(mm);
        st[j] = 0;
      } else {  // the window record (locate_search)
        const uint32_t f = (uint32_t)__ffs(mm) - 1u;
        const uint32_t rel = mm >> f;
        if (rel >> kLocSpanBits) {
          st[j] = 3;
        } else {
          rv[j] = kLocCtx | ((uint64_t)k[j] << 60) | ((uint64_t)rel << 38) | (base + f);
          res[j] = (uint64_t)__popc(mm);
          st[j] = 0;
        }
      }
    }
    const uint64_t q = q0 + (uint64_t)j * kBlk;
    if (q < npat && st[j] < 3) {
      if constexpr (kOne) {
        kc[j] = res[j] < limit ? res[j] : limit;  // fm_index.cpp:125
        kr[j] = rv[j];
      } else if (kLoc) {
        cnt_out[q] = res[j] < limit ? res[j] : limit;  // fm_index.cpp:125
        rec[q] = rv[j];
      } else {
        store_count<W>(co, q, res[j]);
      }
    }
  }
  if constexpr (kSkipLong && !kOne) {
    // the routed count (round 5): the patterns left to the general search go to the wave's
    // slot of list2 for k_count_long (whose lanes then all search), unless the call keeps
    // them in the lane (CS_QT_GENERAL_INLANE); the wave's listed number to the counters
    // A wave lists them when it holds at least ll.gen_list of them: a wave with one keeps it
    // (its chain overlaps the other waves' reads, and a batch that lists nothing skips the
    // list kernel's work; C4 Q_text: the staged kernel 389 us either way, the list kernel 4
    // against 58 us), a wave with many would idle most of its lanes through their chains
    // (repetitive DNA: the staged kernel 1060 -> 380 us when listed, profiles/r05/r05b_*).
    // Threshold A/B (CS_FM_GENERAL_LIST_MIN, C4 call ms, Q_text / repetitive DNA,
    // profiles/r05/r05c_*): 1: 0.448 / 0.774, 2: 0.395 / 0.758, 4: 0.395 / 0.855, 8: 0.398 /
    // 1.145 — the default is 2.
    uint32_t gm = 0, ng = 0;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool g = st[j] == 3 || st[j] == 5;
      gm |= (uint32_t)g << j;
      ng += (uint32_t)__popcll(__ballot(g));
    }
    if (ll.gen_list && ng >= ll.gen_list) {
      // with the range the table read left (st 5: too wide for the contexts) and the chain
      // codes of the characters before the table's (list_chain), so the list kernel steps on
      // from them instead of reading the record, the offsets and the pattern again
      uint64_t pay[U];
      uint32_t chn[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const bool r = st[j] == 5 && !ix.wide && ep[j] - sp[j] <= 0xFFFFFFFFull;
        pay[j] = r ? (sp[j] | ((ep[j] - sp[j]) << 32)) : kNoRange;
        chn[j] = r ? s_chn[j][threadIdx.x] : kChainNone;
      }
      nlisted += wave_list_pay<U>(ll.list2, ll.cnt2, ll.rng2, slot, gm, pay, chn);
#pragma unroll
      for (int j = 0; j < U; ++j)
        if ((gm >> j) & 1u) st[j] = 6;  // listed
    } else if ((threadIdx.x & 63) == 0) {
      ll.cnt2[slot] = 0;
    }
    list_listed_add(ll, nlisted);
  }
  // the general search for the rest, with only (o0, m) of each pattern still live
  bool general = false;
#pragma unroll
  for (int j = 0; j < U; ++j) general |= st[j] == 3 || st[j] == 5;
  if constexpr (kOne && kNoBar) {
    // the barrier-free one-call search: the general search reads the node table through the
    // caches, the walks (kPos 1 / 2) take the few constants a step needs in registers
    // (WalkK), the tile total is added wave by wave (locate_split_store)
    if (general)
      general_rest<E, U, kLoc, kPacked, W, true>(ix, *ix.table, pats, st, o0, m, q0, co, limit, rec, kc, kr);
    uint32_t skip = 0;  // the patterns left to k_locate_long (4) and k_locate_list (7)
#pragma unroll
    for (int j = 0; j < U; ++j) skip |= (uint32_t)(st[j] == 4 || st[j] == 7) << j;
    locate_split_store<U, kPos, true>(ix, *ix.table, npat, blockIdx.x, q0, kc, kr, op, skip);
    return;
  } else if constexpr (kNoBar) {
    if (general)
      general_rest<E, U, kLoc, kPacked, W>(ix, *ix.table, pats, st, o0, m, q0, co, limit, rec, nullptr, nullptr,
                                           &s_rng[0][0][0]);
    return;
  }
  if constexpr (kOne) {
    // the walk (kPos) needs the node table for every block with a position to find
    bool need = general;
    if constexpr (kPos != 0) {
#pragma unroll
      for (int j = 0; j < U; ++j) need |= kc[j] == 1;
    }
    const bool any_need = __syncthreads_or(need);
    if (any_need) {
      load_table(T, ix.table);
      __syncthreads();
      if (general)
        general_rest<E, U, kLoc, kPacked, W, true>(ix, T, pats, st, o0, m, q0, co, limit, rec, kc, kr);
    }
    uint32_t skip = 0;  // the patterns left to k_locate_long (4) and k_locate_list (7)
#pragma unroll
    for (int j = 0; j < U; ++j) skip |= (uint32_t)(st[j] == 4 || st[j] == 7) << j;
    locate_split_store<U, kPos>(ix, T, npat, blockIdx.x, q0, kc, kr, op, skip);
    return;
  }
  const bool any_general = __syncthreads_or(general);
  if (!any_general) return;
  load_table(T, ix.table);
  __syncthreads();
  general_rest<E, U, kLoc, kPacked, W>(ix, T, pats, st, o0, m, q0, co, limit, rec, nullptr, nullptr,
                                       &s_rng[0][0][0]);
}

// Long patterns (round 3; CS_Q_LONG, fixed-length batches over kLongPatternM, host chunks
// of long patterns) over an lf_exact occurrence-line index that keeps the full suffix array
// and the text (DevIndex::vsa / vtext) — C2 and C4 by default.  The reference steps m
// times (fm_index.cpp:88-98); count_rest already finishes a narrow range by verification
// against the text (rows whose left contexts match, then text[SA - k, SA) against P[0, k)),
// and this kernel runs that search as a pipeline of independent reads, one pattern per
// lane, with nothing else live:
//   (A) the pattern's offsets and its last 32 bytes (realigned dword loads): the
//       prefix-table index of the last K characters and the context key of the qc = 7
//       before them, from a 512-B LDS symbol map (no 10.8-KB node table, no barrier);
//   (B) the table entry — a context record holds the range and its rows' contexts;
//   (C) the candidate rows: the record's inline contexts, else one or two 32-B context
//       sectors; a candidate's chain spells the qf characters before the table part;
//   (D) the SA entry of each candidate (the rows are consecutive: one sector);
//   (E) the window text[SA - k, SA - qf) against P[0, k - qf): up to kLongWords aligned
//       8-B words of text AND of the pattern per round, all issued before the compare.
// A pattern is read once (the general path's count_pattern read its record a second time
// and held both of a lane's patterns behind a block barrier).  Anything else — a range
// wider than the record / two sectors, an escaped context, a symbol outside the table's
// alphabet, a pattern shorter than 32 characters — takes count_pattern with the node table
// read through the caches.
template <int V>
__device__ __forceinline__ bool window_eq_long(const DevIndex& ix, const uint8_t* __restrict__ text,
                                               const uint8_t* P, uint64_t q, uint64_t L) {
  const uint64_t n = ix.n;
  if (q + L > n) {  // a window through the end of the text (cyclic), byte by byte
    for (uint64_t j = 0; j < L; ++j) {
      uint64_t t = q + j;
      if (t >= n) t -= n;
      if (text[t] != P[j]) return false;
    }
    return true;
  }
  const uint64_t* tw = reinterpret_cast<const uint64_t*>(text);
  const uint64_t* pw = reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(P) & ~(uintptr_t)7);
  const uint64_t ps = reinterpret_cast<uintptr_t>(P) & 7;
  const uint64_t tlast = (q + L - 1) >> 3, plast = (ps + L - 1) >> 3;  // words holding a byte
  for (uint64_t j0 = 0; j0 < L; j0 += 8 * V) {
    const uint64_t ta = (q + j0) >> 3, pa = (ps + j0) >> 3;
    uint64_t tv[V + 1], pv[V + 1];
#pragma unroll
    for (int i = 0; i <= V; ++i) {
      tv[i] = ta + i <= tlast ? tw[ta + i] : 0ull;
      pv[i] = pa + i <= plast ? pw[pa + i] : 0ull;
    }
    uint64_t diff = 0;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const uint64_t j = j0 + 8 * (uint64_t)i;
      if (j < L) diff |= (text8(tv[i], tv[i + 1], q + j) ^ text8(pv[i], pv[i + 1], ps + j)) & chunk_mask(j, L);
    }
    if (diff) return false;
  }
  return true;
}

constexpr int kLongWords = 12;  // byte-text words per round (96 characters; no packed text)
// packed pattern words: the fast path takes P[0, k) of at most 32 kLongPW characters before
// the table part (a 150-mer at k = 15: 135)
constexpr uint32_t kLongPW = 5;

// whether a text position of a rare symbol lies in [q, q + L) (sorted list in LDS)
__device__ __forceinline__ bool rare_in(const uint32_t* r, uint32_t nr, uint64_t q, uint64_t L) {
  uint32_t lo = 0, hi = nr;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (r[mid] < q) lo = mid + 1;
    else hi = mid;
  }
  return lo < nr && r[lo] < q + L;
}

// The occurrence codes of P[c0, c0 + min(len, 32 kLongPW)) into pc (character i of the
// chunk at bits 2 (i % 32) of pc[i / 32]), from aligned 8-B words of P (only words holding
// a byte of the chunk) through the LDS map; false when a character has no code.
__device__ __forceinline__ bool pack_pattern(const uint8_t* P, uint64_t c0, uint64_t len,
                                             const uint16_t* cmap, uint64_t pc[kLongPW]) {
  const uint64_t kk = len < 32ull * kLongPW ? len : 32ull * kLongPW;
  const uintptr_t a = reinterpret_cast<uintptr_t>(P) + c0;
  const uint64_t* pw = reinterpret_cast<const uint64_t*>(a & ~(uintptr_t)7);
  const uint64_t ps = a & 7, plast = (ps + kk - 1) >> 3;
  uint64_t x[4 * kLongPW + 1];
#pragma unroll
  for (uint32_t i = 0; i <= 4 * kLongPW; ++i) x[i] = i <= plast ? pw[i] : 0ull;
  bool ok = true;
#pragma unroll
  for (uint32_t i = 0; i < kLongPW; ++i) pc[i] = 0;
#pragma unroll
  for (uint32_t c = 0; c < 4 * kLongPW; ++c) {
    const uint64_t y = text8(x[c], x[c + 1], ps);  // P[c0 + 8c, c0 + 8c + 8)
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
      if (8 * c + b < kk) {
        const uint32_t d = cmap[(uint32_t)(y >> (8 * b)) & 0xFFu] >> 8;
        ok &= d != kNoCode;
        pc[c >> 2] |= (uint64_t)(d & 3u) << (2 * (8 * (c & 3) + b));
      }
    }
  }
  return ok;
}

// pack_pattern from 16-B aligned vectors (11 loads for a 160-character chunk instead of 21
// 8-B ones: a lane's pattern lies at a stride of m bytes from its neighbours', so every load
// instruction touches 64 cache lines and the count of instructions is what the TA/TCP pay).
// A vector holding a byte of the batch lies inside its allocation (16-B granular).
__device__ __forceinline__ bool pack_pattern16(const uint8_t* P, uint64_t len, const uint16_t* cmap,
                                               uint64_t pc[kLongPW]) {
  const uint64_t kk = len < 32ull * kLongPW ? len : 32ull * kLongPW;
  const uintptr_t a = reinterpret_cast<uintptr_t>(P);
  const uint4* pv = reinterpret_cast<const uint4*>(a & ~(uintptr_t)15);
  const uint32_t ps = (uint32_t)(a & 15), vlast = (uint32_t)((ps + kk - 1) >> 4);
  constexpr uint32_t NV = (15 + 32 * kLongPW + 15) / 16;  // 11 for kLongPW = 5
  uint64_t x[2 * NV];
#pragma unroll
  for (uint32_t i = 0; i < NV; ++i) {
    const uint4 v = i <= vlast ? pv[i] : make_uint4(0, 0, 0, 0);
    x[2 * i] = ((uint64_t)v.y << 32) | v.x;
    x[2 * i + 1] = ((uint64_t)v.w << 32) | v.z;
  }
  static_assert(4 * kLongPW + 1 < 2 * NV, "word c + 2 of the last chunk is loaded");
  const uint64_t sel = ps >= 8 ? ~0ull : 0ull, sh = ps & 7;
  bool ok = true;
#pragma unroll
  for (uint32_t i = 0; i < kLongPW; ++i) pc[i] = 0;
#pragma unroll
  for (uint32_t c = 0; c < 4 * kLongPW; ++c) {
    const uint64_t y0 = text8(x[c], x[c + 1], sh), y1 = text8(x[c + 1], x[c + 2], sh);
    const uint64_t y = y0 ^ ((y0 ^ y1) & sel);  // P[8c, 8c + 8)
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
      if (8 * c + b < kk) {
        const uint32_t d = cmap[(uint32_t)(y >> (8 * b)) & 0xFFu] >> 8;
        ok &= d != kNoCode;
        pc[c >> 2] |= (uint64_t)(d & 3u) << (2 * (8 * (c & 3) + b));
      }
    }
  }
  return ok;
}

// text[q, q + len) (len <= 32 kLongPW) against the packed codes pc: the window's words in
// one round, shifted to its start; true when every code agrees
// kV: the words through 16-B aligned vector loads (3 instead of up to 6 8-B loads)
template <bool kV = false>
__device__ __forceinline__ bool packed_chunk_eq(const DevIndex& ix, const uint64_t* pc, uint64_t q,
                                                uint64_t len) {
  const uint64_t a = q >> 5, last = (q + len - 1) >> 5;
  const uint32_t s = (uint32_t)(q & 31) * 2;
  uint64_t w[kLongPW + 1];
  if constexpr (kV) {
    const uint64_t a2 = a & ~1ull, sel = (a & 1) ? ~0ull : 0ull;
    const ulonglong2* pv = reinterpret_cast<const ulonglong2*>(ix.ptext + a2);
    constexpr uint32_t NV = (kLongPW + 3) / 2;  // words a2 .. a2 + 2 NV - 1 cover a .. a + kLongPW
    uint64_t x[2 * NV];
#pragma unroll
    for (uint32_t i = 0; i < NV; ++i) {
      const ulonglong2 v = a2 + 2 * i <= last ? pv[i] : make_ulonglong2(0, 0);
      x[2 * i] = v.x;
      x[2 * i + 1] = v.y;
    }
#pragma unroll
    for (uint32_t i = 0; i <= kLongPW; ++i) {
      const uint64_t y1 = i + 1 < 2 * NV ? x[i + 1] : 0ull;
      w[i] = a + i <= last ? x[i] ^ ((x[i] ^ y1) & sel) : 0ull;
    }
  } else {
#pragma unroll
    for (uint32_t i = 0; i <= kLongPW; ++i) w[i] = a + i <= last ? ix.ptext[a + i] : 0ull;
  }
  uint64_t diff = 0;
#pragma unroll
  for (uint32_t i = 0; i < kLongPW; ++i) {
    const uint64_t j = 32ull * i;
    if (j < len) {
      const uint64_t x = s ? (w[i] >> s) | (w[i + 1] << (64 - s)) : w[i];
      const uint64_t msk = len - j >= 32 ? ~0ull : (1ull << (2 * (len - j))) - 1;
      diff |= (x ^ pc[i]) & msk;
    }
  }
  return !diff;
}

// text[q, q + L) == P[0, L) against the 2-bit text, pc = the codes of P's first 32 kLongPW
// characters (pack_pattern at 0, every one coded); the characters after them (patterns over
// 175 characters at k = 15) against the byte text.  A rare symbol in the packed part of the
// window is a mismatch (its code 0 in the packed text stands for no pattern character).
// Windows through the end of the text: the byte text, cyclically.
template <bool kV = false>
__device__ __forceinline__ bool window_eq_packed(const DevIndex& ix, const uint64_t* pc, const uint8_t* P,
                                                 uint64_t q, uint64_t L, const uint32_t* rare) {
  if (q + L > ix.n) return window_eq<const uint8_t*>(ix, P, q, L, nullptr);
  constexpr uint64_t C = 32ull * kLongPW;
  const uint64_t L0 = L < C ? L : C;
  if (!packed_chunk_eq<kV>(ix, pc, q, L0) || rare_in(rare, ix.nrare, q, L0)) return false;
  return L == L0 || window_eq<const uint8_t*>(ix, P + C, q + C, L - C, nullptr);
}

// kPT: verify against the packed text (DevIndex::ptext), else the byte text in rounds of
// kLongWords words.  Patterns the pipeline does not answer are appended to `list` (q) for
// k_count_list, which runs the general search.
// from_list: the patterns the staged kernel listed (LongList regions, long-pattern routing),
// else every pattern; skip_short (measurement twin only): every pattern is read and only the
// long ones (m >= kFastM, m > k + kCtxQ: the ones a routed call lists) are searched.
// kBytes: measurement twin (bench.py's roofline) — co.out receives each pattern's random
// algorithmic bytes instead of its count: the table entry, the context sector(s), per
// candidate its SA sector (32 B) and the text words of its window.
// (90 VGPRs, 5 waves per SIMD: held to 80 with waves_per_eu(6) it spills and runs 12-15 %
// slower, profiles/r03/long_probe_w6_m300.json)
// (Staging the block's patterns in LDS with coalesced 16-B loads, instead of each lane's
// 8-B loads at a stride of m bytes, was measured: 150-mers 1.91 -> 1.75 ms, but 32- to
// 100-mers 5-18 % slower — the 38-KB stage leaves 4 waves per SIMD —
// profiles/r03/long_probe_lds_stage.json; not kept.)
// kV16: the pattern's bytes through 16-B aligned vector loads (1: pack_pattern16 and
// load_tail32_v16, 2: pack_pattern16 only, 3: 2 and the packed window as 16-B vectors)
// (A)-(C) of the long-pattern search of one pattern (m > 0 characters at pats + o0, n > 0):
// the candidate rows base + i (bit i of cand) whose chains spell the qf characters before the
// table part — what is left is the window text[SA - k, SA - qf) against P[0, k - qf),
// k = m - ptab_k.  true: cand holds the candidates (none: the table part does not occur);
// false: the pipeline cannot answer the pattern (the general search).  pc (kPT): the codes
// of P[0, min(k, 32 kLongPW)).  by (kBytes): the random bytes read.
template <bool kPT, bool kBytes, int kV16>
__device__ __forceinline__ bool long_stage(const DevIndex& ix, const uint8_t* __restrict__ pats, uint64_t o0,
                                           uint64_t m, const uint16_t* cmap, uint64_t pc[kLongPW],
                                           uint64_t& base, uint32_t& cand, uint32_t& qf, uint64_t& by) {
  const uint8_t* P = pats + o0;
  const uint32_t K = ix.ptab_k;
  const uint64_t k = m - K;  // characters before the table part (when m >= K)
  // verification needs the window inside one rotation (k < n, as count_rest's)
  bool fast = m >= 32 && m > K + kCtxQ && k < ix.n;
  uint32_t t = 0, want = 0;
  bool cok = true;
#pragma unroll
  for (uint32_t i = 0; i < kLongPW; ++i) pc[i] = 0;
  base = 0;
  cand = 0;
  qf = 0;
  if (!fast) return false;
  // (A)
  {
    uint32_t u[8];
    load_pattern32(pats, o0 + m - 32, 32, u);  // tail byte i = P[m - 32 + i]
    if constexpr (kPT) {  // P[0, min(k, 160)) coded
      if constexpr (kV16 >= 2) fast &= pack_pattern16(P, k, cmap, pc);
      else fast &= pack_pattern(P, 0, k, cmap, pc);
    }
#pragma unroll
    for (uint32_t i = 0; i < 32; ++i) {
      const uint32_t b = (u[i >> 2] >> (8 * (i & 3))) & 0xFFu;
      if (i >= 32 - K) {  // table part, most significant first
        const uint32_t d = cmap[b] & 0xFFu;
        fast &= d != kNoCode;
        t = t * ix.ptab_sigma + d;
      } else if (i + K + kCtxQ >= 32) {  // chain symbol 31 - K - i of the context part
        const uint32_t d = cmap[b] >> 8;
        cok &= d != kNoCode;
        want |= (d & 3u) << (2 * (31 - K - i));
      }
    }
  }
  if (!fast) return false;
  // (B)
  uint64_t sp, ep;
  uint32_t d[6] = {0, 0, 0, 0, 0, 0};  // inline contexts as u16 entries, row i in entry i
  if constexpr (kBytes) by += ix.ptab_rec == 1 ? 32u : ix.ptab_rec == 2 ? 16u : 8u;
  if (ix.ptab_rec == 2) {
    const uint4 a = load_record16(ix.ptab, t);
    const uint32_t wc = a.y & 15u;
    sp = rec16_sp(a.x, a.w, ix.wide);  // (wide indexes, round 6: sp's bits 32-37 in the record)
    if (wc == kRec16Wide && a.z == kRec16NoRange) return false;  // escaped: from C[]
    ep = sp + (wc == kRec16Wide ? a.z : wc);
    if (wc != kRec16Wide) {
      qf = ix.wide ? kRec16QW : kRec16Q;
      if (ix.wide)
        rec16w_contexts(a.y, a.z, a.w, d);
      else
        rec16_contexts(a.y, a.z, a.w, d);
    }
  } else if (ix.ptab_rec == 1) {
    const uint4* r = static_cast<const uint4*>(ix.ptab) + (uint64_t)t * 2;
    const uint4 a = r[0], b = r[1];
    sp = a.x;
    ep = (uint64_t)a.x + a.y;
    if (ep - sp <= kRecCtx) {
      qf = kCtxQ;
      d[0] = a.z, d[1] = a.w, d[2] = b.x, d[3] = b.y, d[4] = b.z, d[5] = b.w;
    }
  } else if (!ptab_at(ix, t, sp, ep)) {  // (a wide packed entry escaped: from C[])
    return false;
  }
  // (C) the candidate rows base + i (bit i of cand)
  base = sp;
  if (sp >= ep) return true;  // the table part does not occur: count 0
  if (!cok) return false;     // a rare symbol among the context characters
  if (qf) {
    const uint32_t msk = qf == kCtxQ ? ((1u << (2 * kCtxQ)) - 1u) | kCtxEsc : (1u << (2 * qf)) - 1u;
    const uint32_t wq = want & ((1u << (2 * qf)) - 1u);
    uint32_t esc = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const uint32_t e = (d[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
      cand |= (uint32_t)((e & msk) == wq) << i;
      esc |= (uint32_t)((e & kCtxEsc) != 0) << i;
    }
    const uint32_t in = (1u << (uint32_t)(ep - sp)) - 1u;
    cand &= in;
    return (esc & in) == 0;  // 32-B records keep the escape bit; compact ones escape whole
  }
  if (ix.lctx && ep - (sp & ~15ull) <= 32) {
    qf = kCtxQ;
    base = sp & ~15ull;
    const uint32_t lo = (uint32_t)(sp - base), hi = (uint32_t)(ep - base);
    const uint4* p = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(ix.lctx) + base);
    const uint4 x0 = p[0], x1 = p[1];
    const uint4 x2 = hi > 16 ? p[2] : make_uint4(0, 0, 0, 0), x3 = hi > 16 ? p[3] : make_uint4(0, 0, 0, 0);
    if constexpr (kBytes) by += hi > 16 ? 64u : 32u;
    const uint32_t dw[16] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w,
                             x2.x, x2.y, x2.z, x2.w, x3.x, x3.y, x3.z, x3.w};
    const uint32_t msk = ((1u << (2 * kCtxQ)) - 1u) | kCtxEsc;
    uint32_t esc = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint32_t e = (dw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
      cand |= (uint32_t)((e & msk) == want) << i;
      esc |= (uint32_t)((e & kCtxEsc) != 0) << i;
    }
    const uint32_t in = (hi >= 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
    cand &= in;
    return (esc & in) == 0;
  }
  return false;  // wider than the record and two sectors: steps first
}

// the general search for the patterns a long-pattern kernel does not answer: listed in the
// slot of pattern q (LongList list2 / cnt2: a slot holds at most its kLongSlot patterns, and
// a pattern is listed there once — by the staged kernel's deferral or here)
__device__ __forceinline__ void long_list_append(bool general, uint64_t q, const LongList& ll) {
  if (!general) return;
  const uint64_t sl = long_slot(q);
  const uint32_t at = atomicAdd(ll.cnt2 + sl, 1u);
  ll.list2[sl * kLongSlot + at] = (uint32_t)(q % kLongRegion);
  if (ll.rng2) ll.rng2[sl * kLongSlot + at] = kNoRange;  // (the search starts over)
}

// The patterns of one list launch (kList): the entries of the slots of block b — slots b,
// b + grid, ... (the grid is launched with at least slots / kBlk blocks, long_list_grid) —
// their lengths read by one load per thread and scanned in LDS, then taken flattened, kBlk
// at a time, so every lane has a pattern while the block has any (an empty list costs one
// load and two barriers).  f(q, active) runs with the whole block in lockstep (active = q is
// a pattern to search; an inactive lane gets the block's first entry), so f may use wave
// collectives — a wave's patterns may lie in several regions (tiles).  Returns the block's
// number of entries (uniform).  Without a list (CS_Q_LONG, fixed-length batches of long
// patterns) the kernels take one pattern per lane over a grid covering the batch, as before
// round 4 (a loop there costs k_count_long 40 VGPRs).  c: the length of the thread's slot
// (slot_count), read before so that a block with nothing listed leaves after one load.
// slot_count's kFresh: the counts were written in this launch (by this block: the slots a
// block owns are the same for every thread of one grid) — read at the device's coherence
// point, past the CU cache another block sharing the line may have filled.
template <bool kFresh = false>
__device__ __forceinline__ uint32_t slot_count(const uint32_t* cnt, uint64_t npat) {
  const uint64_t slots = (npat + kLongRegion - 1) / kLongRegion * kSlotsPerRegion;
  const uint64_t sl = blockIdx.x + (uint64_t)threadIdx.x * gridDim.x;
  if (sl >= slots) return 0u;
  if constexpr (kFresh) return __hip_atomic_load(cnt + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return cnt[sl];
}

template <class T, class F>
__device__ __forceinline__ uint32_t list_for_each(const T* __restrict__ list, uint32_t c, F&& f) {
  static_assert(kBlk == 256, "the slot lookup below searches 256 slots in 8 steps");  // 
  __shared__ uint32_t s_off[kBlk + 1];
  __shared__ uint32_t s_w[kBlk / 64];
  // exclusive scan of the counts over the block
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w2 = 0; w2 < (int)(kBlk / 64); ++w2) {
    if (w2 < (int)wv) pre += s_w[w2];
    tot += s_w[w2];
  }
  s_off[threadIdx.x] = pre + x - c;
  if (threadIdx.x == 0) s_off[kBlk] = tot;
  __syncthreads();
  for (uint32_t e0 = 0; e0 < tot; e0 += kBlk) {
    const uint32_t e = e0 + threadIdx.x < tot ? e0 + threadIdx.x : 0u;
    // the slot holding entry e: the last t with s_off[t] <= e (empty slots share offsets)
    uint32_t lo = 0, hi = kBlk;  // s_off[lo] <= e < s_off[hi]
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const uint32_t mid = (lo + hi) >> 1;
      if (s_off[mid] <= e) lo = mid;
      else hi = mid;
    }
    const uint64_t s2 = blockIdx.x + (uint64_t)lo * gridDim.x;
    const uint64_t q = s2 / kSlotsPerRegion * kLongRegion + (list[s2 * kLongSlot + (e - s_off[lo])] & (kLongRegion - 1));
    f(q, e0 + threadIdx.x < tot);
  }
  return tot;
}

// list_for_each with two entries per thread and round (e and e + kBlk of 2 kBlk): f(q, act)
// with q[2], act[2], the whole block in lockstep
template <class F>
__device__ __forceinline__ uint32_t list_for_each2(uint32_t c, F&& f) {
  static_assert(kBlk == 256, "the slot lookup below searches 256 slots in 8 steps");
  __shared__ uint32_t s_off2[kBlk + 1];
  __shared__ uint32_t s_w2[kBlk / 64];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_w2[wv] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w2 = 0; w2 < (int)(kBlk / 64); ++w2) {
    if (w2 < (int)wv) pre += s_w2[w2];
    tot += s_w2[w2];
  }
  s_off2[threadIdx.x] = pre + x - c;
  if (threadIdx.x == 0) s_off2[kBlk] = tot;
  __syncthreads();
  for (uint32_t e0 = 0; e0 < tot; e0 += 2 * kBlk) {
    uint64_t q[2];
    bool act[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t ee = e0 + threadIdx.x + h * kBlk;
      act[h] = ee < tot;
      const uint32_t e = act[h] ? ee : 0u;
      uint32_t lo = 0, hi = kBlk;  // s_off2[lo] <= e < s_off2[hi]
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_off2[mid] <= e) lo = mid;
        else hi = mid;
      }
      const uint64_t s2 = blockIdx.x + (uint64_t)lo * gridDim.x;
      // (the entry's index in the list: its slot's base + its place)
      q[h] = s2 * kLongSlot + (e - s_off2[lo]);
    }
    f(q, act);
  }
  return tot;
}

// The rest of up to U listed general searches of the routed count from the ranges the
// staged kernel's table reads left (LongList::rng2), k[j] <= kCtxQ characters still to
// step, given by their occurrence codes (cw[j]: the list2 entry's chain, the next character at
// bits 0-1 — no pattern byte is read): count_rest's steps without its verification (k <= kCtxQ
// never verifies), the U patterns in lockstep — every round issues all their line (or
// context-sector) loads before any is used, so a lane keeps U dependent chains in flight —
// and the rows' left contexts once the range fits two sectors (ctx_match; an escaped
// context steps on).  act[j] false on entry: no pattern j.  Reference: fm_index.cpp:90-98.
// (Round 5: the list kernel read each pattern's offsets and bytes before its first step and
// a byte per step — repetitive DNA's list kernel 236 us per 12.5 M 20-mers.)
template <int U>
__device__ __forceinline__ void count_steps(const DevIndex& ix, const NodeTable& T, uint32_t* cw,
                                            uint32_t* k, uint64_t* sp, uint64_t* ep, bool* act,
                                            uint64_t* res) {
  bool ctx[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    ctx[j] = ix.lctx != nullptr;
    res[j] = 0;
  }
  // (every round steps a pattern, finishes it, or turns its contexts off once: at most
  // k + 2 <= kCtxQ + 2 rounds)
  for (;;) {
    uint4 b[U][4];  // the two lines of a step, or the two context sectors
    uint32_t mode[U];  // 0 done, 1 step, 2 contexts
    bool any = false;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      mode[j] = 0;
      if (!act[j]) continue;
      if (sp[j] >= ep[j] || k[j] == 0) {
        res[j] = sp[j] < ep[j] ? ep[j] - sp[j] : 0;
        act[j] = false;
        continue;
      }
      any = true;
      const uint64_t base = sp[j] & ~15ull;
      if (ctx[j] && k[j] <= ix.lctx_q && ep[j] - base <= 32) {
        mode[j] = 2;
        const uint4* p = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(ix.lctx) + base);
        b[j][0] = p[0];
        b[j][1] = p[1];
        if (ep[j] - base > 16) {
          b[j][2] = p[2];
          b[j][3] = p[3];
        } else {
          b[j][2] = b[j][3] = make_uint4(0, 0, 0, 0);
        }
      } else {
        mode[j] = 1;
        const uint64_t qa = sp[j] >> 6, qe = ep[j] >> 6;
        OccLine::Raw va;
        OccLine::load(ix.lines, qa, va);
        b[j][0] = va[0];
        b[j][1] = va[1];
        if (qe != qa) {
          OccLine::Raw ve;
          OccLine::load(ix.lines, qe, ve);
          b[j][2] = ve[0];
          b[j][3] = ve[1];
        } else {
          b[j][2] = va[0];
          b[j][3] = va[1];
        }
      }
    }
    if (!any) break;
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (mode[j] == 2) {
        const uint64_t base = sp[j] & ~15ull;
        const uint32_t lo = (uint32_t)(sp[j] - base), hi = (uint32_t)(ep[j] - base);
        const uint32_t mask = ((1u << (2 * k[j])) - 1u) | kCtxEsc, want = cw[j] & ((1u << (2 * k[j])) - 1u);
        const uint32_t* dw = reinterpret_cast<const uint32_t*>(b[j]);
        uint32_t match = 0, esc = 0;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          const uint32_t e = (dw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
          match |= (uint32_t)((e & mask) == want) << i;
          esc |= (uint32_t)((e & kCtxEsc) != 0) << i;
        }
        const uint32_t in = (hi >= 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
        if (esc & in) {
          ctx[j] = false;  // a rare symbol in a row's chain: step on
        } else {
          res[j] = (uint64_t)__popc(match & in);
          act[j] = false;
        }
      } else if (mode[j] == 1) {
        const uint32_t code = cw[j] & 3u, c = T.occ_sym[code];
        const OccLine::Raw va = {b[j][0], b[j][1]}, ve = {b[j][2], b[j][3]};
        uint64_t rs = OccE::occ_line(va, code, sp[j]), re = OccE::occ_line(ve, code, ep[j]);
        if (code == 0 && T.exc_n) {
          rs -= exc_before(T, sp[j]);
          re -= exc_before(T, ep[j]);
        }
        sp[j] = T.C[c] + rs;
        ep[j] = T.C[c] + re;
        cw[j] >>= 2;
        --k[j];
      }
    }
  }
}

// The routed count's list2 entries (k_count_long kList): two per thread and round; an entry
// with a range and a chain from the staged kernel takes count_steps (the two of a thread in
// lockstep; its list entry, range and chain are its only reads before the first step), any
// other the general search from the start (count_pattern: no range kept, a wide index, a
// symbol without an occurrence code, longer rests that verify against the text).
template <int W>
__device__ __forceinline__ void count_list_general2(const DevIndex& ix, NodeTable& T, const uint8_t* __restrict__ pats,
                                                    const uint64_t* __restrict__ offs, const CountOut& co,
                                                    uint64_t fixed_m, const LongList& ll, uint32_t c) {
  bool staged = false;
  list_for_each2(c, [&](const uint64_t* ei, const bool* act) {
    if (!staged) {  // the first round (uniform): the block has entries
      load_table(T, ix.table);
      __syncthreads();
      staged = true;
    }
    uint64_t q[2], sp[2], ep[2], res[2], r[2];
    uint32_t k[2], cw[2], ch[2];
    bool lean[2], a2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // (the three loads of both entries first)
      const uint64_t e = act[h] ? ei[h] : 0;
      const uint32_t le = ll.list2[e];
      q[h] = e / kLongSlot / kSlotsPerRegion * kLongRegion + (le & (kLongRegion - 1));
      r[h] = ll.rng2[e];
      ch[h] = le >> kChainShift;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      lean[h] = act[h] && r[h] != kNoRange && ((ch[h] >> 17) & 1u);
      a2[h] = lean[h];
      k[h] = lean[h] ? (ch[h] >> 14) & 7u : 0u;
      cw[h] = ch[h] & 0x3FFFu;
      sp[h] = lean[h] ? r[h] & 0xFFFFFFFFull : 0;
      ep[h] = lean[h] ? sp[h] + (r[h] >> 32) : 0;
      if (act[h] && !lean[h]) {
        // (the search from the start, as the staged kernel's general search)
        const uint64_t o0 = offs ? offs[q[h]] : q[h] * fixed_m, m = offs ? offs[q[h] + 1] - o0 : fixed_m;
        store_count<W>(co, q[h], m == 0 ? ix.n : count_pattern<OccE>(ix, T, pats + o0, m));
      }
    }
    if (lean[0] || lean[1]) {
      count_steps<2>(ix, T, cw, k, sp, ep, a2, res);
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (lean[h]) store_count<W>(co, q[h], res[h]);
    }
  });
}

// the general search of the list2 entries of a block's slots (defined below)
template <int W, bool kBytes>
__device__ __forceinline__ void count_list_general(const DevIndex& ix, NodeTable& T, const uint8_t* __restrict__ pats,
                                                   const uint64_t* __restrict__ offs, const CountOut& co,
                                                   uint64_t fixed_m, const LongList& ll, uint32_t c);
__device__ __forceinline__ void locate_list_general(const DevIndex& ix, NodeTable& T, const uint8_t* __restrict__ pats,
                                                    const uint64_t* __restrict__ offs, uint64_t limit,
                                                    const OnePass& op, const LongList& ll, uint32_t c);

// k_count_long's search of one pattern q (< npat, the batch's offsets or fixed_m)
// whether a u64 text position of a rare symbol lies in [q, q + L) (sorted list in global
// memory; walk_verify() indexes hold a handful — C5: the terminator)
__device__ __forceinline__ bool rare_in64(const uint64_t* __restrict__ r, uint32_t nr, uint64_t q, uint64_t L) {
  uint32_t lo = 0, hi = nr;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (r[mid] < q) lo = mid + 1;
    else hi = mid;
  }
  return lo < nr && r[lo] < q + L;
}
// A walk-verified candidate's window text[q, q + L) against P[0, L): 1 equal, 0 not, 2 not
// decidable here (a window through the text's end, or past the packed codes in pc, on an index
// that keeps no byte text): the pattern takes the general search.
template <bool kPT, bool kV>
__device__ __forceinline__ int window_eq_walk(const DevIndex& ix, const uint64_t* pc, const uint8_t* P,
                                              uint64_t q, uint64_t L) {
  if constexpr (kPT) {
    if (q + L <= ix.n && L <= 32ull * kLongPW) {
      if (!packed_chunk_eq<kV>(ix, pc, q, L)) return 0;
      // (a rare symbol's code 0 in the packed text stands for no pattern character)
      return rare_in64(ix.wrare, ix.nwrare, q, L) ? 0 : 1;
    }
  }
  if (ix.wtext) return window_eq_long<kLongWords>(ix, ix.wtext, P, q, L) ? 1 : 0;
  return 2;
}

// kWalk (round 6): an index without the full suffix array (DevIndex::wtext:
// walk lines with text-position marks, the byte text; C5) takes each candidate row's position
// from its short walk (walk_positions_k: <= pstride - 1 LF steps over walk lines, then the
// mark's sample) and verifies the window against the byte text — a 64-mer costs the record,
// the walk (1.4 lines + a sample on C5) and its window, not 48 more backward-search steps.
// 1: narrow walk lines (WalkLine), 2: wide (WalkLineW).
template <int W, bool kPT, bool kBytes, int kV16, int kWalk = 0>
__device__ __forceinline__ void count_long_one(const DevIndex& ix, const uint8_t* __restrict__ pats,
                                               const uint64_t* __restrict__ offs, const CountOut& co,
                                               uint64_t fixed_m, const LongList& ll, bool skip_short,
                                               const uint16_t* cmap, const uint32_t* rare, uint64_t q) {
  const uint64_t o0 = offs ? offs[q] : q * fixed_m;
  const uint64_t m = offs ? offs[q + 1] - o0 : fixed_m;
  // skip_short (the measurement twin of a routed batch): only the patterns the staged
  // kernel lists
  if (skip_short && !(m >= kFastM && m > ix.ptab_k + kCtxQ)) return;
  if (m == 0 || ix.n == 0) {  // fm_index.cpp:80-81
    if constexpr (kBytes) static_cast<uint64_t*>(co.out)[q] = 0;
    else store_count<W>(co, q, m == 0 ? ix.n : 0);
    return;
  }
  uint64_t by = 0;  // kBytes
  uint64_t pc[kLongPW];  // kPT: the codes of P[0, k)
  uint64_t base;
  uint32_t cand, qf;
  bool general = !long_stage<kPT, kBytes, kV16>(ix, pats, o0, m, cmap, pc, base, cand, qf, by);
  bool wgen = false;  // kWalk
  uint64_t res = 0;
  if (!general) {
    // (D) + (E): each candidate's SA entry, then its window (usually one candidate)
    const uint64_t k = m - ix.ptab_k, L = k - qf, n = ix.n;
    while (cand) {
      const uint32_t i = (uint32_t)__ffs(cand) - 1u;
      cand &= cand - 1;
      uint64_t p, wsteps = 0;
      if constexpr (kWalk != 0) {
        using WL = std::conditional_t<kWalk == 1, WalkLine, WalkLineW>;
        if constexpr (kBytes) {  // (the twin counts the walk's lines)
          p = walk_position_steps<WL>(ix, *ix.table, base + i, wsteps);
        } else {
          uint64_t pos[1] = {base + i};
          bool act[1] = {true};
          walk_positions_k<WL, 1>(ix, *ix.table, walk_consts(*ix.table), pos, act);
          p = pos[0];
        }
      } else {
        p = load_sa(ix.vsa, base + i);
      }
      const uint64_t wq = p >= k ? p - k : p + n - k;
      if constexpr (kBytes) {  // the SA sector (walk: its lines and the sample), then the window's words
        constexpr uint64_t C = 32ull * kLongPW;
        by += kWalk ? 32 * (wsteps + 1) + 8 : 32;
        if (wq + L > n) by += 64;  // byte by byte, as window_eq counts it
        else if (!kPT) by += 8 * (((wq + L - 1) >> 3) - (wq >> 3) + 1);
        else  // the packed window's 32-B sectors (its bytes [q / 4, (q + L) / 4) rounded out)
          by += 32 * ((((wq + (L < C ? L : C) - 1) >> 2) >> 5) - ((wq >> 2) >> 5) + 1) +
                (L > C ? 8ull * kVerifyWords * ((L - C + 8 * kVerifyWords - 1) / (8 * kVerifyWords)) : 0);
        continue;
      }
      bool eq;
      if constexpr (kWalk != 0) {
        const int r = window_eq_walk<kPT, kV16 == 3>(ix, pc, pats + o0, wq, L);
        if (r == 2) {
          wgen = true;
          break;
        }
        eq = r == 1;
      } else if constexpr (kPT) {
        eq = window_eq_packed<kV16 == 3>(ix, pc, pats + o0, wq, L, rare);
      } else {
        eq = window_eq_long<kLongWords>(ix, ix.vtext, pats + o0, wq, L);
      }
      res += eq ? 1u : 0u;
    }
  }
  if (wgen) general = true;  // (a window the walk path cannot decide: the general search)
  long_list_append(general, q, ll);
  if (general) return;
  if constexpr (kBytes) static_cast<uint64_t*>(co.out)[q] = by;
  else store_count<W>(co, q, res);
}

template <int W, bool kPT, bool kBytes = false, int kV16 = 0, bool kList = false, int kWalk = 0>
// (list mode held to 4 waves per SIMD: left alone it takes 150 VGPRs, 3 waves — hoisted
// loop invariants and SGPR spills of the list loop — and C4 150-mers routed took 1.93 ms
// against 1.71, profiles/r04/ab_lib_r04j_count_m150.jsonl)
__global__ __launch_bounds__(kBlk) __attribute__((amdgpu_waves_per_eu(kList ? 4 : 1))) void k_count_long(DevIndex ix, const uint8_t* __restrict__ pats,
                                                     const uint64_t* __restrict__ offs, uint64_t npat,
                                                     CountOut co, uint64_t fixed_m, LongList ll,
                                                     bool skip_short) {
  __shared__ uint16_t cmap[256];
  __shared__ uint32_t rare[kMaxExc];
  static_assert(kBlk >= 256, "one map entry per thread");
  uint32_t c1 = 0;
  if constexpr (kList) {
    // nothing listed in the whole call (the counters): every block leaves at its first load;
    // else a block with nothing listed in its slots after one more load (then retired)
    if (!list_any(ll)) return;
    c1 = slot_count(ll.cnt, npat);
    if (!__syncthreads_or(c1 != 0 || slot_count(ll.cnt2, npat) != 0)) {
      list_retire(ll);
      return;
    }
  }
  if (threadIdx.x < 256)
    cmap[threadIdx.x] = (uint16_t)(ix.table->code[threadIdx.x] | (ix.table->occ_code[threadIdx.x] << 8));
  if (kPT && !kWalk && threadIdx.x < ix.nrare) rare[threadIdx.x] = ix.prare[threadIdx.x];
  __syncthreads();
  if constexpr (kList) {
    list_for_each(ll.list, c1, [&](uint64_t q, bool act) {
      if (act) count_long_one<W, kPT, kBytes, kV16, kWalk>(ix, pats, offs, co, fixed_m, ll, false, cmap, rare, q);
    });
    // then the general search of what it listed and what the staged kernel listed there: the
    // same block owns the same slots of list2, so no second launch (k_count_list) waits for
    // the grid
    __shared__ NodeTable T;
    __syncthreads();
    if constexpr (kBytes)
      count_list_general<W, kBytes>(ix, T, pats, offs, co, fixed_m, ll, slot_count<true>(ll.cnt2, npat));
    else  // (the staged kernel's general searches with their ranges, two per thread)
      count_list_general2<W>(ix, T, pats, offs, co, fixed_m, ll, slot_count<true>(ll.cnt2, npat));
    list_retire(ll);
  } else {
    const uint64_t q = blockIdx.x * (uint64_t)kBlk + threadIdx.x;
    if (q < npat) count_long_one<W, kPT, kBytes, kV16, kWalk>(ix, pats, offs, co, fixed_m, ll, skip_short, cmap, rare, q);
  }
}


// Adds each lane's kc (0: nothing) to op.tiles[tile]: one atomic per distinct tile of the
// wave (a list launch's wave holds one or two slots' patterns, so one or two tiles; a
// pattern-per-lane atomic puts 512 same-address atomics on every tile: C4 150-mer locate
// 2.1 -> 3.4 ms).  Every lane of the wave, in uniform control flow.
__device__ __forceinline__ void wave_tile_add(const OnePass& op, uint64_t tile, uint64_t kc) {
  const uint32_t lane = threadIdx.x & 63;
  uint64_t pend = __ballot(kc != 0);
  while (pend) {
    const uint32_t l = (uint32_t)__ffsll((unsigned long long)pend) - 1u;
    const uint64_t t = __shfl(tile, (int)l, 64);
    const bool in = kc != 0 && tile == t;
    uint64_t s = in ? kc : 0;
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) s += __shfl_xor(s, dd, 64);
    if (lane == l) tile_total_add(op, t, s);
    pend &= ~__ballot(in);
  }
}

// The long-pattern search for the one-call locate (launch_locate_onepass over full-SA
// indexes: CS_Q_LONG, host batches of long patterns, and the long patterns the staged kernel
// lists): k_count_long's stages, then per pattern min(count, limit) and its record for
// k_locate_emit — the only position itself (kLocStash: the SA entry the verification read,
// minus k) or a verified window (first row, match bits, k), whose positions the emit kernel
// reads through SA — and the counts added to their tile's total (zeroed before, or holding the
// staged kernel's totals of the short patterns).
// The patterns it cannot finish (as k_count_long's, and windows whose matches lie too far
// apart for the record) go to k_locate_list.  Reference: fm_index.cpp:107-124 (the search),
// :125 (limit).
// k_locate_long's search of pattern q (mine: q is one to search); every lane of the wave
// calls it.
template <int kV16>
__device__ __forceinline__ void locate_long_one(const DevIndex& ix, const uint8_t* __restrict__ pats,
                                                const uint64_t* __restrict__ offs, uint64_t limit,
                                                const OnePass& op, const LongList& ll,
                                                const uint16_t* cmap, const uint32_t* rare, uint64_t q,
                                                bool mine) {
  bool general = false;
  const uint64_t o0 = mine ? offs[q] : 0, m = mine ? offs[q + 1] - o0 : 0;
  uint64_t kc = 0, rec = 0;
  if (mine && m != 0 && ix.n != 0) {  // fm_index.cpp:109: locate("") = {}
    uint64_t by = 0, pc[kLongPW], base;
    uint32_t cand, qf;
    general = !long_stage<true, false, kV16>(ix, pats, o0, m, cmap, pc, base, cand, qf, by);
    if (!general && cand) {
      const uint64_t k = m - ix.ptab_k, L = k - qf, n = ix.n;
      uint32_t mm = 0;
      uint64_t p0 = 0;  // the first matching row's position
      for (uint32_t c = cand; c; c &= c - 1) {
        const uint32_t i = (uint32_t)__ffs(c) - 1u;
        const uint64_t p = load_sa(ix.vsa, base + i);
        const uint64_t wq = p >= k ? p - k : p + n - k;
        if (window_eq_packed<kV16 == 3>(ix, pc, pats + o0, wq, L, rare)) {
          if (!mm) p0 = wq;
          mm |= 1u << i;
        }
      }
      if (mm) {
        const uint64_t c = (uint64_t)__popc(mm);
        const uint32_t f = (uint32_t)__ffs(mm) - 1u, rel = mm >> f;
        kc = c < limit ? c : limit;  // fm_index.cpp:125
        if (kc == 1) rec = kLocStash | p0;
        else if (kc > 1 && ((rel >> kLocVerRelBits) || k > kLocVerMaxK)) general = true;
        else rec = kLocCtx | (k << 50) | ((uint64_t)rel << 38) | (base + f);
      }
    }
  }
  if (general) kc = 0;  // k_locate_list adds it
  long_list_append(mine && general, q, ll);
  if (mine && !general) {
    op.cnt[q] = (uint32_t)kc;
    op.rec[q] = rec;
  }
  wave_tile_add(op, q / kLocTile, kc);
}

template <int kV16, bool kList>
// (list mode held to 4 waves per SIMD as k_count_long's: routed 150-mers 2.13 -> 1.92 ms,
// profiles/r04/ab_lib_r04j_locate_m150.jsonl)
__global__ __launch_bounds__(kBlk) __attribute__((amdgpu_waves_per_eu(kList ? 4 : 1))) void k_locate_long(DevIndex ix, const uint8_t* __restrict__ pats,
                                                      const uint64_t* __restrict__ offs, uint64_t npat,
                                                      uint64_t limit, OnePass op, LongList ll) {
  __shared__ uint16_t cmap[256];
  __shared__ uint32_t rare[kMaxExc];
  uint32_t c1 = 0;
  if constexpr (kList) {
    // nothing listed or deferred in the whole call: every block leaves at its first load;
    // else a block with nothing in its slots after one more load (then retired)
    if (!list_any(ll)) return;
    c1 = slot_count(ll.cnt, npat);
    if (!__syncthreads_or(c1 != 0 || slot_count(ll.cnt2, npat) != 0)) {
      list_retire(ll);
      return;
    }
  }
  if (threadIdx.x < 256)
    cmap[threadIdx.x] = (uint16_t)(ix.table->code[threadIdx.x] | (ix.table->occ_code[threadIdx.x] << 8));
  if (threadIdx.x < ix.nrare) rare[threadIdx.x] = ix.prare[threadIdx.x];
  __syncthreads();
  if constexpr (kList) {
    list_for_each(ll.list, c1, [&](uint64_t q, bool act) {
      locate_long_one<kV16>(ix, pats, offs, limit, op, ll, cmap, rare, q, act);
    });
    // then the general search of what it listed and the staged search deferred (the same
    // block owns the same slots of list2: no k_locate_list launch)
    __shared__ NodeTable T;
    __syncthreads();
    locate_list_general(ix, T, pats, offs, limit, op, ll, slot_count<true>(ll.cnt2, npat));
    list_retire(ll);
  } else {
    const uint64_t q = blockIdx.x * (uint64_t)kBlk + threadIdx.x;
    locate_long_one<kV16>(ix, pats, offs, limit, op, ll, cmap, rare, q, q < npat);
  }
}

// The patterns k_count_long listed (LongList list2 / cnt2): the general search
// (count_pattern), the node table staged in LDS by the blocks that have work; block b takes
// the entries of slots b, b + grid, ... (list_for_each).  kBytes: k_count_long's measurement
// twin (the general search's bytes into co.out).
// the general search of the entries of the block's slots of list2 (c: the thread's slot
// length, slot_count)
template <int W, bool kBytes>
__device__ __forceinline__ void count_list_general(const DevIndex& ix, NodeTable& T, const uint8_t* __restrict__ pats,
                                                   const uint64_t* __restrict__ offs, const CountOut& co,
                                                   uint64_t fixed_m, const LongList& ll, uint32_t c) {
  bool staged = false;
  list_for_each(ll.list2, c, [&](uint64_t q, bool act) {
    if (!staged) {  // the first round (uniform): the block has entries
      load_table(T, ix.table);
      __syncthreads();
      staged = true;
    }
    if (!act) return;
    const uint64_t o0 = offs ? offs[q] : q * fixed_m, m = offs ? offs[q + 1] - o0 : fixed_m;
    if constexpr (kBytes) {
      uint64_t by = 0;
      (void)count_pattern<OccE>(ix, T, pats + o0, m, &by);
      static_cast<uint64_t*>(co.out)[q] = by;
    } else {
      store_count<W>(co, q, count_pattern<OccE>(ix, T, pats + o0, m));
    }
  });
}

template <int W, bool kBytes = false>
__global__ __launch_bounds__(kBlk) void k_count_list(DevIndex ix, const uint8_t* __restrict__ pats,
                                                     const uint64_t* __restrict__ offs, uint64_t npat,
                                                     CountOut co, uint64_t fixed_m, LongList ll) {
  __shared__ NodeTable T;
  const uint32_t c = slot_count(ll.cnt2, npat);
  if (!__syncthreads_or(c != 0)) return;
  count_list_general<W, kBytes>(ix, T, pats, offs, co, fixed_m, ll, c);
}

// The patterns k_locate_long listed and the staged search deferred: locate's general search
// (locate_search), its count and record for k_locate_emit, the count added to the pattern's
// tile; as k_count_list.
// The one-call search of a short pattern (K <= m <= kFastM) whose locate record did not
// answer it (deferred, CS_FM_LOC_DEFER=1), on its own: k_count_ctx kOne's stages for one
// pattern — the context record, its inline contexts or the context sector(s), the window —
// and, for a single position, its SA entry (stashed as the search kernel does); anything
// else (a wide range, an escaped context, a symbol off the table) locate_search with the LDS
// node table T.  Returns min(count, limit); rec as k_locate_emit reads it.
__device__ __forceinline__ uint64_t locate_miss_one(const DevIndex& ix, const NodeTable& T,
                                                    const uint8_t* __restrict__ pats, uint64_t o0, uint32_t m,
                                                    uint64_t limit, const uint32_t* sa, uint64_t& rec) {
  const uint32_t K = ix.ptab_k;
  bool general = m < K || K == 0 || m > kFastM || !ix.lctx || !ix.lf_exact ||
                 (ix.ptab_rec != 1 && ix.ptab_rec != 2) || ix.wide;
  uint64_t res = 0, rv = 0;
  if (!general) {
    uint32_t u[8];
    load_pattern32(pats, o0, m, u);
    const uint32_t kk = m - K;
    bool ok = kk <= kCtxQ;
    uint32_t tt = 0, ww = 0;
#pragma unroll
    for (uint32_t i = 0; i < kFastM; ++i) {
      const uint32_t b = (u[i >> 2] >> (8 * (i & 3))) & 0xFFu;
      if (i >= m - K && i < m) {
        const uint32_t d = T.code[b];
        ok &= d != kNoCode;
        tt = tt * ix.ptab_sigma + d;
      } else if (i < kk && i < kCtxQ) {
        const uint32_t d = T.occ_code[b];
        ok &= d != kNoCode;
        ww |= (d & 3u) << (2 * (kk - 1 - i));
      }
    }
    general = !ok;
    uint64_t sp = 0, ep = 0, bs = 0;
    uint4 w0 = make_uint4(0, 0, 0, 0), w1 = w0, w2 = w0, w3 = w0;
    bool inl = false;
    if (!general) {
      if (ix.ptab_rec == 1) {
        const uint4* r = static_cast<const uint4*>(ix.ptab) + (uint64_t)tt * 2;
        const uint4 a = r[0], b2 = r[1];
        sp = a.x;
        ep = (uint64_t)a.x + a.y;
        w0 = make_uint4(a.z, a.w, b2.x, b2.y);
        w1 = make_uint4(b2.z, b2.w, 0u, 0u);
        inl = ep - sp <= kRecCtx;
      } else {
        const uint4 a = load_record16(ix.ptab, tt);
        const uint32_t wc = a.y & 15u;
        sp = rec16_sp(a.x, a.w, 0);
        inl = wc != kRec16Wide && kk <= kRec16Q;
        ep = sp + (wc == kRec16Wide ? a.z : wc);
        if (wc == kRec16Wide && a.z == kRec16NoRange) general = true;
        uint32_t d[5];
        rec16_contexts(a.y, a.z, a.w, d);
        w0 = make_uint4(d[0], d[1], d[2], d[3]);
        w1 = make_uint4(d[4], 0u, 0u, 0u);
      }
    }
    if (!general && sp < ep && kk == 0) {  // the table part is the whole pattern: its range
      res = ep - sp;
      rv = sp;
    } else if (!general && sp < ep) {
      if (inl) {
        bs = sp;
      } else if (ep - (sp & ~15ull) <= 32) {
        bs = sp & ~15ull;
        const uint4* p = reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(ix.lctx) + bs);
        w0 = p[0];
        w1 = p[1];
        if (ep - bs > 16) {
          w2 = p[2];
          w3 = p[3];
        }
      } else {
        general = true;
      }
    }
    if (!general && sp < ep && kk != 0) {
      const uint32_t mask = ((1u << (2 * kk)) - 1u) | kCtxEsc;
      const uint32_t lo = (uint32_t)(sp - bs), hi = (uint32_t)(ep - bs);
      const uint32_t dw[16] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w,
                               w2.x, w2.y, w2.z, w2.w, w3.x, w3.y, w3.z, w3.w};
      uint32_t match = 0, esc = 0;
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const uint32_t e = (dw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
        match |= (uint32_t)((e & mask) == ww) << i;
        esc |= (uint32_t)((e & kCtxEsc) != 0) << i;
      }
      const uint32_t in = (hi >= 32 ? ~0u : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
      const uint32_t mm = match & in;
      if (esc & in) {
        general = true;
      } else if (mm) {
        const uint32_t f = (uint32_t)__ffs(mm) - 1u, rel = mm >> f;
        if (rel >> kLocSpanBits) general = true;
        else {
          rv = kLocCtx | ((uint64_t)kk << 60) | ((uint64_t)rel << 38) | (bs + f);
          res = (uint64_t)__popc(mm);
        }
      }
    }
  }
  if (general) res = m && ix.n ? locate_search<OccE>(ix, T, pats + o0, m, rv) : 0;
  const uint64_t kc = res < limit ? res : limit;  // fm_index.cpp:125
  if (kc == 1 && sa) {  // the one position now, as locate_split_store does
    uint64_t row = rv, adj = 0;
    uint32_t rel;
    if (rv & kLocCtx) loc_window(rv, row, adj, rel);
    const uint64_t p = load_sa(sa, row);
    rv = kLocStash | (p >= adj ? p - adj : p + ix.n - adj);
  }
  rec = rv;
  return kc;
}

__device__ __forceinline__ void locate_list_general(const DevIndex& ix, NodeTable& T, const uint8_t* __restrict__ pats,
                                                    const uint64_t* __restrict__ offs, uint64_t limit,
                                                    const OnePass& op, const LongList& ll, uint32_t c) {
  bool staged = false;
  list_for_each(ll.list2, c, [&](uint64_t q, bool act) {
    if (!staged) {
      load_table(T, ix.table);
      __syncthreads();
      staged = true;
    }
    uint64_t kc = 0;
    if (act) {
      const uint64_t o0 = offs[q], m = offs[q + 1] - o0;
      uint64_t rr = 0;
      if (m <= kFastM) {  // a pattern the staged search deferred (its locate record missed)
        kc = locate_miss_one(ix, T, pats, o0, (uint32_t)m, limit, op.sa, rr);
      } else {
        const uint64_t cc = ix.n ? locate_search<OccE>(ix, T, pats + o0, m, rr) : 0;
        kc = cc < limit ? cc : limit;  // fm_index.cpp:125
      }
      op.cnt[q] = (uint32_t)kc;
      op.rec[q] = rr;
    }
    wave_tile_add(op, q / kLocTile, kc);
  });
}

__global__ __launch_bounds__(kBlk) void k_locate_list(DevIndex ix, const uint8_t* __restrict__ pats,
                                                      const uint64_t* __restrict__ offs, uint64_t npat,
                                                      uint64_t limit, OnePass op, LongList ll) {
  __shared__ NodeTable T;
  // (hdr: the staged search listed into the counters, list_any / list_retire)
  if (ll.hdr && !list_any(ll)) return;
  const uint32_t c = slot_count(ll.cnt2, npat);
  if (__syncthreads_or(c != 0)) locate_list_general(ix, T, pats, offs, limit, op, ll, c);
  if (ll.hdr) list_retire(ll);
}

// The batch count over the quaternary wavelet matrix with left contexts (C3: sigma = 256,
// k = 4 prefix table of 16-B context records, u32 contexts of lctx_q = 4 dense codes):
// the shape of k_count_ctx for u32 contexts.  (A) the pattern as realigned dword loads,
// the table index and the context key from a 1-KB LDS map (symbol -> table digit,
// dense code); (B) the U table entries — a whole 16-B record {sp, width, contexts of
// rows 0-1} in one load, or the (sp, ep) pair of a plain table; (C) when the record does
// not hold the range, the u32 context sector(s) of rows [sp, ep) (8 rows per 32 B, at
// most two sectors); (D) counts.  Anything else — patterns over 32 bytes, symbols
// outside the table alphabet or without a dense code, wider ranges — takes
// count_pattern, the general search, behind a block-wide node-table copy.
// Exact by the same backward-search invariant as the occurrence engine's contexts
// (count_rest / ctx_match): after the table, the rows r of [sp, ep) whose chain spells
// P[k-1], ..., P[0] are exactly the rows that survive the reference's remaining k steps
// (fm_index.cpp:90-96).
// kOne (round 6): the one-call locate's search (OnePass stage (1)) in the
// same stages — a pattern finished over the contexts stores its window of matching rows at k
// characters before the end (kLocCtx, lf_exact indexes), the rest its range's first row or
// the general search's record (locate_search); the block stores counts, records and its tile
// total as k_count_ctx's kOne form does, so the scan and emit kernels are the occurrence
// engine's.  The loads of a lane's U patterns are issued together (see k_count_ctx (A)).
template <int U, int W, bool kOne = false>
__global__ __launch_bounds__(kBlk) __attribute__((amdgpu_waves_per_eu(6))) void k_count_qctx(DevIndex ix, const uint8_t* __restrict__ pats,
                                                     const uint64_t* __restrict__ offs,
                                                     uint64_t npat, CountOut co, uint64_t fixed_m,
                                                     uint64_t limit = 0, OnePass op = OnePass{}) {
  // bits 0-7 table digit (kNoCode: outside the table alphabet), 8-15 dense code, bit 16 the
  // symbol occurs (every present symbol has a dense code; with 256 symbols one of them is
  // 0xFF, so kNoCode cannot mark "no code" here)
  __shared__ uint32_t cmap[256];
  __shared__ NodeTable T;
  if constexpr (kOne) onepass_zero(op);
  if (threadIdx.x < 256) {
    const NodeTable* g = ix.table;
    const uint32_t c = threadIdx.x;
    cmap[c] = g->code[c] | ((uint32_t)g->occ_code[c] << 8) | (g->C[c] != g->C[c + 1] ? 1u << 16 : 0u);
  }
  __syncthreads();
  const uint32_t K = ix.ptab_k, sb = ix.lctx_sb, Q = ix.lctx_q;
  const uint64_t q0 = blockIdx.x * (uint64_t)(kBlk * U) + threadIdx.x;
  uint64_t o0[U], res[U], sp[U], ep[U], rv[U];
  uint32_t m[U], t[U], want[U], k[U], c0[U], c1[U];
  uint8_t st[U];  // 0 done, 1 table only, 2 table + contexts, 3 general search
  // (A1) offsets (clamped: unconditional loads)
  uint64_t m1[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk, qc = q < npat ? q : npat - 1;
    st[j] = 0;
    res[j] = rv[j] = 0;
    m[j] = 0;
    t[j] = want[j] = k[j] = 0;
    o0[j] = offs ? offs[qc] : qc * fixed_m;
    m1[j] = offs ? offs[qc + 1] : 0;
  }
  // (A2) lengths and the pattern dwords of the patterns the stages search
  uint32_t praw[U][9], fw = 0;
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk;
    const bool live = q < npat;
    const uint64_t mm = offs ? m1[j] - o0[j] : fixed_m;
    m[j] = live ? (uint32_t)(mm < 0xFFFFFFFFull ? mm : 0xFFFFFFFFull) : 0u;
    const bool any = live && mm != 0 && ix.n != 0;  // fm_index.cpp:81
    if (live && mm == 0) res[j] = kOne ? 0 : ix.n;  // fm_index.cpp:80; locate: :109
    st[j] = any ? 3 : 0;
    const bool fast = any && !(mm < K || K == 0 || mm > kFastM);
    fw |= (uint32_t)fast << j;
    load_pattern32_raw(pats, o0[j], fast ? m[j] : 0u, praw[j], reinterpret_cast<const uint32_t*>(ix.table));
  }
  // (A3)
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if (!((fw >> j) & 1u)) continue;
    uint32_t u[8];
    realign_pattern32(o0[j], praw[j], u);
    const uint32_t kk = m[j] - K;
    // (kOne: a window of rows gives positions only when LF is one n-cycle, and its record
    // holds k in 3 bits: k <= 7, as locate_search's windows)
    const bool cq = kk <= Q && sb * kk <= 32 && (!kOne || (ix.lf_exact && kk <= 7));  // the rest fits one context entry
    bool ok = true, cok = cq;
    uint32_t tt = 0, ww = 0;
#pragma unroll
    for (uint32_t i = 0; i < kFastM; ++i) {
      const uint32_t b = (u[i >> 2] >> (8 * (i & 3))) & 0xFFu;
      if (i >= kk && i < m[j]) {  // table part, most significant first
        const uint32_t d = cmap[b] & 0xFFu;
        ok &= d != kNoCode;
        tt = tt * ix.ptab_sigma + d;
      } else if (cq && i < kk) {  // context part: chain symbol kk-1-i
        const uint32_t e = cmap[b];
        cok &= (e >> 16) != 0u;  // an absent symbol: the general search returns 0
        ww |= ((e >> 8) & 0xFFu) << (sb * (kk - 1 - i));
      }
    }
    if (!ok) continue;
    st[j] = cok ? 2 : 1;
    t[j] = tt;
    want[j] = ww;
    k[j] = kk;
  }
  // (B) the table entries, all in flight together (a dummy address for a pattern without one)
  const void* const dummy = static_cast<const void*>(ix.table);
  if (ix.ptab_rec == 3) {
    uint4 ra[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool act = st[j] == 1 || st[j] == 2;
      ra[j] = load_record16(act ? ix.ptab : dummy, act ? (uint64_t)t[j] : 0ull);
    }
    asm volatile("" ::: "memory");  // (keeps the loads together: see k_count_ctx (B))
#pragma unroll
    for (int j = 0; j < U; ++j) {
      sp[j] = ra[j].x;
      ep[j] = (uint64_t)ra[j].x + ra[j].y;
      c0[j] = ra[j].z;
      c1[j] = ra[j].w;
    }
  } else {
    uint2 ra[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const bool act = st[j] == 1 || st[j] == 2;
      ra[j] = (act ? static_cast<const uint2*>(ix.ptab) + t[j] : static_cast<const uint2*>(dummy))[0];
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < U; ++j) {
      sp[j] = ra[j].x;
      ep[j] = ra[j].y;
      c0[j] = c1[j] = 0;
    }
  }
  // (C) the context sector(s), unless the record holds the range's contexts
  uint4 w[U][4];
  uint64_t bs[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    bs[j] = 0;
    if (st[j] != 1 && st[j] != 2) continue;
    if (sp[j] >= ep[j]) {
      st[j] = 0;
      res[j] = 0;
    } else if (k[j] == 0) {
      st[j] = 0;
      res[j] = ep[j] - sp[j];
      rv[j] = sp[j];  // kOne: the range's first row
    } else if (st[j] == 2 && ix.ptab_rec == 3 && ep[j] - sp[j] <= kRecQCtx) {
      bs[j] = sp[j];
      w[j][0] = make_uint4(c0[j], c1[j], 0u, 0u);
      w[j][1] = w[j][2] = w[j][3] = make_uint4(0, 0, 0, 0);
    } else if (st[j] == 2 && ep[j] - (sp[j] & ~7ull) <= 16) {
      bs[j] = sp[j] & ~7ull;
      const uint4* p = reinterpret_cast<const uint4*>(static_cast<const uint32_t*>(ix.lctx) + bs[j]);
      w[j][0] = p[0];
      w[j][1] = p[1];
      if (ep[j] - bs[j] > 8) {
        w[j][2] = p[2];
        w[j][3] = p[3];
      } else {
        w[j][2] = w[j][3] = make_uint4(0, 0, 0, 0);
      }
    } else {
      st[j] = 3;
    }
  }
  // (D)
  uint64_t kc[U], kr[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    if (st[j] == 2) {
      const uint32_t kb = sb * k[j];
      const uint32_t mask = kb >= 32 ? ~0u : ((1u << kb) - 1u);
      const uint32_t lo = (uint32_t)(sp[j] - bs[j]), hi = (uint32_t)(ep[j] - bs[j]);
      const uint32_t* dw = reinterpret_cast<const uint32_t*>(w[j]);
      uint32_t match = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) match |= (uint32_t)((dw[i] & mask) == want[j]) << i;
      const uint32_t in = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
      const uint32_t mm = match & in;
      res[j] = (uint64_t)__popc(mm);
      if (kOne && mm) {  // the window record (locate_search): rows bs + f + the bits of rel
        const uint32_t f = (uint32_t)__ffs(mm) - 1u;
        rv[j] = kLocCtx | ((uint64_t)k[j] << 60) | ((uint64_t)(mm >> f) << 38) | (bs[j] + f);
      }
      st[j] = 0;
    }
    const uint64_t q = q0 + (uint64_t)j * kBlk;
    kc[j] = kr[j] = 0;
    if (kOne) {
      if (q < npat && st[j] != 3) {
        kc[j] = res[j] < limit ? res[j] : limit;  // fm_index.cpp:125
        kr[j] = rv[j];
      }
    } else if (q < npat && st[j] != 3) {
      store_count<W>(co, q, res[j]);
    }
  }
  bool general = false;
#pragma unroll
  for (int j = 0; j < U; ++j) general |= st[j] == 3;
  if (__syncthreads_or(general)) {
    load_table(T, ix.table);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (st[j] != 3) continue;
      if constexpr (kOne) {
        const uint64_t c = locate_search<QWM>(ix, T, pats + o0[j], m[j], kr[j]);
        kc[j] = c < limit ? c : limit;  // fm_index.cpp:125
      } else {
        store_count<W>(co, q0 + (uint64_t)j * kBlk, count_pattern<QWM>(ix, T, pats + o0[j], m[j]));
      }
    }
  }
  if constexpr (kOne) locate_split_store<U, 0>(ix, T, npat, blockIdx.x, q0, kc, kr, op);
}

// Single-pattern count (FMIndex::count, the p50 path): the pattern travels in the
// kernel arguments and the count is stored straight into pinned host memory, so a
// call is one launch and one synchronisation.  One lane; the node table is read
// through the cache hierarchy instead of being staged into LDS.
template <class E>
__global__ void k_count_one(DevIndex ix, OnePattern p, uint64_t* __restrict__ out) {
  // the pattern to LDS first, one dword per lane: searching straight from the kernel
  // argument miscompiled (the first bytes of a chunk of verify_count's came out wrong)
  __shared__ uint32_t pb[OnePattern::kMax / 4];
  if (threadIdx.x < OnePattern::kMax / 4)
    pb[threadIdx.x] = reinterpret_cast<const uint32_t*>(p.b)[threadIdx.x];
  __syncthreads();
  if (threadIdx.x != 0) return;
  const NodeTable& T = *ix.table;
  uint64_t res;
  if (p.m == 0) res = ix.n;       // fm_index.cpp:80
  else if (ix.n == 0) res = 0;    // :81
  else {
    res = count_pattern<E>(ix, T, BytePat{reinterpret_cast<const uint8_t*>(pb)}, p.m);
  }
  // system-scope store: the host polls this word instead of waiting for the stream
  __hip_atomic_store(out, res, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Resident single-pattern server (cs_fm_serve_start; the p50 path without a launch
// per query).  One wave: lanes 0..31 poll the request words in fine-grained pinned
// host memory with system-scope loads; a request is taken when word 0 carries the
// expected tag and so does every word its length uses.  Lane 0 runs the same
// backward search as k_count_one over the LDS copy of the pattern and the node
// table, stores the count and then (release) the tag it answers.  Exits on a stop
// request, after idle_ticks without one, or after life_ticks in total — every exit
// test is wave-uniform (wall clock, shuffled word 0, wave vote), so the wave always
// drains; the exit mark (bit 63 | last tag served) is stored after the last answer.
template <class E>
__global__ __launch_bounds__(64) void k_count_server(DevIndex ix, const uint64_t* mbox,
                                                     uint64_t* resp, uint32_t seq_done,
                                                     uint64_t idle_ticks, uint64_t life_ticks) {
  __shared__ NodeTable T;
  __shared__ __attribute__((aligned(16))) uint8_t pat[kServeWords * 4];
  load_table(T, ix.table);
  __syncthreads();
  const uint32_t lane = threadIdx.x;
  uint32_t want = seq_done + 1;
  const uint64_t t0 = (uint64_t)wall_clock64();
  uint64_t t_last = t0;
  for (;;) {
    const uint64_t w =
        lane < kServeWords
            ? __hip_atomic_load(mbox + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
            : 0ull;
    const uint64_t w0 = __shfl(w, 0);
    if ((uint32_t)(w0 >> 32) == want) {
      const uint32_t m = (uint32_t)w0;
      const uint32_t nw = m == kServeStop ? 1u : 1u + (m + 3) / 4;
      const bool ok = lane >= nw || (uint32_t)(w >> 32) == want;
      if (__all(ok)) {
        if (m == kServeStop) break;
        if (lane >= 1 && lane < nw)
          *reinterpret_cast<uint32_t*>(pat + 4 * (lane - 1)) = (uint32_t)w;
        __syncthreads();
        if (lane == 0) {
          uint64_t res;
          if (m == 0) res = ix.n;        // fm_index.cpp:80
          else if (ix.n == 0) res = 0;   // :81
          else {
            res = count_pattern<E>(ix, T, BytePat{pat}, m);
          }
          __hip_atomic_store(resp, res, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(resp + 1, (uint64_t)want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        ++want;
        t_last = (uint64_t)wall_clock64();
        continue;
      }
    }
    const uint64_t now = (uint64_t)wall_clock64();
    if (now - t_last > idle_ticks || now - t0 > life_ticks) break;
  }
  if (lane == 0)
    __hip_atomic_store(resp + 2, (1ull << 63) | (uint64_t)(want - 1), __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// Measurement twin of k_count: the algorithmic bytes of each query's search —
// distinct lines per rank pair (sp and ep in one line read once) times the line
// size, plus the prefix-table entry — for the roofline in bench.py.
template <class E>
__global__ __launch_bounds__(kBlk) void k_count_bytes(DevIndex ix, const uint8_t* __restrict__ pats,
                                                      const uint64_t* __restrict__ offs,
                                                      uint64_t npat, uint64_t* __restrict__ out) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= npat) return;
  const uint64_t o0 = offs[q], m = offs[q + 1] - o0;
  uint64_t bytes = 0;
  if (m && ix.n) (void)count_pattern<E>(ix, T, pats + o0, m, &bytes);
  out[q] = bytes;
}

// Measurement twin of the one-call locate's locate-record stage (bench.py's locate roofline):
// hit[q] = 1 when the locate record of pattern q answers it in one read — the (A)/(B0) logic
// of k_count_ctx<..., kOne> for one pattern: no matching row, or one whose SA value the
// record holds — else 0 (the context record, its window and SA entries follow).
__global__ __launch_bounds__(kBlk) void k_locrec_hits(DevIndex ix, const uint8_t* __restrict__ pats,
                                                      const uint64_t* __restrict__ offs, uint64_t npat,
                                                      uint8_t* __restrict__ hit) {
  __shared__ uint16_t cmap[256];
  if (threadIdx.x < 256)
    cmap[threadIdx.x] = (uint16_t)(ix.table->code[threadIdx.x] | (ix.table->occ_code[threadIdx.x] << 8));
  __syncthreads();
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= npat) return;
  const uint64_t o0 = offs[q], m = offs[q + 1] - o0;
  const uint32_t K = ix.ptab_k;
  uint8_t h = 0;
  if (ix.lrec && ix.lrec64 && ix.lctx && K && m >= K + 1 && m <= K + kLocRec64Q) {
    const uint32_t kk = (uint32_t)m - K;
    uint32_t tt = 0, ww = 0;
    bool ok = true;
    for (uint32_t i = 0; i < (uint32_t)m; ++i) {
      const uint32_t b = pats[o0 + i];
      const uint32_t d = i >= kk ? cmap[b] & 0xFFu : cmap[b] >> 8;
      ok &= d != kNoCode;
      if (i >= kk) tt = tt * ix.ptab_sigma + d;
      else ww |= (d & 3u) << (2 * (kk - 1 - i));
    }
    if (ok) {
      const uint32_t mask = (1u << (2 * kk)) - 1u;
      uint32_t tot = 0;
      bool none = false;
      for (uint32_t c = 0; c < 4; ++c) {
        const uint4 a = static_cast<const uint4*>(ix.lrec)[(uint64_t)tt * 4 + c];
        const uint32_t vc = a.w >> 30;
        none |= vc == 0 && a.x == ~0u;
        for (uint32_t i = 0; i < vc; ++i) tot += ((a.w >> (10 * i)) & mask) == ww;
      }
      h = !none && tot <= 1;
    }
  } else if (ix.lrec && !ix.lrec64 && ix.lctx && K && m >= K + 1 && m <= K + 1 + kLocRecQ) {
    const uint32_t kk = (uint32_t)m - K;
    uint32_t tt = 0, ww = 0, dl = 0;
    bool ok = true;
    for (uint32_t i = 0; i < (uint32_t)m; ++i) {
      const uint32_t b = pats[o0 + i];
      if (i >= kk) {
        const uint32_t d = cmap[b] & 0xFFu;
        ok &= d != kNoCode;
        tt = tt * ix.ptab_sigma + d;
      } else {
        const uint32_t d = cmap[b] >> 8;
        ok &= d != kNoCode;
        ww |= (d & 3u) << (2 * (kk - 1 - i));
        if (i + 1 == kk) {
          dl = cmap[b] & 0xFFu;
          ok &= dl != kNoCode;
        }
      }
    }
    if (ok) {
      const uint4 a = static_cast<const uint4*>(ix.lrec)[(dl << (2 * K)) + tt];
      const uint32_t c = a.w >> 24, j2 = kk - 1, mask = (1u << (2 * j2)) - 1u;
      uint32_t mm = 0;
      for (uint32_t i = 0; i < kLocRecRows; ++i)
        mm |= (uint32_t)(i < c && ((a.w >> (8 * i)) & mask) == (ww >> 2)) << i;
      h = c != kLocRecNone && !(mm & (mm - 1u));
    }
  }
  hit[q] = h;
}

template <class E>
__global__ __launch_bounds__(kBlk) void k_locate_ranges(DevIndex ix,
                                                        const uint8_t* __restrict__ pats,
                                                        const uint64_t* __restrict__ offs,
                                                        uint64_t npat, uint64_t limit,
                                                        uint64_t* __restrict__ sp_out,
                                                        uint64_t* __restrict__ cnt_out) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q > npat) return;
  if (q == npat) {  // scan slot for the total
    cnt_out[q] = 0;
    return;
  }
  const uint64_t o0 = offs[q], m = offs[q + 1] - o0;
  uint64_t rec = 0, c = 0;
  if (m && ix.n) c = locate_search<E>(ix, T, pats + o0, m, rec);  // fm_index.cpp:109: empty -> {}
  sp_out[q] = rec;
  cnt_out[q] = c < limit ? c : limit;  // fm_index.cpp:125 `positions.size() < limit`
}

// The one-call locate's search (OnePass stage (1)) for any rank engine over an index that
// keeps the full suffix array (round 6): the binary wavelet matrix (the
// reference's own structure), learned occurrence lines, and occurrence-line indexes without
// a prefix table or left contexts — each lane searches its U = 2 patterns with
// locate_search (phase 1's search, k_locate_ranges) and the block stores counts, records and
// its tile total as k_count_ctx's kOne form does, so the scan and emit kernels after it are
// the occurrence engine's.  No host round trip between the phases, no 100-MB count array
// scanned by rocprim.
template <class E>
__global__ __launch_bounds__(kBlk) void k_locate_one_gen(DevIndex ix, const uint8_t* __restrict__ pats,
                                                         const uint64_t* __restrict__ offs, uint64_t npat,
                                                         uint64_t limit, OnePass op) {
  constexpr int U = 2;
  __shared__ NodeTable T;
  onepass_zero(op);
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t q0 = blockIdx.x * (uint64_t)(kBlk * U) + threadIdx.x;
  uint64_t kc[U], kr[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const uint64_t q = q0 + (uint64_t)j * kBlk;
    kc[j] = kr[j] = 0;
    if (q >= npat) continue;
    const uint64_t o0 = offs[q], m = offs[q + 1] - o0;
    if (m && ix.n) {  // fm_index.cpp:109: empty -> {}
      const uint64_t c = locate_search<E>(ix, T, pats + o0, m, kr[j]);
      kc[j] = c < limit ? c : limit;  // fm_index.cpp:125
    }
  }
  locate_split_store<U, 0>(ix, T, npat, blockIdx.x, q0, kc, kr, op);
}

// The reported rows of pattern q in row order (fm_index.cpp:125): sp[q] + (j -
// offs[q]) for a plain record, else the window's matching rows, tagged with k.
__global__ void k_expand_rows(const uint64_t* __restrict__ sp, const uint64_t* __restrict__ offs,
                              uint64_t npat, uint64_t* __restrict__ rows) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < npat; q += stride) {
    const uint64_t a = offs[q], b = offs[q + 1], s = sp[q];
    if (s & kLocCtx) {
      const uint64_t r0 = s & kLocRowMask, tag = ((s >> 60) & 7u) << kWalkAdjShift;
      uint32_t rel = (uint32_t)(s >> 38) & ((1u << kLocSpanBits) - 1u);
      for (uint64_t j = a; j < b; ++j) {
        const uint32_t f = (uint32_t)__ffs(rel) - 1u;
        rows[j] = (r0 + f) | tag;
        rel &= rel - 1u;
      }
    } else {
      for (uint64_t j = a; j < b; ++j) rows[j] = s + (j - a);
    }
  }
}

template <bool POW2>
__device__ __forceinline__ bool is_sampled(const DevIndex& ix, uint64_t row) {
  if (POW2) return (row & ((1ull << ix.stride_shift) - 1)) == 0;
  return row % ix.stride == 0;
}

template <bool POW2>
__device__ __forceinline__ uint64_t sample_index(const DevIndex& ix, uint64_t row) {
  if (POW2) return row >> ix.stride_shift;
  return row / ix.stride;
}

// Persistent LF walk (fm_index.cpp:125-153).  Block b owns rows [b*chunk, ...);
// lanes pull rows from an LDS counter and cycle FETCH -> WALK -> SAMPLE as in
// k_walk_lines below (the SSA read of a finishing lane does not add a round trip
// to its wave's LF step).
template <class E, bool POW2>
__global__ __launch_bounds__(kBlk) void k_walk(DevIndex ix, const uint64_t* __restrict__ rows,
                                               uint64_t total, uint64_t chunk,
                                               uint64_t* __restrict__ out,
                                               unsigned long long* __restrict__ err,
                                               uint32_t steps_only) {
  enum : uint32_t { kFetch = 0, kWalk = 1, kSample = 2, kDone = 3 };
  __shared__ NodeTable T;
  __shared__ unsigned long long next;
  const uint64_t a = blockIdx.x * chunk;
  const uint64_t end = (a + chunk < total) ? a + chunk : total;
  load_table(T, ix.table);
  if (threadIdx.x == 0) next = a;
  __syncthreads();
  if (a >= total) return;
  const uint64_t n = ix.n;
  uint64_t j = 0, pos = 0, steps = 0, adj = 0;
  uint32_t phase = kFetch;
  for (;;) {
    if (phase == kFetch) {
      j = atomicAdd(&next, 1ull);
      if (j >= end) phase = kDone;
    }
    if (!__any(phase != kDone)) break;
    uint64_t row = 0, smp = 0;
    if (phase == kFetch) row = rows[j];
    if (phase == kSample) smp = ssa_at(ix, sample_index<POW2>(ix, pos));
    if (phase == kFetch) {
      pos = row & kWalkRowMask;
      adj = row >> kWalkAdjShift;
      steps = 0;
      phase = kWalk;
    } else if (phase == kSample) {
      uint64_t s = smp + steps;  // :147-153
      s = s >= n ? s - n : s;
      st_out(out + j, steps_only ? steps : s >= adj ? s - adj : s + n - adj);
      phase = kFetch;
    } else if (phase == kWalk) {
      // loop condition of fm_index.cpp:130: stop at a sampled row or after n steps
      if (is_sampled<POW2>(ix, pos) || steps >= n) {
        if (steps >= n) {
          atomicMin(err, (unsigned long long)j);  // fm_index.cpp:136-138
          phase = kFetch;
        } else {
          phase = kSample;
        }
      } else {
        pos = E::lf(ix, T, pos);
        ++steps;
      }
    }
  }
}

// The same walk over walk lines (occurrence engine, fm_device.hpp WalkLine): one
// line per step gives the mark, the sample index and LF.
__device__ __forceinline__ uint64_t wssa_at(const DevIndex& ix, uint64_t k) {
  if (ix.wssa_eb == 5) {  // 40-bit entries (wide position samples): the two dwords holding them
    const uint64_t b = 5 * k;
    const uint32_t* d = static_cast<const uint32_t*>(ix.wssa) + (b >> 2);
    const uint64_t x = ((uint64_t)d[1] << 32) | d[0];
    return (x >> (8 * (b & 3))) & ((1ull << 40) - 1);
  }
  return ix.wssa_eb == 8 ? static_cast<const uint64_t*>(ix.wssa)[k] : static_cast<const uint32_t*>(ix.wssa)[k];
}

// LF(pos) from pos's walk line v (line q, offset o): C[c] + occ(c, pos) from the same
// line (OccE::lf), or for the quaternary matrix level 0 from the walk line and levels
// 1.. as QWM::lf.
template <class W, bool kQ>
__device__ __forceinline__ uint64_t walk_lf(const DevIndex& ix, const NodeTable& T,
                                            const typename W::Raw& v, uint64_t q, uint32_t o,
                                            uint64_t pos) {
  if (!kQ) {
    const uint32_t code = W::code(v, o);
    uint32_t c = T.occ_sym[code];
    uint64_t r = W::occ(v, code, q, o);
    if (code == 0 && T.exc_n) {
      const uint32_t e = exc_before(T, pos);
      if (e < T.exc_n && T.exc_row[e] == pos) {
        c = T.exc_sym[e];
        r = exc_rank(T, c, pos);
      } else {
        r -= e;
      }
    }
    return T.C[c] + r;
  }
  const uint32_t d0 = W::code(v, o);
  uint64_t p = T.qZ[0][d0] + W::occ(v, d0, q, o);
  uint32_t x = d0;
  const int L = (int)T.qlevels;
  for (int l = 1; l < L; ++l) {
    const int nid = qnode_id(l, x);
    const uint8_t f = T.flags[nid];
    uint32_t d;
    if (f & kPure) {
      d = (f >> 2) & 3u;
      p = T.qZ[l][d] + T.R[nid] + (p - T.S[nid]);
    } else {
      OccLine::Raw lv;
      const uint64_t lq = p >> 6;
      OccLine::load(QWM::level(ix, l), lq, lv);
      const uint32_t lo = (uint32_t)(p & 63);
      d = OccLine::code(lv, lo);
      p = T.qZ[l][d] + OccLine::base(lv, d, lq) + OccLine::prefix(lv, d, lo);
    }
    x = (x << 2) | d;
  }
  return T.C[T.qsym[x]] + (p - T.S8[x]);
}

// Short walks (walk lines with text-position marks, lf_exact): every walk ends within
// pstride - 1 steps, so one lane per reported row — coalesced row reads, no work
// queue — and finished waves make room for new ones, as in the count kernels.
// One short walk (walk lines with text-position marks): from BWT row `pos` by LF to the
// first marked row or row the reference samples; writes out[j] = its text position
// minus adj (mod n), or the LF steps when steps_only; an overrun records j in err.
template <class W, bool kQ>
__device__ __forceinline__ void walk_short_one(const DevIndex& ix, const NodeTable& T, uint64_t pos,
                                               uint64_t adj, uint64_t j, uint64_t* __restrict__ out,
                                               unsigned long long* __restrict__ err,
                                               uint32_t steps_only) {
  const uint64_t n = ix.n;
  const uint64_t row_mask = ix.stride_shift != 0xFFFFFFFFu ? (1ull << ix.stride_shift) - 1 : 0;
  uint64_t steps = 0;
  for (;;) {
    uint64_t q;
    uint32_t o;
    typename W::Raw v;
    W::locate(pos, q, o);
    W::load(ix.walk, q, v);
    const bool mk = W::mark(v, o);
    const bool rs = row_mask ? (pos & row_mask) == 0 : pos % ix.stride == 0;
    if (mk || rs || steps >= n) {  // fm_index.cpp:130 loop condition
      if (steps >= n) {            // :136-138
        atomicMin(err, (unsigned long long)j);
        return;
      }
      const uint64_t sidx = mk ? W::mark_rank(v, o) : (row_mask ? pos >> ix.stride_shift : pos / ix.stride);
      uint64_t s = (mk ? wssa_at(ix, sidx) : ssa_at(ix, sidx)) + steps;  // :147-153
      s = s >= n ? s - n : s;
      st_out(out + j, steps_only ? steps : s >= adj ? s - adj : s + n - adj);
      return;
    }
    pos = walk_lf<W, kQ>(ix, T, v, q, o, pos);
    ++steps;
  }
}

template <class W>
__device__ __forceinline__ uint64_t walk_position(const DevIndex& ix, const NodeTable& T, uint64_t pos) {
  // as walk_short_one; an lf_exact index with text-position marks ends every walk within
  // pstride - 1 steps (the bound below is never reached)
  const uint64_t n = ix.n;
  const uint64_t row_mask = ix.stride_shift != 0xFFFFFFFFu ? (1ull << ix.stride_shift) - 1 : 0;
  for (uint64_t steps = 0; steps < n; ++steps) {
    uint64_t q;
    uint32_t o;
    typename W::Raw v;
    W::locate(pos, q, o);
    W::load(ix.walk, q, v);
    const bool mk = W::mark(v, o);
    const bool rs = row_mask ? (pos & row_mask) == 0 : pos % ix.stride == 0;
    if (mk || rs) {  // fm_index.cpp:147-153
      const uint64_t sidx = mk ? W::mark_rank(v, o) : (row_mask ? pos >> ix.stride_shift : pos / ix.stride);
      const uint64_t s = (mk ? wssa_at(ix, sidx) : ssa_at(ix, sidx)) + steps;
      return s >= n ? s - n : s;
    }
    pos = walk_lf<W, false>(ix, T, v, q, o, pos);
  }
  return 0;
}

// walk_position and the LF steps it took (measurement twin: bench.py's walk bytes)
template <class W>
__device__ __forceinline__ uint64_t walk_position_steps(const DevIndex& ix, const NodeTable& T, uint64_t pos,
                                                        uint64_t& steps_out) {
  const uint64_t n = ix.n;
  const uint64_t row_mask = ix.stride_shift != 0xFFFFFFFFu ? (1ull << ix.stride_shift) - 1 : 0;
  for (uint64_t steps = 0; steps < n; ++steps) {
    uint64_t q;
    uint32_t o;
    typename W::Raw v;
    W::locate(pos, q, o);
    W::load(ix.walk, q, v);
    const bool mk = W::mark(v, o);
    const bool rs = row_mask ? (pos & row_mask) == 0 : pos % ix.stride == 0;
    if (mk || rs) {
      const uint64_t sidx = mk ? W::mark_rank(v, o) : (row_mask ? pos >> ix.stride_shift : pos / ix.stride);
      const uint64_t s = (mk ? wssa_at(ix, sidx) : ssa_at(ix, sidx)) + steps;
      steps_out = steps;
      return s >= n ? s - n : s;
    }
    pos = walk_lf<W, false>(ix, T, v, q, o, pos);
  }
  steps_out = n;
  return 0;
}

template <class W, int U>
__device__ __forceinline__ void walk_positions(const DevIndex& ix, const NodeTable& T, uint64_t* pos,
                                               bool* act) {
  const uint64_t n = ix.n;
  const uint64_t row_mask = ix.stride_shift != 0xFFFFFFFFu ? (1ull << ix.stride_shift) - 1 : 0;
  uint64_t steps[U];
#pragma unroll
  for (int j = 0; j < U; ++j) steps[j] = 0;
  for (uint64_t it = 0; it < n; ++it) {
    bool any = false;
#pragma unroll
    for (int j = 0; j < U; ++j) any |= act[j];
    if (!any) return;
    uint64_t q[U];
    uint32_t o[U];
    typename W::Raw v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {  // the lines of every active walk first
      q[j] = 0, o[j] = 0;
      if (act[j]) {
        W::locate(pos[j], q[j], o[j]);
        W::load(ix.walk, q[j], v[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (!act[j]) continue;
      const bool mk = W::mark(v[j], o[j]);
      const bool rs = row_mask ? (pos[j] & row_mask) == 0 : pos[j] % ix.stride == 0;
      if (mk || rs) {  // fm_index.cpp:147-153
        const uint64_t sidx = mk ? W::mark_rank(v[j], o[j])
                                 : (row_mask ? pos[j] >> ix.stride_shift : pos[j] / ix.stride);
        const uint64_t s = (mk ? wssa_at(ix, sidx) : ssa_at(ix, sidx)) + steps[j];
        pos[j] = s >= n ? s - n : s;
        act[j] = false;
      } else {
        pos[j] = walk_lf<W, false>(ix, T, v[j], q[j], o[j], pos[j]);
        ++steps[j];
      }
    }
  }
}

// walk_lf over the occurrence-line walk lines with the step's constants in registers (K);
// more than one rare row takes the table (through the caches) as walk_lf does
template <class W>
__device__ __forceinline__ uint64_t walk_lf_k(const NodeTable& T, const WalkK& K, const typename W::Raw& v,
                                              uint64_t q, uint32_t o, uint64_t pos) {
  const uint32_t code = W::code(v, o);
  uint64_t r = W::occ(v, code, q, o);
  const uint64_t cc = code == 0 ? K.C[0] : code == 1 ? K.C[1] : code == 2 ? K.C[2] : K.C[3];
  if (code == 0 && K.nexc) {
    if (K.nexc == 1) {
      if (pos == K.exc_row0) return K.exc_c0;  // the rare row: no earlier row holds its symbol
      r -= K.exc_row0 < pos ? 1u : 0u;
    } else {
      const uint32_t e = exc_before(T, pos);
      if (e < T.exc_n && T.exc_row[e] == pos) {
        const uint32_t c = T.exc_sym[e];
        return T.C[c] + exc_rank(T, c, pos);
      }
      r -= e;
    }
  }
  return cc + r;
}

template <class W, int U>
__device__ __forceinline__ void walk_positions_k(const DevIndex& ix, const NodeTable& T, const WalkK& K,
                                                 uint64_t* pos, bool* act) {
  const uint64_t n = ix.n;
  const uint64_t row_mask = ix.stride_shift != 0xFFFFFFFFu ? (1ull << ix.stride_shift) - 1 : 0;
  uint64_t steps[U];
#pragma unroll
  for (int j = 0; j < U; ++j) steps[j] = 0;
  for (uint64_t it = 0; it < n; ++it) {
    bool any = false;
#pragma unroll
    for (int j = 0; j < U; ++j) any |= act[j];
    if (!any) return;
    uint64_t q[U];
    uint32_t o[U];
    typename W::Raw v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {  // the lines of every active walk first
      q[j] = 0, o[j] = 0;
      if (act[j]) {
        W::locate(pos[j], q[j], o[j]);
        W::load(ix.walk, q[j], v[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (!act[j]) continue;
      const bool mk = W::mark(v[j], o[j]);
      const bool rs = row_mask ? (pos[j] & row_mask) == 0 : pos[j] % ix.stride == 0;
      if (mk || rs) {  // fm_index.cpp:147-153
        const uint64_t sidx = mk ? W::mark_rank(v[j], o[j])
                                 : (row_mask ? pos[j] >> ix.stride_shift : pos[j] / ix.stride);
        const uint64_t s = (mk ? wssa_at(ix, sidx) : ssa_at(ix, sidx)) + steps[j];
        pos[j] = s >= n ? s - n : s;
        act[j] = false;
      } else {
        pos[j] = walk_lf_k<W>(T, K, v[j], q[j], o[j], pos[j]);
        ++steps[j];
      }
    }
  }
}

template <class W, bool kQ>
__global__ __launch_bounds__(kBlk) void k_walk_short(DevIndex ix, const uint64_t* __restrict__ rows,
                                                     uint64_t total, uint64_t* __restrict__ out,
                                                     unsigned long long* __restrict__ err,
                                                     uint32_t steps_only) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (j >= total) return;
  const uint64_t row = rows[j];
  walk_short_one<W, kQ>(ix, T, row & kWalkRowMask, row >> kWalkAdjShift, j, out, err, steps_only);
}

// Phase 2 over walk lines with text-position marks, fused with the records (no rows
// buffer, as k_locate_sa for the full SA): a lane takes a pattern's reported rows —
// a context window's matching rows (subtracting k) or a plain range of at most
// kLocSmall rows — and walks each; wider ranges are listed for k_walk_fused_wide.
template <class W, bool kQ>
__global__ __launch_bounds__(kBlk) void k_walk_fused(DevIndex ix, const uint64_t* __restrict__ sp,
                                                     const uint64_t* __restrict__ offs, uint64_t npat,
                                                     uint64_t* __restrict__ out,
                                                     uint64_t* __restrict__ wide,
                                                     unsigned long long* __restrict__ nwide,
                                                     unsigned long long* __restrict__ err,
                                                     uint32_t steps_only) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= npat) return;
  const uint64_t a = offs[q], c = offs[q + 1] - a, s = sp[q];
  if (!c) return;
  if (s & kLocCtx) {
    const uint64_t r0 = s & kLocRowMask, adj = (s >> 60) & 7u;
    uint32_t rel = (uint32_t)(s >> 38) & ((1u << kLocSpanBits) - 1u);
    for (uint64_t j = 0; j < c; ++j) {
      const uint32_t f = (uint32_t)__ffs(rel) - 1u;
      walk_short_one<W, kQ>(ix, T, r0 + f, adj, a + j, out, err, steps_only);
      rel &= rel - 1u;
    }
  } else if (c <= kLocSmall) {
    for (uint64_t j = 0; j < c; ++j) walk_short_one<W, kQ>(ix, T, s + j, 0, a + j, out, err, steps_only);
  } else {
    wide[atomicAdd(nwide, 1ull)] = q;
  }
}

// the listed wide ranges: a block per range, its threads over the rows
template <class W, bool kQ>
__global__ __launch_bounds__(kBlk) void k_walk_fused_wide(DevIndex ix, const uint64_t* __restrict__ sp,
                                                          const uint64_t* __restrict__ offs,
                                                          uint64_t* __restrict__ out,
                                                          const uint64_t* __restrict__ wide,
                                                          const unsigned long long* __restrict__ nwide,
                                                          unsigned long long* __restrict__ err,
                                                          uint32_t steps_only) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t nw = *nwide;
  for (uint64_t e = blockIdx.x; e < nw; e += gridDim.x) {
    const uint64_t q = wide[e], a = offs[q], c = offs[q + 1] - a, s = sp[q];
    for (uint64_t j = threadIdx.x; j < c; j += blockDim.x)
      walk_short_one<W, kQ>(ix, T, s + j, 0, a + j, out, err, steps_only);
  }
}

template <class W, bool kQ>
__global__ __launch_bounds__(kBlk) void k_walk_lines(DevIndex ix, const uint64_t* __restrict__ rows,
                                                     uint64_t total, uint64_t chunk,
                                                     uint64_t* __restrict__ out,
                                                     unsigned long long* __restrict__ err,
                                                     uint32_t steps_only) {
  // Each lane cycles FETCH (row from the block's slice) -> WALK (one line per LF
  // step) -> SAMPLE (the mark's SA sample, with the next row's index) -> WALK ...
  // Every loop iteration issues at most one dependent load per lane and kind,
  // whatever its phase, so a wave waits one memory round trip per iteration even
  // when some of its lanes are starting or finishing a walk.
  enum : uint32_t { kFetch = 0, kWalk = 1, kSample = 2, kDone = 3 };
  __shared__ NodeTable T;
  __shared__ unsigned long long next;
  const uint64_t a = blockIdx.x * chunk;
  const uint64_t end = (a + chunk < total) ? a + chunk : total;
  load_table(T, ix.table);
  if (threadIdx.x == 0) next = a;
  __syncthreads();
  if (a >= total) return;
  const uint64_t n = ix.n;
  uint64_t j = 0, pos = 0, steps = 0, sidx = 0, adj = 0;
  uint32_t phase = kFetch;
  bool from_ssa = false;  // the stop row is one of the reference's sampled rows
  const uint64_t row_mask = ix.stride_shift != 0xFFFFFFFFu ? (1ull << ix.stride_shift) - 1 : 0;
  for (;;) {
    if (phase == kFetch) {
      j = atomicAdd(&next, 1ull);
      if (j >= end) phase = kDone;
    }
    if (!__any(phase != kDone)) break;
    // ---- issue this iteration's load ----
    uint64_t row = 0, smp = 0, q = 0;
    uint32_t o = 0;
    typename W::Raw v;
    if (phase == kFetch) row = rows[j];
    if (phase == kWalk) {
      W::locate(pos, q, o);
      W::load(ix.walk, q, v);
    }
    uint64_t jn = 0;
    if (phase == kSample) {
      smp = from_ssa ? ssa_at(ix, sidx) : wssa_at(ix, sidx);
      // the next row's index travels with the sample: a walk of s steps costs s + 1
      // round trips instead of s + 2 (walks average ~3 steps at pstride 8)
      jn = atomicAdd(&next, 1ull);
      if (jn < end) row = rows[jn];
    }
    // ---- consume ----
    if (phase == kFetch) {
      pos = row & kWalkRowMask;
      adj = row >> kWalkAdjShift;
      steps = 0;
      phase = kWalk;
    } else if (phase == kWalk) {
      // a walk may stop at a marked row or at a row the reference samples
      // (row % stride == 0, SSA): both give SA[start] = sample + steps, and the
      // first of the two comes sooner (mean 11 steps at stride 32 instead of 15.5)
      const bool mk = W::mark(v, o);
      const bool rs = row_mask ? (pos & row_mask) == 0 : pos % ix.stride == 0;
      if (mk || rs || steps >= n) {  // fm_index.cpp:130 loop condition
        if (steps >= n) {            // :136-138, checked first
          atomicMin(err, (unsigned long long)j);
          phase = kFetch;
        } else {
          from_ssa = !mk;
          sidx = mk ? W::mark_rank(v, o) : (row_mask ? pos >> ix.stride_shift : pos / ix.stride);
          phase = kSample;
        }
      } else {
        pos = walk_lf<W, kQ>(ix, T, v, q, o, pos);
        ++steps;
      }
    } else if (phase == kSample) {
      uint64_t s = smp + steps;  // :147-153
      s = s >= n ? s - n : s;
      st_out(out + j, steps_only ? steps : s >= adj ? s - adj : s + n - adj);
      if (jn < end) {
        j = jn;
        pos = row & kWalkRowMask;
        adj = row >> kWalkAdjShift;
        steps = 0;
        phase = kWalk;
      } else {
        phase = kDone;
      }
    }
  }
}

// ---- building-block kernels for parity tests ----
template <class F>
__global__ void k_level_rank1(DevIndex ix, int level, const uint64_t* __restrict__ pos, uint64_t k,
                              uint64_t* __restrict__ out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= k) return;
  uint64_t p = pos[t];
  // BitVector::rank1(i >= size) = count_ones() (bitvector.cpp:168-170)
  if (p > ix.n) p = ix.n;
  out[t] = rank1_at<F>(level_ptr<F>(ix, level), p);
}

template <class E>
__global__ void k_wt_rank(DevIndex ix, const uint8_t* __restrict__ syms,
                          const uint64_t* __restrict__ pos, uint64_t k, uint64_t* __restrict__ out) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= k) return;
  const uint32_t c = syms[t];
  const uint64_t i = pos[t];
  uint64_t d = 0;
  if (i != 0 && i <= ix.n && T.C[c] != T.C[c + 1]) d = E::rank(ix, T, c, i);  // wavelet.cpp:60
  out[t] = d;
}

template <class E>
__global__ void k_lf(DevIndex ix, const uint64_t* __restrict__ rows, uint64_t k,
                     uint64_t* __restrict__ out, uint8_t* __restrict__ sym) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (t >= k) return;
  const uint64_t i = rows[t];
  if (i >= ix.n) {  // fm_index.hpp:63 / wavelet.cpp:104
    if (out) out[t] = 0;
    if (sym) sym[t] = 0;
    return;
  }
  uint32_t c;
  const uint64_t v = E::lf(ix, T, i, &c);
  if (out) out[t] = v;
  if (sym) sym[t] = (uint8_t)c;
}

// extract(pos, len) (fm_index.cpp:163-167) without the text: start at the
// inverse-SA sample of the first sampled text position e >= pos+len (position n =
// suffix 0 cyclically, whose BWT symbol is T[n-1]) and invert LF down to pos; each
// LF step yields BWT[row] = T[cur-1].  One lane per query; requires lf_exact.
template <class E>
__global__ __launch_bounds__(kBlk) void k_extract(DevIndex ix, const uint64_t* __restrict__ pos,
                                                  const uint64_t* __restrict__ len,
                                                  const uint64_t* __restrict__ out_offs,
                                                  uint64_t k, uint8_t* __restrict__ out) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= k) return;
  const uint64_t n = ix.n;
  const uint64_t p = pos[q];
  if (p >= n) return;  // fm_index.cpp:164: empty
  uint64_t L = len[q];
  if (L > n - p) L = n - p;
  const uint64_t end = p + L;
  const uint64_t s = ix.pstride;
  uint64_t e = ((end + s - 1) / s) * s;
  if (e >= n) e = n;
  uint64_t row = isa_at(ix, e == n ? 0 : e / s);
  uint8_t* o = out + out_offs[q];
  for (uint64_t cur = e; cur > p; --cur) {
    uint32_t c;
    const uint64_t nxt = E::lf(ix, T, row, &c);
    if (cur - 1 < end) o[cur - 1 - p] = (uint8_t)c;
    row = nxt;
  }
}

// extract(pos, len) (fm_index.cpp:163-167) as the reference does it — a copy of
// text_[pos, pos+len) — from the text kept in HBM (keep_device_text).  One lane per
// query: the queries' strings are short and start at random positions, so each lane
// reads its own 1-2 cache lines; dword loads when source and destination line up.
__global__ __launch_bounds__(kBlk) void k_extract_text(const uint8_t* __restrict__ text, uint64_t n,
                                                       const uint64_t* __restrict__ pos,
                                                       const uint64_t* __restrict__ len,
                                                       const uint64_t* __restrict__ out_offs,
                                                       uint64_t k, uint8_t* __restrict__ out) {
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q >= k) return;
  const uint64_t p = pos[q];
  if (p >= n) return;  // fm_index.cpp:164: empty
  uint64_t L = len[q];
  if (L > n - p) L = n - p;  // :165
  const uint8_t* s = text + p;
  uint8_t* o = out + out_offs[q];
  uint64_t i = 0;
  if ((((uintptr_t)s ^ (uintptr_t)o) & 3) == 0) {
    for (; i < L && ((uintptr_t)(s + i) & 3); ++i) o[i] = s[i];
    for (; i + 4 <= L; i += 4)
      *reinterpret_cast<uint32_t*>(o + i) = *reinterpret_cast<const uint32_t*>(s + i);
  }
  for (; i < L; ++i) o[i] = s[i];
}

// WaveletTree::access for every row (the BWT), grid-stride.
template <class E>
__global__ __launch_bounds__(kBlk) void k_bwt(DevIndex ix, uint8_t* __restrict__ out) {
  __shared__ NodeTable T;
  load_table(T, ix.table);
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ix.n; i += stride) {
    uint32_t c;
    (void)E::lf(ix, T, i, &c);
    out[i] = (uint8_t)c;
  }
}

}  // namespace


cs_status launch_extract(const cs_fm_index* h, const uint64_t* d_pos, const uint64_t* d_len,
                         const uint64_t* d_out_offs, uint64_t k, uint8_t* d_out, hipStream_t st) {
  if (!k) return CS_OK;
  if (h->d_dtext) {
    k_extract_text<<<grid_for(k, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(
        static_cast<const uint8_t*>(h->d_dtext), h->n, d_pos, d_len, d_out_offs, k, d_out);
    FMX_HIP(hipGetLastError());
    return CS_OK;
  }
  FMX_DISPATCH(h, k_extract, grid_for(k, kBlk, 0xFFFFFFFFu), h->dev(), d_pos, d_len, d_out_offs, k,
               d_out);
  return CS_OK;
}

cs_status launch_bwt(const cs_fm_index* h, uint8_t* d_out, hipStream_t st) {
  FMX_DISPATCH(h, k_bwt, grid_for(h->n, kBlk, 65536), h->dev(), d_out);
  return CS_OK;
}

// The index as one query sees it under the caller's query flags (cs_fmindex.h CS_Q_*):
// the same structures with the prefix table, the left contexts / context records or the
// walk lines left out, so a search runs the plain backward-search steps of the
// reference (fm_index.cpp:84-98) and a walk its row-sampled SSA walk (:125-153).
DevIndex query_dev(const cs_fm_index* h, uint32_t flags) {
  DevIndex d = h->dev();
  if (flags & CS_Q_NO_PREFIX) d.ptab_k = 0;
  if (flags & CS_Q_NO_CONTEXTS) {
    d.lctx = nullptr;
    d.lctx_q = 0;
  }
  // CS_Q_NO_FULL_SA: locate's phase 2 walks, and a walk takes no verified windows
  if (flags & (CS_Q_NO_CONTEXTS | CS_Q_NO_VERIFY | CS_Q_NO_FULL_SA))
    d.vsa = nullptr, d.vtext = nullptr, d.ptext = nullptr, d.wtext = nullptr;
  if (flags & CS_Q_NO_WALK_LINES) d.walk = nullptr, d.wtext = nullptr;
  if (flags & CS_QT_MAP_LDS) d.dna_std = 0;
  if (flags & (CS_Q_NO_PREFIX | CS_Q_NO_CONTEXTS | CS_Q_NO_FULL_SA | CS_Q_NO_LOC_RECORDS)) d.lrec = nullptr;
  return d;
}

cs_status launch_count(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                       uint64_t npat, uint64_t* d_out, hipStream_t st, uint64_t fixed_m,
                       uint32_t flags) {
  CountOut co{d_out, nullptr, nullptr, 0, 8};
  return launch_count_ex(h, d_pats, d_offs, npat, co, flags, st, fixed_m, false);
}

// Tuning selectors (round 5): the query paths read no environment.
// A handle takes its defaults from the CS_FM_* variables once, when it is created
// (read_tuning, fm_capi.hip: cs_fm_index::tune), and a call's flags add CS_QT_* bits over
// them (cs_fmindex.h), so tests and A/Bs select kernels per call without touching the
// environment — and a thread that changes the environment cannot race a call.
//
// CS_QT_BARRIER (CS_FM_COUNT_NOBAR=0): the staged kernel's general search behind a block-wide
// LDS copy of the node table; the default (since round 4) reads the node table through the
// caches with no block barrier, so a wave whose patterns are done leaves at once instead of
// waiting at the barrier for the block's slowest record read.  C4 headline A/Bs in one
// process: 0.417 against 0.456 ms per call unrouted (profiles/r04/ab_nobar_unrouted.json),
// 0.401 against 0.413 back to back routed (ab_nobar_b2b.json).  A template parameter (a
// runtime flag kept both general searches in one kernel: 100 VGPRs, 4 waves per SIMD instead
// of 79 / 6), honoured for the two-patterns-per-lane forms over occurrence lines and learned
// lines (byte strings, routed or not, and 2-bit packed) and locate's phase 1.
inline bool count_nobar(uint32_t flags) { return !(flags & CS_QT_BARRIER); }

// CS_QT_QCTX_UNSTAGED (CS_FM_QCTX_STAGED=0): the quaternary matrix counts through k_count (one
// pattern per lane) instead of the staged k_count_qctx
inline bool qctx_staged(uint32_t flags) { return !(flags & CS_QT_QCTX_UNSTAGED); }

// the call's flags with the handle's tuning defaults
inline uint32_t call_flags(const cs_fm_index* h, uint32_t flags) { return flags | h->tune; }

// k_count_long over the batch (skip_short: only its long patterns, as k_count_ctx's kSkipLong),
// then k_count_list over the patterns it listed; byte_text: the byte text even when the
// index has the packed one (tuning hook CS_FM_LONG_KERNEL=2)
// The call's long-pattern lists (LongList): the counters' header (kListHdrBytes, zero between
// calls), slot lists of the staged kernel (list / cnt, unless `direct`) and of k_count_long /
// k_locate_long for the general search (list2 / cnt2), offsets inside the slots' regions (u16; list2 u32 with the chain);
// in the caller's workspace (round 5: cs_fm_workspace_bytes, no allocation in the call) or in
// one stream-ordered allocation whose header is zeroed here.  Direct launches (every pattern
// to the long kernel, no staged kernel before it) zero cnt2 here and use no counters;
// otherwise the staged kernel writes every slot's counts, wave by wave.
static_assert(kLongRegion == 2 * kBlk && kLongSlot == 2 * 64, "a slot is one wave's patterns (U = 2)");
static_assert(kListHdrBytes % 256 == 0, "the lists start 256-B aligned");
struct LongBufs {
  StreamBuf buf;
  LongList ll;
  static uint64_t bytes(uint64_t npat, bool direct) {
    const uint64_t slots = (npat + kLongRegion - 1) / kLongRegion * kSlotsPerRegion;
    // list2 (u32 entries) and cnt2; unless direct, list (u16), cnt and the ranges of the
    // general-search entries (8 B each)
    return kListHdrBytes + slots * (kLongSlot * 4 + 4) + (direct ? 0 : slots * (kLongSlot * (2 + 8) + 4));
  }
  // into `at` (bytes(npat, direct) of it: the caller's workspace, whose header the calls keep
  // zeroed, or the call's own allocation when `fresh`), or an allocation of its own
  cs_status alloc(uint64_t npat, bool direct, hipStream_t st, void* at = nullptr, bool fresh = true) {
    const uint64_t regions = (npat + kLongRegion - 1) / kLongRegion, slots = regions * kSlotsPerRegion;
    const uint64_t entries = slots * kLongSlot;
    const uint64_t lists = entries * 4 + (direct ? 0 : entries * 2);
    if (!at) FMX_HIP(buf.alloc(bytes(npat, direct), st));
    uint8_t* p = at ? static_cast<uint8_t*>(at) : buf.as<uint8_t>();
    ll.hdr = reinterpret_cast<uint32_t*>(p);
    if ((!at || fresh) && !direct) FMX_HIP(hipMemsetAsync(p, 0, kListHdrBytes, st));
    p += kListHdrBytes;
    ll.list2 = reinterpret_cast<uint32_t*>(p);
    ll.cnt2 = reinterpret_cast<uint32_t*>(p + lists);
    if (!direct) {
      ll.list = reinterpret_cast<uint16_t*>(p + entries * 4);
      ll.cnt = ll.cnt2 + slots;
      ll.rng2 = reinterpret_cast<uint64_t*>(p + lists + 2 * slots * 4);  // (8-B aligned: slots % 4 == 0)
    } else {
      ll.hdr = nullptr;
      FMX_HIP(hipMemsetAsync(ll.cnt2, 0, slots * 4, st));
    }
    return CS_OK;
  }
};


// blocks of the list kernels (list_for_each): one generation of the blocks resident at their
// 4 waves per SIMD — 4 blocks of 4 waves per CU, 1024 on the MI355X's 256 CUs — and at least
// slots / kBlk so that a block's slots fit one load per thread.  Round 5 A/B (CS_FM_LIST_GRID,
// C4 ms per 12.5 M, repetitive DNA / Q_text 64-mers / 150-mers, profiles/r05/r05f, r05g):
// 512: 0.679 / 1.93 / 2.42; 768: 0.667 / 1.53 / 1.94; 1024: 0.68 / 1.38-1.40 / 1.78-1.79;
// 1280: 0.744 / 1.72 / 2.12; 2560 (round 4): 0.755 / 1.49 / 1.83 — a second, partial
// generation of blocks costs a whole chain of dependent reads.
constexpr unsigned kLongListGrid = 0;  // (0: 4 blocks per CU of the device)
unsigned list_blocks_per_device() {
  static std::once_flag once[64];
  static unsigned g[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1024;
  std::call_once(once[dev], [dev] {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) {
      (void)hipGetLastError();
      ncu = 256;
    }
    g[dev] = 4u * (unsigned)ncu;
  });
  return g[dev];
}
unsigned long_list_grid(uint64_t npat, uint32_t want = kLongListGrid) {
  const uint64_t slots = (npat + kLongRegion - 1) / kLongRegion * kSlotsPerRegion;
  const uint64_t g = std::max<uint64_t>(std::min<uint64_t>(slots, want ? want : list_blocks_per_device()),
                                        (slots + kBlk - 1) / kBlk);
  return (unsigned)std::max<uint64_t>(g, 1);
}

// k_count_long over the batch (from_list: the staged kernel's lists in ll), then k_count_list
// over what it could not finish.  skip_short (twin): every pattern read, only the long ones
// searched.
// whether k_count_long verifies long patterns at their walks' positions (round 6): the
// index keeps no full SA (DevIndex::vsa) but walk lines and a text to compare against
inline bool walk_verify(const DevIndex& ix) {
  return !ix.vsa && ix.walk && ix.wssa && ix.lf_exact && (ix.wtext || (ix.ptext && ix.wrare));
}
template <bool kBytes>
cs_status launch_count_long_t(const DevIndex& ix, const uint8_t* d_pats, const uint64_t* d_offs,
                              uint64_t npat, const CountOut& co, hipStream_t st, uint64_t fixed_m,
                              const LongList* routed, bool skip_short, bool byte_text, bool loads8) {
  LongBufs own;
  LongList ll;
  if (routed) {
    ll = *routed;
  } else {
    cs_status s = own.alloc(npat, true, st);
    if (s != CS_OK) return s;
    ll = own.ll;
  }
  const unsigned g = routed ? long_list_grid(npat, routed->grid) : grid_for(npat, kBlk, 0xFFFFFFFFu);
  // CS_QT_LONG_LOADS8 (CS_FM_LONG_V16=0): 8-B pattern / window loads; the default 16-B vectors
  // for the pattern's packed part and the window (C4 150-mers 1.87 -> 1.55 ms, 64-mers 1.25 ->
  // 1.16-1.21, profiles/r03/long_probe_v16.json; round 4's partial forms 1 / 2 are gone)
  const int walk = walk_verify(ix) ? (ix.wide ? 2 : 1) : 0;
  if (walk && kBytes) {  // the measurement twin of the walk forms (direct launches only)
    if (walk == 2 && ix.ptext)
      k_count_long<0, true, true, 3, false, 2><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
    else if (walk == 2)
      k_count_long<0, false, true, 0, false, 2><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
    else if (ix.ptext)
      k_count_long<0, true, true, 3, false, 1><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
    else
      k_count_long<0, false, true, 0, false, 1><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
  } else if (walk) {  // (round 6) candidates positioned by their short walks (no full SA)
    // against the 2-bit text when the index has it (C5), else the byte text
    const bool pt = ix.ptext != nullptr && !byte_text;
    if (routed && walk == 2 && pt)
      k_count_long<0, true, false, 3, true, 2><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, false);
    else if (routed && walk == 2)
      k_count_long<0, false, false, 0, true, 2><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, false);
    else if (routed && pt)
      k_count_long<0, true, false, 3, true, 1><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, false);
    else if (routed)
      k_count_long<0, false, false, 0, true, 1><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, false);
    else if (walk == 2 && pt)
      k_count_long<0, true, false, 3, false, 2><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
    else if (walk == 2)
      k_count_long<0, false, false, 0, false, 2><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
    else if (pt)
      k_count_long<0, true, false, 3, false, 1><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
    else
      k_count_long<0, false, false, 0, false, 1><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
  } else if (routed && ix.ptext && !byte_text && !loads8)  // the routed default
    k_count_long<0, true, kBytes, 3, true><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, false);
  else if (routed && ix.ptext && !byte_text)
    k_count_long<0, true, kBytes, 0, true><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, false);
  else if (routed)
    k_count_long<0, false, kBytes, 0, true><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, false);
  else if (ix.ptext && !byte_text && !loads8)
    k_count_long<0, true, kBytes, 3><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
  else if (ix.ptext && !byte_text)
    k_count_long<0, true, kBytes><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
  else
    k_count_long<0, false, kBytes><<<g, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m, ll, skip_short);
  FMX_HIP(hipGetLastError());
  if (!routed) {  // (a routed k_count_long searches what it listed itself)
    k_count_list<0, kBytes><<<long_list_grid(npat), kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, fixed_m, ll);
    FMX_HIP(hipGetLastError());
  }
  return CS_OK;
}
cs_status launch_count_long(const DevIndex& ix, const uint8_t* d_pats, const uint64_t* d_offs,
                            uint64_t npat, const CountOut& co, hipStream_t st, uint64_t fixed_m,
                            const LongList* routed, uint32_t flags) {
  return launch_count_long_t<false>(ix, d_pats, d_offs, npat, co, st, fixed_m, routed, false,
                                    (flags & CS_QT_LONG_BYTE_TEXT) != 0, (flags & CS_QT_LONG_LOADS8) != 0);
}

// Whether a device batch is routed (the staged kernel lists its long patterns — and, for
// counts, the patterns left to the general search — for k_count_long / k_locate_long in the
// same call): every batch on the indexes k_count_long serves (occurrence lines, the full SA
// and the text).  Round 4 routed only batches of 4 M patterns or more (kRouteMin): the lists
// cost a call ≈ 8 µs whatever it held — one stream-ordered allocation and a list kernel that
// scanned every slot's count (C4's 12.5 M 20-mers 0.381 -> 0.397 ms, C2's 1 M 36 -> 47 µs).
// Round 5 takes both out: the lists live in the caller's workspace (cs_fm_workspace_bytes)
// and a list kernel whose counters read 0 leaves at its first load (list_any), so every batch
// routes and the production path is the one the tests run.
// CS_QT_NO_ROUTE (CS_FM_LONG_ROUTE=0): never route (the staged kernel alone, round 2's path).
bool can_route(const cs_fm_index* h, const DevIndex& ix, uint32_t flags) {
  // (round 6: also indexes without the full SA whose long patterns k_count_long verifies at
  // their walks' positions, DevIndex::wtext — C5)
  if (h->line_fmt != kFmtOcc || !(ix.vsa || walk_verify(ix)) || !ix.ptab_k) return false;
  return !(flags & CS_QT_NO_ROUTE);
}

// the staged kernel at count width W: table entries (context records) of U patterns per
// lane in flight together, then their context sectors or rank steps
template <int W>
cs_status launch_count_staged(const cs_fm_index* h, const DevIndex& ix, const uint8_t* d_pats,
                              const uint64_t* d_offs, uint64_t npat, const CountOut& co,
                              hipStream_t st, uint64_t fixed_m, bool packed, uint32_t flags,
                              const Work& work) {
  // patterns per lane: CS_QT_COUNT_U1 / CS_QT_COUNT_U4 (CS_FM_COUNT_U=1 / 4), else 2
  const int U = (flags & CS_QT_COUNT_U1) ? 1 : (flags & CS_QT_COUNT_U4) ? 4 : 2;
  const bool nobar = count_nobar(flags);
  const bool lo = h->line_fmt == kFmtLOcc;
  const unsigned g2 = grid_for((npat + 1) / 2, kBlk, 0xFFFFFFFFu);
  if (packed && lo && nobar)
    k_count_ctx<LOccE, 2, false, true, W, true><<<g2, kBlk, 0, st>>>(ix, d_pats, nullptr, npat, co, 0,
                                                                      nullptr, fixed_m);
  else if (packed && lo)
    k_count_ctx<LOccE, 2, false, true, W><<<g2, kBlk, 0, st>>>(ix, d_pats, nullptr, npat, co, 0,
                                                                nullptr, fixed_m);
  else if (packed && nobar)
    k_count_ctx<OccE, 2, false, true, W, true><<<g2, kBlk, 0, st>>>(ix, d_pats, nullptr, npat, co, 0,
                                                                     nullptr, fixed_m);
  else if (packed)
    k_count_ctx<OccE, 2, false, true, W><<<g2, kBlk, 0, st>>>(ix, d_pats, nullptr, npat, co, 0,
                                                               nullptr, fixed_m);
  else if (lo && nobar)
    k_count_ctx<LOccE, 2, false, false, W, true><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, 0,
                                                                       nullptr, fixed_m);
  else if (lo)
    k_count_ctx<LOccE, 2, false, false, W><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, 0,
                                                                 nullptr, fixed_m);
  else if (W == 8 && U == 1)
    k_count_ctx<OccE, 1, false, false, 8><<<grid_for(npat, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, 0, nullptr, fixed_m);
  else if (W == 8 && U == 4)
    k_count_ctx<OccE, 4, false, false, 8><<<grid_for((npat + 3) / 4, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, 0, nullptr, fixed_m);
  else if (d_offs && can_route(h, ix, flags)) {
    // routing inside the call: the staged kernel counts what its one read answers and lists
    // the long patterns and (unless CS_QT_GENERAL_INLANE) the general-search ones;
    // k_count_long takes both lists from the workspace (or the call's allocation)
    LongBufs lb;
    const bool ws = work.p && work.bytes >= LongBufs::bytes(npat, false);
    cs_status s = lb.alloc(npat, false, st, ws ? work.p : nullptr, false);
    if (s != CS_OK) return s;
    // the general searches a wave lists from (LongList::gen_list): CS_QT_GENERAL_INLANE none,
    // CS_QT_GENERAL_LIST_ALL every one, else the handle's threshold (CS_FM_GENERAL_LIST_MIN)
    // (an index routed for its walk-verified long patterns only, ix.wtext: its general
    // searches stay in the lane unless the call lists every one — C5's 20-mer count is
    // unchanged by the routing)
    lb.ll.gen_list = (flags & CS_QT_GENERAL_INLANE) ? 0u : (flags & CS_QT_GENERAL_LIST_ALL) ? 1u
                     : ix.vsa ? h->gen_list_min : 0u;
    lb.ll.grid = h->list_grid;
    if (nobar)
      k_count_ctx<OccE, 2, false, false, W, true, false, true><<<g2, kBlk, 0, st>>>(
          ix, d_pats, d_offs, npat, co, 0, nullptr, fixed_m, OnePass{}, lb.ll);
    else
      k_count_ctx<OccE, 2, false, false, W, false, false, true><<<g2, kBlk, 0, st>>>(
          ix, d_pats, d_offs, npat, co, 0, nullptr, fixed_m, OnePass{}, lb.ll);
    FMX_HIP(hipGetLastError());
    return launch_count_long(ix, d_pats, d_offs, npat, co, st, fixed_m, &lb.ll, flags);
  } else if (nobar)
    k_count_ctx<OccE, 2, false, false, W, true><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, 0,
                                                                      nullptr, fixed_m);
  else
    k_count_ctx<OccE, 2, false, false, W><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, 0,
                                                                nullptr, fixed_m);
  FMX_HIP(hipGetLastError());
  return CS_OK;
}

uint64_t count_workspace_bytes(const cs_fm_index* h, uint64_t npat) {
  (void)h;
  return LongBufs::bytes(npat, false);
}

cs_status launch_count_ex(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                          uint64_t npat, const CountOut& co, uint32_t flags, hipStream_t st,
                          uint64_t fixed_m, bool packed, const Work& work) {
  if (!npat) return CS_OK;
  flags = call_flags(h, flags);
  const DevIndex ix = query_dev(h, flags);
  if (h->line_fmt == kFmtQwm && ix.ptab_k && ix.lctx && !ix.wide && !packed && qctx_staged(flags)) {
    // the staged quaternary-matrix kernel (C3)
    const unsigned g2 = grid_for((npat + 1) / 2, kBlk, 0xFFFFFFFFu);
    if (co.width == 8)
      k_count_qctx<2, 8><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m);
    else if (co.width == 4)
      k_count_qctx<2, 4><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m);
    else
      k_count_qctx<2, 1><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, fixed_m);
    FMX_HIP(hipGetLastError());
    return CS_OK;
  }
  if (h->line_fmt == kFmtOcc && ix.ptab_k && (ix.vsa || walk_verify(ix)) && !packed &&
      ((flags & CS_Q_LONG) || (!d_offs && fixed_m > kLongPatternM))) {
    // long patterns: one per lane in k_count_long (record, candidates, SA, text window as
    // independent rounds; against the 2-bit text when the index has it), the patterns it
    // does not answer listed for k_count_list; kept out of the staged kernel, whose
    // registers the pattern and text words would take from the 20-mer path.
    // CS_QT_LONG_ROUND2 (CS_FM_LONG_KERNEL=0): round 2's kernel (the general search with
    // look-ahead rounds, k_count<OccE, false, true>); CS_QT_LONG_BYTE_TEXT (=2): the byte text
    // even when the packed text is there.
    if (flags & CS_QT_LONG_ROUND2) {
      k_count<OccE, false, true><<<grid_for(npat, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(ix, d_pats, d_offs,
                                                                                    npat, co, fixed_m);
    } else {
      cs_status r = launch_count_long(ix, d_pats, d_offs, npat, co, st, fixed_m, nullptr, flags);
      if (r != CS_OK) return r;
    }
    FMX_HIP(hipGetLastError());
    return CS_OK;
  }
  if ((h->line_fmt == kFmtOcc || h->line_fmt == kFmtLOcc) && ix.ptab_k) {
    if (co.width == 8) return launch_count_staged<8>(h, ix, d_pats, d_offs, npat, co, st, fixed_m, packed, flags, work);
    if (co.width == 4) return launch_count_staged<4>(h, ix, d_pats, d_offs, npat, co, st, fixed_m, packed, flags, work);
    return launch_count_staged<1>(h, ix, d_pats, d_offs, npat, co, st, fixed_m, packed, flags, work);
  }
  const unsigned g = grid_for(npat, kBlk, 0xFFFFFFFFu);
  if (packed)
    FMX_DISPATCH2(h, k_count, true, g, ix, d_pats, nullptr, npat, co, fixed_m);
  else
    FMX_DISPATCH2(h, k_count, false, g, ix, d_pats, d_offs, npat, co, fixed_m);
  return CS_OK;
}

cs_status launch_count_one(const cs_fm_index* h, const OnePattern& p, uint64_t* out_host,
                           hipStream_t st) {
  FMX_DISPATCH1(h, k_count_one, h->dev(), p, out_host);
  return CS_OK;
}

cs_status launch_count_server(const cs_fm_index* h, uint32_t seq_done, uint64_t idle_ticks,
                              uint64_t life_ticks) {
  hipStream_t st = h->server.st;
  FMX_DISPATCH1(h, k_count_server, h->dev(), h->server.mbox, h->server.resp, seq_done, idle_ticks,
                life_ticks);
  return CS_OK;
}

cs_status launch_count_bytes(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                             uint64_t npat, uint64_t* d_out, hipStream_t st, uint32_t flags) {
  if (!npat) return CS_OK;
  flags = call_flags(h, flags);
  const DevIndex ix = query_dev(h, flags);
  // the patterns k_count_long counts (CS_Q_LONG: all of them; routed device batches: those
  // of kFastM characters or more) take its twin, the rest the general search's
  const bool lk = h->line_fmt == kFmtOcc && ix.ptab_k && (ix.vsa || walk_verify(ix));
  const bool old = (flags & CS_QT_LONG_ROUND2) != 0;
  if (!(lk && (flags & CS_Q_LONG) && !old))
    FMX_DISPATCH(h, k_count_bytes, grid_for(npat, kBlk, 0xFFFFFFFFu), ix, d_pats, d_offs, npat, d_out);
  // (a routed call's long patterns: can_route; ADVICE r03: the twin now follows the call)
  if (lk && !old && ((flags & CS_Q_LONG) || (d_offs && can_route(h, ix, flags)))) {
    const CountOut co{d_out, nullptr, nullptr, 0, 8};
    return launch_count_long_t<true>(ix, d_pats, d_offs, npat, co, st, 0, nullptr, !(flags & CS_Q_LONG),
                                     (flags & CS_QT_LONG_BYTE_TEXT) != 0, (flags & CS_QT_LONG_LOADS8) != 0);
  }
  return CS_OK;
}

cs_status launch_locrec_hits(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                             uint64_t npat, uint8_t* d_hit, hipStream_t st) {
  if (!npat) return CS_OK;
  const DevIndex ix = h->dev();
  k_locrec_hits<<<grid_for(npat, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(ix, d_pats, d_offs, npat, d_hit);
  FMX_HIP(hipGetLastError());
  return CS_OK;
}

// Batch locate in one call (OnePass above): occurrence lines with a prefix table, left
// contexts and the full suffix array (C2, C4).  *done = false when the index has another
// shape (the caller runs the two phases).  Writes d_out_offs (npat + 1) and, when the
// total fits `cap`, every position; synchronises `st` for *total.  CS_QT_NO_ONEPASS
// (CS_FM_LOCATE_ONEPASS=0) turns it off.
// The call's buffers (the lists, then per pattern its count and record, the tiles, the wide
// ranges) in the caller's workspace when it holds locate_workspace_bytes(npat), else in one
// stream-ordered allocation.
// (+ on walk-line indexes the walk list: kLocTile (output index, row) pairs per tile and the
// tiles' counts)
uint64_t locate_walk_bytes(const cs_fm_index* h, uint64_t npat) {
  const uint64_t tiles = (npat + kLocTile - 1) / kLocTile;
  return h->d_sa ? 0 : ((tiles * 4 + 7) & ~7ull) + tiles * kLocTile * 16;
}
uint64_t locate_lo_bytes(const cs_fm_index* h, uint64_t npat, uint64_t wide_cap) {
  const uint64_t tiles = (npat + kLocTile - 1) / kLocTile;
  const uint64_t cb = h->wide ? 8 : 4;  // count bytes (a wide index's counts pass 2^32)
  return ((npat * (8 + cb) + tiles * 8 + 8 + wide_cap * 16 + 7) & ~7ull) + locate_walk_bytes(h, npat) +
         (kScanMaxBlocks + 1) * 8;
}
uint64_t locate_workspace_bytes(const cs_fm_index* h, uint64_t npat) {
  return LongBufs::bytes(npat, false) + locate_lo_bytes(h, npat, npat);
}
cs_status launch_locate_onepass(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                                uint64_t npat, uint64_t limit, uint64_t* d_out_offs,
                                uint64_t* d_out_pos, uint64_t cap, uint64_t* total, hipStream_t st,
                                bool* done, uint32_t flags, const Work& work) {
  *done = false;
  flags = call_flags(h, flags);
  if (flags & CS_QT_NO_ONEPASS) return CS_OK;
  DevIndex ix = h->dev();
  if (flags & CS_Q_NO_LOC_RECORDS) ix.lrec = nullptr;
  // positions from the full SA (narrow), or by the short walk over walk lines with
  // text-position marks (OnePass above); CS_QT_ONEPASS_SA (CS_FM_LOCATE_ONEPASS=2): the full
  // SA only (a walk index takes the two phases)
  const bool by_sa = h->d_sa && !h->wide;
  const bool by_walk = !h->d_sa && h->d_walk && h->d_wssa && h->walk_marks == 2 && !(flags & CS_QT_ONEPASS_SA);
  // the occurrence engine's staged search (context records, locate records, routing), or —
  // round 6 — over the full suffix array any other index: the quaternary matrix's staged
  // search (C3) or the generic one (k_locate_one_gen: the binary wavelet matrix, learned
  // occurrence lines, indexes without prefix table or contexts)
  const bool occ_fast = h->line_fmt == kFmtOcc && ix.ptab_k && ix.lctx && h->lf_exact && (by_sa || by_walk);
  const bool gen = !occ_fast && by_sa;
  if (!occ_fast && !gen) return CS_OK;
  const int kpos = by_sa ? 0 : h->wide ? 2 : 1;
  *done = true;
  if (!npat) {
    FMX_HIP(hipMemsetAsync(d_out_offs, 0, 8, st));
    FMX_HIP(hipStreamSynchronize(st));
    *total = 0;
    return CS_OK;
  }
  constexpr int U = 2;
  const uint64_t tiles = (npat + kBlk * U - 1) / (kBlk * U);
  if (tiles > 0xFFFFFFFFull) {
    set_error("batch too large for one launch");
    return CS_ERR_INVALID;
  }
  // a range wider than kLocSmall rows takes over kLocSmall positions of the capacity, and
  // a pattern has at most one
  const uint64_t wide_cap = std::min<uint64_t>(cap / (kLocSmall + 1) + 1, npat);
  // long patterns (full-SA indexes with the 2-bit text): k_locate_long takes every pattern
  // of a CS_Q_LONG batch (host batches of long patterns pass it) and, routed (can_route),
  // the long patterns the staged kernel lists in the same call
  const bool lk = occ_fast && kpos == 0 && ix.ptext && ix.vtext && ix.vsa;
  const bool long_only = lk && (flags & CS_Q_LONG);
  const bool routed = lk && !long_only && can_route(h, ix, flags);
  static_assert(kLocTile == (uint64_t)kBlk * U, "k_locate_long's tiles are the staged kernel's");
  // locate records: a pattern its record does not answer reads its context record in the
  // same lane (the default), or is listed for the list kernels (CS_QT_LOC_DEFER,
  // CS_FM_LOC_DEFER=1), which search it with the staged stages (locate_miss_one).  Deferring
  // shortens the search kernel (C4 Q_text: 468 -> 410 us) but the 7 % it lists cost the list kernel 130 us of dependent chains: 0.665 against 0.612 ms
  // per call (profiles/r04/ab_defer_fast_misses.json; 0.786 / 0.631 when the list kernel ran
  // the general search, ab_defer.json)
  const bool defer = occ_fast && (flags & CS_QT_LOC_DEFER) && kpos == 0 && ix.lrec;
  // (the long-pattern lists, when the call has them, first, in the same buffer: one
  // stream-ordered allocation per call without a workspace, not two)
  const bool lists = long_only || routed || defer;
  const uint64_t lb_bytes = lists ? LongBufs::bytes(npat, long_only) : 0;
  const uint64_t lo = locate_lo_bytes(h, npat, wide_cap);
  const bool use_ws = work.p && work.bytes >= LongBufs::bytes(npat, false) + lo;
  StreamBuf wsb;
  uint8_t* base;
  uint64_t lo_at;
  if (use_ws) {
    base = static_cast<uint8_t*>(work.p);
    lo_at = LongBufs::bytes(npat, false);  // (the workspace's lists sit where a count's do)
  } else {
    FMX_HIP(wsb.alloc(lb_bytes + lo, st));
    base = wsb.as<uint8_t>();
    lo_at = lb_bytes;
  }
  OnePass op;
  op.rec = reinterpret_cast<uint64_t*>(base + lo_at);
  op.tiles = op.rec + npat;
  op.nwide = reinterpret_cast<unsigned long long*>(op.tiles + tiles);
  op.wide = reinterpret_cast<uint64_t*>(op.nwide + 1);
  if (h->wide) op.cnt64 = op.wide + 2 * wide_cap;
  else op.cnt = reinterpret_cast<uint32_t*>(op.wide + 2 * wide_cap);
  {
    // after the counts (8-B aligned): on walk-line indexes the tiles' walk counts and slots,
    // then the chained scan's flags
    const uint64_t cb = h->wide ? 8 : 4;
    uint8_t* w = reinterpret_cast<uint8_t*>(op.wide + 2 * wide_cap) + ((npat * cb + 7) & ~7ull);
    if (kpos != 0) {
      op.wcnt = reinterpret_cast<uint32_t*>(w);
      op.walks = reinterpret_cast<uint64_t*>(w + ((tiles * 4 + 7) & ~7ull));
    }
    op.sflags = reinterpret_cast<unsigned long long*>(w + locate_walk_bytes(h, npat));
  }
  op.sa = static_cast<const uint32_t*>(h->d_sa);
  op.out_offs = d_out_offs;
  op.out_pos = d_out_pos;
  op.cap = d_out_pos ? cap : 0;
  op.wide_cap = wide_cap;
  // the search kernel's blocks zero their tiles (and block 0 the wide-range counter); a
  // CS_Q_LONG call, which runs no search kernel, zeroes them here
  const bool nobar = count_nobar(flags);
  if (long_only) {
    FMX_HIP(hipMemsetAsync(op.tiles, 0, tiles * 8 + 8, st));
    FMX_HIP(hipMemsetAsync(op.sflags, 0, (kScanMaxBlocks + 1) * 8, st));
  }
  const CountOut co{nullptr, nullptr, nullptr, 0, 8};
  op.defer = defer ? 1u : 0u;
  if (gen) {
    if (h->line_fmt == kFmtQwm && ix.ptab_k && ix.lctx && !ix.wide && qctx_staged(flags))
      k_count_qctx<U, 8, true><<<(unsigned)tiles, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, 0, limit, op);
    else
      FMX_DISPATCH(h, k_locate_one_gen, (unsigned)tiles, ix, d_pats, d_offs, npat, limit, op);
  } else if (long_only || routed || defer) {
    LongBufs lb;
    cs_status ls = lb.alloc(npat, long_only, st, base, !use_ws);
    if (ls != CS_OK) return ls;
    if (long_only)
      ;  // (tiles zeroed above)
    else if (routed && nobar)
      k_count_ctx<OccE, U, true, false, 8, true, true, true><<<(unsigned)tiles, kBlk, 0, st>>>(
          ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op, lb.ll);
    else if (routed)
      k_count_ctx<OccE, U, true, false, 8, false, true, true><<<(unsigned)tiles, kBlk, 0, st>>>(
          ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op, lb.ll);
    else if (nobar)
      k_count_ctx<OccE, U, true, false, 8, true, true><<<(unsigned)tiles, kBlk, 0, st>>>(
          ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op, lb.ll);
    else
      k_count_ctx<OccE, U, true, false, 8, false, true><<<(unsigned)tiles, kBlk, 0, st>>>(
          ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op, lb.ll);
    FMX_HIP(hipGetLastError());
    if (long_only || routed) {
      const unsigned g1 = routed ? long_list_grid(npat, h->list_grid) : grid_for(npat, kBlk, 0xFFFFFFFFu);
      // CS_QT_LONG_LOADS8 (k_count_long's): 8-B pattern / window loads
      const bool v0 = (flags & CS_QT_LONG_LOADS8) != 0;
      if (routed && v0)
        k_locate_long<0, true><<<g1, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, limit, op, lb.ll);
      else if (routed)
        k_locate_long<3, true><<<g1, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, limit, op, lb.ll);
      else if (v0)
        k_locate_long<0, false><<<g1, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, limit, op, lb.ll);
      else
        k_locate_long<3, false><<<g1, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, limit, op, lb.ll);
      FMX_HIP(hipGetLastError());
    }
    if (!routed)  // (a routed k_locate_long searches what it listed and what was deferred)
      k_locate_list<<<long_list_grid(npat, h->list_grid), kBlk, 0, st>>>(ix, d_pats, d_offs, npat, limit, op, lb.ll);
  } else if (kpos == 0 && nobar)
    k_count_ctx<OccE, U, true, false, 8, true, true><<<(unsigned)tiles, kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op);
  else if (kpos == 0)
    k_count_ctx<OccE, U, true, false, 8, false, true><<<(unsigned)tiles, kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op);
  else if (kpos == 1 && nobar)
    k_count_ctx<OccE, U, true, false, 8, true, true, false, true, 1><<<(unsigned)tiles, kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op);
  else if (kpos == 1)
    k_count_ctx<OccE, U, true, false, 8, false, true, false, true, 1><<<(unsigned)tiles, kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op);
  else if (nobar)
    k_count_ctx<OccE, U, true, false, 8, true, true, false, true, 2><<<(unsigned)tiles, kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op);
  else
    k_count_ctx<OccE, U, true, false, 8, false, true, false, true, 2><<<(unsigned)tiles, kBlk, 0, st>>>(
        ix, d_pats, d_offs, npat, co, limit, nullptr, 0, op);
  FMX_HIP(hipGetLastError());
  // (k_locate_walks: 4 blocks per CU, and one tile per thread)
  const unsigned walk_grid = (unsigned)std::max<uint64_t>(list_blocks_per_device(), (tiles + kBlk - 1) / kBlk);
  // the chained scan (a block per 1024 tiles) while its look-back fits a block, else one block
  const uint64_t sblocks = (tiles + kScanBlock - 1) / kScanBlock;
  if (sblocks <= kScanMaxBlocks)
    k_scan_chained<<<(unsigned)sblocks, kScanBlock, 0, st>>>(op.tiles, tiles, d_out_offs + npat, op.sflags);
  else
    k_scan_tiles<<<1, 1024, 0, st>>>(op.tiles, tiles, d_out_offs + npat);
  FMX_HIP(hipGetLastError());
  if (kpos == 0) {
    k_locate_emit<U, 0><<<(unsigned)tiles, kBlk, 0, st>>>(ix, npat, op);
    k_locate_emit_wide<0><<<1024, kBlk, 0, st>>>(ix, op, d_out_offs, d_out_pos);
  } else if (kpos == 1) {
    k_locate_emit<U, 1><<<(unsigned)tiles, kBlk, 0, st>>>(ix, npat, op);
    k_locate_walks<1><<<walk_grid, kBlk, 0, st>>>(ix, op, tiles);
    k_locate_emit_wide<1><<<1024, kBlk, 0, st>>>(ix, op, d_out_offs, d_out_pos);
  } else {
    k_locate_emit<U, 2><<<(unsigned)tiles, kBlk, 0, st>>>(ix, npat, op);
    k_locate_walks<2><<<walk_grid, kBlk, 0, st>>>(ix, op, tiles);
    k_locate_emit_wide<2><<<1024, kBlk, 0, st>>>(ix, op, d_out_offs, d_out_pos);
  }
  FMX_HIP(hipGetLastError());
  FMX_HIP(hipMemcpyAsync(total, d_out_offs + npat, 8, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  return CS_OK;
}

cs_status launch_locate_ranges(const cs_fm_index* h, const uint8_t* d_pats,
                               const uint64_t* d_offs, uint64_t npat, uint64_t limit,
                               uint64_t* d_sp, uint64_t* d_out_offs, uint64_t* total,
                               hipStream_t st, uint32_t flags) {
  StreamBuf cnt, tmp;
  FMX_HIP(cnt.alloc((npat + 1) * 8, st));
  flags = call_flags(h, flags);
  const DevIndex ix = query_dev(h, flags);
  if ((h->line_fmt == kFmtOcc || h->line_fmt == kFmtLOcc) && ix.lctx && ix.ptab_k) {
    // patterns per lane: CS_QT_LOCATE_U1 (CS_FM_LOCATE_U=1) one, else two
    const int U = (flags & CS_QT_LOCATE_U1) ? 1 : 2;
    const CountOut co{cnt.p, nullptr, nullptr, 0, 8};
    const unsigned g2 = grid_for((npat + 1) / 2, kBlk, 0xFFFFFFFFu);
    if (h->line_fmt == kFmtOcc && U == 1)
      k_count_ctx<OccE, 1, true, false, 8><<<grid_for(npat, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(
          ix, d_pats, d_offs, npat, co, limit, d_sp, 0);
    else if (h->line_fmt == kFmtOcc && count_nobar(flags))
      k_count_ctx<OccE, 2, true, false, 8, true><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co,
                                                                      limit, d_sp, 0);
    else if (h->line_fmt == kFmtOcc)  // staged, two patterns per lane
      k_count_ctx<OccE, 2, true, false, 8><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, limit,
                                                                 d_sp, 0);
    else
      k_count_ctx<LOccE, 2, true, false, 8><<<g2, kBlk, 0, st>>>(ix, d_pats, d_offs, npat, co, limit,
                                                                  d_sp, 0);
    FMX_HIP(hipGetLastError());
  } else {
    FMX_DISPATCH(h, k_locate_ranges, grid_for(npat + 1, kBlk, 0xFFFFFFFFu), ix, d_pats,
                 d_offs, npat, limit, d_sp, cnt.as<uint64_t>());
  }
  size_t tb = 0;
  FMX_HIP(rocprim::exclusive_scan(nullptr, tb, cnt.as<uint64_t>(), d_out_offs, (uint64_t)0,
                                  npat + 1, rocprim::plus<uint64_t>(), st));
  FMX_HIP(tmp.alloc(tb, st));
  FMX_HIP(rocprim::exclusive_scan(tmp.p, tb, cnt.as<uint64_t>(), d_out_offs, (uint64_t)0,
                                  npat + 1, rocprim::plus<uint64_t>(), st));
  FMX_HIP(hipMemcpyAsync(total, d_out_offs + npat, 8, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  return CS_OK;
}

// Phase 2 with the full suffix array, fused (no rows buffer): each pattern's rows come
// from its record (as k_expand_rows) and go straight through SA: SA[row] - k (mod n) for
// a window row k characters before the end, SA[row] otherwise.  A lane
// takes a pattern of at most kLocSmall rows (every context window: <= kLocSpanBits);
// wider plain ranges are listed for k_locate_sa_wide, a block per range.
__global__ __launch_bounds__(kBlk) void k_locate_sa(const uint32_t* __restrict__ sa, uint64_t n,
                                                    const uint64_t* __restrict__ sp,
                                                    const uint64_t* __restrict__ offs, uint64_t npat,
                                                    uint64_t* __restrict__ out,
                                                    uint64_t* __restrict__ wide,
                                                    unsigned long long* __restrict__ nwide) {
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < npat; q += gs) {
    const uint64_t a = offs[q], c = offs[q + 1] - a, s = sp[q];
    if (!c) continue;
    if (s & kLocCtx) {
      uint64_t r0, adj;
      uint32_t rel;
      loc_window(s, r0, adj, rel);
      for (uint64_t j = 0; j < c; ++j) {
        const uint32_t f = (uint32_t)__ffs(rel) - 1u;
        const uint64_t p = load_sa(sa, r0 + f);
        st_out(out + a + j, p >= adj ? p - adj : p + n - adj);
        rel &= rel - 1u;
      }
    } else if (c <= kLocSmall) {
      for (uint64_t j = 0; j < c; ++j) st_out(out + a + j, (uint64_t)sa[s + j]);
    } else {
      wide[atomicAdd(nwide, 1ull)] = q;
    }
  }
}

__global__ __launch_bounds__(kBlk) void k_locate_sa_wide(const uint32_t* __restrict__ sa,
                                                         const uint64_t* __restrict__ sp,
                                                         const uint64_t* __restrict__ offs,
                                                         uint64_t* __restrict__ out,
                                                         const uint64_t* __restrict__ wide,
                                                         const unsigned long long* __restrict__ nwide) {
  const uint64_t nw = *nwide;
  for (uint64_t e = blockIdx.x; e < nw; e += gridDim.x) {
    const uint64_t q = wide[e], a = offs[q], c = offs[q + 1] - a, s = sp[q];
    for (uint64_t j = threadIdx.x; j < c; j += blockDim.x) st_out(out + a + j, (uint64_t)sa[s + j]);
  }
}


cs_status launch_locate_walk(const cs_fm_index* h, const uint64_t* d_sp,
                             const uint64_t* d_out_offs, uint64_t npat, uint64_t total,
                             uint64_t* d_out_pos, hipStream_t st, unsigned long long* err_word,
                             uint32_t flags, uint32_t steps_only) {
  if (!total) return CS_OK;
  flags = call_flags(h, flags);
  if (h->d_sa && h->lf_exact && !(flags & CS_Q_NO_FULL_SA)) {  // full suffix array: one read per position
    if (steps_only) {  // no LF steps: one SA read per position
      FMX_HIP(hipMemsetAsync(d_out_pos, 0, total * 8, st));
      return CS_OK;
    }
    StreamBuf wide;
    FMX_HIP(wide.alloc((total / (kLocSmall + 1) + 1) * 8 + 8, st));
    unsigned long long* nwide = wide.as<unsigned long long>();
    FMX_HIP(hipMemsetAsync(nwide, 0, 8, st));
    const uint32_t* sa = static_cast<const uint32_t*>(h->d_sa);
    k_locate_sa<<<grid_for(npat, kBlk, 0xFFFFFFFFu), kBlk, 0, st>>>(
        sa, h->n, d_sp, d_out_offs, npat, d_out_pos, wide.as<uint64_t>() + 1, nwide);
    FMX_HIP(hipGetLastError());
    k_locate_sa_wide<<<1024, kBlk, 0, st>>>(sa, d_sp, d_out_offs, d_out_pos,
                                             wide.as<uint64_t>() + 1, nwide);
    FMX_HIP(hipGetLastError());
    return CS_OK;
  }
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const uint64_t max_blocks = (uint64_t)ncu * 8;  // 8 x 256 threads = full CU
  uint64_t chunk = (total + max_blocks - 1) / max_blocks;
  if (chunk < 64) chunk = 64;
  const unsigned blocks = (unsigned)((total + chunk - 1) / chunk);
  const DevIndex ix = query_dev(h, flags);
  unsigned long long* err =
      err_word ? err_word : reinterpret_cast<unsigned long long*>(h->d_err);
  const bool pow2 = ix.stride_shift != 0xFFFFFFFFu;
  // CS_QT_WALK_PERSISTENT (CS_FM_WALK_PERSISTENT=1): the persistent walk over a rows buffer;
  // CS_QT_WALK_ROWS (CS_FM_WALK_ROWS=1): short walks from an expanded rows buffer
  // (k_expand_rows + k_walk_short) instead of straight from the records
  const bool persistent = (flags & CS_QT_WALK_PERSISTENT) != 0;
  if (ix.walk && h->walk_marks == 2 && !persistent && !(flags & CS_QT_WALK_ROWS)) {
    // short walks straight from the records (no rows buffer)
    StreamBuf wide;
    FMX_HIP(wide.alloc((total / (kLocSmall + 1) + 1) * 8 + 8, st));
    unsigned long long* nwide = wide.as<unsigned long long>();
    FMX_HIP(hipMemsetAsync(nwide, 0, 8, st));
    uint64_t* wl = wide.as<uint64_t>() + 1;
    const bool q = h->line_fmt == kFmtQwm;
    const unsigned g = grid_for(npat, kBlk, 0xFFFFFFFFu);
    if (h->wide && q) {
      k_walk_fused<WalkLineW, true><<<g, kBlk, 0, st>>>(ix, d_sp, d_out_offs, npat, d_out_pos, wl, nwide, err, steps_only);
      k_walk_fused_wide<WalkLineW, true><<<1024, kBlk, 0, st>>>(ix, d_sp, d_out_offs, d_out_pos, wl, nwide, err, steps_only);
    } else if (h->wide) {
      k_walk_fused<WalkLineW, false><<<g, kBlk, 0, st>>>(ix, d_sp, d_out_offs, npat, d_out_pos, wl, nwide, err, steps_only);
      k_walk_fused_wide<WalkLineW, false><<<1024, kBlk, 0, st>>>(ix, d_sp, d_out_offs, d_out_pos, wl, nwide, err, steps_only);
    } else if (q) {
      k_walk_fused<WalkLine, true><<<g, kBlk, 0, st>>>(ix, d_sp, d_out_offs, npat, d_out_pos, wl, nwide, err, steps_only);
      k_walk_fused_wide<WalkLine, true><<<1024, kBlk, 0, st>>>(ix, d_sp, d_out_offs, d_out_pos, wl, nwide, err, steps_only);
    } else {
      k_walk_fused<WalkLine, false><<<g, kBlk, 0, st>>>(ix, d_sp, d_out_offs, npat, d_out_pos, wl, nwide, err, steps_only);
      k_walk_fused_wide<WalkLine, false><<<1024, kBlk, 0, st>>>(ix, d_sp, d_out_offs, d_out_pos, wl, nwide, err, steps_only);
    }
    FMX_HIP(hipGetLastError());
    return CS_OK;
  }
  StreamBuf rows;
  FMX_HIP(rows.alloc(total * 8, st));
  k_expand_rows<<<grid_for(npat, kBlk, 65536), kBlk, 0, st>>>(d_sp, d_out_offs, npat,
                                                              rows.as<uint64_t>());
  FMX_HIP(hipGetLastError());
  const uint64_t* r = rows.as<uint64_t>();
  if (ix.walk && h->walk_marks == 2 && !persistent) {
    const bool q = h->line_fmt == kFmtQwm;
    const unsigned g = grid_for(total, kBlk, 0xFFFFFFFFu);
    if (h->wide && q)
      k_walk_short<WalkLineW, true><<<g, kBlk, 0, st>>>(ix, r, total, d_out_pos, err, steps_only);
    else if (h->wide)
      k_walk_short<WalkLineW, false><<<g, kBlk, 0, st>>>(ix, r, total, d_out_pos, err, steps_only);
    else if (q)
      k_walk_short<WalkLine, true><<<g, kBlk, 0, st>>>(ix, r, total, d_out_pos, err, steps_only);
    else
      k_walk_short<WalkLine, false><<<g, kBlk, 0, st>>>(ix, r, total, d_out_pos, err, steps_only);
  } else if (ix.walk) {
    const bool q = h->line_fmt == kFmtQwm;
    if (h->wide && q)
      k_walk_lines<WalkLineW, true><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else if (h->wide)
      k_walk_lines<WalkLineW, false><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else if (q)
      k_walk_lines<WalkLine, true><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else
      k_walk_lines<WalkLine, false><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
  } else if (h->line_fmt == kFmtQwm) {
    if (pow2) k_walk<QWM, true><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else k_walk<QWM, false><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
  } else if (h->line_fmt == kFmtOcc) {
    if (pow2) k_walk<OccE, true><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else k_walk<OccE, false><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
  } else if (h->line_fmt == kFmtLOcc) {
    if (pow2) k_walk<LOccE, true><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else k_walk<LOccE, false><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
  } else if (h->line_fmt == kFmtLine32) {
    if (pow2) k_walk<WM<Line32>, true><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else k_walk<WM<Line32>, false><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
  } else if (h->line_fmt == kFmtLine32W) {
    if (pow2) k_walk<WM<Line32W>, true><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else k_walk<WM<Line32W>, false><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
  } else {
    if (pow2) k_walk<WM<Line64>, true><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
    else k_walk<WM<Line64>, false><<<blocks, kBlk, 0, st>>>(ix, r, total, chunk, d_out_pos, err, steps_only);
  }
  FMX_HIP(hipGetLastError());
  return CS_OK;  // rows are freed in stream order after the walk
}

void keep_pool(int device) {
  static std::once_flag once[64];
  if (device < 0 || device >= 64) return;
  std::call_once(once[device], [device] {
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    uint64_t keep = ~0ull;  // never trim the pool back on synchronisation
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    (void)hipGetLastError();
  });
}

cs_status check_locate_error(const cs_fm_index* h, unsigned long long* err, hipStream_t st) {
  if (!err) err = reinterpret_cast<unsigned long long*>(h->d_err);
  uint64_t bad = ~0ull;
  FMX_HIP(hipMemcpyAsync(&bad, err, 8, hipMemcpyDeviceToHost, st));
  FMX_HIP(hipStreamSynchronize(st));
  if (bad == ~0ull) return CS_OK;
  FMX_HIP(hipMemsetAsync(err, 0xFF, 8, st));
  FMX_HIP(hipStreamSynchronize(st));
  set_error("locate: LF walk exceeded text length");  // fm_index.cpp:137
  return CS_ERR_LF_OVERRUN;
}

cs_status launch_level_rank1(const cs_fm_index* h, int level, const uint64_t* d_pos, uint64_t k,
                             uint64_t* d_out, hipStream_t st) {
  if (h->line_fmt == kFmtOcc || h->line_fmt == kFmtQwm || h->line_fmt == kFmtLOcc) {
    set_error("level rank1: this index has no binary wavelet levels (occurrence lines)");
    return CS_ERR_UNSUPPORTED;
  }
  if (!k) return CS_OK;
  const unsigned g = grid_for(k, kBlk, 0xFFFFFFFFu);
  if (h->line_fmt == kFmtLine32)
    k_level_rank1<Line32><<<g, kBlk, 0, st>>>(h->dev(), level, d_pos, k, d_out);
  else if (h->line_fmt == kFmtLine32W)
    k_level_rank1<Line32W><<<g, kBlk, 0, st>>>(h->dev(), level, d_pos, k, d_out);
  else
    k_level_rank1<Line64><<<g, kBlk, 0, st>>>(h->dev(), level, d_pos, k, d_out);
  FMX_HIP(hipGetLastError());
  return CS_OK;
}

cs_status launch_wt_rank(const cs_fm_index* h, const uint8_t* d_syms, const uint64_t* d_pos,
                         uint64_t k, uint64_t* d_out, hipStream_t st) {
  if (!k) return CS_OK;
  FMX_DISPATCH(h, k_wt_rank, grid_for(k, kBlk, 0xFFFFFFFFu), h->dev(), d_syms, d_pos, k, d_out);
  return CS_OK;
}

cs_status launch_wt_access(const cs_fm_index* h, const uint64_t* d_pos, uint64_t k,
                           uint8_t* d_out, hipStream_t st) {
  if (!k) return CS_OK;
  FMX_DISPATCH(h, k_lf, grid_for(k, kBlk, 0xFFFFFFFFu), h->dev(), d_pos, k, (uint64_t*)nullptr,
               d_out);
  return CS_OK;
}

cs_status launch_lf(const cs_fm_index* h, const uint64_t* d_rows, uint64_t k, uint64_t* d_out,
                    hipStream_t st) {
  if (!k) return CS_OK;
  FMX_DISPATCH(h, k_lf, grid_for(k, kBlk, 0xFFFFFFFFu), h->dev(), d_rows, k, d_out,
               (uint8_t*)nullptr);
  return CS_OK;
}

}  // namespace fmx
