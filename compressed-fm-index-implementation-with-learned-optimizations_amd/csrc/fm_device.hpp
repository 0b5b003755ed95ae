// fm_device.hpp — HBM layout of the index and the device-side rank primitives.
//
// Wavelet matrix (the reference's "WaveletTree", src/core/wavelet.cpp:14-53): 8
// levels, level l holds bit (7-l) of the level-l sequence; the next sequence is the
// stable zeros-then-ones partition.  Each level's BitVector (src/core/bitvector.hpp:
// 95-98: bits_ + super_ u32 every 2048 bits + blocks_ u16 every 256 bits) is stored
// re-laid-out as 64-byte RANK LINES:
//
//     struct RankLine { u64 base; u64 w[7]; }   // 64 B, 64-B aligned
//
// covering 448 bits: base = rank1 at the line's first bit (absolute), w[k] = bits
// [448L + 64k, +64) LSB-first.  rank1(i) = base + popcount of the bits of line i/448
// below i — one 64-B HBM granule per rank instead of the reference's three arrays.
// rank1(i) equals BitVector::rank1(i) for every 0 <= i <= n (tests/test_gpu_parity
// checks every position against the oracle).  A sentinel line past n makes
// rank1(n) (the reference's count_ones() special case, bitvector.cpp:168-170) a
// plain line read.
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
constexpr int kLineWords = 7;                 // payload words per line
constexpr uint32_t kLineBits = 64 * kLineWords;  // 448
constexpr int kNodes = 255;                   // internal nodes, levels 0..7
constexpr uint8_t kPure = 1, kPureBit = 2;

struct alignas(64) RankLine {
  uint64_t base;
  uint64_t w[kLineWords];
};
static_assert(sizeof(RankLine) == 64, "rank line must be one 64-B granule");

// Everything the query kernels read besides the rank lines; copied into LDS by
// every block (8.5 KB).
struct NodeTable {
  uint64_t S[kNodes];        // node start in its level
  uint64_t R[kNodes];        // rank1_l(S)
  uint64_t Z[kLevels];       // zeros per level (size - ones)
  uint64_t C[257];           // fm_index.cpp:36-47 (u64)
  uint64_t S8[256];          // start of each symbol's run after the last level
  uint8_t flags[256];        // kPure | kPureBit per node
};

struct DevIndex {
  const RankLine* lines;     // kLevels * nlines
  uint64_t nlines;           // per level = n/448 + 1
  uint64_t n;
  const uint32_t* ssa;       // row-sampled SA (fm_index.cpp:57-66), u32 as the reference
  uint64_t nsamples;
  uint32_t stride;
  uint32_t stride_shift;     // log2(stride) when stride is a power of two, else 0xFFFFFFFF
  const NodeTable* table;    // global copy
};

__host__ __device__ inline int node_id(int level, uint32_t prefix) {
  return (1 << level) - 1 + (int)prefix;
}

// Line index / offset of bit position p.  p < 2^38 so p>>6 fits 32 bits and the
// division by 7 is a 32-bit multiply-high.
__device__ __forceinline__ void line_of(uint64_t p, uint32_t& q, uint32_t& o) {
  const uint32_t g = (uint32_t)(p >> 6);
  q = g / (uint32_t)kLineWords;
  o = (uint32_t)(p - (uint64_t)q * kLineBits);
}

// Load one rank line as four 16-B vector loads (global_load_dwordx4).
__device__ __forceinline__ void load_line(const RankLine* __restrict__ lines, uint64_t idx,
                                          uint4 (&v)[4]) {
  const uint4* p = reinterpret_cast<const uint4*>(lines + idx);
  v[0] = p[0];
  v[1] = p[1];
  v[2] = p[2];
  v[3] = p[3];
}

__device__ __forceinline__ uint64_t u64_of(uint32_t lo, uint32_t hi) {
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// popcount of the first o bits of the 448-bit payload (o in [0, 448]).
__device__ __forceinline__ uint32_t prefix_pop(const uint4 (&v)[4], uint32_t o) {
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

__device__ __forceinline__ uint32_t bit_at(const uint4 (&v)[4], uint32_t o) {
  const uint32_t wd = 2 + (o >> 5);  // dword index within the 16-dword line
  const uint32_t dw[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                           v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
  uint32_t d = 0;
#pragma unroll
  for (int k = 2; k < 16; ++k) d = (wd == (uint32_t)k) ? dw[k] : d;
  return (d >> (o & 31)) & 1u;
}

__device__ __forceinline__ uint64_t line_base(const uint4 (&v)[4]) {
  return u64_of(v[0].x, v[0].y);
}

// rank1_l(p) with one 64-B line read.
__device__ __forceinline__ uint64_t rank1_dev(const DevIndex& ix, int level, uint64_t p) {
  uint32_t q, o;
  line_of(p, q, o);
  uint4 v[4];
  load_line(ix.lines, (uint64_t)level * ix.nlines + q, v);
  return line_base(v) + prefix_pop(v, o);
}

}  // namespace fmx
