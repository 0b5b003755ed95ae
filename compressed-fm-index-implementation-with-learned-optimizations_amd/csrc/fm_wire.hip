// fm_wire.hip — the wire form of a count vector for the cross-GPU gather of
// per-shard counts (shard.py).  The reference returns one
// uint64_t per count() (src/api/fm_index.cpp:79-101); shipping those across xGMI
// costs 8 B per pattern, which at 12.5 M patterns per 0.4 ms step and 7 peers per
// receiving GPU is more than the links carry.  The wire form is exact and 1 B per
// pattern: min(count, 255) as uint8 plus a (pattern index, count) pair for every
// count >= 255, in one fixed-size buffer so the gather is a plain collective:
//
//   [u64 pairs][u64 cap][cap x (u64 index, u64 count)][npat x u8]
//
// `pairs` may exceed `cap` (the pairs past it are not stored): the receiver then
// fetches those shards' counts another way (shard.unpack_counts raises).
#include "fm_internal.hpp"

namespace fmx {
namespace {

constexpr unsigned kWireBlk = 256;

// Four counts per lane (one dword of the u8 area), so the stores are coalesced dwords.
__global__ __launch_bounds__(kWireBlk) void k_pack_wire(const uint64_t* __restrict__ counts,
                                                        uint64_t npat, uint64_t cap,
                                                        uint64_t* __restrict__ hdr,
                                                        uint8_t* __restrict__ u8) {
  if (blockIdx.x == 0 && threadIdx.x == 0) hdr[1] = cap;
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; 4 * w < npat; w += gs) {
    uint32_t packed = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t q = 4 * w + i;
      if (q >= npat) break;
      const uint64_t v = counts[q];
      packed |= (uint32_t)(v < 255 ? v : 255) << (8 * i);
      if (v >= 255) {
        const unsigned long long e = atomicAdd(reinterpret_cast<unsigned long long*>(hdr), 1ull);
        if (e < cap) {
          hdr[2 + 2 * e] = q;
          hdr[3 + 2 * e] = v;
        }
      }
    }
    if (4 * w + 4 <= npat) {
      reinterpret_cast<uint32_t*>(u8)[w] = packed;
    } else {
      for (uint64_t q = 4 * w; q < npat; ++q) u8[q] = (uint8_t)(packed >> (8 * (q - 4 * w)));
    }
  }
}

}  // namespace
}  // namespace fmx

using namespace fmx;

extern "C" {

uint64_t cs_counts_wire_bytes(uint64_t npat, uint64_t cap) {
  return 16 + 16 * cap + ((npat + 7) & ~7ull);
}

cs_status cs_counts_pack_wire(const uint64_t* d_counts, uint64_t npat, uint64_t cap, void* d_wire,
                              void* stream) {
  if (!d_wire || (npat && !d_counts)) {
    set_error("null wire pointer");
    return CS_ERR_INVALID;
  }
  hipStream_t st = (hipStream_t)stream;
  uint64_t* hdr = static_cast<uint64_t*>(d_wire);
  FMX_HIP(hipMemsetAsync(hdr, 0, 8, st));  // the pair counter; the kernel writes cap
  uint8_t* u8 = static_cast<uint8_t*>(d_wire) + 16 + 16 * cap;
  k_pack_wire<<<grid_for((npat + 3) / 4 + 1, kWireBlk, 65536), kWireBlk, 0, st>>>(
      d_counts, npat, cap, hdr, u8);
  FMX_HIP(hipGetLastError());
  return CS_OK;
}

}  // extern "C"
