// fm_synth.hip — synthetic texts and Q_text pattern batches in HBM (SURVEY.md
// §8(d)); bit-identical to oracle/fm_oracle.c's generators.
#include "../../include/cs_synth.h"
#include "fm_internal.hpp"

namespace fmx {
namespace {

constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// one thread per draw
__global__ void k_text(int kind, uint64_t seed, uint64_t len, uint8_t* __restrict__ out) {
  const uint64_t per = kind == 0 ? 32 : 8;
  const uint64_t ndraw = (len + per - 1) / per;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t d = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; d < ndraw; d += stride) {
    const uint64_t x = mix64(seed + (d + 1) * kGamma);
    const uint64_t base = d * per;
    if (kind == 0) {
      const char acgt[4] = {'A', 'C', 'G', 'T'};
      if (base + 32 <= len) {
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          uint32_t v = 0;
#pragma unroll
          for (int b = 0; b < 4; ++b) v |= (uint32_t)acgt[(x >> (2 * (4 * k + b))) & 3u] << (8 * b);
          w[k] = v;
        }
        uint4* o = reinterpret_cast<uint4*>(out + base);
        o[0] = make_uint4(w[0], w[1], w[2], w[3]);
        o[1] = make_uint4(w[4], w[5], w[6], w[7]);
      } else {
        for (uint64_t k = 0; base + k < len; ++k) out[base + k] = acgt[(x >> (2 * k)) & 3u];
      }
    } else {
      for (uint64_t k = 0; k < 8 && base + k < len; ++k) {
        const uint64_t b = (x >> (8 * k)) & 0xFFu;
        out[base + k] = (uint8_t)(1 + ((b * 255) >> 8));
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[len] = kind == 0 ? '$' : 0;
}

// Repetitive DNA (kind 2): copies of a 2^20-base seed sequence — the first 2^20 bases
// of the kind-0 stream — each base substituted with probability 655/65536 by a
// uniform one; one thread per 32 positions (they share the seed draw).
constexpr uint64_t kRdnaSeedBits = 20;
constexpr uint64_t kRdnaSalt = 0x5DEECE66Dull;
constexpr uint32_t kRdnaRate = 655;  // of 65536: ~1.0 % drawn, ~0.75 % changed
__global__ void k_text_rdna(uint64_t seed, uint64_t len, uint8_t* __restrict__ out) {
  const char acgt[4] = {'A', 'C', 'G', 'T'};
  const uint64_t ngroup = (len + 31) / 32;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < ngroup; g += stride) {
    const uint64_t i0 = g * 32, o0 = i0 & ((1ull << kRdnaSeedBits) - 1);
    const uint64_t x = mix64(seed + (o0 / 32 + 1) * kGamma);
    uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint64_t h = mix64((seed ^ kRdnaSalt) + (i0 + k + 1) * kGamma);
      const uint32_t b = (h & 0xFFFFu) < kRdnaRate ? (uint32_t)(h >> 16) & 3u : (uint32_t)(x >> (2 * k)) & 3u;
      w[k >> 2] |= (uint32_t)acgt[b] << (8 * (k & 3));
    }
    if (i0 + 32 <= len) {
      uint4* o = reinterpret_cast<uint4*>(out + i0);
      o[0] = make_uint4(w[0], w[1], w[2], w[3]);
      o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
      for (uint64_t k = 0; i0 + k < len; ++k) out[i0 + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[len] = '$';
}

__global__ void k_patterns(const uint8_t* __restrict__ text, uint64_t N, uint64_t m, uint64_t first,
                           uint64_t npat, uint64_t seed, uint8_t* __restrict__ pats,
                           uint64_t* __restrict__ offs) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < npat; q += stride) {
    const uint64_t k = first + q;
    const uint64_t pos = mix64(seed + (k + 1) * kGamma) % (N - m);
    for (uint64_t j = 0; j < m; ++j) pats[q * m + j] = text[pos + j];
    if (offs) {
      offs[q] = q * m;
      if (q + 1 == npat) offs[npat] = npat * m;
    }
  }
}

// Q_unif pattern k: m symbols from the draws x_0 = mix(seed + (k+1)*gamma),
// x_{i+1} = mix(x_i + gamma); DNA takes 2 bits per symbol (32 per draw) -> "ACGT",
// bytes take 8 bits per symbol (8 per draw) -> 1 + ((b*255)>>8), LSB first.
__global__ void k_patterns_unif(int kind, uint64_t m, uint64_t first, uint64_t npat, uint64_t seed,
                                uint8_t* __restrict__ pats, uint64_t* __restrict__ offs) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const char* acgt = "ACGT";
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < npat; q += stride) {
    uint64_t x = mix64(seed + (first + q + 1) * kGamma);
    const uint32_t per = kind == 0 ? 32u : 8u;
    for (uint64_t j = 0; j < m; ++j) {
      if (j && j % per == 0) x = mix64(x + kGamma);
      const uint32_t sh = (uint32_t)(j % per);
      pats[q * m + j] = kind == 0 ? (uint8_t)acgt[(x >> (2 * sh)) & 3u]
                                  : (uint8_t)(1u + ((((x >> (8 * sh)) & 0xFFu) * 255u) >> 8));
    }
    if (offs) {
      offs[q] = q * m;
      if (q + 1 == npat) offs[npat] = npat * m;
    }
  }
}

}  // namespace
}  // namespace fmx

using namespace fmx;

extern "C" {

cs_status cs_synth_text_device(int kind, uint64_t seed, uint64_t len, uint8_t* d_out, void* stream) {
  if (!d_out || kind < 0 || kind > 2) {
    set_error("cs_synth_text_device: bad argument");
    return CS_ERR_INVALID;
  }
  if (kind == 2) {
    k_text_rdna<<<grid_for((len + 31) / 32 + 1, 256, 65536), 256, 0, (hipStream_t)stream>>>(seed, len,
                                                                                          d_out);
    FMX_HIP(hipGetLastError());
    return CS_OK;
  }
  const uint64_t ndraw = (len + 7) / 8;
  k_text<<<grid_for(ndraw, 256, 65536), 256, 0, (hipStream_t)stream>>>(kind, seed, len, d_out);
  FMX_HIP(hipGetLastError());
  return CS_OK;
}

cs_status cs_synth_patterns_device(const uint8_t* d_text, uint64_t N, uint64_t m, uint64_t first,
                                   uint64_t npat, uint64_t seed, uint8_t* d_pats, uint64_t* d_offs,
                                   void* stream) {
  if (!d_text || !d_pats || m == 0 || N <= m) {
    set_error("cs_synth_patterns_device: bad argument");
    return CS_ERR_INVALID;
  }
  if (!npat) return CS_OK;
  k_patterns<<<grid_for(npat, 256, 65536), 256, 0, (hipStream_t)stream>>>(d_text, N, m, first, npat,
                                                                         seed, d_pats, d_offs);
  FMX_HIP(hipGetLastError());
  return CS_OK;
}

cs_status cs_synth_random_patterns_device(int kind, uint64_t m, uint64_t first, uint64_t npat,
                                          uint64_t seed, uint8_t* d_pats, uint64_t* d_offs,
                                          void* stream) {
  if ((kind != 0 && kind != 1) || (npat && !d_pats)) {
    set_error("cs_synth_random_patterns_device: bad argument");
    return CS_ERR_INVALID;
  }
  if (!npat) return CS_OK;
  k_patterns_unif<<<grid_for(npat, 256, 65536), 256, 0, (hipStream_t)stream>>>(
      kind, m, first, npat, seed, d_pats, d_offs);
  FMX_HIP(hipGetLastError());
  return CS_OK;
}

}  // extern "C"
