/*
 * cs_synth.h — synthetic workloads of SURVEY.md §8(d), generated in HBM.
 *
 * Bench/test plumbing (not part of the reference's API): the same splitmix64
 * streams as oracle/fm_oracle.c (orc_gen_dna / orc_gen_bytes /
 * orc_gen_patterns_text), so host and device agree bit for bit.  splitmix64 is
 * counter-based — draw k = mix(seed + (k+1)*0x9E3779B97F4A7C15) — so any slice of
 * a stream (e.g. one rank's query shard) is generated independently.
 */
#ifndef CS_SYNTH_H
#define CS_SYNTH_H

#include <stdint.h>

#include "cs_fmindex.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kind 0: DNA, 32 bases per draw (2 bits each, LSB first) -> "ACGT", then '$'.
 * kind 1: bytes, 8 per draw, b -> 1 + ((b*255)>>8), then 0x00.
 * kind 2: repetitive DNA — position i copies base i mod 2^20 of the kind-0 stream (the
 *         seed sequence), substituted when h_i = splitmix64((seed ^ 0x5DEECE66D) +
 *         (i+1)*0x9E3779B97F4A7C15) has (h_i & 0xFFFF) < 655 by "ACGT"[(h_i >> 16) & 3]
 *         (~0.75 % of bases changed); then '$'.  Substrings recur in every copy: ranges
 *         thousands of rows wide, the heavy-tailed case of genomic text.
 * Writes len+1 bytes to d_out (device).  Asynchronous on stream. */
cs_status cs_synth_text_device(int kind, uint64_t seed, uint64_t len, uint8_t* d_out, void* stream);

/* Q_text patterns first..first+npat-1 of the stream `seed`: pattern k =
 * text[x_k % (N-m), +m).  Writes npat*m bytes (fixed stride m) to d_pats and, if
 * d_offs is not NULL, npat+1 offsets (q*m). */
cs_status cs_synth_patterns_device(const uint8_t* d_text, uint64_t N, uint64_t m, uint64_t first,
                                   uint64_t npat, uint64_t seed, uint8_t* d_pats, uint64_t* d_offs,
                                   void* stream);

/* Q_unif patterns first..first+npat-1 (SURVEY.md §8(d) secondary batch): uniform
 * random symbols, kind 0 ACGT (2 bits per symbol, 32 per draw), kind 1 the σ=256
 * text alphabet (8 bits per symbol, b -> 1 + ((b*255)>>8)); draws x_0 =
 * splitmix64(seed + (k+1)*0x9E3779B97F4A7C15), x_{i+1} = splitmix64(x_i + that
 * constant), symbols LSB first.  Same output layout as cs_synth_patterns_device. */
cs_status cs_synth_random_patterns_device(int kind, uint64_t m, uint64_t first, uint64_t npat,
                                          uint64_t seed, uint8_t* d_pats, uint64_t* d_offs,
                                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CS_SYNTH_H */
