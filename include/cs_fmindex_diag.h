/*
 * cs_fmindex_diag.h — measurement twins and parity building blocks of the engine's C ABI.
 *
 * Not part of the drop-in interface (include/cs_fmindex.h): bench.py's roofline accounting
 * (the algorithmic bytes of each query's search, which patterns the locate records answer,
 * the LF steps of each walk) and the parity tests' layer-by-layer checks against the oracle.
 */
#ifndef CS_FMINDEX_DIAG_H
#define CS_FMINDEX_DIAG_H

#include <stdint.h>

#include "cs_fmindex.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Measurement twin of cs_fm_count_device: d_out[q] = the algorithmic HBM bytes of query q's
 * search (distinct rank/occurrence lines per rank pair x line size + the prefix-table entry,
 * records and context sectors), for roofline accounting (bench.py); flags CS_Q_*. */
cs_status cs_fm_count_bytes_device(const cs_fm_index* h, const uint8_t* d_pats,
                                   const uint64_t* d_offs, uint64_t npat, uint64_t* d_out,
                                   uint32_t flags, void* stream);
/* Measurement twin of the one-call locate's locate records (bench.py's locate roofline):
 * d_hit[q] = 1 when the index's locate records (cs_fm_info.locate_record_bytes) answer
 * pattern q in one read, else 0. */
cs_status cs_fm_locate_record_hits_device(const cs_fm_index* h, const uint8_t* d_pats,
                                          const uint64_t* d_offs, uint64_t npat, uint8_t* d_hit,
                                          void* stream);
/* Measurement twin of phase 2 (bench.py's walk roofline): d_steps[j] = the LF steps the
 * walk of reported row j takes before its sample (0 with the full suffix array). */
cs_status cs_fm_locate_walk_steps_device(const cs_fm_index* h, const uint64_t* d_sp,
                                         const uint64_t* d_out_offs, uint64_t npat,
                                         uint64_t total, uint64_t* d_steps, uint32_t flags,
                                         void* stream);

/* Building blocks, for parity tests (host arrays in/out):
 *   level rank1   — BitVector::rank1 of wavelet level l (src/core/bitvector.cpp:165-230);
 *                   CS_ERR_UNSUPPORTED on an occurrence-line index (no levels)
 *   wavelet rank  — WaveletTree::rank (src/core/wavelet.cpp:59-96)
 *   access        — WaveletTree::access (src/core/wavelet.cpp:102-128) = BWT[i]
 *   LF            — FMIndex::LF (src/api/fm_index.hpp:62-66) */
cs_status cs_fm_level_rank1(const cs_fm_index* h, int level, const uint64_t* pos, uint64_t k,
                            uint64_t* out);
cs_status cs_fm_wt_rank(const cs_fm_index* h, const uint8_t* syms, const uint64_t* pos,
                        uint64_t k, uint64_t* out);
cs_status cs_fm_wt_access(const cs_fm_index* h, const uint64_t* pos, uint64_t k, uint8_t* out);
cs_status cs_fm_lf(const cs_fm_index* h, const uint64_t* rows, uint64_t k, uint64_t* out);
cs_status cs_fm_get_C(const cs_fm_index* h, uint64_t* out257);
/* The whole BWT (WaveletTree::access for every row) into device memory d_out (n
 * bytes), asynchronous on stream. */
cs_status cs_fm_bwt_device(const cs_fm_index* h, uint8_t* d_out, void* stream);
cs_status cs_fm_get_ssa(const cs_fm_index* h, uint64_t* out, uint64_t cap, uint64_t* len);

/* Suffix array of text (host in/out) by the device builder — src/core/sais.hpp:8-16
 * order (a proper prefix sorts first). */
cs_status cs_sa_build(const uint8_t* text, uint64_t n, uint32_t* sa_out, int device);


#ifdef __cplusplus
}
#endif
#endif /* CS_FMINDEX_DIAG_H */
