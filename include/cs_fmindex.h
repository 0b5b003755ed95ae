/*
 * cs_fmindex.h — C ABI of the MI355X-native batched FM-index engine.
 *
 * Drop-in boundary for the reference's query path.  The reference exposes no FFI:
 * its boundary is the C++ class cs::FMIndex (src/api/fm_index.hpp:17-67), linked
 * statically by every caller (the tools/ and tests/ programs).  Each entry point below
 * names the member it replaces.  include/cs/fm_index.hpp re-creates that class on
 * top of this ABI (same names, argument meaning and exceptions), so a caller of the
 * reference swaps the header and links libcs_fmindex.so — see INTEGRATION.md.
 *
 * Conventions
 *  - plain pointers and sizes; no HIP or torch types.  `stream` is a hipStream_t
 *    passed as void* (NULL = the legacy default stream of the handle's device).
 *  - *_device entry points take device pointers (inputs already resident in HBM);
 *    the others take host pointers and stage through HBM themselves.
 *  - a handle is immutable after creation and may be used from several host
 *    threads on distinct streams.
 *  - positions and counts are uint64 (the reference's uint64_t return types,
 *    src/api/fm_index.hpp:26,32).  Texts up to n < 2^38 bytes are indexed (the
 *    reference's uint32 SA/C/SSA stop at 2^32): from n >= 2^32 the
 *    index is "wide" (u64 samples and packed 8-B prefix-table entries, a bucketed
 *    suffix sorter); cs_fm_create takes the reference's own u32 arrays, so n < 2^32.
 *  - on a non-OK status, cs_fm_last_error() returns this thread's message; for
 *    CS_ERR_LF_OVERRUN it is the reference's exact text
 *    "locate: LF walk exceeded text length" (src/api/fm_index.cpp:137).
 */
#ifndef CS_FMINDEX_H
#define CS_FMINDEX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum cs_status {
  CS_OK = 0,
  CS_ERR_INVALID = 1,        /* bad argument (null pointer, n >= 2^32, ...) */
  CS_ERR_OOM = 2,            /* device allocation failed */
  CS_ERR_HIP = 3,            /* HIP runtime error (message in cs_fm_last_error) */
  CS_ERR_LF_OVERRUN = 4,     /* fm_index.cpp:136-138 */
  CS_ERR_SSA_RANGE = 5,      /* fm_index.cpp:141-146 */
  CS_ERR_CAPACITY = 6,       /* caller's output buffer too small; *total says how big */
  CS_ERR_UNSUPPORTED = 7,    /* e.g. open_directory (fm_index.cpp:71-73 throws) */
  CS_ERR_NO_DEVICE = 8       /* no HIP device: the engine never falls back to the CPU */
} cs_status;

/* BuildParams — src/api/fm_index.hpp:11-14.  Only ssa_stride changes the index,
 * as in the reference (S, s and eps are accepted and ignored there too). */
typedef struct cs_build_params {
  uint32_t S;           /* 512 */
  uint32_t s;           /* 64 */
  uint32_t ssa_stride;  /* 32 */
  double eps;           /* 1.0 */
} cs_build_params;

typedef struct cs_fm_index cs_fm_index;

/* Memory / geometry summary of a built index. */
typedef struct cs_fm_info {
  uint64_t n;              /* text length incl. any terminator the caller appended */
  uint32_t ssa_stride;
  uint32_t line_bits;      /* positions per line (224 / 192 / 448 bits; 64 rows in occurrence lines) */
  uint64_t lines_per_level;
  uint64_t rank_bytes;     /* all rank lines in HBM */
  uint64_t ssa_bytes;
  uint32_t active_levels[256]; /* per symbol: bitmask of levels needing a memory access */
  int device;
  uint32_t prefix_k;       /* prefix table: k-mers whose (sp, ep) is precomputed (0 = none) */
  uint32_t prefix_sigma;   /* its alphabet size */
  uint64_t prefix_bytes;
  uint8_t prefix_code[256];/* digit of each symbol in the table alphabet, 255 = not in it */
  uint32_t engine;         /* 0 = binary wavelet matrix in rank lines, 1 = occurrence lines,
                              2 = quaternary wavelet matrix of occurrence lines,
                              3 = learned occurrence lines (model + residual counters) */
  uint32_t line_bytes;     /* bytes per rank / occurrence line (32 or 64) */
  uint32_t levels;         /* rank-line sequences: 8 binary levels, 1..4 quaternary, or 1 */
  uint32_t rare_rows;      /* occurrence lines: BWT rows of rare symbols kept in the table */
  uint32_t walk_marks;     /* locate walk lines: 0 none, 1 sampled rows (row % stride == 0),
                              2 sampled text positions (needs a unique smallest terminator) */
  uint64_t walk_bytes;
  uint32_t context_q;      /* left contexts: symbols per BWT row a count may finish with
                              in one read (0 = none; occurrence lines only) */
  uint32_t position_stride; /* text-position samples (extract, locate walk marks) every
                              position_stride positions; the SSA keeps ssa_stride */
  uint64_t context_bytes;
  uint64_t full_sa_bytes;  /* full suffix array kept for locate (lf_exact builds), 0 = none */
  uint32_t record_bytes;   /* prefix-table entries are context records of 32 or 16 B; 0 = plain table */
  uint32_t text_in_hbm;    /* 1: the text is kept in HBM and extract copies it (as text_.substr) */
  uint64_t packed_text_bytes; /* 2-bit copy of the text (occurrence lines, lf_exact, full SA and
                              text in HBM) that long patterns are verified against; 0 = none.
                              Derived from the text on build / open / import, not saved. */
  uint64_t locate_record_bytes; /* locate records (one-call locate: the SA values of the
                              rows of every k-mer with at most 12 rows (64-B records, read by
                              four lanes together), or of every (k+1)-mer with at most 3 (16 B),
                              beside their contexts, so a 20-mer's position is one read);
                              0 = none.  Derived on build / open / import, not saved. */
  uint64_t locate_record_width; /* 64 or 16 (bytes per record); 0 = none */
  uint64_t device_bytes;   /* round 5: every device allocation the handle owns — each image
                              part with its pad, the derived parts (2-bit text, locate
                              records, rare-symbol positions), the node table, the overrun
                              word and the small-batch arena — i.e. the HBM the index holds */
} cs_fm_info;

void cs_default_build_params(cs_build_params* p);

/* FMIndex::build_from_text — fm_index.hpp:19, fm_index.cpp:16-69.
 * Builds the whole index on `device` (suffix array by prefix doubling, cyclic BWT,
 * C[], row-sampled SSA, and the rank structure: occurrence lines when at most four
 * symbols hold all but 128 BWT rows, else a quaternary wavelet matrix of occurrence
 * lines; environment CS_FM_ENGINE=wavelet selects the reference's binary 8-level
 * wavelet matrix instead).  `text` is a host pointer.
 * HBM footprint: besides the base structures (rank lines, SSA, inverse-SA samples) the
 * build adds optional speed structures while an eighth of the device stays free — walk
 * lines, the k-mer prefix table, left contexts, context records, the full suffix array,
 * the text.  Environment CS_FM_HBM_BUDGET=<bytes>[K|M|G|T] (powers of 1000) caps the
 * whole index instead: the structures are added in that order while the index fits (the
 * prefix table takes the largest k that fits; the full suffix array, when it fits,
 * replaces the walk lines).  Results never depend on the budget, only throughput does
 * (bench.py legs "footprint" and "budget"). */
cs_status cs_fm_build_from_text(const uint8_t* text, uint64_t n, const cs_build_params* p,
                                int device, cs_fm_index** out);
/* Same, with the text already in device memory on `device`. */
cs_status cs_fm_build_from_device_text(const uint8_t* d_text, uint64_t n,
                                       const cs_build_params* p, int device,
                                       cs_fm_index** out);
/* Create from host index arrays built elsewhere — the members the reference's
 * build_from_text leaves in bwt_ (the cyclic BWT, n bytes) and ssa_ (u32 samples
 * SA[k * ssa_stride], ceil(n / ssa_stride) of them), src/api/fm_index.cpp:49-66 —
 * without suffix sorting.  `text` (n bytes, optional, may be NULL) is kept on the
 * host for extract, as text_; without it extract returns CS_ERR_UNSUPPORTED
 * (the arrays carry no inverse-SA samples).  n < 2^32. */
cs_status cs_fm_create(const uint8_t* bwt, uint64_t n, const uint32_t* ssa, uint64_t nsamples,
                       uint32_t ssa_stride, const uint8_t* text, int device, cs_fm_index** out);
/* FMIndex::open_directory — fm_index.hpp:20 ("TODO: on-disk format"); the reference
 * throws (fm_index.cpp:71-73).  Here it opens an index written by
 * cs_fm_save_directory onto device CS_FM_DEVICE (default 0).
 * A reference-style directory holding only its source text (text.txt, as the shipped
 * sample.csidx/) is built on the device the way tools/build_index.cpp builds it ('$'
 * appended unless the text ends in '$' or '\0', ssa_stride 32).  A missing or foreign
 * directory fails with CS_ERR_INVALID ("cannot open: <path>"). */
cs_status cs_fm_open_directory(const char* dir, cs_fm_index** out);
cs_status cs_fm_open_directory_on(const char* dir, int device, cs_fm_index** out);
/* The reference's designed single-file format, CSIDX (src/serialization/serialization.hpp:
 * 1-83: 88-B header "CSIDX", version 1, text_len, eight 8-B-aligned section offsets; the
 * mmap reader serialization.cpp:153-335).  The reference never wired it to FMIndex and its
 * writer does not terminate (serialization.cpp:44-54), so these follow the documented
 * layout: text [u64 len][bytes], bwt [u64 n][bytes], C [u64 257][u32], ssa [u32 stride][pad]
 * [u64 count][u32], footer "CSEND"; the wavelet and vEB sections are neither written nor
 * read (the engine builds its own rank structures from the BWT).
 * cs_fm_open_csidx: the BWT and the SSA as cs_fm_create takes them (no suffix sorting; the
 * C array, when present, must match the BWT), the text when present for extract;
 * cs_fm_open_directory(_on) given a path to such a file opens it the same way.
 * cs_fm_save_csidx: writes one (n < 2^32).  cs_csidx_check: validates a file on the CPU
 * (no device): CS_OK with its n, stride and whether it holds the text. */
cs_status cs_fm_open_csidx(const char* path, int device, cs_fm_index** out);
cs_status cs_fm_save_csidx(const cs_fm_index* h, const char* path);
cs_status cs_csidx_check(const char* path, uint64_t* n, uint32_t* ssa_stride, int* has_text);
/* Write a CSIDX file from host index arrays, on the host (no device): the reference's
 * members bwt_ (n bytes), ssa_ (ceil(n / ssa_stride) u32 samples) and, optional (NULL),
 * text_ — the file IndexWriter would write for them (serialization.cpp:64-147: header,
 * text, BWT, C_ = the BWT's cumulative histogram, SSA, footer; 8-B aligned sections).
 * cs_fm_save_csidx writes through the same writer. */
cs_status cs_csidx_write(const char* path, const uint8_t* bwt, uint64_t n, const uint32_t* ssa,
                         uint64_t nsamples, uint32_t ssa_stride, const uint8_t* text);
/* Writes the index (HBM images of every structure, plus the text when kept) to dir. */
cs_status cs_fm_save_directory(const cs_fm_index* h, const char* dir);
/* Replication of an index across GPUs (export / import of its device image) and the wire
 * form of per-shard counts: include/cs_fmindex_replica.h. */
void cs_fm_destroy(cs_fm_index* h);
cs_status cs_fm_get_info(const cs_fm_index* h, cs_fm_info* out);
const char* cs_fm_last_error(void);

/* FMIndex::count — fm_index.hpp:26, fm_index.cpp:79-101 (one pattern, host). */
cs_status cs_fm_count(const cs_fm_index* h, const uint8_t* pattern, uint64_t m, uint64_t* out);
/* Serving mode for single-pattern count (the p50 path; no reference counterpart —
 * it replaces the per-query kernel launch behind FMIndex::count, fm_index.cpp:79-101).
 * cs_fm_serve_start keeps one wave resident on a private non-blocking stream that
 * polls a request mailbox in pinned host memory; while it is on, cs_fm_count and
 * single-pattern cs_fm_count_batch calls with m <= 124 are answered by it (same
 * results), longer patterns take the launch path.  The wave exits after idle_us
 * without requests (0 = 10 ms) and is relaunched by the next request.  While it is
 * resident, device-wide synchronisation (hipDeviceSynchronize, hipFree, …) waits
 * for it to go idle.  cs_fm_serve_stop shuts it down and waits; cs_fm_destroy
 * does it too.  Calls on one handle are serialised. */
cs_status cs_fm_serve_start(const cs_fm_index* h, uint32_t idle_us);
cs_status cs_fm_serve_stop(const cs_fm_index* h);
/* FMIndex::locate — fm_index.hpp:32, fm_index.cpp:107-157 (one pattern, host).
 * Positions in BWT-row order; at most min(limit, cap) written; *nout = number. */
cs_status cs_fm_locate(const cs_fm_index* h, const uint8_t* pattern, uint64_t m, uint64_t limit,
                       uint64_t* out, uint64_t cap, uint64_t* nout);
/* FMIndex::extract — fm_index.hpp:37, fm_index.cpp:163-167 (clamped substring). */
cs_status cs_fm_extract(const cs_fm_index* h, uint64_t pos, uint64_t len, uint8_t* out,
                        uint64_t* nout);

/* Batched extract on the device (fm_index.cpp:163-167 semantics: pos >= n gives
 * "", len clamped to n - pos) by LF inversion from inverse-SA samples — the text
 * itself is not needed.  Requires a text whose last symbol is unique and the
 * smallest (the standard terminator) and inverse-SA samples; otherwise the host
 * copy of the text (as text_) serves, else CS_ERR_UNSUPPORTED.  out_offs has
 * k+1 entries (CSR into out); if *total > cap: CS_ERR_CAPACITY, out_offs valid. */
cs_status cs_fm_extract_batch(const cs_fm_index* h, const uint64_t* pos, const uint64_t* len,
                              uint64_t k, uint64_t* out_offs, uint8_t* out, uint64_t cap,
                              uint64_t* total);
/* Same with device buffers, asynchronous on `stream`: d_out_offs (k+1 entries) must
 * already hold the clamped lengths' exclusive scan (d_out_offs[q] = sum over r < q of
 * min(len[r], n - pos[r]) for pos[r] < n, else 0); d_out receives the bytes. */
cs_status cs_fm_extract_device(const cs_fm_index* h, const uint64_t* d_pos, const uint64_t* d_len,
                               const uint64_t* d_out_offs, uint64_t k, uint8_t* d_out,
                               void* stream);

/* Batched count: pattern q = pats[offs[q] .. offs[q+1]).  Host buffers; offsets must
 * be non-decreasing (checked: CS_ERR_INVALID).  cs_fm_count_device takes the same
 * layout in device memory, unchecked.  A batch of more than CS_FM_HOST_CHUNK patterns
 * (environment when the handle is created, default 2^21) runs in chunks: each chunk's caller pages are page-locked
 * while the earlier chunks' copies and counts run, and its offsets are checked just before
 * it is queued — so on CS_ERR_INVALID the contents of out_counts are unspecified (the
 * counts of earlier chunks may have been written). */
cs_status cs_fm_count_batch(const cs_fm_index* h, const uint8_t* pats, const uint64_t* offs,
                            uint64_t npat, uint64_t* out_counts, void* stream);
/* Batched locate, host buffers.  out_offs has npat+1 entries (CSR into out_pos).
 * *total = sum_q min(count_q, limit) (0 for empty patterns, fm_index.cpp:109).
 * If *total > cap: CS_ERR_CAPACITY, out_offs valid, out_pos untouched. */
cs_status cs_fm_locate_batch(const cs_fm_index* h, const uint8_t* pats, const uint64_t* offs,
                             uint64_t npat, uint64_t limit, uint64_t* out_offs, uint64_t* out_pos,
                             uint64_t cap, uint64_t* total, void* stream);

/* Device-resident batches (no host staging, asynchronous on `stream` unless stated).
 * Round 6: one count entry and one locate entry, each with query flags
 * and an optional caller workspace, replace rounds 2-5's _ex / _ws / _async / fixed ladders.
 * d_pats may be NULL when every pattern of the batch is empty (the count / locate forms then
 * read d_offs[0] and d_offs[npat] back, synchronising `stream`, and return CS_ERR_INVALID
 * unless they are equal). */
/* Query flags (the `flags` argument of the device entry points).  Every flag leaves the results unchanged and
 * only selects which structures a search may read, so the reference's own loop can
 * be run and timed on any index:
 *   CS_Q_NO_PREFIX     start every search from C[] (fm_index.cpp:84-89): no prefix table
 *   CS_Q_NO_CONTEXTS   step every remaining character through the rank structure
 *                      (fm_index.cpp:90-96): no left contexts, no context records, no
 *                      verification against the text
 *   CS_Q_NO_VERIFY     no verification of narrow ranges against the text (an index
 *                      keeping the full suffix array and the text finishes a search
 *                      whose range is at most 8 rows by comparing the characters left
 *                      with the text before each row's suffix)
 *   CS_Q_NO_FULL_SA    locate phase 2: walk LF to the sampled rows (fm_index.cpp:125-153)
 *                      even when the full suffix array is kept
 *   CS_Q_NO_WALK_LINES locate phase 2: walk the rank structure to the reference's row
 *                      samples (row % ssa_stride == 0) even when walk lines exist
 *   CS_Q_LONG          count and the one-call locate: a hint that the batch holds long
 *                      patterns (32 characters and more) — one pattern per lane in the
 *                      long-pattern kernels (record, candidates, SA entry, 2-bit text
 *                      window), outside the 20-mer kernel (occurrence-line indexes that
 *                      keep the full suffix array and the text; implied by a fixed-length
 *                      batch with m > 31 and by a host batch, cs_fm_count_batch /
 *                      cs_fm_locate_batch, whose patterns are all longer than 31).  Without
 *                      it, the long patterns of a device batch are routed to the same
 *                      kernels inside the call (the 20-mer kernel lists them in the call's
 *                      own buffer; the handle holds no routing state).
 *   CS_Q_NO_LOC_RECORDS the one-call locate without the locate records (the context
 *                      record, then the matching row's SA entry: two dependent reads)
 *                      Results never change. */
#define CS_Q_NO_PREFIX 1u
#define CS_Q_NO_CONTEXTS 2u
#define CS_Q_NO_FULL_SA 4u
#define CS_Q_NO_WALK_LINES 8u
#define CS_Q_NO_VERIFY 16u
#define CS_Q_LONG 32u
#define CS_Q_NO_LOC_RECORDS 64u
/* Tuning selectors (flags bits 8-23: equivalent kernels for tests and A/B measurements,
 * results never change) are declared in cs_fmindex_tuning.h (round 6: kept out of the
 * drop-in API; a caller of the reference's interface never needs them). */

/* Where a batch count writes.  width 8: uint64 counts (the reference's return type,
 * fm_index.hpp:26).  width 4: uint32, exact while n < 2^32 (CS_ERR_INVALID otherwise).
 * width 1: uint8 — a count >= 255 is stored as 255 and listed as a (pattern index, count)
 * pair of uint64 in d_exc (capacity exc_cap pairs); *d_exc_n (device, caller-zeroed)
 * receives the number of such patterns, which may exceed exc_cap: the pairs past it are
 * then not stored.  Narrow widths cut the HBM bytes written per pattern and the bytes a
 * gather of the counts across GPUs moves (bench.py, shard.py). */
typedef struct cs_count_out {
  void* d_counts;
  uint32_t width;
  uint64_t* d_exc;
  uint64_t exc_cap;
  uint64_t* d_exc_n;
} cs_count_out;

/* Device workspace: a count of a device batch routes its long patterns and the patterns its
 * one read cannot finish to lists the next kernel takes, and the one-call locate keeps
 * per-pattern counts, records and tile totals between its kernels.  Without a workspace
 * (d_work NULL or work_bytes too small) a call allocates that memory itself (stream-ordered);
 * cs_fm_workspace_bytes(h, npat) bytes serve a count or a one-call locate of up to npat
 * patterns.  Zero-fill it once before its first use: the calls leave it that way (the list
 * kernel's last block re-zeroes the counters it used).  Results do not depend on it — each
 * call's first kernel claims the list kernels' retire word itself — but a first call on
 * memory that was not zero-filled may scan every list slot.  One workspace serves one call at
 * a time: calls that share it must be ordered (one stream, or events). */
uint64_t cs_fm_workspace_bytes(const cs_fm_index* h, uint64_t npat);

/* FMIndex::count (fm_index.cpp:79-101) of every pattern of a device batch: pattern q =
 * d_pats[d_offs[q] .. d_offs[q+1]) (non-decreasing offsets, unchecked), or, with d_offs NULL,
 * npat patterns of one length fixed_m back to back (pattern q at d_pats + q*fixed_m; k-mer
 * batches read no offsets array); counts as *out says (uint64 = the reference's type); flags
 * CS_Q_* (and CS_QT_*, cs_fmindex_tuning.h); d_work / work_bytes the optional workspace. */
cs_status cs_fm_count_device(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                             uint64_t fixed_m, uint64_t npat, const cs_count_out* out, uint32_t flags,
                             void* d_work, uint64_t work_bytes, void* stream);
/* The same for 2-bit packed DNA patterns (not a reference form: 8 B per pattern
 * instead of m bytes plus an 8-B offset): pattern q is d_packed[q], character i is
 * "ACGT"[(d_packed[q] >> 2i) & 3], i = 0 .. m-1, m <= 32.  Counts equal count() of the
 * byte string those characters spell. */
cs_status cs_fm_count_packed_device(const cs_fm_index* h, const uint64_t* d_packed, uint32_t m,
                                    uint64_t npat, const cs_count_out* out, uint32_t flags,
                                    void* stream);

/* FMIndex::locate (fm_index.cpp:107-157) of every pattern of a device batch in one call:
 * d_out_offs (npat + 1 entries) = the exclusive scan of min(count, limit), and
 * d_out_pos[d_out_offs[q] ..] pattern q's positions in the reference's row order.  Every
 * index that keeps the full suffix array (occurrence lines, the quaternary and binary wavelet
 * matrices, learned lines) and occurrence-line indexes with walk lines and text-position
 * marks (C5) take three launches — search, scan of the per-block totals, positions — and one
 * host synchronisation; otherwise (and under a CS_Q_NO_* structure flag) the two phases below
 * run back to back.  CS_Q_LONG sends every pattern to the long-pattern search.  Returns
 * CS_ERR_CAPACITY with *total set and the offsets written when the positions do not fit `cap`
 * (positions are then incomplete).  Synchronises `stream`. */
cs_status cs_fm_locate_device(const cs_fm_index* h, const uint8_t* d_pats, const uint64_t* d_offs,
                              uint64_t npat, uint64_t limit, uint64_t* d_out_offs, uint64_t* d_out_pos,
                              uint64_t cap, uint64_t* total, uint32_t flags, void* d_work,
                              uint64_t work_bytes, void* stream);
/* locate in two phases, under query flags (e.g. CS_Q_NO_FULL_SA | CS_Q_NO_WALK_LINES runs the
 * reference's row-sampled SSA walk, fm_index.cpp:125-153, on any index).
 * Phase 1, the backward search: d_sp[q] = the pattern's record for phase 2 (the first row of
 * its range, or an encoded window of matching rows when the search finished over the left
 * contexts — treat it as opaque), d_out_offs = exclusive scan of min(count, limit) (npat+1
 * entries).  Synchronises `stream` to return *total. */
cs_status cs_fm_locate_ranges_device(const cs_fm_index* h, const uint8_t* d_pats,
                                     const uint64_t* d_offs, uint64_t npat, uint64_t limit,
                                     uint64_t* d_sp, uint64_t* d_out_offs, uint64_t* total,
                                     uint32_t flags, void* stream);
/* Phase 2: LF walk to the sampled rows and SSA lookup for every reported row (d_out_pos has
 * `total` entries).  sync != 0: synchronises `stream` and returns the LF-overrun error
 * (CS_ERR_LF_OVERRUN, fm_index.cpp:136-138); sync == 0: asynchronous, for timing loops — the
 * overrun is reported by the next cs_fm_locate_check. */
cs_status cs_fm_locate_walk_device(const cs_fm_index* h, const uint64_t* d_sp,
                                   const uint64_t* d_out_offs, uint64_t npat, uint64_t total,
                                   uint64_t* d_out_pos, uint32_t flags, int sync, void* stream);
cs_status cs_fm_locate_check(const cs_fm_index* h, void* stream);

/* Measurement twins and the parity tests' building blocks (per-level BitVector::rank1,
 * WaveletTree::rank / access, LF, C[], the BWT, the SSA, the suffix array): see
 * include/cs_fmindex_diag.h. */

#ifdef __cplusplus
}
#endif
#endif /* CS_FMINDEX_H */
