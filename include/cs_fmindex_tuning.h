/*
 * cs_fmindex_tuning.h — per-call tuning selectors of the C ABI (include/cs_fmindex.h).
 *
 * Not part of the drop-in interface: a caller of the reference's cs::FMIndex never sets
 * these.  They are flags bits that choose among kernels computing the same results, for
 * the parity tests (every kernel a selector reaches is checked against the oracle) and for
 * A/B timing of one kernel against another on one index.
 */
#ifndef CS_FMINDEX_TUNING_H
#define CS_FMINDEX_TUNING_H

/* Tuning selectors (round 5): flags bits 8-24 choose among equivalent kernels for tests and
 * A/B measurements — results never change.  A handle takes its defaults from the CS_FM_*
 * environment once, when it is created (build, create, open, import: the variable named
 * beside each bit), and a call's flags are ORed over them: a call can add a selector but
 * cannot clear one the handle's environment set (a handle created with CS_FM_LONG_ROUTE=0
 * never routes).  No count, locate or extract call reads the environment.
 *   CS_QT_BARRIER         staged count / locate phase 1: the general search behind a block-wide
 *                         LDS copy of the node table (CS_FM_COUNT_NOBAR=0)
 *   CS_QT_NO_ROUTE        no routing inside the call: the staged kernel searches long
 *                         patterns itself (CS_FM_LONG_ROUTE=0)
 *   CS_QT_COUNT_U1 / _U4  staged count: one / four patterns per lane (CS_FM_COUNT_U=1 / 4)
 *   CS_QT_LONG_LOADS8     long-pattern kernels: 8-B pattern and window loads (CS_FM_LONG_V16=0)
 *   CS_QT_LONG_ROUND2     CS_Q_LONG counts through round 2's kernel (CS_FM_LONG_KERNEL=0)
 *   CS_QT_LONG_BYTE_TEXT  long-pattern kernels against the byte text (CS_FM_LONG_KERNEL=2)
 *   CS_QT_QCTX_UNSTAGED   quaternary matrix: one pattern per lane (CS_FM_QCTX_STAGED=0)
 *   CS_QT_NO_ONEPASS      cs_fm_locate_device runs the two phases (CS_FM_LOCATE_ONEPASS=0)
 *   CS_QT_ONEPASS_SA      the one-call locate only over the full SA (CS_FM_LOCATE_ONEPASS=2)
 *   CS_QT_LOC_DEFER       one-call locate: locate-record misses to the list kernel
 *                         (CS_FM_LOC_DEFER=1)
 *   CS_QT_LOCATE_U1       locate phase 1: one pattern per lane (CS_FM_LOCATE_U=1)
 *   CS_QT_WALK_ROWS       phase 2 walks from an expanded rows buffer (CS_FM_WALK_ROWS=1)
 *   CS_QT_WALK_PERSISTENT phase 2: the persistent walk kernel (CS_FM_WALK_PERSISTENT=1)
 *   CS_QT_GENERAL_INLANE  routed count: the staged kernel's lanes run the general searches
 *                         (patterns the one read cannot finish) themselves; by default a wave
 *                         holding at least CS_FM_GENERAL_LIST_MIN (2) of them lists them for
 *                         the list kernel (CS_FM_GENERAL_INLANE=1)
 *   CS_QT_GENERAL_LIST_ALL routed count: every wave lists its general searches
 *                         (CS_FM_GENERAL_LIST_ALL=1)
 *   CS_QT_MAP_LDS         staged count / locate: characters mapped through the LDS symbol table
 *                         even for the standard DNA code (default: four per dword in registers;
 *                         CS_FM_MAP_LDS=1) */
#define CS_QT_BARRIER (1u << 8)
#define CS_QT_NO_ROUTE (1u << 9)
#define CS_QT_COUNT_U1 (1u << 10)
#define CS_QT_COUNT_U4 (1u << 11)
#define CS_QT_LONG_LOADS8 (1u << 12)
#define CS_QT_LONG_ROUND2 (1u << 13)
#define CS_QT_LONG_BYTE_TEXT (1u << 14)
#define CS_QT_QCTX_UNSTAGED (1u << 15)
#define CS_QT_NO_ONEPASS (1u << 16)
#define CS_QT_ONEPASS_SA (1u << 17)
#define CS_QT_LOC_DEFER (1u << 18)
#define CS_QT_LOCATE_U1 (1u << 19)
#define CS_QT_WALK_ROWS (1u << 20)
#define CS_QT_WALK_PERSISTENT (1u << 21)
#define CS_QT_GENERAL_INLANE (1u << 22)
#define CS_QT_GENERAL_LIST_ALL (1u << 23)
#define CS_QT_MAP_LDS (1u << 24)

#include "cs_fmindex.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Build options (round 6): the engine, footprint and tuning-default choices of a build as
 * "NAME=VALUE" pairs separated by spaces, commas or semicolons.  NAME is one of the CS_FM_*
 * variables cs_fm_build_from_text reads from the environment, with or without the CS_FM_
 * prefix, in any case: ENGINE=wavelet|occ|qwm|learned, HBM_BUDGET=40G, FULL_SA=0, WALK=0,
 * WALK_MARKS=row, PREFIX_K=12, LCTX=0, CTX_RECORDS=0|1|16, LOC_RECORDS=0, LOC_REC64=1,
 * DEVICE_TEXT=0, PACKED_TEXT=0, WIDE=1, PSTRIDE=8, LINE_BYTES=64, SA_BUILDER=bucketed,
 * PASS_MAX=<bytes>, the handle defaults of the selectors above (LONG_ROUTE=0, COUNT_U=4 ...),
 * GENERAL_LIST_MIN, LIST_GRID, HOST_CHUNK.  With an options string (empty included) the build
 * reads no environment variable: a name not given takes its default.  options == NULL is
 * cs_fm_build_from_text / cs_fm_build_from_device_text (text_on_device != 0), which read the
 * environment.  A malformed pair or an unknown name fails with CS_ERR_INVALID
 * (cs_fm_last_error names it).  Results never depend on the options, only footprint and
 * throughput do. */
cs_status cs_fm_build_with_options(const uint8_t* text, uint64_t n, int text_on_device,
                                   const cs_build_params* p, const char* options, int device,
                                   cs_fm_index** out);
/* The calling thread's build options for every handle it constructs from now on — build,
 * create, open_directory, import — in the same "NAME=VALUE" form; NULL returns the thread to
 * the environment.  cs_fm_build_with_options's own options take precedence for that call. */
cs_status cs_fm_set_build_options(const char* options);

#ifdef __cplusplus
}
#endif

#endif /* CS_FMINDEX_TUNING_H */
