/*
 * cs_fmindex_replica.h — replication of an index across GPUs and the wire form of per-shard
 * counts (shard.py, bench.py --gpus N).
 *
 * Not part of the drop-in interface (include/cs_fmindex.h): the reference has one process
 * and one index; these move an index's device image between GPUs (a broadcast over RCCL
 * instead of building on every GPU) and pack counts for the gather to rank 0.
 */
#ifndef CS_FMINDEX_REPLICA_H
#define CS_FMINDEX_REPLICA_H

#include <stdint.h>

#include "cs_fmindex.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The index as a device image, for replication across GPUs (e.g. a broadcast over
 * RCCL instead of building on every GPU): export_meta returns the meta text (the
 * directory format's cs_fmindex.meta) and the byte size of each part; export_parts
 * copies the parts into caller device buffers (asynchronous on stream); import
 * creates an index on `device` from a meta and device buffers holding the parts
 * (copied; the buffers may be freed after the call).  The host text is not part of
 * the image. */
cs_status cs_fm_export_meta(const cs_fm_index* h, char* meta, uint64_t cap, uint64_t* meta_len,
                            uint64_t* part_bytes, uint32_t* nparts);
cs_status cs_fm_export_parts(const cs_fm_index* h, void* const* d_dst, void* stream);
cs_status cs_fm_import(const char* meta, uint64_t meta_len, const void* const* d_src,
                       uint32_t nparts, int device, cs_fm_index** out);
/* The same without staging copies (replication at one index's worth of HBM per GPU):
 * export_part_ptrs gives the device address of each of the index's own parts
 * (read-only, valid while h lives) so a broadcast can send straight from them;
 * import_alloc creates a handle on `device` with its parts allocated (contents
 * undefined) and returns their addresses for the caller to fill, e.g. by receiving the
 * broadcast into them; import_commit (after those copies, on any stream) completes the
 * handle — it must not be queried before. */
cs_status cs_fm_export_part_ptrs(const cs_fm_index* h, const void** d_parts, uint32_t cap);
cs_status cs_fm_import_alloc(const char* meta, uint64_t meta_len, int device, cs_fm_index** out,
                             void** d_parts, uint32_t nparts);
cs_status cs_fm_import_commit(cs_fm_index* h);

/* Wire form of a device count vector for the cross-GPU gather of per-shard counts
 * (shard.py): exact and 1 B per pattern — min(count, 255) as uint8
 * plus a (pattern index, count) pair for each count >= 255 — in one fixed-size buffer
 * of cs_counts_wire_bytes(npat, cap) bytes:
 *   [u64 pairs][u64 cap][cap x (u64 index, u64 count)][npat x u8]
 * `pairs` may exceed cap (the pairs past it are not stored).  Asynchronous on stream. */
uint64_t cs_counts_wire_bytes(uint64_t npat, uint64_t cap);
cs_status cs_counts_pack_wire(const uint64_t* d_counts, uint64_t npat, uint64_t cap, void* d_wire,
                              void* stream);


#ifdef __cplusplus
}
#endif
#endif /* CS_FMINDEX_REPLICA_H */
