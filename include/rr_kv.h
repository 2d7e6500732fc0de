/*
 * rr_kv.h — batched key-value I/O around the GPU path.
 *
 * The reference moves one value per RocksDB call: rocksdbapi_write (rocksdbapi.cc:258-274,
 * from dumpValToRock, rock.c:682-697) and rocksdbapi_read (rocksdbapi.cc:206-230, from the
 * rock thread's restore, rock.c:457-474), each wrapped around one serObject / desObject.
 * These calls move a batch per store call and keep the bytes on the GPU in between:
 *
 *   dump     flat values (host) -> one upload -> rr_encode_batch -> [rr_snappy_compress_batch]
 *            -> one download -> ONE write_batch of k puts (RocksDB: a WriteBatch)
 *   restore  ONE multi_get of k keys (RocksDB: MultiGet) -> one upload ->
 *            [rr_snappy_decompress_batch] -> rr_decode_batch -> one download of the flat batch
 *
 * The store is the caller's, through rr_kv_ops (RocksDB's MultiGet / WriteBatch in RedRock;
 * RocksDB is not part of this build).  With RR_KV_SNAPPY the stored values are snappy streams
 * (rr_snappy.h): store-side compression is then turned off (kNoCompression), since the value
 * arrives compressed.
 */
#ifndef RR_KV_H
#define RR_KV_H

#include <stddef.h>
#include <stdint.h>
#include "rr_serdes.h"
#include "rr_rdb.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RR_KV_SNAPPY 1   /* values are stored as snappy raw streams, (de)compressed on the GPU */

typedef struct rr_kv_ops {
    void *user;
    /* k keys of database dbi -> vals[i] / val_lens[i] (allocated by the store, released with
     * free_val); a missing key leaves vals[i] == NULL.  Returns 0 or nonzero on failure. */
    int (*multi_get)(void *user, int dbi, size_t k, const char *const *keys, const size_t *key_lens, void **vals,
                     size_t *val_lens);
    /* k puts applied as one batch.  Returns 0 or nonzero on failure. */
    int (*write_batch)(void *user, int dbi, size_t k, const char *const *keys, const size_t *key_lens,
                       const void *const *vals, const size_t *val_lens);
    void (*free_val)(void *user, void *val);
} rr_kv_ops;

/* Dump k values (host flat batch: values[k], elems[n_elems], arena[arena_bytes]) under keys.
 * A value that cannot be encoded (rr_encode_batch's RR_E_ENCODE) fails the call before any
 * write (RR_API_EINVAL); nothing is written then. */
int rr_kv_dump_batch(rr_ctx *ctx, const rr_kv_ops *kv, int dbi, size_t k, const char *const *keys,
                     const size_t *key_lens, const rr_value *values, const rr_elem *elems, uint64_t n_elems,
                     const uint8_t *arena, uint64_t arena_bytes, int flags);

/* Restore k keys into *out (malloc'd; rr_rdb_flat_free): records, descriptors (slots per
 * rr_format.h) and the arena, which mirrors the k blobs back to back.  A missing key, or a
 * stored value that does not decompress, fails the call (RR_API_EINVAL); a blob that does not
 * decode keeps its nonzero rr_value.status, as rr_decode_batch reports it. */
int rr_kv_restore_batch(rr_ctx *ctx, const rr_kv_ops *kv, int dbi, size_t k, const char *const *keys,
                        const size_t *key_lens, int flags, rr_rdb_flat *out);

#ifdef __cplusplus
}
#endif
#endif
