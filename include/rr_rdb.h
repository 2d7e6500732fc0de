/*
 * rr_rdb.h — batched snapshot restore for BGSAVE / AOF rewrite.
 *
 * RedRock's fork child (rdb.c:1017-1071 rdbSaveKeyValuePair, aof.c:1308-1387) meets every
 * evicted value as shared.valueInRock and asks the parent for it one key at a time over two
 * pipes (rock_rdb.c:240-267 requestSnapshotValByKeyInRdbProcess; the parent's service thread,
 * rock_rdb.c:126-230, reads the RocksDB snapshot and answers), then desObject()s the blob
 * (rock.c:527-550).  One round trip and one decode per key.
 *
 * These calls keep that protocol and batch both ends:
 *
 *   RAW   the reference's wire format unchanged — request {int dbi, size_t key_len, key},
 *         response {size_t val_len, val} — with k requests in flight: rr_rdb_request_batch
 *         writes requests while it reads responses (poll(), so neither pipe can fill up and
 *         deadlock), and rr_rdb_serve answers everything queued with one multi-get.  Either end
 *         interoperates with the reference's serial other end.
 *   FLAT  one request carries k keys (dbi = RR_RDB_FLAT_TAG, then size_t k, then the k RAW
 *         requests); the service decodes the k blobs on its GPU (rr_decode_batch_host — the
 *         parent process holds the GPU; a fork child must not touch the HIP runtime its parent
 *         initialised) and answers with the flat batch: u64 n, u64 n_elems, u64 bytes, then the
 *         n rr_value records, the n_elems rr_elem descriptors and the arena (bytes).  The child
 *         builds robj straight from the records (rr_compat_rdb_load_batch in
 *         rock_serdes_compat.h): no parse on the CPU.
 *
 * The service stops on the request pipe's close (return 0), like the reference's thread.
 */
#ifndef RR_RDB_H
#define RR_RDB_H

#include <stddef.h>
#include <stdint.h>
#include "rr_serdes.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RR_RDB_FLAT_TAG (-0x5244)   /* a dbi no RedRock database has: marks a FLAT request */

/* blobs of one batch: data (16-byte aligned, zero-padded to 16) and offsets[n+1] (malloc'd) */
typedef struct rr_rdb_blobs {
    uint8_t *data;
    uint64_t *offsets;
    uint64_t n;
} rr_rdb_blobs;

/* a decoded batch received over the pipe (malloc'd) */
typedef struct rr_rdb_flat {
    rr_value *values;
    rr_elem *elems;
    uint8_t *arena;
    uint64_t n, n_elems, bytes;
} rr_rdb_flat;

/* the service's snapshot lookup: k keys at once (a RocksDB MultiGet over the snapshot in
 * RedRock).  vals[i] / val_lens[i] out; a missing key is vals[i] == NULL.  Returns 0, or
 * nonzero to stop the service. */
typedef int (*rr_rdb_multiget_fn)(void *user, size_t k, const int *dbis, const char *const *keys,
                                  const size_t *key_lens, void **vals, size_t *val_lens);

/* Child side, RAW: k requests pipelined on fd_req, k responses read from fd_resp into *out.
 * Returns RR_API_OK, or RR_API_EINVAL / RR_API_EHIP-style errors (rr_last_error()); a closed
 * pipe returns RR_API_EINVAL with "pipe closed". */
int rr_rdb_request_batch(int fd_req, int fd_resp, const int *dbis, const char *const *keys, const size_t *key_lens,
                         size_t k, rr_rdb_blobs *out);
void rr_rdb_blobs_free(rr_rdb_blobs *b);

/* Child side, FLAT: one batch request, the decoded batch back. */
int rr_rdb_request_flat(int fd_req, int fd_resp, const int *dbis, const char *const *keys, const size_t *key_lens,
                        size_t k, rr_rdb_flat *out);
void rr_rdb_flat_free(rr_rdb_flat *f);

/* Service side: answers RAW and FLAT requests until fd_req closes (returns 0) or an error
 * (returns nonzero: a missing key, a write error — the reference's `goto err`).  RAW requests
 * already queued are answered together (up to max_batch per multi-get).  ctx: the GPU engine
 * context FLAT requests decode on (NULL: FLAT requests are an error). */
int rr_rdb_serve(int fd_req, int fd_resp, rr_rdb_multiget_fn get, void (*free_val)(void *), void *user,
                 rr_ctx *ctx, size_t max_batch);

#ifdef __cplusplus
}
#endif
#endif
