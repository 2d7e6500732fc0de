/*
 * rr_oracle.h — CPU restatement of RedRock's value serdes (src/rock_serdes.c) in plain C.
 *
 * TEST INFRASTRUCTURE: the checker for the HIP engine and the timed CPU baseline of bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.  The product
 * library (redrock_old_amd/) never links or calls it.
 *
 * Parity: pinned by SURVEY.md §8c known-answer vectors K1-K9 and the reference's own vectors
 * (ziplist.c:114-149 byte example, util.c:754-897 string2ll/ll2string, intset.c:361-375) —
 * see tests/golden/.  The reference itself cannot be built or run here (SURVEY.md §8c denial).
 *
 * Two modes:
 *   flat      rro_decode / rro_encode: the same flat form the GPU produces (rr_format.h),
 *             pthreads over value ranges (nthreads >= 1).
 *   faithful  rro_faithful_*: one thread, per-value allocation pattern of serObject/desObject
 *             (sds doubling growth, one malloc per element, dict/skiplist/quicklist builds).
 */
#ifndef RR_ORACLE_H
#define RR_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/rr_format.h"
#include "../include/rr_serdes.h"

#ifdef __cplusplus
extern "C" {
#endif

int rro_string2ll(const char *s, size_t slen, long long *value);   /* util.c:360-424 */
int rro_ll2str(char *buf, long long value);                        /* sds.c:450-479 */
int rro_zip_try_encoding(const uint8_t *s, uint64_t len, long long *v); /* ziplist.c:480 */

/* Parse one ziplist of L bytes.  If out != NULL, writes up to cap entry descriptors whose STR
 * offsets are base + offset-in-ziplist.  Returns RR_OK or RR_E_ZL_CORRUPT; *count = entries. */
int rro_parse_ziplist(const uint8_t *zl, uint64_t L, uint64_t base, rr_elem *out, uint64_t cap,
                      uint64_t *count);

/* Decode blob at data[off, off+len).  Counting mode when out == NULL.  *n_slots = descriptors
 * the blob's members occupy before SET_HT de-duplication (== its reservation when valid);
 * *n_elems = descriptors the value keeps. */
int rro_decode_one(const uint8_t *data, uint64_t off, uint64_t len, rr_value *v,
                   rr_elem *out, uint64_t *n_elems, uint64_t *n_slots, uint64_t *payload);

/* Descriptor slots value b[0, L) owns in a decoded batch (== its descriptor count if valid). */
uint64_t rro_reserve(const uint8_t *b, uint64_t L);

/* Flat batch decode; arena receives the mirror copy of data[0, offsets[n]). */
int rro_decode(const uint8_t *data, const uint64_t *offsets, uint64_t n, rr_value *values,
               rr_elem *elems, uint64_t elem_cap, uint8_t *arena, rr_totals *t, int nthreads);

/* Blob size of one flat value (0 and *status != 0 if it cannot be encoded); elems is the
 * batch's descriptor array (elem_cap entries), arena_cap the arena's size. */
uint64_t rro_encode_size(const rr_value *v, const rr_elem *elems, uint64_t elem_cap, uint64_t arena_cap,
                         int *status);
int rro_encode(const rr_value *values, const rr_elem *elems, uint64_t elem_cap, const uint8_t *arena,
               uint64_t arena_cap, uint64_t n, uint8_t *data, uint64_t data_cap, uint64_t *offsets, rr_totals *t,
               int nthreads);

/* Reference-faithful single-thread mode (rro_faithful.c). Returns 0 on success.
 * decode: blobs -> heap objects (kept alive in an opaque store), then encode them back. */
typedef struct rro_store rro_store;
rro_store *rro_faithful_decode(const uint8_t *data, const uint64_t *offsets, uint64_t n,
                               uint64_t *n_bad);
/* serObject every stored object into out (offsets written); returns total bytes. */
uint64_t rro_faithful_encode(rro_store *s, uint8_t *out, uint64_t cap, uint64_t *offsets);
void rro_store_free(rro_store *s);

int rro_nprocs(void);

#ifdef __cplusplus
}
#endif
#endif
