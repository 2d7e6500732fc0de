/*
 * rr_serdes.h — batch C-ABI of the MI355X value serialize/deserialize engine.
 *
 * Replaces, for batches, the reference hot path of RedRock:
 *   robj *desObject(void *buf, size_t len)   rock_serdes.h:49, defined rock_serdes.c:538
 *   sds   serObject(robj *o)                 rock_serdes.h:48, defined rock_serdes.c:512
 *   robj *desString(char *s, size_t len)     rock_serdes.h:47, defined rock_serdes.c:133
 * The reference is one value per call and builds Redis heap objects; a GPU cannot build robj
 * (host pointers), so the batch entry points below decode blobs into the flat device form of
 * rr_format.h and encode that form back into blobs, bit-exact.  The single-value legacy
 * signatures live in rock_serdes_compat.h.
 *
 * Conventions:
 *   - return value: RR_API_OK (0) or a negative RR_API_E* code for the whole call;
 *   - per-value status in rr_value.status (0 = OK), counted into rr_totals.n_bad;
 *   - caller-owned buffers; one rr_ctx per host thread, and a context's calls never run at the
 *     same time on the device (one stream, or streams the caller orders): they share the
 *     context's scratch and its zero-between-calls sums; no hidden host synchronisation in the
 *     device entry points (graph-capturable after rr_ctx_reserve: decode = 2 kernels,
 *     encode = 3 kernels, a batch of at most 4096 values in at most 128 KiB = ONE kernel; all
 *     on the caller's stream).  The only wait is when the context's scratch must grow: it
 *     waits for the whole device (hipDeviceSynchronize: other streams' and contexts' work too)
 *     before freeing the old buffer — rr_ctx_reserve sizes it up front so a hot path never
 *     grows — and under graph capture it fails instead.
 * Plain C: no HIP or torch types in any signature.  Streams are passed as void* (hipStream_t).
 */
#ifndef RR_SERDES_H
#define RR_SERDES_H

#include <stddef.h>
#include <stdint.h>
#include "rr_format.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RR_API_OK        0
#define RR_API_EINVAL   -1   /* bad argument (null pointer, misaligned buffer, n too large) */
#define RR_API_EHIP     -2   /* a HIP runtime call failed */
#define RR_API_ENOMEM   -3   /* device/host allocation failed */
#define RR_API_ENODEV   -4   /* no usable GPU */
#define RR_API_EDEVICE  -5   /* the device reported a failure (rr_totals.bytes == UINT64_MAX) */

/* Value indices and descriptor positions are 32-bit: a batch holds fewer than 2^32 - 1 values
 * (larger n is RR_API_EINVAL) and at most 2^32 - 1 descriptors (later values: RR_E_CAPACITY). */
#define RR_MAX_VALUES   0xFFFFFFFFull

typedef struct rr_ctx rr_ctx;

/* Blob batch: n blobs concatenated; blob i is data[offsets[i] .. offsets[i+1]). */
typedef struct rr_blob_batch {
    uint8_t  *data;         /* 16-byte aligned */
    uint64_t *offsets;      /* n+1 entries, offsets[0] == 0, non-decreasing */
    uint64_t  n;
    uint64_t  data_cap;     /* bytes available at data (encode output capacity) */
} rr_blob_batch;

/* Flat decoded batch (rr_format.h). */
typedef struct rr_flat_batch {
    rr_value *values;       /* n records */
    rr_elem  *elems;        /* elem_cap descriptors */
    uint8_t  *arena;        /* arena_cap bytes, 16-byte aligned */
    uint64_t  n;
    uint64_t  elem_cap;
    uint64_t  arena_cap;
} rr_flat_batch;

/* Written by the device at the end of every batch call.  bytes == UINT64_MAX means the call
 * failed on the device (a look-back wait was cut off) and its outputs must not be used; the
 * host entry points return RR_API_EDEVICE then. */
typedef struct rr_totals {
    uint64_t n_elems;       /* descriptors written (decode) / read (encode) */
    uint64_t bytes;         /* blob bytes read (decode) / written (encode) */
    uint64_t n_bad;         /* values whose status != RR_OK */
    uint64_t payload;       /* payload bytes (string/ziplist bytes) copied */
} rr_totals;

/* ---- context ------------------------------------------------------------------------ */
int  rr_ctx_create(int device, rr_ctx **out);
void rr_ctx_destroy(rr_ctx *ctx);
/* Make scratch space for batches up to n_values values / n_bytes blob bytes (the device calls
 * grow it on demand too, but growing allocates; call this first when capturing graphs).  This
 * also sizes the context's window-sums buffer, which the calls keep zero between calls (their
 * own last workgroups zero it: no zeroing launch). */
int  rr_ctx_reserve(rr_ctx *ctx, uint64_t n_values, uint64_t n_bytes);
/* Options of a context (RR_CTX_* flags; 0 by default).  RR_CTX_NO_SMALL: every call takes the
 * batch pipeline, also a batch small enough for the one-launch kernels (at most 4096 values in
 * at most 128 KiB: decode by in->data_cap, encode by out->data_cap) — for tests and timing. */
#define RR_CTX_NO_SMALL 1u
int  rr_ctx_set_options(rr_ctx *ctx, unsigned flags);
const char *rr_last_error(void);

/* ---- device-resident entry points (all pointers on ctx's device) -------------------- */
/* Decode: needs out->n == in->n; in->data_cap a multiple of 16 with
 * offsets[n] <= data_cap (the work grid is sized from data_cap, so keep it tight) and
 * in->data readable for data_cap bytes; out->arena_cap >= in->data_cap;
 * out->elem_cap >= number of descriptors (an upper bound is rr_decode_elem_bound()). */
int rr_decode_batch(rr_ctx *ctx, const rr_blob_batch *in, rr_flat_batch *out,
                    rr_totals *d_totals, void *stream);
/* Encode: writes out->offsets[0..n] and out->data; out->data_cap bounds the bytes written
 * (values that would not fit are counted bad and not written).  A value is unencodable —
 * size 0, counted in rr_totals.n_bad — when its status is not RR_OK, when its descriptors
 * [elem_base, elem_base + n_elems) pass in->elem_cap, when a payload it references passes
 * in->arena_cap, or when its descriptor kinds do not fit its type (RR_E_ENCODE rules,
 * rr_format.h).  Nothing outside [elems, elems + elem_cap) or [arena, arena + arena_cap) is read. */
int rr_encode_batch(rr_ctx *ctx, const rr_flat_batch *in, rr_blob_batch *out,
                    rr_totals *d_totals, void *stream);

/* Upper bound on descriptors a decode of `bytes` blob bytes in `n` values can produce. */
uint64_t rr_decode_elem_bound(uint64_t n, uint64_t bytes);

/* ---- host entry points (host pointers; stage through the ctx's device buffers; block) */
/* A batch of more than 16 MiB of blobs is decoded in chunks of whole values whose uploads,
 * decodes and downloads overlap on separate streams (results identical to one call); with
 * pinned host buffers (hipHostMalloc / hipHostRegister) the two PCIe directions then run at
 * once.  A batch whose descriptors overflow elem_cap is decoded again in one call.
 * arena may be NULL: the arena is a byte-for-byte mirror of `data` (rr_format.h), so a caller
 * that keeps `data` can index it with the descriptors and skip the arena's download. */
int rr_decode_batch_host(rr_ctx *ctx, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                         rr_value *values, rr_elem *elems, uint64_t elem_cap,
                         uint8_t *arena, rr_totals *totals);
/* Returns bytes via totals->bytes; data_cap bounds the output. */
int rr_encode_batch_host(rr_ctx *ctx, const rr_value *values, const rr_elem *elems,
                         uint64_t n_elems, const uint8_t *arena, uint64_t arena_bytes,
                         uint64_t n, uint8_t *data, uint64_t data_cap, uint64_t *offsets,
                         rr_totals *totals);

/* ---- multi-GPU sharding ---------------------------------------------- */
/* Values are independent: a batch splits into G contiguous value ranges balanced by bytes,
 * shard k starting at the first value whose first byte is at or after k * total / G; each GPU
 * decodes / encodes its shard with the single-GPU calls, and RCCL over xGMI moves data only
 * for a root split or gather (one process per GPU, one rr_comm per process). */
typedef struct rr_shard {
    uint64_t v0, v1;        /* values [v0, v1) of the whole batch */
    uint64_t b0, b1;        /* their bytes [b0, b1) = offsets[v0], offsets[v1] */
} rr_shard;

/* Host: the byte-balanced plan of a batch (host offsets, n+1 entries) into g shards. */
int rr_shard_plan(const uint64_t *offsets, uint64_t n, uint32_t g, rr_shard *plan);
/* Device, in place: place a decoded shard in the whole batch — values' elem_base += elem_add,
 * STR / ZLRAW arena offsets += byte_add (zero-filled slots of malformed values stay zero). */
int rr_flat_rebase(rr_ctx *ctx, rr_value *values, uint64_t n, rr_elem *elems, uint64_t n_elems,
                   uint64_t elem_add, uint64_t byte_add, void *stream);
/* The same placement in host memory (a caller gathering decoded shards on the host).  Both
 * refuse (RR_API_EINVAL) a placement past 2^32 - 1 descriptors: elem_base is 32-bit. */
int rr_flat_rebase_host(rr_value *values, uint64_t n, rr_elem *elems, uint64_t n_elems, uint64_t elem_add,
                        uint64_t byte_add);
/* Where a gather places shard k's descriptors (elem_at[k] = the descriptors of the shards before
 * it, also its rebase's elem_add; its records go at the plan's value range).  Returns the total
 * descriptor count, UINT64_MAX past 2^32 - 1.  rr_gather uses it; elem_at may be NULL. */
uint64_t rr_gather_layout(const uint64_t *shard_elems, int nranks, uint64_t *elem_at);

typedef struct rr_comm rr_comm;
#define RR_COMM_ID_BYTES 128
/* One rank creates the id and hands it to every rank by its own means (MPI, a file, a
 * torch.distributed broadcast, ...); every rank then calls rr_comm_init (collective). */
int rr_comm_get_id(uint8_t id[RR_COMM_ID_BYTES]);
int rr_comm_init(rr_ctx *ctx, int nranks, int rank, const uint8_t id[RR_COMM_ID_BYTES], rr_comm **out);
void rr_comm_destroy(rr_comm *comm);

/* Collective.  The root holds the whole batch (device); every rank gets the plan (nranks
 * entries, host memory) so it can size its shard buffers.  Blocks until the plan is known. */
int rr_split_plan(rr_comm *comm, const rr_blob_batch *whole, int root, rr_shard *plan, void *stream);

/* The point-to-point transfers rr_split / rr_gather post, as data: each entry is one transfer
 * this rank makes — send (RR_XFER_SEND) or receive (RR_XFER_RECV) `bytes` bytes at byte
 * `offset` of the buffer `buf` names, to / from rank `peer`.  rr_split and rr_gather post
 * exactly these lists, in this order, inside one ncclGroup; a caller with another transport
 * (the CPU tests' gloo ranks) runs the same lists.  Zero-byte transfers are left out on both
 * sides.  At most 2 * nranks entries; the count is returned, -1 for a bad argument (and for a
 * gather placed past 2^32 - 1 descriptors). */
enum { RR_XFER_SEND = 0, RR_XFER_RECV = 1 };
enum {
    RR_BUF_WHOLE_DATA = 0, RR_BUF_WHOLE_OFFSETS = 1, RR_BUF_MINE_DATA = 2, RR_BUF_MINE_OFFSETS = 3,   /* split */
    RR_BUF_MINE_VALUES = 4, RR_BUF_MINE_ELEMS = 5, RR_BUF_WHOLE_VALUES = 6, RR_BUF_WHOLE_ELEMS = 7   /* gather */
};
typedef struct {
    int32_t peer, dir, buf, rsv;
    uint64_t offset, bytes;
} rr_xfer;
/* split: the root sends rank k (k != root) its bytes [b0, b1) and offsets [v0, v1]; rank k
 * receives them at offset 0 of its shard buffers (the root's own shard is a local copy) */
int rr_split_schedule(const rr_shard *plan, int nranks, int rank, int root, rr_xfer *out);
/* gather: rank k (k != root) sends the root its records and its shard_elems[k] descriptors;
 * the root receives them at the plan's value range and at rr_gather_layout's position */
int rr_gather_schedule(const rr_shard *plan, const uint64_t *shard_elems, int nranks, int rank, int root,
                       rr_xfer *out);

/* rr_split and rr_gather agree on every rank's arguments (a one-word all-reduce) before any
 * point-to-point call, so a bad argument on one rank returns RR_API_EINVAL on every rank
 * instead of leaving the others' sends and receives waiting.  That agreement reads one word
 * back to the host, so both calls BLOCK the host until the work queued on `stream` before them
 * has run; the transfers themselves are queued on `stream` and not waited for. */
/* Collective.  Each rank receives its shard: mine->data (>= its b1 - b0 bytes, 16-byte
 * aligned) and mine->offsets (v1 - v0 + 1 entries, rebased to 0); mine->n is set.  The root
 * sends ncclSend slices over xGMI (rr_split_schedule).  The root may take its shard in place
 * (mine->data == whole->data + b0, mine->offsets == whole->offsets + v0) only when its shard
 * starts at byte 0 (root 0): the rebase rewrites those offsets. */
int rr_split(rr_comm *comm, const rr_blob_batch *whole, const rr_shard *plan, int root, rr_blob_batch *mine,
             void *stream);
/* Collective.  Every rank passes its decoded shard (mine: n values, mine_elems descriptor
 * slots = that decode's rr_totals.n_elems); the root receives all shards into whole->values /
 * whole->elems (whole->n >= the batch's values, whole->elem_cap >= all shards' descriptors) at
 * their places (rr_gather_layout) and rebases them, so whole equals a decode of the whole batch
 * (whose arena is the whole blob buffer: the arena mirrors it, nothing moves).  Blocks until
 * the shards' sizes are known (an all-gather of one word per rank). */
int rr_gather(rr_comm *comm, const rr_flat_batch *mine, uint64_t mine_elems, const rr_shard *plan, int root,
              rr_flat_batch *whole, void *stream);

/* ---- diagnostics ------------------------------------------------------------------------ */
/* The engine's streaming device copy (16-byte buffer loads, 8 in flight per lane, nontemporal
 * stores): the measured copy bandwidth bench.py prices the decode's roofline against
 * (SURVEY.md §8d).  16-byte aligned device pointers, any byte count; asynchronous on `stream`. */
int rr_copy_device(rr_ctx *ctx, void *dst, const void *src, uint64_t bytes, void *stream);

/* ---- synthetic batches (BASELINE.json configs) ------------------------ */
/* config: 1 = 64-B RAW strings, 2 = Zipf 16B-4KiB strings, 3 = 16-pair hash ziplists,
 *         4 = mixed (config-4 proportions; also the 1M headline batch),
 *         5 = config-4 proportions, seekable: value i drawn from its own seed (the 100M batch
 *             of BASELINE config 5, any shard of it generated alone — rr_gen_range),
 *         10 = edge cases, 11 = mixed with large values.  Host memory, malloc'd. */
typedef struct rr_host_batch {
    uint8_t  *data;
    uint64_t *offsets;
    uint64_t  n;
    uint64_t  bytes;
} rr_host_batch;
int  rr_gen_batch(int config, uint64_t n, uint64_t seed, rr_host_batch *out);
void rr_host_batch_free(rr_host_batch *b);
uint64_t rr_gen_default_seed(int config);   /* 0x5EED0000 + config */
/* Config 5 only, nthreads host threads: blob bytes and descriptor counts (either may be NULL) of
 * values [v0, v1) of the seeded batch, without keeping their bytes; and the blobs of values
 * [v0, v1) (out->offsets relative to the range's first byte) — equal to the same range of
 * rr_gen_batch(5, n, seed) for any n >= v1. */
int rr_gen_sizes(int config, uint64_t v0, uint64_t v1, uint64_t seed, uint64_t *bytes, uint32_t *descs,
                 int nthreads);
int rr_gen_range(int config, uint64_t v0, uint64_t v1, uint64_t seed, rr_host_batch *out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
