/* rr_internal.h — what the C host files of the engine share (rr_api.c, rr_shard.c, rr_snappy_api.c). */
#ifndef RR_INTERNAL_H
#define RR_INTERNAL_H

#include "rr_kernels.h"

#define RR_HOST_CHUNK (16ull << 20)   /* pipelined host decode: bytes per chunk (at least) */
#define RR_HOST_MAXCHUNK 64

struct rr_ctx {
    int device;
    unsigned options;            /* RR_CTX_* */
    hipStream_t stream;          /* used by the host entry points */
    uint64_t *scratch;           /* look-back words + counters */
    uint64_t scratch_words;
    int scratch_used;            /* a call has used the scratch (growing it then waits for the device) */
    /* The zero-between-calls sums: [encode group sums, enc words][decode half 0, dec words]
     * [decode half 1][decode half for graph-captured calls].  A decode call adds its window and
     * group sums into one half while its count_kernel zeroes what the previous call left in the
     * other; the calls alternate (dphase), so no kernel has to find out that it finishes last. */
    uint64_t *dsums;
    uint64_t dsums_enc, dsums_dec;   /* words of the encode region / of each decode half */
    uint64_t dext[2];                /* words each decode half holds non-zero (its last call's sums) */
    int dphase;                      /* the half the next decode call uses */
    int dsums_dirty;                 /* a call failed midway: re-zero the whole buffer first */
    int fail_second;             /* test hooks: 1 (rr_debug_fail_second) the next pipeline call stops after its first
                                    kernel; 2 (rr_debug_one_help) the next one-launch decode helps every window */
    /* device staging for host entry points */
    void *d_in, *d_off, *d_vals, *d_elems, *d_arena, *d_out, *d_ooff;
    size_t c_in, c_off, c_vals, c_elems, c_arena, c_out, c_ooff;
    rr_totals *d_totals;
    /* pipelined host decode (rr_api.c): transfer streams, per-chunk events and totals */
    int pipe_ready;
    hipStream_t up, down, aux;
    hipEvent_t ev_up[RR_HOST_MAXCHUNK], ev_dec[RR_HOST_MAXCHUNK];
    rr_totals *d_ktot, *h_ktot;   /* device / pinned host, RR_HOST_MAXCHUNK each */
    uint64_t *h_need;             /* pinned, mapped: per chunk, the arena bytes its encode reads */
    hipEvent_t ev_arena[RR_HOST_MAXCHUNK], ev_enc[RR_HOST_MAXCHUNK], ev_need[RR_HOST_MAXCHUNK];
    /* small batches through the host entry points: one pinned buffer mapped into the device,
     * which the one-launch kernels read their input from and write their output to */
    uint8_t *h_small, *d_small;
    uint32_t small_seq;   /* the one-launch kernels' completion words (small_wait) */
    hipStream_t sstream;  /* the one-launch host calls' stream: the device's highest priority, so a
                           * per-key call is dispatched ahead of batch work queued elsewhere */
    size_t c_small;
};

/* the context's scratch: grow to `words` (waits on the previous call through an event; fails
 * under graph capture), and mark the end of a call's use of it */
int rr_ensure_scratch(rr_ctx *c, uint64_t words, hipStream_t stream);
int rr_mark_scratch(rr_ctx *c, hipStream_t stream);
/* grow a device staging buffer of the host entry points */
int rr_dgrow(void **p, size_t *cap, size_t need);

/* sets rr_last_error() and returns code */
int rr_fail(int code, const char *fmt, ...);
#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) \
    return rr_fail(RR_API_EHIP, "%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); } while (0)

#endif
