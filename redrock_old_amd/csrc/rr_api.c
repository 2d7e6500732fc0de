/*
 * rr_api.c — the C host layer of the engine (plain C99 over the HIP runtime C API).
 *
 * Implements include/rr_serdes.h: contexts, argument checks, device-resident batch calls
 * (a hipMemsetAsync of the look-back words + one kernel, no host sync) and host-pointer
 * variants that stage through pinned buffers and the context's device buffers.
 */
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rr_internal.h"

static __thread char g_err[256];
const char *rr_last_error(void) { return g_err; }
int rr_fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}
#define fail rr_fail
#define ensure_scratch rr_ensure_scratch
#define mark_scratch rr_mark_scratch
#define dgrow rr_dgrow

int rr_ctx_create(int device, rr_ctx **out) {
    if (!out) return fail(RR_API_EINVAL, "out is NULL");
    *out = NULL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RR_API_ENODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RR_API_EINVAL, "device %d out of range", device);
    HIPCHK(hipSetDevice(device));
    rr_ctx *c = (rr_ctx *)calloc(1, sizeof *c);
    if (!c) return fail(RR_API_ENOMEM, "calloc");
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        free(c);
        return fail(RR_API_EHIP, "hipStreamCreate");
    }
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (hipStreamCreateWithPriority(&c->sstream, hipStreamNonBlocking, prio_hi) != hipSuccess) {
        hipStreamDestroy(c->stream);
        free(c);
        return fail(RR_API_EHIP, "hipStreamCreateWithPriority");
    }
    if (hipMalloc((void **)&c->d_totals, sizeof(rr_totals)) != hipSuccess) {
        hipStreamDestroy(c->sstream);
        hipStreamDestroy(c->stream);
        free(c);
        return fail(RR_API_ENOMEM, "hipMalloc totals");
    }
    *out = c;
    return RR_API_OK;
}

static void dfree(void **p, size_t *c) { if (*p) hipFree(*p); *p = NULL; *c = 0; }

void rr_ctx_destroy(rr_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->scratch) hipFree(c->scratch);
    if (c->dsums) hipFree(c->dsums);
    dfree(&c->d_in, &c->c_in); dfree(&c->d_off, &c->c_off); dfree(&c->d_vals, &c->c_vals);
    dfree(&c->d_elems, &c->c_elems); dfree(&c->d_arena, &c->c_arena); dfree(&c->d_out, &c->c_out);
    dfree(&c->d_ooff, &c->c_ooff);
    if (c->d_totals) hipFree(c->d_totals);
    if (c->h_small) hipHostFree(c->h_small);
    if (c->pipe_ready) {
        for (int k = 0; k < RR_HOST_MAXCHUNK; k++) {
            hipEventDestroy(c->ev_up[k]); hipEventDestroy(c->ev_dec[k]);
            hipEventDestroy(c->ev_arena[k]); hipEventDestroy(c->ev_enc[k]); hipEventDestroy(c->ev_need[k]);
        }
        hipStreamDestroy(c->up);
        hipStreamDestroy(c->down);
        hipStreamDestroy(c->aux);
        hipHostFree(c->h_need);
        hipFree(c->d_ktot);
        hipHostFree(c->h_ktot);
    }
    hipStreamDestroy(c->sstream);
    hipStreamDestroy(c->stream);
    free(c);
}

/* Grow the scratch.  Kernels of earlier calls — on whatever stream, or replays of a captured
 * graph — may still be using the old buffer: growing (rare: rr_ctx_reserve sizes it up front)
 * waits for the whole device (hipDeviceSynchronize: every stream on it, other contexts', torch's
 * and RCCL's work included — rr_ctx_reserve is the way to never pay it on a hot path).  (Round 4 recorded an event after every call for this wait: one HIP call
 * more per call, on the path small batches are bound by.)  Growing allocates, which a stream
 * under graph capture cannot do: size the scratch with rr_ctx_reserve before capturing. */
int rr_ensure_scratch(rr_ctx *c, uint64_t words, hipStream_t stream) {
    if (c->scratch && words <= c->scratch_words) return RR_API_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (stream && hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
        return fail(RR_API_EINVAL, "scratch too small under graph capture: call rr_ctx_reserve first");
    HIPCHK(hipSetDevice(c->device));
    if (c->scratch) {
        if (c->scratch_used) HIPCHK(hipDeviceSynchronize());
        hipFree(c->scratch);
        c->scratch = NULL;
    }
    uint64_t want = words + words / 4 + 64;
    if (hipMalloc((void **)&c->scratch, want * sizeof(uint64_t)) != hipSuccess)
        return fail(RR_API_ENOMEM, "hipMalloc scratch (%llu words)", (unsigned long long)want);
    c->scratch_words = want;
    c->scratch_used = 0;
    return RR_API_OK;
}

/* The zero-between-calls sums (rr_internal.h): the encode's group sums, E4's block 0 zeroes
 * what E3 read; the decode's window and group sums, double-buffered — each call adds into one
 * half while its count_kernel (or the one-launch decode) zeroes what the previous call left in the
 * other — plus a half for graph-captured decodes, which a captured zeroing kernel re-zeroes at every
 * replay.  So no two-launch kernel has to learn that it finishes last (round 4 found that with a
 * returning atomic at every window's end); the one-launch form's last window by index gathers the
 * others' end words and leaves its words zero itself.
 * Zeroed once when (re)allocated; like the scratch, growing waits on the previous call and is
 * refused under graph capture.  A call that failed midway leaves dsums_dirty: the next call
 * zeroes the whole buffer first. */
static int is_capturing(hipStream_t stream) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return stream && hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
static int ensure_dsums(rr_ctx *c, uint64_t dec_words, uint64_t enc_words, hipStream_t stream) {
    if (c->dsums && dec_words <= c->dsums_dec && enc_words <= c->dsums_enc) {
        /* a failed call left sums non-zero: a captured call would bake them into its graph (its
         * first replay's offsets wrong), so it is refused until an uncaptured call re-zeroes them
         *  */
        if (c->dsums_dirty && is_capturing(stream))
            return fail(RR_API_EINVAL, "a failed call left the context's sums dirty: make one call outside the capture first");
        if (c->dsums_dirty) {
            HIPCHK(hipMemsetAsync(c->dsums, 0, (c->dsums_enc + 3 * c->dsums_dec) * sizeof(uint64_t), stream));
            c->dsums_dirty = 0;
            c->dext[0] = c->dext[1] = 0;
        }
        return RR_API_OK;
    }
    if (is_capturing(stream)) return fail(RR_API_EINVAL, "decode sums too small under graph capture: call rr_ctx_reserve first");
    HIPCHK(hipSetDevice(c->device));
    if (c->dsums) {
        if (c->scratch_used) HIPCHK(hipDeviceSynchronize());
        hipFree(c->dsums);
        c->dsums = NULL;
    }
    uint64_t d = dec_words > c->dsums_dec ? dec_words : c->dsums_dec, e = enc_words > c->dsums_enc ? enc_words : c->dsums_enc;
    d += d / 4 + 64;
    e += e / 4 + 64;
    if (hipMalloc((void **)&c->dsums, (e + 3 * d) * sizeof(uint64_t)) != hipSuccess)
        return fail(RR_API_ENOMEM, "hipMalloc decode sums (%llu words)", (unsigned long long)(e + 3 * d));
    HIPCHK(hipMemsetAsync(c->dsums, 0, (e + 3 * d) * sizeof(uint64_t), stream));
    if (!stream) HIPCHK(hipStreamSynchronize(NULL));
    c->dsums_enc = e;
    c->dsums_dec = d;
    c->dext[0] = c->dext[1] = 0;
    c->dsums_dirty = 0;
    return RR_API_OK;
}

/* after a call's launches: the scratch has been used (a later growth waits for the device) */
int rr_mark_scratch(rr_ctx *c, hipStream_t stream) {
    (void)stream;
    c->scratch_used = 1;
    return RR_API_OK;
}

int rr_ctx_set_options(rr_ctx *c, unsigned flags) {
    if (!c || (flags & ~RR_CTX_NO_SMALL)) return fail(RR_API_EINVAL, "rr_ctx_set_options: bad argument");
    c->options = flags;
    return RR_API_OK;
}
/* test hook (not in rr_serdes.h): the context's next pipeline decode or encode launches only
 * its first kernel and fails, leaving the zero-between-calls sums as a failed second launch or
 * an aborted stream would (tests/test_gpu_small.py) */
int rr_debug_fail_second(rr_ctx *c) {
    if (!c) return fail(RR_API_EINVAL, "ctx is NULL");
    c->fail_second = 1;
    return RR_API_OK;
}
/* test hook (not in rr_serdes.h): the context's next one-launch decode sums every earlier
 * window itself, as for windows whose workgroups have not started (the look-back's help path) */
int rr_debug_one_help(rr_ctx *c) {
    if (!c) return fail(RR_API_EINVAL, "ctx is NULL");
    c->fail_second = 2;
    return RR_API_OK;
}
#define SMALL_DEC(c, n, cap) (!((c)->options & RR_CTX_NO_SMALL) && rr_small_decode_fits((n), (cap)))
#define SMALL_ENC(c, n, cap) (!((c)->options & RR_CTX_NO_SMALL) && rr_small_encode_fits((n), (cap)))

int rr_ctx_reserve(rr_ctx *c, uint64_t n_values, uint64_t n_bytes) {
    if (!c) return fail(RR_API_EINVAL, "ctx is NULL");
    uint64_t a = rr_encode_scratch_words(n_values, (n_bytes + 15) & ~15ull), b = rr_decode_scratch_words((n_bytes + 15) & ~15ull, n_values);
    int rc = ensure_scratch(c, a > b ? a : b, NULL);
    const uint64_t sd = rr_decode_sums_words((n_bytes + 15) & ~15ull), se = rr_encode_sums_words(n_values);
    return rc ? rc : ensure_dsums(c, sd, se, NULL);
}


uint64_t rr_decode_elem_bound(uint64_t n, uint64_t bytes) {
    /* every descriptor but a value's first consumes >= 2 blob bytes (ziplist entry / intset
     * member minimum); the first may come from the 5-byte header alone. */
    return n + bytes / 2;
}

static int aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

int rr_decode_batch(rr_ctx *c, const rr_blob_batch *in, rr_flat_batch *out, rr_totals *d_totals, void *stream) {
    if (!c || !in || !out) return fail(RR_API_EINVAL, "NULL argument");
    if (out->n != in->n) return fail(RR_API_EINVAL, "out->n != in->n");
    if (in->n >= RR_MAX_VALUES) return fail(RR_API_EINVAL, "batch too large (value indices are 32-bit)");
    if (in->n && (!in->data || !in->offsets || !out->values || !out->arena))
        return fail(RR_API_EINVAL, "NULL buffer");
    if (!aligned16(in->data) || !aligned16(out->arena)) return fail(RR_API_EINVAL, "data/arena not 16-byte aligned");
    if (in->data_cap & 15) return fail(RR_API_EINVAL, "data_cap must be a multiple of 16");
    if (out->arena_cap < in->data_cap) return fail(RR_API_EINVAL, "arena_cap < data_cap");
    HIPCHK(hipSetDevice(c->device));   /* (the launch helpers' per-device facts: this context's device) */
    if (SMALL_DEC(c, in->n, in->data_cap)) {   /* one launch, no scratch */
        HIPCHK(rr_launch_decode_small(in->data, in->offsets, in->n, out->values, out->elems, out->elem_cap, out->arena,
                                      in->data_cap, d_totals, NULL, 0, (hipStream_t)stream));
        return RR_API_OK;
    }
    const uint64_t nsums = rr_decode_sums_words(in->data_cap);
    int rc = ensure_scratch(c, rr_decode_scratch_words(in->data_cap, in->n), (hipStream_t)stream);
    if (!rc) rc = ensure_dsums(c, nsums, 0, (hipStream_t)stream);
    if (rc) return rc;
    const int first_only = c->fail_second;
    c->fail_second = 0;
    const int capturing = is_capturing((hipStream_t)stream);
    uint64_t *half[3];
    for (int h = 0; h < 3; h++) half[h] = c->dsums + c->dsums_enc + (uint64_t)h * c->dsums_dec;
    uint64_t *use, *zero = NULL, nzero = 0;
    if (capturing) {   /* the graph's own half, re-zeroed by a captured kernel at every replay */
        use = half[2];
        HIPCHK(rr_launch_zero_words(use, nsums, (hipStream_t)stream));
    } else {           /* this call's half; the call zeroes what the previous call left in the other */
        const int x = c->dphase, y = 1 - x;
        use = half[x];
        zero = half[y];
        nzero = c->dext[y];
        c->dext[y] = 0;
        c->dext[x] = nsums;
        c->dphase = y;
    }
    const hipError_t e = rr_launch_decode(in->data, in->offsets, in->n, out->values, out->elems, out->elem_cap,
                                          out->arena, c->scratch, use, zero, nzero, in->data_cap, d_totals,
                                          (hipStream_t)stream, first_only);
    rc = mark_scratch(c, (hipStream_t)stream);
    if (e != hipSuccess || first_only == 1) {
        c->dsums_dirty = 1;
        return first_only == 1 ? fail(RR_API_EHIP, "decode: second launch withheld (rr_debug_fail_second)")
                          : fail(RR_API_EHIP, "decode launch: %s", hipGetErrorString(e));
    }
    return rc;
}

int rr_encode_batch(rr_ctx *c, const rr_flat_batch *in, rr_blob_batch *out, rr_totals *d_totals, void *stream) {
    if (!c || !in || !out) return fail(RR_API_EINVAL, "NULL argument");
    if (out->n != in->n) return fail(RR_API_EINVAL, "out->n != in->n");
    if (in->n >= RR_MAX_VALUES) return fail(RR_API_EINVAL, "batch too large (value indices are 32-bit)");
    if (!out->offsets) return fail(RR_API_EINVAL, "NULL offsets");
    if (in->n && (!in->values || !out->data)) return fail(RR_API_EINVAL, "NULL buffer");
    if ((uintptr_t)out->data & 15) return fail(RR_API_EINVAL, "out->data must be 16-byte aligned");
    HIPCHK(hipSetDevice(c->device));
    if (SMALL_ENC(c, in->n, out->data_cap)) {   /* one launch, no scratch */
        HIPCHK(rr_launch_encode_small(in->values, in->elems, in->elem_cap, in->arena, in->arena_cap, in->n, out->data,
                                      out->data_cap, out->offsets, d_totals, NULL, 0, (hipStream_t)stream));
        return RR_API_OK;
    }
    int rc = ensure_scratch(c, rr_encode_scratch_words(in->n, out->data_cap), (hipStream_t)stream);
    if (!rc) rc = ensure_dsums(c, 0, rr_encode_sums_words(in->n), (hipStream_t)stream);
    if (rc) return rc;
    const int first_only = c->fail_second == 1;   /* (2: the decode's help hook, not an encode's) */
    c->fail_second = 0;
    const hipError_t e = rr_launch_encode(in->values, in->elems, in->elem_cap, in->arena, in->arena_cap, in->n,
                                          out->data, out->data_cap, out->offsets, c->scratch, c->dsums, d_totals,
                                          (hipStream_t)stream, first_only);
    rc = mark_scratch(c, (hipStream_t)stream);
    if (e != hipSuccess || first_only) {
        c->dsums_dirty = 1;
        return first_only ? fail(RR_API_EHIP, "encode: second launch withheld (rr_debug_fail_second)")
                          : fail(RR_API_EHIP, "encode launch: %s", hipGetErrorString(e));
    }
    return rc;
}

/* diagnostics (tools/time_copy.py; not in rr_serdes.h): one of the copy kernel's shapes */
int rr_copy_shape(rr_ctx *c, void *dst, const void *src, uint64_t bytes, int shape, void *stream) {
    if (!c || (bytes && (!dst || !src)) || (((uintptr_t)dst | (uintptr_t)src) & 15)) return fail(RR_API_EINVAL, "rr_copy_shape");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(rr_launch_copy_shape((uint8_t *)dst, (const uint8_t *)src, bytes, shape, (hipStream_t)stream));
    return RR_API_OK;
}

int rr_copy_device(rr_ctx *c, void *dst, const void *src, uint64_t bytes, void *stream) {
    if (!c || (bytes && (!dst || !src))) return fail(RR_API_EINVAL, "NULL argument");
    if (((uintptr_t)dst | (uintptr_t)src) & 15) return fail(RR_API_EINVAL, "rr_copy_device: pointers must be 16-byte aligned");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(rr_launch_copy((uint8_t *)dst, (const uint8_t *)src, bytes, (hipStream_t)stream));
    return RR_API_OK;
}

/* grow a device staging buffer (host entry points only) */
int rr_dgrow(void **p, size_t *cap, size_t need) {
    if (need <= *cap && *p) return RR_API_OK;
    if (*p) hipFree(*p);
    *p = NULL;
    *cap = 0;
    size_t want = need + need / 8 + 256;
    if (hipMalloc(p, want) != hipSuccess) return fail(RR_API_ENOMEM, "hipMalloc %zu", want);
    *cap = want;
    return RR_API_OK;
}
#define GROW(P, C, N) do { int r_ = dgrow((void **)&(P), &(C), (N)); if (r_) return r_; } while (0)

/* ---- pipelined host decode -------------------------------------------------------------
 * A batch of more than one RR_HOST_CHUNK goes in chunks of whole values (at most
 * RR_HOST_MAXCHUNK): every chunk's blob bytes and offsets are queued up at once on the `up`
 * stream; chunk k decodes on the context stream once its bytes are in (its descriptors placed
 * after the earlier chunks', its elem_base rebased on the device), and its records, descriptors
 * and arena slice go down on the `down` stream while later chunks are still going up.  With
 * pinned host buffers (hipHostMalloc / hipHostRegister) the two PCIe directions overlap;
 * pageable buffers still work, staged by the runtime.  The device layout is the whole batch's
 * (offsets, arena mirror and data_cap are global), so a chunk's decode is the whole-batch decode
 * restricted to its values: results are identical to the one-call path. */
static int pipe_init(rr_ctx *c) {
    if (c->pipe_ready) return RR_API_OK;
    HIPCHK(hipStreamCreateWithFlags(&c->up, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->down, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    for (int k = 0; k < RR_HOST_MAXCHUNK; k++) {
        HIPCHK(hipEventCreateWithFlags(&c->ev_up[k], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_dec[k], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_arena[k], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_enc[k], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->ev_need[k], hipEventDisableTiming));
    }
    HIPCHK(hipHostMalloc((void **)&c->h_need, RR_HOST_MAXCHUNK * RR_NEED_BLOCKS * sizeof(uint64_t), hipHostMallocMapped));
    HIPCHK(hipMalloc((void **)&c->d_ktot, RR_HOST_MAXCHUNK * sizeof(rr_totals)));
    HIPCHK(hipHostMalloc((void **)&c->h_ktot, RR_HOST_MAXCHUNK * sizeof(rr_totals), hipHostMallocDefault));
    c->pipe_ready = 1;
    return RR_API_OK;
}

/* chunk cuts: cut[k] = first value whose first byte is at or after k * bytes / K */
static int plan_chunks(const uint64_t *offsets, uint64_t n, uint64_t bytes, uint64_t *cut) {
    uint64_t K = (bytes + RR_HOST_CHUNK - 1) / RR_HOST_CHUNK;
    if (K > RR_HOST_MAXCHUNK) K = RR_HOST_MAXCHUNK;
    int m = 0;
    cut[m++] = 0;
    for (uint64_t k = 1; k < K; k++) {
        const uint64_t target = bytes / K * k;
        uint64_t lo = cut[m - 1], hi = n;   /* first v in [lo, n] with offsets[v] >= target */
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo) / 2;
            if (offsets[mid] >= target) hi = mid; else lo = mid + 1;
        }
        if (lo > cut[m - 1] && lo < n) cut[m++] = lo;
    }
    cut[m] = n;
    return m;   /* chunks */
}

static int decode_host_pipelined_run(rr_ctx *c, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                                     rr_value *values, rr_elem *elems, uint64_t elem_cap, uint8_t *arena,
                                     rr_totals *totals, uint64_t bytes, size_t pbytes, const uint64_t *cut, int K) {
    int rc;
    uint8_t *d_in = (uint8_t *)c->d_in, *d_arena = (uint8_t *)c->d_arena;
    uint64_t *d_off = (uint64_t *)c->d_off;
    rr_value *d_vals = (rr_value *)c->d_vals;
    rr_elem *d_elems = (rr_elem *)c->d_elems;
    /* the stream of the previous host call is done with the staging buffers: wait for it */
    HIPCHK(hipEventRecord(c->ev_dec[0], c->stream));
    HIPCHK(hipStreamWaitEvent(c->up, c->ev_dec[0], 0));
    HIPCHK(hipMemsetAsync(d_in + bytes, 0, pbytes + 16 - bytes, c->up));
    HIPCHK(hipMemsetAsync(d_arena + bytes, 0, pbytes + 16 - bytes, c->up));
    for (int k = 0; k < K; k++) {
        const uint64_t v0 = cut[k], v1 = cut[k + 1], b0 = offsets[v0], b1 = offsets[v1];
        if (b1 > b0) HIPCHK(hipMemcpyAsync(d_in + b0, data + b0, b1 - b0, hipMemcpyHostToDevice, c->up));
        HIPCHK(hipMemcpyAsync(d_off + v0, offsets + v0, (v1 - v0 + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->up));
        HIPCHK(hipEventRecord(c->ev_up[k], c->up));
    }
    rr_totals sum = {0, 0, 0, 0};
    uint64_t E = 0;   /* descriptor slots of the earlier chunks */
    for (int k = 0; k < K; k++) {
        const uint64_t v0 = cut[k], v1 = cut[k + 1], nk = v1 - v0, b0 = offsets[v0], b1 = offsets[v1];
        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_up[k], 0));
        rr_blob_batch in = {d_in, d_off + v0, nk, pbytes};
        const uint64_t ek = E < elem_cap ? E : elem_cap;   /* (past elem_cap: nothing is written) */
        rr_flat_batch out = {d_vals + v0, d_elems + ek, d_arena, nk, elem_cap - ek, pbytes};
        rc = rr_decode_batch(c, &in, &out, c->d_ktot + k, c->stream);
        if (rc) return rc;
        HIPCHK(rr_launch_flat_rebase(d_vals + v0, nk, NULL, 0, E, 0, c->stream));
        HIPCHK(hipMemcpyAsync(&c->h_ktot[k], c->d_ktot + k, sizeof(rr_totals), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipEventRecord(c->ev_dec[k], c->stream));
        HIPCHK(hipEventSynchronize(c->ev_dec[k]));   /* (later chunks keep going up meanwhile) */
        const rr_totals t = c->h_ktot[k];
        if (t.bytes == ~0ull) return fail(RR_API_EDEVICE, "decode: device-side failure (look-back timeout)");
        HIPCHK(hipStreamWaitEvent(c->down, c->ev_dec[k], 0));
        HIPCHK(hipMemcpyAsync(values + v0, d_vals + v0, nk * sizeof(rr_value), hipMemcpyDeviceToHost, c->down));
        const uint64_t ne = E >= elem_cap ? 0 : t.n_elems < elem_cap - E ? t.n_elems : elem_cap - E;
        if (ne && elems) HIPCHK(hipMemcpyAsync(elems + E, d_elems + E, ne * sizeof(rr_elem), hipMemcpyDeviceToHost, c->down));
        if (b1 > b0 && arena) HIPCHK(hipMemcpyAsync(arena + b0, d_arena + b0, b1 - b0, hipMemcpyDeviceToHost, c->down));
        E += t.n_elems;
        sum.n_elems += t.n_elems;
        sum.bytes = t.bytes;   /* (the offsets are the whole batch's: a chunk reports its end) */
        sum.n_bad += t.n_bad;
        sum.payload += t.payload;
    }
    HIPCHK(hipStreamSynchronize(c->down));
    if (E > elem_cap) return 1;   /* the batch overflows elem_cap: the caller redoes it in one call */
    if (totals) *totals = sum;
    return RR_API_OK;
}

/* On an error after the uploads are queued, the transfers still in flight would keep writing
 * the caller's host buffers (downloads) and the staging buffers the next call reuses (uploads):
 * wait for both transfer streams before reporting it. */
static int decode_host_pipelined(rr_ctx *c, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                                 rr_value *values, rr_elem *elems, uint64_t elem_cap, uint8_t *arena,
                                 rr_totals *totals, uint64_t bytes, size_t pbytes, const uint64_t *cut, int K) {
    int rc = pipe_init(c);
    if (rc) return rc;
    rc = decode_host_pipelined_run(c, data, offsets, n, values, elems, elem_cap, arena, totals, bytes, pbytes, cut, K);
    if (rc != RR_API_OK && rc != 1) {
        c->dsums_dirty = 1;   /* a chunk's kernels may not all have run */
        (void)hipStreamSynchronize(c->up);
        (void)hipStreamSynchronize(c->down);
        (void)hipStreamSynchronize(c->stream);
    }
    return rc;
}

/* ---- small batches through the host entry points --------------------------------------
 * One pinned host buffer, mapped into the device, holds the call's input and output: the
 * one-launch kernel reads the input from it (16-byte loads over PCIe) and writes the records
 * there; the host copies in before the launch and out after one stream synchronisation.  No
 * device staging, no transfer calls: the per-value path of the compat shim (desObject /
 * serObject) pays one launch and one synchronisation. */
static int small_grow(rr_ctx *c, size_t need) {
    if (need <= c->c_small && c->h_small) return RR_API_OK;
    if (c->h_small) HIPCHK(hipHostFree(c->h_small));
    c->h_small = c->d_small = NULL;
    c->c_small = 0;
    const size_t want = need + need / 2 + 4096;
    HIPCHK(hipHostMalloc((void **)&c->h_small, want, hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer((void **)&c->d_small, c->h_small, 0));
    c->c_small = want;
    return RR_API_OK;
}
#define AL16(x) (((x) + 15) & ~(size_t)15)

/* Wait for a one-launch kernel by its completion word in the mapped staging (signal_done in
 * rr_kernels.hip) instead of a stream synchronisation.  The stream is polled now and then, so a
 * kernel that faulted (the stream reports an error) or ended without the word cannot hang it. */
static int small_wait(rr_ctx *c, const uint32_t *flag, uint32_t seq) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int yielding = 0;
    for (uint64_t k = 1;; ++k) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return RR_API_OK;
        /* spin ~50 us (a lone call's kernel ends well inside it), then give the core away
         * between polls: behind another context's long batch the caller (the Redis main
         * thread, through the shim) must not burn a core until that batch drains */
        if (yielding) sched_yield();
        else if ((k & 255) == 0) {
            clock_gettime(CLOCK_MONOTONIC, &t1);
            yielding = (t1.tv_sec - t0.tv_sec) * 1000000000L + (t1.tv_nsec - t0.tv_nsec) > 50000L;
        }
        if ((k & 4095) == 0 || (yielding && (k & 63) == 0)) {
            const hipError_t q = hipStreamQuery(c->sstream);
            if (q == hipSuccess) {
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return RR_API_OK;
                return fail(RR_API_EDEVICE, "one-launch kernel ended without its completion word");
            }
            if (q != hipErrorNotReady) {
                c->dsums_dirty = 1;   /* (an earlier pipeline call on the stream may have stopped midway) */
                (void)hipGetLastError();
                return fail(RR_API_EDEVICE, hipGetErrorString(q));
            }
        }
        __builtin_ia32_pause();
    }
}

static int decode_host_small(rr_ctx *c, const uint8_t *data, const uint64_t *offsets, uint64_t n, rr_value *values,
                             rr_elem *elems, uint64_t elem_cap, uint8_t *arena, rr_totals *totals) {
    const uint64_t bytes = offsets[n];
    const size_t o_off = 0, o_dat = AL16((n + 1) * sizeof(uint64_t)), o_tot = o_dat + AL16(bytes) + 16,
                 o_flag = o_tot + sizeof(rr_totals), o_val = AL16(o_flag + 4), o_el = AL16(o_val + n * sizeof(rr_value)),
                 end = o_el + elem_cap * sizeof(rr_elem);
    int rc = small_grow(c, end);
    if (rc) return rc;
    uint8_t *h = c->h_small, *d = c->d_small;
    /* the previous call on this context is done with the buffer (its own synchronisation) */
    memcpy(h + o_off, offsets, (n + 1) * sizeof(uint64_t));
    if (bytes) memcpy(h + o_dat, data, bytes);
    memset(h + o_dat + bytes, 0, AL16(bytes) + 16 - bytes);
    uint32_t seq = ++c->small_seq;
    if (!seq) seq = ++c->small_seq;   /* (0 is the cleared word) */
    __atomic_store_n((uint32_t *)(h + o_flag), 0u, __ATOMIC_RELAXED);
    HIPCHK(rr_launch_decode_small(d + o_dat, (const uint64_t *)(d + o_off), n, (rr_value *)(d + o_val),
                                  (rr_elem *)(d + o_el), elem_cap, NULL, AL16(bytes), (rr_totals *)(d + o_tot),
                                  (uint32_t *)(d + o_flag), seq, c->sstream));
    rc = small_wait(c, (const uint32_t *)(h + o_flag), seq);
    if (rc) return rc;
    rr_totals t;
    memcpy(&t, h + o_tot, sizeof t);
    if (n) memcpy(values, h + o_val, n * sizeof(rr_value));
    const uint64_t ne = t.n_elems < elem_cap ? t.n_elems : elem_cap;
    if (ne && elems) memcpy(elems, h + o_el, ne * sizeof(rr_elem));
    if (bytes && arena) memcpy(arena, data, bytes);   /* the arena mirrors the blob bytes */
    if (totals) *totals = t;
    return RR_API_OK;
}

int rr_decode_batch_host(rr_ctx *c, const uint8_t *data, const uint64_t *offsets, uint64_t n, rr_value *values,
                         rr_elem *elems, uint64_t elem_cap, uint8_t *arena, rr_totals *totals) {
    if (!c || !offsets || (n && (!data || !values))) return fail(RR_API_EINVAL, "NULL argument");
    if (n >= RR_MAX_VALUES) return fail(RR_API_EINVAL, "batch too large (value indices are 32-bit)");
    /* elem_base is 32-bit (rr_format.h): past 2^32 - 1 descriptors a value gets RR_E_CAPACITY,
     * as in the one-call path, and the chunks' running descriptor base never wraps */
    if (elem_cap > 0xFFFFFFFFull) elem_cap = 0xFFFFFFFFull;
    HIPCHK(hipSetDevice(c->device));
    uint64_t bytes = offsets[n];
    size_t pbytes = (size_t)((bytes + 15) & ~15ull);
    if (SMALL_DEC(c, n, pbytes)) return decode_host_small(c, data, offsets, n, values, elems, elem_cap, arena, totals);
    GROW(c->d_in, c->c_in, pbytes + 16);
    GROW(c->d_off, c->c_off, (n + 1) * sizeof(uint64_t));
    GROW(c->d_vals, c->c_vals, (n ? n : 1) * sizeof(rr_value));
    GROW(c->d_elems, c->c_elems, (elem_cap ? elem_cap : 1) * sizeof(rr_elem));
    GROW(c->d_arena, c->c_arena, pbytes + 16);
    /* chunked when the batch is big enough.  While the descriptors fit elem_cap a chunk's
     * capacity check is the whole batch's; a batch that overflows it (the pipelined pass
     * returns 1) is decoded again in one call, so capacity statuses match it exactly. */
    if (bytes > RR_HOST_CHUNK) {
        uint64_t cut[RR_HOST_MAXCHUNK + 1];
        const int K = plan_chunks(offsets, n, bytes, cut);
        if (K > 1) {
            const int rc = decode_host_pipelined(c, data, offsets, n, values, elems, elem_cap, arena, totals, bytes,
                                                 pbytes, cut, K);
            if (rc != 1) return rc;
        }
    }
    HIPCHK(hipMemsetAsync(c->d_in, 0, pbytes + 16, c->stream));
    if (bytes) HIPCHK(hipMemcpyAsync(c->d_in, data, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_off, offsets, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->d_arena, 0, pbytes ? pbytes : 16, c->stream));
    rr_blob_batch in = {(uint8_t *)c->d_in, (uint64_t *)c->d_off, n, pbytes};
    rr_flat_batch out = {(rr_value *)c->d_vals, (rr_elem *)c->d_elems, (uint8_t *)c->d_arena, n, elem_cap, pbytes};
    int rc = rr_decode_batch(c, &in, &out, c->d_totals, c->stream);
    if (rc) return rc;
    rr_totals t;
    HIPCHK(hipMemcpyAsync(&t, c->d_totals, sizeof t, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (t.bytes == ~0ull) return fail(RR_API_EDEVICE, "decode: device-side failure (look-back timeout)");
    if (n) HIPCHK(hipMemcpyAsync(values, c->d_vals, n * sizeof(rr_value), hipMemcpyDeviceToHost, c->stream));
    uint64_t ne = t.n_elems < elem_cap ? t.n_elems : elem_cap;
    if (ne && elems) HIPCHK(hipMemcpyAsync(elems, c->d_elems, ne * sizeof(rr_elem), hipMemcpyDeviceToHost, c->stream));
    if (bytes && arena) HIPCHK(hipMemcpyAsync(arena, c->d_arena, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (n == 0) memset(&t, 0, sizeof t);
    if (totals) *totals = t;
    return RR_API_OK;
}

static int encode_host_small(rr_ctx *c, const rr_value *values, const rr_elem *elems, uint64_t n_elems,
                             const uint8_t *arena, uint64_t arena_bytes, uint64_t n, uint8_t *data, uint64_t data_cap,
                             uint64_t *offsets, rr_totals *totals) {
    const size_t o_val = 0, o_el = AL16(n * sizeof(rr_value)), o_ar = o_el + AL16(n_elems * sizeof(rr_elem)),
                 o_off = o_ar + AL16(arena_bytes), o_tot = o_off + AL16((n + 1) * sizeof(uint64_t)),
                 o_flag = o_tot + 32, o_out = o_flag + 16, end = o_out + AL16(data_cap) + 16;
    int rc = small_grow(c, end);
    if (rc) return rc;
    uint8_t *h = c->h_small, *d = c->d_small;
    memcpy(h + o_val, values, n * sizeof(rr_value));
    if (n_elems) memcpy(h + o_el, elems, n_elems * sizeof(rr_elem));
    if (arena_bytes) memcpy(h + o_ar, arena, arena_bytes);
    uint32_t seq = ++c->small_seq;
    if (!seq) seq = ++c->small_seq;   /* (0 is the cleared word) */
    __atomic_store_n((uint32_t *)(h + o_flag), 0u, __ATOMIC_RELAXED);
    HIPCHK(rr_launch_encode_small((const rr_value *)(d + o_val), (const rr_elem *)(d + o_el), n_elems, d + o_ar,
                                  arena_bytes, n, d + o_out, data_cap, (uint64_t *)(d + o_off),
                                  (rr_totals *)(d + o_tot), (uint32_t *)(d + o_flag), seq, c->sstream));
    rc = small_wait(c, (const uint32_t *)(h + o_flag), seq);
    if (rc) return rc;
    rr_totals t;
    memcpy(&t, h + o_tot, sizeof t);
    memcpy(offsets, h + o_off, (n + 1) * sizeof(uint64_t));
    const uint64_t nb = t.bytes < data_cap ? t.bytes : data_cap;
    if (nb) memcpy(data, h + o_out, nb);
    if (totals) *totals = t;
    return RR_API_OK;
}

/* ---- pipelined host encode -------------------------------------------------------------
 * A batch whose records + descriptors + arena pass RR_HOST_CHUNK goes in chunks of whole values
 * (balanced by descriptors; at most RR_HOST_MAXCHUNK).  Everything goes up on the `up` stream,
 * queued at once: the records, then per chunk the descriptors its values reach (from their
 * records: a growing prefix) and one slice of the arena.  Chunk k's encode runs on the context
 * stream once its descriptors are in and the arena prefix its payloads reach (arena_need_kernel,
 * on the `aux` stream as soon as those descriptors land) has been uploaded; it writes its blobs
 * into its own 16-byte aligned region of the output staging, its offsets are rebased past the
 * earlier chunks' bytes on the device, and its blobs and offsets go down on the `down` stream
 * while later chunks are still going up.  Every chunk's encode is the whole call's restricted to
 * its values (full descriptor and arena capacities, the output capacity left after the earlier
 * chunks): results are identical to one call. */
#define RR_NEED_MAXK RR_HOST_MAXCHUNK
static int encode_host_pipelined_run(rr_ctx *c, const rr_value *values, const rr_elem *elems, uint64_t n_elems,
                                     const uint8_t *arena, uint64_t arena_bytes, uint64_t n, uint8_t *data,
                                     uint64_t data_cap, uint64_t *offsets, rr_totals *totals, const uint64_t *cut,
                                     const uint64_t *eneed, int K) {
    rr_value *d_vals = (rr_value *)c->d_vals;
    rr_elem *d_elems = (rr_elem *)c->d_elems;
    uint8_t *d_arena = (uint8_t *)c->d_arena, *d_out = (uint8_t *)c->d_out;
    uint64_t *d_ooff = (uint64_t *)c->d_ooff;
    /* the previous host call on this context is done with the staging buffers */
    HIPCHK(hipEventRecord(c->ev_dec[0], c->stream));
    HIPCHK(hipStreamWaitEvent(c->up, c->ev_dec[0], 0));
    if (n) HIPCHK(hipMemcpyAsync(d_vals, values, n * sizeof(rr_value), hipMemcpyHostToDevice, c->up));
    uint64_t e_done = 0;
    for (int k = 0; k < K; k++) {
        if (eneed[k] > e_done) {
            HIPCHK(hipMemcpyAsync(d_elems + e_done, elems + e_done, (eneed[k] - e_done) * sizeof(rr_elem),
                                  hipMemcpyHostToDevice, c->up));
            e_done = eneed[k];
        }
        HIPCHK(hipEventRecord(c->ev_up[k], c->up));
        const uint64_t a0 = arena_bytes * (uint64_t)k / K, a1 = arena_bytes * (uint64_t)(k + 1) / K;
        if (a1 > a0) HIPCHK(hipMemcpyAsync(d_arena + a0, arena + a0, a1 - a0, hipMemcpyHostToDevice, c->up));
        HIPCHK(hipEventRecord(c->ev_arena[k], c->up));
        /* which arena bytes the chunk reads: as soon as its descriptors are in */
        HIPCHK(hipStreamWaitEvent(c->aux, c->ev_up[k], 0));
        HIPCHK(rr_launch_arena_need(d_vals + cut[k], cut[k + 1] - cut[k], d_elems, n_elems, arena_bytes,
                                    (uint64_t *)c->h_need + (size_t)k * RR_NEED_BLOCKS, c->aux));
        HIPCHK(hipEventRecord(c->ev_need[k], c->aux));
    }
    rr_totals sum = {0, 0, 0, 0};
    uint64_t base = 0, region = 0;   /* output bytes of the earlier chunks; their staging space */
    for (int k = 0; k < K; k++) {
        const uint64_t v0 = cut[k], nk = cut[k + 1] - v0;
        HIPCHK(hipEventSynchronize(c->ev_need[k]));
        uint64_t need = 0;
        for (int b = 0; b < RR_NEED_BLOCKS; b++) {
            const uint64_t x = c->h_need[(size_t)k * RR_NEED_BLOCKS + b];
            need = x > need ? x : need;
        }
        int j = -1;   /* the last arena slice the chunk reads */
        for (int s = 0; s < K && need; s++)
            if (arena_bytes * (uint64_t)s / K < need) j = s;
        HIPCHK(hipStreamWaitEvent(c->stream, c->ev_up[k], 0));
        if (j >= 0) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_arena[j], 0));
        const uint64_t cap = data_cap > base ? data_cap - base : 0;
        rr_flat_batch in = {d_vals + v0, d_elems, d_arena, nk, n_elems, arena_bytes};
        rr_blob_batch out = {d_out + region, d_ooff + v0, nk, cap};
        int rc = rr_encode_batch(c, &in, &out, c->d_ktot + k, c->stream);
        if (rc) return rc;
        HIPCHK(rr_launch_offsets_rebase(d_ooff + v0, nk + 1, 0ull - base, c->stream));
        HIPCHK(hipMemcpyAsync(&c->h_ktot[k], c->d_ktot + k, sizeof(rr_totals), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipEventRecord(c->ev_enc[k], c->stream));
        HIPCHK(hipEventSynchronize(c->ev_enc[k]));   /* (later chunks keep going up meanwhile) */
        const rr_totals t = c->h_ktot[k];
        if (t.bytes == ~0ull) return fail(RR_API_EDEVICE, "encode: device-side failure (look-back timeout)");
        HIPCHK(hipStreamWaitEvent(c->down, c->ev_enc[k], 0));
        HIPCHK(hipMemcpyAsync(offsets + v0, d_ooff + v0, (nk + (k == K - 1)) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                              c->down));
        const uint64_t nb = t.bytes < cap ? t.bytes : cap;
        if (nb) HIPCHK(hipMemcpyAsync(data + base, d_out + region, nb, hipMemcpyDeviceToHost, c->down));
        base += t.bytes;
        region += (nb + 15) & ~15ull;
        sum.n_elems += t.n_elems;
        sum.n_bad += t.n_bad;
        sum.payload += t.payload;
    }
    HIPCHK(hipStreamSynchronize(c->down));
    sum.bytes = base;
    if (totals) *totals = sum;
    return RR_API_OK;
}

/* Cuts by descriptors (the encode's work) and, per chunk, the descriptor prefix its values
 * reach (the valid ones: status RR_OK, descriptors inside n_elems — what the encode reads).  The
 * staging output needs room for every chunk's 16-byte aligned region. */
static int encode_host_pipelined(rr_ctx *c, const rr_value *values, const rr_elem *elems, uint64_t n_elems,
                                 const uint8_t *arena, uint64_t arena_bytes, uint64_t n, uint8_t *data,
                                 uint64_t data_cap, uint64_t *offsets, rr_totals *totals) {
    int rc = pipe_init(c);
    if (rc) return rc;
    uint64_t cut[RR_HOST_MAXCHUNK + 1], eneed[RR_HOST_MAXCHUNK];
    const uint64_t in_bytes = n * sizeof(rr_value) + n_elems * sizeof(rr_elem) + arena_bytes;
    uint64_t K = (in_bytes + RR_HOST_CHUNK - 1) / RR_HOST_CHUNK;
    if (K > RR_HOST_MAXCHUNK) K = RR_HOST_MAXCHUNK;
    if (K > n) K = n;
    uint64_t tot = 0;
    for (uint64_t v = 0; v < n; v++) tot += values[v].n_elems + 1;   /* (+1: every value costs) */
    int m = 0;
    uint64_t acc = 0, emax = 0;
    cut[0] = 0;
    for (uint64_t v = 0; v < n; v++) {
        const uint64_t eb = values[v].elem_base, ne = values[v].n_elems;
        if (values[v].status == RR_OK && eb + ne <= n_elems && eb + ne > emax) emax = eb + ne;
        acc += ne + 1;
        if (m + 1 < (int)K && acc >= tot / K * (uint64_t)(m + 1) && v + 1 < n) {
            eneed[m] = emax;
            cut[++m] = v + 1;
        }
    }
    eneed[m] = emax;
    cut[++m] = n;
    GROW(c->d_out, c->c_out, data_cap + 16 * (size_t)m + 16);
    rc = encode_host_pipelined_run(c, values, elems, n_elems, arena, arena_bytes, n, data, data_cap, offsets, totals,
                                   cut, eneed, m);
    if (rc != RR_API_OK) {   /* transfers in flight must not outlive the call */
        c->dsums_dirty = 1;   /* a chunk's kernels may not all have run */
        (void)hipStreamSynchronize(c->up);
        (void)hipStreamSynchronize(c->aux);
        (void)hipStreamSynchronize(c->down);
        (void)hipStreamSynchronize(c->stream);
    }
    return rc;
}

int rr_encode_batch_host(rr_ctx *c, const rr_value *values, const rr_elem *elems, uint64_t n_elems,
                         const uint8_t *arena, uint64_t arena_bytes, uint64_t n, uint8_t *data, uint64_t data_cap,
                         uint64_t *offsets, rr_totals *totals) {
    if (!c || !offsets || (n && (!values || !data))) return fail(RR_API_EINVAL, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    if (SMALL_ENC(c, n, data_cap))
        return encode_host_small(c, values, elems, n_elems, arena, arena_bytes, n, data, data_cap, offsets, totals);
    GROW(c->d_vals, c->c_vals, (n ? n : 1) * sizeof(rr_value));
    GROW(c->d_elems, c->c_elems, (n_elems ? n_elems : 1) * sizeof(rr_elem));
    GROW(c->d_arena, c->c_arena, arena_bytes + 16);
    GROW(c->d_out, c->c_out, data_cap + 16);
    GROW(c->d_ooff, c->c_ooff, (n + 1) * sizeof(uint64_t));
    if (n > 1 && n * sizeof(rr_value) + n_elems * sizeof(rr_elem) + arena_bytes > RR_HOST_CHUNK)
        return encode_host_pipelined(c, values, elems, n_elems, arena, arena_bytes, n, data, data_cap, offsets, totals);
    if (n) HIPCHK(hipMemcpyAsync(c->d_vals, values, n * sizeof(rr_value), hipMemcpyHostToDevice, c->stream));
    if (n_elems) HIPCHK(hipMemcpyAsync(c->d_elems, elems, n_elems * sizeof(rr_elem), hipMemcpyHostToDevice, c->stream));
    if (arena_bytes) HIPCHK(hipMemcpyAsync(c->d_arena, arena, arena_bytes, hipMemcpyHostToDevice, c->stream));
    rr_flat_batch in = {(rr_value *)c->d_vals, (rr_elem *)c->d_elems, (uint8_t *)c->d_arena, n, n_elems, arena_bytes};
    rr_blob_batch out = {(uint8_t *)c->d_out, (uint64_t *)c->d_ooff, n, data_cap};
    int rc = rr_encode_batch(c, &in, &out, c->d_totals, c->stream);
    if (rc) return rc;
    rr_totals t;
    HIPCHK(hipMemcpyAsync(&t, c->d_totals, sizeof t, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(offsets, c->d_ooff, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (t.bytes == ~0ull) return fail(RR_API_EDEVICE, "encode: device-side failure (look-back timeout)");
    uint64_t nb = t.bytes < data_cap ? t.bytes : data_cap;
    if (nb) HIPCHK(hipMemcpyAsync(data, c->d_out, nb, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (n == 0) memset(&t, 0, sizeof t);
    if (totals) *totals = t;
    return RR_API_OK;
}
