/*
 * rr_shard.c — multi-GPU sharding in the C host layer (include/rr_serdes.h "multi-GPU",
 * SURVEY.md §8e): the byte-balanced plan, and the root split / gather of device-resident
 * batches with RCCL point-to-point transfers over xGMI.  One process per GPU, one rr_comm per
 * process.  Nothing here touches the decode: values are independent, so each rank decodes its
 * shard with rr_decode_batch and only the split and the gather move data between GPUs.
 */
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

#include "rr_internal.h"

struct rr_comm {
    ncclComm_t nc;
    int nranks, rank, device;
    uint64_t *d_words;   /* 4 * nranks words: the plan / the all-gathered shard sizes */
};

#define NCCLCHK(x) do { ncclResult_t r_ = (x); if (r_ != ncclSuccess) \
    return rr_fail(RR_API_EHIP, "%s:%d %s: %s", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); } while (0)

/* the same rule as shard_plan_kernel: shard k starts at the first value whose first byte is at
 * or after floor(total * k / g) */
int rr_shard_plan(const uint64_t *offsets, uint64_t n, uint32_t g, rr_shard *plan) {
    if (!offsets || !plan || g == 0) return rr_fail(RR_API_EINVAL, "rr_shard_plan: bad argument");
    const uint64_t total = offsets[n];
    uint64_t prev = 0;
    for (uint32_t k = 0; k < g; k++) {
        uint64_t cut = n;
        if (k + 1 < g) {
            const uint64_t target = (uint64_t)(((unsigned __int128)total * (k + 1)) / g);
            uint64_t lo = 0, hi = n;
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                if (offsets[mid] < target) lo = mid + 1;
                else hi = mid;
            }
            cut = lo;
        }
        plan[k].v0 = prev;
        plan[k].v1 = cut;
        plan[k].b0 = offsets[prev];
        plan[k].b1 = offsets[cut];
        prev = cut;
    }
    return RR_API_OK;
}

/* elem_base is 32-bit (rr_format.h): a shard placed past 2^32 - 1 descriptors cannot be
 * represented, so an elem_add that large is refused instead of wrapping in the kernel */
int rr_flat_rebase(rr_ctx *ctx, rr_value *values, uint64_t n, rr_elem *elems, uint64_t n_elems, uint64_t elem_add,
                   uint64_t byte_add, void *stream) {
    if (!ctx) return rr_fail(RR_API_EINVAL, "ctx is NULL");
    if (elem_add > 0xFFFFFFFFull || n_elems > 0xFFFFFFFFull - elem_add)
        return rr_fail(RR_API_EINVAL, "rr_flat_rebase: descriptors past 2^32 - 1 (elem_base is 32-bit)");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(rr_launch_flat_rebase(values, n, elems, n_elems, elem_add, byte_add, (hipStream_t)stream));
    return RR_API_OK;
}

/* Host forms of the placement rr_gather makes on the device (flat_rebase_kernel's rule), for a
 * caller that gathers decoded shards in host memory: values' elem_base += elem_add, STR /
 * ZLRAW arena offsets += byte_add, zero-filled slots of malformed values left zero. */
int rr_flat_rebase_host(rr_value *values, uint64_t n, rr_elem *elems, uint64_t n_elems, uint64_t elem_add,
                        uint64_t byte_add) {
    if ((n && !values) || (n_elems && !elems)) return rr_fail(RR_API_EINVAL, "rr_flat_rebase_host: NULL buffer");
    if (elem_add > 0xFFFFFFFFull || n_elems > 0xFFFFFFFFull - elem_add)
        return rr_fail(RR_API_EINVAL, "rr_flat_rebase_host: descriptors past 2^32 - 1 (elem_base is 32-bit)");
    for (uint64_t i = 0; i < n; i++) values[i].elem_base += (uint32_t)elem_add;
    for (uint64_t i = 0; i < n_elems; i++) {
        rr_elem *e = &elems[i];
        if ((e->kind == RR_K_STR || e->kind == RR_K_ZLRAW) && (e->data | e->len) != 0) e->data += byte_add;
    }
    return RR_API_OK;
}

/* Where the gather puts shard k: its records at values + plan[k].v0 (the plan's value range),
 * its descriptors at elems + elem_at[k] = the descriptors of the shards before it, which is
 * also the elem_add its rebase applies.  Returns the total, or UINT64_MAX past 2^32 - 1. */
uint64_t rr_gather_layout(const uint64_t *shard_elems, int nranks, uint64_t *elem_at) {
    uint64_t e = 0;
    for (int k = 0; k < nranks; k++) {
        if (elem_at) elem_at[k] = e;
        e += shard_elems[k];
        if (e > 0xFFFFFFFFull) return UINT64_MAX;
    }
    return e;
}

/* ---- the transfer schedules (rr_serdes.h): the pairing rr_split / rr_gather post ---------- */
static int xfer(rr_xfer *out, int m, int peer, int dir, int buf, uint64_t offset, uint64_t bytes) {
    if (bytes == 0) return m;   /* (both sides skip it: both know the plan) */
    out[m].peer = peer;
    out[m].dir = dir;
    out[m].buf = buf;
    out[m].rsv = 0;
    out[m].offset = offset;
    out[m].bytes = bytes;
    return m + 1;
}

int rr_split_schedule(const rr_shard *plan, int nranks, int rank, int root, rr_xfer *out) {
    if (!plan || !out || nranks < 1 || rank < 0 || rank >= nranks || root < 0 || root >= nranks) return -1;
    int m = 0;
    if (rank == root) {
        for (int k = 0; k < nranks; k++) {
            if (k == root) continue;
            const rr_shard *p = &plan[k];
            m = xfer(out, m, k, RR_XFER_SEND, RR_BUF_WHOLE_DATA, p->b0, p->b1 - p->b0);
            m = xfer(out, m, k, RR_XFER_SEND, RR_BUF_WHOLE_OFFSETS, p->v0 * sizeof(uint64_t),
                     (p->v1 - p->v0 + 1) * sizeof(uint64_t));
        }
    } else {
        const rr_shard *p = &plan[rank];
        m = xfer(out, m, root, RR_XFER_RECV, RR_BUF_MINE_DATA, 0, p->b1 - p->b0);
        m = xfer(out, m, root, RR_XFER_RECV, RR_BUF_MINE_OFFSETS, 0, (p->v1 - p->v0 + 1) * sizeof(uint64_t));
    }
    return m;
}

int rr_gather_schedule(const rr_shard *plan, const uint64_t *shard_elems, int nranks, int rank, int root,
                       rr_xfer *out) {
    if (!plan || !shard_elems || !out || nranks < 1 || rank < 0 || rank >= nranks || root < 0 || root >= nranks)
        return -1;
    int m = 0;
    if (rank == root) {
        uint64_t at = 0;   /* rr_gather_layout's placement, shard by shard */
        for (int k = 0; k < nranks; k++) {
            const uint64_t nv = plan[k].v1 - plan[k].v0;
            if (k != root) {
                m = xfer(out, m, k, RR_XFER_RECV, RR_BUF_WHOLE_VALUES, plan[k].v0 * sizeof(rr_value), nv * sizeof(rr_value));
                m = xfer(out, m, k, RR_XFER_RECV, RR_BUF_WHOLE_ELEMS, at * sizeof(rr_elem), shard_elems[k] * sizeof(rr_elem));
            }
            at += shard_elems[k];
            if (at > 0xFFFFFFFFull) return -1;   /* elem_base is 32-bit */
        }
    } else {
        const uint64_t nv = plan[rank].v1 - plan[rank].v0;
        m = xfer(out, m, root, RR_XFER_SEND, RR_BUF_MINE_VALUES, 0, nv * sizeof(rr_value));
        m = xfer(out, m, root, RR_XFER_SEND, RR_BUF_MINE_ELEMS, 0, shard_elems[rank] * sizeof(rr_elem));
    }
    return m;
}

/* post a schedule inside one ncclGroup (the group is always closed, whatever a call inside it
 * returns); bufs[] = the device base of each RR_BUF_* */
static ncclResult_t post_schedule(rr_comm *c, const rr_xfer *x, int m, uint8_t *const *bufs, hipStream_t s) {
    ncclResult_t r = ncclGroupStart();
    for (int i = 0; i < m && r == ncclSuccess; i++) {
        uint8_t *p = bufs[x[i].buf] + x[i].offset;
        r = x[i].dir == RR_XFER_SEND ? ncclSend(p, x[i].bytes, ncclUint8, x[i].peer, c->nc, s)
                                     : ncclRecv(p, x[i].bytes, ncclUint8, x[i].peer, c->nc, s);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    return r == ncclSuccess ? r2 : r;
}

int rr_comm_get_id(uint8_t id[RR_COMM_ID_BYTES]) {
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    memcpy(id, &u, RR_COMM_ID_BYTES);
    return RR_API_OK;
}

int rr_comm_init(rr_ctx *ctx, int nranks, int rank, const uint8_t id[RR_COMM_ID_BYTES], rr_comm **out) {
    if (!ctx || !out || nranks < 1 || rank < 0 || rank >= nranks) return rr_fail(RR_API_EINVAL, "rr_comm_init: bad argument");
    *out = NULL;
    HIPCHK(hipSetDevice(ctx->device));
    rr_comm *c = (rr_comm *)calloc(1, sizeof *c);
    if (!c) return rr_fail(RR_API_ENOMEM, "calloc");
    ncclUniqueId u;
    memcpy(&u, id, RR_COMM_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&c->nc, nranks, u, rank);
    if (r != ncclSuccess) { free(c); return rr_fail(RR_API_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r)); }
    if (hipMalloc((void **)&c->d_words, sizeof(uint64_t) * 4 * (size_t)nranks) != hipSuccess) {
        ncclCommDestroy(c->nc);
        free(c);
        return rr_fail(RR_API_ENOMEM, "hipMalloc comm words");
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = ctx->device;
    *out = c;
    return RR_API_OK;
}

void rr_comm_destroy(rr_comm *c) {
    if (!c) return;
    hipSetDevice(c->device);
    ncclCommDestroy(c->nc);
    hipFree(c->d_words);
    free(c);
}

int rr_split_plan(rr_comm *c, const rr_blob_batch *whole, int root, rr_shard *plan, void *stream) {
    if (!c || !plan || root < 0 || root >= c->nranks) return rr_fail(RR_API_EINVAL, "rr_split_plan: bad argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(c->device));
    if (c->rank == root) {
        if (!whole || !whole->offsets) return rr_fail(RR_API_EINVAL, "rr_split_plan: root needs the whole batch");
        HIPCHK(rr_launch_shard_plan(whole->offsets, whole->n, (uint32_t)c->nranks, c->d_words, s));
    }
    NCCLCHK(ncclBroadcast(c->d_words, c->d_words, 4 * (size_t)c->nranks, ncclUint64, root, c->nc, s));
    HIPCHK(hipMemcpyAsync(plan, c->d_words, sizeof(rr_shard) * (size_t)c->nranks, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return RR_API_OK;
}

/* Every rank's verdict on its own arguments, agreed before any point-to-point call: a rank
 * that returned early would leave its peers' sends / receives waiting forever on their
 * streams.  bad = this rank's local verdict; returns whether ANY rank is bad (or a transport
 * error: RR_API_EHIP).  An all-reduce (max) of one word, then a host sync. */
static int agree(rr_comm *c, int bad, hipStream_t s, int *any_bad) {
    uint64_t w = bad ? 1 : 0;
    HIPCHK(hipMemcpyAsync(c->d_words, &w, sizeof w, hipMemcpyHostToDevice, s));
    NCCLCHK(ncclAllReduce(c->d_words, c->d_words, 1, ncclUint64, ncclMax, c->nc, s));
    HIPCHK(hipMemcpyAsync(&w, c->d_words, sizeof w, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *any_bad = w != 0;
    return RR_API_OK;
}

int rr_split(rr_comm *c, const rr_blob_batch *whole, const rr_shard *plan, int root, rr_blob_batch *mine,
             void *stream) {
    /* (arguments every rank shares: a bad one fails on every rank alike, before any collective) */
    if (!c || !plan || root < 0 || root >= c->nranks) return rr_fail(RR_API_EINVAL, "rr_split: bad argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(c->device));
    const rr_shard *me = &plan[c->rank];
    const uint64_t nb = me->b1 - me->b0, nv = me->v1 - me->v0;
    int bad = 0;
    if (!mine || mine->data_cap < ((nb + 15) & ~15ull) || !mine->offsets || (nb && !mine->data))
        bad = rr_fail(RR_API_EINVAL, "rr_split: shard buffers too small");
    else if (c->rank == root && (!whole || !whole->data || !whole->offsets))
        bad = rr_fail(RR_API_EINVAL, "rr_split: root needs the whole batch");
    else if (c->rank == root && mine->offsets == whole->offsets + me->v0 && me->b0 != 0)
        bad = rr_fail(RR_API_EINVAL, "rr_split: in-place offsets need the root's shard to start at byte 0");
    int any_bad = 0;
    int rc = agree(c, bad, s, &any_bad);
    if (rc) return rc;
    if (bad) return bad;
    if (any_bad) return rr_fail(RR_API_EINVAL, "rr_split: another rank's arguments are invalid");
    rr_xfer *x = (rr_xfer *)malloc(sizeof(rr_xfer) * 2 * (size_t)c->nranks);
    if (!x) return rr_fail(RR_API_ENOMEM, "malloc");
    const int m = rr_split_schedule(plan, c->nranks, c->rank, root, x);
    uint8_t *bufs[8] = {0};
    if (c->rank == root) {
        bufs[RR_BUF_WHOLE_DATA] = (uint8_t *)whole->data;
        bufs[RR_BUF_WHOLE_OFFSETS] = (uint8_t *)whole->offsets;
    }
    bufs[RR_BUF_MINE_DATA] = mine->data;
    bufs[RR_BUF_MINE_OFFSETS] = (uint8_t *)mine->offsets;
    const ncclResult_t r = m < 0 ? ncclInvalidArgument : post_schedule(c, x, m, bufs, s);
    free(x);
    if (r != ncclSuccess) return rr_fail(RR_API_EHIP, "rr_split: %s", ncclGetErrorString(r));
    if (c->rank == root) {   /* the root's own shard: a device copy (nothing if it decodes in place) */
        if (mine->data != whole->data + me->b0 && nb)
            HIPCHK(hipMemcpyAsync(mine->data, whole->data + me->b0, nb, hipMemcpyDeviceToDevice, s));
        if (mine->offsets != whole->offsets + me->v0)
            HIPCHK(hipMemcpyAsync(mine->offsets, whole->offsets + me->v0, (nv + 1) * sizeof(uint64_t),
                                  hipMemcpyDeviceToDevice, s));
    }
    const int in_place = c->rank == root && mine->data == whole->data + me->b0;
    if (nb < mine->data_cap && !in_place)   /* the shard's tail padding reads as zeros */
        HIPCHK(hipMemsetAsync(mine->data + nb, 0, mine->data_cap - nb, s));
    HIPCHK(rr_launch_offsets_rebase(mine->offsets, nv + 1, me->b0, s));
    mine->n = nv;
    return RR_API_OK;
}

int rr_gather(rr_comm *c, const rr_flat_batch *mine, uint64_t mine_elems, const rr_shard *plan, int root,
              rr_flat_batch *whole, void *stream) {
    if (!c || !plan || root < 0 || root >= c->nranks) return rr_fail(RR_API_EINVAL, "rr_gather: bad argument");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipSetDevice(c->device));
    const int R = c->nranks;
    const uint64_t my_nv = plan[c->rank].v1 - plan[c->rank].v0;
    int bad = 0;
    if (!mine || (my_nv && !mine->values) || (mine_elems && !mine->elems))
        bad = rr_fail(RR_API_EINVAL, "rr_gather: NULL shard buffer");
    /* every rank's {descriptor count, verdict} (the root places the shards with the counts) */
    uint64_t w2[2] = {mine_elems, bad ? 1u : 0u};
    HIPCHK(hipMemcpyAsync(c->d_words + 2 * c->rank, w2, sizeof w2, hipMemcpyHostToDevice, s));
    NCCLCHK(ncclAllGather(c->d_words + 2 * c->rank, c->d_words, 2, ncclUint64, c->nc, s));
    uint64_t *got = (uint64_t *)malloc(sizeof(uint64_t) * 4 * (size_t)R);
    if (!got) return rr_fail(RR_API_ENOMEM, "malloc");
    uint64_t *cnt = got + 2 * R, *at = got + 3 * R;   /* descriptor counts, shard placements */
    hipError_t he = hipMemcpyAsync(got, c->d_words, sizeof(uint64_t) * 2 * (size_t)R, hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    if (he != hipSuccess) { free(got); return rr_fail(RR_API_EHIP, "rr_gather sizes: %s", hipGetErrorString(he)); }
    int any_bad = 0;
    for (int k = 0; k < R; k++) { cnt[k] = got[2 * k]; any_bad |= got[2 * k + 1] != 0; }
    /* the root's verdict on the whole batch needs the counts: one more agreement round */
    int rbad = 0;
    if (c->rank == root && !any_bad) {
        const uint64_t tot = rr_gather_layout(cnt, R, NULL);
        if (tot == UINT64_MAX) rbad = rr_fail(RR_API_EINVAL, "rr_gather: descriptors past 2^32 - 1 (elem_base is 32-bit)");
        else if (!whole || (plan[R - 1].v1 && !whole->values) || (tot && !whole->elems) || whole->elem_cap < tot ||
                 whole->n < plan[R - 1].v1)
            rbad = rr_fail(RR_API_EINVAL, "rr_gather: root's whole batch too small");
    }
    int root_bad = 0;
    int rc = any_bad ? RR_API_OK : agree(c, rbad, s, &root_bad);
    if (rc == RR_API_OK && (any_bad || root_bad))
        rc = bad ? bad : rbad ? rbad : rr_fail(RR_API_EINVAL, "rr_gather: another rank's arguments are invalid");
    if (rc == RR_API_OK) rr_gather_layout(cnt, R, at);
    if (rc == RR_API_OK) {
        rr_xfer *x = (rr_xfer *)malloc(sizeof(rr_xfer) * 2 * (size_t)R);
        const int m = x ? rr_gather_schedule(plan, cnt, R, c->rank, root, x) : -1;
        uint8_t *bufs[8] = {0};
        bufs[RR_BUF_MINE_VALUES] = (uint8_t *)mine->values;
        bufs[RR_BUF_MINE_ELEMS] = (uint8_t *)mine->elems;
        if (c->rank == root) {
            bufs[RR_BUF_WHOLE_VALUES] = (uint8_t *)whole->values;
            bufs[RR_BUF_WHOLE_ELEMS] = (uint8_t *)whole->elems;
        }
        const ncclResult_t r = m < 0 ? ncclInvalidArgument : post_schedule(c, x, m, bufs, s);
        free(x);
        if (r != ncclSuccess) rc = rr_fail(RR_API_EHIP, "rr_gather: %s", ncclGetErrorString(r));
    }
    if (rc == RR_API_OK && c->rank == root) {
        for (int k = 0; k < R && rc == RR_API_OK; k++) {
            const uint64_t nv = plan[k].v1 - plan[k].v0;
            rr_value *dv = whole->values + plan[k].v0;
            rr_elem *de = whole->elems + at[k];
            if (k == root) {   /* the root's own shard: copy it in, unless it decoded in place */
                hipError_t e2 = hipSuccess;
                if (nv && (void *)mine->values != (void *)dv)
                    e2 = hipMemcpyAsync(dv, mine->values, nv * sizeof(rr_value), hipMemcpyDeviceToDevice, s);
                if (e2 == hipSuccess && cnt[k] && (void *)mine->elems != (void *)de)
                    e2 = hipMemcpyAsync(de, mine->elems, cnt[k] * sizeof(rr_elem), hipMemcpyDeviceToDevice, s);
                if (e2 != hipSuccess) rc = rr_fail(RR_API_EHIP, "rr_gather copy: %s", hipGetErrorString(e2));
            }
            if (rc == RR_API_OK) {
                hipError_t e3 = rr_launch_flat_rebase(dv, nv, de, cnt[k], at[k], plan[k].b0, s);
                if (e3 != hipSuccess) rc = rr_fail(RR_API_EHIP, "rr_gather rebase: %s", hipGetErrorString(e3));
            }
        }
    }
    free(got);
    return rc;
}
