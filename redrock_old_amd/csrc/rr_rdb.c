/*
 * rr_rdb.c — batched snapshot restore over RedRock's fork-child pipes (include/rr_rdb.h;
 * SURVEY.md §8f row f4).  The wire format of a RAW request / response is the reference's
 * (rock_rdb.c:126-267): {int dbi, size_t key_len, key} / {size_t val_len, val}.
 */
#include <errno.h>
#include <fcntl.h>
#include <poll.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "rr_internal.h"
#include "../../include/rr_rdb.h"

#define fail rr_fail

/* read / write exactly len bytes on a blocking fd: 1 done, 0 closed, -1 error
 * (the reference's _read_pipe_by_length / _write_pipe_by_length, rock_rdb.c:64-103) */
static int read_full(int fd, void *buf, size_t len) {
    char *p = (char *)buf;
    while (len) {
        ssize_t r = read(fd, p, len);
        if (r == 0) return 0;
        if (r < 0) { if (errno == EINTR) continue; return -1; }
        p += r;
        len -= (size_t)r;
    }
    return 1;
}
static int write_full(int fd, const void *buf, size_t len) {
    const char *p = (const char *)buf;
    while (len) {
        ssize_t r = write(fd, p, len);
        if (r < 0) { if (errno == EINTR) continue; return -1; }
        p += r;
        len -= (size_t)r;
    }
    return 1;
}

static uint8_t *pack_requests(const int *dbis, const char *const *keys, const size_t *key_lens, size_t k,
                              size_t *out_len, int tag) {
    size_t len = tag ? sizeof(int) + sizeof(size_t) : 0;
    for (size_t i = 0; i < k; i++) len += sizeof(int) + sizeof(size_t) + key_lens[i];
    uint8_t *b = (uint8_t *)malloc(len ? len : 1), *p = b;
    if (!b) return NULL;
    if (tag) {
        const int t = RR_RDB_FLAT_TAG;
        const size_t kk = k;
        memcpy(p, &t, sizeof t); p += sizeof t;
        memcpy(p, &kk, sizeof kk); p += sizeof kk;
    }
    for (size_t i = 0; i < k; i++) {
        memcpy(p, &dbis[i], sizeof(int)); p += sizeof(int);
        memcpy(p, &key_lens[i], sizeof(size_t)); p += sizeof(size_t);
        memcpy(p, keys[i], key_lens[i]); p += key_lens[i];
    }
    *out_len = len;
    return b;
}

void rr_rdb_blobs_free(rr_rdb_blobs *b) {
    if (!b) return;
    free(b->data);
    free(b->offsets);
    memset(b, 0, sizeof *b);
}

void rr_rdb_flat_free(rr_rdb_flat *f) {
    if (!f) return;
    free(f->values);
    free(f->elems);
    free(f->arena);
    memset(f, 0, sizeof *f);
}

/* RAW: write the k requests while reading the k responses (both fds non-blocking for the call) */
int rr_rdb_request_batch(int fd_req, int fd_resp, const int *dbis, const char *const *keys, const size_t *key_lens,
                         size_t k, rr_rdb_blobs *out) {
    if (!out || (k && (!dbis || !keys || !key_lens))) return fail(RR_API_EINVAL, "rr_rdb_request_batch: NULL argument");
    memset(out, 0, sizeof *out);
    size_t wlen = 0, wpos = 0;
    uint8_t *req = pack_requests(dbis, keys, key_lens, k, &wlen, 0);
    uint64_t *offs = (uint64_t *)calloc(k + 1, sizeof(uint64_t));
    size_t cap = 4096, used = 0;
    uint8_t *data = (uint8_t *)malloc(cap);
    if (!req || !offs || !data) { free(req); free(offs); free(data); return fail(RR_API_ENOMEM, "malloc"); }
    const int f1 = fcntl(fd_req, F_GETFL), f2 = fcntl(fd_resp, F_GETFL);
    fcntl(fd_req, F_SETFL, f1 | O_NONBLOCK);
    fcntl(fd_resp, F_SETFL, f2 | O_NONBLOCK);
    size_t got = 0, hdr_have = 0, val_len = 0, val_have = 0;
    uint8_t hdr[sizeof(size_t)];
    int in_val = 0, rc = RR_API_OK;
    uint8_t tmp[65536];
    while (rc == RR_API_OK && (wpos < wlen || got < k)) {
        struct pollfd pf[2] = {{fd_req, POLLOUT, 0}, {fd_resp, POLLIN, 0}};
        const int nf = wpos < wlen ? 2 : 1;
        struct pollfd *ps = wpos < wlen ? pf : pf + 1;
        if (poll(ps, (nfds_t)nf, -1) < 0) {
            if (errno == EINTR) continue;
            rc = fail(RR_API_EINVAL, "poll failed");
            break;
        }
        if (wpos < wlen && (pf[0].revents & (POLLOUT | POLLERR | POLLHUP))) {
            ssize_t w = write(fd_req, req + wpos, wlen - wpos);
            if (w > 0) wpos += (size_t)w;
            else if (w < 0 && errno != EAGAIN && errno != EINTR) { rc = fail(RR_API_EINVAL, "request pipe write failed"); break; }
        }
        if (ps[nf - 1].revents & (POLLIN | POLLERR | POLLHUP)) {
            ssize_t r = read(fd_resp, tmp, sizeof tmp);
            if (r == 0) { rc = fail(RR_API_EINVAL, "pipe closed after %zu of %zu values", got, k); break; }
            if (r < 0) { if (errno == EAGAIN || errno == EINTR) continue; rc = fail(RR_API_EINVAL, "response read failed"); break; }
            size_t i = 0;
            while (i < (size_t)r && got < k) {   /* response parser: {size_t len, bytes}* */
                if (!in_val) {
                    const size_t t = sizeof hdr - hdr_have < (size_t)r - i ? sizeof hdr - hdr_have : (size_t)r - i;
                    memcpy(hdr + hdr_have, tmp + i, t);
                    hdr_have += t;
                    i += t;
                    if (hdr_have == sizeof hdr) {
                        memcpy(&val_len, hdr, sizeof val_len);
                        hdr_have = 0;
                        val_have = 0;
                        in_val = 1;
                        if (used + val_len + 16 > cap) {
                            while (used + val_len + 16 > cap) cap *= 2;
                            uint8_t *nd = (uint8_t *)realloc(data, cap);
                            if (!nd) { rc = fail(RR_API_ENOMEM, "realloc"); break; }
                            data = nd;
                        }
                    }
                }
                if (in_val) {
                    const size_t t = val_len - val_have < (size_t)r - i ? val_len - val_have : (size_t)r - i;
                    memcpy(data + used + val_have, tmp + i, t);
                    val_have += t;
                    i += t;
                    if (val_have == val_len) {
                        used += val_len;
                        offs[++got] = used;
                        in_val = 0;
                    }
                }
            }
        }
    }
    fcntl(fd_req, F_SETFL, f1);
    fcntl(fd_resp, F_SETFL, f2);
    free(req);
    if (rc != RR_API_OK) { free(offs); free(data); return rc; }
    memset(data + used, 0, ((used + 15) & ~15ull) - used);
    out->data = data;
    out->offsets = offs;
    out->n = k;
    return RR_API_OK;
}

int rr_rdb_request_flat(int fd_req, int fd_resp, const int *dbis, const char *const *keys, const size_t *key_lens,
                        size_t k, rr_rdb_flat *out) {
    if (!out || (k && (!dbis || !keys || !key_lens))) return fail(RR_API_EINVAL, "rr_rdb_request_flat: NULL argument");
    memset(out, 0, sizeof *out);
    size_t wlen = 0;
    uint8_t *req = pack_requests(dbis, keys, key_lens, k, &wlen, 1);
    if (!req) return fail(RR_API_ENOMEM, "malloc");
    const int w = write_full(fd_req, req, wlen);   /* the service reads a whole FLAT request before it answers */
    free(req);
    if (w != 1) return fail(RR_API_EINVAL, "request pipe write failed");
    uint64_t h[3];
    if (read_full(fd_resp, h, sizeof h) != 1) return fail(RR_API_EINVAL, "pipe closed (flat header)");
    out->n = h[0];
    out->n_elems = h[1];
    out->bytes = h[2];
    out->values = (rr_value *)malloc((h[0] ? h[0] : 1) * sizeof(rr_value));
    out->elems = (rr_elem *)malloc((h[1] ? h[1] : 1) * sizeof(rr_elem));
    out->arena = (uint8_t *)malloc(h[2] + 16);
    if (!out->values || !out->elems || !out->arena) { rr_rdb_flat_free(out); return fail(RR_API_ENOMEM, "malloc"); }
    if (read_full(fd_resp, out->values, h[0] * sizeof(rr_value)) != 1 ||
        read_full(fd_resp, out->elems, h[1] * sizeof(rr_elem)) != 1 || read_full(fd_resp, out->arena, h[2]) != 1) {
        rr_rdb_flat_free(out);
        return fail(RR_API_EINVAL, "pipe closed (flat body)");
    }
    return RR_API_OK;
}

/* ---- service ------------------------------------------------------------------------------ */
typedef struct {
    int *dbis;
    char **keys;
    size_t *lens;
    void **vals;
    size_t *vlens;
    size_t n, cap;
} reqs_t;

static void reqs_clear(reqs_t *r) {
    for (size_t i = 0; i < r->n; i++) free(r->keys[i]);
    r->n = 0;
}
static void reqs_free(reqs_t *r) {
    reqs_clear(r);
    free(r->dbis); free(r->keys); free(r->lens); free(r->vals); free(r->vlens);
}
static int reqs_push(reqs_t *r, int dbi, char *key, size_t len) {
    if (r->n == r->cap) {
        size_t c = r->cap ? 2 * r->cap : 64;
        int *d = realloc(r->dbis, c * sizeof(int));
        if (d) r->dbis = d;
        char **k = realloc(r->keys, c * sizeof(char *));
        if (k) r->keys = k;
        size_t *l = realloc(r->lens, c * sizeof(size_t));
        if (l) r->lens = l;
        void **v = realloc(r->vals, c * sizeof(void *));
        if (v) r->vals = v;
        size_t *vl = realloc(r->vlens, c * sizeof(size_t));
        if (vl) r->vlens = vl;
        if (!d || !k || !l || !v || !vl) return -1;
        r->cap = c;
    }
    r->dbis[r->n] = dbi;
    r->keys[r->n] = key;
    r->lens[r->n] = len;
    r->n++;
    return 0;
}
/* the rest of a request whose dbi was read: size_t key_len, key */
static int read_key(int fd, int dbi, reqs_t *r) {
    size_t len;
    if (read_full(fd, &len, sizeof len) != 1) return -1;
    char *key = (char *)malloc(len ? len : 1);
    if (!key) return -1;
    if (len && read_full(fd, key, len) != 1) { free(key); return -1; }
    if (reqs_push(r, dbi, key, len)) { free(key); return -1; }
    return 0;
}
static int lookup(reqs_t *r, rr_rdb_multiget_fn get, void *user) {
    memset(r->vals, 0, r->n * sizeof(void *));
    if (get(user, r->n, r->dbis, (const char *const *)r->keys, r->lens, r->vals, r->vlens)) return -1;
    for (size_t i = 0; i < r->n; i++)
        if (!r->vals[i]) return -1;   /* not found: the reference's goto err (rock_rdb.c:176-181) */
    return 0;
}
static void drop_vals(reqs_t *r, void (*free_val)(void *)) {
    for (size_t i = 0; i < r->n; i++)
        if (r->vals[i] && free_val) free_val(r->vals[i]);
}

static int serve_flat(int fd_req, int fd_resp, reqs_t *r, rr_rdb_multiget_fn get, void (*free_val)(void *), void *user,
                      rr_ctx *ctx) {
    size_t k;
    if (read_full(fd_req, &k, sizeof k) != 1) return -1;
    for (size_t i = 0; i < k; i++) {
        int dbi;
        if (read_full(fd_req, &dbi, sizeof dbi) != 1 || read_key(fd_req, dbi, r)) return -1;
    }
    if (!ctx || lookup(r, get, user)) { drop_vals(r, free_val); return -1; }
    uint64_t *offs = (uint64_t *)malloc((r->n + 1) * sizeof(uint64_t));
    uint64_t bytes = 0;
    if (!offs) { drop_vals(r, free_val); return -1; }
    offs[0] = 0;
    for (size_t i = 0; i < r->n; i++) offs[i + 1] = bytes += r->vlens[i];
    const uint64_t padded = (bytes + 15) & ~15ull, cap = rr_decode_elem_bound(r->n, bytes);
    uint8_t *data = (uint8_t *)calloc(padded + 16, 1), *arena = (uint8_t *)malloc(padded + 16);
    rr_value *vals = (rr_value *)malloc((r->n ? r->n : 1) * sizeof(rr_value));
    rr_elem *els = (rr_elem *)malloc((cap ? cap : 1) * sizeof(rr_elem));
    int rc = -1;
    rr_totals t;
    if (data && arena && vals && els) {
        for (size_t i = 0; i < r->n; i++) memcpy(data + offs[i], r->vals[i], r->vlens[i]);
        if (rr_decode_batch_host(ctx, data, offs, r->n, vals, els, cap, arena, &t) == RR_API_OK) {
            const uint64_t h[3] = {r->n, t.n_elems < cap ? t.n_elems : cap, bytes};
            rc = (write_full(fd_resp, h, sizeof h) == 1 && write_full(fd_resp, vals, h[0] * sizeof(rr_value)) == 1 &&
                  write_full(fd_resp, els, h[1] * sizeof(rr_elem)) == 1 && write_full(fd_resp, arena, bytes) == 1)
                     ? 0 : -1;
        }
    }
    drop_vals(r, free_val);
    free(offs); free(data); free(arena); free(vals); free(els);
    return rc;
}

int rr_rdb_serve(int fd_req, int fd_resp, rr_rdb_multiget_fn get, void (*free_val)(void *), void *user, rr_ctx *ctx,
                 size_t max_batch) {
    if (!get) return fail(RR_API_EINVAL, "rr_rdb_serve: no lookup");
    if (max_batch == 0) max_batch = 1;
    reqs_t r = {0};
    int rc = 0, have_next = 0, next = 0;
    for (;;) {
        int dbi;
        if (have_next) { dbi = next; have_next = 0; }
        else {
            const int g = read_full(fd_req, &dbi, sizeof dbi);
            if (g == 0) break;                              /* normal exit: the child closed the pipe */
            if (g < 0) { rc = fail(RR_API_EINVAL, "request read error"); break; }
        }
        if (dbi == RR_RDB_FLAT_TAG) {
            if (serve_flat(fd_req, fd_resp, &r, get, free_val, user, ctx)) { rc = fail(RR_API_EINVAL, "flat request failed"); break; }
            reqs_clear(&r);
            continue;
        }
        if (read_key(fd_req, dbi, &r)) { rc = fail(RR_API_EINVAL, "request read error"); break; }
        /* every RAW request already queued joins the batch (stop at a FLAT request) */
        while (r.n < max_batch) {
            struct pollfd pf = {fd_req, POLLIN, 0};
            if (poll(&pf, 1, 0) <= 0 || !(pf.revents & POLLIN)) break;
            int d2;
            const int g = read_full(fd_req, &d2, sizeof d2);
            if (g != 1) break;   /* (a close is seen again at the top of the loop) */
            if (d2 == RR_RDB_FLAT_TAG) { have_next = 1; next = d2; break; }
            if (read_key(fd_req, d2, &r)) { rc = -1; break; }
        }
        if (rc || lookup(&r, get, user)) { drop_vals(&r, free_val); rc = fail(RR_API_EINVAL, "lookup failed (missing key)"); break; }
        for (size_t i = 0; i < r.n && !rc; i++) {
            if (write_full(fd_resp, &r.vlens[i], sizeof(size_t)) != 1 || write_full(fd_resp, r.vals[i], r.vlens[i]) != 1)
                rc = fail(RR_API_EINVAL, "response write error");
        }
        drop_vals(&r, free_val);
        reqs_clear(&r);
        if (rc) break;
    }
    reqs_free(&r);
    return rc;
}
