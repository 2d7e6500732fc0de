/*
 * test_rdb.c — unit test of the batched snapshot restore (include/rr_rdb.h, row f4) over real
 * pipes, a snapshot store of the golden fixtures' valid blobs, and the minimal Redis model.
 *
 *   cpu  RAW protocol only (no GPU):
 *        1. rr_rdb_request_batch against rr_rdb_serve, 20000 keys in one call (far more than a
 *           pipe holds in either direction: the pipelining must not deadlock);
 *        2. the reference's serial child (restated from rock_rdb.c:240-267) against
 *           rr_rdb_serve;
 *        3. rr_rdb_request_batch against the reference's serial service thread (restated from
 *           rock_rdb.c:126-230);
 *   gpu  + 4. FLAT: rr_compat_rdb_load_batch (the fork child's side: robj from the records the
 *           parent decoded on its GPU) equals desObject on every blob, checked through
 *           serObject, for 5000 keys.
 * Exit status 0 when every check passes.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "server.h"
#include "rock_serdes_compat.h"
#include "fixtures.h"

static int fails;
#define CHECK(c, ...) do { if (!(c)) { fails++; printf("FAIL: "); printf(__VA_ARGS__); printf("\n"); } } while (0)

/* ---- the snapshot store: key "k:<i>" -> valid fixture i % nvalid, or (bench with a config)
 * value i of a generated batch ---- */
static const fixture_t *valid[N_FIXTURES];
static int nvalid;
static rr_host_batch gen;   /* gen.n > 0: the store serves this batch */
typedef struct { const uint8_t *blob; size_t len; } val_t;
static int blob_of(const char *key, size_t len, val_t *v) {
    char buf[32];
    if (len < 3 || len >= sizeof buf) return 0;
    memcpy(buf, key, len);
    buf[len] = 0;
    long i = strtol(buf + 2, NULL, 10);
    if (i < 0) return 0;
    if (gen.n) {
        const uint64_t j = (uint64_t)i % gen.n;
        v->blob = gen.data + gen.offsets[j];
        v->len = gen.offsets[j + 1] - gen.offsets[j];
    } else {
        v->blob = valid[i % nvalid]->blob;
        v->len = valid[i % nvalid]->len;
    }
    return 1;
}
static int store_get(void *user, size_t k, const int *dbis, const char *const *keys, const size_t *lens, void **vals,
                     size_t *vlens) {
    (void)user;
    for (size_t i = 0; i < k; i++) {
        val_t f;
        vals[i] = NULL;
        if (dbis[i] != 3 || !blob_of(keys[i], lens[i], &f)) continue;
        vals[i] = malloc(f.len ? f.len : 1);
        memcpy(vals[i], f.blob, f.len);
        vlens[i] = f.len;
    }
    return 0;
}

typedef struct { int rfd, wfd; rr_ctx *ctx; int rc; int serial; } server_t;
static void *serve_thread(void *a) {
    server_t *s = (server_t *)a;
    s->rc = rr_rdb_serve(s->rfd, s->wfd, store_get, free, NULL, s->ctx, 4096);
    close(s->wfd);
    return NULL;
}

/* the reference's service thread, one request at a time (rock_rdb.c:126-230) */
static int rd(int fd, void *b, size_t n) { char *p = b; while (n) { ssize_t r = read(fd, p, n); if (r <= 0) return (int)r; p += r; n -= (size_t)r; } return 1; }
static int wr(int fd, const void *b, size_t n) { const char *p = b; while (n) { ssize_t r = write(fd, p, n); if (r < 0) return -1; p += r; n -= (size_t)r; } return 1; }
static void *serial_server(void *a) {
    server_t *s = (server_t *)a;
    for (;;) {
        int dbi;
        size_t klen;
        if (rd(s->rfd, &dbi, sizeof dbi) != 1) break;
        if (rd(s->rfd, &klen, sizeof klen) != 1) { s->rc = -1; break; }
        char key[64];
        if (klen >= sizeof key || rd(s->rfd, key, klen) != 1) { s->rc = -1; break; }
        val_t f;
        if (dbi != 3 || !blob_of(key, klen, &f)) { s->rc = -1; break; }
        size_t vlen = f.len;
        if (wr(s->wfd, &vlen, sizeof vlen) != 1 || wr(s->wfd, f.blob, vlen) != 1) { s->rc = -1; break; }
    }
    close(s->wfd);
    return NULL;
}

static void make_keys(size_t k, char **keys, size_t *lens, int *dbis) {
    for (size_t i = 0; i < k; i++) {
        keys[i] = malloc(24);
        lens[i] = (size_t)snprintf(keys[i], 24, "k:%zu", i);
        dbis[i] = 3;
    }
}

static void start(server_t *s, int *cfd_req, int *cfd_resp, int serial, rr_ctx *ctx, pthread_t *th) {
    int a[2], b[2];
    if (pipe(a) || pipe(b)) { perror("pipe"); exit(2); }
    s->rfd = a[0]; s->wfd = b[1]; s->ctx = ctx; s->rc = 0; s->serial = serial;
    *cfd_req = a[1];
    *cfd_resp = b[0];
    pthread_create(th, NULL, serial ? serial_server : serve_thread, s);
}
static void stop(server_t *s, int cfd_req, int cfd_resp, pthread_t th) {
    close(cfd_req);
    pthread_join(th, NULL);
    close(cfd_resp);
    close(s->rfd);
}

static void check_blobs(const rr_rdb_blobs *b, size_t k, char **keys, size_t *lens, const char *what) {
    CHECK(b->n == k, "%s: %llu values for %zu keys", what, (unsigned long long)b->n, k);
    for (size_t i = 0; i < k && i < b->n; i++) {
        val_t f;
        blob_of(keys[i], lens[i], &f);
        const uint64_t len = b->offsets[i + 1] - b->offsets[i];
        if (len != f.len || memcmp(b->data + b->offsets[i], f.blob, f.len)) {
            CHECK(0, "%s: value %zu differs", what, i);
            break;
        }
    }
}

#include <time.h>
static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }

/* bench: keys/s of the reference's serial fetch, the pipelined RAW batch and the FLAT restore
 * (fetch + GPU decode in the service + robj in the child) over the same pipes.  With the oracle
 * linked (RR_RDB_BENCH_ORACLE, test infrastructure), the RAW legs also run the child's CPU
 * desObject on every fetched value (oracle/rro_faithful.c: the reference's allocation pattern),
 * so the child's whole restore is timed on both sides. */
#ifdef RR_RDB_BENCH_ORACLE
#include "rr_oracle.h"
#endif
static int bench(size_t k, char **keys, size_t *lens, int *dbis) {
    server_t s;
    pthread_t th;
    int fq, fr;
    start(&s, &fq, &fr, 0, NULL, &th);
    double t0 = now();
    for (size_t i = 0; i < k; i++) {
        size_t vlen = 0;
        wr(fq, &dbis[i], sizeof(int)); wr(fq, &lens[i], sizeof(size_t)); wr(fq, keys[i], lens[i]);
        rd(fr, &vlen, sizeof vlen);
        char *v = malloc(vlen ? vlen : 1);
        rd(fr, v, vlen);
        free(v);
    }
    const double t_serial = now() - t0;
    stop(&s, fq, fr, th);
    double t_serial_des = 0, t_batch_des = 0;
#ifdef RR_RDB_BENCH_ORACLE
    /* the reference child: one round trip, then desObject, per key (rock.c:527-550) */
    start(&s, &fq, &fr, 0, NULL, &th);
    t0 = now();
    for (size_t i = 0; i < k; i++) {
        size_t vlen = 0;
        wr(fq, &dbis[i], sizeof(int)); wr(fq, &lens[i], sizeof(size_t)); wr(fq, keys[i], lens[i]);
        rd(fr, &vlen, sizeof vlen);
        uint8_t *v = malloc(vlen ? vlen : 1);
        rd(fr, v, vlen);
        const uint64_t o[2] = {0, vlen};
        uint64_t nbad = 0;
        rro_store *st = rro_faithful_decode(v, o, 1, &nbad);
        rro_store_free(st);
        free(v);
    }
    t_serial_des = now() - t0;
    stop(&s, fq, fr, th);
#endif
    /* the product paths of a child linked with the shim: desObject is the host codec (f1) —
     * the unchanged serial child (rock.c:527-550), and the pipelined RAW batch */
    start(&s, &fq, &fr, 0, NULL, &th);
    t0 = now();
    for (size_t i = 0; i < k; i++) {
        size_t vlen = 0;
        wr(fq, &dbis[i], sizeof(int)); wr(fq, &lens[i], sizeof(size_t)); wr(fq, keys[i], lens[i]);
        rd(fr, &vlen, sizeof vlen);
        char *v = malloc(vlen ? vlen : 1);
        rd(fr, v, vlen);
        decrRefCount(desObject(v, vlen));
        free(v);
    }
    const double t_serial_shim = now() - t0;
    stop(&s, fq, fr, th);
    start(&s, &fq, &fr, 0, NULL, &th);
    rr_rdb_blobs b;
    t0 = now();
    rr_rdb_request_batch(fq, fr, dbis, (const char *const *)keys, lens, k, &b);
    const double t_batch = now() - t0;
    double t_batch_shim;
    {
        const double t1 = now();
        for (size_t i = 0; i < k; i++) decrRefCount(desObject(b.data + b.offsets[i], b.offsets[i + 1] - b.offsets[i]));
        t_batch_shim = t_batch + (now() - t1);
    }
#ifdef RR_RDB_BENCH_ORACLE
    {   /* the pipelined RAW batch + the child's CPU desObject on every value */
        uint64_t nbad = 0;
        const double t1 = now();
        rro_store *st = rro_faithful_decode(b.data, b.offsets, b.n, &nbad);
        t_batch_des = t_batch + (now() - t1);
        rro_store_free(st);
    }
#endif
    rr_rdb_blobs_free(&b);
    stop(&s, fq, fr, th);
    rr_ctx *ctx = NULL;
    if (rr_ctx_create(0, &ctx) != RR_API_OK) return 2;
    robj **objs = malloc(sizeof(robj *) * k);
    sds *sk = malloc(sizeof(sds) * k);
    for (size_t i = 0; i < k; i++) sk[i] = sdsnewlen(keys[i], lens[i]);
    start(&s, &fq, &fr, 0, ctx, &th);
    rr_compat_rdb_load_batch(fq, fr, 3, sk, 1000, objs);   /* warm the GPU context */
    for (size_t i = 0; i < 1000; i++) decrRefCount(objs[i]);
    t0 = now();
    rr_compat_rdb_load_batch(fq, fr, 3, sk, k, objs);
    const double t_flat = now() - t0;
    stop(&s, fq, fr, th);
    for (size_t i = 0; i < k; i++) { decrRefCount(objs[i]); sdsfree(sk[i]); }
    free(objs); free(sk);
    rr_ctx_destroy(ctx);
    uint64_t bytes = 0;
    for (size_t i = 0; i < k; i++) {
        val_t f;
        blob_of(keys[i], lens[i], &f);
        bytes += f.len;
    }
    printf("{\"keys\": %zu, \"bytes\": %llu, \"store\": \"%s\", \"serial_fetch_keys_per_s\": %.0f, "
           "\"batch_fetch_keys_per_s\": %.0f, \"flat_restore_keys_per_s\": %.0f",
           k, (unsigned long long)bytes, gen.n ? "generated batch" : "golden fixtures", k / t_serial, k / t_batch,
           k / t_flat);
    printf(", \"serial_fetch_shim_desobject_keys_per_s\": %.0f, \"batch_fetch_shim_desobject_keys_per_s\": %.0f",
           k / t_serial_shim, k / t_batch_shim);
    if (t_serial_des > 0)
        printf(", \"serial_fetch_cpu_desobject_keys_per_s\": %.0f, \"batch_fetch_cpu_desobject_keys_per_s\": %.0f",
               k / t_serial_des, k / t_batch_des);
    printf("}\n");
    return 0;
}

int main(int argc, char **argv) {
    const int gpu = argc > 1 && !strcmp(argv[1], "gpu");
    for (int i = 0; i < N_FIXTURES; i++)
        if (FIXTURES[i].status == 0) valid[nvalid++] = &FIXTURES[i];
    enum { K = 20000, KB = 200000 };
    static char *keys[KB];
    static size_t lens[KB];
    static int dbis[KB];
    make_keys(KB, keys, lens, dbis);
    if (argc > 1 && !strcmp(argv[1], "bench")) {   /* bench [config k]: a generated store of k values */
        size_t k = K;
        if (argc > 3) {
            k = (size_t)strtoull(argv[3], NULL, 10);
            if (k == 0 || k > KB || rr_gen_batch(atoi(argv[2]), k, rr_gen_default_seed(atoi(argv[2])), &gen) != 0) return 2;
        }
        return bench(k, keys, lens, dbis);
    }
    server_t s;
    pthread_t th;
    int fq, fr;

    /* 1. batch client vs batch service */
    start(&s, &fq, &fr, 0, NULL, &th);
    rr_rdb_blobs b;
    int rc = rr_rdb_request_batch(fq, fr, dbis, (const char *const *)keys, lens, K, &b);
    CHECK(rc == RR_API_OK, "batch vs batch: %s", rr_last_error());
    if (rc == RR_API_OK) check_blobs(&b, K, keys, lens, "batch vs batch");
    CHECK(((uintptr_t)b.data & 15) == 0, "blob buffer not 16-byte aligned");
    rr_rdb_blobs_free(&b);
    stop(&s, fq, fr, th);
    CHECK(s.rc == 0, "service did not exit cleanly (%d)", s.rc);

    /* 2. the reference's serial child vs the batch service */
    start(&s, &fq, &fr, 0, NULL, &th);
    for (size_t i = 0; i < 300; i++) {
        size_t vlen = 0;
        wr(fq, &dbis[i], sizeof(int));
        wr(fq, &lens[i], sizeof(size_t));
        wr(fq, keys[i], lens[i]);
        if (rd(fr, &vlen, sizeof vlen) != 1) { CHECK(0, "serial child: no response"); break; }
        char *v = malloc(vlen ? vlen : 1);
        rd(fr, v, vlen);
        val_t f;
        blob_of(keys[i], lens[i], &f);
        CHECK(vlen == f.len && !memcmp(v, f.blob, vlen), "serial child: value %zu differs", i);
        free(v);
    }
    stop(&s, fq, fr, th);

    /* 3. the batch child vs the reference's serial service */
    start(&s, &fq, &fr, 1, NULL, &th);
    rc = rr_rdb_request_batch(fq, fr, dbis, (const char *const *)keys, lens, K, &b);
    CHECK(rc == RR_API_OK, "batch vs serial: %s", rr_last_error());
    if (rc == RR_API_OK) check_blobs(&b, K, keys, lens, "batch vs serial");
    rr_rdb_blobs_free(&b);
    stop(&s, fq, fr, th);
    CHECK(s.rc == 0, "serial service error");

    /* a missing key ends the service (the reference's goto err) and the child sees the close */
    start(&s, &fq, &fr, 0, NULL, &th);
    int bad = 9;
    rc = rr_rdb_request_batch(fq, fr, &bad, (const char *const *)keys, lens, 1, &b);
    CHECK(rc != RR_API_OK, "missing key accepted");
    stop(&s, fq, fr, th);
    CHECK(s.rc != 0, "service kept going after a missing key");

    if (gpu) {   /* 4. FLAT: decode in the service (GPU), robj in the child */
        rr_ctx *ctx = NULL;
        if (rr_ctx_create(0, &ctx) != RR_API_OK) { printf("no GPU: %s\n", rr_last_error()); return 2; }
        enum { KF = 5000 };
        static robj *objs[KF];
        sds skeys[KF];
        for (size_t i = 0; i < KF; i++) skeys[i] = sdsnewlen(keys[i], lens[i]);
        start(&s, &fq, &fr, 0, ctx, &th);
        rr_compat_rdb_load_batch(fq, fr, 3, skeys, KF, objs);
        stop(&s, fq, fr, th);
        CHECK(s.rc == 0, "flat service error");
        for (size_t i = 0; i < KF; i++) {
            val_t f;
            blob_of(keys[i], lens[i], &f);
            robj *o = desObject((void *)f.blob, f.len);
            sds a = serObject(objs[i]), c = serObject(o);
            if (sdslen(a) != sdslen(c) || memcmp(a, c, sdslen(a))) { CHECK(0, "flat restore: value %zu differs", i); }
            CHECK(objs[i]->lru == o->lru && objs[i]->type == o->type && objs[i]->encoding == o->encoding,
                  "flat restore: value %zu header differs", i);
            sdsfree(a); sdsfree(c);
            decrRefCount(o);
            decrRefCount(objs[i]);
            sdsfree(skeys[i]);
        }
        rr_ctx_destroy(ctx);
    }
    for (size_t i = 0; i < KB; i++) free(keys[i]);
    printf("%d failures (%d valid fixtures, %s)\n", fails, nvalid, gpu ? "cpu+gpu" : "cpu");
    return fails ? 1 : 0;
}
