/*
 * rock_serdes_compat.c — bodies of RedRock's legacy serdes signatures (rock_serdes.h:47-49)
 * over the MI355X batch engine (include/rock_serdes_compat.h).
 *
 * Built inside a Redis tree: it includes the tree's server.h and uses only the Redis API the
 * reference rock_serdes.c itself uses (robj constructors, sds, dict, quicklist, intset,
 * zslInsert, zmalloc).  The decode and encode of the bytes run on the GPU through
 * rr_decode_batch_host / rr_encode_batch_host; this file only turns flat records into heap
 * objects and back, which a GPU cannot do.  Abort semantics are the reference's: a blob the
 * reference would reject (any nonzero rr_value.status) ends in serverPanic.
 *
 * The repo's own unit test compiles this file against a minimal Redis model
 * (tests/c/miniredis) instead of a Redis tree.
 */
#ifndef RR_REDIS_TREE
#define RR_REDIS_TREE 1
#endif
#include <poll.h>
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include "server.h"

#include "rock_serdes_compat.h"

static int g_device;
static __thread rr_ctx *g_ctx;   /* one engine context per host thread (rr_serdes.h) */

void rr_compat_set_device(int device) { g_device = device; }

/* ---- fork children (rock.c:527-550: BGSAVE / AOF rewrite call desObject in a fork()ed child).
 * A child must not touch the HIP runtime its parent initialised, so in a child desObject does
 * not decode itself: it sends the blob over a socket to a decode service thread in the parent
 * (rr_rdb_serve's FLAT request, the blob standing in for the key) and builds the robj from the
 * flat records that come back.  rock.c needs no change.
 *
 * Every fork gets a connection of its own: right before the fork (pthread_atfork prepare) the
 * parent opens a socketpair and starts a service thread on one end; after the fork the parent
 * closes the child's end and the child closes every service end it inherited.  So the service
 * sees EOF when its child exits (killRDBChild on FLUSHALL, SHUTDOWN, replication changes) and
 * drops any response it still owed, and a later child can never read an earlier child's reply
 * or send into the middle of its request.  A service that fails (a decode error, a device
 * failure, a write error) closes its end: the child's request then fails and it panics instead
 * of waiting forever. */
static pid_t g_owner;                     /* the process whose threads own GPU contexts */
static pthread_mutex_t g_svc_mu = PTHREAD_MUTEX_INITIALIZER;
#define RR_COMPAT_MAX_SVC 64
static int g_svc_fds[RR_COMPAT_MAX_SVC];  /* service ends of the live connections (parent) */
static int g_nsvc;
/* the service threads, joinable: a thread still inside the HIP runtime (its context's teardown
 * after its child exited) when the process exits would race the runtime's own teardown, so the
 * owner's exit ends and joins them (compat_exit); a finished thread is joined when its slot is
 * next needed.  0 free, 1 running, 2 finished */
static pthread_t g_th[RR_COMPAT_MAX_SVC];
static int g_th_state[RR_COMPAT_MAX_SVC];
static int g_child_fd = -1;               /* this process's own connection (child end) */
static int g_fork_fd = -1;                /* the connection opened for the fork in progress */
static int g_as_child;                    /* test hook: route this process as a child would */

static int in_child(void) { return g_as_child || (g_owner && getpid() != g_owner); }

static void compat_exit(void);
static int g_exit_hooked;
static void exit_hook(void) {
    if (!__atomic_exchange_n(&g_exit_hooked, 1, __ATOMIC_SEQ_CST)) atexit(compat_exit);
}

static rr_ctx *engine(void) {
    if (in_child()) serverPanic("rock serdes: the GPU engine cannot be used in a fork child (HIP is the parent's)");
    if (!g_ctx) {
        if (rr_ctx_create(g_device, &g_ctx) != RR_API_OK) serverPanic("rock serdes engine: %s", rr_last_error());
        if (!g_owner) g_owner = getpid();
        exit_hook();
    }
    return g_ctx;
}

static int echo_blob(void *user, size_t k, const int *dbis, const char *const *keys, const size_t *key_lens,
                     void **vals, size_t *val_lens) {
    (void)user; (void)dbis;
    for (size_t i = 0; i < k; i++) { vals[i] = (void *)keys[i]; val_lens[i] = key_lens[i]; }
    return 0;
}

/* one connection's service: until its child closes the other end, or a request fails */
static void *decode_service(void *arg) {
    const int slot = (int)((intptr_t)arg >> 32), fd = (int)(uint32_t)(intptr_t)arg;
    sigset_t pipe_set;   /* a reply to a child that is gone: EPIPE on this thread, not SIGPIPE */
    sigemptyset(&pipe_set);
    sigaddset(&pipe_set, SIGPIPE);
    pthread_sigmask(SIG_BLOCK, &pipe_set, NULL);
    /* the engine context only once the child's first request is there: the thread starts inside
     * fork()'s prepare handler, and a child that never asks must cost no GPU context */
    rr_ctx *ctx = NULL;
    struct pollfd pf = {fd, POLLIN, 0};
    char peek;
    if (poll(&pf, 1, -1) > 0 && recv(fd, &peek, 1, MSG_PEEK) == 1 && rr_ctx_create(g_device, &ctx) == RR_API_OK) {
        exit_hook();
        rr_rdb_serve(fd, fd, echo_blob, NULL, NULL, ctx, 64);
        rr_ctx_destroy(ctx);
    }
    pthread_mutex_lock(&g_svc_mu);
    for (int i = 0; i < g_nsvc; i++)
        if (g_svc_fds[i] == fd) { g_svc_fds[i] = g_svc_fds[--g_nsvc]; break; }
    close(fd);   /* the child's read sees EOF */
    g_th_state[slot] = 2;
    pthread_mutex_unlock(&g_svc_mu);
    return NULL;
}

/* a new connection with its own service thread (g_svc_mu held): the child end, or -1 */
static int open_connection(void) {
    int sv[2];
    pthread_t th;
    int slot = -1;
    for (int i = 0; i < RR_COMPAT_MAX_SVC; i++) {
        if (g_th_state[i] == 2) { pthread_join(g_th[i], NULL); g_th_state[i] = 0; }   /* (it has returned) */
        if (g_th_state[i] == 0 && slot < 0) slot = i;
    }
    if (slot < 0 || g_nsvc == RR_COMPAT_MAX_SVC || socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return -1;
    g_svc_fds[g_nsvc++] = sv[0];
    if (pthread_create(&th, NULL, decode_service, (void *)(((intptr_t)slot << 32) | (intptr_t)(uint32_t)sv[0])) != 0) {
        g_nsvc--;
        close(sv[0]);
        close(sv[1]);
        return -1;
    }
    g_th[slot] = th;
    g_th_state[slot] = 1;
    return sv[1];
}

/* this process's own connection (the in-process child route of the tests) */
int rr_compat_service_start(void) {
    pthread_mutex_lock(&g_svc_mu);
    if (g_child_fd < 0) g_child_fd = open_connection();
    const int rc = g_child_fd >= 0 ? 0 : -1;
    pthread_mutex_unlock(&g_svc_mu);
    return rc;
}

/* the lock is held across the fork, so the child's copy of the registry is consistent */
static void atfork_prepare(void) {
    pthread_mutex_lock(&g_svc_mu);
    if (g_owner && getpid() == g_owner && !g_as_child) g_fork_fd = open_connection();
}
static void atfork_parent(void) {
    if (g_fork_fd >= 0) close(g_fork_fd);   /* the child's end is the child's alone */
    g_fork_fd = -1;
    pthread_mutex_unlock(&g_svc_mu);
}
static void atfork_child(void) {
    g_ctx = NULL;   /* (the parent's context is not ours) */
    memset(g_th_state, 0, sizeof g_th_state);   /* (nor its threads) */
    for (int i = 0; i < g_nsvc; i++) close(g_svc_fds[i]);   /* the parent's service ends */
    g_nsvc = 0;
    if (g_child_fd >= 0) close(g_child_fd);   /* the parent's own connection */
    g_child_fd = g_fork_fd;
    g_fork_fd = -1;
    pthread_mutex_unlock(&g_svc_mu);
}
/* the owner's exit: every service's connection shut down (its thread sees EOF, destroys its
 * context, returns), then every thread joined, before the HIP runtime's own teardown (exit_hook
 * registers this once the runtime is up, so it runs before every handler the runtime registered) */
static void compat_exit(void) {
    if (g_owner && getpid() != g_owner) return;   /* (a fork child: no threads of its own) */
    pthread_mutex_lock(&g_svc_mu);
    for (int i = 0; i < g_nsvc; i++) shutdown(g_svc_fds[i], SHUT_RDWR);
    pthread_t th[RR_COMPAT_MAX_SVC];
    int n = 0;
    for (int i = 0; i < RR_COMPAT_MAX_SVC; i++)
        if (g_th_state[i]) { th[n++] = g_th[i]; g_th_state[i] = 0; }
    pthread_mutex_unlock(&g_svc_mu);
    for (int i = 0; i < n; i++) pthread_join(th[i], NULL);
}
__attribute__((constructor)) static void compat_atfork_register(void) {
    pthread_atfork(atfork_prepare, atfork_parent, atfork_child);
}

void rr_compat_test_as_child(int on) { g_as_child = on; }

/* test hooks: a child that dies after sending a request (its reply must never reach another
 * child), and the parent's services ending (a waiting child must fail, not hang) */
int rr_compat_test_send_only(const void *blob, size_t len) {
    const int dbi = RR_RDB_FLAT_TAG, zero = 0;
    const size_t one = 1;
    return g_child_fd >= 0 && write(g_child_fd, &dbi, sizeof dbi) == sizeof dbi &&
                   write(g_child_fd, &one, sizeof one) == sizeof one && write(g_child_fd, &zero, sizeof zero) == sizeof zero &&
                   write(g_child_fd, &len, sizeof len) == sizeof len && write(g_child_fd, blob, len) == (ssize_t)len
               ? 0 : -1;
}
void rr_compat_test_drop_services(void) {
    pthread_mutex_lock(&g_svc_mu);
    for (int i = 0; i < g_nsvc; i++) shutdown(g_svc_fds[i], SHUT_RDWR);
    pthread_mutex_unlock(&g_svc_mu);
}

static const char *status_name(unsigned st) {
    static const char *names[RR_N_STATUS] = {"ok", "short blob", "unknown type", "string encoding",
                                             "INT string length", "EMBSTR length", "truncated element",
                                             "element count", "intset", "ziplist length", "ziplist",
                                             "capacity", "encode", "duplicate hash field", "NaN score"};
    return st < RR_N_STATUS ? names[st] : "?";
}

/* ---------------------------------------------------------------- flat -> robj (desObject) */

/* skiplist pairs in blob order (a member's arena offset is its blob offset): desZset inserts
 * them in that order, which decides which copy of a repeated member its dict keeps */
static int pair_by_offset(const void *a, const void *b) {
    const rr_elem *x = (const rr_elem *)a, *y = (const rr_elem *)b;
    return x->data < y->data ? -1 : x->data > y->data;
}

/* The object desObject (rock_serdes.c:538-564) builds for one decoded value: every
 * descriptor already says what the reference derives from the bytes (rr_format.h). */
static robj *robj_from_flat(const rr_value *v, const rr_elem *el, const uint8_t *arena) {
    robj *o = NULL;
    const uint32_t n = v->n_elems;
    switch (v->type) {
    case RR_TYPE_STRING:                                                      /* :133-158 */
        if (v->enc == RR_ENC_INT) o = createStringObjectFromLongLongForValue((long long)el[0].data);
        else if (v->enc == RR_ENC_RAW) o = createRawStringObject((const char *)arena + el[0].data, el[0].len);
        else o = createEmbeddedStringObject((const char *)arena + el[0].data, el[0].len);
        break;
    case RR_TYPE_LIST_QUICKLIST:                                              /* :191-214 */
        o = createQuicklistObject();
        quicklistSetOptions(o->ptr, server.list_max_ziplist_size, server.list_compress_depth);
        for (uint32_t i = 0; i < n; i++) {
            if (el[i].kind == RR_K_INT) {   /* the element's bytes were this integer's decimal */
                char buf[32];
                int l = ll2string(buf, sizeof buf, (long long)el[i].data);
                quicklistPushTail(o->ptr, buf, (size_t)l);
            } else {
                quicklistPushTail(o->ptr, (void *)(arena + el[i].data), el[i].len);
            }
        }
        break;
    case RR_TYPE_SET_INTSET: {                                                /* :255-276 */
        o = createIntsetObject();
        const uint32_t w = v->enc;
        intset *is = zrealloc(o->ptr, sizeof(intset) + (size_t)w * n);
        is->encoding = w;
        is->length = n;
        for (uint32_t i = 0; i < n; i++) memcpy((char *)is->contents + (size_t)i * w, &el[i].data, w);
        o->ptr = is;
        break;
    }
    case RR_TYPE_SET_HT:                                                      /* :277-303 */
        o = createSetObject();
        if (n > DICT_HT_INITIAL_SIZE) dictExpand(o->ptr, n);
        for (uint32_t i = 0; i < n; i++) dictAdd(o->ptr, sdsnewlen(arena + el[i].data, el[i].len), NULL);
        break;
    case RR_TYPE_HASH_ZIPLIST:                                                /* :356-366 */
    case RR_TYPE_ZSET_ZIPLIST: {                                              /* :455-466 */
        unsigned char *zl = zmalloc(el[0].len);
        memcpy(zl, arena + el[0].data, el[0].len);
        o = createObject(v->type == RR_TYPE_HASH_ZIPLIST ? OBJ_HASH : OBJ_ZSET, zl);
        o->encoding = OBJ_ENCODING_ZIPLIST;
        break;
    }
    case RR_TYPE_HASH_HT: {                                                   /* :368-407 */
        dict *d = dictCreate(&hashDictType, NULL);
        if (n / 2 > DICT_HT_INITIAL_SIZE) dictExpand(d, n / 2);
        for (uint32_t i = 0; i < n; i += 2)
            dictAdd(d, sdsnewlen(arena + el[i].data, el[i].len), sdsnewlen(arena + el[i + 1].data, el[i + 1].len));
        o = createObject(OBJ_HASH, d);
        o->encoding = OBJ_ENCODING_HT;
        break;
    }
    case RR_TYPE_ZSET_SKIPLIST: {                                             /* :467-501 */
        o = createZsetObject();
        zset *zs = o->ptr;
        const uint32_t np = n / 2;
        if (np > DICT_HT_INITIAL_SIZE) dictExpand(zs->dict, np);
        /* the flat pairs are in serZset's order; desZset inserted them in blob order */
        const rr_elem (*pr)[2] = (const rr_elem (*)[2])el;
        rr_elem (*tmp)[2] = NULL;
        for (uint32_t i = 1; i < np; i++)
            if (pr[i][0].data < pr[i - 1][0].data) {
                tmp = zmalloc(sizeof(rr_elem) * 2 * (size_t)np);
                memcpy(tmp, el, sizeof(rr_elem) * 2 * (size_t)np);
                qsort(tmp, np, sizeof(rr_elem) * 2, pair_by_offset);
                pr = (const rr_elem (*)[2])tmp;
                break;
            }
        for (uint32_t i = 0; i < np; i++) {
            sds ele = sdsnewlen(arena + pr[i][0].data, pr[i][0].len);
            double score;
            memcpy(&score, &pr[i][1].data, sizeof score);
            zskiplistNode *zn = zslInsert(zs->zsl, score, ele);
            dictAdd(zs->dict, ele, &zn->score);
        }
        if (tmp) zfree(tmp);
        break;
    }
    default:
        serverPanic("desObject type error!");
    }
    o->lru = v->lru;
    return o;
}

/* a child's batch: the parent's decode service decodes it, the robj are built here */
static void des_batch_in_child(void *const *bufs, const size_t *lens, size_t n, robj **out) {
    if (g_child_fd < 0)
        serverPanic("desObject in a fork child: the parent's decode service is not running "
                    "(the parent must use the engine before it forks)");
    int *dbis = zmalloc(sizeof(int) * n);
    for (size_t i = 0; i < n; i++) dbis[i] = 0;
    rr_rdb_flat f;
    if (rr_rdb_request_flat(g_child_fd, g_child_fd, dbis, (const char *const *)bufs, lens, n, &f) != RR_API_OK || f.n != n)
        serverPanic("desObject in a fork child: %s", rr_last_error());
    for (size_t i = 0; i < n; i++) {
        if (f.values[i].status != RR_OK)   /* the reference's serverAssert / serverPanic site */
            serverPanic("desObject: bad blob (%s, status %u)", status_name(f.values[i].status), f.values[i].status);
        out[i] = robj_from_flat(&f.values[i], f.elems + f.values[i].elem_base, f.arena);
    }
    rr_rdb_flat_free(&f);
    zfree(dbis);
}

void rr_compat_des_batch(void *const *bufs, const size_t *lens, size_t n, robj **out) {
    if (n == 0) return;
    if (in_child()) { des_batch_in_child(bufs, lens, n, out); return; }
    uint64_t *offs = zmalloc(sizeof(uint64_t) * (n + 1));
    offs[0] = 0;
    for (size_t i = 0; i < n; i++) offs[i + 1] = offs[i] + lens[i];
    const uint64_t bytes = offs[n], padded = (bytes + 15) & ~15ull;
    uint8_t *data = zmalloc(padded ? padded : 16);
    for (size_t i = 0; i < n; i++) memcpy(data + offs[i], bufs[i], lens[i]);
    memset(data + bytes, 0, padded - bytes);
    const uint64_t cap = rr_decode_elem_bound(n, bytes);
    rr_value *vals = zmalloc(sizeof(rr_value) * n);
    rr_elem *els = zmalloc(sizeof(rr_elem) * (cap ? cap : 1));
    rr_totals t;
    /* no arena download: it would mirror `data` byte for byte, so the descriptors index it */
    if (rr_decode_batch_host(engine(), data, offs, n, vals, els, cap, NULL, &t) != RR_API_OK)
        serverPanic("desObject: %s", rr_last_error());
    for (size_t i = 0; i < n; i++) {
        if (vals[i].status != RR_OK)   /* the reference's serverAssert / serverPanic site */
            serverPanic("desObject: bad blob (%s, status %u)", status_name(vals[i].status), vals[i].status);
        out[i] = robj_from_flat(&vals[i], els + vals[i].elem_base, data);
    }
    zfree(offs); zfree(data); zfree(vals); zfree(els);
}

void rr_compat_rdb_load_batch(int fd_req, int fd_resp, int dbid, sds *keys, size_t k, robj **out) {
    if (k == 0) return;
    int *dbis = zmalloc(sizeof(int) * k);
    size_t *lens = zmalloc(sizeof(size_t) * k);
    for (size_t i = 0; i < k; i++) { dbis[i] = dbid; lens[i] = sdslen(keys[i]); }
    rr_rdb_flat f;
    if (rr_rdb_request_flat(fd_req, fd_resp, dbis, (const char *const *)keys, lens, k, &f) != RR_API_OK || f.n != k)
        serverPanic("rock rdb batch restore: %s", rr_last_error());
    for (size_t i = 0; i < k; i++) {
        if (f.values[i].status != RR_OK)   /* desObject's assert sites, as in rr_compat_des_batch */
            serverPanic("desObject: bad blob (%s, status %u)", status_name(f.values[i].status), f.values[i].status);
        out[i] = robj_from_flat(&f.values[i], f.elems + f.values[i].elem_base, f.arena);
    }
    rr_rdb_flat_free(&f);
    zfree(dbis);
    zfree(lens);
}

robj *desObject(void *buf, size_t len) {
    robj *o = NULL;
    rr_compat_des_batch(&buf, &len, 1, &o);
    return o;
}

robj *desString(char *s, size_t len, uint32_t lru) {
    serverAssert(len >= 2 + sizeof(lru));                                   /* :134-135 */
    serverAssert(s[0] == RR_TYPE_STRING);
    robj *o = desObject(s, len);
    o->lru = lru;
    return o;
}

/* ---------------------------------------------------------------- robj -> flat (serObject) */
typedef struct {
    rr_value *vals;
    rr_elem *els;
    uint8_t *arena;
    uint64_t nv, ne, na, cap_v, cap_e, cap_a, out_bound;
} flat_t;

static rr_elem *add_elem(flat_t *f) {
    if (f->ne == f->cap_e) {
        f->cap_e = f->cap_e ? 2 * f->cap_e : 64;
        f->els = zrealloc(f->els, sizeof(rr_elem) * f->cap_e);
    }
    rr_elem *e = &f->els[f->ne++];
    memset(e, 0, sizeof *e);
    return e;
}
static void add_str(flat_t *f, const void *p, size_t len) {
    if (f->na + len > f->cap_a) {
        while (f->na + len > f->cap_a) f->cap_a = f->cap_a ? 2 * f->cap_a : 4096;
        f->arena = zrealloc(f->arena, f->cap_a);
    }
    rr_elem *e = add_elem(f);
    e->kind = RR_K_STR;
    e->data = f->na;
    e->len = (uint32_t)len;
    if (len) memcpy(f->arena + f->na, p, len);
    f->na += len;
    f->out_bound += 8 + len;
}
static void add_int(flat_t *f, long long v) {
    rr_elem *e = add_elem(f);
    e->kind = RR_K_INT;
    e->data = (uint64_t)v;
    f->out_bound += 8 + 24;
}

/* serObject (rock_serdes.c:512-535): the value's type tag (serObjectType :62-110), its lru and
 * its elements in the order ser* walks them */
static void flatten(flat_t *f, robj *o) {
    rr_value *v = &f->vals[f->nv++];
    memset(v, 0, sizeof *v);
    v->lru = o->lru;
    v->elem_base = (uint32_t)f->ne;
    f->out_bound += 13;
    switch (o->type) {
    case OBJ_STRING:                                                          /* :114-128 */
        v->type = RR_TYPE_STRING;
        v->enc = (uint8_t)o->encoding;
        if (o->encoding == OBJ_ENCODING_INT) add_int(f, (long long)(intptr_t)o->ptr);
        else {
            serverAssert(o->encoding == OBJ_ENCODING_RAW || o->encoding == OBJ_ENCODING_EMBSTR);
            add_str(f, o->ptr, sdslen(o->ptr));
        }
        break;
    case OBJ_LIST: {                                                          /* :162-188 */
        serverAssert(o->encoding == OBJ_ENCODING_QUICKLIST);
        v->type = RR_TYPE_LIST_QUICKLIST;
        quicklistIter *it = quicklistGetIterator(o->ptr, AL_START_HEAD);
        quicklistEntry entry;
        while (quicklistNext(it, &entry)) {
            if (entry.value) add_str(f, entry.value, entry.sz);
            else add_int(f, entry.longval);
        }
        quicklistReleaseIterator(it);
        break;
    }
    case OBJ_SET:                                                             /* :217-245 */
        if (o->encoding == OBJ_ENCODING_INTSET) {
            intset *is = o->ptr;
            v->type = RR_TYPE_SET_INTSET;
            v->enc = (uint8_t)is->encoding;
            for (uint32_t i = 0; i < is->length; i++) {
                int64_t x = 0;
                if (is->encoding == 2) { int16_t y; memcpy(&y, (char *)is->contents + 2 * (size_t)i, 2); x = y; }
                else if (is->encoding == 4) { int32_t y; memcpy(&y, (char *)is->contents + 4 * (size_t)i, 4); x = y; }
                else memcpy(&x, (char *)is->contents + 8 * (size_t)i, 8);
                add_int(f, x);
            }
        } else if (o->encoding == OBJ_ENCODING_HT) {
            v->type = RR_TYPE_SET_HT;
            dictIterator *di = dictGetIterator(o->ptr);
            dictEntry *de;
            while ((de = dictNext(di))) { sds ele = dictGetKey(de); add_str(f, ele, sdslen(ele)); }
            dictReleaseIterator(di);
        } else serverPanic("serSet()!");
        break;
    case OBJ_HASH:                                                            /* :314-346 */
        if (o->encoding == OBJ_ENCODING_ZIPLIST) {
            v->type = RR_TYPE_HASH_ZIPLIST;
            add_str(f, o->ptr, ziplistBlobLen(o->ptr));
            f->els[f->ne - 1].kind = RR_K_ZLRAW;
        } else if (o->encoding == OBJ_ENCODING_HT) {
            v->type = RR_TYPE_HASH_HT;
            dictIterator *di = dictGetIterator(o->ptr);
            dictEntry *de;
            while ((de = dictNext(di))) {
                sds field = dictGetKey(de), val = dictGetVal(de);
                add_str(f, field, sdslen(field));
                add_str(f, val, sdslen(val));
            }
            dictReleaseIterator(di);
        } else serverPanic("serHash()");
        break;
    case OBJ_ZSET:                                                            /* :417-446 */
        if (o->encoding == OBJ_ENCODING_ZIPLIST) {
            v->type = RR_TYPE_ZSET_ZIPLIST;
            add_str(f, o->ptr, ziplistBlobLen(o->ptr));
            f->els[f->ne - 1].kind = RR_K_ZLRAW;
        } else if (o->encoding == OBJ_ENCODING_SKIPLIST) {
            v->type = RR_TYPE_ZSET_SKIPLIST;
            zset *zs = o->ptr;
            for (zskiplistNode *zn = zs->zsl->tail; zn; zn = zn->backward) {   /* tail -> head */
                add_str(f, zn->ele, sdslen(zn->ele));
                rr_elem *e = add_elem(f);
                e->kind = RR_K_SCORE;
                memcpy(&e->data, &zn->score, 8);
                f->out_bound += 8;
            }
        } else serverPanic("serZset()");
        break;
    default:
        serverPanic("Unknown object type");
    }
    v->n_elems = (uint32_t)(f->ne - v->elem_base);
}

/* The serialize path's buffers, per thread and kept across calls: the evictor's per-key
 * serObject allocates nothing here after its first calls (a one-off large batch's growth is
 * given back at the end of rr_compat_ser_batch). */
static __thread flat_t t_flat;
static __thread uint64_t *t_offs;
static __thread uint8_t *t_data;
static __thread size_t t_offs_cap, t_data_cap;

void rr_compat_ser_batch(robj *const *objs, size_t n, sds *out) {
    if (n == 0) return;
    flat_t *f = &t_flat;
    f->nv = f->ne = f->na = f->out_bound = 0;
    if (n > f->cap_v) {
        f->vals = zrealloc(f->vals, sizeof(rr_value) * n);
        f->cap_v = n;
    }
    for (size_t i = 0; i < n; i++) flatten(f, objs[i]);
    if (n + 1 > t_offs_cap) {
        t_offs = zrealloc(t_offs, sizeof(uint64_t) * (n + 1));
        t_offs_cap = n + 1;
    }
    if (f->out_bound + 16 > t_data_cap) {
        t_data = zrealloc(t_data, f->out_bound + 16);
        t_data_cap = f->out_bound + 16;
    }
    rr_totals t;
    if (rr_encode_batch_host(engine(), f->vals, f->els, f->ne, f->arena, f->na, n, t_data, f->out_bound + 16, t_offs,
                             &t) != RR_API_OK)
        serverPanic("serObject: %s", rr_last_error());
    if (t.n_bad) serverPanic("serObject: %llu unencodable objects", (unsigned long long)t.n_bad);
    for (size_t i = 0; i < n; i++) out[i] = sdsnewlen(t_data + t_offs[i], t_offs[i + 1] - t_offs[i]);
    /* the thread's buffers keep their size between calls (the per-key serObject allocates
     * nothing), but not a one-off large batch's: past 1 MiB and 4x this call's need, give it back */
    const size_t big = 1u << 20;
    if (t_data_cap > big && t_data_cap > 4 * (f->out_bound + 16)) { zfree(t_data); t_data = NULL; t_data_cap = 0; }
    if (f->cap_a > big && f->cap_a > 4 * f->na) { zfree(f->arena); f->arena = NULL; f->cap_a = 0; }
    if (f->cap_e * sizeof(rr_elem) > big && f->cap_e > 4 * f->ne) { zfree(f->els); f->els = NULL; f->cap_e = 0; }
    if (f->cap_v * sizeof(rr_value) > big && f->cap_v > 4 * n) { zfree(f->vals); f->vals = NULL; f->cap_v = 0; }
    if (t_offs_cap * sizeof(uint64_t) > big && t_offs_cap > 4 * (n + 1)) { zfree(t_offs); t_offs = NULL; t_offs_cap = 0; }
}

sds serObject(robj *o) {
    sds s = NULL;
    rr_compat_ser_batch(&o, 1, &s);
    return s;
}

/* ---------------------------------------------------------------- rock_serdes.h:51-55
 * The debug round trips `ROCK testserdes{str,list,set,hash,zset}` runs (rock.c:170-184), with
 * the reference's inputs (rock_serdes.c:626-901): a live key of db 0 ("abc"; "def" for the set)
 * of the encoding the reference's hook exercises goes through serObject + desObject (here: the
 * GPU engine) and the result is logged; the string hook round-trips its three literal strings
 * through desString.  Like the reference they only log, they assert nothing. */

/* the value of `name` in db 0 when it has the given type and encoding, else a logged NULL */
static robj *test_value(const char *name, unsigned type, unsigned enc) {
    sds key = sdsnewlen(name, strlen(name));
    dictEntry *de = dictFind(server.db[0].dict, key);
    sdsfree(key);
    if (!de) {
        serverLog(LL_NOTICE, "de is null for key = %s", name);
        return NULL;
    }
    robj *o = dictGetVal(de);
    if (o->type != type || o->encoding != enc) {
        serverLog(LL_NOTICE, "val type or encoding not correct! type = %u, encoding = %u", o->type, o->encoding);
        return NULL;
    }
    return o;
}

static robj *test_round_trip(robj *o) {
    sds blob = serObject(o);
    robj *back = desObject(blob, sdslen(blob));
    sdsfree(blob);
    return back;
}

static void test_log_quicklist(quicklist *ql) {
    quicklistIter *it = quicklistGetIterator(ql, AL_START_HEAD);
    quicklistEntry e;
    for (int i = 0; quicklistNext(it, &e); i++) {
        if (e.value) serverLog(LL_NOTICE, "index = %d, entry sz = %u, entry val = %.*s", i, e.sz, (int)e.sz, e.value);
        else serverLog(LL_NOTICE, "index = %d, entry long value = %lld", i, e.longval);
    }
    quicklistReleaseIterator(it);
}

void _test_ser_des_string(void) {                                             /* :829-901 */
    serverLog(LL_NOTICE, "_test_ser_des_string");
    static const char raw60[] = "aadfcrghsdgggggggggggadbAFWEdsar4dadsrd423FASFASXASDFASR3ADFASDFASFASR34RFADSFSADFSAFXEEdsdec";
    robj *src[3] = {createStringObjectFromLongLongForValue(134123), createEmbeddedStringObject("abc", 3),
                    createRawStringObject(raw60, 60)};
    for (int k = 0; k < 3; k++) {
        sds blob = serObject(src[k]);
        const size_t len = sdslen(blob);
        char *copy = zmalloc(len);   /* desString borrows a caller buffer, as rock.c's zmalloc'd read */
        memcpy(copy, blob, len);
        robj *d = desString(copy, len, src[k]->lru);
        serverAssert(d->refcount == 1);
        const char *what = NULL;
        if (src[k]->type != d->type) what = "type";
        else if (src[k]->encoding != d->encoding) what = "encoding";
        else if (src[k]->encoding == OBJ_ENCODING_INT) { if (src[k]->ptr != d->ptr) what = "long val"; }
        else if (sdslen(src[k]->ptr) != sdslen(d->ptr)) what = "sds len";
        else if (memcmp(src[k]->ptr, d->ptr, sdslen(d->ptr))) what = "memcmp";
        if (what) serverLog(LL_NOTICE, "%d %s!", k + 1, what);
        else serverLog(LL_NOTICE, "%d round trip ok, blob len = %zu", k + 1, len);
        decrRefCount(d);
        zfree(copy);
        sdsfree(blob);
        decrRefCount(src[k]);
    }
}

void _test_ser_des_list(void) {                                               /* :792-827 */
    serverLog(LL_NOTICE, "_test_ser_des_list");
    robj *o = test_value("abc", OBJ_LIST, OBJ_ENCODING_QUICKLIST);
    if (!o) return;
    test_log_quicklist(o->ptr);
    robj *list = createQuicklistObject();
    quicklistSetOptions(list->ptr, server.list_max_ziplist_size, server.list_compress_depth);
    sds xxx = sdsnewlen("xxx", 3), num = sdsfromlonglong(-1234567);
    quicklistPushTail(list->ptr, xxx, sdslen(xxx));
    quicklistPushTail(list->ptr, num, sdslen(num));
    sdsfree(xxx);
    sdsfree(num);
    test_log_quicklist(list->ptr);
    robj *back = test_round_trip(list);
    test_log_quicklist(back->ptr);
    decrRefCount(back);
    decrRefCount(list);
}

void _test_ser_des_set(void) {                                                /* :741-773 (HT) */
    robj *o = test_value("def", OBJ_SET, OBJ_ENCODING_HT);
    if (!o) return;
    robj *back = test_round_trip(o);
    dictIterator *di = dictGetIterator(back->ptr);
    dictEntry *de;
    while ((de = dictNext(di)))
        serverLog(LL_NOTICE, "set ht, key = %s, val is %s", (char *)dictGetKey(de), dictGetVal(de) ? "not null" : "null");
    dictReleaseIterator(di);
    decrRefCount(back);
}

void _test_ser_des_hash(void) {                                               /* :694-718 (HT) */
    robj *o = test_value("abc", OBJ_HASH, OBJ_ENCODING_HT);
    if (!o) return;
    robj *back = test_round_trip(o);
    serverLog(LL_NOTICE, "des encoding = %s", back->encoding == OBJ_ENCODING_HT ? "ht" : "not ht!!!");
    if (back->encoding == OBJ_ENCODING_HT) {
        dictIterator *di = dictGetIterator(back->ptr);
        dictEntry *de;
        for (int no = 0; (de = dictNext(di)); no++)
            serverLog(LL_NOTICE, "no = %d, field = %s, val = %s", no, (char *)dictGetKey(de), (char *)dictGetVal(de));
        dictReleaseIterator(di);
    }
    decrRefCount(back);
}

void _test_ser_des_zset(void) {                                               /* :647-671 (skiplist) */
    robj *o = test_value("abc", OBJ_ZSET, OBJ_ENCODING_SKIPLIST);
    if (!o) return;
    robj *back = test_round_trip(o);
    serverLog(LL_NOTICE, "des encoding = %s", back->encoding == OBJ_ENCODING_SKIPLIST ? "skiplist" : "not skiplist!!!");
    if (back->encoding == OBJ_ENCODING_SKIPLIST) {
        zset *zs = back->ptr;
        serverAssert(zs->zsl->length == dictSize(zs->dict));
        int i = 0;
        for (zskiplistNode *zn = zs->zsl->tail; zn; zn = zn->backward, i++)   /* tail -> head */
            serverLog(LL_NOTICE, "zset skiplist i = %d, key = %s, score = %lf", i, zn->ele, zn->score);
    }
    decrRefCount(back);
}
