/*
 * rock_serdes_compat.c — bodies of RedRock's legacy serdes signatures (rock_serdes.h:47-55)
 * over the engine (include/rock_serdes_compat.h).
 *
 * Built inside a Redis tree: it includes the tree's server.h and uses only the Redis API the
 * reference rock_serdes.c itself uses (robj constructors, sds, dict, quicklist, intset,
 * zslInsert, zmalloc).  Abort semantics are the reference's: a blob the reference would reject
 * (any nonzero rr_value.status) ends in serverPanic.
 *
 * Routing.  RedRock's call sites are per key — desObject per rock-thread job (rock.c:468) and per
 * key in the BGSAVE child (rock.c:538), serObject per evicted key (rock.c:691) — so a call of one
 * value, and a batch form below the measured crossover, runs the engine's host codec
 * (include/rr_host.h) on the calling thread: the GPU path's exact flat form, no launch, no PCIe.
 * A batch at or above the crossover goes through the GPU entry points (rr_decode_batch_host /
 * rr_encode_batch_host).  A fork child always takes the host codec: it must not touch the HIP
 * runtime its parent initialised, and on the CPU it needs no help from the parent.  Either way
 * this file turns flat records into heap objects and back, which a GPU cannot do.
 *
 * Process exit.  Threads that call in here are not the shim's own: RedRock's rock thread
 * (rock.c:615) is never joined and loops on desObject (rock.c:552-596).  A thread inside the HIP
 * runtime while exit() tears the runtime down crashes the process, so every engine (HIP) call
 * is counted in flight; the owner's exit raises a closing flag, waits (bounded) for the count to
 * drain, and any later caller parks instead of entering the runtime.  Host-codec calls touch no
 * runtime and are never held.
 *
 * The repo's own unit tests compile this file against a minimal Redis model (tests/c/miniredis)
 * instead of a Redis tree.
 */
#ifndef RR_REDIS_TREE
#define RR_REDIS_TREE 1
#endif
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "server.h"

#include "rock_serdes_compat.h"
#include "rr_host.h"

static int g_device;
static __thread rr_ctx *g_ctx;   /* one engine context per host thread (rr_serdes.h) */

void rr_compat_set_device(int device) { g_device = device; }

/* ---------------------------------------------------------------- routing */

/* The crossovers (values per call) from which a batch form goes to the GPU, measured with
 * tests/c/bench_callpattern.c on the GPU box (profiles/r6_callpattern_cfg4.json): the robj a call
 * builds or walks cost the same on either route, and a GPU call adds a launch, the staging copies
 * and the PCIe round trip.  Serialize: the GPU route is 7-10 % faster from 16,384 values.
 * Deserialize: the host route is as fast or faster at every k measured (1 to 65,536), so it
 * never goes to the GPU by default.  RR_COMPAT_GPU_MIN_SER / RR_COMPAT_GPU_MIN_DES override them
 * (values; 0 = never). */
#define RR_COMPAT_GPU_MIN_SER_DEFAULT 16384
#define RR_COMPAT_GPU_MIN_DES_DEFAULT 0
static int g_route = RR_COMPAT_ROUTE_AUTO;
static uint64_t g_gpu_min_ser, g_gpu_min_des;
static pthread_once_t g_cfg_once = PTHREAD_ONCE_INIT;

static void read_config(void) {
    const char *s = getenv("RR_COMPAT_GPU_MIN_SER"), *d = getenv("RR_COMPAT_GPU_MIN_DES");
    g_gpu_min_ser = s ? strtoull(s, NULL, 10) : RR_COMPAT_GPU_MIN_SER_DEFAULT;
    g_gpu_min_des = d ? strtoull(d, NULL, 10) : RR_COMPAT_GPU_MIN_DES_DEFAULT;
}

void rr_compat_set_route(int route) { g_route = route; }

static pid_t g_owner;    /* the process whose threads own GPU contexts */
static int g_forked;     /* this process is a fork child of an owner (its HIP runtime is the parent's) */
static int g_as_child;   /* test hook: route this process as a fork child would */

/* (set in the child by pthread_atfork: no getpid() system call per desObject) */
static void atfork_child(void) {
    if (g_owner) g_forked = 1;
}
__attribute__((constructor)) static void compat_atfork_register(void) { pthread_atfork(NULL, NULL, atfork_child); }

static int in_child(void) { return g_as_child || g_forked; }

/* n values (encode: ser = 1) through the GPU entry points? */
static int use_gpu(size_t n, int ser) {
    if (in_child()) return g_route == RR_COMPAT_ROUTE_GPU;   /* (the engine then refuses, below) */
    if (g_route != RR_COMPAT_ROUTE_AUTO) return g_route == RR_COMPAT_ROUTE_GPU;
    pthread_once(&g_cfg_once, read_config);
    const uint64_t min = ser ? g_gpu_min_ser : g_gpu_min_des;
    return min && n >= min;
}

void rr_compat_test_as_child(int on) { g_as_child = on; }

/* ---------------------------------------------------------------- engine calls and exit */

static int g_inflight;          /* threads inside an engine (HIP) call */
static int g_closing;           /* the owner's exit has begun */
static pthread_t g_closer;      /* the thread running it (its own later calls pass) */
static __thread int t_inflight; /* this thread's share of g_inflight */
static int g_test_hold_ms, g_test_holding;

/* The process is exiting under us: this thread must never enter (or re-enter) the runtime. */
static __attribute__((noreturn)) void park(void) {
    for (;;) pause();
}

static void engine_enter(void) {
    __atomic_add_fetch(&g_inflight, 1, __ATOMIC_SEQ_CST);
    t_inflight++;
    if (__atomic_load_n(&g_closing, __ATOMIC_SEQ_CST) && !pthread_equal(pthread_self(), g_closer)) {
        t_inflight--;
        __atomic_sub_fetch(&g_inflight, 1, __ATOMIC_SEQ_CST);
        park();
    }
}

static void engine_leave(void) {
    t_inflight--;
    __atomic_sub_fetch(&g_inflight, 1, __ATOMIC_SEQ_CST);
}

/* The owner's exit: no new engine call, then the calls in flight drain (at most 10 s; a call
 * stuck longer than that is a hung device, and the exit goes on).  exit_hook registers this once
 * the runtime is up, so it runs before every exit handler the runtime registered. */
static void compat_exit(void) {
    if (g_forked) return;   /* (a fork child has no engine calls) */
    g_closer = pthread_self();
    __atomic_store_n(&g_closing, 1, __ATOMIC_SEQ_CST);
    const struct timespec ms = {0, 1000000};
    for (int i = 0; i < 10000 && __atomic_load_n(&g_inflight, __ATOMIC_SEQ_CST) > t_inflight; i++)
        nanosleep(&ms, NULL);
}

static int g_exit_hooked;
static void exit_hook(void) {
    if (!__atomic_exchange_n(&g_exit_hooked, 1, __ATOMIC_SEQ_CST)) atexit(compat_exit);
}

/* A thread's context is destroyed when the thread ends (a context per host thread), inside the
 * engine count so an exit meanwhile waits for it. */
static pthread_key_t g_ctx_key;
static pthread_once_t g_key_once = PTHREAD_ONCE_INIT;

static void ctx_at_thread_exit(void *p) {
    if (in_child()) return;   /* (not ours to destroy) */
    engine_enter();
    const int hold = __atomic_exchange_n(&g_test_hold_ms, 0, __ATOMIC_SEQ_CST);
    if (hold) {   /* test hook: a teardown still running when the process exits */
        __atomic_store_n(&g_test_holding, 1, __ATOMIC_SEQ_CST);
        const struct timespec t = {hold / 1000, (long)(hold % 1000) * 1000000};
        nanosleep(&t, NULL);
    }
    rr_ctx_destroy((rr_ctx *)p);
    g_ctx = NULL;
    engine_leave();
}

static void make_key(void) { pthread_key_create(&g_ctx_key, ctx_at_thread_exit); }

void rr_compat_test_hold_teardown(int ms) { __atomic_store_n(&g_test_hold_ms, ms, __ATOMIC_SEQ_CST); }
int rr_compat_test_holding(void) { return __atomic_load_n(&g_test_holding, __ATOMIC_SEQ_CST); }
int rr_compat_in_flight(void) { return __atomic_load_n(&g_inflight, __ATOMIC_SEQ_CST); }

/* This thread's context, inside engine_enter / engine_leave. */
static rr_ctx *engine(void) {
    if (in_child()) {
        engine_leave();
        serverPanic("rock serdes: the GPU engine cannot be used in a fork child (HIP is the parent's)");
    }
    if (!g_ctx) {
        if (rr_ctx_create(g_device, &g_ctx) != RR_API_OK) {
            engine_leave();
            serverPanic("rock serdes engine: %s", rr_last_error());
        }
        if (!g_owner) g_owner = getpid();
        exit_hook();
        pthread_once(&g_key_once, make_key);
        pthread_setspecific(g_ctx_key, g_ctx);
    }
    return g_ctx;
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
 * descriptor already says what the reference derives from the bytes (rr_format.h).  blob (may be
 * NULL) = the value's own bytes, for the copies the reference makes straight from them. */
static robj *robj_from_flat(const rr_value *v, const rr_elem *el, const uint8_t *arena, const uint8_t *blob) {
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
        if (blob) memcpy(is->contents, blob + 13, (size_t)w * n);   /* the blob's contents, as :270-273 */
        else for (uint32_t i = 0; i < n; i++) memcpy((char *)is->contents + (size_t)i * w, &el[i].data, w);
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

/* desObject on the calling thread: the host codec into a stack buffer (a value of more than 64
 * descriptors asks for its exact count and decodes again into the heap), then the robj. */
static robj *des_host(const void *buf, size_t len) {
    rr_elem local[64], *el = local;
    rr_value v;
    uint64_t need;
    const uint8_t *b = buf;
    if (len >= 13 && (b[0] == RR_TYPE_HASH_ZIPLIST || b[0] == RR_TYPE_ZSET_ZIPLIST)) {
        /* kept as its raw bytes (:356-366, :455-466): the ziplist's verdict, no entry descriptors */
        const int st = rr_host_check_value(b, len, &v);
        if (st != RR_OK) serverPanic("desObject: bad blob (%s, status %u)", status_name((unsigned)st), (unsigned)st);
        local[0].kind = RR_K_ZLRAW;
        local[0].data = 13;
        local[0].len = (uint32_t)(len - 13);
        return robj_from_flat(&v, local, b, b);
    }
    int st = rr_host_decode_value(buf, len, 0, &v, el, 64, &need);
    if (st == RR_E_CAPACITY) {
        el = zmalloc(sizeof(rr_elem) * need);
        st = rr_host_decode_value(buf, len, 0, &v, el, need, NULL);
    }
    if (st != RR_OK) {   /* the reference's serverAssert / serverPanic site */
        if (el != local) zfree(el);
        serverPanic("desObject: bad blob (%s, status %u)", status_name((unsigned)st), (unsigned)st);
    }
    robj *o = robj_from_flat(&v, el, buf, buf);
    if (el != local) zfree(el);
    return o;
}

/* n blobs through the GPU: one rr_decode_batch_host, then the robj from the records */
static void des_batch_gpu(void *const *bufs, const size_t *lens, size_t n, robj **out) {
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
    engine_enter();
    /* no arena download: it would mirror `data` byte for byte, so the descriptors index it */
    const int rc = rr_decode_batch_host(engine(), data, offs, n, vals, els, cap, NULL, &t);
    engine_leave();
    if (rc != RR_API_OK) serverPanic("desObject: %s", rr_last_error());
    for (size_t i = 0; i < n; i++) {
        if (vals[i].status != RR_OK)   /* the reference's serverAssert / serverPanic site */
            serverPanic("desObject: bad blob (%s, status %u)", status_name(vals[i].status), vals[i].status);
        out[i] = robj_from_flat(&vals[i], els + vals[i].elem_base, data, data + offs[i]);
    }
    zfree(offs); zfree(data); zfree(vals); zfree(els);
}

void rr_compat_des_batch(void *const *bufs, const size_t *lens, size_t n, robj **out) {
    if (n == 0) return;
    if (use_gpu(n, 0)) { des_batch_gpu(bufs, lens, n, out); return; }
    for (size_t i = 0; i < n; i++) out[i] = des_host(bufs[i], lens[i]);
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
        out[i] = robj_from_flat(&f.values[i], f.elems + f.values[i].elem_base, f.arena, NULL);
    }
    rr_rdb_flat_free(&f);
    zfree(dbis);
    zfree(lens);
}

robj *desObject(void *buf, size_t len) {
    if (use_gpu(1, 0)) {
        robj *o = NULL;
        des_batch_gpu(&buf, &len, 1, &o);
        return o;
    }
    return des_host(buf, len);
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
    int by_ref;   /* STR descriptors hold the payload's address (the host codec, arena NULL) */
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
    rr_elem *e = add_elem(f);
    e->kind = RR_K_STR;
    e->len = (uint32_t)len;
    f->out_bound += 8 + len;
    if (f->by_ref) {
        e->data = (uint64_t)(uintptr_t)p;
        return;
    }
    if (f->na + len > f->cap_a) {
        while (f->na + len > f->cap_a) f->cap_a = f->cap_a ? 2 * f->cap_a : 4096;
        f->arena = zrealloc(f->arena, f->cap_a);
    }
    e->data = f->na;
    if (len) memcpy(f->arena + f->na, p, len);
    f->na += len;
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
 * given back at the end of ser_batch_gpu). */
static __thread flat_t t_flat;
static __thread uint64_t *t_offs;
static __thread uint8_t *t_data;
static __thread size_t t_offs_cap, t_data_cap;

static void flat_reset(flat_t *f, size_t n, int by_ref) {
    f->nv = f->ne = f->na = f->out_bound = 0;
    f->by_ref = by_ref;
    if (n > f->cap_v) {
        f->vals = zrealloc(f->vals, sizeof(rr_value) * n);
        f->cap_v = n;
    }
}

/* serObject on the calling thread: the robj described in place (descriptors hold its strings'
 * addresses, nothing is copied), sized, and written by the host codec straight into the sds. */
static sds ser_host(robj *o) {
    if (o->type == OBJ_SET && o->encoding == OBJ_ENCODING_INTSET) {   /* :220-226: the intset's own bytes */
        const intset *is = o->ptr;
        const size_t nb = (size_t)is->encoding * is->length;
        sds s = sdsnewlen(SDS_NOINIT, 13 + nb);
        const uint32_t lru = o->lru, hdr[2] = {is->encoding, is->length};
        s[0] = RR_TYPE_SET_INTSET;
        memcpy(s + 1, &lru, 4);
        memcpy(s + 5, hdr, 8);
        memcpy(s + 13, is->contents, nb);
        return s;
    }
    flat_t *f = &t_flat;
    flat_reset(f, 1, 1);
    flatten(f, o);
    uint64_t size;
    if (rr_host_encode_size(&f->vals[0], f->els, f->ne, UINT64_MAX, &size) != RR_OK)
        serverPanic("serObject: unencodable object (type %u, encoding %u)", o->type, o->encoding);
    sds s = sdsnewlen(SDS_NOINIT, size);
    rr_host_encode_value(&f->vals[0], f->els, NULL, (uint8_t *)s);
    return s;
}

static void ser_batch_gpu(robj *const *objs, size_t n, sds *out) {
    flat_t *f = &t_flat;
    flat_reset(f, n, 0);
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
    engine_enter();
    const int rc = rr_encode_batch_host(engine(), f->vals, f->els, f->ne, f->arena, f->na, n, t_data,
                                        f->out_bound + 16, t_offs, &t);
    engine_leave();
    if (rc != RR_API_OK) serverPanic("serObject: %s", rr_last_error());
    if (t.n_bad) serverPanic("serObject: %llu unencodable objects", (unsigned long long)t.n_bad);
    for (size_t i = 0; i < n; i++) out[i] = sdsnewlen(t_data + t_offs[i], t_offs[i + 1] - t_offs[i]);
    /* the thread's buffers keep their size between calls, but not a one-off large batch's: past
     * 1 MiB and 4x this call's need, give it back */
    const size_t big = 1u << 20;
    if (t_data_cap > big && t_data_cap > 4 * (f->out_bound + 16)) { zfree(t_data); t_data = NULL; t_data_cap = 0; }
    if (f->cap_a > big && f->cap_a > 4 * f->na) { zfree(f->arena); f->arena = NULL; f->cap_a = 0; }
    if (f->cap_e * sizeof(rr_elem) > big && f->cap_e > 4 * f->ne) { zfree(f->els); f->els = NULL; f->cap_e = 0; }
    if (f->cap_v * sizeof(rr_value) > big && f->cap_v > 4 * n) { zfree(f->vals); f->vals = NULL; f->cap_v = 0; }
    if (t_offs_cap * sizeof(uint64_t) > big && t_offs_cap > 4 * (n + 1)) { zfree(t_offs); t_offs = NULL; t_offs_cap = 0; }
}

void rr_compat_ser_batch(robj *const *objs, size_t n, sds *out) {
    if (n == 0) return;
    if (use_gpu(n, 1)) { ser_batch_gpu(objs, n, out); return; }
    for (size_t i = 0; i < n; i++) out[i] = ser_host(objs[i]);
}

sds serObject(robj *o) {
    if (use_gpu(1, 1)) {
        sds s = NULL;
        ser_batch_gpu(&o, 1, &s);
        return s;
    }
    return ser_host(o);
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
