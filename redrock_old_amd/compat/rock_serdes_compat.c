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
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "server.h"

#include "rock_serdes_compat.h"

static int g_device;
static __thread rr_ctx *g_ctx;   /* one engine context per host thread (rr_serdes.h) */

void rr_compat_set_device(int device) { g_device = device; }

static rr_ctx *engine(void) {
    if (!g_ctx && rr_ctx_create(g_device, &g_ctx) != RR_API_OK)
        serverPanic("rock serdes engine: %s", rr_last_error());
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

void rr_compat_des_batch(void *const *bufs, const size_t *lens, size_t n, robj **out) {
    if (n == 0) return;
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
    uint64_t nv, ne, na, cap_e, cap_a, out_bound;
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

void rr_compat_ser_batch(robj *const *objs, size_t n, sds *out) {
    if (n == 0) return;
    flat_t f;
    memset(&f, 0, sizeof f);
    f.vals = zmalloc(sizeof(rr_value) * n);
    for (size_t i = 0; i < n; i++) flatten(&f, objs[i]);
    uint64_t *offs = zmalloc(sizeof(uint64_t) * (n + 1));
    uint8_t *data = zmalloc(f.out_bound + 16);
    rr_totals t;
    if (rr_encode_batch_host(engine(), f.vals, f.els, f.ne, f.arena, f.na, n, data, f.out_bound + 16, offs, &t) !=
        RR_API_OK)
        serverPanic("serObject: %s", rr_last_error());
    if (t.n_bad) serverPanic("serObject: %llu unencodable objects", (unsigned long long)t.n_bad);
    for (size_t i = 0; i < n; i++) out[i] = sdsnewlen(data + offs[i], offs[i + 1] - offs[i]);
    zfree(offs); zfree(data); zfree(f.vals); zfree(f.els); zfree(f.arena);
}

sds serObject(robj *o) {
    sds s = NULL;
    rr_compat_ser_batch(&o, 1, &s);
    return s;
}
