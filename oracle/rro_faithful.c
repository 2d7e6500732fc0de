/*
 * rro_faithful.c — reference-faithful CPU restatement of serObject/desObject
 * (TEST INFRASTRUCTURE: bench.py cpu_baseline "faithful" leg and tests only).
 *
 * Restates the work the reference does per value on its single main / rock thread, with the
 * same data structures and allocation pattern (SURVEY.md §3, §8d "CPU baseline" mode 1):
 *   desObject  rock_serdes.c:538  -> robj per value (object.c:41-171)
 *     String   createRawStringObject / createEmbeddedStringObject / INT in ptr      :133-158
 *     List     quicklist of <=8 KiB ziplists, quicklistPushTail + zipTryEncoding      :191-214
 *              (quicklist.c:420-520, ziplist.c:480, list-max-ziplist-size -2)
 *     Set      intset zrealloc+memcpy / dict of sds (dictExpand, sdsnewlen, dictAdd)   :248-311
 *     Hash     ziplist zmalloc+memcpy / dict sds->sds                                 :349-414
 *     ZSet     ziplist zmalloc+memcpy / skiplist zslInsert + dictAdd                  :448-508
 *   serObject  rock_serdes.c:512  -> sds with sdsMakeRoomFor growth (sds.c:204-247)
 *     List ints re-rendered by sdsfromlonglong (malloc/free per integer)             :177-181
 *     HT types walked in dict bucket order (siphash-1-2 keyed, dict.c:562)
 * HT blobs therefore come back as a permutation (SURVEY.md §8c HT parity note); every other
 * type round-trips byte for byte.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "rr_oracle.h"

/* ------------------------------------------------------------------ sds (sds.h type 64) */
typedef struct { uint64_t len, alloc; } sdshdr;
typedef char *sds;
#define SDSH(s) ((sdshdr *)((s) - sizeof(sdshdr)))
static sds sdsnewlen(const void *init, uint64_t len) {
    sdshdr *h = (sdshdr *)malloc(sizeof(sdshdr) + len + 1);
    h->len = len; h->alloc = len;
    char *s = (char *)(h + 1);
    if (len && init) memcpy(s, init, len);
    s[len] = 0;
    return s;
}
static void sdsfree(sds s) { if (s) free(SDSH(s)); }
static uint64_t sdslen(const sds s) { return SDSH(s)->len; }
/* sds.c:204-247 sdsMakeRoomFor: double below 1 MiB, then +1 MiB */
static sds sdscatlen(sds s, const void *t, uint64_t len) {
    sdshdr *h = SDSH(s);
    if (h->alloc - h->len < len) {
        uint64_t newlen = h->len + len;
        if (newlen < 1024 * 1024) newlen *= 2; else newlen += 1024 * 1024;
        h = (sdshdr *)realloc(h, sizeof(sdshdr) + newlen + 1);
        h->alloc = newlen;
        s = (char *)(h + 1);
    }
    memcpy(s + h->len, t, len);
    h->len += len;
    s[h->len] = 0;
    return s;
}
static sds sdsfromlonglong(long long v) { char buf[24]; int l = rro_ll2str(buf, v); return sdsnewlen(buf, (uint64_t)l); }

/* ------------------------------------------------------------------ siphash-1-2 (siphash.c) */
static uint8_t g_seed[16] = {7, 1, 3, 9, 11, 2, 5, 8, 13, 4, 6, 10, 12, 14, 15, 0};
#define ROTL(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
#define SIPROUND do { v0 += v1; v1 = ROTL(v1, 13); v1 ^= v0; v0 = ROTL(v0, 32); v2 += v3; v3 = ROTL(v3, 16); \
        v3 ^= v2; v0 += v3; v3 = ROTL(v3, 21); v3 ^= v0; v2 += v1; v1 = ROTL(v1, 17); v1 ^= v2; v2 = ROTL(v2, 32); } while (0)
static uint64_t siphash(const uint8_t *in, uint64_t inlen) {
    uint64_t k0, k1, v0, v1, v2, v3, b = inlen << 56, m;
    memcpy(&k0, g_seed, 8); memcpy(&k1, g_seed + 8, 8);
    v0 = 0x736f6d6570736575ULL ^ k0; v1 = 0x646f72616e646f6dULL ^ k1;
    v2 = 0x6c7967656e657261ULL ^ k0; v3 = 0x7465646279746573ULL ^ k1;
    const uint8_t *end = in + inlen - (inlen % 8);
    for (; in != end; in += 8) { memcpy(&m, in, 8); v3 ^= m; SIPROUND; v0 ^= m; }
    switch (inlen & 7) {
    case 7: b |= ((uint64_t)in[6]) << 48; /* fallthrough */
    case 6: b |= ((uint64_t)in[5]) << 40; /* fallthrough */
    case 5: b |= ((uint64_t)in[4]) << 32; /* fallthrough */
    case 4: b |= ((uint64_t)in[3]) << 24; /* fallthrough */
    case 3: b |= ((uint64_t)in[2]) << 16; /* fallthrough */
    case 2: b |= ((uint64_t)in[1]) << 8;  /* fallthrough */
    case 1: b |= ((uint64_t)in[0]); break;
    case 0: break;
    }
    v3 ^= b; SIPROUND; v0 ^= b; v2 ^= 0xff; SIPROUND; SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

/* ------------------------------------------------------------------ dict (dict.c, no rehash step) */
typedef struct dictEntry { sds key; void *val; struct dictEntry *next; } dictEntry;
typedef struct { dictEntry **table; uint64_t size, used; } dict;
static dict *dictCreate(void) { dict *d = (dict *)calloc(1, sizeof(dict)); return d; }
static void dictExpand(dict *d, uint64_t n) {   /* dict.c:147, power of two >= n */
    uint64_t sz = 4;
    while (sz < n) sz <<= 1;
    dictEntry **nt = (dictEntry **)calloc(sz, sizeof(dictEntry *));
    for (uint64_t i = 0; i < d->size; i++)
        for (dictEntry *e = d->table[i], *nx; e; e = nx) {
            nx = e->next;
            uint64_t h = siphash((uint8_t *)e->key, sdslen(e->key)) & (sz - 1);
            e->next = nt[h]; nt[h] = e;
        }
    free(d->table);
    d->table = nt; d->size = sz;
}
static int dictAdd(dict *d, sds key, void *val) {   /* dict.c:265: DICT_ERR on duplicates */
    if (d->size == 0) dictExpand(d, 4);
    if (d->used >= d->size) dictExpand(d, d->used * 2);
    uint64_t h = siphash((uint8_t *)key, sdslen(key)) & (d->size - 1);
    for (dictEntry *e = d->table[h]; e; e = e->next)
        if (sdslen(e->key) == sdslen(key) && !memcmp(e->key, key, sdslen(key))) return 1;
    dictEntry *e = (dictEntry *)malloc(sizeof *e);
    e->key = key; e->val = val; e->next = d->table[h]; d->table[h] = e;
    d->used++;
    return 0;
}
static void dictRelease(dict *d, int free_vals) {
    for (uint64_t i = 0; i < d->size; i++)
        for (dictEntry *e = d->table[i], *nx; e; e = nx) {
            nx = e->next; sdsfree(e->key);
            if (free_vals) sdsfree((sds)e->val);
            free(e);
        }
    free(d->table); free(d);
}

/* ------------------------------------------------------------------ skiplist (t_zset.c:132) */
#define ZSKIPLIST_MAXLEVEL 32
typedef struct zskiplistNode {
    sds ele; double score; struct zskiplistNode *backward;
    struct { struct zskiplistNode *forward; unsigned long span; } level[];
} zskiplistNode;
typedef struct { zskiplistNode *header, *tail; unsigned long length; int level; } zskiplist;
typedef struct { dict *dict; zskiplist *zsl; } zset;
static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static int zslRandomLevel(void) {   /* p = 0.25 */
    int level = 1;
    for (;;) {
        g_rng ^= g_rng << 13; g_rng ^= g_rng >> 7; g_rng ^= g_rng << 17;
        if ((g_rng & 0xFFFF) < (0xFFFF >> 2) && level < ZSKIPLIST_MAXLEVEL) level++; else break;
    }
    return level;
}
static zskiplistNode *zslCreateNode(int level, double score, sds ele) {
    zskiplistNode *zn = (zskiplistNode *)malloc(sizeof(*zn) + (size_t)level * sizeof(zn->level[0]));
    zn->score = score; zn->ele = ele;
    return zn;
}
static zskiplist *zslCreate(void) {
    zskiplist *zsl = (zskiplist *)malloc(sizeof *zsl);
    zsl->level = 1; zsl->length = 0;
    zsl->header = zslCreateNode(ZSKIPLIST_MAXLEVEL, 0, NULL);
    for (int j = 0; j < ZSKIPLIST_MAXLEVEL; j++) { zsl->header->level[j].forward = NULL; zsl->header->level[j].span = 0; }
    zsl->header->backward = NULL; zsl->tail = NULL;
    return zsl;
}
static int sdscmp(const sds a, const sds b) {
    uint64_t l1 = sdslen(a), l2 = sdslen(b), m = l1 < l2 ? l1 : l2;
    int c = memcmp(a, b, m);
    if (c) return c;
    return l1 < l2 ? -1 : l1 > l2;
}
/* (score, ele) of node x sorts before (score, ele): zslInsert's walk predicate */
static int node_before(const zskiplistNode *x, double score, const sds ele) {
    return x->score < score || (x->score == score && sdscmp(x->ele, ele) < 0);
}
/* zslInsert (t_zset.c:132-180) restated: on every level find the last node before the new key
 * (and how many level-0 nodes precede it), draw the node's height, splice it in on each of its
 * levels with the spans split, then fix the backward link.  A NaN score is the assert at
 * t_zset.c:137: the caller rejects it before calling. */
static zskiplistNode *zslInsert(zskiplist *sl, double score, sds ele) {
    zskiplistNode *prev[ZSKIPLIST_MAXLEVEL], *cur = sl->header;
    unsigned long pos[ZSKIPLIST_MAXLEVEL], walked = 0;
    for (int lv = sl->level - 1; lv >= 0; lv--) {
        for (zskiplistNode *nx; (nx = cur->level[lv].forward) != NULL && node_before(nx, score, ele); cur = nx)
            walked += cur->level[lv].span;
        prev[lv] = cur;
        pos[lv] = walked;
    }
    const int h = zslRandomLevel();
    for (int lv = sl->level; lv < h; lv++) {
        prev[lv] = sl->header;
        pos[lv] = 0;
        sl->header->level[lv].span = sl->length;
    }
    if (h > sl->level) sl->level = h;
    zskiplistNode *node = zslCreateNode(h, score, ele);
    for (int lv = 0; lv < h; lv++) {
        const unsigned long gap = pos[0] - pos[lv];
        node->level[lv].forward = prev[lv]->level[lv].forward;
        prev[lv]->level[lv].forward = node;
        node->level[lv].span = prev[lv]->level[lv].span - gap;
        prev[lv]->level[lv].span = gap + 1;
    }
    for (int lv = h; lv < sl->level; lv++) prev[lv]->level[lv].span++;
    node->backward = prev[0] == sl->header ? NULL : prev[0];
    if (node->level[0].forward) node->level[0].forward->backward = node;
    else sl->tail = node;
    sl->length++;
    return node;
}
static void zslFree(zskiplist *zsl) {
    zskiplistNode *node = zsl->header->level[0].forward, *next;
    free(zsl->header);
    while (node) { next = node->level[0].forward; free(node); node = next; }   /* ele owned by dict */
    free(zsl);
}

/* ------------------------------------------------------------------ quicklist of ziplists */
typedef struct qlnode { struct qlnode *next; uint8_t *zl; uint32_t sz, count; } qlnode;
typedef struct { qlnode *head, *tail; uint64_t count; } quicklist;
#define QL_NODE_MAX 8192   /* list-max-ziplist-size -2 (config.c:2212, quicklist.c:47) */
static uint32_t zl_entry_size(uint32_t prev_raw, const uint8_t *s, uint32_t len, long long *iv, int *isint) {
    uint32_t sz = prev_raw < 254 ? 1 : 5;
    *isint = rro_zip_try_encoding(s, len, iv);
    if (*isint) {
        long long v = *iv;
        if (v >= 0 && v <= 12) sz += 1;
        else if (v >= -128 && v <= 127) sz += 2;
        else if (v >= -32768 && v <= 32767) sz += 3;
        else if (v >= -8388608 && v <= 8388607) sz += 4;
        else if (v >= INT32_MIN && v <= INT32_MAX) sz += 5;
        else sz += 9;
    } else sz += (len <= 0x3F ? 1 : len <= 0x3FFF ? 2 : 5) + len;
    return sz;
}
/* ziplistPush at tail: zrealloc + write entry (ziplist.c:743-839) */
static void zl_push(qlnode *n, uint32_t *prev_raw, const uint8_t *s, uint32_t len) {
    long long iv; int isint;
    uint32_t es = zl_entry_size(*prev_raw, s, len, &iv, &isint);
    n->zl = (uint8_t *)realloc(n->zl, n->sz + es);
    uint8_t *p = n->zl + n->sz - 1;   /* overwrite the end byte */
    uint8_t *e = p;
    if (*prev_raw < 254) *p++ = (uint8_t)*prev_raw; else { *p++ = 0xFE; memcpy(p, prev_raw, 4); p += 4; }
    if (isint) {
        long long v = iv;
        if (v >= 0 && v <= 12) *p++ = (uint8_t)(0xF1 + v);
        else if (v >= -128 && v <= 127) { *p++ = 0xFE; *p++ = (uint8_t)v; }
        else if (v >= -32768 && v <= 32767) { *p++ = 0xC0; int16_t x = (int16_t)v; memcpy(p, &x, 2); p += 2; }
        else if (v >= -8388608 && v <= 8388607) { *p++ = 0xF0; int32_t x = (int32_t)v; memcpy(p, &x, 3); p += 3; }
        else if (v >= INT32_MIN && v <= INT32_MAX) { *p++ = 0xD0; int32_t x = (int32_t)v; memcpy(p, &x, 4); p += 4; }
        else { *p++ = 0xE0; memcpy(p, &v, 8); p += 8; }
    } else {
        if (len <= 0x3F) *p++ = (uint8_t)len;
        else if (len <= 0x3FFF) { *p++ = (uint8_t)(0x40 | (len >> 8)); *p++ = (uint8_t)len; }
        else { *p++ = 0x80; *p++ = (uint8_t)(len >> 24); *p++ = (uint8_t)(len >> 16); *p++ = (uint8_t)(len >> 8); *p++ = (uint8_t)len; }
        memcpy(p, s, len); p += len;
    }
    *p = 0xFF;
    uint32_t tail = (uint32_t)(e - n->zl);
    n->sz += es;
    memcpy(n->zl, &n->sz, 4); memcpy(n->zl + 4, &tail, 4);
    n->count++;
    uint16_t c16 = n->count < 0xFFFF ? (uint16_t)n->count : 0xFFFF;
    memcpy(n->zl + 8, &c16, 2);
    *prev_raw = es;
}
typedef struct { qlnode *node; uint32_t prev_raw; } qlcursor;
static void qlPushTail(quicklist *ql, qlcursor *cur, const uint8_t *s, uint32_t len) {
    /* _quicklistNodeAllowInsert quicklist.c:420: new node when the ziplist would pass 8 KiB */
    if (!ql->tail || ql->tail->sz + len + 11 > QL_NODE_MAX) {
        qlnode *n = (qlnode *)calloc(1, sizeof *n);
        n->zl = (uint8_t *)malloc(11);
        uint32_t L = 11, t = 10; uint16_t c = 0;
        memcpy(n->zl, &L, 4); memcpy(n->zl + 4, &t, 4); memcpy(n->zl + 8, &c, 2); n->zl[10] = 0xFF;
        n->sz = 11;
        if (ql->tail) ql->tail->next = n; else ql->head = n;
        ql->tail = n;
        cur->node = n; cur->prev_raw = 0;
    }
    zl_push(ql->tail, &cur->prev_raw, s, len);
    ql->count++;
}

/* ------------------------------------------------------------------ robj */
enum { OBJ_STRING, OBJ_LIST, OBJ_SET, OBJ_ZSET, OBJ_HASH };
enum { ENC_RAW = 0, ENC_INT = 1, ENC_HT = 2, ENC_ZIPLIST = 5, ENC_INTSET = 6, ENC_SKIPLIST = 7, ENC_EMBSTR = 8, ENC_QUICKLIST = 9 };
typedef struct robj { unsigned type : 4, encoding : 4, lru : 24; int refcount; void *ptr; } robj;
static robj *createObject(int type, void *ptr) {
    robj *o = (robj *)malloc(sizeof *o);
    o->type = (unsigned)type; o->encoding = ENC_RAW; o->ptr = ptr; o->refcount = 1; o->lru = 0;
    return o;
}
static robj *createEmbeddedStringObject(const uint8_t *s, uint64_t len) {   /* object.c:84 */
    robj *o = (robj *)malloc(sizeof(robj) + sizeof(sdshdr) + len + 1);
    sdshdr *h = (sdshdr *)(o + 1);
    h->len = len; h->alloc = len;
    char *p = (char *)(h + 1);
    memcpy(p, s, len); p[len] = 0;
    o->type = OBJ_STRING; o->encoding = ENC_EMBSTR; o->ptr = p; o->refcount = 1;
    return o;
}

struct rro_store { robj **objs; uint64_t n; };

static inline uint32_t L32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t L64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

static robj *desObject(const uint8_t *b, uint64_t len) {
    if (len < 5) return NULL;
    uint32_t lru = L32(b + 1);
    const uint8_t *s = b + 5;
    uint64_t rem = len - 5;
    robj *o = NULL;
    switch (b[0]) {
    case RR_TYPE_STRING: {
        if (rem < 1) return NULL;
        uint8_t enc = s[0]; s++; rem--;
        if (enc == RR_ENC_INT) { if (rem != 8) return NULL; o = createObject(OBJ_STRING, (void *)(intptr_t)L64(s)); o->encoding = ENC_INT; }
        else if (enc == RR_ENC_RAW) { o = createObject(OBJ_STRING, sdsnewlen(s, rem)); }
        else if (enc == RR_ENC_EMBSTR) { if (rem > 44) return NULL; o = createEmbeddedStringObject(s, rem); }
        else return NULL;
        break;
    }
    case RR_TYPE_LIST_QUICKLIST: {
        quicklist *ql = (quicklist *)calloc(1, sizeof *ql);
        qlcursor cur = {0};
        while (rem) {
            if (rem < 4) return NULL;
            uint32_t l = L32(s); s += 4; rem -= 4;
            if (l > rem) return NULL;
            qlPushTail(ql, &cur, s, l);
            s += l; rem -= l;
        }
        o = createObject(OBJ_LIST, ql); o->encoding = ENC_QUICKLIST;
        break;
    }
    case RR_TYPE_SET_INTSET: {
        if (rem < 8) return NULL;
        uint32_t w = L32(s), cnt = L32(s + 4);
        uint32_t content = w * cnt;                               /* u32 product, rock_serdes.c:268 */
        if (rem - 8 != (uint64_t)content) return NULL;            /* :274 */
        uint8_t *is = (uint8_t *)malloc(8);                     /* createIntsetObject */
        is = (uint8_t *)realloc(is, 8 + (size_t)content);       /* zrealloc */
        memcpy(is, s, 8 + (size_t)content);
        o = createObject(OBJ_SET, is); o->encoding = ENC_INTSET;
        break;
    }
    case RR_TYPE_SET_HT:
    case RR_TYPE_HASH_HT: {
        if (rem < 8) return NULL;
        uint64_t cnt = L64(s); s += 8; rem -= 8;
        dict *d = dictCreate();
        if (cnt > 4) dictExpand(d, cnt);
        int hash = b[0] == RR_TYPE_HASH_HT;
        while (rem) {
            if (rem < 8) return NULL;
            uint64_t l = L64(s); s += 8; rem -= 8;
            if (l > rem) return NULL;
            sds k = sdsnewlen(s, l); s += l; rem -= l;
            sds v = NULL;
            if (hash) {
                if (rem < 8) return NULL;
                uint64_t vl = L64(s); s += 8; rem -= 8;
                if (vl > rem) return NULL;
                v = sdsnewlen(s, vl); s += vl; rem -= vl;
            }
            if (dictAdd(d, k, v)) {
                sdsfree(k); sdsfree(v);
                if (hash) return NULL;   /* serverAssert(ret == DICT_OK), rock_serdes.c:399-400 */
            }                            /* a set ignores the duplicate (rock_serdes.c:297) */
            cnt--;
        }
        if (cnt) return NULL;
        o = createObject(hash ? OBJ_HASH : OBJ_SET, d); o->encoding = ENC_HT;
        break;
    }
    case RR_TYPE_HASH_ZIPLIST:
    case RR_TYPE_ZSET_ZIPLIST: {
        if (rem < 8) return NULL;
        uint64_t L = L64(s); s += 8; rem -= 8;
        if (rem != L) return NULL;
        uint8_t *zl = (uint8_t *)malloc(L);
        memcpy(zl, s, L);
        o = createObject(b[0] == RR_TYPE_HASH_ZIPLIST ? OBJ_HASH : OBJ_ZSET, zl); o->encoding = ENC_ZIPLIST;
        break;
    }
    case RR_TYPE_ZSET_SKIPLIST: {
        if (rem < 8) return NULL;
        uint64_t cnt = L64(s); s += 8; rem -= 8;
        zset *zs = (zset *)malloc(sizeof *zs);
        zs->dict = dictCreate(); zs->zsl = zslCreate();
        if (cnt > 4) dictExpand(zs->dict, cnt);
        while (cnt--) {
            if (rem < 8) return NULL;
            uint64_t l = L64(s); s += 8; rem -= 8;
            if (l > rem) return NULL;
            sds e = sdsnewlen(s, l); s += l; rem -= l;
            if (rem < 8) return NULL;
            double sc; memcpy(&sc, s, 8); s += 8; rem -= 8;
            if (isnan(sc)) return NULL;  /* zslInsert's serverAssert(!isnan(score)), t_zset.c:137 */
            zskiplistNode *zn = zslInsert(zs->zsl, sc, e);
            dictAdd(zs->dict, e, &zn->score);
        }
        if (rem) return NULL;
        o = createObject(OBJ_ZSET, zs); o->encoding = ENC_SKIPLIST;
        break;
    }
    default:
        return NULL;
    }
    o->lru = lru & RR_LRU_MASK;
    return o;
}

static sds serObject(robj *o) {
    uint8_t t;
    switch (o->type) {
    case OBJ_STRING: t = RR_TYPE_STRING; break;
    case OBJ_LIST: t = RR_TYPE_LIST_QUICKLIST; break;
    case OBJ_SET: t = o->encoding == ENC_INTSET ? RR_TYPE_SET_INTSET : RR_TYPE_SET_HT; break;
    case OBJ_ZSET: t = o->encoding == ENC_ZIPLIST ? RR_TYPE_ZSET_ZIPLIST : RR_TYPE_ZSET_SKIPLIST; break;
    default: t = o->encoding == ENC_ZIPLIST ? RR_TYPE_HASH_ZIPLIST : RR_TYPE_HASH_HT; break;
    }
    sds dst = sdsnewlen(&t, 1);
    uint32_t lru = o->lru;
    dst = sdscatlen(dst, &lru, 4);
    switch (t) {
    case RR_TYPE_STRING: {
        uint8_t enc = (uint8_t)o->encoding;
        dst = sdscatlen(dst, &enc, 1);
        if (enc == ENC_INT) { long long v = (long long)(intptr_t)o->ptr; dst = sdscatlen(dst, &v, 8); }
        else dst = sdscatlen(dst, o->ptr, sdslen((sds)o->ptr));
        break;
    }
    case RR_TYPE_LIST_QUICKLIST: {   /* quicklistNext over every node's ziplist */
        quicklist *ql = (quicklist *)o->ptr;
        for (qlnode *n = ql->head; n; n = n->next) {
            uint64_t cnt;
            rr_elem *tmp = (rr_elem *)malloc(sizeof(rr_elem) * (n->count ? n->count : 1));
            rro_parse_ziplist(n->zl, n->sz, 0, tmp, n->count, &cnt);
            for (uint64_t i = 0; i < cnt; i++) {
                if (tmp[i].kind == RR_K_STR) {
                    uint32_t l = tmp[i].len;
                    dst = sdscatlen(dst, &l, 4);
                    dst = sdscatlen(dst, n->zl + tmp[i].data, l);
                } else {
                    sds str = sdsfromlonglong((long long)tmp[i].data);
                    uint32_t l = (uint32_t)sdslen(str);
                    dst = sdscatlen(dst, &l, 4);
                    dst = sdscatlen(dst, str, l);
                    sdsfree(str);
                }
            }
            free(tmp);
        }
        break;
    }
    case RR_TYPE_SET_INTSET: {
        uint8_t *is = (uint8_t *)o->ptr;
        uint32_t w = L32(is), cnt = L32(is + 4);
        dst = sdscatlen(dst, is, 4);
        dst = sdscatlen(dst, is + 4, 4);
        dst = sdscatlen(dst, is + 8, (uint32_t)(w * cnt));       /* u32 product, rock_serdes.c:224 */
        break;
    }
    case RR_TYPE_SET_HT:
    case RR_TYPE_HASH_HT: {
        dict *d = (dict *)o->ptr;
        uint64_t cnt = d->used;
        dst = sdscatlen(dst, &cnt, 8);
        for (uint64_t i = 0; i < d->size; i++)
            for (dictEntry *e = d->table[i]; e; e = e->next) {
                uint64_t l = sdslen(e->key);
                dst = sdscatlen(dst, &l, 8);
                dst = sdscatlen(dst, e->key, l);
                if (t == RR_TYPE_HASH_HT) {
                    uint64_t vl = sdslen((sds)e->val);
                    dst = sdscatlen(dst, &vl, 8);
                    dst = sdscatlen(dst, e->val, vl);
                }
            }
        break;
    }
    case RR_TYPE_HASH_ZIPLIST:
    case RR_TYPE_ZSET_ZIPLIST: {
        uint64_t L = L32((uint8_t *)o->ptr);   /* ziplistBlobLen */
        dst = sdscatlen(dst, &L, 8);
        dst = sdscatlen(dst, o->ptr, L);
        break;
    }
    case RR_TYPE_ZSET_SKIPLIST: {
        zset *zs = (zset *)o->ptr;
        uint64_t len = zs->zsl->length;
        dst = sdscatlen(dst, &len, 8);
        for (zskiplistNode *zn = zs->zsl->tail; zn; zn = zn->backward) {
            uint64_t l = sdslen(zn->ele);
            dst = sdscatlen(dst, &l, 8);
            dst = sdscatlen(dst, zn->ele, l);
            dst = sdscatlen(dst, &zn->score, 8);
        }
        break;
    }
    }
    return dst;
}

static void decrRefCount(robj *o) {
    switch (o->type) {
    case OBJ_STRING:
        if (o->encoding == ENC_RAW) sdsfree((sds)o->ptr);
        break;
    case OBJ_LIST: {
        quicklist *ql = (quicklist *)o->ptr;
        for (qlnode *n = ql->head, *nx; n; n = nx) { nx = n->next; free(n->zl); free(n); }
        free(ql);
        break;
    }
    case OBJ_SET:
    case OBJ_HASH:
        if (o->encoding == ENC_HT) dictRelease((dict *)o->ptr, o->type == OBJ_HASH);
        else free(o->ptr);
        break;
    case OBJ_ZSET:
        if (o->encoding == ENC_SKIPLIST) {
            zset *zs = (zset *)o->ptr;
            zslFree(zs->zsl);
            dictRelease(zs->dict, 0);
            free(zs);
        } else free(o->ptr);
        break;
    }
    free(o);
}

rro_store *rro_faithful_decode(const uint8_t *data, const uint64_t *offsets, uint64_t n, uint64_t *n_bad) {
    rro_store *s = (rro_store *)malloc(sizeof *s);
    s->objs = (robj **)malloc(sizeof(robj *) * (n ? n : 1));
    s->n = n;
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; i++) {
        s->objs[i] = desObject(data + offsets[i], offsets[i + 1] - offsets[i]);
        if (!s->objs[i]) bad++;
    }
    if (n_bad) *n_bad = bad;
    return s;
}

uint64_t rro_faithful_encode(rro_store *s, uint8_t *out, uint64_t cap, uint64_t *offsets) {
    uint64_t pos = 0;
    for (uint64_t i = 0; i < s->n; i++) {
        if (offsets) offsets[i] = pos;
        if (!s->objs[i]) continue;
        sds b = serObject(s->objs[i]);
        uint64_t l = sdslen(b);
        if (out && pos + l <= cap) memcpy(out + pos, b, l);
        pos += l;
        sdsfree(b);   /* rock.c:693 */
    }
    if (offsets) offsets[s->n] = pos;
    return pos;
}

void rro_store_free(rro_store *s) {
    if (!s) return;
    for (uint64_t i = 0; i < s->n; i++) if (s->objs[i]) decrRefCount(s->objs[i]);
    free(s->objs);
    free(s);
}
