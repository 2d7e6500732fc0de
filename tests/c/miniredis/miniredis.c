/* miniredis.c — the minimal Redis model of server.h (TEST INFRASTRUCTURE, see there). */
#include "server.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---- zmalloc / sds ---- */
void *zmalloc(size_t size) { void *p = malloc(size ? size : 1); if (!p) abort(); return p; }
void *zrealloc(void *ptr, size_t size) { void *p = realloc(ptr, size ? size : 1); if (!p) abort(); return p; }
void zfree(void *ptr) { free(ptr); }

typedef struct { size_t len; } sdshdr_t;
const char *SDS_NOINIT = "SDS_NOINIT";
sds sdsnewlen(const void *init, size_t initlen) {
    sdshdr_t *h = zmalloc(sizeof *h + initlen + 1);
    h->len = initlen;
    char *s = (char *)(h + 1);
    if (init == SDS_NOINIT) init = NULL;
    if (initlen && init) memcpy(s, init, initlen);
    s[initlen] = 0;
    return s;
}
size_t sdslen(const sds s) { return ((const sdshdr_t *)s - 1)->len; }
void sdsfree(sds s) { if (s) zfree((sdshdr_t *)s - 1); }

/* ---- util.c:360-424 string2ll, :294 ll2string ---- */
static int string2ll(const char *s, size_t slen, long long *value) {
    size_t i = 0;
    int neg = 0;
    unsigned long long v;
    if (slen == 0) return 0;
    if (slen == 1 && s[0] == '0') { *value = 0; return 1; }
    if (s[0] == '-') { neg = 1; if (++i == slen) return 0; }
    if (s[i] < '1' || s[i] > '9') return 0;
    v = (unsigned long long)(s[i++] - '0');
    for (; i < slen; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        if (v > ~0ULL / 10) return 0;
        v *= 10;
        if (v > ~0ULL - (unsigned long long)(s[i] - '0')) return 0;
        v += (unsigned long long)(s[i] - '0');
    }
    if (neg) { if (v > (1ULL << 63)) return 0; *value = (long long)(0ULL - v); }
    else { if (v > 0x7FFFFFFFFFFFFFFFULL) return 0; *value = (long long)v; }
    return 1;
}
int ll2string(char *s, size_t len, long long value) {
    char buf[32];
    unsigned long long v = value < 0 ? 0ULL - (unsigned long long)value : (unsigned long long)value;
    int n = 0;
    do { buf[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    if (value < 0) buf[n++] = '-';
    if ((size_t)n >= len) return 0;
    for (int i = 0; i < n; i++) s[i] = buf[n - 1 - i];
    s[n] = 0;
    return n;
}

/* ---- dict (insertion-ordered; keys compared as sds) ---- */
dictType setDictType, hashDictType, zsetDictType;
dict *dictCreate(dictType *type, void *privDataPtr) {
    (void)privDataPtr;
    dict *d = zmalloc(sizeof *d);
    d->ents = NULL; d->used = d->cap = 0; d->type = type;
    return d;
}
int dictExpand(dict *d, unsigned long size) {
    if (size > d->cap) { d->ents = zrealloc(d->ents, size * sizeof(dictEntry)); d->cap = size; }
    return DICT_OK;
}
int dictAdd(dict *d, void *key, void *val) {
    for (unsigned long i = 0; i < d->used; i++)
        if (sdslen(d->ents[i].key) == sdslen(key) && !memcmp(d->ents[i].key, key, sdslen(key))) return DICT_ERR;
    if (d->used == d->cap) dictExpand(d, d->cap ? 2 * d->cap : 4);
    d->ents[d->used].key = key;
    d->ents[d->used].v.val = val;
    d->used++;
    return DICT_OK;
}
dictEntry *dictFind(dict *d, const void *key) {
    for (unsigned long i = 0; i < d->used; i++)
        if (sdslen(d->ents[i].key) == sdslen((const sds)key) && !memcmp(d->ents[i].key, key, sdslen((const sds)key)))
            return &d->ents[i];
    return NULL;
}
dictIterator *dictGetIterator(dict *d) { dictIterator *it = zmalloc(sizeof *it); it->d = d; it->i = 0; return it; }
dictEntry *dictNext(dictIterator *it) { return it->i < it->d->used ? &it->d->ents[it->i++] : NULL; }
void dictReleaseIterator(dictIterator *it) { zfree(it); }

/* ---- quicklist: one array; pushes re-try integer encoding (zipTryEncoding, ziplist.c:480) ---- */
typedef struct { int isint; long long v; unsigned char *s; size_t sz; } qlent_t;
struct quicklist { qlent_t *e; size_t n, cap; };
struct quicklistIter { const quicklist *ql; size_t i; };
void quicklistSetOptions(quicklist *ql, int fill, int depth) { (void)ql; (void)fill; (void)depth; }
int quicklistPushTail(quicklist *ql, void *value, size_t sz) {
    if (ql->n == ql->cap) { ql->cap = ql->cap ? 2 * ql->cap : 8; ql->e = zrealloc(ql->e, ql->cap * sizeof(qlent_t)); }
    qlent_t *e = &ql->e[ql->n++];
    long long v;
    if (sz > 0 && sz < 32 && string2ll(value, sz, &v)) { e->isint = 1; e->v = v; e->s = NULL; e->sz = 0; }
    else { e->isint = 0; e->s = zmalloc(sz ? sz : 1); memcpy(e->s, value, sz); e->sz = sz; }
    return 0;
}
quicklistIter *quicklistGetIterator(const quicklist *ql, int direction) {
    (void)direction;
    quicklistIter *it = zmalloc(sizeof *it); it->ql = ql; it->i = 0; return it;
}
int quicklistNext(quicklistIter *it, quicklistEntry *entry) {
    if (it->i >= it->ql->n) return 0;
    const qlent_t *e = &it->ql->e[it->i++];
    memset(entry, 0, sizeof *entry);
    if (e->isint) entry->longval = e->v;
    else { entry->value = e->s ? e->s : (unsigned char *)""; entry->sz = (unsigned int)e->sz; }
    return 1;
}
void quicklistReleaseIterator(quicklistIter *it) { zfree(it); }

/* ---- sorted set: ascending (score, member), a new node before equal ones (t_zset.c:132) ---- */
static int sdscmp(const sds a, const sds b) {
    size_t la = sdslen(a), lb = sdslen(b), m = la < lb ? la : lb;
    int c = m ? memcmp(a, b, m) : 0;
    if (c) return c;
    return la < lb ? -1 : la > lb;
}
zskiplistNode *zslInsert(zskiplist *zsl, double score, sds ele) {
    zskiplistNode *x = zmalloc(sizeof *x), *prev = NULL, *cur = zsl->header;
    x->ele = ele; x->score = score;
    while (cur && (cur->score < score || (cur->score == score && sdscmp(cur->ele, ele) < 0))) { prev = cur; cur = cur->forward; }
    x->backward = prev; x->forward = cur;
    if (prev) prev->forward = x; else zsl->header = x;
    if (cur) cur->backward = x; else zsl->tail = x;
    zsl->length++;
    return x;
}

size_t ziplistBlobLen(unsigned char *zl) { uint32_t l; memcpy(&l, zl, 4); return l; }

/* ---- objects ---- */
robj *createObject(int type, void *ptr) {
    robj *o = zmalloc(sizeof *o);
    o->type = (unsigned)type; o->encoding = OBJ_ENCODING_RAW; o->ptr = ptr; o->refcount = 1; o->lru = 0;
    return o;
}
robj *createRawStringObject(const char *ptr, size_t len) { return createObject(OBJ_STRING, sdsnewlen(ptr, len)); }
robj *createEmbeddedStringObject(const char *ptr, size_t len) {   /* object.c:84: robj + sds, one allocation */
    robj *o = zmalloc(sizeof(robj) + sizeof(sdshdr_t) + len + 1);
    sdshdr_t *h = (sdshdr_t *)(o + 1);
    char *s = (char *)(h + 1);
    h->len = len;
    if (len && ptr && ptr != SDS_NOINIT) memcpy(s, ptr, len);
    s[len] = 0;
    o->type = OBJ_STRING; o->encoding = OBJ_ENCODING_EMBSTR; o->ptr = s; o->refcount = 1; o->lru = 0;
    return o;
}
robj *createStringObjectFromLongLongForValue(long long value) {
    robj *o = createObject(OBJ_STRING, (void *)(intptr_t)value);
    o->encoding = OBJ_ENCODING_INT;
    return o;
}
robj *createQuicklistObject(void) {
    quicklist *ql = zmalloc(sizeof *ql);
    ql->e = NULL; ql->n = ql->cap = 0;
    robj *o = createObject(OBJ_LIST, ql);
    o->encoding = OBJ_ENCODING_QUICKLIST;
    return o;
}
robj *createSetObject(void) {
    robj *o = createObject(OBJ_SET, dictCreate(&setDictType, NULL));
    o->encoding = OBJ_ENCODING_HT;
    return o;
}
robj *createIntsetObject(void) {
    intset *is = zmalloc(sizeof(intset));
    is->encoding = 2; is->length = 0;
    robj *o = createObject(OBJ_SET, is);
    o->encoding = OBJ_ENCODING_INTSET;
    return o;
}
robj *createZsetObject(void) {
    zset *zs = zmalloc(sizeof *zs);
    zs->dict = dictCreate(&zsetDictType, NULL);
    zs->zsl = zmalloc(sizeof(zskiplist));
    zs->zsl->header = zs->zsl->tail = NULL; zs->zsl->length = 0; zs->zsl->level = 1;
    robj *o = createObject(OBJ_ZSET, zs);
    o->encoding = OBJ_ENCODING_SKIPLIST;
    return o;
}
static void dictFree(dict *d, int keys, int vals) {
    for (unsigned long i = 0; i < d->used; i++) {
        if (keys) sdsfree(d->ents[i].key);
        if (vals) sdsfree(d->ents[i].v.val);
    }
    zfree(d->ents); zfree(d);
}
void decrRefCount(robj *o) {
    switch (o->type) {
    case OBJ_STRING: if (o->encoding == OBJ_ENCODING_RAW) sdsfree(o->ptr); break;   /* (EMBSTR: inside o) */
    case OBJ_LIST: {
        quicklist *ql = o->ptr;
        for (size_t i = 0; i < ql->n; i++) zfree(ql->e[i].s);
        zfree(ql->e); zfree(ql);
        break;
    }
    case OBJ_SET: if (o->encoding == OBJ_ENCODING_HT) dictFree(o->ptr, 1, 0); else zfree(o->ptr); break;
    case OBJ_HASH: if (o->encoding == OBJ_ENCODING_HT) dictFree(o->ptr, 1, 1); else zfree(o->ptr); break;
    case OBJ_ZSET:
        if (o->encoding == OBJ_ENCODING_SKIPLIST) {
            zset *zs = o->ptr;
            for (zskiplistNode *n = zs->zsl->header, *nx; n; n = nx) { nx = n->forward; sdsfree(n->ele); zfree(n); }
            zfree(zs->zsl); zfree(zs->dict->ents); zfree(zs->dict); zfree(zs);
        } else zfree(o->ptr);
        break;
    }
    zfree(o);
}

struct redisServer server = {-2, 0, NULL};   /* list-max-ziplist-size -2, list-compress-depth 0 */
static redisDb mr_db0;
void mr_init_db(void) {
    if (!mr_db0.dict) mr_db0.dict = dictCreate(NULL, NULL);
    server.db = &mr_db0;
}

sds sdsfromlonglong(long long value) {
    char buf[32];
    int l = ll2string(buf, sizeof buf, value);
    return sdsnewlen(buf, (size_t)l);
}

char *mr_log;
size_t mr_log_len;
static size_t mr_log_cap;
void mr_log_reset(void) { mr_log_len = 0; if (mr_log) mr_log[0] = 0; }
void serverLog(int level, const char *fmt, ...) {
    char line[1024];
    va_list ap;
    va_start(ap, fmt);
    int l = vsnprintf(line, sizeof line, fmt, ap);
    va_end(ap);
    if (l < 0) return;
    if ((size_t)l >= sizeof line) l = (int)sizeof line - 1;
    if (mr_log_len + (size_t)l + 2 > mr_log_cap) {
        mr_log_cap = (mr_log_len + (size_t)l + 2) * 2;
        mr_log = zrealloc(mr_log, mr_log_cap);
    }
    memcpy(mr_log + mr_log_len, line, (size_t)l);
    mr_log_len += (size_t)l;
    mr_log[mr_log_len++] = '\n';
    mr_log[mr_log_len] = 0;
    printf("[log %d] %s\n", level, line);
}

jmp_buf *mr_panic_jmp;
char mr_panic_msg[256];
void _serverPanic(const char *file, int line, const char *msg, ...) {
    va_list ap;
    va_start(ap, msg);
    vsnprintf(mr_panic_msg, sizeof mr_panic_msg, msg, ap);
    va_end(ap);
    (void)file; (void)line;
    if (mr_panic_jmp) longjmp(*mr_panic_jmp, 1);
    fprintf(stderr, "PANIC: %s\n", mr_panic_msg);
    abort();
}
void _serverAssert(const char *estr, const char *file, int line) {
    snprintf(mr_panic_msg, sizeof mr_panic_msg, "assert %s (%s:%d)", estr, file, line);
    if (mr_panic_jmp) longjmp(*mr_panic_jmp, 1);
    fprintf(stderr, "ASSERT: %s\n", mr_panic_msg);
    abort();
}
