/*
 * rr_oracle.c — flat-mode CPU restatement of src/rock_serdes.c (TEST INFRASTRUCTURE ONLY;
 * see rr_oracle.h for who may use it and how parity is pinned).
 *
 * Every function cites the reference lines it restates.  Error codes map the reference's
 * serverAssert/serverPanic sites to per-value status codes (rr_format.h).
 */
#define _GNU_SOURCE
#include "rr_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t ld64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline void st32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static inline void st64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }

/* util.c:360-424 — strict: no '+', no spaces, no leading zeros, overflow checked. */
int rro_string2ll(const char *s, size_t slen, long long *value) {
    const char *p = s;
    size_t plen = 0;
    int negative = 0;
    unsigned long long v;
    if (slen == 0) return 0;
    if (slen == 1 && p[0] == '0') { if (value) *value = 0; return 1; }
    if (p[0] == '-') {
        negative = 1; p++; plen++;
        if (plen == slen) return 0;
    }
    if (p[0] >= '1' && p[0] <= '9') { v = (unsigned long long)(p[0] - '0'); p++; plen++; }
    else return 0;
    while (plen < slen && p[0] >= '0' && p[0] <= '9') {
        if (v > (~0ULL / 10)) return 0;
        v *= 10;
        if (v > (~0ULL - (unsigned long long)(p[0] - '0'))) return 0;
        v += (unsigned long long)(p[0] - '0');
        p++; plen++;
    }
    if (plen < slen) return 0;
    if (negative) {
        if (v > (1ULL << 63)) return 0;
        if (value) *value = (long long)(0ULL - v);
    } else {
        if (v > (unsigned long long)0x7FFFFFFFFFFFFFFFLL) return 0;
        if (value) *value = (long long)v;
    }
    return 1;
}

/* sds.c:450-479 — reversed-digit rendering; for LLONG_MIN the negation wraps to 2^63. */
int rro_ll2str(char *s, long long value) {
    unsigned long long v = (value < 0) ? 0ULL - (unsigned long long)value : (unsigned long long)value;
    char *p = s;
    do { *p++ = (char)('0' + (v % 10)); v /= 10; } while (v);
    if (value < 0) *p++ = '-';
    int l = (int)(p - s);
    *p = '\0';
    p--;
    while (s < p) { char a = *s; *s = *p; *p = a; s++; p--; }
    return l;
}

/* ziplist.c:480-503 — only 1..31-byte strings are tried. */
int rro_zip_try_encoding(const uint8_t *s, uint64_t len, long long *v) {
    if (len >= 32 || len == 0) return 0;
    return rro_string2ll((const char *)s, (size_t)len, v);
}

/* ziplist.c:300-447 (ZIP_DECODE_PREVLEN / ZIP_DECODE_LENGTH / zipIntSize / zipLoadInteger),
 * header :193-256.  Bounds-checked; the reference trusts the bytes (rock_serdes.c:356-366). */
int rro_parse_ziplist(const uint8_t *zl, uint64_t L, uint64_t base, rr_elem *out, uint64_t cap,
                      uint64_t *count) {
    *count = 0;
    if (L < 11 || ld32(zl) != L) return RR_E_ZL_CORRUPT;
    uint32_t zltail = ld32(zl + 4);
    uint16_t zllen = (uint16_t)(zl[8] | (zl[9] << 8));
    uint64_t p = 10, prev_raw = 0, last = 10, n = 0;
    for (;;) {
        if (p >= L) return RR_E_ZL_CORRUPT;
        if (zl[p] == 0xFF) break;
        uint64_t pl, pls;
        if (zl[p] < 254) { pl = zl[p]; pls = 1; }
        else {
            if (p + 5 > L - 1) return RR_E_ZL_CORRUPT;
            pl = ld32(zl + p + 1); pls = 5;
        }
        if (pl != prev_raw) return RR_E_ZL_CORRUPT;
        uint64_t q = p + pls;
        if (q >= L - 1) return RR_E_ZL_CORRUPT;
        uint8_t enc = zl[q];
        uint64_t end;
        rr_elem e;
        memset(&e, 0, sizeof e);
        if (enc < 0xC0) {
            uint8_t cls = enc & 0xC0;
            uint64_t ls, sl;
            if (cls == 0x00) { ls = 1; sl = enc & 0x3F; }
            else if (cls == 0x40) {
                if (q + 2 > L - 1) return RR_E_ZL_CORRUPT;
                ls = 2; sl = ((uint64_t)(enc & 0x3F) << 8) | zl[q + 1];
            } else {
                if (q + 5 > L - 1) return RR_E_ZL_CORRUPT;
                ls = 5;
                sl = ((uint64_t)zl[q + 1] << 24) | ((uint64_t)zl[q + 2] << 16) |
                     ((uint64_t)zl[q + 3] << 8) | zl[q + 4];
            }
            uint64_t d = q + ls;
            end = d + sl;
            if (end > L - 1) return RR_E_ZL_CORRUPT;
            e.kind = RR_K_STR; e.data = base + d; e.len = (uint32_t)sl; e.zenc = cls;
        } else {
            uint64_t isz;
            switch (enc) {
            case 0xFE: isz = 1; break;
            case 0xC0: isz = 2; break;
            case 0xF0: isz = 3; break;
            case 0xD0: isz = 4; break;
            case 0xE0: isz = 8; break;
            default:
                if (enc >= 0xF1 && enc <= 0xFD) isz = 0;
                else return RR_E_ZL_CORRUPT;
            }
            uint64_t d = q + 1;
            end = d + isz;
            if (end > L - 1) return RR_E_ZL_CORRUPT;
            int64_t v;
            if (isz == 0) v = (int64_t)(enc & 0x0F) - 1;
            else if (isz == 1) v = (int8_t)zl[d];
            else if (isz == 2) v = (int16_t)(zl[d] | (zl[d + 1] << 8));
            else if (isz == 3) { /* zipLoadInteger :552-556: i32 built from 3 high bytes, >> 8 */
                int32_t i32 = (int32_t)(((uint32_t)zl[d] << 8) | ((uint32_t)zl[d + 1] << 16) |
                                        ((uint32_t)zl[d + 2] << 24));
                v = i32 >> 8;
            } else if (isz == 4) v = (int32_t)ld32(zl + d);
            else v = (int64_t)ld64(zl + d);
            e.kind = RR_K_INT; e.data = (uint64_t)v; e.zenc = enc;
        }
        if (out) { if (n >= cap) return RR_E_CAPACITY; out[n] = e; }
        n++;
        prev_raw = end - p;
        last = p;
        p = end;
    }
    if (p != L - 1) return RR_E_ZL_CORRUPT;
    if (zllen != 0xFFFF && zllen != n) return RR_E_ZL_CORRUPT;
    if (zltail != last) return RR_E_ZL_CORRUPT;
    *count = n;
    return RR_OK;
}

#define EMIT(K, D, LEN, Z) do { \
        if (out) { rr_elem *e_ = &out[n]; e_->data = (uint64_t)(D); e_->len = (uint32_t)(LEN); \
                   e_->kind = (K); e_->zenc = (Z); e_->rsv = 0; } \
        n++; } while (0)

/* Members of one HT / skiplist value while it is parsed: batch offset + length of the string,
 * the raw score bits (skiplist), the position in the blob, and a duplicate mark. */
typedef struct { uint64_t off, len, score; uint64_t idx; int dup; } mem_t;
static __thread mem_t *g_mem;
static __thread uint64_t g_mem_cap;
static __thread const uint8_t *g_base;   /* batch base for the qsort comparators */

static mem_t *mem_slot(uint64_t i) {
    if (i >= g_mem_cap) {
        uint64_t c = g_mem_cap ? g_mem_cap * 2 : 64;
        while (c <= i) c *= 2;
        g_mem = (mem_t *)realloc(g_mem, c * sizeof(mem_t));
        g_mem_cap = c;
    }
    return &g_mem[i];
}

/* sdscmp (sds.c:814-824): memcmp of the common prefix, then the shorter string first */
static int sdscmp_raw(const uint8_t *a, uint64_t la, const uint8_t *b, uint64_t lb) {
    uint64_t m = la < lb ? la : lb;
    int c = m ? memcmp(a, b, m) : 0;
    if (c) return c;
    return la < lb ? -1 : la > lb ? 1 : 0;
}

/* content order for duplicate detection: (len, bytes), then blob position */
static int key_cmp(const void *x, const void *y) {
    const mem_t *a = *(mem_t *const *)x, *b = *(mem_t *const *)y;
    if (a->len != b->len) return a->len < b->len ? -1 : 1;
    int c = a->len ? memcmp(g_base + a->off, g_base + b->off, a->len) : 0;
    if (c) return c;
    return a->idx < b->idx ? -1 : a->idx > b->idx;
}

/* Marks every key equal to an earlier key (dictAdd's DICT_ERR, dict.c:265 via
 * dictAddRaw/_dictKeyIndex); returns how many.  keys[] point into the member table. */
static uint64_t mark_dups(mem_t **keys, uint64_t k) {
    if (k < 2) return 0;
    qsort(keys, k, sizeof(mem_t *), key_cmp);
    uint64_t d = 0;
    for (uint64_t i = 1; i < k; i++)
        if (keys[i]->len == keys[i - 1]->len &&
            (!keys[i]->len || !memcmp(g_base + keys[i]->off, g_base + keys[i - 1]->off, keys[i]->len))) {
            keys[i]->dup = 1;   /* the earlier blob position sorted first: it is the one dictAdd kept */
            d++;
        }
    return d;
}

/* The order serZset writes the skiplist desZset rebuilt: zslInsert (t_zset.c:132-180) keeps
 * the list ascending by (score, sdscmp(ele)) with a new node placed before equal ones, and
 * serZset walks it tail->head (rock_serdes.c:430-440) — i.e. descending by (score, ele),
 * equal keys in blob order.  Scores compare as doubles (-0.0 == 0.0); NaN never gets here. */
static int sl_cmp(const void *x, const void *y) {
    const mem_t *a = (const mem_t *)x, *b = (const mem_t *)y;
    double sa, sb;
    memcpy(&sa, &a->score, 8);
    memcpy(&sb, &b->score, 8);
    if (sa > sb) return -1;
    if (sa < sb) return 1;
    int c = sdscmp_raw(g_base + a->off, a->len, g_base + b->off, b->len);
    if (c) return c > 0 ? -1 : 1;
    return a->idx < b->idx ? -1 : a->idx > b->idx;
}

static int is_nan_bits(uint64_t s) {
    return (s & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (s & 0x000FFFFFFFFFFFFFull);
}

/* desObject rock_serdes.c:538-564 and des{String,List,Set,Hash,Zset} :133-508. */
int rro_decode_one(const uint8_t *data, uint64_t off, uint64_t len, rr_value *v,
                   rr_elem *out, uint64_t *n_elems, uint64_t *n_slots, uint64_t *payload) {
    const uint8_t *b = data + off;
    uint64_t n = 0, pay = 0, slots = 0;
    int st = RR_OK;
    g_base = data;
    v->type = len ? b[0] : 0;
    v->enc = 0;
    v->lru = len >= 5 ? (ld32(b + 1) & RR_LRU_MASK) : 0;
    *n_elems = 0; *payload = 0; *n_slots = 0;
    if (len < 5) { st = RR_E_SHORT; goto done; }                       /* :539-542 */
    uint64_t p = 5, rem = len - 5;
    switch (b[0]) {
    case RR_TYPE_STRING: {                                               /* :133-158 */
        if (len < 6) { st = RR_E_SHORT; break; }
        uint8_t enc = b[5];
        v->enc = enc;
        uint64_t rest = len - 6;
        if (enc == RR_ENC_INT) {
            if (rest != 8) { st = RR_E_STR_INTLEN; break; }
            EMIT(RR_K_INT, ld64(b + 6), 0, 0);
        } else if (enc == RR_ENC_RAW || enc == RR_ENC_EMBSTR) {
            if (enc == RR_ENC_EMBSTR && rest > RR_EMBSTR_SIZE_LIMIT) { st = RR_E_EMBSTR_LEN; break; }
            if (rest > 0xFFFFFFFFull) { st = RR_E_CAPACITY; break; }
            EMIT(RR_K_STR, off + 6, rest, 0);
            pay += rest;
        } else st = RR_E_STR_ENC;
        break;
    }
    case RR_TYPE_LIST_QUICKLIST:                                         /* :191-214 */
        while (rem) {
            if (rem < 4) { st = RR_E_TRUNC; break; }
            uint64_t l = ld32(b + p);
            p += 4; rem -= 4;
            if (l > rem) { st = RR_E_TRUNC; break; }
            long long iv;
            if (rro_zip_try_encoding(b + p, l, &iv)) EMIT(RR_K_INT, iv, 0, 0);
            else { EMIT(RR_K_STR, off + p, l, 0); pay += l; }
            p += l; rem -= l;
        }
        break;
    case RR_TYPE_SET_INTSET: {                                           /* :255-276 */
        if (rem < 8) { st = RR_E_SHORT; break; }
        uint64_t w = ld32(b + p), cnt = ld32(b + p + 4);
        p += 8; rem -= 8;
        if ((w != 2 && w != 4 && w != 8) || rem != w * cnt) { st = RR_E_INTSET; break; }
        v->enc = (uint8_t)w;
        for (uint64_t i = 0; i < cnt; i++) {
            const uint8_t *q = b + p + i * w;
            int64_t x = w == 2 ? (int16_t)(q[0] | (q[1] << 8)) : w == 4 ? (int32_t)ld32(q) : (int64_t)ld64(q);
            EMIT(RR_K_INT, x, 0, 0);
        }
        break;
    }
    case RR_TYPE_SET_HT:                                                 /* :277-303 */
    case RR_TYPE_HASH_HT: {                                              /* :368-404 */
        if (rem < 8) { st = RR_E_SHORT; break; }
        uint64_t cnt = ld64(b + p), got = 0, m = 0;
        int per = b[0] == RR_TYPE_SET_HT ? 1 : 2;
        p += 8; rem -= 8;
        while (rem && st == RR_OK) {
            for (int k = 0; k < per; k++) {
                if (rem < 8) { st = RR_E_TRUNC; break; }
                uint64_t l = ld64(b + p);
                p += 8; rem -= 8;
                if (l > rem) { st = RR_E_TRUNC; break; }
                mem_t *e = mem_slot(m);
                e->off = off + p; e->len = l; e->idx = m; e->dup = 0;
                m++;
                p += l; rem -= l;
            }
            got++;
        }
        if (st == RR_OK && got != cnt) st = RR_E_COUNT;
        if (st != RR_OK) break;
        slots = m;
        /* keys: every member of a set, the fields (even positions) of a hash */
        uint64_t nk = per == 1 ? m : m / 2;
        mem_t **keys = (mem_t **)malloc(sizeof(mem_t *) * (nk ? nk : 1));
        for (uint64_t i = 0; i < nk; i++) keys[i] = &g_mem[i * (uint64_t)per];
        uint64_t d = mark_dups(keys, nk);
        free(keys);
        if (d && per == 2) { st = RR_E_DUP; break; }                   /* :399-400 */
        for (uint64_t i = 0; i < m; i++) {                               /* :297 keeps the first */
            if (g_mem[i].dup) continue;
            EMIT(RR_K_STR, g_mem[i].off, g_mem[i].len, 0);
            pay += g_mem[i].len;
        }
        break;
    }
    case RR_TYPE_HASH_ZIPLIST:                                           /* :356-366 */
    case RR_TYPE_ZSET_ZIPLIST: {                                         /* :455-466 */
        if (rem < 8) { st = RR_E_SHORT; break; }
        uint64_t L = ld64(b + p);
        p += 8; rem -= 8;
        if (rem != L) { st = RR_E_ZL_LEN; break; }
        uint64_t cnt;
        st = rro_parse_ziplist(b + p, L, off + p, out ? out + 1 : NULL, (uint64_t)-1, &cnt);
        if (st == RR_OK && (cnt & 1)) st = RR_E_ZL_CORRUPT;
        if (st != RR_OK) break;
        if (out) { out[0].data = off + p; out[0].len = (uint32_t)L; out[0].kind = RR_K_ZLRAW;
                   out[0].zenc = 0; out[0].rsv = 0; }
        n = 1 + cnt;
        pay += L;
        break;
    }
    case RR_TYPE_ZSET_SKIPLIST: {                                        /* :467-501 */
        if (rem < 8) { st = RR_E_SHORT; break; }
        uint64_t cnt = ld64(b + p), m = 0;
        p += 8; rem -= 8;
        for (uint64_t i = 0; i < cnt; i++) {
            if (rem < 8) { st = RR_E_TRUNC; break; }
            uint64_t l = ld64(b + p);
            p += 8; rem -= 8;
            if (l > rem) { st = RR_E_TRUNC; break; }
            mem_t *e = mem_slot(m);
            e->off = off + p; e->len = l; e->idx = m; e->dup = 0;
            p += l; rem -= l;
            if (rem < 8) { st = RR_E_TRUNC; break; }
            e->score = ld64(b + p);
            m++;
            p += 8; rem -= 8;
        }
        if (st == RR_OK && rem != 0) st = RR_E_COUNT;
        if (st != RR_OK) break;
        for (uint64_t i = 0; i < m; i++)
            if (is_nan_bits(g_mem[i].score)) { st = RR_E_NAN; break; }  /* t_zset.c:137 */
        if (st != RR_OK) break;
        int sorted = 1;
        for (uint64_t i = 1; i < m && sorted; i++) sorted = sl_cmp(&g_mem[i - 1], &g_mem[i]) < 0;
        if (!sorted) qsort(g_mem, m, sizeof(mem_t), sl_cmp);
        slots = 2 * m;
        for (uint64_t i = 0; i < m; i++) {
            EMIT(RR_K_STR, g_mem[i].off, g_mem[i].len, 0);
            EMIT(RR_K_SCORE, g_mem[i].score, 0, 0);
            pay += g_mem[i].len;
        }
        break;
    }
    default:
        st = RR_E_TYPE;                                                  /* :560-562 */
    }
done:
    if (st != RR_OK) { n = 0; pay = 0; slots = 0; }
    else if (b[0] != RR_TYPE_SET_HT && b[0] != RR_TYPE_HASH_HT && b[0] != RR_TYPE_ZSET_SKIPLIST) slots = n;
    v->status = (uint16_t)st;
    *n_elems = n;
    *n_slots = slots;
    *payload = pay;
    return st;
}

/* Descriptor slots a value owns (rr_format.h "descriptor slots"): from the header alone, plus
 * the length chain of a List.  Equals the decoded count for every valid blob; a malformed
 * value keeps its slots zero-filled. */
static uint64_t zl_walk_count(const uint8_t *zl, uint64_t L) {
    uint64_t p = 10, n = 0;
    while (p < L - 1 && zl[p] != 0xFF) {
        uint64_t q = p + (zl[p] < 254 ? 1 : 5), e;
        if (q >= L - 1) break;
        uint8_t enc = zl[q];
        if (enc < 0xC0) {
            uint8_t cls = enc & 0xC0;
            if (cls == 0x00) e = q + 1 + (enc & 0x3F);
            else if (cls == 0x40) { if (q + 2 > L - 1) break; e = q + 2 + (((uint64_t)(enc & 0x3F) << 8) | zl[q + 1]); }
            else {
                if (q + 5 > L - 1) break;
                e = q + 5 + (((uint64_t)zl[q + 1] << 24) | ((uint64_t)zl[q + 2] << 16) | ((uint64_t)zl[q + 3] << 8) | zl[q + 4]);
            }
        } else if (enc == 0xFE) e = q + 2;
        else if (enc == 0xC0) e = q + 3;
        else if (enc == 0xF0) e = q + 4;
        else if (enc == 0xD0) e = q + 5;
        else if (enc == 0xE0) e = q + 9;
        else if (enc >= 0xF1 && enc <= 0xFD) e = q + 1;
        else break;
        if (e > L - 1) break;
        n++;
        p = e;
    }
    return n;
}

uint64_t rro_reserve(const uint8_t *b, uint64_t L) {
    if (L < 5) return 0;
    switch (b[0]) {
    case RR_TYPE_STRING: return L >= 6 ? 1 : 0;
    case RR_TYPE_LIST_QUICKLIST: {
        uint64_t p = 5, n = 0;
        while (p < L) {
            if (L - p < 4) break;
            uint64_t l = ld32(b + p);
            if (l > L - p - 4) break;
            n++;
            p += 4 + l;
        }
        return n;
    }
    default: break;
    }
    if (L < 13) return 0;
    switch (b[0]) {
    case RR_TYPE_SET_INTSET: {
        uint64_t w = ld32(b + 5), c = ld32(b + 9);
        return ((w == 2 || w == 4 || w == 8) && L - 13 == w * c) ? c : 0;
    }
    case RR_TYPE_SET_HT: { uint64_t c = ld64(b + 5), m = (L - 13) / 8; return c < m ? c : m; }
    case RR_TYPE_HASH_HT: { uint64_t c = ld64(b + 5), m = (L - 13) / 8; return c > m / 2 ? m : 2 * c; }
    case RR_TYPE_ZSET_SKIPLIST: { uint64_t c = ld64(b + 5), m = (L - 13) / 16; return 2 * (c < m ? c : m); }
    case RR_TYPE_HASH_ZIPLIST:
    case RR_TYPE_ZSET_ZIPLIST: {
        uint64_t Lz = ld64(b + 5);
        if (Lz != L - 13 || Lz < 11) return 0;
        uint64_t zllen = (uint64_t)b[21] | ((uint64_t)b[22] << 8);
        if (zllen != 0xFFFF) { uint64_t m = (Lz - 11) / 2; return 1 + (zllen < m ? zllen : m); }
        return 1 + zl_walk_count(b + 13, Lz);
    }
    default: return 0;
    }
}

/* ---------------------------------------------------------------- batch, pthreads */

typedef struct {
    const uint8_t *data; const uint64_t *off;
    rr_value *values; rr_elem *elems; uint64_t cap;
    const rr_elem *ielems; const uint8_t *arena; uint8_t *odata; uint64_t *ooff;
    uint64_t v0, v1;
    uint64_t base;        /* in: running base for pass 2 */
    uint64_t count, payload, bad;
    uint64_t *sizes;
    uint64_t ecap, acap;  /* encode: elem_cap / arena_cap of the flat input */
    int pass;
} job_t;

static void *dec_worker(void *arg) {
    job_t *j = (job_t *)arg;
    uint64_t base = j->base, cnt = 0, pay = 0, bad = 0;
    for (uint64_t i = j->v0; i < j->v1; i++) {
        uint64_t o = j->off[i], len = j->off[i + 1] - o, ne, ns, pl;
        rr_value *v = &j->values[i];
        if (j->pass == 1) {
            uint64_t r = rro_reserve(j->data + o, len);
            v->elem_base = (uint32_t)r;          /* stash the reservation for pass 2 */
            cnt += r;
        } else {
            uint64_t r = v->elem_base;
            rro_decode_one(j->data, o, len, v, NULL, &ne, &ns, &pl);
            if (v->status == RR_OK && ns != r) { v->status = RR_E_COUNT; ne = 0; }
            v->elem_base = (uint32_t)base;
            if (v->status != RR_OK) {
                /* malformed: its slots are zero-filled (when they fit) and it owns no descriptors */
                if (base + r <= j->cap) memset(j->elems + base, 0, sizeof(rr_elem) * r);
                ne = 0;
            } else if (base + r > j->cap) {
                v->status = RR_E_CAPACITY;                 /* keeps its count, writes nothing */
            } else {
                rro_decode_one(j->data, o, len, v, j->elems + base, &ne, &ns, &pl);
                if (ne < r) memset(j->elems + base + ne, 0, sizeof(rr_elem) * (r - ne));   /* SET_HT dedup */
                pay += pl;
            }
            v->n_elems = (uint32_t)ne;
            if (v->status != RR_OK) bad++;
            base += r;
        }
    }
    j->count = cnt; j->payload = pay; j->bad = bad;
    return NULL;
}

int rro_nprocs(void) {
    long n = sysconf(_SC_NPROCESSORS_ONLN);
    return n > 0 ? (int)n : 1;
}

static void run_jobs(job_t *jobs, int nt, void *(*fn)(void *)) {
    if (nt == 1) { fn(&jobs[0]); return; }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nt);
    for (int t = 0; t < nt; t++) pthread_create(&th[t], NULL, fn, &jobs[t]);
    for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
    free(th);
}

/* Byte-balanced value ranges (SURVEY.md §8e partition rule, applied to host threads). */
static void split_ranges(const uint64_t *off, uint64_t n, int nt, job_t *jobs) {
    uint64_t total = off[n], v = 0;
    for (int t = 0; t < nt; t++) {
        uint64_t target = total / (uint64_t)nt * (uint64_t)(t + 1);
        uint64_t v1 = v;
        if (t == nt - 1) v1 = n;
        else while (v1 < n && off[v1] < target) v1++;
        jobs[t].v0 = v; jobs[t].v1 = v1; v = v1;
    }
}

int rro_decode(const uint8_t *data, const uint64_t *offsets, uint64_t n, rr_value *values,
               rr_elem *elems, uint64_t elem_cap, uint8_t *arena, rr_totals *t, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    split_ranges(offsets, n, nthreads, jobs);
    for (int k = 0; k < nthreads; k++) {
        jobs[k].data = data; jobs[k].off = offsets; jobs[k].values = values;
        jobs[k].elems = elems; jobs[k].cap = elem_cap; jobs[k].pass = 1;
    }
    run_jobs(jobs, nthreads, dec_worker);
    uint64_t base = 0;
    for (int k = 0; k < nthreads; k++) { jobs[k].base = base; base += jobs[k].count; jobs[k].pass = 2; }
    run_jobs(jobs, nthreads, dec_worker);
    if (arena && offsets[n]) memcpy(arena, data, offsets[n]);   /* mirror arena */
    rr_totals tt = {base, offsets[n], 0, 0};
    for (int k = 0; k < nthreads; k++) { tt.n_bad += jobs[k].bad; tt.payload += jobs[k].payload; }
    if (t) *t = tt;
    free(jobs);
    return RR_OK;
}

/* ---------------------------------------------------------------- encode */

static inline uint64_t dec_len(long long v) {
    char buf[24];
    return (uint64_t)rro_ll2str(buf, v);
}

static int fits_width(int64_t x, unsigned w) {
    if (w == 8) return 1;
    if (w == 4) return x >= INT32_MIN && x <= INT32_MAX;
    return x >= INT16_MIN && x <= INT16_MAX;
}

/* serObject rock_serdes.c:512-535 sizes.  A value is unencodable (RR_E_ENCODE, size 0) when
 * its status is not RR_OK, its descriptor range passes elem_cap, a payload it references
 * passes arena_cap, or its descriptors do not have the kinds its type needs. */
#define ARENA_OK(E) ((E).data <= arena_cap && (uint64_t)(E).len <= arena_cap - (E).data)
uint64_t rro_encode_size(const rr_value *v, const rr_elem *elems, uint64_t elem_cap, uint64_t arena_cap,
                         int *status) {
    uint64_t n = v->n_elems, s = 5;
    *status = RR_OK;
    if (v->status != RR_OK || (uint64_t)v->elem_base + n > elem_cap) goto bad;
    const rr_elem *el = elems + v->elem_base;
    switch (v->type) {
    case RR_TYPE_STRING:
        if (n != 1) goto bad;
        if (v->enc == RR_ENC_INT) { if (el[0].kind != RR_K_INT) goto bad; return 14; }
        if ((v->enc != RR_ENC_RAW && v->enc != RR_ENC_EMBSTR) || el[0].kind != RR_K_STR || !ARENA_OK(el[0])) goto bad;
        return 6 + el[0].len;
    case RR_TYPE_LIST_QUICKLIST:
        for (uint64_t i = 0; i < n; i++) {
            if (el[i].kind == RR_K_INT) s += 4 + dec_len((long long)el[i].data);
            else if (el[i].kind == RR_K_STR && ARENA_OK(el[i])) s += 4 + el[i].len;
            else goto bad;
        }
        return s;
    case RR_TYPE_SET_INTSET:
        if (v->enc != 2 && v->enc != 4 && v->enc != 8) goto bad;
        for (uint64_t i = 0; i < n; i++)
            if (el[i].kind != RR_K_INT || !fits_width((int64_t)el[i].data, v->enc)) goto bad;
        return 13 + (uint64_t)v->enc * n;
    case RR_TYPE_SET_HT:
    case RR_TYPE_HASH_HT:
        if (v->type == RR_TYPE_HASH_HT && (n & 1)) goto bad;
        s += 8;
        for (uint64_t i = 0; i < n; i++) {
            if (el[i].kind != RR_K_STR || !ARENA_OK(el[i])) goto bad;
            s += 8 + el[i].len;
        }
        return s;
    case RR_TYPE_HASH_ZIPLIST:
    case RR_TYPE_ZSET_ZIPLIST:
        if (n < 1 || el[0].kind != RR_K_ZLRAW || !ARENA_OK(el[0])) goto bad;
        return 13 + el[0].len;
    case RR_TYPE_ZSET_SKIPLIST:
        if (n & 1) goto bad;
        s += 8;
        for (uint64_t i = 0; i < n; i += 2) {
            if (el[i].kind != RR_K_STR || !ARENA_OK(el[i]) || el[i + 1].kind != RR_K_SCORE) goto bad;
            s += 16 + el[i].len;
        }
        return s;
    default:
        break;
    }
bad:
    *status = RR_E_ENCODE;
    return 0;
}

static void encode_one(const rr_value *v, const rr_elem *el, const uint8_t *arena, uint8_t *o) {
    uint64_t n = v->n_elems, p = 5;
    o[0] = v->type;
    st32(o + 1, v->lru & RR_LRU_MASK);
    switch (v->type) {
    case RR_TYPE_STRING:                                                 /* :114-128 */
        o[5] = v->enc;
        if (v->enc == RR_ENC_INT) st64(o + 6, el[0].data);
        else memcpy(o + 6, arena + el[0].data, el[0].len);
        break;
    case RR_TYPE_LIST_QUICKLIST:                                         /* :162-188 */
        for (uint64_t i = 0; i < n; i++) {
            if (el[i].kind == RR_K_INT) {
                char buf[24];
                uint32_t l = (uint32_t)rro_ll2str(buf, (long long)el[i].data);
                st32(o + p, l); memcpy(o + p + 4, buf, l); p += 4 + l;
            } else {
                st32(o + p, el[i].len); memcpy(o + p + 4, arena + el[i].data, el[i].len);
                p += 4 + el[i].len;
            }
        }
        break;
    case RR_TYPE_SET_INTSET: {                                           /* :220-226 */
        uint32_t w = v->enc;
        st32(o + p, w); st32(o + p + 4, (uint32_t)n); p += 8;
        for (uint64_t i = 0; i < n; i++) { uint64_t x = el[i].data; memcpy(o + p, &x, w); p += w; }
        break;
    }
    case RR_TYPE_SET_HT:                                                 /* :227-239 */
    case RR_TYPE_HASH_HT:                                                /* :322-339 */
        st64(o + p, v->type == RR_TYPE_SET_HT ? n : n / 2); p += 8;
        for (uint64_t i = 0; i < n; i++) {
            st64(o + p, el[i].len); memcpy(o + p + 8, arena + el[i].data, el[i].len);
            p += 8 + el[i].len;
        }
        break;
    case RR_TYPE_HASH_ZIPLIST:                                           /* :317-320 */
    case RR_TYPE_ZSET_ZIPLIST:                                           /* :420-423 */
        st64(o + p, el[0].len);
        memcpy(o + p + 8, arena + el[0].data, el[0].len);
        break;
    case RR_TYPE_ZSET_SKIPLIST:                                          /* :425-440 */
        st64(o + p, n / 2); p += 8;
        for (uint64_t i = 0; i < n; i += 2) {
            st64(o + p, el[i].len); memcpy(o + p + 8, arena + el[i].data, el[i].len);
            p += 8 + el[i].len;
            st64(o + p, el[i + 1].data); p += 8;
        }
        break;
    }
}

static void *enc_worker(void *arg) {
    job_t *j = (job_t *)arg;
    uint64_t base = j->base, tot = 0, bad = 0, pay = 0;
    for (uint64_t i = j->v0; i < j->v1; i++) {
        const rr_value *v = &j->values[i];
        int st;
        if (j->pass == 1) {
            uint64_t s = rro_encode_size(v, j->ielems, j->ecap, j->acap, &st);
            j->sizes[i] = s;
            tot += s;
        } else {
            uint64_t s = j->sizes[i];
            j->ooff[i] = base;
            rro_encode_size(v, j->ielems, j->ecap, j->acap, &st);
            if (st != RR_OK || base + s > j->cap) bad++;
            else {
                encode_one(v, j->ielems + v->elem_base, j->arena, j->odata + base);
                const rr_elem *el = j->ielems + v->elem_base;
                for (uint32_t k = 0; k < v->n_elems; k++)
                    if (el[k].kind == RR_K_STR || el[k].kind == RR_K_ZLRAW) {
                        pay += el[k].len;
                        if (el[k].kind == RR_K_ZLRAW) break;
                    }
            }
            base += s;
        }
    }
    j->count = tot; j->bad = bad; j->payload = pay;
    return NULL;
}

int rro_encode(const rr_value *values, const rr_elem *elems, uint64_t elem_cap, const uint8_t *arena,
               uint64_t arena_cap, uint64_t n, uint8_t *data, uint64_t data_cap, uint64_t *offsets, rr_totals *t,
               int nthreads) {
    if (nthreads < 1) nthreads = 1;
    uint64_t *sizes = (uint64_t *)malloc(sizeof(uint64_t) * (n ? n : 1));
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    /* value ranges balanced by descriptor count */
    uint64_t tot_el = 0, v = 0, run = 0, v1 = 0;
    for (uint64_t i = 0; i < n; i++) tot_el += values[i].n_elems;
    for (int k = 0; k < nthreads; k++) {
        uint64_t target = tot_el / (uint64_t)nthreads * (uint64_t)(k + 1);
        v1 = v;
        if (k == nthreads - 1) v1 = n;
        else while (v1 < n && run < target) run += values[v1++].n_elems;
        jobs[k].v0 = v; jobs[k].v1 = v1; v = v1;
        jobs[k].values = (rr_value *)values; jobs[k].ielems = elems; jobs[k].arena = arena;
        jobs[k].odata = data; jobs[k].ooff = offsets; jobs[k].cap = data_cap; jobs[k].sizes = sizes;
        jobs[k].ecap = elem_cap; jobs[k].acap = arena_cap;
        jobs[k].pass = 1;
    }
    run_jobs(jobs, nthreads, enc_worker);
    uint64_t base = 0;
    for (int k = 0; k < nthreads; k++) { jobs[k].base = base; base += jobs[k].count; jobs[k].pass = 2; }
    run_jobs(jobs, nthreads, enc_worker);
    offsets[n] = base;
    rr_totals tt = {tot_el, base, 0, 0};
    for (int k = 0; k < nthreads; k++) { tt.n_bad += jobs[k].bad; tt.payload += jobs[k].payload; }
    if (t) *t = tt;
    free(jobs); free(sizes);
    return RR_OK;
}
