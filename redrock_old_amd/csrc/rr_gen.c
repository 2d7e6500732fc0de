/*
 * rr_gen.c — seeded synthetic value batches for the BASELINE.json configs.
 *
 * Blobs are produced the way RedRock would produce them: the value is first shaped like the
 * Redis object the reference serializes (ziplists built by tail pushes with zipTryEncoding,
 * intsets sorted with the smallest width that holds their members, skiplists walked
 * tail->head, list integers re-rendered by sdsll2str), then laid out per serObject
 * (rock_serdes.c:512-535).  This is a third, independent writer of the format: the tests
 * check that both oracles and the GPU decoder accept every generated blob and that every
 * encoder reproduces it byte for byte.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rr_serdes.h"

/* ------------------------------------------------------------------ rng: xoshiro256** */
typedef struct { uint64_t s[4]; } rng_t;
static uint64_t splitmix(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t *r, uint64_t seed) { for (int i = 0; i < 4; i++) r->s[i] = splitmix(&seed); }
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static uint64_t rnd(rng_t *r) {
    uint64_t *s = r->s, res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static uint64_t rnd_below(rng_t *r, uint64_t n) { return n ? rnd(r) % n : 0; }
static uint64_t rnd_range(rng_t *r, uint64_t lo, uint64_t hi) { return lo + rnd_below(r, hi - lo + 1); }
static double rnd_unit(rng_t *r) { return (double)(rnd(r) >> 11) * (1.0 / 9007199254740992.0); }

/* ------------------------------------------------------------------ byte buffer */
typedef struct { uint8_t *p; uint64_t n, cap; } buf_t;
static void bgrow(buf_t *b, uint64_t need) {
    if (b->n + need <= b->cap) return;
    uint64_t c = b->cap ? b->cap : 4096;
    while (c < b->n + need) c *= 2;
    b->p = (uint8_t *)realloc(b->p, c);
    b->cap = c;
}
static void bput(buf_t *b, const void *d, uint64_t n) { bgrow(b, n); memcpy(b->p + b->n, d, n); b->n += n; }
static void bu8(buf_t *b, uint8_t v) { bput(b, &v, 1); }
static void bu32(buf_t *b, uint32_t v) { bput(b, &v, 4); }
static void bu64(buf_t *b, uint64_t v) { bput(b, &v, 8); }

/* ------------------------------------------------------------------ helpers from Redis text */
/* util.c:360-424 */
static int s2ll(const uint8_t *s, uint64_t slen, long long *value) {
    uint64_t i = 0; int neg = 0; unsigned long long v;
    if (slen == 0) return 0;
    if (slen == 1 && s[0] == '0') { *value = 0; return 1; }
    if (s[0] == '-') { neg = 1; i = 1; if (i == slen) return 0; }
    if (s[i] >= '1' && s[i] <= '9') v = (unsigned long long)(s[i++] - '0'); else return 0;
    while (i < slen && s[i] >= '0' && s[i] <= '9') {
        if (v > ~0ULL / 10) return 0;
        v *= 10;
        if (v > ~0ULL - (unsigned long long)(s[i] - '0')) return 0;
        v += (unsigned long long)(s[i++] - '0');
    }
    if (i < slen) return 0;
    if (neg) { if (v > (1ULL << 63)) return 0; *value = (long long)(0ULL - v); }
    else { if (v > 0x7FFFFFFFFFFFFFFFull) return 0; *value = (long long)v; }
    return 1;
}
/* sds.c:450-479 */
static int ll2s(char *s, long long value) {
    unsigned long long v = value < 0 ? 0ULL - (unsigned long long)value : (unsigned long long)value;
    char *p = s;
    do { *p++ = (char)('0' + v % 10); v /= 10; } while (v);
    if (value < 0) *p++ = '-';
    int l = (int)(p - s);
    for (char *a = s, *z = p - 1; a < z; a++, z--) { char t = *a; *a = *z; *z = t; }
    return l;
}
/* util.c:517-552 */
static int d2s(char *buf, size_t len, double value) {
    if (isnan(value)) return snprintf(buf, len, "nan");
    if (isinf(value)) return snprintf(buf, len, value < 0 ? "-inf" : "inf");
    if (value == 0) return snprintf(buf, len, (1.0 / value < 0) ? "-0" : "0");
    double mn = -4503599627370495.0, mx = 4503599627370496.0;
    if (value > mn && value < mx && value == (double)((long long)value))
        return ll2s(buf, (long long)value);
    return snprintf(buf, len, "%.17g", value);
}

/* ------------------------------------------------------------------ ziplist writer */
/* Tail push, __ziplistInsert ziplist.c:743-839 with zipTryEncoding :480 and
 * zipStoreEntryEncoding :326 / zipStorePrevEntryLength :391. */
typedef struct { buf_t b; uint64_t prev_raw, last, count; } zl_t;
static void zl_init(zl_t *z) {
    memset(z, 0, sizeof *z);
    uint8_t hdr[10] = {0};
    bput(&z->b, hdr, 10);
    z->last = 10;
}
static void zl_push(zl_t *z, const uint8_t *s, uint64_t len, int force_big_prevlen) {
    uint64_t start = z->b.n;
    if (z->prev_raw < 254 && !force_big_prevlen) bu8(&z->b, (uint8_t)z->prev_raw);
    else { bu8(&z->b, 0xFE); bu32(&z->b, (uint32_t)z->prev_raw); }
    long long v;
    if (len > 0 && len < 32 && s2ll(s, len, &v)) {
        if (v >= 0 && v <= 12) bu8(&z->b, (uint8_t)(0xF1 + v));
        else if (v >= -128 && v <= 127) { bu8(&z->b, 0xFE); bu8(&z->b, (uint8_t)(int8_t)v); }
        else if (v >= -32768 && v <= 32767) { bu8(&z->b, 0xC0); int16_t x = (int16_t)v; bput(&z->b, &x, 2); }
        else if (v >= -8388608 && v <= 8388607) {
            bu8(&z->b, 0xF0); uint32_t x = (uint32_t)(int32_t)v; bput(&z->b, &x, 3);
        } else if (v >= INT32_MIN && v <= INT32_MAX) { bu8(&z->b, 0xD0); int32_t x = (int32_t)v; bput(&z->b, &x, 4); }
        else { bu8(&z->b, 0xE0); bput(&z->b, &v, 8); }
    } else {
        if (len <= 0x3F) bu8(&z->b, (uint8_t)len);
        else if (len <= 0x3FFF) { bu8(&z->b, (uint8_t)(0x40 | (len >> 8))); bu8(&z->b, (uint8_t)len); }
        else { bu8(&z->b, 0x80); bu8(&z->b, (uint8_t)(len >> 24)); bu8(&z->b, (uint8_t)(len >> 16));
               bu8(&z->b, (uint8_t)(len >> 8)); bu8(&z->b, (uint8_t)len); }
        bput(&z->b, s, len);
    }
    z->prev_raw = z->b.n - start;
    z->last = start;
    z->count++;
}
static void zl_finish(zl_t *z) {
    bu8(&z->b, 0xFF);
    uint32_t L = (uint32_t)z->b.n, tail = (uint32_t)z->last;
    uint16_t n = z->count < 0xFFFF ? (uint16_t)z->count : 0xFFFF;
    memcpy(z->b.p, &L, 4); memcpy(z->b.p + 4, &tail, 4); memcpy(z->b.p + 8, &n, 2);
}

/* ------------------------------------------------------------------ value shapes */
static const char ALNUM[] = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz";
static void rand_alnum(rng_t *r, uint8_t *d, uint64_t n, int letter_first) {
    for (uint64_t i = 0; i < n; i++) d[i] = (uint8_t)ALNUM[rnd_below(r, 62)];
    if (letter_first && n) d[0] = (uint8_t)ALNUM[10 + rnd_below(r, 52)];
}
/* log-uniform magnitude, random sign: hits every ziplist integer width */
static long long rand_logint(rng_t *r) {
    unsigned b = (unsigned)rnd_below(r, 64);
    unsigned long long m = b == 0 ? 0 : (rnd(r) >> (64 - b));
    if (b == 63 && (rnd(r) & 1)) return (long long)0x8000000000000000ull;  /* LLONG_MIN */
    long long v = (long long)(m & 0x7FFFFFFFFFFFFFFFull);
    return (rnd(r) & 1) ? -v : v;
}

typedef struct { uint8_t *s; uint64_t n; double score; } item_t;
static int item_cmp(const item_t *a, const item_t *b) {   /* sdscmp, sds.c:814 */
    uint64_t m = a->n < b->n ? a->n : b->n;
    int c = memcmp(a->s, b->s, m);
    if (c) return c;
    return a->n < b->n ? -1 : a->n > b->n ? 1 : 0;
}
static int zcmp_asc(const void *x, const void *y) {        /* zslInsert order, t_zset.c:132 */
    const item_t *a = (const item_t *)x, *b = (const item_t *)y;
    if (a->score < b->score) return -1;
    if (a->score > b->score) return 1;
    return item_cmp(a, b);
}
static int zcmp_desc(const void *x, const void *y) { return zcmp_asc(y, x); }
static int icmp64(const void *x, const void *y) {
    long long a = *(const long long *)x, b = *(const long long *)y;
    return a < b ? -1 : a > b;
}

static void hdr(buf_t *o, rng_t *r, uint8_t type) {
    bu8(o, type);
    bu32(o, (uint32_t)rnd_below(r, 1u << 24));
}

/* unique random members (alnum, letter first) of length in [lo,hi] */
static item_t *rand_members(rng_t *r, uint64_t n, uint64_t lo, uint64_t hi) {
    item_t *it = (item_t *)calloc(n ? n : 1, sizeof(item_t));
    for (uint64_t i = 0; i < n; i++) {
        for (;;) {
            uint64_t l = rnd_range(r, lo, hi);
            it[i].s = (uint8_t *)malloc(l ? l : 1); it[i].n = l;
            rand_alnum(r, it[i].s, l, 1);
            int dup = 0;
            for (uint64_t j = 0; j < i && !dup; j++) dup = item_cmp(&it[i], &it[j]) == 0;
            if (!dup || l == 0) break;
            free(it[i].s);
            if (l == 0) break;
        }
    }
    return it;
}
static void free_items(item_t *it, uint64_t n) { for (uint64_t i = 0; i < n; i++) free(it[i].s); free(it); }

static void gen_string(buf_t *o, rng_t *r, int enc, uint64_t len, long long ival, int alnum) {
    hdr(o, r, RR_TYPE_STRING);
    bu8(o, (uint8_t)enc);
    if (enc == RR_ENC_INT) { bu64(o, (uint64_t)ival); return; }
    bgrow(o, len);
    if (alnum) rand_alnum(r, o->p + o->n, len, 1);
    else for (uint64_t i = 0; i < len; i++) o->p[o->n + i] = (uint8_t)rnd(r);
    o->n += len;
}

/* List: quicklist entries; ints rendered via sdsll2str (rock_serdes.c:177) */
static void gen_list(buf_t *o, rng_t *r, uint64_t n, int int_pct, uint64_t slo, uint64_t shi) {
    hdr(o, r, RR_TYPE_LIST_QUICKLIST);
    for (uint64_t i = 0; i < n; i++) {
        if ((int)rnd_below(r, 100) < int_pct) {
            char buf[24]; uint32_t l = (uint32_t)ll2s(buf, rand_logint(r));
            bu32(o, l); bput(o, buf, l);
        } else {
            uint32_t l = (uint32_t)rnd_range(r, slo, shi);
            bu32(o, l); bgrow(o, l); rand_alnum(r, o->p + o->n, l, 0); o->n += l;
        }
    }
}

/* intset: sorted unique, width = the smallest that holds every member (intset.c:45) */
static void gen_intset(buf_t *o, rng_t *r, uint64_t n, unsigned width) {
    long long *v = (long long *)malloc(sizeof(long long) * (n ? n : 1));
    for (uint64_t i = 0; i < n; i++) {
        for (;;) {
            long long x;
            if (width == 2) x = (int16_t)rnd(r);
            else if (width == 4) x = (i == 0) ? (long long)(int32_t)(0x8000u | (uint32_t)rnd_below(r, 0x7FFF0000u)) * ((rnd(r) & 1) ? 1 : -1) : (int32_t)rnd(r);
            else x = (i == 0) ? (long long)(0x100000000ull + rnd_below(r, 1ull << 40)) * ((rnd(r) & 1) ? 1 : -1) : (long long)rnd(r);
            int dup = 0;
            for (uint64_t j = 0; j < i && !dup; j++) dup = v[j] == x;
            if (!dup) { v[i] = x; break; }
        }
    }
    qsort(v, n, sizeof(long long), icmp64);
    hdr(o, r, RR_TYPE_SET_INTSET);
    bu32(o, width); bu32(o, (uint32_t)n);
    for (uint64_t i = 0; i < n; i++) bput(o, &v[i], width);
    free(v);
}

static void gen_set_ht(buf_t *o, rng_t *r, uint64_t n, uint64_t lo, uint64_t hi) {
    item_t *m = rand_members(r, n, lo, hi);
    hdr(o, r, RR_TYPE_SET_HT);
    bu64(o, n);
    for (uint64_t i = 0; i < n; i++) { bu64(o, m[i].n); bput(o, m[i].s, m[i].n); }
    free_items(m, n);
}

static uint64_t rand_value_str(rng_t *r, uint8_t *d, uint64_t lo, uint64_t hi, int int_pct) {
    if ((int)rnd_below(r, 100) < int_pct) return (uint64_t)ll2s((char *)d, rand_logint(r));
    uint64_t l = rnd_range(r, lo, hi);
    rand_alnum(r, d, l, 1);
    return l;
}

/* Hash ziplist: field,value tail pushes (hashTypeSet t_hash.c:225-231) */
static void gen_hash_zl(buf_t *o, rng_t *r, uint64_t pairs, uint64_t vlo, uint64_t vhi, int int_pct) {
    zl_t z; zl_init(&z);
    uint8_t *vb = (uint8_t *)malloc(vhi + 32);
    for (uint64_t i = 0; i < pairs; i++) {
        char f[32]; int fl = snprintf(f, sizeof f, "field:%02llu", (unsigned long long)i);
        zl_push(&z, (const uint8_t *)f, (uint64_t)fl, 0);
        uint64_t vl = rand_value_str(r, vb, vlo, vhi, int_pct);
        zl_push(&z, vb, vl, 0);
    }
    zl_finish(&z);
    free(vb);
    hdr(o, r, RR_TYPE_HASH_ZIPLIST);
    bu64(o, z.b.n); bput(o, z.b.p, z.b.n);
    free(z.b.p);
}

static void gen_hash_ht(buf_t *o, rng_t *r, uint64_t pairs, uint64_t vlo, uint64_t vhi) {
    hdr(o, r, RR_TYPE_HASH_HT);
    bu64(o, pairs);
    uint8_t *vb = (uint8_t *)malloc(vhi + 32);
    for (uint64_t i = 0; i < pairs; i++) {
        char f[32]; int fl = snprintf(f, sizeof f, "field:%02llu", (unsigned long long)i);
        bu64(o, (uint64_t)fl); bput(o, f, (uint64_t)fl);
        uint64_t vl = rnd_range(r, vlo, vhi);
        rand_alnum(r, vb, vl, 0);
        bu64(o, vl); bput(o, vb, vl);
    }
    free(vb);
}

static double rand_score(rng_t *r) {
    if (rnd(r) & 1) return (double)((long long)rnd_below(r, 2000001) - 1000000);
    return rnd_unit(r) * 2e6 - 1e6;
}

/* ZSet ziplist: member, d2string(score) pairs in ascending order (zzlInsertAt t_zset.c:1029) */
static void gen_zset_zl(buf_t *o, rng_t *r, uint64_t n, uint64_t lo, uint64_t hi) {
    item_t *m = rand_members(r, n, lo, hi);
    for (uint64_t i = 0; i < n; i++) m[i].score = rand_score(r);
    qsort(m, n, sizeof(item_t), zcmp_asc);
    zl_t z; zl_init(&z);
    for (uint64_t i = 0; i < n; i++) {
        char sb[128]; int sl = d2s(sb, sizeof sb, m[i].score);
        zl_push(&z, m[i].s, m[i].n, 0);
        zl_push(&z, (const uint8_t *)sb, (uint64_t)sl, 0);
    }
    zl_finish(&z);
    hdr(o, r, RR_TYPE_ZSET_ZIPLIST);
    bu64(o, z.b.n); bput(o, z.b.p, z.b.n);
    free(z.b.p);
    free_items(m, n);
}

/* ZSet skiplist: tail->head = descending (rock_serdes.c:430-440) */
static void gen_zset_sl(buf_t *o, rng_t *r, uint64_t n, uint64_t lo, uint64_t hi) {
    item_t *m = rand_members(r, n, lo, hi);
    for (uint64_t i = 0; i < n; i++) m[i].score = rand_score(r);
    qsort(m, n, sizeof(item_t), zcmp_desc);
    hdr(o, r, RR_TYPE_ZSET_SKIPLIST);
    bu64(o, n);
    for (uint64_t i = 0; i < n; i++) { bu64(o, m[i].n); bput(o, m[i].s, m[i].n); bput(o, &m[i].score, 8); }
    free_items(m, n);
}

/* Zipf sizes in [lo, hi], P(s) ∝ 1/(s-lo+1) — inverse CDF table */
typedef struct { double *cdf; uint64_t lo, n; } zipf_t;
static void zipf_init(zipf_t *z, uint64_t lo, uint64_t hi) {
    z->lo = lo; z->n = hi - lo + 1;
    z->cdf = (double *)malloc(sizeof(double) * z->n);
    double acc = 0;
    for (uint64_t k = 0; k < z->n; k++) { acc += 1.0 / (double)(k + 1); z->cdf[k] = acc; }
    for (uint64_t k = 0; k < z->n; k++) z->cdf[k] /= acc;
}
static uint64_t zipf_draw(zipf_t *z, rng_t *r) {
    double u = rnd_unit(r);
    uint64_t a = 0, b = z->n - 1;
    while (a < b) { uint64_t m = (a + b) / 2; if (z->cdf[m] < u) a = m + 1; else b = m; }
    return z->lo + a;
}

/* config-4 proportions: 40% String (INT 10 / EMBSTR 45 / RAW 45),
 * 15% List (16, 50% ints), 15% Set (intset 16 w=2/4/8 | HT 16, 50/50),
 * 15% Hash (ziplist 16 pairs 80% | HT 16 pairs 20%), 15% ZSet (ziplist 80% | skiplist 20%). */
/* returns the descriptors the value decodes to (rr_format.h element layout), from what it
 * generated: String 1, List / intset / HT set n, hash / zset ziplist 1 + 2n, HT hash / skiplist 2n */
static uint64_t gen_mixed(buf_t *o, rng_t *r, zipf_t *zraw, uint64_t scale) {
    uint64_t t = rnd_below(r, 100), u = rnd_below(r, 100);
    uint64_t ne = 16 * scale;
    if (t < 40) {
        if (u < 10) gen_string(o, r, RR_ENC_INT, 0, rand_logint(r), 0);
        else if (u < 55) gen_string(o, r, RR_ENC_EMBSTR, rnd_range(r, 1, 44), 0, 1);
        else gen_string(o, r, RR_ENC_RAW, zipf_draw(zraw, r) * scale, 0, 1);
        return 1;
    } else if (t < 55) { gen_list(o, r, ne, 50, 1, 64); return ne; }
    else if (t < 70) {
        if (u < 50) gen_intset(o, r, ne, (unsigned[]){2, 4, 8}[rnd_below(r, 3)]);
        else gen_set_ht(o, r, ne, 1, 64);
        return ne;
    } else if (t < 85) {
        if (u < 80) { gen_hash_zl(o, r, ne, 1, 64, 25); return 1 + 2 * ne; }
        gen_hash_ht(o, r, ne, 65, 128);
        return 2 * ne;
    } else {
        if (u < 80) { gen_zset_zl(o, r, ne, 1, 64); return 1 + 2 * ne; }
        gen_zset_sl(o, r, ne, 65, 128);
        return 2 * ne;
    }
}

/* ------------------------------------------------------------------ edge cases (config 10) */
static void put_raw_blob(buf_t *o, uint8_t type, uint32_t lru, const void *body, uint64_t n) {
    bu8(o, type); bu32(o, lru); bput(o, body, n);
}
static void gen_list_items(buf_t *o, uint32_t lru, const char **items, int n) {
    bu8(o, RR_TYPE_LIST_QUICKLIST); bu32(o, lru);
    for (int i = 0; i < n; i++) { uint32_t l = (uint32_t)strlen(items[i]); bu32(o, l); bput(o, items[i], l); }
}
static void gen_edge(buf_t *o, rng_t *r, uint64_t k) {
    switch (k % 24) {
    case 0: { long long vs[] = {0, -1, (long long)0x8000000000000000ull, 0x7FFFFFFFFFFFFFFFll, 134123};
              gen_string(o, r, RR_ENC_INT, 0, vs[(k / 24) % 5], 0); break; }
    case 1: { uint64_t ls[] = {0, 1, 44}; gen_string(o, r, RR_ENC_EMBSTR, ls[(k / 24) % 3], 0, 1); break; }
    case 2: { uint64_t ls[] = {0, 44, 45, 1000, 70000}; gen_string(o, r, RR_ENC_RAW, ls[(k / 24) % 5], 0, 0); break; }
    case 3: { static const char *it[] = {"0", "12", "13", "-1", "127", "128", "-128", "-129", "32767", "32768",
                                        "-32768", "-32769", "8388607", "8388608", "-8388608", "-8388609",
                                        "2147483647", "2147483648", "-2147483648", "-2147483649",
                                        "9223372036854775807", "-9223372036854775808"};
              gen_list_items(o, (uint32_t)rnd_below(r, 1u << 24), it, 22); break; }
    case 4: { static const char *it[] = {"99999999999999999999", "-0", "+1", "01", " 1", "1 ", "",
                                        "9223372036854775808", "-9223372036854775809", "abc",
                                        "1234567890123456789012345678901"};
              gen_list_items(o, (uint32_t)rnd_below(r, 1u << 24), it, 11); break; }
    case 5: gen_list_items(o, 7, NULL, 0); break;                   /* empty list body */
    case 6: gen_intset(o, r, 1 + rnd_below(r, 40), 2); break;
    case 7: gen_intset(o, r, 1 + rnd_below(r, 40), 4); break;
    case 8: gen_intset(o, r, 1 + rnd_below(r, 40), 8); break;
    case 9: { uint8_t body[8] = {2, 0, 0, 0, 0, 0, 0, 0}; put_raw_blob(o, RR_TYPE_SET_INTSET, 1, body, 8); break; }
    case 10: { /* HT set with the empty string (rock_serdes.c:291) */
              bu8(o, RR_TYPE_SET_HT); bu32(o, 3); bu64(o, 2); bu64(o, 0); bu64(o, 1); bu8(o, 'x'); break; }
    case 11: gen_set_ht(o, r, 1000, 1, 64); break;
    case 12: { /* hash ziplist with 14-bit and 32-bit lengths, entries >= 254 B (5-byte prevlen) */
              zl_t z; zl_init(&z);
              uint64_t lens[] = {63, 64, 253, 254, 300, 16383, 16384, 20000};
              uint8_t *s = (uint8_t *)malloc(20000);
              for (int i = 0; i < 8; i++) {
                  char f[16]; int fl = snprintf(f, sizeof f, "f%d", i);
                  zl_push(&z, (uint8_t *)f, (uint64_t)fl, 0);
                  rand_alnum(r, s, lens[i], 1);
                  zl_push(&z, s, lens[i], 0);
              }
              free(s);
              zl_finish(&z);
              hdr(o, r, RR_TYPE_HASH_ZIPLIST); bu64(o, z.b.n); bput(o, z.b.p, z.b.n); free(z.b.p);
              break; }
    case 13: { /* non-minimal 5-byte prevlen for a small previous entry (cascade leftovers) */
              zl_t z; zl_init(&z);
              zl_push(&z, (const uint8_t *)"a", 1, 0);
              zl_push(&z, (const uint8_t *)"1", 1, 1);
              zl_push(&z, (const uint8_t *)"bb", 2, 1);
              zl_push(&z, (const uint8_t *)"-70000", 6, 0);
              zl_finish(&z);
              hdr(o, r, RR_TYPE_ZSET_ZIPLIST); bu64(o, z.b.n); bput(o, z.b.p, z.b.n); free(z.b.p);
              break; }
    case 14: { /* zset ziplist with inf/-inf/-0 scores */
              zl_t z; zl_init(&z);
              const char *sc[] = {"-inf", "-0", "0", "1.5", "inf", "3"};
              for (int i = 0; i < 6; i++) {
                  char m[8]; int ml = snprintf(m, sizeof m, "m%d", i);
                  zl_push(&z, (uint8_t *)m, (uint64_t)ml, 0);
                  zl_push(&z, (const uint8_t *)sc[i], strlen(sc[i]), 0);
              }
              zl_finish(&z);
              hdr(o, r, RR_TYPE_ZSET_ZIPLIST); bu64(o, z.b.n); bput(o, z.b.p, z.b.n); free(z.b.p);
              break; }
    case 15: { /* skiplist with ±inf, -0.0, tied scores */
              double sc[] = {INFINITY, 2.0, 2.0, -0.0, -INFINITY};
              const char *m[] = {"z", "b", "a", "c", "d"};
              bu8(o, RR_TYPE_ZSET_SKIPLIST); bu32(o, 42); bu64(o, 5);
              for (int i = 0; i < 5; i++) { bu64(o, 1); bput(o, m[i], 1); bput(o, &sc[i], 8); }
              break; }
    case 16: { /* hash HT with empty field and value */
              bu8(o, RR_TYPE_HASH_HT); bu32(o, 9); bu64(o, 2);
              bu64(o, 0); bu64(o, 0); bu64(o, 1); bu8(o, 'k'); bu64(o, 3); bput(o, "v\0v", 3); break; }
    case 17: { /* empty hash ziplist */
              zl_t z; zl_init(&z); zl_finish(&z);
              hdr(o, r, RR_TYPE_HASH_ZIPLIST); bu64(o, z.b.n); bput(o, z.b.p, z.b.n); free(z.b.p); break; }
    case 18: { /* binary RAW with NULs (HLL-like) */
              uint8_t b[300]; for (int i = 0; i < 300; i++) b[i] = (uint8_t)(i % 3 ? 0 : rnd(r));
              bu8(o, RR_TYPE_STRING); bu32(o, 0xFFFFFF); bu8(o, RR_ENC_RAW); bput(o, b, 300); break; }
    case 19: gen_zset_sl(o, r, 1 + rnd_below(r, 300), 1, 200); break;
    case 20: gen_hash_ht(o, r, 1 + rnd_below(r, 300), 0, 300); break;
    case 21: gen_list(o, r, 1 + rnd_below(r, 2000), 50, 0, 300); break;
    case 22: gen_hash_zl(o, r, 1 + rnd_below(r, 200), 1, 64, 50); break;
    case 23: gen_zset_zl(o, r, 1 + rnd_below(r, 64), 1, 64); break;
    }
}

/* ------------------------------------------------------------------ config 5: seekable */
/* BASELINE config 5 (100M values in config-4 proportions over 8 GPUs): value i is drawn from
 * its own seed, so any value range of the batch — one GPU's shard — can be generated alone,
 * and the sizes of all 100M values without keeping their bytes. */
static uint64_t value_seed(uint64_t seed, uint64_t i) {
    uint64_t x = seed ^ (i * 0xD1B54A32D192ED03ull);
    return splitmix(&x);
}

typedef struct {
    uint64_t v0, v1, seed;
    const zipf_t *z;
    uint64_t *bytes;    /* sizes pass: per-value blob bytes (or NULL) */
    uint32_t *descs;    /* per-value descriptor counts (or NULL) */
    buf_t out;          /* range pass: the chunk's blobs */
    uint64_t *offs;     /* range pass: v1 - v0 + 1 chunk-relative offsets */
    int keep;           /* range pass: keep the bytes */
} genjob_t;

static void *gen_worker(void *arg) {
    genjob_t *j = (genjob_t *)arg;
    buf_t tmp = {0};
    buf_t *o = j->keep ? &j->out : &tmp;
    if (j->offs) j->offs[0] = 0;
    for (uint64_t i = j->v0; i < j->v1; i++) {
        rng_t r; rng_seed(&r, value_seed(j->seed, i));
        const uint64_t start = o->n;
        const uint64_t nd = gen_mixed(o, &r, (zipf_t *)j->z, 1);
        if (j->bytes) j->bytes[i - j->v0] = o->n - start;
        if (j->descs) j->descs[i - j->v0] = (uint32_t)nd;
        if (j->offs) j->offs[i - j->v0 + 1] = o->n;
        if (!j->keep) o->n = 0;
    }
    free(tmp.p);
    return NULL;
}

static int run_jobs(genjob_t *jobs, int nt) {
    pthread_t th[64];
    int started = 0, rc = RR_API_OK;
    for (int k = 1; k < nt; k++) {
        if (pthread_create(&th[k], NULL, gen_worker, &jobs[k]) != 0) { rc = RR_API_ENOMEM; break; }
        started = k;
    }
    gen_worker(&jobs[0]);
    for (int k = 1; k <= started; k++) pthread_join(th[k], NULL);
    if (rc != RR_API_OK)   /* the jobs that never started: run them here */
        for (int k = started + 1; k < nt; k++) gen_worker(&jobs[k]);
    return RR_API_OK;
}

static int clamp_threads(int nt, uint64_t n) {
    if (nt < 1) nt = 1;
    if (nt > 64) nt = 64;
    if ((uint64_t)nt > n / 4096 + 1) nt = (int)(n / 4096 + 1);
    return nt;
}

int rr_gen_sizes(int config, uint64_t v0, uint64_t v1, uint64_t seed, uint64_t *bytes, uint32_t *descs, int nthreads) {
    if (config != 5 || v1 < v0 || (!bytes && !descs)) return RR_API_EINVAL;
    zipf_t z = {0};
    zipf_init(&z, 45, 4096);
    const uint64_t n = v1 - v0;
    const int nt = clamp_threads(nthreads, n);
    genjob_t jobs[64];
    memset(jobs, 0, sizeof jobs);
    for (int k = 0; k < nt; k++) {
        jobs[k].v0 = v0 + n * (uint64_t)k / (uint64_t)nt;
        jobs[k].v1 = v0 + n * (uint64_t)(k + 1) / (uint64_t)nt;
        jobs[k].seed = seed;
        jobs[k].z = &z;
        jobs[k].bytes = bytes ? bytes + (jobs[k].v0 - v0) : NULL;
        jobs[k].descs = descs ? descs + (jobs[k].v0 - v0) : NULL;
    }
    const int rc = run_jobs(jobs, nt);
    free(z.cdf);
    return rc;
}

int rr_gen_range(int config, uint64_t v0, uint64_t v1, uint64_t seed, rr_host_batch *out, int nthreads) {
    if (!out || config != 5 || v1 < v0) return RR_API_EINVAL;
    memset(out, 0, sizeof *out);
    zipf_t z = {0};
    zipf_init(&z, 45, 4096);
    const uint64_t n = v1 - v0;
    const int nt = clamp_threads(nthreads, n);
    genjob_t jobs[64];
    memset(jobs, 0, sizeof jobs);
    int rc = RR_API_OK;
    for (int k = 0; k < nt; k++) {
        jobs[k].v0 = v0 + n * (uint64_t)k / (uint64_t)nt;
        jobs[k].v1 = v0 + n * (uint64_t)(k + 1) / (uint64_t)nt;
        jobs[k].seed = seed;
        jobs[k].z = &z;
        jobs[k].keep = 1;
        jobs[k].offs = (uint64_t *)malloc(sizeof(uint64_t) * (jobs[k].v1 - jobs[k].v0 + 1));
        if (!jobs[k].offs) rc = RR_API_ENOMEM;
    }
    uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    if (!off) rc = RR_API_ENOMEM;
    if (rc == RR_API_OK) rc = run_jobs(jobs, nt);
    uint64_t total = 0;
    for (int k = 0; k < nt; k++) total += jobs[k].out.n;
    const uint64_t padded = (total + 15) & ~15ull;
    uint8_t *data = NULL;
    if (rc == RR_API_OK && posix_memalign((void **)&data, 64, padded ? padded : 16)) rc = RR_API_ENOMEM;
    if (rc == RR_API_OK) {
        uint64_t base = 0;
        off[0] = 0;
        for (int k = 0; k < nt; k++) {
            const uint64_t m = jobs[k].v1 - jobs[k].v0;
            if (jobs[k].out.n) memcpy(data + base, jobs[k].out.p, jobs[k].out.n);
            for (uint64_t i = 1; i <= m; i++) off[jobs[k].v0 - v0 + i] = base + jobs[k].offs[i];
            base += jobs[k].out.n;
        }
        memset(data + total, 0, padded - total);
        out->data = data; out->offsets = off; out->n = n; out->bytes = total;
    } else {
        free(off);
    }
    for (int k = 0; k < nt; k++) { free(jobs[k].out.p); free(jobs[k].offs); }
    free(z.cdf);
    return rc;
}

/* ------------------------------------------------------------------ API */
uint64_t rr_gen_default_seed(int config) { return 0x5EED0000ull + (uint64_t)config; }

int rr_gen_batch(int config, uint64_t n, uint64_t seed, rr_host_batch *out) {
    if (!out) return RR_API_EINVAL;
    memset(out, 0, sizeof *out);
    rng_t r; rng_seed(&r, seed);
    buf_t o = {0};
    uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    if (!off) return RR_API_ENOMEM;
    zipf_t zs = {0}, zr = {0};
    if (config == 2) zipf_init(&zs, 16, 4096);
    if (config == 4 || config == 5 || config == 11) zipf_init(&zr, 45, 4096);
    off[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        switch (config) {
        case 1: gen_string(&o, &r, RR_ENC_RAW, 64, 0, 0); break;
        case 2: { uint64_t s = zipf_draw(&zs, &r);
                  gen_string(&o, &r, s <= RR_EMBSTR_SIZE_LIMIT ? RR_ENC_EMBSTR : RR_ENC_RAW, s, 0, 1); break; }
        case 3: gen_hash_zl(&o, &r, 16, 1, 64, 25); break;
        case 4: gen_mixed(&o, &r, &zr, 1); break;
        case 5: {   /* seekable: value i from its own seed (rr_gen_range) */
            rng_t ri; rng_seed(&ri, value_seed(seed, i));
            gen_mixed(&o, &ri, &zr, 1);
            break; }
        case 10: gen_edge(&o, &r, i); break;
        case 11: {
            uint64_t u = rnd_below(&r, 100);
            if (u < 5) gen_string(&o, &r, RR_ENC_RAW, rnd_range(&r, 5000, 300000), 0, 0);
            else if (u < 8) gen_list(&o, &r, rnd_range(&r, 500, 3000), 50, 0, 80);
            else if (u < 11) gen_set_ht(&o, &r, rnd_range(&r, 500, 1500), 1, 40);
            else if (u < 14) gen_hash_zl(&o, &r, rnd_range(&r, 100, 600), 1, 64, 25);
            else if (u < 17) gen_zset_sl(&o, &r, rnd_range(&r, 200, 800), 1, 64);
            else if (u < 20) gen_intset(&o, &r, rnd_range(&r, 100, 512), (unsigned[]){2, 4, 8}[rnd_below(&r, 3)]);
            else gen_mixed(&o, &r, &zr, 1);
            break; }
        default:
            free(off); free(o.p); free(zs.cdf); free(zr.cdf);
            return RR_API_EINVAL;
        }
        off[i + 1] = o.n;
    }
    free(zs.cdf); free(zr.cdf);
    /* 16-byte aligned, padded to a multiple of 16 */
    uint64_t padded = (o.n + 15) & ~15ull;
    uint8_t *data = NULL;
    if (posix_memalign((void **)&data, 64, padded ? padded : 16)) { free(off); free(o.p); return RR_API_ENOMEM; }
    if (o.n) memcpy(data, o.p, o.n);
    memset(data + o.n, 0, padded - o.n);
    free(o.p);
    out->data = data; out->offsets = off; out->n = n; out->bytes = o.n;
    return RR_API_OK;
}

void rr_host_batch_free(rr_host_batch *b) {
    if (!b) return;
    free(b->data); free(b->offsets);
    memset(b, 0, sizeof *b);
}
