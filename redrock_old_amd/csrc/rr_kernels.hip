// rr_kernels.hip — CDNA4 (gfx950) decode and encode kernels for RedRock value blobs.
//
// Decode (blob batch -> flat batch): zero + count + decode launches.
//   count: thread per value, descriptor reservation + walk class, per-window reservation sums;
//   decode: workgroup per byte window (~72 KiB), its first slot from the sums, streams the
//   window into the MIRROR arena (every payload lands at its blob offset) and into LDS, sorts
//   each chunk of its values by class, walks + emits single-class batches.  Details at K1/K3.
// Encode (flat batch -> blob batch): zero + size + index + emit launches.
//   size: blob sizes and in-block offsets per 256 values; index: global offsets and the first
//   value of each 16 KiB output window; emit: workgroup per output window builds the window's
//   bytes in LDS (element-parallel tasks, aligned stores) and stores it coalesced.  Details at
//   E1-E4.
// Small batches (<= 4096 values, <= 128 KiB): one workgroup, one launch each way.
//
// No MFMA: this is byte/record work bounded by HBM.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "rr_decode_class.h"
#include "rr_device.h"
#include "rr_kernels.h"

using namespace rr;

namespace {



struct Parsed {
    uint32_t status;
    uint32_t enc;
    uint64_t n;        // descriptors
    uint64_t payload;  // payload bytes (string / ziplist bytes)
    bool unsorted;     // EMIT, skiplist: pairs not in serZset's order (descending (score, member))
};

// sdscmp (sds.c:814-824) of two byte strings
template <typename P>
__device__ __forceinline__ int sdscmp_p(P a, uint64_t la, P b, uint64_t lb) {
    const uint64_t m = la < lb ? la : lb;
    for (uint64_t x = 0; x < m; ++x) {
        const uint32_t ca = ld_u8(a + x), cb = ld_u8(b + x);
        if (ca != cb) return ca < cb ? -1 : 1;
    }
    return la < lb ? -1 : la > lb ? 1 : 0;
}

__device__ __forceinline__ void put_elem(rr_elem *e, uint64_t data, uint32_t len, uint32_t kind, uint32_t zenc) {
    uint4 w;
    w.x = (uint32_t)data;
    w.y = (uint32_t)(data >> 32);
    w.z = len;
    w.w = kind | (zenc << 8);
    *reinterpret_cast<uint4 *>(e) = w;
}

// ziplist walk, ziplist.c:300-447; bounds checked.  zl points at the ziplist (L bytes),
// zoff is its offset in the batch (arena offsets of string entries = zoff + position).
template <bool EMIT, typename P>
__device__ __forceinline__ uint32_t parse_ziplist(P zl, uint64_t L, uint64_t zoff, rr_elem *out, uint64_t &count) {
    count = 0;
    if (L < 11 || ld_u32(zl) != L) return RR_E_ZL_CORRUPT;
    uint32_t zltail = ld_u32(zl + 4);
    uint32_t zllen = ld_u8(zl + 8) | (ld_u8(zl + 9) << 8);
    uint64_t p = 10, prev_raw = 0, last = 10, n = 0;
    for (;;) {
        if (p >= L) return RR_E_ZL_CORRUPT;
        uint32_t b0 = ld_u8(zl + p);
        if (b0 == 0xFF) break;
        uint64_t pl, pls;
        if (b0 < 254) { pl = b0; pls = 1; }
        else {
            if (p + 5 > L - 1) return RR_E_ZL_CORRUPT;
            pl = ld_u32(zl + p + 1);
            pls = 5;
        }
        if (pl != prev_raw) return RR_E_ZL_CORRUPT;
        uint64_t q = p + pls;
        if (q >= L - 1) return RR_E_ZL_CORRUPT;
        uint32_t enc = ld_u8(zl + q);
        uint64_t end;
        if (enc < 0xC0) {
            uint32_t cls = enc & 0xC0;
            uint64_t ls, sl;
            if (cls == 0x00) { ls = 1; sl = enc & 0x3F; }
            else if (cls == 0x40) {
                if (q + 2 > L - 1) return RR_E_ZL_CORRUPT;
                ls = 2;
                sl = ((uint64_t)(enc & 0x3F) << 8) | ld_u8(zl + q + 1);
            } else {
                if (q + 5 > L - 1) return RR_E_ZL_CORRUPT;
                ls = 5;
                sl = ((uint64_t)ld_u8(zl + q + 1) << 24) | ((uint64_t)ld_u8(zl + q + 2) << 16) |
                     ((uint64_t)ld_u8(zl + q + 3) << 8) | ld_u8(zl + q + 4);
            }
            uint64_t d = q + ls;
            end = d + sl;
            if (end > L - 1) return RR_E_ZL_CORRUPT;
            if (EMIT) put_elem(out + n, zoff + d, (uint32_t)sl, RR_K_STR, cls);
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
            if (EMIT) {
                int64_t v;
                P x = zl + d;
                if (isz == 0) v = (int64_t)(enc & 0x0F) - 1;
                else if (isz == 1) v = (int8_t)ld_u8(x);
                else if (isz == 2) v = (int16_t)(ld_u8(x) | (ld_u8(x + 1) << 8));
                else if (isz == 3) v = ((int32_t)((ld_u8(x) << 8) | (ld_u8(x + 1) << 16) | (ld_u8(x + 2) << 24))) >> 8;
                else if (isz == 4) v = (int32_t)ld_u32(x);
                else v = (int64_t)ld_u64(x);
                put_elem(out + n, (uint64_t)v, 0, RR_K_INT, enc);
            }
        }
        ++n;
        prev_raw = end - p;
        last = p;
        p = end;
    }
    if (p != L - 1) return RR_E_ZL_CORRUPT;
    if (zllen != 0xFFFF && zllen != n) return RR_E_ZL_CORRUPT;
    if (zltail != last) return RR_E_ZL_CORRUPT;
    count = n;
    return RR_OK;
}

// desObject rock_serdes.c:538-564 and des* :133-508, on one blob at b (batch offset off).
template <bool EMIT, typename P>
__device__ __forceinline__ Parsed parse_value(P b, uint64_t off, uint64_t len, rr_elem *out) {
    Parsed r{RR_OK, 0, 0, 0, false};
    uint64_t n = 0, pay = 0;
    if (len < 5) { r.status = RR_E_SHORT; return r; }
    uint32_t type = ld_u8(b);
    uint64_t p = 5, rem = len - 5;
    uint32_t st = RR_OK;
    switch (type) {
        case RR_TYPE_STRING: {
            if (len < 6) { st = RR_E_SHORT; break; }
            uint32_t enc = ld_u8(b + 5);
            r.enc = enc;
            uint64_t rest = len - 6;
            if (enc == RR_ENC_INT) {
                if (rest != 8) { st = RR_E_STR_INTLEN; break; }
                if (EMIT) put_elem(out, ld_u64(b + 6), 0, RR_K_INT, 0);
                n = 1;
            } else if (enc == RR_ENC_RAW || enc == RR_ENC_EMBSTR) {
                if (enc == RR_ENC_EMBSTR && rest > RR_EMBSTR_SIZE_LIMIT) { st = RR_E_EMBSTR_LEN; break; }
                if (rest > 0xFFFFFFFFull) { st = RR_E_CAPACITY; break; }
                if (EMIT) put_elem(out, off + 6, (uint32_t)rest, RR_K_STR, 0);
                n = 1;
                pay = rest;
            } else st = RR_E_STR_ENC;
            break;
        }
        case RR_TYPE_LIST_QUICKLIST:
            while (rem) {
                if (rem < 4) { st = RR_E_TRUNC; break; }
                uint64_t l = ld_u32(b + p);
                p += 4;
                rem -= 4;
                if (l > rem) { st = RR_E_TRUNC; break; }
                if (EMIT) {
                    int64_t iv;
                    if (zip_try_int(b + p, (uint32_t)l, iv)) put_elem(out + n, (uint64_t)iv, 0, RR_K_INT, 0);
                    else { put_elem(out + n, off + p, (uint32_t)l, RR_K_STR, 0); pay += l; }
                }
                ++n;
                p += l;
                rem -= l;
            }
            break;
        case RR_TYPE_SET_INTSET: {
            if (rem < 8) { st = RR_E_SHORT; break; }
            uint64_t w = ld_u32(b + p), cnt = ld_u32(b + p + 4);
            p += 8;
            rem -= 8;
            if ((w != 2 && w != 4 && w != 8) || rem != w * cnt) { st = RR_E_INTSET; break; }
            r.enc = (uint32_t)w;
            if (EMIT) {
                for (uint64_t i = 0; i < cnt; ++i) {
                    P q = b + p + i * w;
                    int64_t x = w == 2 ? (int64_t)(int16_t)ld_u16(q)
                              : w == 4 ? (int64_t)(int32_t)ld_u32(q) : (int64_t)ld_u64(q);
                    put_elem(out + i, (uint64_t)x, 0, RR_K_INT, 0);
                }
            }
            n = cnt;
            break;
        }
        case RR_TYPE_SET_HT:
        case RR_TYPE_HASH_HT: {
            if (rem < 8) { st = RR_E_SHORT; break; }
            uint64_t cnt = ld_u64(b + p), got = 0;
            uint32_t per = type == RR_TYPE_SET_HT ? 1 : 2;
            p += 8;
            rem -= 8;
            while (rem && st == RR_OK) {
                for (uint32_t k = 0; k < per; ++k) {
                    if (rem < 8) { st = RR_E_TRUNC; break; }
                    uint64_t l = ld_u64(b + p);
                    p += 8;
                    rem -= 8;
                    if (l > rem) { st = RR_E_TRUNC; break; }
                    if (EMIT) put_elem(out + n, off + p, (uint32_t)l, RR_K_STR, 0);
                    ++n;
                    pay += l;
                    p += l;
                    rem -= l;
                }
                ++got;
            }
            if (st == RR_OK && got != cnt) st = RR_E_COUNT;
            break;
        }
        case RR_TYPE_HASH_ZIPLIST:
        case RR_TYPE_ZSET_ZIPLIST: {
            if (rem < 8) { st = RR_E_SHORT; break; }
            uint64_t L = ld_u64(b + p);
            p += 8;
            rem -= 8;
            if (rem != L) { st = RR_E_ZL_LEN; break; }
            uint64_t cnt;
            st = parse_ziplist<EMIT, P>(b + p, L, off + p, out + 1, cnt);
            if (st == RR_OK && (cnt & 1)) st = RR_E_ZL_CORRUPT;
            if (st != RR_OK) break;
            if (EMIT) put_elem(out, off + p, (uint32_t)L, RR_K_ZLRAW, 0);
            n = 1 + cnt;
            pay = L;
            break;
        }
        case RR_TYPE_ZSET_SKIPLIST: {
            if (rem < 8) { st = RR_E_SHORT; break; }
            uint64_t cnt = ld_u64(b + p);
            p += 8;
            rem -= 8;
            bool nan = false;
            double prev = 0.0;
            uint64_t pm = 0, pl = 0;   // previous member (position in b, length)
            for (uint64_t i = 0; i < cnt; ++i) {
                if (rem < 8) { st = RR_E_TRUNC; break; }
                uint64_t l = ld_u64(b + p);
                p += 8;
                rem -= 8;
                if (l > rem) { st = RR_E_TRUNC; break; }
                if (EMIT) put_elem(out + n, off + p, (uint32_t)l, RR_K_STR, 0);
                const uint64_t mp = p;
                pay += l;
                p += l;
                rem -= l;
                if (rem < 8) { st = RR_E_TRUNC; break; }
                const uint64_t bits = ld_u64(b + p);
                const double sc = __longlong_as_double((long long)bits);
                nan |= sc != sc;   // zslInsert serverAssert(!isnan(score)), t_zset.c:137
                if (EMIT) {
                    put_elem(out + n + 1, bits, 0, RR_K_SCORE, 0);
                    // serZset's order: descending score, then descending member (equal keys stay)
                    if (i > 0 && !r.unsorted)
                        r.unsorted = sc > prev || (sc == prev && sdscmp_p(b + pm, pl, b + mp, l) < 0);
                }
                prev = sc;
                pm = mp;
                pl = l;
                n += 2;
                p += 8;
                rem -= 8;
            }
            if (st == RR_OK && rem != 0) st = RR_E_COUNT;
            if (st == RR_OK && nan) st = RR_E_NAN;
            break;
        }
        default:
            st = RR_E_TYPE;
    }
    if (st != RR_OK) { n = 0; pay = 0; }
    r.status = st;
    r.n = n;
    r.payload = pay;
    return r;
}

// The encode's totals: E1's and E3's per-tile partials {bad, payload, descriptors} (3 words a
// tile), folded by E4's block 0 into the call's totals (zeroed by E1's block 0); bytes =
// offsets[n], or UINT64_MAX when the call's error word is set (device-side failure).
__device__ __forceinline__ void fold_totals(const uint64_t *__restrict__ stats, uint32_t ntiles,
                                            const uint64_t *__restrict__ offsets, uint64_t n, rr_totals *out,
                                            uint64_t *err) {
    __shared__ uint64_t red[3][4];
    uint64_t b = 0, p = 0, c = 0;
    for (uint32_t t = threadIdx.x; t < ntiles; t += blockDim.x) {
        b += stats[3 * (uint64_t)t + 0];
        p += stats[3 * (uint64_t)t + 1];
        c += stats[3 * (uint64_t)t + 2];
    }
    b = wave_sum(b);
    p = wave_sum(p);
    c = wave_sum(c);
    const uint32_t w = threadIdx.x / RR_WAVE;
    if (lane_id() == 0) { red[0][w] = b; red[1][w] = p; red[2][w] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t tb = 0, tp = 0, tc = 0;
        for (uint32_t k = 0; k < blockDim.x / RR_WAVE; ++k) { tb += red[0][k]; tp += red[1][k]; tc += red[2][k]; }
        if (tb) atomicAdd((unsigned long long *)&out->n_bad, (unsigned long long)tb);
        if (tp) atomicAdd((unsigned long long *)&out->payload, (unsigned long long)tp);
        if (tc) atomicAdd((unsigned long long *)&out->n_elems, (unsigned long long)tc);
        out->bytes = lb_load(err) ? ~0ull : offsets[n];
    }
}

// ---------------------------------------------------------------------------------------- decode
// Two launches, no inter-workgroup waits (a batch of one window generation: decode_kernel's ONE
// form alone, which does count_kernel's part in each window):
//   K1 count_kernel   thread per value: its descriptor reservation (rr_format.h) and its walk
//                     class (rr_decode_class.h; header checks done here), first_val per byte
//                     window, the reservations summed per window and per group of windows;
//   K3 decode_kernel  workgroup per byte window: its first slot from the window / group sums,
//                     the window's bytes into the mirror arena and an LDS stage, then per chunk
//                     of 512 values a class sort and a slot scan in LDS, and single-class batches
//                     (heaviest class first) walked from the stage by the waves; the window's
//                     marked values fixed at its end, its totals added atomically.

#ifndef RR_ABLATE   // timing-only ablations (tools/, wrong results; the decode's 1-4 below): count_kernel 5 no
#define RR_ABLATE 0       // List stage or walk, 6 the stage lands but no walk; enc_emit_kernel 7 no header,
#endif                    // length or decimal field writes, 8 no payload copies, 9 no decimals, 10 no task fields
// ---- K1: reservation + class per value ------------------------------------------------
// reserve(i) = the descriptor slots value i owns (rr_format.h): header fields only, plus the
// length chain of a List.  Equal to the decoded count for every valid blob.
template <typename P>
__device__ __forceinline__ uint64_t zl_walk_count_g(P zl, uint64_t L) {
    uint64_t p = 10, n = 0;
    while (p < L - 1 && zl[p] != 0xFF) {
        const uint64_t q = p + (zl[p] < 254 ? 1 : 5);
        if (q >= L - 1) break;
        const uint32_t enc = zl[q];
        uint64_t e;
        if (enc < 0xC0) {
            const uint32_t cls = enc & 0xC0;
            if (cls == 0x00) e = q + 1 + (enc & 0x3F);
            else if (cls == 0x40) { if (q + 2 > L - 1) break; e = q + 2 + (((uint64_t)(enc & 0x3F) << 8) | zl[q + 1]); }
            else { if (q + 5 > L - 1) break; e = q + 5 + __builtin_bswap32(ld_u32(zl + q + 1)); }
        } else if (enc == 0xFE) e = q + 2;
        else if (enc == 0xC0) e = q + 3;
        else if (enc == 0xF0) e = q + 4;
        else if (enc == 0xD0) e = q + 5;
        else if (enc == 0xE0) e = q + 9;
        else if (enc >= 0xF1 && enc <= 0xFD) e = q + 1;
        else break;
        if (e > L - 1) break;
        ++n;
        p = e;
    }
    return n;
}

// The first 24 bytes of a value as six dwords, from at most three aligned 16-byte loads
// (granules past the value's end are not read: they may lie past the padded batch), instead
// of one scattered byte load per header byte.  Bytes past the value's end are don't-cares:
// every use below is guarded by a length check, as in reserve_g / classify_g.
__device__ __forceinline__ void head24(const uint8_t *blob, uint64_t o, uint64_t b1, uint32_t (&d)[6]) {
    const uint64_t a = o & ~15ull;
    const u32x4 *g = reinterpret_cast<const u32x4 *>(blob + a);
    uint32_t h[12];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const u32x4 x = a + 16 * k < b1 ? g[k] : u32x4{0u, 0u, 0u, 0u};
        h[4 * k] = x[0]; h[4 * k + 1] = x[1]; h[4 * k + 2] = x[2]; h[4 * k + 3] = x[3];
    }
    const uint32_t q = (uint32_t)(o >> 2) & 3, sh = (uint32_t)o & 3;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t lo = q == 0 ? h[j] : q == 1 ? h[j + 1] : q == 2 ? h[j + 2] : h[j + 3];
        const uint32_t hi = q == 0 ? h[j + 1] : q == 1 ? h[j + 2] : q == 2 ? h[j + 3] : h[j + 4];
        d[j] = __builtin_amdgcn_alignbyte(hi, lo, sh);
    }
}
typedef uint32_t u32_ua __attribute__((aligned(1)));   // unaligned dword (one global_load_dword)
// a List length field: one unaligned dword load from global memory (gfx950 serves it from one
// line; an aligned pair + alignbyte measured count 52.5 -> 54.6 us), byte reads from LDS
__device__ __forceinline__ uint32_t len_u32(const uint8_t *p) { return *reinterpret_cast<const u32_ua *>(p); }
__device__ __forceinline__ uint32_t len_u32(lds_cptr p) { return ld_u32(p); }
// A List's reservation: its element count, from the chain of u32 length fields (b: the value's
// bytes, in global memory or an LDS stage)
template <typename P>
__device__ __forceinline__ uint64_t list_count(P b, uint64_t L) {
    uint64_t p = 5, n = 0;
    while (p < L) {
        if (L - p < 4) break;
        const uint64_t l = len_u32(b + p);
        if (l > L - p - 4) break;
        ++n;
        p += 4 + l;
    }
    return n;
}
// The same from a List staged in LDS (count_kernel; L < 2^32): 32-bit positions, each length
// field from two aligned dword reads and an alignbyte (one LDS round trip per element)
__device__ __forceinline__ uint32_t list_count_lds(uint32_t b, uint32_t L) {   // b: LDS byte address of byte 0
    typedef const __attribute__((address_space(3))) uint32_t *lds_u32p;
    uint32_t p = 5, n = 0;
    while (p <= L && L - p >= 4) {
        const uint32_t a = b + p, a4 = a & ~3u;
        const uint32_t lo = *(lds_u32p)(uintptr_t)a4, hi = *(lds_u32p)(uintptr_t)(a4 + 4);
        const uint32_t l = __builtin_amdgcn_alignbyte(hi, lo, a & 3);
        if (l > L - p - 4) break;
        ++n;
        p += 4 + l;
    }
    return n;
}
// The descriptor reservation (rr_format.h) and the walk class of a value from its header dwords
// (b: the value's bytes, in global memory or an LDS stage).  LIST_LATER: a List's count is left
// to the caller (count_kernel walks it from LDS), r = 0.
template <bool LIST_LATER = false, typename P>
__device__ __forceinline__ void reserve_classify(P b, uint64_t L, const uint32_t (&d)[6], uint64_t &r, uint32_t &c) {
    r = 0;
    c = C_EXACT;
    if (L < 5) return;
    const uint32_t t = d[0] & 0xFF;
    const uint32_t f5 = __builtin_amdgcn_alignbyte(d[2], d[1], 1), f9 = __builtin_amdgcn_alignbyte(d[3], d[2], 1);
    const uint32_t f13 = __builtin_amdgcn_alignbyte(d[4], d[3], 1);
    const uint64_t u5 = (uint64_t)f5 | ((uint64_t)f9 << 32);
    switch (t) {
        case RR_TYPE_STRING: {
            if (L < 6) return;
            r = 1;
            const uint32_t enc = (d[1] >> 8) & 0xFF;
            const uint64_t rest = L - 6;
            if (enc == RR_ENC_INT) c = rest == 8 ? C_STR : C_EXACT;
            else if (enc == RR_ENC_EMBSTR) c = rest <= RR_EMBSTR_SIZE_LIMIT ? C_STR : C_EXACT;
            else if (enc == RR_ENC_RAW) c = rest <= 0xFFFFFFFFull ? C_STR : C_EXACT;
            return;
        }
        case RR_TYPE_LIST_QUICKLIST: {
            c = C_LIST;
            if (!LIST_LATER) r = list_count(b, L);
            return;
        }
        default:
            break;
    }
    if (L < 13) return;
    switch (t) {
        case RR_TYPE_SET_INTSET: {
            const uint64_t w = f5, cnt = f9;
            const bool ok = (w == 2 || w == 4 || w == 8) && L - 13 == w * cnt;
            r = ok ? cnt : 0;
            c = ok ? C_IS : C_EXACT;
            return;
        }
        case RR_TYPE_SET_HT: { const uint64_t m = (L - 13) / 8; r = u5 < m ? u5 : m; c = C_HT; return; }
        case RR_TYPE_HASH_HT: { const uint64_t m = (L - 13) / 8; r = u5 > m / 2 ? m : 2 * u5; c = C_HH; return; }
        case RR_TYPE_ZSET_SKIPLIST: { const uint64_t m = (L - 13) / 16; r = 2 * (u5 < m ? u5 : m); c = C_SL; return; }
        case RR_TYPE_HASH_ZIPLIST:
        case RR_TYPE_ZSET_ZIPLIST: {
            const uint64_t Lz = u5;
            c = (L >= 24 && Lz == L - 13 && f13 == Lz) ? C_ZL : C_EXACT;
            if (Lz != L - 13 || Lz < 11) return;
            const uint64_t zllen = (d[5] >> 8) & 0xFFFF;
            if (zllen != 0xFFFF) { const uint64_t m = (Lz - 11) / 2; r = 1 + (zllen < m ? zllen : m); return; }
            r = 1 + zl_walk_count_g(b + 13, Lz);
            return;
        }
        default:
            return;
    }
}

// Block 0 also zeroes the pipeline's per-call words (look-back state, fixup header) and the
// totals: later kernels of the same stream use them, so no separate launch is needed.
__device__ __forceinline__ void zero_call_words(uint64_t *words, uint32_t nwords, rr_totals *tot) {
    if (blockIdx.x != 0) return;
    for (uint32_t k = threadIdx.x; k < nwords; k += blockDim.x) words[k] = 0;
    if (tot && threadIdx.x < 4) reinterpret_cast<uint64_t *>(tot)[threadIdx.x] = 0;
}

// Per value: its reservation (u32; a value that would need 2^32 slots fails capacity anyway),
// its class and first_val.  Per window: the reservations of its values summed into wtot[w], and
// per group of WGROUP windows into gtot[w / WGROUP] (both zero on entry: the previous call's
// count_kernel zeroed this half of the context's double buffer; this call zeroes the other).
// A window's values are consecutive, so each run of one window (group) in a wave adds its sum
// with two LDS atomics — the inclusive wave scan at its last lane, minus the exclusive scan at
// its first — into the workgroup's table of the windows (groups) it touches; the table then
// goes to global memory with one atomic per touched window (group) per workgroup.  (Global
// atomics straight from the waves serialize on the same words: ~16 waves per 72 KiB window and
// ~1K per group of config 1's 70-byte values — count 52 -> 162 us.)  decode_kernel then finds
// its first descriptor slot from at most two loads per lane (the groups before it, the windows
// before it in its group): no scan launch.
// o / win for the call's (runtime) window size without a 64-bit integer division (~50
// instructions): a double-precision reciprocal — o < 2^53, so the product is within one of the
// quotient — and one correction
__device__ __forceinline__ uint64_t div_win(uint64_t o, uint32_t win, double rcp) {
    uint64_t q = (uint64_t)((double)o * rcp);
    const int64_t rem = (int64_t)(o - q * win);
    q = rem < 0 ? q - 1 : rem >= (int64_t)win ? q + 1 : q;
    return q;
}
// The same for a batch under 4 GiB in single precision: (float)o * (1 / win) is within one of the
// quotient for o < 2^32 and win >= 1024 (relative error < 2^-22 on a quotient < 2^22), and the
// correction needs 32-bit integers only — about a third of the double form's instructions
__device__ __forceinline__ uint32_t div_win32(uint32_t o, uint32_t win, float rcpf) {
    uint32_t q = (uint32_t)((float)o * rcpf);
    const int32_t rem = (int32_t)(o - q * win);
    q = rem < 0 ? q - 1 : rem >= (int32_t)win ? q + 1 : q;
    return q;
}
constexpr uint32_t WGROUP = 16;   // (64: ~260 same-address atomics per group sum on config 1)
// (The sums are zero on entry without a zeroing launch: they are double-buffered, and each
// call's count_kernel zeroes the half the previous call used.  A zeroing kernel cost ~4.5 us a
// call, hipMemsetAsync of a size that is not a multiple of 16 bytes two fill kernels of ~4.7 us
// — a sixth of config 1's 100K-value call.  Round 4 had decode_kernel's last workgroup zero them,
// found by a returning atomic at every window's end: ~2 us of idle workgroup slot per window.)
constexpr uint32_t CNT_NT = 256, CNT_LW = CNT_NT, CNT_LG = 8;   // (a workgroup's values start in <= 256 windows)
// a wave's List stage (16 KiB a workgroup: 8 workgroups still fit a CU; measured count_kernel
// 53.5 us at 4 KiB, 53.8 at 8 KiB, 62.7 at 2 KiB; walking from global memory 58.1, with no List
// walk at all — a timing-only build — 30.9)
constexpr uint32_t CNT_LB = 4096;
template <bool W32>   // (the batch's bytes < 2^32: the window divisions in single precision)
__global__ __launch_bounds__(CNT_NT) void count_kernel(const uint8_t *__restrict__ blob,
                                                       const uint64_t *__restrict__ offsets, uint64_t n,
                                                       uint32_t *__restrict__ first_val, uint64_t *__restrict__ first_off,
                                                       uint32_t nwin, uint32_t win,
                                                       uint32_t *__restrict__ counts, uint8_t *__restrict__ cls,
                                                       uint64_t *wtot, uint64_t *gtot,
                                                       uint64_t *zero_words, uint64_t nzero, rr_totals *tot) {
    __shared__ uint64_t lw[CNT_LW], lg[CNT_LG];
    __shared__ __attribute__((aligned(16))) uint8_t lstage[CNT_NT / RR_WAVE][CNT_LB];
    if (blockIdx.x == 0 && tot && threadIdx.x < 4) reinterpret_cast<uint64_t *>(tot)[threadIdx.x] = 0;
    {   // the other half of the context's sums, for the next call: a slice per block
        const uint64_t per = (nzero + gridDim.x - 1) / gridDim.x, z0 = (uint64_t)blockIdx.x * per;
        const uint64_t z1 = z0 + per < nzero ? z0 + per : nzero;
        for (uint64_t k = z0 + threadIdx.x; k < z1; k += CNT_NT) zero_words[k] = 0;
    }
    const uint32_t tid = threadIdx.x;
    lw[tid] = 0;
    if (tid < CNT_LG) lg[tid] = 0;
    const uint64_t b0 = (uint64_t)blockIdx.x * CNT_NT;
    const uint64_t i = b0 + tid;
    const uint64_t ic = i < n ? i : n;   // (every lane stays for the wave scans; i == n: first_val's sentinel)
    // the three offsets in one round trip (loads at clamped indices, no guard branch whose join
    // made the compiler wait for the first two before issuing the third), the header granules
    // in the next, issued before the first_val stores
    const uint64_t o_hi = offsets[ic];
    const uint64_t o_lo = offsets[ic ? ic - 1 : 0];
    const uint64_t b1 = offsets[ic < n ? ic + 1 : n];
    const double rcp = W32 ? 0.0 : 1.0 / (double)win;
    const float rcpf = W32 ? 1.0f / (float)win : 0.0f;
    auto dw = [&](uint64_t o) __attribute__((always_inline)) -> uint64_t {
        return W32 ? (uint64_t)div_win32((uint32_t)o, win, rcpf) : div_win(o, win, rcp);
    };
    const uint32_t wf = (uint32_t)dw(offsets[b0 < n ? b0 : n]), gf = wf / WGROUP;   // the block's first window / group
    uint32_t d[6];
    if (i < n) head24(blob, o_hi, b1, d);
    if (i <= n) {
        // first_val[w] = first value whose first byte is at or after w*win (windows past the
        // last value start, and the sentinel nwin, get n), first_off[w] = that value's offset
        const uint64_t w_lo = i == 0 ? 0 : dw(o_lo) + 1;
        const uint64_t w_hi = i == n ? nwin : dw(o_hi);
        for (uint64_t w = w_lo; w <= w_hi && w <= nwin; ++w) {
            first_val[w] = (uint32_t)i;
            first_off[w] = o_hi;   // (its first byte: decode_kernel's stage range without an offsets round trip)
        }
    }
    uint64_t r = 0;
    uint32_t w = 0xFFFFFFFFu;   // (lanes past n: a window no value has)
    uint32_t c = C_N;
    if (i < n) {
        reserve_classify<true>(blob + o_hi, b1 - o_hi, d, r, c);
        cls[i] = (uint8_t)c;
        w = (uint32_t)dw(o_hi);
    }
    // Lists: the length chain from LDS.  The wave stages its Lists' bytes with direct-to-LDS
    // loads, CNT_LB bytes at a time (Lists in lane order, as many as fit), then each List lane
    // walks its copy: a memory round trip per pack instead of one per element (a dependent
    // global load per element made the wave's longest List its critical path).  A List longer
    // than the stage walks from global memory.
    const uint32_t lane = lane_id(), wave = tid / RR_WAVE;
#if RR_ABLATE == 5   // timing only (wrong results): no List staging, no walk
    if (i < n && c == C_LIST) r = (b1 - o_hi) >> 4;
    if (0)
#endif
    {
        const uint64_t L = b1 - o_hi, s0 = (o_hi + 5) & ~15ull;
        const bool lst = i < n && c == C_LIST && L > 5;
        const uint32_t ng = lst ? (uint32_t)((((o_hi + L + 15) & ~15ull) - s0) >> 4) : 0u;   // its granules
        if (lst && ng > CNT_LB / 16) r = list_count(blob + o_hi, L);
        uint64_t todo = __ballot(lst && ng <= CNT_LB / 16);
        while (todo) {
            const bool mine = (todo >> lane) & 1;
            const uint32_t incl = wave_incl_scan_u32(mine ? ng : 0u), ex = incl - (mine ? ng : 0u);
            const bool inpack = mine && incl <= CNT_LB / 16;   // (the first List of todo always fits)
            const uint64_t pack = __ballot(inpack);
            for (uint64_t m = pack; m; m &= m - 1) {
                const int j = __builtin_ctzll(m);
                const uint64_t sj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s0, j) |
                                    ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s0 >> 32), j) << 32);
                const uint32_t gj = (uint32_t)__builtin_amdgcn_readlane((int)ng, j);
                const uint32_t ej = (uint32_t)__builtin_amdgcn_readlane((int)ex, j);
                for (uint32_t k0 = 0; k0 < gj; k0 += RR_WAVE)
                    if (k0 + lane < gj)
                        __builtin_amdgcn_global_load_lds((const void *)(blob + sj + 16ull * (k0 + lane)),
                                                         (__attribute__((address_space(3))) void *)(lstage[wave] + 16 * (ej + k0)),
                                                         16, 0, 0);
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the pack has landed (this wave's own stage)
#if RR_ABLATE == 6   // timing only (wrong results): the stage lands, no walk
            if (inpack) r = L >> 4 | (lstage[wave][16 * ex] & 1);
            else
#endif
            if (inpack)
                r = list_count_lds((uint32_t)(uintptr_t)(lds_cptr)(lstage[wave] + 16 * ex + ((o_hi + 5) & 15)) - 5u, (uint32_t)L);
            todo &= ~pack;
        }
    }
    if (i < n) counts[i] = (uint32_t)(r < 0xFFFFFFFFull ? r : 0xFFFFFFFFull);
    const uint64_t incl = wave_incl_scan_fast(r);
    const uint32_t wp = wave_from_prev(w), wn = wave_from_next(w);
    const bool in = i < n;
    lds_barrier();   // (the tables are zero)
    // a run's sum into the table slot k (u64 adds wrap: a slot's total is its runs' sum), or
    // straight to global memory past the table (values longer than a window: rare)
    auto run_sum = [&](uint64_t *lt, uint32_t nl, uint64_t *t, uint32_t k, uint32_t k0, bool head, bool tail)
        __attribute__((always_inline)) {
        uint64_t *dst = k - k0 < nl ? lt + (k - k0) : t + k;
        if (head && tail) {
            if (r) atomicAdd((unsigned long long *)dst, (unsigned long long)r);
        } else {
            if (head && incl != r) atomicAdd((unsigned long long *)dst, (unsigned long long)(0ull - (incl - r)));
            if (tail && incl) atomicAdd((unsigned long long *)dst, (unsigned long long)incl);
        }
    };
    run_sum(lw, CNT_LW, wtot, w, wf, in & (lane == 0 || wp != w), in & (lane == RR_WAVE - 1 || wn != w));
    const uint32_t g = w / WGROUP;
    run_sum(lg, CNT_LG, gtot, g, gf, in & (lane == 0 || wp / WGROUP != g), in & (lane == RR_WAVE - 1 || wn / WGROUP != g));
    lds_barrier();
    if (lw[tid]) atomicAdd((unsigned long long *)&wtot[wf + tid], (unsigned long long)lw[tid]);
    if (tid < CNT_LG && lg[tid]) atomicAdd((unsigned long long *)&gtot[gf + tid], (unsigned long long)lg[tid]);
}

// ---- exclusive scan of u64 sizes (rr_launch_scan_u64: the snappy kernels' block lengths) ----
// 4096 values per 256-thread workgroup, tile ids from an atomic ticket (so a tile only waits
// on tiles already running), decoupled look-back between tiles (two-level, rr_device.h).
constexpr uint32_t SCAN_PER_THREAD = 16;
constexpr uint32_t SCAN_TILE = 256 * SCAN_PER_THREAD;

__global__ __launch_bounds__(256) void scan_kernel(uint64_t *__restrict__ counts, uint64_t n, uint64_t *lb,
                                                   uint32_t ntiles, uint64_t *err) {
    __shared__ uint64_t wsum[4];
    __shared__ uint64_t sh_prefix;
    __shared__ uint32_t sh_tile;
    uint64_t *ticket = lb;
    uint64_t *state = lb + 1;
    uint64_t *groups = state + ntiles;
    if (threadIdx.x == 0) sh_tile = (uint32_t)atomicAdd((unsigned long long *)ticket, 1ull);
    __syncthreads();
    const uint32_t tile = sh_tile;
    const uint64_t base = (uint64_t)tile * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_PER_THREAD;
    uint64_t x[SCAN_PER_THREAD];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER_THREAD; ++k) {
        x[k] = base + k < n ? counts[base + k] : 0;
        sum += x[k];
    }
    const uint64_t incl = wave_incl_scan_fast(sum);
    const uint32_t w = threadIdx.x / RR_WAVE;
    if (lane_id() == RR_WAVE - 1) wsum[w] = incl;
    __syncthreads();
    uint64_t wpre = 0, agg = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        if (k < w) wpre += wsum[k];
        agg += wsum[k];
    }
    if (w == 0) {
        const uint64_t pre = lookback(state, groups, tile, ntiles, agg, err);
        if (lane_id() == 0) sh_prefix = pre;
    }
    __syncthreads();
    uint64_t run = sh_prefix + wpre + incl - sum;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER_THREAD; ++k) {
        if (base + k < n) counts[base + k] = run;
        run += x[k];
    }
    if (tile == ntiles - 1 && threadIdx.x == 255) counts[n] = sh_prefix + agg;
}

// ---- K3: windows: mirror copy + class sort + single-class batches -----------------------
// per-value contribution to the window totals (returned by value: accumulators passed by
// reference were merged into one dynamically-addressed update and spilled to scratch)
struct Acc {
    uint32_t bad;
    uint64_t pay;
};

// Values whose descriptors need a whole-value pass the walks cannot make (duplicate keys of a
// hash table, re-sorting a skiplist) are marked for the window's fixup (fixup_window): FIX_MARK
// in the record's status, and a count in the window's LDS word.
constexpr uint32_t FIX_MARK_ST = 0x8000;   // (= FIX_MARK, below)
__device__ __forceinline__ uint32_t mark_fixup(uint32_t *nfix) {
    atomicAdd(nfix, 1u);
    return FIX_MARK_ST;
}

// The exact parser, lane = value v: the reference's status codes for malformed values,
// zero-filled slots, capacity handling.  src: the batch's bytes from batch offset src0 on
// (global memory, or an LDS stage); eb, r: the value's first descriptor slot and its reservation.
template <typename P>
__device__ __forceinline__ Acc exact_value(P src, uint64_t src0, uint64_t v, const uint64_t *__restrict__ offsets,
                                           uint64_t eb, uint64_t r, rr_value *__restrict__ values,
                                           rr_elem *__restrict__ elems, uint64_t cap, uint32_t *nfix) {
    uint64_t pay = 0;
    const uint64_t o_lo = offsets[v], o_hi = offsets[v + 1];
    const P b = src + (o_lo - src0);
    Parsed pr = parse_value<false, P>(b, o_lo, o_hi - o_lo, nullptr);
    uint32_t status = pr.status;
    uint64_t ne = pr.n;
    if (status == RR_OK && ne != r) status = RR_E_COUNT;
    const bool fits = eb + r <= cap;
    if (status != RR_OK) {
        ne = 0;
        if (fits)
            for (uint64_t k = 0; k < r; ++k) put_elem(elems + eb + k, 0, 0, 0, 0);
    } else if (!fits) {
        status = RR_E_CAPACITY;
    } else {
        Parsed e = parse_value<true, P>(b, o_lo, o_hi - o_lo, elems + eb);
        pay += e.payload;
        const uint32_t t = ld_u8(b);
        const uint64_t keys = t == RR_TYPE_HASH_HT ? ne / 2 : ne;
        if (((t == RR_TYPE_SET_HT || t == RR_TYPE_HASH_HT) && keys >= 2) || e.unsorted) status |= mark_fixup(nfix);
    }
    const uint32_t len = (uint32_t)(o_hi - o_lo);
    put_value(values + v, len ? ld_u8(b) : 0, pr.enc, status, len >= 5 ? ld_u32(b + 1) : 0, (uint32_t)ne,
              (uint32_t)eb);
    return Acc{(status & ~FIX_MARK_ST) != RR_OK ? 1u : 0u, pay};
}

// Values per batch of a class (a class with more values in the chunk gets several batches):
// the grouped walks give each value G = min(GMAX, 64 / count) lanes, so fewer values per batch
// means more lanes per value.  Measured: 8 or 12 ziplists per batch 3-15 % slower than 16,
// 32 ziplists 7 % slower; 8 or 16 Lists per batch within noise.
#ifndef RR_ZL_VPB
#define RR_ZL_VPB 16
#endif
#ifndef RR_HH_VPB
#define RR_HH_VPB 8
#endif
#ifndef RR_HT_VPB
#define RR_HT_VPB 16
#endif
#ifndef RR_LIST_VPB
#define RR_LIST_VPB 16
#endif
__device__ __forceinline__ uint32_t class_vpb(uint32_t c) {
    return c == C_ZL ? RR_ZL_VPB : c == C_HH ? RR_HH_VPB : c == C_HT ? RR_HT_VPB : c == C_LIST ? RR_LIST_VPB : RR_WAVE;
}
// class batch order: heaviest walks first (longest-job-first over the window's waves; hash-first
// instead of ziplist-first measured within noise)
__device__ __forceinline__ constexpr uint32_t class_at(uint32_t k) {   // {ZL, SL, HH, HT, LIST, EXACT, IS, STR}[k]
    return k == 0 ? C_ZL : k == 1 ? C_SL : k == 2 ? C_HH : k == 3 ? C_HT : k == 4 ? C_LIST : k == 5 ? C_EXACT
                                                                                              : k == 6 ? C_IS : C_STR;
}

// One single-class batch, run by the whole wave: lane < cnt (active) decodes value v (byte
// offsets relative to the source, whose byte 0 is batch offset B).  The walks run the wave in
// lock-step (rr_decode_class.h); values they reject, and the EXACT class, go to the exact
// parser lane by lane.  G lanes per value (grouped walks), this lane being lane g of its group;
// the group's lane 0 records the value (or runs the exact parser), every lane returns the
// payload of the elements it stored.  (eb_v, r_v: value v's first descriptor slot and its
// reservation, for active lanes)
template <class Src>
__device__ __forceinline__ Acc run_batch(const Src &src, uint32_t c, bool active, uint64_t v, uint32_t G, uint32_t g,
                                         uint64_t B, rsrc_t E, uint64_t eb0, const uint8_t *__restrict__ blob,
                                         const uint64_t *__restrict__ offsets, uint64_t eb_v, uint64_t r_v,
                                         rr_value *__restrict__ values, rr_elem *__restrict__ elems, uint64_t cap,
                                         uint32_t *nfix) {
    // (one exact_value call site: the parser is large and every inlined copy costs I-cache)
    bool exact = c == C_EXACT;
    Acc acc{0, 0};
    if (!exact) {
        uint64_t eb = eb0, r = 0;
        Lane l{};
        l.B = B;
        l.E = E;
        if (active) {
            const uint64_t o = offsets[v], o1 = offsets[v + 1];
            eb = eb_v;
            r = r_v;
            l.q = (uint32_t)(o - B);
            l.L = (uint32_t)(o1 - o);
            l.so = (uint32_t)(eb - eb0) * 16;
            l.r = (uint32_t)r;
            l.ok = eb + r <= cap;
        }
        Head H;
        src.template get<4>(l.q, H.h);
        uint32_t ne = 1, enc = 0;
        uint64_t vp = 0;   // this value's payload bytes (counted once it is emitted)
        bool fail = false, fixup = false;
        if (c == C_STR) {
            if (active) do_string(H, l, vp);
            enc = H.b5();
        } else if (c == C_IS) {
            do_intset_g(src, H, l, active, G, g);
            ne = H.f9();
            enc = H.f5();
        } else if (c == C_LIST) {   // grouped, software-pipelined (G a power of two)
            if (G >= 16) fail = do_list_bp<16>(src, l, active, g, ne, vp);
            else if (G >= 8) fail = do_list_bp<8>(src, l, active, g, ne, vp);
            else if (G >= 4) fail = do_list_bp<4>(src, l, active, g, ne, vp);
            else if (G >= 2) fail = do_list_bp<2>(src, l, active, g, ne, vp);
            else fail = do_list_bp<1>(src, l, active, g, ne, vp);
        } else if (c == C_HT || c == C_HH) {   // grouped (G > 1) or lane per value (do_ht)
            if (G > 1) fail = do_ht_g(src, H, l, active, G, g, ne, vp, fixup, c == C_HH);
            else fail = do_ht(src, H, l, active, ne, vp, fixup, c == C_HH);
        } else if (c == C_SL) {
            fail = do_skiplist_g(src, H, l, active, G, g, ne, vp);
        } else {   // C_ZL: grouped on one backward prevlen chain, software-pipelined (G 4, 8 or 16)
            if (G >= 16) fail = do_ziplist_bp<16>(src, l, active, g, ne, vp);
            else if (G >= 8) fail = do_ziplist_bp<8>(src, l, active, g, ne, vp);
            else fail = do_ziplist_bp<4>(src, l, active, g, ne, vp);
        }
        exact = fail;
        if (active && !fail) {
            if (g == 0) {
                const uint32_t st = !l.ok ? (uint32_t)RR_E_CAPACITY : fixup ? mark_fixup(nfix) : (uint32_t)RR_OK;
                put_value(values + v, H.type(), enc, st, H.lru(), ne, (uint32_t)eb);
                acc.bad = l.ok ? 0u : 1u;
            }
            acc.pay = l.ok ? vp : 0;
        }
        active &= g == 0;   // the exact parser runs once per value, on the group's lane 0
    }
    if (active && exact) acc = exact_value(blob, 0, v, offsets, eb_v, r_v, values, elems, cap, nfix);
    return acc;
}

struct ElemV {
    uint64_t data;
    uint32_t len;
    uint32_t kind;
};
__device__ __forceinline__ ElemV get_elem(const rr_elem *e) {
    uint4 w = *reinterpret_cast<const uint4 *>(e);
    return ElemV{(uint64_t)w.x | ((uint64_t)w.y << 32), w.z, w.w & 0xFF};
}

template <uint32_t NT>
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t x, uint64_t *wsum, uint64_t &total) {
    // (the wave scan in DPP when no lane's value reaches 2^26: the wave's sum fits 32 bits)
    const uint64_t incl = wave_incl_scan_fast(x);
    const uint32_t wv = threadIdx.x / RR_WAVE;
    if (lane_id() == RR_WAVE - 1) wsum[wv] = incl;
    lds_barrier();
    uint64_t pre = 0, t = 0;
#pragma unroll
    for (uint32_t k = 0; k < NT / RR_WAVE; ++k) {
        const uint64_t s = wsum[k];
        pre += k < wv ? s : 0;
        t += s;
    }
    total = t;
    return pre + incl - x;
}

// ---- the fixup of marked values (end of a window) ---------------------------------------
// Values whose descriptors need a whole-value pass the walks cannot make carry FIX_MARK in their
// record's status and are counted in the window's LDS word; after its batches the window's
// workgroup finds them among its value records and fixes each one with all its threads:
//   SET_HT / HASH_HT  exact duplicate-key test — fingerprints of (length, first and last 8
//                     bytes) in an LDS open-addressing table (the window's stage, now free),
//                     byte comparison on a fingerprint match; a value with more keys than fit
//                     runs in several passes, each over one residue class of the fingerprints.
//                     A hash with a repeated field gets RR_E_DUP (desHash's serverAssert,
//                     rock_serdes.c:399-400); a set keeps the first copy of each member
//                     (desSet's dictAdd, :297): later copies are marked and the descriptors
//                     compacted in place, the freed tail slots zeroed.
//   ZSET_SKIPLIST     pairs re-sorted in place into serZset's order (descending score, then
//                     member, equal keys in blob order — the skiplist desZset builds, t_zset.c:
//                     132-180) by a bitonic network over the descriptor pairs in global memory.
// Totals changes go straight into the call's totals.  Only values the walks could not clear are
// marked: none in a batch of serObject output whose hash tables hold at most HT_FP_KEYS keys,
// barring 16-bit fingerprint collisions.  (Round 3 ran this as a fourth launch over a global
// queue: 5.6 us with an empty queue.)
constexpr uint32_t FIX_MARK = FIX_MARK_ST;   // rr_value.status bit: the value awaits its fixup
constexpr uint32_t FIX_TAB = 8192, FIX_TAB_BITS = 13, FIX_PASS_KEYS = 2048;
constexpr uint32_t FIX_LDS = FIX_TAB * 8 + 64 * 8 + 64;   // table, wave sums, flag (bytes of the stage)

// 32-bit fingerprint of a member: length, first and last 8 bytes (bytes of the member only)
__device__ __forceinline__ uint32_t member_fp(const uint8_t *__restrict__ blob, uint64_t off, uint32_t len) {
    uint64_t a = 0, z = 0;
    if (len >= 8) {
        __builtin_memcpy(&a, blob + off, 8);
        __builtin_memcpy(&z, blob + off + len - 8, 8);
    } else {
        for (uint32_t i = 0; i < len; ++i) a |= (uint64_t)blob[off + i] << (8 * i);
    }
    uint64_t h = (a ^ 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (h >> 31) ^ z ^ ((uint64_t)len << 32)) * 0x94D049BB133111EBull;
    return (uint32_t)(h ^ (h >> 32));
}
__device__ __forceinline__ bool bytes_equal(const uint8_t *__restrict__ blob, uint64_t a, uint64_t b, uint32_t len) {
    uint32_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t x, y;
        __builtin_memcpy(&x, blob + a + i, 8);
        __builtin_memcpy(&y, blob + b + i, 8);
        if (x != y) return false;
    }
    for (; i < len; ++i)
        if (blob[a + i] != blob[b + i]) return false;
    return true;
}

// pair a sorts before pair b in serZset's order
__device__ __forceinline__ bool pair_before(const uint8_t *__restrict__ blob, const uint4 &am, uint64_t as,
                                            const uint4 &bm, uint64_t bs) {
    const double sa = __longlong_as_double((long long)as), sb = __longlong_as_double((long long)bs);
    if (sa != sb) return sa > sb;
    const uint64_t oa = (uint64_t)am.x | ((uint64_t)am.y << 32), ob = (uint64_t)bm.x | ((uint64_t)bm.y << 32);
    const int c = sdscmp_p(blob + oa, am.z, blob + ob, bm.z);
    if (c) return c > 0;
    return oa < ob;   // equal keys: blob order (the member's arena offset is its blob offset)
}

template <uint32_t NT>
__device__ void fix_sort_skiplist(const uint8_t *__restrict__ blob, rr_elem *__restrict__ el, uint32_t np) {
    uint4 *P = reinterpret_cast<uint4 *>(el);   // pair i = P[2i] (member), P[2i + 1] (score)
    uint32_t m = 1;
    while (m < np) m <<= 1;
    // bitonic network with every comparator ascending (first step of each merge compares
    // mirrored positions): positions >= np act as +infinity and are never touched
    for (uint32_t k = 2; k <= m; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < m / 2; t += NT) {
                uint32_t lo, hi;
                if (j == k >> 1) {
                    const uint32_t blk = t / j, o = t % j;
                    lo = blk * k + o;
                    hi = blk * k + k - 1 - o;
                } else {
                    const uint32_t blk = t / j, o = t % j;
                    lo = blk * 2 * j + o;
                    hi = lo + j;
                }
                if (hi >= np) continue;
                const uint4 am = P[2 * lo], as = P[2 * lo + 1], bm = P[2 * hi], bs = P[2 * hi + 1];
                const uint64_t sa = (uint64_t)as.x | ((uint64_t)as.y << 32), sb = (uint64_t)bs.x | ((uint64_t)bs.y << 32);
                if (pair_before(blob, bm, sb, am, sa)) {
                    P[2 * lo] = bm; P[2 * lo + 1] = bs;
                    P[2 * hi] = am; P[2 * hi + 1] = as;
                }
            }
            __syncthreads();
        }
    }
}

// One marked value v, by the whole workgroup (every thread calls it with the same v); lds:
// FIX_LDS bytes.  Clears the mark.
template <uint32_t NT>
__device__ void fixup_value(const uint8_t *__restrict__ blob, uint64_t v, rr_value *__restrict__ values,
                            rr_elem *__restrict__ elems, rr_totals *out, uint8_t *lds) {
    unsigned long long *tab = reinterpret_cast<unsigned long long *>(lds);
    uint64_t *wsum = reinterpret_cast<uint64_t *>(lds + FIX_TAB * 8);
    uint32_t *flag = reinterpret_cast<uint32_t *>(lds + FIX_TAB * 8 + 64 * 8);   // bit 0: a duplicate key,
                                                                                  // bit 1: a pass overflowed
    const uint32_t tid = threadIdx.x;
    if (tid == 0) *flag = 0;
    __syncthreads();
    const uint4 rv = reinterpret_cast<const uint4 *>(values)[v];
    const uint32_t type = rv.x & 0xFF, n = rv.z;
    rr_elem *el = elems + rv.w;
    bool drop_all = false;   // (a hash with a repeated field)
    if (type == RR_TYPE_ZSET_SKIPLIST) {
        fix_sort_skiplist<NT>(blob, el, n / 2);
    } else {
        const uint32_t per = type == RR_TYPE_SET_HT ? 1 : 2, nk = n / per;
        uint32_t K = (nk + FIX_PASS_KEYS - 1) / FIX_PASS_KEYS;
        for (;;) {
            for (uint32_t r = 0; r < K; ++r) {
                for (uint32_t j = tid; j < FIX_TAB; j += NT) tab[j] = 0;
                __syncthreads();
                for (uint32_t i = tid; i < nk; i += NT) {
                    const ElemV e = get_elem(el + (uint64_t)i * per);
                    const uint32_t fp = member_fp(blob, e.data, e.len);
                    if (fp % K != r) continue;
                    const unsigned long long ent = ((unsigned long long)fp << 32) | (i + 1u);
                    uint32_t h = (fp * 0x9E3779B1u) >> (32 - FIX_TAB_BITS), probes = 0;
                    for (;;) {
                        unsigned long long cur = tab[h];
                        if (cur == 0) {
                            cur = atomicCAS(&tab[h], 0ull, ent);
                            if (cur == 0) break;   // first of its key so far
                        }
                        if ((uint32_t)(cur >> 32) == fp) {
                            const uint32_t j = (uint32_t)cur - 1u;
                            const ElemV o = get_elem(el + (uint64_t)j * per);
                            if (o.len == e.len && bytes_equal(blob, o.data, e.data, e.len)) {
                                uint32_t later = i;
                                if (i < j) {   // this copy comes first: it takes the slot
                                    if (atomicCAS(&tab[h], cur, ent) != cur) continue;
                                    later = j;
                                }
                                // mark the later copy (rsv = 1) for compaction
                                reinterpret_cast<uint16_t *>(el + (uint64_t)later * per)[7] = 1;
                                atomicOr(flag, 1u);
                                break;
                            }
                        }
                        h = (h + 1) & (FIX_TAB - 1);
                        if (++probes == FIX_TAB) { atomicOr(flag, 2u); break; }
                    }
                }
                __syncthreads();
                if (*flag & 2) break;
            }
            if (!(*flag & 2)) break;
            K *= 2;   // a residue class overflowed the table: finer classes (marks stay valid)
            __syncthreads();
            if (tid == 0) *flag &= ~2u;
            __syncthreads();
        }
        if (*flag & 1) {
            // compact the kept descriptors forward (a chunk is read before it is written, and
            // writes never pass the chunk's own positions), zero the freed tail
            drop_all = per == 2;
            uint64_t kept = 0, dropped = 0;
            for (uint32_t c0 = 0; c0 < n; c0 += NT) {
                const uint32_t i = c0 + tid;
                uint4 d = make_uint4(0, 0, 0, 0);
                if (i < n) d = reinterpret_cast<const uint4 *>(el)[i];
                const bool keep = i < n && (per == 2 || (d.w >> 16) == 0);
                uint64_t tot;
                const uint64_t pos = block_excl_scan<NT>(keep ? 1u : 0u, wsum, tot);
                dropped += i < n && !keep ? d.z : 0;
                __syncthreads();
                if (keep && per == 1) reinterpret_cast<uint4 *>(el)[kept + pos] = d;
                if (per == 2 && i < n) dropped += d.z;   // a hash with a repeated field loses all
                kept += tot;
                __syncthreads();
            }
            const uint32_t nk2 = per == 2 ? 0u : (uint32_t)kept;
            for (uint32_t i = nk2 + tid; i < n; i += NT) reinterpret_cast<uint4 *>(el)[i] = make_uint4(0, 0, 0, 0);
            dropped = wave_sum(dropped);
            if (lane_id() == 0 && dropped && out)
                atomicAdd((unsigned long long *)&out->payload, (unsigned long long)(0ull - dropped));
            if (tid == 0) {
                uint4 w = rv;
                w.z = nk2;
                if (per == 2 && out) atomicAdd((unsigned long long *)&out->n_bad, 1ull);
                w.x = (rv.x & 0xFFFFu) | ((per == 2 ? (uint32_t)RR_E_DUP : (uint32_t)RR_OK) << 16);
                reinterpret_cast<uint4 *>(values)[v] = w;
            }
        }
    }
    if (tid == 0 && !drop_all && !(*flag & 1)) {   // the mark cleared (the status is RR_OK)
        uint4 w = rv;
        w.x = rv.x & 0xFFFFu;
        reinterpret_cast<uint4 *>(values)[v] = w;
    }
    __syncthreads();
}

// The window's marked values [v_lo, v_hi): found by their records' status (every thread one
// value per round, a ballot and an LDS list), fixed one by one.  The caller makes the window's
// record and descriptor stores visible to the workgroup first (__syncthreads).
template <uint32_t NT>
__device__ void fixup_window(const uint8_t *__restrict__ blob, uint64_t v_lo, uint64_t v_hi,
                             rr_value *__restrict__ values, rr_elem *__restrict__ elems, rr_totals *out,
                             uint8_t *lds) {
    uint32_t *list = reinterpret_cast<uint32_t *>(lds + FIX_LDS);   // NT + 1 words past the fixup's own
    for (uint64_t r0 = v_lo; r0 < v_hi; r0 += NT) {
        if (threadIdx.x == 0) list[NT] = 0;
        __syncthreads();
        const uint64_t v = r0 + threadIdx.x;
        if (v < v_hi && ((reinterpret_cast<const uint4 *>(values)[v].x >> 16) & FIX_MARK))
            list[atomicAdd(&list[NT], 1u)] = threadIdx.x;
        __syncthreads();
        const uint32_t m = list[NT];
        for (uint32_t k = 0; k < m; ++k) fixup_value<NT>(blob, r0 + list[k], values, elems, out, lds);
    }
}

// a wave-uniform 64-bit value into SGPRs
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    return (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)x) |
           ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32);
}

// Probe build (tools/probe_decode.py, -DRR_PROBE): per-window phase cycles and per-class batch
// cycles / counts / lanes into a buffer set by rr_probe_set (PROBE_WORDS u64 per window).
// Diagnostics only; the product build has none of it.
#ifdef RR_PROBE
constexpr uint32_t PROBE_WORDS = 37;   // ([32, 36): the one-launch form's phases, [36] batch start -> offsets)
__device__ uint64_t *g_probe;
extern "C" int rr_probe_set(void *p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_probe), &p, sizeof(p)) == hipSuccess ? 0 : -1; }
#define PROBE(...) __VA_ARGS__
#else
#define PROBE(...)
#endif
// Timing-only ablations (tools/, wrong results): -DRR_ABLATE=1 copy + stage only, 2 + the class
// sort (no batches), 3 no arena copy, 4 no descriptor stores (rr_decode_class.h).

// Window granules (16 B) per thread loaded before the first_val -> offsets / class-byte loads
// (the rest after the class bytes): measured 8 before 6 % slower, none before 2 % slower.
constexpr uint32_t DEC_KE = 2;
// Two 512-thread workgroups per CU = 4 waves per SIMD, so at most 128 VGPRs: the allocator is
// told so (left to itself it takes 137 for the hash-table walk and the CU holds one workgroup).
constexpr int DEC_WPE = 4;

// The one-launch decode's words in the context's sums (zero on entry, zero again when the call's
// last window is done): [6] a wait that never ended (the error word), then per window its
// look-back word (ONE_RUN once it runs, ONE_AGG | its reservations once it knows them) and its
// end word (ONE_AGG | n_bad << 40 | payload).
constexpr uint32_t ONE_HDR = 8;
constexpr uint64_t ONE_AGG = 1ull << 63, ONE_RUN = 1ull << 62, ONE_VAL = ONE_RUN - 1;
__host__ __device__ constexpr uint64_t one_words(uint64_t nwin) { return ONE_HDR + 2 * nwin; }

// The window's values [v[0], v[1]) and their first offsets f[0], f[1]: count_kernel's first_val
// of the window and of the next, i.e. min{i <= n : i == n or offsets[i] >= T} for T = tile * win
// and (tile + 1) * win.  Round 1 reads NT consecutive offsets from just before the guess
// n * T / data_cap (exact for evenly sized values: config 1's windows resolve both bounds in this
// one round, and the window's own offsets come out of the same samples, a[0, NT) from position
// *base); a bound outside them narrows by NT / 2 samples a round.  a: 3 * NT u64 of LDS,
// cnt: 2 * NW u64.
// issue(): the caller's loads, issued right behind the first samples (vmcnt retires in order, so
// the samples are waited for without them).
template <uint32_t NT, typename F>
__device__ __forceinline__ void one_locate(const uint64_t *__restrict__ offsets, uint64_t n, uint32_t win,
                                           uint64_t data_cap, uint32_t tile, uint64_t on, uint64_t *a, uint64_t *cnt,
                                           uint64_t (&v)[2], uint64_t (&f)[2], uint64_t &base, F &&issue) {
    constexpr uint32_t H = NT / 2, NWV = NT / RR_WAVE;
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid / RR_WAVE;
    const uint64_t T[2] = {(uint64_t)tile * win, (uint64_t)(tile + 1) * win};
    const uint64_t g = (uint64_t)((double)n * (double)T[0] / (double)(data_cap ? data_cap : 1));
    base = rfl64(g > NT / 8 ? (g - NT / 8 < n ? g - NT / 8 : n) : 0);
    const uint64_t q1 = base + tid < n ? base + tid : n;
    const uint64_t a1 = q1 < n ? offsets[q1] : on;
    issue();
    a[tid] = a1;
    const uint64_t m0 = __ballot(q1 < n && a1 < T[0]), m1 = __ballot(q1 < n && a1 < T[1]);
    if (lane == 0) cnt[wave] = (uint64_t)__popcll(m0) | ((uint64_t)__popcll(m1) << 32);
    lds_barrier();
    uint64_t lo[2], hi[2], oh[2];
    {
        uint32_t c[2] = {0, 0};
#pragma unroll
        for (uint32_t w = 0; w < NWV; ++w) { c[0] += (uint32_t)cnt[w]; c[1] += (uint32_t)(cnt[w] >> 32); }
#pragma unroll
        for (int k = 0; k < 2; ++k) {   // (position j of the samples: min(base + j, n))
            const uint64_t qc = base + c[k] < n ? base + c[k] : n;
            lo[k] = c[k] ? qc : 0;   // (samples 0 .. c - 1 lie below T: the bound is past them)
            hi[k] = c[k] < NT ? qc : n;
            oh[k] = rfl64(c[k] < NT ? a[c[k]] : on);
        }
    }
    // later rounds (rare): threads [0, H) search T[0], [H, NT) T[1]; buffers 1 and 2 alternate
    for (uint32_t r = 1; lo[0] < hi[0] || lo[1] < hi[1]; ++r) {
        const uint32_t k = tid / H, j = tid % H, b = 1 + (r & 1);
        const uint64_t span = hi[k] - lo[k];
        const uint64_t p = span <= H ? lo[k] + j : lo[k] + span * j / H;
        const bool valid = p < hi[k];
        const uint64_t x = valid ? offsets[p] : 0;
        a[b * NT + tid] = x;
        const uint64_t m = __ballot(valid && x < T[k]);
        if (lane == 0) cnt[(r & 1) * NWV + wave] = (uint64_t)__popcll(m);
        lds_barrier();
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            if (lo[kk] >= hi[kk]) continue;
            uint32_t c = 0;
#pragma unroll
            for (uint32_t w = 0; w < NWV / 2; ++w) c += (uint32_t)cnt[(r & 1) * NWV + kk * (NWV / 2) + w];
            const uint64_t sp = hi[kk] - lo[kk];
            const uint32_t nv = sp <= H ? (uint32_t)sp : H;   // the valid samples
            auto pos = [&](uint32_t q) { return sp <= H ? lo[kk] + q : lo[kk] + sp * q / H; };
            const uint64_t nlo = c ? pos(c - 1) + 1 : lo[kk];
            if (c < nv) { hi[kk] = rfl64(pos(c)); oh[kk] = rfl64(a[b * NT + kk * H + c]); }
            lo[kk] = rfl64(nlo);
        }
    }
    v[0] = rfl64(lo[0]); v[1] = rfl64(lo[1]);
    f[0] = oh[0]; f[1] = oh[1];
}

// The same bound by one wave alone, 64 samples a round (the look-back's help below)
__device__ __forceinline__ uint64_t wave_lower_bound(const uint64_t *__restrict__ offsets, uint64_t n, uint64_t T) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t sp = hi - lo;
        const uint32_t j = lane_id(), nv = sp <= RR_WAVE ? (uint32_t)sp : RR_WAVE;
        auto pos = [&](uint32_t q) { return sp <= RR_WAVE ? lo + q : lo + sp * q / RR_WAVE; };
        const uint64_t p = pos(j);
        const uint32_t c = (uint32_t)__popcll(__ballot(j < nv && offsets[p] < T));
        const uint64_t nlo = c ? pos(c - 1) + 1 : lo;
        if (c < nv) hi = pos(c);
        lo = nlo;
    }
    return lo;
}

// A window's reservations (unsaturated, as count_kernel's window sums), by one wave from global
// memory: the look-back's help for a window that has not started (its workgroup not yet
// dispatched), so that a window never waits on one that is not running.
__device__ uint64_t one_window_sum(const uint8_t *__restrict__ blob, const uint64_t *__restrict__ offsets, uint64_t n,
                                   uint32_t win, uint32_t p) {
    const uint64_t v0 = wave_lower_bound(offsets, n, (uint64_t)p * win);
    const uint64_t v1 = wave_lower_bound(offsets, n, (uint64_t)(p + 1) * win);
    uint64_t sum = 0;
    for (uint64_t v = v0 + lane_id(); v < v1; v += RR_WAVE) {
        const uint64_t o = offsets[v], o1 = offsets[v + 1];
        uint32_t d[6], c;
        uint64_t r;
        head24(blob, o, o1, d);
        reserve_classify(blob + o, o1 - o, d, r, c);
        sum += r;
    }
    return wave_sum(sum);
}

// Workgroup per byte WINDOW of W bytes: window t owns the values whose first byte lies in
// [t*W, (t+1)*W) (first_val from K1).  The workgroup
//   1. loads the window (buffer resources: no exec-mask branches; loads past the range read
//      zeros, stores past it are dropped, unstaged granules go to a dummy LDS slot) and the tail
//      of its last value (up to SLACK more) while it
//   2. counting-sorts a chunk of <= PMAX of its values by class in LDS (the sort reads no
//      global memory, so none of its waits drain the loads), then writes the window to the
//      mirror arena (nontemporal) and the LDS stage;
//   3. its waves take single-class batches of <= 64 values, heaviest class first, and walk +
//      emit them from LDS (from global memory when the values did not fit the stage).
// Every barrier orders LDS only (lds_barrier): __syncthreads() would make each wave wait for
// the acknowledgement of its streaming arena stores.
//
// Descriptor slots: the window's first slot eb0 is the sum of count_kernel's totals of the
// windows before it (two loads per lane: the groups before its group, the windows before it in
// its group); each chunk scans its values' reservations in LDS (eloc) while it sorts them, so
// no scan launch runs between count_kernel and this kernel.
//
// ONE (a batch of one generation of windows, no count_kernel): the window finds its values by
// two lower-bound searches of offsets (one_locate), classifies them from its stage itself
// (count_kernel's rule) and finds its first slot by a flat look-back over the earlier windows'
// words, waiting only on windows that run (one not dispatched yet is summed here); each window
// stores its totals in its end word and the last window stores the call's totals and leaves the
// words zero (one_words).
template <uint32_t W, uint32_t SLACK, uint32_t NW, uint32_t PMAX, bool ONE = false>
__global__ __launch_bounds__(NW * RR_WAVE) __attribute__((amdgpu_waves_per_eu(DEC_WPE))) void decode_kernel(
    const uint8_t *__restrict__ blob, uint64_t data_cap, const uint64_t *__restrict__ offsets, uint64_t n,
    const uint32_t *__restrict__ first_val, const uint64_t *__restrict__ first_off, uint8_t *__restrict__ cls, uint32_t *__restrict__ counts,
    const uint64_t *wtot, const uint64_t *gtot, rr_value *__restrict__ values,
    rr_elem *__restrict__ elems, uint64_t elem_cap, uint8_t *__restrict__ arena, uint32_t nwin, uint32_t win,
    rr_totals *tot, uint64_t *one, uint64_t *zero_words, uint64_t nzero, uint32_t help_all) {
    constexpr uint32_t NT = NW * RR_WAVE, STAGE = W + SLACK;
    static_assert(PMAX == NT, "a chunk is one value per thread (the slot scan)");
    static_assert(W % 16 == 0 && SLACK % 16 == 0, "tile shape");
    static_assert(FIX_LDS + 4 * (NT + 1) <= STAGE, "the fixup reuses the stage");
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE + 64];
    __shared__ uint32_t nfix;             // values of the window marked for the fixup
    __shared__ uint16_t perm[PMAX];
    __shared__ uint32_t eloc[PMAX + 1];   // chunk-relative first slot of each value, then the chunk's slots
    __shared__ uint64_t wpart[2][NW];     // wave sums: [0] the window's first slot, [1] the chunk's slot scan
    __shared__ uint32_t ccount[C_N], cbase[C_N], wcnt[NW][C_N];
    __shared__ uint64_t bend;   // the batch prefix ends in batch order, a byte each (<= 72 batches a chunk)
    __shared__ uint32_t next_batch;
    __shared__ uint64_t red[2][NW];
    PROBE(__shared__ uint64_t prb[PROBE_WORDS]; uint64_t pt0 = __builtin_amdgcn_s_memtime(), pt1 = 0, pt2 = 0;
          const uint64_t prt0 = __builtin_amdgcn_s_memrealtime(); uint64_t pa = 0, pb = 0, pc = 0, pd = 0, pe = 0; uint32_t pit = 0;
          if (threadIdx.x < PROBE_WORDS) prb[threadIdx.x] = 0;)
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid / RR_WAVE;
    // (A persistent form — the resident grid walking windows b, b + grid, ..., no workgroup
    // teardown and dispatch between a CU slot's windows, ~1.6 us of idle slot each — costs 61
    // spilled VGPRs at the 128 cap, a 2-window unrolled form 57: decode_kernel 285 -> 366 us,
    // round 6, profiles/r6_decode_persist_ab.txt.)
    const uint32_t tile = blockIdx.x;
    if (tid == 0) nfix = 0;   // (ordered before the batches by the sort's first barrier)
    __shared__ rr_totals s_fix;   // (ONE: the fixup's adjustments of the window's totals)
    if (ONE && tid < 4) reinterpret_cast<uint64_t *>(&s_fix)[tid] = 0;
    uint64_t *const state = one + ONE_HDR, *const fin = state + nwin;   // (ONE)
    const uint64_t W0 = (uint64_t)tile * win;   // (win <= W: the call's window size, launch_decode)
    constexpr uint32_t KM = W / 16 / NT;   // granules per thread of a whole window
    static_assert(W % 16 == 0 && W % (16 * NT) == 0, "window granules per thread");
    u32x4 ov_m[KM];
    uint64_t pre = 0, padded, W1, A0, ov_a, v_lo, v_hi, f_lo, f_hi, sbase = 0;
    uint32_t ov_mb;
    rsrc_t ov_RM;
    uint32_t cls0 = C_N, cnt0 = 0;
    if constexpr (ONE) {
        if (tid == 0) lb_store(&state[tile], ONE_RUN);   // (the look-back waits only on windows that run)
        // count_kernel's other duty: the other half of the context's sums, a slice per window
        const uint64_t per = (nzero + gridDim.x - 1) / gridDim.x, z0 = (uint64_t)blockIdx.x * per;
        const uint64_t z1 = z0 + per < nzero ? z0 + per : nzero;
        for (uint64_t k = z0 + tid; k < z1; k += NT) zero_words[k] = 0;
        // the window's granules [W0, W0 + win) go out right behind the search's first samples
        // (bounded by data_cap, not offsets[n]: no round trip first; granules past the batch are
        // not staged and their arena stores are dropped, below)
        const uint64_t LE = W0 + win < data_cap ? W0 + win : data_cap;
        ov_a = W0 >> 4;
        ov_mb = LE > W0 ? (uint32_t)(LE - W0) : 0u;
        ov_RM = make_rsrc(blob + W0, ov_mb);
        const uint64_t on = offsets[n];
        uint64_t vv[2], ff[2];
        one_locate<NT>(offsets, n, win, data_cap, tile, on, reinterpret_cast<uint64_t *>(stage), &wpart[0][0], vv, ff,
                       sbase, [&]() __attribute__((always_inline)) {
#pragma unroll
                           for (uint32_t k = 0; k < KM; ++k)
                               ov_m[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                       ov_RM, (int)((tid + k * NT) * 16), 0, 0));
                       });
        PROBE(pa = __builtin_amdgcn_s_memtime();)
        v_lo = vv[0]; v_hi = vv[1]; f_lo = ff[0]; f_hi = ff[1];
        padded = (on + 15) & ~15ull;
        W1 = W0 + win < padded ? W0 + win : padded;
        A0 = W0 > (offsets[0] & ~15ull) ? W0 : (offsets[0] & ~15ull);
    } else {
        // 0. the loads of the window's first slot go out first (reduced under the sort)
        const uint32_t grp = tile / WGROUP, gi = tile % WGROUP;
        pre = tid < gi ? wtot[(uint64_t)grp * WGROUP + tid] : 0;
        for (uint32_t k = tid; k < grp; k += NT) pre += gtot[k];
        padded = (offsets[n] + 15) & ~15ull;
        W1 = W0 + win < padded ? W0 + win : padded;
        // the arena copy starts at the call's first value (a call over a slice of a larger buffer —
        // the chunks of rr_decode_batch_host — copies only its own bytes); the stage always lies
        // past it (S0 >= offsets[v_lo] >= offsets[0])
        A0 = W0 > (offsets[0] & ~15ull) ? W0 : (offsets[0] & ~15ull);
        // the window's own granules [A0, W1) first: their range needs only offsets[0] and
        // offsets[n], not first_val -> offsets, so the loads go out at the window's start; the
        // stage's tail [W1, ov_te) (the last values' bytes past the window) follows.  The arena
        // gets [A0, W1) (stores past it are dropped); granule A0 / 16 + tid + k * NT is at byte
        // offset 16 (tid + k NT)
        ov_a = A0 >> 4;
        ov_mb = (W1 >> 4) > ov_a ? (uint32_t)(((W1 >> 4) - ov_a) * 16) : 0u;
        ov_RM = make_rsrc(blob + A0, ov_mb);
        // KE granules per thread go out before the first_val -> offsets / class-byte loads, the
        // rest after the class bytes: the sort waits (vmcnt, in issue order) for the class bytes
        // and therefore for the early granules only
        constexpr uint32_t KE = DEC_KE < KM ? DEC_KE : KM;
#pragma unroll
        for (uint32_t k = 0; k < KE; ++k)
            ov_m[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ov_RM, (int)((tid + k * NT) * 16), 0, 0));
        // (the values' first offsets come with first_val: one round trip, not first_val -> offsets)
        v_lo = first_val[tile]; v_hi = first_val[tile + 1];
        f_lo = first_off[tile]; f_hi = first_off[tile + 1];
        // the first chunk's class bytes and reservations, loaded before the rest of the window so
        // their latency hides under it
        cls0 = v_lo + tid < v_hi ? (uint32_t)cls[v_lo + tid] : C_N;
        cnt0 = v_lo + tid < v_hi ? counts[v_lo + tid] : 0u;
#pragma unroll
        for (uint32_t k = KE; k < KM; ++k)
            ov_m[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ov_RM, (int)((tid + k * NT) * 16), 0, 0));
    }
    const uint64_t ov_w1 = W1 >> 4;
    // the arena gets [A0, W1): in the ONE form the loads start at W0, so granules below A0 (the
    // call's first value, in window 0 or in a slice of a larger buffer) are dropped
    const rsrc_t ov_RA = make_rsrc(arena + ov_a * 16, ov_w1 > ov_a ? (uint32_t)((ov_w1 - ov_a) * 16) : 0u);
    uint64_t S0 = W0, S1 = W0;
    if (v_hi > v_lo) {
        S0 = f_lo & ~15ull;
        S1 = (f_hi + 15) & ~15ull;
    }
    // the stage's tail [W1, S1) comes from KT granules per thread past the window; a window is
    // staged when its values' bytes [S0, S1) fit the stage and its tail fits those granules (a
    // call window smaller than W leaves stage room unused: a longer tail walks from global
    // memory)
    constexpr uint32_t KT = (SLACK / 16 + NT - 1) / NT;
    const uint64_t ov_t0 = ov_w1 > ov_a ? ov_w1 : ov_a;
    const bool staged = S1 - S0 <= STAGE && (S1 >> 4) <= ov_t0 + (uint64_t)KT * NT;
    const uint64_t cap = elem_cap < 0xFFFFFFFFull ? elem_cap : 0xFFFFFFFFull;   // elem_base is 32-bit
    // (ONE: the first chunk's offsets, from the search's first samples when they hold them)
    uint64_t o_v = 0, o_v1 = 0;
    if constexpr (ONE) {
        const uint64_t *a = reinterpret_cast<const uint64_t *>(stage);
        const uint64_t i0 = v_lo + tid < n ? v_lo + tid : n, i1 = v_lo + tid + 1 < n ? v_lo + tid + 1 : n;
        o_v = i0 >= sbase && i0 - sbase < NT ? a[i0 - sbase] : offsets[i0];
        o_v1 = i1 >= sbase && i1 - sbase < NT ? a[i1 - sbase] : offsets[i1];
    }
    // the stage's tail, also in flight under the sort
    const uint64_t ov_te = (staged && S1 > W1 ? S1 : W1) >> 4;
    const rsrc_t ov_RT = make_rsrc(blob + ov_t0 * 16, ov_te > ov_t0 ? (uint32_t)((ov_te - ov_t0) * 16) : 0u);
    u32x4 ov_t[KT];
#pragma unroll
    for (uint32_t k = 0; k < KT; ++k)
        ov_t[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ov_RT, (int)((tid + k * NT) * 16), 0, 0));

    if constexpr (!ONE) {
        pre = wave_sum_fast(pre);
        if (lane == 0) wpart[0][wave] = pre;   // (read after the sort's first barrier)
    }
    auto first_slot = [&]() __attribute__((always_inline)) {
        uint64_t s = 0;
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) s += wpart[0][w];
        return s;
    };
    const uint64_t ov_s0 = S0 >> 4;
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    lds_u32x4 *ov_lds = (lds_u32x4 *)(__attribute__((address_space(3))) uint8_t *)stage;
    // granule g's stage slot, or the dummy slot just past the stage (reads past the stage see
    // garbage there, which the walks never use: every read is checked against its value's end)
    auto ov_slot = [&](uint64_t g) __attribute__((always_inline)) -> uint32_t {
        return (staged & (g >= ov_s0) & (g < ov_te)) ? (uint32_t)(g - ov_s0) : STAGE / 16;
    };
    // the window's loads have landed (under the sort): arena stores, LDS stage writes
    auto ov_finish = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t k = 0; k < KM; ++k) {
            // (a window smaller than W: the main loads' granules past W1 read zeros, and the
            // tail loads bring those stage slots)
            const uint64_t g = ov_a + tid + (uint64_t)k * NT;
            // (ONE: granules below A0 go to an offset past the resource, which drops the store)
            const int so = ONE && g < (A0 >> 4) ? 0x7FFFFFF0 : (int)((tid + k * NT) * 16);
            if (RR_ABLATE != 3) __builtin_amdgcn_raw_buffer_store_b128(ov_m[k], ov_RA, so, 0, 2 /* nt */);
            ov_lds[g < ov_w1 ? ov_slot(g) : STAGE / 16] = ov_m[k];
        }
        // the stage's tail [W1, ov_te): LDS only
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k) ov_lds[ov_slot(ov_t0 + tid + (uint64_t)k * NT)] = ov_t[k];
    };

    // values that do not fit the stage are read from global memory; if even their 32-bit
    // window-relative byte or slot offsets could overflow, the exact parser takes them (the
    // slots bounded as rr_decode_elem_bound does: a value's descriptors past its first take >= 2
    // bytes each; a staged window never comes near)
    const bool far = (!staged && S1 - S0 > 0xFFFFFF00ull) || ((S1 - S0) / 2 + (v_hi - v_lo)) * 16 >= NOSLOT;
    const LdsSrc lsrc{(lds_cptr)stage};
    const GlbSrc gsrc{make_rsrc(blob + S0, (uint32_t)(data_cap - S0 < 0xFFFFFFFFull ? data_cap - S0 : 0xFFFFFFFFull))};
    // ONE: a value's reservation and class (count_kernel's rule: reserve_classify, a List's
    // length chain) from the stage once it has landed, or from global memory for a window that
    // is not staged
    auto one_class = [&](uint64_t o, uint64_t o1, uint64_t &r, uint32_t &c) __attribute__((always_inline)) {
        uint32_t d[6];
        if (staged) {
            const uint32_t q = (uint32_t)(o - S0);
            lsrc.get<6>(q, d);   // (reads up to 28 bytes past q: inside the stage's slack)
            reserve_classify(lsrc.S + q, o1 - o, d, r, c);
        } else {
            head24(blob, o, o1, d);
            reserve_classify(blob + o, o1 - o, d, r, c);
        }
    };

    uint64_t bad = 0, pay = 0, eb0 = 0, run = 0;   // run: the slots of the earlier chunks
    const uint64_t v_end = RR_ABLATE == 1 ? v_lo : v_hi;
    // 2. counting sort of a chunk of values by class into perm, class bases and batch prefixes,
    //    and the scan of the chunk's reservations into eloc (returns the chunk's slots).  One
    //    barrier: each wave's class counts go to LDS (a ballot per class), then every wave finds
    //    its own class bases from them (lane c: class c's total and its part in earlier waves, the
    //    bases in batch order by readlane) and places its values with no atomics (three barriers
    //    and a returning LDS atomic per class and wave before: config 1's one-launch windows sort
    //    in 3.9K cycles instead of 5.6K; config 4 at 1M values 0.348-0.353 -> 0.332-0.334 ms).
    auto sort_chunk = [&](uint64_t c0) __attribute__((always_inline)) -> uint64_t {
        const uint32_t nv = (uint32_t)(v_hi - c0 < PMAX ? v_hi - c0 : PMAX);
        if (tid == 0) next_batch = 0;
        PROBE(if (c0 == v_lo) pt1 = __builtin_amdgcn_s_memtime();)
        const uint32_t i = tid;
        // (ONE: a later chunk's classes and reservations were stored by the window's first pass)
        const uint32_t ci = c0 == v_lo ? cls0 : i < nv ? (uint32_t)cls[c0 + i] : C_N;
        const uint32_t ri = c0 == v_lo ? cnt0 : i < nv ? counts[c0 + i] : 0u;
        const uint32_t myc = i < nv ? (far ? C_EXACT : ci) : C_N;
        uint32_t cntc = 0;   // lane c < C_N: this wave's values of class c
        uint64_t mm = 0;     // the wave's ballot of my class
#pragma unroll
        for (uint32_t c = 0; c < C_N; ++c) {
            const uint64_t m = __ballot(myc == c);
            cntc = lane == c ? (uint32_t)__popcll(m) : cntc;
            mm = myc == c ? m : mm;
        }
        if (lane < C_N) wcnt[wave][lane] = cntc;
        const uint64_t incl = wave_incl_scan_fast((uint64_t)ri);
        if (lane == RR_WAVE - 1) wpart[1][wave] = incl;
        lds_barrier();
        uint32_t tot_c = 0, below_c = 0;   // lane c < C_N: class c's total, and in earlier waves
        if (lane < C_N) {
#pragma unroll
            for (uint32_t w = 0; w < NW; ++w) {
                const uint32_t x = wcnt[w][lane];
                tot_c += x;
                below_c += w < wave ? x : 0u;
            }
        }
        uint32_t base_c = 0, s = 0, bs = 0;   // lane c: class c's first perm slot
        uint64_t be = 0;
#pragma unroll
        for (uint32_t k = 0; k < C_N; ++k) {
            const uint32_t c = class_at(k), vpb = class_vpb(c);
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)tot_c, (int)c);
            base_c = lane == c ? s : base_c;
            if (tid == 0) { cbase[c] = s; ccount[c] = t; }   // (the batch loop's)
            s += t;
            bs += (t + vpb - 1) / vpb;
            be |= (uint64_t)bs << (8 * k);
        }
        static_assert(PMAX / 8 + C_N < 256, "batch prefix ends fit a byte (vpb >= 8)");
        if (tid == 0) bend = be;
        const uint32_t myb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((myc & (RR_WAVE - 1)) * 4), (int)(base_c + below_c));
        uint64_t wpre = 0, ctot = 0;
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) {
            const uint64_t x = wpart[1][w];
            wpre += w < wave ? x : 0;
            ctot += x;
        }
        // (u32, saturated: slots past 2^32 - 1 fail capacity whatever their exact place)
        const uint64_t mine = wpre + incl - ri;
        if (i < nv) {
            eloc[i] = (uint32_t)(mine < 0xFFFFFFFFull ? mine : 0xFFFFFFFFull);
            perm[myb + (uint32_t)__popcll(mm & ((1ull << lane) - 1))] = (uint16_t)i;
        }
        if (tid == 0) eloc[nv] = (uint32_t)(ctot < 0xFFFFFFFFull ? ctot : 0xFFFFFFFFull);
        return rfl64(ctot);   // (wave-uniform: kept in SGPRs)
    };
    uint64_t ctot = 0;
    if constexpr (ONE) {
        // the stage first, then the classes and reservations from it; the window's sum (of the
        // unsaturated reservations, as count_kernel's window sums) published before the sort and
        // the look-back resolved after it
        lds_barrier();   // (every wave has read its offsets from the search's samples)
        ov_finish();
        lds_barrier();
        PROBE(pb = __builtin_amdgcn_s_memtime();)
        uint64_t ragg = 0;
        if (v_lo + tid < v_hi) {
            one_class(o_v, o_v1, ragg, cls0);
            cnt0 = (uint32_t)(ragg < 0xFFFFFFFFull ? ragg : 0xFFFFFFFFull);
        }
        if (v_hi - v_lo > PMAX) {   // a window of more than one chunk: the later chunks' classes
            for (uint64_t c0 = v_lo + PMAX; c0 < v_hi; c0 += PMAX) {   // and reservations kept in the scratch
                if (c0 + tid < v_hi) {
                    uint64_t r;
                    uint32_t c;
                    one_class(offsets[c0 + tid], offsets[c0 + tid + 1], r, c);
                    ragg += r;
                    cls[c0 + tid] = (uint8_t)c;
                    counts[c0 + tid] = (uint32_t)(r < 0xFFFFFFFFull ? r : 0xFFFFFFFFull);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (read back by other waves of the window)
        }
        ragg = wave_sum_fast(ragg);
        if (lane == 0) red[0][wave] = ragg;
        lds_barrier();
        uint64_t agg = 0;
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) agg += red[0][w];
        // the window's look-back word, then the sort; then every earlier window's word, a thread
        // each (at most 511: one generation): a window that has not published yet but runs is
        // waited for; one not running yet (its workgroup not dispatched) is summed here instead,
        // by wave 0 from global memory (one_window_sum), so no window waits on one that does not run
        if (tid == 0) lb_store(&state[tile], ONE_RUN | ONE_AGG | agg);
        PROBE(pd = __builtin_amdgcn_s_memtime();)
        if (v_end > v_lo) ctot = sort_chunk(v_lo);
        PROBE(pe = __builtin_amdgcn_s_memtime();)
        __shared__ uint64_t lbw[2][2][NW];   // [round parity][waiting, to help][wave]
        uint64_t got = 0;
        bool have = tid >= tile;
        for (uint32_t it = 0;; ++it) {
            bool help = false;
            if (!have) {
                const uint64_t x = lb_load(&state[tid]);   // (after the sort: issued before it, the
                                                           // first read finds fewer words, 14.0 -> 15.1 us)
                if (x & ONE_AGG) { got = x & ONE_VAL; have = true; }
                else help = help_all || !(x & ONE_RUN);   // (help_all: the test hook's forced help)
            }
            const uint32_t b = it & 1;
            const uint64_t wm = __ballot(!have), hm = __ballot(help);
            if (lane == 0) { lbw[b][0][wave] = wm; lbw[b][1][wave] = hm; }
            lds_barrier();
            uint64_t anyw = 0, anyh = 0;
#pragma unroll
            for (uint32_t w = 0; w < NW; ++w) { anyw |= lbw[b][0][w]; anyh |= lbw[b][1][w]; }
            PROBE(pit = it + 1;)
            if (!anyw) break;
            if (it > (1u << 22)) {   // bounded: never hang the GPU (the call reports bytes = ~0)
                if (tid == 0) lb_store(one + 6, 1);
                break;
            }
            if (anyh) {
                if (wave == 0) {
                    for (uint32_t w = 0; w < NW; ++w)
                        for (uint64_t m = lbw[b][1][w]; m; m &= m - 1) {
                            const uint32_t q = w * RR_WAVE + (uint32_t)__builtin_ctzll(m);
                            const uint64_t sq = one_window_sum(blob, offsets, n, win, q);
                            if (lane == 0) lb_store(&state[q], ONE_AGG | sq);
                        }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (visible before the next round)
                }
            } else {
                __builtin_amdgcn_s_sleep(1);
            }
        }
        got = wave_sum_fast(got);
        if (lane == 0) red[1][wave] = got;
        lds_barrier();
        uint64_t e = 0;
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) e += red[1][w];
        eb0 = rfl64(e);
        PROBE(pc = __builtin_amdgcn_s_memtime();)
    } else {
        if (v_end > v_lo) {
            ctot = sort_chunk(v_lo);       // (with the window's loads still in flight)
            eb0 = rfl64(first_slot());     // (the waves' sums are behind the sort's first barrier)
        }
        ov_finish();                       // they have landed under the sort
    }
    for (uint64_t c0 = v_lo; c0 < v_end; c0 += PMAX) {
        if (c0 != v_lo) {
            lds_barrier();   // every wave is done with the previous chunk's batches
            run += ctot;
            ctot = sort_chunk(c0);
        }
        lds_barrier();   // the stage and the chunk's sort are complete
        // the chunk's descriptor slots [eb_c, eb_c + ctot), cut at the capacity
        const uint64_t eb_c = eb0 + run, ecut = eb_c + ctot < cap ? eb_c + ctot : cap;
        const rsrc_t E = make_rsrc(reinterpret_cast<const uint8_t *>(elems + eb_c),
                                   far || ecut <= eb_c ? 0u : (uint32_t)((ecut - eb_c) * 16));

        PROBE(if (c0 == v_lo) pt2 = __builtin_amdgcn_s_memtime();)
        // 3. single-class batches, taken dynamically by the waves
        const uint64_t be = rfl64(bend);   // (uniform: SGPRs)
        const uint32_t nb = RR_ABLATE == 2 ? 0u : (uint32_t)(be >> 56);
        for (;;) {
            uint32_t bi = 0;
            if (lane == 0) bi = atomicAdd(&next_batch, 1u);
            bi = __builtin_amdgcn_readfirstlane(bi);
            if (bi >= nb) break;
            // the batch's class from the packed prefix ends by scalar compares, not an LDS read per
            // class passed (round 6: config 3 at 1M 0.445 -> 0.438 ms, config 1 at 100K 13.5 -> 13.2 us)
            uint32_t k = 0, b0 = 0;   // (bi < nb)
#pragma unroll
            for (int j = 0; j < C_N - 1; ++j) {
                const uint32_t e = (uint32_t)(be >> (8 * j)) & 0xFFu;
                b0 = bi >= e ? e : b0;
                k += bi >= e;
            }
            const uint32_t c = class_at(k);
            const uint32_t vpb = class_vpb(c);
            const uint32_t first = cbase[c] + (bi - b0) * vpb;
            const uint32_t cnt = min(ccount[c] - (bi - b0) * vpb, vpb);
            PROBE(const uint64_t tb0 = __builtin_amdgcn_s_memtime();)
            // lanes per value: the chained classes 64 / cnt (grouped walks; a power of two for
            // Lists, ziplists and hash tables, so a value's lanes lie in one DPP row), hash
            // tables grouped only when a value gets lanes enough to hold its keys (do_ht_g)
            const bool grouped = c == C_LIST || c == C_SL || c == C_IS || c == C_ZL;
            const uint32_t Gw = max(1u, min(GMAX, (uint32_t)RR_WAVE / cnt));
            const bool htg = (c == C_HT || c == C_HH) && Gw >= ht_group_min(c == C_HH);
            const uint32_t Gh = 1u << (31 - __builtin_clz(Gw));
            const bool pow2 = htg || c == C_ZL || c == C_LIST;
            const uint32_t G = __builtin_amdgcn_readfirstlane(pow2 ? Gh : grouped ? Gw : 1u);
            const uint32_t li = lane / G, g = lane - li * G;   // the value's index in the batch
            const bool active = li < cnt;
            const uint32_t pi = active ? perm[first + li] : 0u;
            const uint64_t v = c0 + pi;
            uint64_t eb_v = eb_c, r_v = 0;
            if (active) {
                const uint32_t e0 = eloc[pi], e1 = eloc[pi + 1];
                eb_v = e1 == 0xFFFFFFFFu ? 1ull << 40 : eb_c + e0;   // (saturated: past every capacity)
                r_v = e1 - e0;
            }
            PROBE({   // cycles from the batch's start until its values' offsets are in registers
                const uint64_t ox = active ? offsets[v] : 0ull;
                const uint64_t tof = __builtin_amdgcn_s_memtime() - tb0 + (ox == ~0ull ? 1u : 0u);
                if (lane == 0) atomicAdd((unsigned long long *)&prb[36], (unsigned long long)tof);
            })
            const Acc a = staged ? run_batch(lsrc, c, active, v, G, g, S0, E, eb_c, blob, offsets, eb_v, r_v, values,
                                             elems, cap, &nfix)
                                 : run_batch(gsrc, c, active, v, G, g, S0, E, eb_c, blob, offsets, eb_v, r_v, values,
                                             elems, cap, &nfix);
            bad += a.bad;
            pay += a.pay;
            PROBE(if (lane == 0) {
                atomicAdd((unsigned long long *)&prb[3 + c], (unsigned long long)(__builtin_amdgcn_s_memtime() - tb0));
                atomicAdd((unsigned long long *)&prb[3 + C_N + c], 1ull);
                atomicAdd((unsigned long long *)&prb[3 + 2 * C_N + c], (unsigned long long)cnt);
            })
        }
    }
    bad = wave_sum_fast(bad);
    pay = wave_sum_fast(pay);
    if (lane == 0) { red[0][wave] = bad; red[1][wave] = pay; }
    lds_barrier();
    // 4. the window's marked values (rare: none in serObject output but fingerprint collisions),
    //    in the stage's LDS once every wave's records and descriptors are visible to the others
    if (nfix) {
        __syncthreads();
        fixup_window<NT>(blob, v_lo, v_hi, values, elems, ONE ? &s_fix : tot, stage);
        if (ONE) lds_barrier();   // (s_fix complete)
    }
    if constexpr (ONE) {
        // the window's totals into its end word; the call's last window waits for every other
        // window's, stores the call's totals and leaves the call's words zero (every look-back is
        // over once every window has ended)
        uint64_t tb = 0, tp = 0;
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) { tb += red[0][w]; tp += red[1][w]; }
        tb += s_fix.n_bad;
        tp += s_fix.payload;   // (u64 wrap: the fixup's adjustments are negative)
        if (tile != nwin - 1) {
            if (tid == 0) lb_store(&fin[tile], ONE_AGG | tb << 40 | (tp & ((1ull << 40) - 1)));
        } else {
            uint64_t xb = 0, xp = 0;
            if (tid < tile) {
                uint64_t x = 0;
                for (uint32_t sp = 0; !((x = lb_load(&fin[tid])) & ONE_AGG); ++sp) {
                    if (sp > (1u << 22)) { lb_store(one + 6, 1); break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                xb = (x & ~ONE_AGG) >> 40;
                xp = x & ((1ull << 40) - 1);
            }
            lds_barrier();   // (every wave is past its reads of red)
            xb = wave_sum_fast(xb);
            xp = wave_sum_fast(xp);
            if (lane == 0) { red[0][wave] = xb; red[1][wave] = xp; }
            lds_barrier();
            if (tid == 0) {
                for (uint32_t w = 0; w < NW; ++w) { tb += red[0][w]; tp += red[1][w]; }
                const uint64_t err = lb_load(one + 6);
                if (tot) {
                    tot->n_elems = eb0 + run + ctot;
                    tot->bytes = err ? ~0ull : offsets[n];   // (a wait that never ended)
                    tot->n_bad = tb;
                    tot->payload = tp;
                }
                lb_store(one + 6, 0);
            }
            if (tid < nwin) { lb_store(&state[tid], 0); lb_store(&fin[tid], 0); }
        }
        // (probe: [0] locate, [1] stage .. first slot, [2] the rest, [32] locate .. stage landed,
        //  [33] classification + publish, [34] the first chunk's sort, [35] look-back rounds)
        PROBE(if (tid == 0) {
              prb[0] = pa - pt0; prb[1] = pc - pa; prb[2] = __builtin_amdgcn_s_memtime() - pc; prb[32] = pb - pa; prb[33] = pd - pb; prb[34] = pe - pd; prb[35] = pit;
              prb[28] = v_hi - v_lo; prb[27] = prt0; prb[30] = __builtin_amdgcn_s_memrealtime();
              prb[31] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                        ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)) << 32);
              prb[29] = staged; if (g_probe) for (uint32_t i = 0; i < PROBE_WORDS; ++i) g_probe[(uint64_t)tile * PROBE_WORDS + i] = prb[i]; })
    }
    if (!ONE && tid == 0) {
        uint64_t tb = 0, tp = 0;
        for (uint32_t w = 0; w < NW; ++w) { tb += red[0][w]; tp += red[1][w]; }
        // the window's {bad, payload} straight into the call's totals (zeroed by count_kernel):
        // two non-returning atomics per window, ~7K per call spread over the kernel
        if (tot && tb) atomicAdd((unsigned long long *)&tot->n_bad, (unsigned long long)tb);
        if (tot && tp) atomicAdd((unsigned long long *)&tot->payload, (unsigned long long)tp);
        // the call's bytes, and its descriptor slots: the last window's first slot + its own
        // (plain stores, one writer each: no fold launch)
        if (tot && tile == 0) tot->bytes = offsets[n];
        if (tot && tile == nwin - 1) tot->n_elems = first_slot() + run + ctot;
        // (timeline: start / end on the 100 MHz realtime clock, and where the workgroup ran:
        //  HW_ID = wave, simd, pipe, CU, SH, SE bits; XCC_ID in bits 32+)
        PROBE(prb[0] = pt1 - pt0; prb[1] = pt2 - pt1; prb[2] = __builtin_amdgcn_s_memtime() - pt2; prb[28] = v_hi - v_lo;
              prb[27] = prt0; prb[30] = __builtin_amdgcn_s_memrealtime();
              prb[31] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                        ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)) << 32);
              prb[29] = staged; if (g_probe) for (uint32_t i = 0; i < PROBE_WORDS; ++i) g_probe[(uint64_t)tile * PROBE_WORDS + i] = prb[i];)
        // (no returning atomic, no barrier after it: the workgroup's slot frees as soon as its
        //  waves end — the sums are zeroed by the next call's count_kernel)
    }
}

// ---- small batches: the whole decode in one launch --------------------------------------
// The per-value callers (desObject on the rock thread, rock.c:468; the restore queue,
// rock.c:302-383) hand over one or a few values at a time, where the pipeline's launches, not
// bytes, are the cost.  A batch of at most SMALL_N values in at most SMALL_BYTES is decoded by
// ONE workgroup in ONE launch: its bytes staged into LDS with 16-byte loads (the source may be
// pinned host memory mapped into the device: rr_decode_batch_host), the reservations from the
// headers (count_kernel's rule), an in-block scan for the slots, the exact parser per value
// from LDS (the reference's statuses; the walks' results are the parser's by construction), the
// fixup of marked values, and the totals — the same records, descriptors, arena and totals as
// the pipeline, byte for byte.
constexpr uint32_t SMALL_NT = 1024, SMALL_VPT = 4, SMALL_N = SMALL_NT * SMALL_VPT;
constexpr uint32_t SMALL_BYTES = 128 * 1024;   // (one workgroup: up to 160 KiB of LDS)
// batches of at most this many values: one wave per value (the class walks on a wave / the
// whole wave emitting one value); larger ones one lane per value (the exact parser / the byte
// emitter) — which the host takes only for values of at most SMALL_LANE_BYTES on average
// (rr_small_decode_fits): a lane walking a 500-byte value costs ~20 us (round 4: 64 config-4
// values took 368 us through the lane path)
constexpr uint32_t SMALL_GW = 256;
constexpr uint64_t SMALL_LANE_BYTES = 64;
constexpr uint32_t SMALL_EIN = 16 * 1024;   // encode inputs up to this size staged in LDS
constexpr uint32_t SMALL_STAGE = SMALL_BYTES + 8192;   // + the reads past a value's end; >= the fixup's LDS
static_assert(FIX_LDS + 4 * (SMALL_NT + 1) <= SMALL_STAGE, "the fixup reuses the stage");

// The host entry points wait for a one-launch kernel by spinning on a word of their mapped
// staging instead of a stream synchronisation (~4 us less per call).  The producer form of
// MI355X_MICROARCH.md (inter-workgroup visibility, "valid forms"): every wave waits for its
// OWN stores to be acknowledged (s_waitcnt vmcnt(0): on gfx950 __syncthreads() is a bare
// s_barrier that waits for nothing in flight), then the barrier, so lane 0 signals only after
// every wave's records, descriptors and totals have landed; lane 0's ONE system-scope release
// (one L2 writeback), an explicit vmcnt(0) wait after it (the compiler may drop its own wait
// after the writeback when the scoreboard looks empty), and the store of the call's sequence
// number.  (A system fence in every thread — sixteen waves, sixteen L2 writebacks — cost ~8 us
// a call: tools/micro/lat_probe.hip, launch + spin 19.4 us against 11.4 us between HIP events.)
__device__ __forceinline__ void signal_done(uint32_t *done, uint32_t seq) {
    if (!done) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // (system scope)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(SMALL_NT) void decode_small_kernel(const uint8_t *__restrict__ blob,
                                                                const uint64_t *__restrict__ offsets, uint64_t n,
                                                                rr_value *__restrict__ values,
                                                                rr_elem *__restrict__ elems, uint64_t elem_cap,
                                                                uint8_t *__restrict__ arena, uint64_t data_cap,
                                                                rr_totals *tot, uint32_t *done, uint32_t seq) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[SMALL_STAGE];
    __shared__ uint64_t wsum[SMALL_NT / RR_WAVE], red[2][SMALL_NT / RR_WAVE];
    __shared__ uint32_t nfix;
    __shared__ uint64_t s_off[SMALL_GW + 1], s_eb[SMALL_GW], s_r[SMALL_GW];
    __shared__ uint32_t s_cls[SMALL_GW];
    __shared__ rr_totals s_tot;   // (the fixup's adjustments; the call's totals are stored once, at the end)
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid / RR_WAVE;
    if (tid == 0) nfix = 0;
    if (tid < 4) reinterpret_cast<uint64_t *>(&s_tot)[tid] = 0;
    // 1. the whole buffer [0, data_cap) into the stage, 16-byte granules, every load in flight
    //    beside the offsets loads (no wait for offsets[0] / offsets[n] first: the inputs may be
    //    the host entry point's mapped staging, a PCIe round trip each); the mirror arena gets
    //    [offsets[0], offsets[n]) rounded to granules, as the pipeline's window copy
    constexpr uint64_t B0 = 0;
    const uint32_t ng = (uint32_t)(data_cap >> 4);
    const u32x4 *src4 = reinterpret_cast<const u32x4 *>(blob);
    constexpr uint32_t SG = SMALL_BYTES / 16 / SMALL_NT;
    u32x4 gx[SG];
#pragma unroll
    for (uint32_t k = 0; k < SG; ++k) {
        const uint32_t g = tid + k * SMALL_NT;
        gx[k] = g < ng ? src4[g] : u32x4{0u, 0u, 0u, 0u};
    }
    // my values: v0 .. v0 + SMALL_VPT - 1 (consecutive: the block scan runs in value order)
    const uint64_t v0 = (uint64_t)tid * SMALL_VPT;
    uint64_t o[SMALL_VPT + 1];
#pragma unroll
    for (uint32_t j = 0; j <= SMALL_VPT; ++j) o[j] = offsets[v0 + j < n ? v0 + j : n];
    const uint64_t on = offsets[n], a0 = offsets[0] >> 4, a1 = (on + 15) >> 4;   // (uniform)
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    lds_u32x4 *st4 = (lds_u32x4 *)(__attribute__((address_space(3))) uint8_t *)stage;
#pragma unroll
    for (uint32_t k = 0; k < SG; ++k) {
        const uint32_t g = tid + k * SMALL_NT;
        if (g < ng) {
            st4[g] = gx[k];
            if (arena && g >= a0 && g < a1) reinterpret_cast<u32x4 *>(arena)[g] = gx[k];
        }
    }
    // LDS-only barriers from here to the fixup: __syncthreads() would wait for the arena stores'
    // acknowledgements — a PCIe round trip when the arena is the host entry point's mapped staging
    lds_barrier();
    const lds_cptr S = (lds_cptr)stage;
    // 2. reservations and walk classes from the headers (count_kernel's rule) and their block scan
    uint64_t r[SMALL_VPT], sum = 0;
    uint32_t cl[SMALL_VPT];
#pragma unroll
    for (uint32_t j = 0; j < SMALL_VPT; ++j) {
        r[j] = 0;
        cl[j] = C_EXACT;
        if (v0 + j < n) {
            const uint32_t q = (uint32_t)(o[j] - B0);
            uint32_t d[6];
            LdsSrc{S}.get<6>(q, d);   // (reads up to 28 bytes past q: inside the stage's slack)
            reserve_classify(S + q, o[j + 1] - o[j], d, r[j], cl[j]);
        }
        sum += r[j];
    }
    uint64_t total;
    uint64_t eb = block_excl_scan<SMALL_NT>(sum, wsum, total);
    const uint64_t cap = elem_cap < 0xFFFFFFFFull ? elem_cap : 0xFFFFFFFFull;   // elem_base is 32-bit
    uint64_t bad = 0, pay = 0;
    if (n <= SMALL_GW) {
        // 3a. a few values (the per-key calls): one wave per value, the value's class walk on
        //     all the lanes the batch loop would give a lone value (rr_decode_class.h), its
        //     offsets from LDS; the exact parser for the EXACT class and for values a walk rejects
        if (v0 <= n) {
#pragma unroll
            for (uint32_t j = 0; j <= SMALL_VPT; ++j)
                if (v0 + j <= n) s_off[v0 + j] = o[j];
#pragma unroll
            for (uint32_t j = 0; j < SMALL_VPT; ++j)
                if (v0 + j < n) { s_cls[v0 + j] = cl[j]; s_eb[v0 + j] = eb; s_r[v0 + j] = r[j]; eb += r[j]; }
        }
        lds_barrier();
        const LdsSrc lsrc{S};
        for (uint32_t v = wave; v < n; v += SMALL_NT / RR_WAVE) {
            const uint32_t c = s_cls[v];
            const uint64_t ev = s_eb[v], rv = s_r[v];
            Acc a{0, 0};
            if (c == C_EXACT) {
                if (lane == 0) a = exact_value(S, B0, v, s_off, ev, rv, values, elems, cap, &nfix);
            } else {
                const bool grouped = c == C_LIST || c == C_SL || c == C_IS || c == C_ZL;
                const bool htg = (c == C_HT || c == C_HH) && GMAX >= ht_group_min(c == C_HH);
                const uint32_t G = grouped || htg ? GMAX : 1u;
                const rsrc_t E = make_rsrc(reinterpret_cast<const uint8_t *>(elems + ev),
                                           ev < cap ? (uint32_t)((cap - ev < rv ? cap - ev : rv) * 16) : 0u);
                a = run_batch(lsrc, c, lane < G, v, G, lane & (G - 1), B0, E, ev, blob, s_off, ev, rv, values, elems, cap,
                              &nfix);
            }
            bad += a.bad;
            pay += a.pay;
        }
    } else {
        // 3b. the exact parser per value, from the stage
#pragma unroll 1
        for (uint32_t j = 0; j < SMALL_VPT; ++j) {
            if (v0 + j < n) {
                const Acc a = exact_value(S, B0, v0 + j, offsets, eb, r[j], values, elems, cap, &nfix);
                bad += a.bad;
                pay += a.pay;
            }
            eb += r[j];
        }
    }
    bad = wave_sum_fast(bad);
    pay = wave_sum_fast(pay);
    if (lane == 0) { red[0][wave] = bad; red[1][wave] = pay; }
    lds_barrier();
    // 4. marked values (duplicate keys, unsorted skiplists), in the stage's LDS, once every
    //    record and descriptor is visible to the workgroup (a full barrier only then)
    if (nfix) {
        __syncthreads();
        fixup_window<SMALL_NT>(blob, 0, n, values, elems, &s_tot, stage);
    }
    if (tid == 0) {
        uint64_t tb = 0, tp = 0;
        for (uint32_t w = 0; w < SMALL_NT / RR_WAVE; ++w) { tb += red[0][w]; tp += red[1][w]; }
        tot->n_bad = tb + s_tot.n_bad;
        tot->payload = tp + s_tot.payload;
        tot->n_elems = total;
        tot->bytes = on;
    }
    signal_done(done, seq);
}

// ---------------------------------------------------------------------------------------- encode
__device__ __forceinline__ bool fits_width(int64_t x, uint32_t w) {
    if (w == 8) return true;
    if (w == 4) return x >= INT32_MIN && x <= INT32_MAX;
    return x >= INT16_MIN && x <= INT16_MAX;
}


// Decimal digits of an unsigned magnitude (sdsll2str's length without the sign): compares,
// no divisions.
__constant__ uint64_t P10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                 100000000ull, 1000000000ull, 10000000000ull, 100000000000ull, 1000000000000ull,
                                 10000000000000ull, 100000000000000ull, 1000000000000000ull, 10000000000000000ull,
                                 100000000000000000ull, 1000000000000000000ull, 10000000000000000000ull};
// decimal digits of v: t = floor(bits(v) * log10 2) (1233 / 4096) is the count or one less, and
// v >= 10^t says which (one table read instead of 19 64-bit compares, ~75 VALU a call: round 6,
// E1 71.0 -> 58.1 us, E4 296 -> 292 us on config 4; profiles/r6_encode_pieces_ab.txt)
__device__ __forceinline__ uint32_t udigits(uint64_t v) {
    const uint32_t b = 64u - (uint32_t)__builtin_clzll(v | 1ull), t = (b * 1233u) >> 12;
    const uint32_t d = t + (v >= P10[t] ? 1u : 0u);
    return d ? d : 1u;
}
// Length of sdsll2str(x) (sds.c:450-479).
__device__ __forceinline__ uint32_t sdec_len(int64_t x) {
    return x < 0 ? 1u + udigits(0ull - (uint64_t)x) : udigits((uint64_t)x);
}

// Per-descriptor contribution to a value's blob bytes and payload, and whether the
// descriptor kind is legal for the value type (see enc_emit_kernel's layout table).
struct ElemCost {
    uint64_t bytes, pay;
    bool bad;
};
// a STR / ZLRAW descriptor's payload lies inside the caller's arena
__device__ __forceinline__ bool in_arena(const ElemV &e, uint64_t acap) { return e.data <= acap && e.len <= acap - e.data; }
__device__ __forceinline__ ElemCost elem_cost(uint32_t type, uint32_t enc, uint64_t i, const ElemV &e, uint64_t acap) {
    switch (type) {
        case RR_TYPE_LIST_QUICKLIST:
            if (e.kind == RR_K_INT) return {4 + (uint64_t)sdec_len((int64_t)e.data), 0, false};
            return {4 + (uint64_t)e.len, e.len, e.kind != RR_K_STR || !in_arena(e, acap)};
        case RR_TYPE_SET_INTSET:
            return {enc, 0, e.kind != RR_K_INT || !fits_width((int64_t)e.data, enc)};
        case RR_TYPE_ZSET_SKIPLIST:
            if (i & 1) return {8, 0, e.kind != RR_K_SCORE};
            return {8 + (uint64_t)e.len, e.len, e.kind != RR_K_STR || !in_arena(e, acap)};
        default:   // SET_HT / HASH_HT members
            return {8 + (uint64_t)e.len, e.len, e.kind != RR_K_STR || !in_arena(e, acap)};
    }
}

// serObject rock_serdes.c:512-535: blob size of one flat value, 0 + status if unencodable:
// a value whose status is not RR_OK, whose descriptor range passes elem_cap or whose payloads
// pass arena_cap is never read further (RR_E_ENCODE).  Descriptors are read four at a time
// (independent 16-byte loads in flight per lane).  Used by E3 for the values past data_cap;
// E1 computes the same sizes element-parallel.
__device__ uint64_t encode_size(uint32_t type, uint32_t enc, uint32_t vstatus, uint64_t eb, uint64_t n,
                                const rr_elem *elems, uint64_t ecap, uint64_t acap, uint32_t &st, uint64_t &pay) {
    st = RR_OK;
    pay = 0;
    const rr_elem *el = elems + eb;
    if (vstatus != RR_OK || eb + n > ecap) type = 0xFF;   // falls to the unencodable default
    switch (type) {
        case RR_TYPE_STRING: {
            if (n != 1) break;
            ElemV e = get_elem(el);
            if (enc == RR_ENC_INT) {
                if (e.kind != RR_K_INT) break;
                return 14;
            }
            if ((enc != RR_ENC_RAW && enc != RR_ENC_EMBSTR) || e.kind != RR_K_STR || !in_arena(e, acap)) break;
            pay = e.len;
            return 6 + (uint64_t)e.len;
        }
        case RR_TYPE_HASH_ZIPLIST:
        case RR_TYPE_ZSET_ZIPLIST: {
            if (n < 1) break;
            ElemV e = get_elem(el);
            if (e.kind != RR_K_ZLRAW || !in_arena(e, acap)) break;
            pay = e.len;
            return 13 + (uint64_t)e.len;
        }
        case RR_TYPE_SET_INTSET:
            if (enc != 2 && enc != 4 && enc != 8) break;
            [[fallthrough]];
        case RR_TYPE_LIST_QUICKLIST:
        case RR_TYPE_SET_HT:
        case RR_TYPE_HASH_HT:
        case RR_TYPE_ZSET_SKIPLIST: {
            if ((type == RR_TYPE_HASH_HT || type == RR_TYPE_ZSET_SKIPLIST) && (n & 1)) break;
            uint64_t sz = type == RR_TYPE_LIST_QUICKLIST ? 5 : 13, p = 0;
            bool bad = false;
            for (uint64_t i = 0; i < n; i += 4) {
                ElemV e[4];
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) e[k] = i + k < n ? get_elem(el + i + k) : ElemV{0, 0, RR_K_INT};
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) {
                    if (i + k < n) {
                        const ElemCost c = elem_cost(type, enc, i + k, e[k], acap);
                        sz += c.bytes;
                        p += c.pay;
                        bad |= c.bad;
                    }
                }
            }
            if (bad) { st = RR_E_ENCODE; return 0; }
            pay = p;
            return sz;
        }
        default:
            break;
    }
    st = RR_E_ENCODE;
    pay = 0;
    return 0;
}

// Encode runs as three kernels, with no inter-workgroup waits (E4's block 0 zeroes the group
// sums for the next call):
//   E1 enc_size_kernel  workgroup per 256 values, element-parallel: blob size (0 for an
//                       unencodable value), its offset inside the block into offsets[v], the
//                       block's bytes into btot[b] and (atomically) its group's of 64 blocks
//                       into gtot; per-tile {bad, payload, descriptors};
//   E3 enc_index_kernel thread per value, the same blocks: the block's first byte from the
//                       group and block sums before it (two loads per lane), offsets[v] made
//                       global, the first value of every W-byte output window, and the values
//                       that would cross data_cap (RR_E_CAPACITY, payload taken back);
//   E4 enc_emit_kernel  workgroup per W-byte output window: builds the window's bytes in an
//                       LDS image (headers and length fields by element-parallel tasks,
//                       payloads by 64-byte copy pieces), then stores it with 16-byte
//                       coalesced stores; its block 0 folds the totals.
// (Round 3 ran a look-back scan of the sizes as E2, 15 us on config 4.)
// Output bytes past the last value that fits (and of a value that does not fit) are zero.

// ---- E1: blob size per value -----------------------------------------------------------
// Workgroup per NT values, element-parallel: a value's descriptors are "tasks" (one for a
// STRING or a ziplist: the payload / ZLRAW descriptor; n for the others); a block scan of the
// task counts maps task t to its value (binary search of the task bases in LDS), the tasks are
// costed NT per round (U rounds' descriptors loaded at once), and a value's size is the
// difference of the running task-byte scan between its first and its last task.  The cost
// of a value is then additive in its descriptors, not the longest value of the wave.  Values
// of at most ENC_SHORT tasks (strings, ziplists, small collections) skip the rounds: their own
// lane costs them, as a thread-per-value pass would.
// Sizes are serObject's (encode_size, same statuses).
__device__ __forceinline__ ElemCost task_cost(uint32_t type, uint32_t enc, uint64_t k, const ElemV &e, uint64_t acap) {
    switch (type) {
        case RR_TYPE_STRING:
            if (enc == RR_ENC_INT) return {8, 0, e.kind != RR_K_INT};
            return {e.len, e.len, e.kind != RR_K_STR || !in_arena(e, acap)};
        case RR_TYPE_HASH_ZIPLIST:
        case RR_TYPE_ZSET_ZIPLIST:
            return {e.len, e.len, e.kind != RR_K_ZLRAW || !in_arena(e, acap)};
        default:
            return elem_cost(type, enc, k, e, acap);
    }
}
// E1 constants: task rounds whose descriptors are loaded together; values with at most ENC_SHORT
// tasks are costed by their own lane
constexpr uint32_t ENC_SIZE_U = 2, ENC_SHORT = 4;
constexpr uint32_t ENC_MAPCAP = 4096;
// Task -> value map of a round of NT values (the value's index at each of its tasks, u8), from
// the task bases: the value with tasks writes its index at its first task (the head), then a
// running max fills the runs — heads increase along the map, so the zeros between them (the map
// was zeroed beforehand, ordered by a barrier) never win: 16 positions a thread, the carry across
// threads by a DPP max scan and the waves' maxima in LDS.  Returns whether the round's tt tasks
// fit the map (block-uniform); ends with an LDS barrier either way.
template <uint32_t NT>
__device__ __forceinline__ bool build_task_map(uint8_t *tmap, uint32_t *wmax, uint32_t base, uint32_t ntask,
                                               uint64_t tt) {
    static_assert(NT <= 256 && ENC_MAPCAP == 16 * NT, "u8 map, 16 bytes per thread");
    const uint32_t tid = threadIdx.x;
    const bool usemap = tt <= ENC_MAPCAP;
    if (usemap && ntask) tmap[base] = (uint8_t)tid;
    lds_barrier();
    if (usemap && tt) {
        const uint4 q = reinterpret_cast<uint4 *>(tmap)[tid];
        uint32_t w[4] = {q.x, q.y, q.z, q.w}, m = 0;
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) m = max(m, (w[k >> 2] >> (8 * (k & 3))) & 0xFF);
        const uint32_t im = wave_incl_max_u32(m);
        if (lane_id() == RR_WAVE - 1) wmax[tid / RR_WAVE] = im;
        lds_barrier();
        uint32_t carry = 0;
#pragma unroll
        for (uint32_t k = 0; k < NT / RR_WAVE; ++k) carry = k < tid / RR_WAVE ? max(carry, wmax[k]) : carry;
        const uint32_t prev = wave_from_prev(im);
        carry = max(carry, lane_id() ? prev : 0u);
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            carry = max(carry, (w[k >> 2] >> (8 * (k & 3))) & 0xFF);
            w[k >> 2] = (w[k >> 2] & ~(0xFFu << (8 * (k & 3)))) | (carry << (8 * (k & 3)));
        }
        reinterpret_cast<uint4 *>(tmap)[tid] = make_uint4(w[0], w[1], w[2], w[3]);
        lds_barrier();
    }
    return usemap;
}
#ifdef RR_PROBE
// Encode probe (tools/probe_encode.py): per window {init, headers, tasks, copy, store, total,
// values, tasks, pieces} in s_memrealtime ticks (100 MHz); diagnostics only.
constexpr uint32_t EPROBE_WORDS = 13;
__device__ uint64_t *g_eprobe;
extern "C" int rr_eprobe_set(void *p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_eprobe), &p, sizeof(p)) == hipSuccess ? 0 : -1; }
__device__ __forceinline__ uint64_t rr_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define EPROBE(...) __VA_ARGS__
// E1 (enc_size_kernel) phases summed over the call's blocks: [0] head (records, the short
// values' descriptors, the task scan and map), [1] the task rounds, [2] the sizes' scan and
// stores, [3] blocks, [4] tasks, [5] rounds; s_memtime after every outstanding memory operation
__device__ unsigned long long g_e1probe[6];
extern "C" int rr_e1probe_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_e1probe), sizeof(g_e1probe)) == hipSuccess ? 0 : -1;
}
extern "C" int rr_e1probe_reset() {
    static const unsigned long long z[6] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_e1probe), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
__device__ __forceinline__ uint64_t e1_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#else
#define EPROBE(...)
#endif

template <uint32_t NT, uint32_t U>
__global__ __launch_bounds__(NT) void enc_size_kernel(const rr_value *__restrict__ values,
                                                      const rr_elem *__restrict__ elems, uint64_t n,
                                                      uint64_t ecap, uint64_t acap,
                                                      uint64_t *__restrict__ sizes, uint64_t *__restrict__ stats,
                                                      uint64_t *__restrict__ btot, uint64_t *gtot,
                                                      uint64_t *zero_words, uint32_t nzero, rr_totals *tot) {
    zero_call_words(zero_words, nzero, tot);
    EPROBE(const uint64_t e1t0 = e1_stamp(); uint64_t e1t1 = 0, e1nr = 0;)
    __shared__ uint32_t tb[NT + 1];                  // first task of each value
    __shared__ uint32_t s_el[NT], s_te[NT], s_bad[NT];
    __shared__ uint64_t s_b1[NT], s_p1[NT];   // the value's byte / payload sums (short values: their own lane's)
    __shared__ uint64_t ws0[NT / RR_WAVE];
    __shared__ uint64_t red[3][NT / RR_WAVE];
    // task -> value map of the block when it has at most ENC_MAPCAP tasks (build_task_map): one
    // LDS read per task instead of a binary search of the task bases
    __shared__ __attribute__((aligned(16))) uint8_t tmap[ENC_MAPCAP];
    __shared__ uint32_t wmax[NT / RR_WAVE];
    reinterpret_cast<uint4 *>(tmap)[threadIdx.x] = make_uint4(0, 0, 0, 0);   // (ordered before the
                                                                             // heads by the scan's barrier)
    const uint32_t tid = threadIdx.x;
    const uint64_t v = (uint64_t)blockIdx.x * NT + tid;
    uint32_t type = 0, enc = 0, ntask = 0, hdr = 0, bad = 0;
    uint64_t ne = 0, eb = 0;
    if (v < n) {
        const uint4 w = reinterpret_cast<const uint4 *>(values)[v];
        type = w.x & 0xFF;
        enc = (w.x >> 8) & 0xFF;
        ne = w.z;
        eb = w.w;
        bad = 1;
        if ((w.x >> 16) == RR_OK && eb + ne <= ecap) {
            switch (type) {
                case RR_TYPE_STRING:
                    if (ne == 1 && (enc == RR_ENC_INT || enc == RR_ENC_RAW || enc == RR_ENC_EMBSTR)) { bad = 0; hdr = 6; ntask = 1; }
                    break;
                case RR_TYPE_HASH_ZIPLIST:
                case RR_TYPE_ZSET_ZIPLIST:
                    if (ne >= 1) { bad = 0; hdr = 13; ntask = 1; }
                    break;
                case RR_TYPE_SET_INTSET:
                    if (enc == 2 || enc == 4 || enc == 8) { bad = 0; hdr = 13; ntask = (uint32_t)ne; }
                    break;
                case RR_TYPE_LIST_QUICKLIST: bad = 0; hdr = 5; ntask = (uint32_t)ne; break;
                case RR_TYPE_SET_HT: bad = 0; hdr = 13; ntask = (uint32_t)ne; break;
                case RR_TYPE_HASH_HT:
                case RR_TYPE_ZSET_SKIPLIST:
                    if (!(ne & 1)) { bad = 0; hdr = 13; ntask = (uint32_t)ne; }
                    break;
                default: break;
            }
        }
    }
    // a short value is costed here, by its own lane (its loads in flight under the scan)
    uint64_t sh_b = 0, sh_p = 0;
    if (ntask <= ENC_SHORT) {
        ElemV e[ENC_SHORT];
#pragma unroll
        for (uint32_t k = 0; k < ENC_SHORT; ++k) e[k] = k < ntask ? get_elem(elems + eb + k) : ElemV{0, 0, 0};
#pragma unroll
        for (uint32_t k = 0; k < ENC_SHORT; ++k) {
            if (k < ntask) {
                const ElemCost c = task_cost(type, enc, k, e[k], acap);
                sh_b += c.bytes;
                sh_p += c.pay;
                bad |= c.bad ? 1u : 0u;
            }
        }
        ntask = 0;
    }
    s_el[tid] = (uint32_t)eb;
    s_te[tid] = type | (enc << 8);
    s_bad[tid] = bad;
    s_b1[tid] = sh_b;
    s_p1[tid] = sh_p;
    uint64_t TT;
    const uint32_t base = (uint32_t)block_excl_scan<NT>(ntask, ws0, TT);
    tb[tid] = base;
    if (tid == NT - 1) tb[NT] = base + ntask;
    const bool usemap = build_task_map<NT>(tmap, wmax, base, ntask, TT);
    EPROBE(e1t1 = e1_stamp();)
    auto fetch = [&](uint64_t t, uint32_t &pj, ElemV &pe) {
        pj = 0;
        pe = ElemV{0, 0, 0};
        if (t < TT) {
            uint32_t lo = 0;
            if (usemap) lo = tmap[t];
            else
#pragma unroll
                for (uint32_t s = NT / 2; s > 0; s >>= 1)
                    if (tb[lo + s] <= t) lo += s;
            pj = lo;
            pe = get_elem(elems + s_el[lo] + (uint32_t)(t - tb[lo]));
        }
    };
    for (uint64_t g0 = 0; g0 < TT; g0 += U * NT) {
        uint32_t j[U];
        ElemV e[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) fetch(g0 + u * NT + tid, j[u], e[u]);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            if (g0 + u * NT >= TT) break;
            const uint64_t t = g0 + u * NT + tid;
            const bool act = t < TT;
            ElemCost c{0, 0, false};
            if (act) {
                const uint32_t te = s_te[j[u]];
                c = task_cost(te & 0xFF, te >> 8, (uint32_t)(t - tb[j[u]]), e[u], acap);
            }
            // wave-segmented sums, no block barrier per round: a wave's tasks run over a few
            // values in order; each value's run in the wave adds (inclusive scan at its last
            // task) - (exclusive scan at its first task) to the value's sums with two LDS atomics
            // (a block scan and barrier per round measured 81 -> 73 us without)
            const bool small = __ballot((c.bytes | c.pay) >= (1ull << 26)) == 0;
            const uint64_t ib = small ? (uint64_t)wave_incl_scan_u32((uint32_t)c.bytes) : wave_incl_scan(c.bytes);
            const uint64_t ip = small ? (uint64_t)wave_incl_scan_u32((uint32_t)c.pay) : wave_incl_scan(c.pay);
            const uint32_t jp = wave_from_prev(j[u]), jn = wave_from_next(j[u]);
            const uint32_t ln = lane_id();
            const bool first = act && (ln == 0 || jp != j[u]);
            const bool last = act && (ln == RR_WAVE - 1 || t + 1 >= TT || jn != j[u]);
            if (first) {
                atomicAdd((unsigned long long *)&s_b1[j[u]], (unsigned long long)(0ull - (ib - c.bytes)));
                atomicAdd((unsigned long long *)&s_p1[j[u]], (unsigned long long)(0ull - (ip - c.pay)));
            }
            if (last) {
                atomicAdd((unsigned long long *)&s_b1[j[u]], (unsigned long long)ib);
                atomicAdd((unsigned long long *)&s_p1[j[u]], (unsigned long long)ip);
            }
            if (act && c.bad) s_bad[j[u]] = 1;
        }
    }
    lds_barrier();
    EPROBE(const uint64_t e1t2 = e1_stamp(); e1nr = (TT + U * NT - 1) / (U * NT);)
    uint64_t size = 0, pay = 0;
    if (v < n) {
        bad = s_bad[tid];
        size = bad ? 0 : hdr + s_b1[tid];
        pay = bad ? 0 : s_p1[tid];
    }
    // the value's offset inside the block; the block's bytes (E3 adds the blocks before it)
    uint64_t btotal;
    const uint64_t inb = block_excl_scan<NT>(size, ws0, btotal);
    if (v < n) sizes[v] = inb;
    if (tid == 0) {
        btot[blockIdx.x] = btotal;
        if (btotal) atomicAdd((unsigned long long *)&gtot[blockIdx.x / WGROUP], (unsigned long long)btotal);
    }
    uint64_t sb = wave_sum_fast(bad), sp = wave_sum_fast(pay), sn = wave_sum_fast(ne);
    const uint32_t wv = tid / RR_WAVE;
    if (lane_id() == 0) { red[0][wv] = sb; red[1][wv] = sp; red[2][wv] = sn; }
    __syncthreads();
    if (tid < 3) {
        uint64_t sum = 0;
        for (uint32_t k = 0; k < NT / RR_WAVE; ++k) sum += red[tid][k];
        stats[3 * (uint64_t)blockIdx.x + tid] = sum;
    }
    EPROBE(const uint64_t e1t3 = e1_stamp();
           if (tid == 0) {
               atomicAdd(&g_e1probe[0], (unsigned long long)(e1t1 - e1t0)); atomicAdd(&g_e1probe[1], (unsigned long long)(e1t2 - e1t1));
               atomicAdd(&g_e1probe[2], (unsigned long long)(e1t3 - e1t2)); atomicAdd(&g_e1probe[3], 1ull);
               atomicAdd(&g_e1probe[4], (unsigned long long)TT); atomicAdd(&g_e1probe[5], (unsigned long long)e1nr);
           })
}

// ---- E3: window index + capacity check ---------------------------------------------------
// fv[w] = the value holding output byte w*W (values of size 0 hold none).  A value whose end
// passes data_cap is not written (rock_serdes has no such case: sds grows; the batch API
// bounds the output): it counts as bad and its payload is taken back out of the totals
// (stored as a two's-complement negative, folded by the same modular sum).
template <uint32_t W>
__global__ __launch_bounds__(256) void enc_index_kernel(const rr_value *__restrict__ values,
                                                        const rr_elem *__restrict__ elems, uint64_t n,
                                                        uint64_t ecap, uint64_t acap, uint64_t *__restrict__ offsets,
                                                        const uint64_t *__restrict__ btot,
                                                        const uint64_t *__restrict__ gtot, uint64_t cap,
                                                        uint32_t *__restrict__ fv, uint64_t nwin,
                                                        uint64_t *__restrict__ stats) {
    __shared__ uint64_t red[2][4], wpre[4];
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    const uint64_t v = (uint64_t)blk * blockDim.x + tid;
    // the block's first byte: the groups of WGROUP blocks before it, the blocks before it in its
    // group (E1's sums)
    const uint32_t grp = blk / WGROUP, gi = blk % WGROUP;
    uint64_t pre = tid < gi ? btot[(uint64_t)grp * WGROUP + tid] : 0;
    for (uint32_t k = tid; k < grp; k += blockDim.x) pre += gtot[k];
    pre = wave_sum_fast(pre);
    if (lane_id() == 0) wpre[tid / RR_WAVE] = pre;
    // my offset inside the block and the next value's (the block's last: the block's bytes), read
    // before any thread of the block overwrites offsets with the global ones
    uint64_t ia = 0, ib = 0;
    if (v < n) {
        ia = offsets[v];
        ib = tid + 1 < blockDim.x && v + 1 < n ? offsets[v + 1] : btot[blk];
    }
    __syncthreads();
    const uint64_t P = wpre[0] + wpre[1] + wpre[2] + wpre[3];
    uint64_t bad = 0, pay = 0;
    if (v < n) {
        const uint64_t a = P + ia, b = P + ib;
        offsets[v] = a;
        if (v + 1 == n) offsets[n] = b;
        if (b > a) {
            uint64_t w_hi = (b - 1) / W;
            if (w_hi > nwin) w_hi = nwin;
            for (uint64_t w = (a + W - 1) / W; w <= w_hi; ++w) fv[w] = (uint32_t)v;
            if (b > cap) {
                const uint4 x = reinterpret_cast<const uint4 *>(values)[v];
                uint32_t st;
                encode_size(x.x & 0xFF, (x.x >> 8) & 0xFF, x.x >> 16, x.w, x.z, elems, ecap, acap, st, pay);
                bad = 1;
                pay = 0ull - pay;
            }
        }
    }
    bad = wave_sum_fast(bad);
    pay = wave_sum_fast(pay);
    const uint32_t wv = threadIdx.x / RR_WAVE;
    if (lane_id() == 0) { red[0][wv] = bad; red[1][wv] = pay; }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint64_t s = 0;
        if (threadIdx.x < 2)
            for (uint32_t k = 0; k < blockDim.x / RR_WAVE; ++k) s += red[threadIdx.x][k];
        stats[3 * (uint64_t)blockIdx.x + threadIdx.x] = s;
    }
}




// ---- E4: window emission -------------------------------------------------------------------
// Blob layout per type (serObject rock_serdes.c:512-535): a value is a header of h bytes then
// one "task" per descriptor, each task writing es bytes:
//   STRING    h=6  (type, lru, enc)            INT: 8 (i64)           STR: len (payload)
//   LIST      h=5                              INT: 4 + decimal       STR: 4 + len
//   INTSET    h=13 (+ u32 enc, u32 count)      enc bytes of the int
//   SET/HASH HT  h=13 (+ u64 count)            8 + len
//   ZIPLIST   h=5,  one task (descriptor 0, the raw ziplist): 8 + len
//   SKIPLIST  h=13 (+ u64 count)               member: 8 + len        score: 8 (raw f64)
__device__ __forceinline__ uint32_t enc_hdr(uint32_t type) {
    return type == RR_TYPE_STRING ? 6u : (type == RR_TYPE_LIST_QUICKLIST || type == RR_TYPE_HASH_ZIPLIST ||
                                          type == RR_TYPE_ZSET_ZIPLIST) ? 5u : 13u;
}

// Naturally aligned LDS stores only in the window image: a misaligned ds_write costs ~7 aligned
// ones on gfx950 (tools/micro/lds_align.hip: misaligned b32/b64/b128 all ~0.45 ms vs 0.06-0.10
// ms aligned).

// x < 10^8 as 8 ASCII digits, the most significant in byte 0: 4-digit halves, 2-digit pairs,
// digits (exact reciprocal multiplies for these ranges)
__device__ __forceinline__ uint64_t swar8(uint32_t x) {
    const uint32_t hi = x / 10000u, lo = x - hi * 10000u;
    auto two = [](uint32_t p) {   // p < 100 -> tens | units << 8
        const uint32_t t = (p * 103u) >> 10;
        return t | ((p - t * 10u) << 8);
    };
    auto four = [&](uint32_t h) {   // h < 10^4 -> 4 digits
        const uint32_t a = (h * 5243u) >> 19;
        return two(a) | (two(h - a * 100u) << 16);
    };
    return ((uint64_t)four(hi) | ((uint64_t)four(lo) << 32)) + 0x3030303030303030ull;
}

// lds_or writes the low nb (<= 8) bytes of v at image offset d into an image whose bytes there
// are still zero (the image is zeroed first and no two fields overlap): the field OR-ed into the
// one or two naturally aligned 8-byte words it touches, no-return LDS atomics, no branches on
// the alignment (lds_put takes up to seven conditional stores).
__device__ __forceinline__ void lds_or(uint8_t *img, uint32_t d, uint64_t v, uint32_t nb) {
    v = nb >= 8 ? v : v & ((1ull << (8 * nb)) - 1);
    const uint32_t s = (d & 7u) * 8u;
    uint64_t *w = reinterpret_cast<uint64_t *>(img + (d & ~7u));
    __hip_atomic_fetch_or(w, v << s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (s && s + 8 * nb > 64) __hip_atomic_fetch_or(w + 1, v >> (64 - s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The window image: writes at absolute output positions, clipped to [w0, w0 + span).
struct Img {
    uint8_t *img;
    uint64_t w0;
    uint64_t span;
    // little-endian field of nb (<= 8) bytes, clipped to the window with no byte loop: the bytes
    // before w0 shifted out, those past the span cut from the length.  (Until round 6 a byte loop
    // handled the window's two straddling values, inlined at every call site: the emit kernel
    // took 79 VGPRs instead of 72, and encode config 4 / 3 ran 2.6 % slower;
    // profiles/r6_encode_pieces_ab.txt)
    __device__ __forceinline__ void field(uint64_t pos, uint64_t v, uint32_t nb) const {
        const int64_t d = (int64_t)(pos - w0), e = d + (int64_t)nb;
        const int64_t lo = d > 0 ? d : 0, hi = e < (int64_t)span ? e : (int64_t)span;
        if (hi > lo) lds_or(img, (uint32_t)lo, v >> (8 * (uint32_t)(lo - d)), (uint32_t)(hi - lo));
    }
    // the same with the bytes before `from` dropped too
    __device__ __forceinline__ void field_from(uint64_t pos, uint64_t v, uint32_t nb, uint64_t from) const {
        const int64_t d = (int64_t)(pos - w0), e = d + (int64_t)nb, f = (int64_t)(from - w0);
        int64_t lo = d > f ? d : f;
        lo = lo > 0 ? lo : 0;
        const int64_t hi = e < (int64_t)span ? e : (int64_t)span;
        if (hi > lo) lds_or(img, (uint32_t)lo, v >> (8 * (uint32_t)(lo - d)), (uint32_t)(hi - lo));
    }
    // chunk c (0: the last 8 digits, 1: the 8 before, 2: the first 3) of sdsll2str(x) at pos, l
    // characters: the chunk's 8 digits right-aligned at their place, the leading zeros dropped by
    // the clip at the first digit; chunk 0 also writes the sign
    __device__ __forceinline__ void decimal_chunk(uint64_t pos, int64_t x, uint32_t l, uint32_t c) const {
        const uint64_t u = x < 0 ? 0ull - (uint64_t)x : (uint64_t)x;
        const uint64_t q = u / 100000000ull, q2 = q / 100000000ull;
        const uint64_t ch = c == 0 ? u - q * 100000000ull : c == 1 ? q - q2 * 100000000ull : q2;
        const uint64_t end = pos + l, from = pos + (x < 0 ? 1u : 0u);
        field_from(end - 8 * (c + 1), swar8((uint32_t)ch), 8, from);
        if (c == 0 && x < 0) field(pos, '-', 1);
    }
    // sdsll2str(x) (sds.c:450-479), l characters at pos: |x| as three 8-digit chunks, each
    // turned into 8 ASCII digits at once (SWAR), the 24-character string shifted right past
    // its leading zeros (first character in byte 0), the sign prepended, then stored as up to
    // three fields
    __device__ __forceinline__ void decimal(uint64_t pos, int64_t x, uint32_t l) const {
        const uint64_t u = x < 0 ? 0ull - (uint64_t)x : (uint64_t)x;
        const uint64_t q = u / 100000000ull, q2 = q / 100000000ull;
        uint64_t w[3] = {swar8((uint32_t)q2), swar8((uint32_t)(q - q2 * 100000000ull)),
                         swar8((uint32_t)(u - q * 100000000ull))};
        const uint32_t neg = x < 0 ? 1u : 0u, zb = 8u * (24u - (l - neg)), ws = zb >> 6, bs = zb & 63;
        auto word = [&](uint32_t i) { return i == 0 ? w[0] : i == 1 ? w[1] : i == 2 ? w[2] : 0ull; };
        auto shr = [&](uint32_t i) {
            const uint64_t lo = word(ws + i), hi = word(ws + i + 1);
            return bs ? (lo >> bs) | (hi << (64 - bs)) : lo;
        };
        uint64_t a0 = shr(0), a1 = shr(1), a2 = shr(2);
        if (neg) {
            a2 = (a2 << 8) | (a1 >> 56);
            a1 = (a1 << 8) | (a0 >> 56);
            a0 = (a0 << 8) | '-';
        }
        for (uint32_t k = 0; 8 * k < l; ++k)
            field(pos + 8 * k, k == 0 ? a0 : k == 1 ? a1 : a2, l - 8 * k < 8 ? l - 8 * k : 8);
    }
};

// Copy piece: arena bytes [src, src+len) -> image bytes [d, d+len), the piece inside one
// 64-byte aligned image block.  Destination-aligned plan: ascending head steps (1, 2, 4, 8)
// to a 16-byte boundary, up to four 16-byte chunks, descending tail (8, 4, 2, 1).  Source
// loads are unaligned (allowed for global memory) and all issued before the stores.  Macros
// over plain locals: the same code on struct members went through scratch memory.
#define RR_PIECE_LOAD(P, SRC, DST, LEN)                                                          \
    uint4 P##m0, P##m1, P##m2, P##m3;                                                            \
    uint64_t P##h8 = 0, P##t8 = 0;                                                               \
    uint32_t P##h4 = 0, P##t4 = 0, P##h2 = 0, P##t2 = 0, P##h1 = 0, P##t1 = 0;                   \
    {                                                                                            \
        uint32_t p_ = (DST), r_ = (LEN);                                                         \
        const uint8_t *q_ = (SRC);                                                               \
        if ((p_ & 1) && r_ >= 1) { P##h1 = q_[0]; p_ += 1; r_ -= 1; q_ += 1; }                   \
        if ((p_ & 2) && r_ >= 2) { uint16_t x_; __builtin_memcpy(&x_, q_, 2); P##h2 = x_; p_ += 2; r_ -= 2; q_ += 2; } \
        if ((p_ & 4) && r_ >= 4) { __builtin_memcpy(&P##h4, q_, 4); p_ += 4; r_ -= 4; q_ += 4; } \
        if ((p_ & 8) && r_ >= 8) { __builtin_memcpy(&P##h8, q_, 8); p_ += 8; r_ -= 8; q_ += 8; } \
        const uint32_t nm_ = r_ >> 4;                                                            \
        if (nm_ > 0) __builtin_memcpy(&P##m0, q_, 16);                                           \
        if (nm_ > 1) __builtin_memcpy(&P##m1, q_ + 16, 16);                                      \
        if (nm_ > 2) __builtin_memcpy(&P##m2, q_ + 32, 16);                                      \
        if (nm_ > 3) __builtin_memcpy(&P##m3, q_ + 48, 16);                                      \
        q_ += 16 * nm_;                                                                          \
        r_ &= 15;                                                                                \
        if (r_ & 8) { __builtin_memcpy(&P##t8, q_, 8); q_ += 8; }                                \
        if (r_ & 4) { __builtin_memcpy(&P##t4, q_, 4); q_ += 4; }                                \
        if (r_ & 2) { uint16_t x_; __builtin_memcpy(&x_, q_, 2); P##t2 = x_; q_ += 2; }          \
        if (r_ & 1) P##t1 = q_[0];                                                               \
    }
#define RR_PIECE_STORE(P, IMG, DST, LEN)                                                         \
    {                                                                                            \
        uint8_t *i_ = (IMG);                                                                     \
        uint32_t p_ = (DST), r_ = (LEN);                                                         \
        if ((p_ & 1) && r_ >= 1) { i_[p_] = (uint8_t)P##h1; p_ += 1; r_ -= 1; }                  \
        if ((p_ & 2) && r_ >= 2) { *reinterpret_cast<uint16_t *>(i_ + p_) = (uint16_t)P##h2; p_ += 2; r_ -= 2; } \
        if ((p_ & 4) && r_ >= 4) { *reinterpret_cast<uint32_t *>(i_ + p_) = P##h4; p_ += 4; r_ -= 4; } \
        if ((p_ & 8) && r_ >= 8) { *reinterpret_cast<uint64_t *>(i_ + p_) = P##h8; p_ += 8; r_ -= 8; } \
        const uint32_t nm_ = r_ >> 4;                                                            \
        uint4 *m_ = reinterpret_cast<uint4 *>(i_ + p_);                                          \
        if (nm_ > 0) m_[0] = P##m0;                                                              \
        if (nm_ > 1) m_[1] = P##m1;                                                              \
        if (nm_ > 2) m_[2] = P##m2;                                                              \
        if (nm_ > 3) m_[3] = P##m3;                                                              \
        p_ += 16 * nm_;                                                                          \
        r_ &= 15;                                                                                \
        if (r_ & 8) { *reinterpret_cast<uint64_t *>(i_ + p_) = P##t8; p_ += 8; }                 \
        if (r_ & 4) { *reinterpret_cast<uint32_t *>(i_ + p_) = P##t4; p_ += 4; }                 \
        if (r_ & 2) { *reinterpret_cast<uint16_t *>(i_ + p_) = (uint16_t)P##t2; p_ += 2; }       \
        if (r_ & 1) i_[p_] = (uint8_t)P##t1;                                                     \
    }

// Granule copy of a piece aligned with its image offset mod 16 (RR_ENC_ALIGNED): up to four
// aligned 16-byte loads, each clamped to the piece's last granule; full granules stored as
// they are, partial ones masked and OR-ed into the zeroed image (no-return 64-bit LDS atomics).
// The piece's granules are visited in an order rotated by R (0-3): X##k holds granule (k + R) & 3
// of the piece.  With R = (lane / 4) mod 4, the 16 lanes a ds_write_b128 serves together — which
// hold consecutive 64-byte image blocks, i.e. four block phases mod 256 bytes — write 16
// distinct bank groups at every step instead of four lanes per 16-byte bank group.
#define RR_AL_LOAD(X, S, D, L, R)                                                                \
    u32x4 X##0 = {0u, 0u, 0u, 0u}, X##1 = X##0, X##2 = X##0, X##3 = X##0;                      \
    if ((L) > 0) {                                                                               \
        const uint32_t c0_ = (D) & ~15u, cl_ = ((D) + (L) - 1) & ~15u;                           \
        const u32x4 *g_ = reinterpret_cast<const u32x4 *>(arena + (S) - ((D) - c0_));            \
        X##0 = g_[c0_ + 16 * (((R) + 0) & 3) <= cl_ ? (((R) + 0) & 3) : 0];                      \
        X##1 = g_[c0_ + 16 * (((R) + 1) & 3) <= cl_ ? (((R) + 1) & 3) : 0];                      \
        X##2 = g_[c0_ + 16 * (((R) + 2) & 3) <= cl_ ? (((R) + 2) & 3) : 0];                      \
        X##3 = g_[c0_ + 16 * (((R) + 3) & 3) <= cl_ ? (((R) + 3) & 3) : 0];                      \
    }
#define RR_AL_CHUNK(XK, K, D, L)                                                                 \
    {                                                                                            \
        const uint32_t dc_ = ((D) & ~15u) + 16u * (K), e_ = (D) + (L);                           \
        if ((L) > 0 && dc_ < e_) {                                                               \
            const uint32_t lo_ = (D) > dc_ ? (D) - dc_ : 0u, hi_ = e_ < dc_ + 16u ? e_ - dc_ : 16u; \
            if (lo_ == 0 && hi_ == 16) {                                                         \
                img4[dc_ >> 4] = make_uint4(XK[0], XK[1], XK[2], XK[3]);                         \
            } else {                                                                             \
                _Pragma("unroll") for (uint32_t h_ = 0; h_ < 2; ++h_) {                          \
                    const uint32_t a_ = lo_ > 8 * h_ ? lo_ - 8 * h_ : 0u;                         \
                    const uint32_t b0_ = hi_ > 8 * h_ ? hi_ - 8 * h_ : 0u, b_ = b0_ < 8 ? b0_ : 8u; \
                    if (b_ > a_) {                                                               \
                        const uint64_t m_ = (~0ull >> (64 - 8 * (b_ - a_))) << (8 * a_);         \
                        const uint64_t v_ = (h_ ? ((uint64_t)XK[3] << 32 | XK[2])                \
                                                : ((uint64_t)XK[1] << 32 | XK[0])) & m_;         \
                        __hip_atomic_fetch_or(reinterpret_cast<uint64_t *>(img + dc_ + 8 * h_), v_, \
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);   \
                    }                                                                            \
                }                                                                                \
            }                                                                                    \
        }                                                                                        \
    }
#define RR_AL_STORE(X, D, L, R)                                                                  \
    RR_AL_CHUNK(X##0, ((R) + 0) & 3, D, L) RR_AL_CHUNK(X##1, ((R) + 1) & 3, D, L)                \
    RR_AL_CHUNK(X##2, ((R) + 2) & 3, D, L) RR_AL_CHUNK(X##3, ((R) + 3) & 3, D, L)

// Copy-run queue: one entry per payload (arena offset (40 bits) | length << 40, image offset,
// first piece); the copy phase splits the runs into 64-byte image-block pieces.
constexpr uint64_t JQ_SRC = (1ull << 40) - 1;


// copy pieces: 2^ENC_PS-byte image blocks (round 6: 16-byte pieces, one aligned load each and four
// pieces a thread in flight, measured within noise of 64-byte pieces: encode config 4 0.3748 vs
// 0.3754 ms, configs 3 and 2 +1 %; profiles/r6_encode_pieces_ab.txt)
constexpr uint32_t ENC_PS = 6;
// waves per SIMD the emit kernel is built for (74 VGPRs, no spills; 5: E4 345 us, 6: 307 us)
constexpr int ENC_WPE = 6;
template <uint32_t W, uint32_t NT, uint32_t RCAP>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(ENC_WPE))) void enc_emit_kernel(const rr_value *__restrict__ values,
                                                      const rr_elem *__restrict__ elems,
                                                      const uint8_t *__restrict__ arena, uint64_t n,
                                                      uint8_t *__restrict__ out, uint64_t cap,
                                                      const uint64_t *__restrict__ offsets,
                                                      const uint32_t *__restrict__ fv,
                                                      const uint64_t *__restrict__ stats, uint32_t ntiles,
                                                      rr_totals *tot, uint64_t *err, uint64_t *zsums, uint32_t nzsums) {
    static_assert(W <= 65536 && W % 64 == 0, "image offsets are 16-bit, pieces 64-byte blocks");
    static_assert(W % (16 * NT) == 0, "image stores: whole 16-byte chunks per thread");
    // block 0 also zeroes E1's group sums, which E3 (done) read: they are zero for the next call
    // without a zeroing launch (the context keeps them in its zero-between-calls buffer)
    if (blockIdx.x == 0)
        for (uint32_t k = threadIdx.x; k < nzsums; k += NT) zsums[k] = 0;
    // block 0 folds E1's and E3's tile totals into the call's totals before its window (a
    // separate finalize launch's work, hidden under the other windows: encode cfg 4 -1 %)
    if (tot && blockIdx.x == 0) fold_totals(stats, ntiles, offsets, n, tot, err);
    static_assert(RCAP >= 2 && (W >> ENC_PS) + RCAP < 65536, "run piece bases are 16-bit");
    __shared__ uint4 img4[W / 16];
    __shared__ uint64_t rq_a[RCAP];        // run: arena offset | length << 40
    __shared__ uint32_t rq_dp[RCAP];       // run: image offset | first piece (pieces of earlier runs) << 16
    __shared__ __attribute__((aligned(16))) uint32_t tb[NT + 1];   // task base of each value of the round
    // per value of the round: sv_pos, the output position of its first task (less the element-byte
    // scan there once its first task is costed), sv_el its elem_base, sv_te type | enc << 8
    __shared__ __attribute__((aligned(16))) uint64_t sv_raw[2 * NT];
    uint64_t *const sv_pos = sv_raw;
    uint32_t *const sv_el = reinterpret_cast<uint32_t *>(sv_raw + NT), *const sv_te = sv_el + NT;
    __shared__ uint64_t wsum[2][NT / RR_WAVE];
    __shared__ uint8_t dsrc[NT / RR_WAVE][RR_WAVE / 3 + 1];   // a wave's decimal lanes, in lane order
    __shared__ uint64_t sh_nrp;            // runs reserved | pieces reserved << 32
    __shared__ uint32_t sh_pend;           // pieces of the queued runs, when the queue overflowed
    __shared__ uint32_t sh_unal;           // some queued run is not aligned with its image offset mod 16
    uint8_t *img = reinterpret_cast<uint8_t *>(img4);
    const uint64_t total = offsets[n];
    const uint64_t lim = total < cap ? total : cap;
    const uint64_t w0 = (uint64_t)blockIdx.x * W;
    if (w0 >= lim) return;
    // the first round of the window's records and offsets, at the kernel's start: buffer loads (no
    // branches; lanes past the window's values read zeros), in flight under the image's zeroing
    // (encode config 4 -1.5 %, config 2 -5 %, profiles/r5_encode_persistent_ab.txt "p0")
    auto first_round = [&](uint64_t v0, uint64_t vend, uint64_t &a, uint64_t &b, uint4 &x) {
        const uint32_t nv = vend - v0 < NT ? (uint32_t)(vend - v0) : NT;
        const rsrc_t RO = make_rsrc(reinterpret_cast<const uint8_t *>(offsets + v0), (nv + 1) * 8u);
        const rsrc_t RV = make_rsrc(reinterpret_cast<const uint8_t *>(values + v0), nv * 16u);
        const uint32_t t = threadIdx.x;
        a = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(RO, (int)(t * 8), 0, 0));
        b = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(RO, (int)(t * 8 + 8), 0, 0));
        x = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(RV, (int)(t * 16), 0, 0));
    };
    // the window's value range [v0, vend): the values holding its bytes (fv from E3)
    const uint64_t v0 = fv[blockIdx.x];
    const uint64_t vend = w0 + W < total ? (uint64_t)fv[blockIdx.x + 1] + 1 : n;
    uint64_t pa, pb;
    uint4 px;
    first_round(v0, vend, pa, pb, px);
    const uint32_t tid = threadIdx.x;
    EPROBE(uint64_t et0 = rr_stamp(), etk = 0, ent = 0, tf = 0, tsc = 0, twr = 0, tw1 = 0, tw2 = 0;)
    const uint64_t span = lim - w0 < W ? lim - w0 : W;
    const Img I{img, w0, span};
#pragma unroll
    for (uint32_t k = tid; k < W / 16; k += NT) img4[k] = make_uint4(0, 0, 0, 0);
    if (tid == 0) { sh_nrp = 0; sh_pend = 0xFFFFFFFFu; sh_unal = 0; }
    lds_barrier();
    EPROBE(const uint64_t et1 = rr_stamp();)

    // Payload bytes [pos, pos+len) <- arena[src..]: clipped to the window and queued as one
    // run for the copy phase.  Called by every lane of the wave (want = false for none): the
    // run slot and its pieces are reserved together with one 64-bit LDS atomic per wave over
    // two wave prefix sums, so run order and piece order agree.
    auto payload = [&](bool want, uint64_t pos, uint64_t src, uint64_t len) {
        uint64_t d0 = pos < w0 ? w0 : pos, d1 = pos + len;
        if (d1 > w0 + span) d1 = w0 + span;
        want = want && d0 < d1;
        src += want ? d0 - pos : 0;
        const uint32_t dst = want ? (uint32_t)(d0 - w0) : 0, l = want ? (uint32_t)(d1 - d0) : 0;
        const bool queued = want && src + l <= JQ_SRC;
        const uint32_t np = queued ? ((dst + l - 1) >> ENC_PS) - (dst >> ENC_PS) + 1 : 0;
        const uint64_t mine = queued ? (1ull | ((uint64_t)np << 32)) : 0;
        // (the two 32-bit fields scanned apart in DPP: a wave's runs and pieces stay far below 2^32)
        const uint64_t incl = (uint64_t)wave_incl_scan_u32(queued ? 1u : 0u) |
                              ((uint64_t)wave_incl_scan_u32(queued ? np : 0u) << 32);
        const uint64_t wtot = ((uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)(incl >> 32), RR_WAVE - 1) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)incl, RR_WAVE - 1);
        uint64_t base = 0;
        if (wtot && lane_id() == RR_WAVE - 1) base = atomicAdd((unsigned long long *)&sh_nrp, (unsigned long long)wtot);
        base = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(base >> 32), RR_WAVE - 1) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, RR_WAVE - 1);   // (lane 63 took the atomic)
        if (!want) return;
        const uint64_t at = base + incl - mine;
        const uint32_t r = (uint32_t)at, p0 = (uint32_t)(at >> 32);
        if (queued && r < RCAP) {
            rq_a[r] = src | ((uint64_t)l << 40);
            rq_dp[r] = dst | (p0 << 16);
            if ((reinterpret_cast<uintptr_t>(arena) + src - dst) & 15) sh_unal = 1;
        } else {   // queue full (rare; keeps the kernel small): byte copy
            if (queued && r == RCAP) sh_pend = p0;
            for (uint32_t i = 0; i < l; ++i) img[dst + i] = arena[src + i];
        }
    };

    for (uint64_t vb = v0; vb < vend; vb += NT) {
        const uint64_t v = vb + tid;
        uint32_t tasks = 0;
        uint64_t a = pa, b = pb;
        uint4 x = px;
        if (vb != v0 && v < vend) {   // (rounds past the first: values of a window past NT)
            a = offsets[v];
            b = offsets[v + 1];
            x = reinterpret_cast<const uint4 *>(values)[v];
        }
        if (v < vend) {
            if (b > a && b <= cap) {
                const uint32_t type = x.x & 0xFF, enc = (x.x >> 8) & 0xFF, ne = x.z;
                // type, lru (5 bytes) then the type's fixed field: STRING enc (1), INTSET enc +
                // count (8), HT / skiplist count (8)
                const uint32_t fnb = type == RR_TYPE_STRING ? 1u : (type == RR_TYPE_SET_INTSET || type == RR_TYPE_SET_HT ||
                                                                    type == RR_TYPE_HASH_HT || type == RR_TYPE_ZSET_SKIPLIST) ? 8u : 0u;
                const uint64_t fv8 = type == RR_TYPE_STRING ? enc : type == RR_TYPE_SET_INTSET ? (enc | ((uint64_t)ne << 32))
                                   : type == RR_TYPE_SET_HT ? ne : (uint64_t)(ne / 2);
                for (uint32_t f = 0; f < 2; ++f) {
                    const uint32_t nb = f == 0 ? 5u : fnb;
                    if (nb && RR_ABLATE != 7) I.field(a + 5 * f, f == 0 ? (type | ((uint64_t)(x.y & RR_LRU_MASK) << 8)) : fv8, nb);
                }
                tasks = (type == RR_TYPE_HASH_ZIPLIST || type == RR_TYPE_ZSET_ZIPLIST) ? 1u : ne;
                sv_pos[tid] = a + enc_hdr(type);
                sv_el[tid] = x.w;
                sv_te[tid] = type | (enc << 8);
            }
        }
        uint64_t tt;
        const uint32_t base = (uint32_t)block_excl_scan<NT>(tasks, wsum[0], tt);
        tb[tid] = base;
        if (tid == NT - 1) tb[NT] = base + tasks;
        lds_barrier();
        EPROBE(const uint64_t eth = rr_stamp(); ent += tt;)
        uint64_t run = 0;   // element bytes of the earlier task rounds
        // (an LDS task -> value map as in E1 measured E4 +2 %, its 4 KiB more LDS per workgroup;
        // the search in two rounds of independent LDS reads +6 %: more LDS instructions in an
        // issue-bound kernel; four rounds' descriptors loaded together +12 %)
        auto fetch = [&](uint64_t t, uint32_t &pj, ElemV &pe) {
            pj = 0;
            pe = ElemV{0, 0, 0};
            if (t < tt) {
                // last value j with tb[j] <= t
                // (a per-chunk LDS task -> value map instead, built with a block-wide max fill:
                // encode config 4 +8-10 %, the fill's three barriers a chunk cost more than the
                // search's dependent reads; round 6, profiles/r6_encode_pieces_ab.txt)
                uint32_t lo = 0;
#pragma unroll
                for (uint32_t s = NT / 2; s > 0; s >>= 1)
                    if (tb[lo + s] <= t) lo += s;
                pj = lo;
                pe = get_elem(elems + sv_el[lo] + (uint32_t)(t - tb[lo]));
            }
        };
        auto round = [&](uint64_t r0, const uint32_t j, const ElemV &e) {
            EPROBE(const uint64_t rs0 = rr_stamp();)
            const uint64_t t = r0 + tid;
            const bool act = t < tt;
            uint64_t es = 0;
            uint32_t type = 0, enc = 0, k = 0;
            if (act) {
                k = (uint32_t)(t - tb[j]);
                type = sv_te[j] & 0xFF;
                enc = sv_te[j] >> 8;
                switch (type) {
                    case RR_TYPE_STRING: es = enc == RR_ENC_INT ? 8 : e.len; break;
                    case RR_TYPE_LIST_QUICKLIST:
                        es = 4 + (e.kind == RR_K_INT ? sdec_len((int64_t)e.data) : e.len);
                        break;
                    case RR_TYPE_SET_INTSET: es = enc; break;
                    case RR_TYPE_ZSET_SKIPLIST: es = (k & 1) ? 8 : 8 + (uint64_t)e.len; break;
                    default: es = 8 + (uint64_t)e.len; break;   // HT members, ziplist raw
                }
            }
            uint64_t rt;
            const uint64_t ex = run + block_excl_scan<NT>(es, wsum[1], rt);
            if (act && k == 0) sv_pos[j] -= ex;
            lds_barrier();
            EPROBE(const uint64_t rs1 = rr_stamp(); tsc += rs1 - rs0;)
            bool pay = false;
            uint64_t ppos = 0;
            [[maybe_unused]] bool isd = false;
            [[maybe_unused]] uint64_t dpos = 0;
            [[maybe_unused]] uint32_t dlen = 0;
            if (act) {
                const uint64_t p = sv_pos[j] + ex;
                // one fixed field, then a decimal or a payload (single call sites keep the
                // kernel small enough for the instruction cache)
                uint64_t fval = e.len;
                uint32_t fnb = 8, hdr = 8;
                pay = true;
                if (type == RR_TYPE_STRING) { fnb = 0; hdr = 0; if (enc == RR_ENC_INT) { fval = e.data; fnb = 8; pay = false; } }
                else if (type == RR_TYPE_LIST_QUICKLIST) { fval = es - 4; fnb = 4; hdr = 4; pay = e.kind != RR_K_INT; }
                else if (type == RR_TYPE_SET_INTSET) { fval = e.data; fnb = enc; pay = false; }
                else if (type == RR_TYPE_ZSET_SKIPLIST && (k & 1)) { fval = e.data; pay = false; }
                if (fnb && RR_ABLATE != 7 && RR_ABLATE != 10) I.field(p, fval, fnb);
                EPROBE(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const uint64_t rw1 = rr_stamp(); tw1 += rw1 - rs1;)
                if (type == RR_TYPE_LIST_QUICKLIST && !pay) { isd = true; dpos = p + 4; dlen = (uint32_t)(es - 4); }
                EPROBE(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const uint64_t rw2 = rr_stamp(); tw2 += rw2 - rw1;)
                ppos = p + hdr;
            }
            // integer List elements' decimals: a wave with at most 21 spreads each one's three
            // 8-digit chunks over three lanes (one SWAR conversion a lane instead of three: the
            // decimals were ~20 % of the kernel's VALU); lane 3i + c takes chunk c of the wave's
            // i-th decimal, whose lane it finds through a per-wave LDS list.  Round 6: E4 297.5 ->
            // 282.7 us, encode config 4 -2.3 % (profiles/r6_encode_pieces_ab.txt)
            {
                const uint64_t dm = __ballot(isd);
                const uint32_t nd = (uint32_t)__popcll(dm);
                if (nd && nd <= RR_WAVE / 3 && RR_ABLATE != 7 && RR_ABLATE != 9) {   // (wave-uniform)
                    const uint32_t ln = lane_id(), wv = tid / RR_WAVE;
                    if (isd) dsrc[wv][__builtin_amdgcn_mbcnt_hi((uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0u))] = (uint8_t)ln;
                    const uint32_t i = ln / 3, c = ln - 3 * i;
                    const uint32_t src = i < nd ? dsrc[wv][i] : ln;
                    const int64_t x = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * src), (int)(uint32_t)e.data)) |
                                                ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * src), (int)(uint32_t)(e.data >> 32)) << 32));
                    const uint64_t xp = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * src), (int)(uint32_t)dpos)) |
                                        ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * src), (int)(uint32_t)(dpos >> 32)) << 32);
                    const uint32_t xl = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * src), (int)dlen);
                    if (i < nd) I.decimal_chunk(xp, x, xl, c);
                } else if (isd && RR_ABLATE != 7 && RR_ABLATE != 9) {
                    I.decimal(dpos, (int64_t)e.data, dlen);
                }
            }
            payload(pay, ppos, e.data, e.len);
            run += rt;
            EPROBE(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const uint64_t rs2 = rr_stamp(); twr += rs2 - rs1;)
        };
        for (uint64_t g0 = 0; g0 < tt; g0 += NT) {
            uint32_t j0;
            ElemV e0;
            fetch(g0 + tid, j0, e0);
            round(g0, j0, e0);
        }
        lds_barrier();
        EPROBE(const uint64_t ett = rr_stamp(); etk += ett - eth;)
    }
    EPROBE(const uint64_t et2 = rr_stamp();)

    // payload pieces: piece b of the window -> its run (last run whose first piece <= b) ->
    // the run's k-th 64-byte image block
    const uint32_t nr = (uint32_t)sh_nrp < RCAP ? (uint32_t)sh_nrp : RCAP;
    const uint32_t npc = sh_pend != 0xFFFFFFFFu ? sh_pend : (uint32_t)(sh_nrp >> 32);
    // piece -> run map in the rounds' value arrays (free now): each queued run writes its index at
    // its first piece, then a block-wide running max fills the pieces after it (heads increase
    // along the map, the zeros between them never win) — one LDS read per piece instead of a
    // binary search of the runs' first pieces (9 dependent LDS reads per piece).  Round 6: encode
    // config 4 0.382 -> 0.371 ms and 0.384 -> 0.372 on one box, config 2 -1.5 %, config 3 within
    // noise (profiles/r6_encode_pieces_ab.txt)
    uint16_t *const pmap = reinterpret_cast<uint16_t *>(sv_raw);
    static_assert(8 * NT >= (W >> ENC_PS) + RCAP && 16 * NT <= sizeof(sv_raw), "piece map: 8 pieces a thread");
    if (npc) {   // (block-uniform)
        reinterpret_cast<uint4 *>(pmap)[tid] = make_uint4(0, 0, 0, 0);
        lds_barrier();
        for (uint32_t r = tid; r < nr; r += NT) pmap[rq_dp[r] >> 16] = (uint16_t)r;
        lds_barrier();
        const uint4 q = reinterpret_cast<const uint4 *>(pmap)[tid];
        const uint32_t qw[4] = {q.x, q.y, q.z, q.w};
        uint32_t m[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) m[k] = (qw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
#pragma unroll
        for (uint32_t k = 1; k < 8; ++k) m[k] = max(m[k], m[k - 1]);
        const uint32_t im = wave_incl_max_u32(m[7]);
        const uint32_t wv = tid / RR_WAVE;
        if (lane_id() == RR_WAVE - 1) wsum[0][wv] = im;
        lds_barrier();
        uint32_t carry = wave_from_prev(im);   // (lane 0: 0; every lane runs the DPP)
#pragma unroll
        for (uint32_t k = 0; k < NT / RR_WAVE; ++k) carry = k < wv ? max(carry, (uint32_t)wsum[0][k]) : carry;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) m[k] = max(carry, m[k]);
        reinterpret_cast<uint4 *>(pmap)[tid] = make_uint4(m[0] | m[1] << 16, m[2] | m[3] << 16, m[4] | m[5] << 16, m[6] | m[7] << 16);
        lds_barrier();
    }
    auto piece = [&](uint32_t b, uint64_t &ps, uint32_t &pd, uint32_t &pl) {
        const uint32_t lo = pmap[b];
        const uint64_t a = rq_a[lo];
        const uint32_t dp = rq_dp[lo], dst = dp & 0xFFFF, l = (uint32_t)(a >> 40),
                       k = b - (dp >> 16);
        const uint32_t d0 = k == 0 ? dst : ((dst >> ENC_PS) + k) << ENC_PS;
        const uint32_t e1 = (((dst >> ENC_PS) + k + 1) << ENC_PS), e = e1 < dst + l ? e1 : dst + l;
        ps = (a & JQ_SRC) + (d0 - dst);
        pd = d0;
        pl = e > d0 ? e - d0 : 0;   // (inside one 2^ENC_PS-byte block by construction)
    };
    // Every run aligned with its image offset mod 16 (any arena that keeps the blob layout, the
    // decode's mirror arena included): pieces move whole granules (RR_AL_LOAD / RR_AL_STORE).
    // A window with any other run takes the byte plan below for all its pieces.
    if (RR_ABLATE == 8) {   // timing only (wrong results): no payload copies
    } else if (sh_unal == 0) {
        for (uint32_t j = tid; j < npc; j += 2 * NT) {
            const bool two = j + NT < npc;
            uint64_t s0, s1 = 0;
            uint32_t d0, l0, d1 = 0, l1 = 0;
            piece(j, s0, d0, l0);
            if (two) piece(j + NT, s1, d1, l1);
            const uint32_t rot = 0;   // (rotated per lane group for LDS bank spread: within noise)
            RR_AL_LOAD(xa, s0, d0, l0, rot)
            RR_AL_LOAD(xb, s1, d1, l1, rot)
            RR_AL_STORE(xa, d0, l0, rot)
            RR_AL_STORE(xb, d1, l1, rot)
        }
    } else
        for (uint32_t j = tid; j < npc; j += 2 * NT) {
        const bool two = j + NT < npc;
        uint64_t s0, s1 = 0;
        uint32_t d0, l0, d1 = 0, l1 = 0;
        piece(j, s0, d0, l0);
        if (two) piece(j + NT, s1, d1, l1);
        RR_PIECE_LOAD(a_, arena + s0, d0, l0)
        RR_PIECE_LOAD(b_, arena + s1, d1, l1)
        RR_PIECE_STORE(a_, img, d0, l0)
        RR_PIECE_STORE(b_, img, d1, l1)
    }
    lds_barrier();
    EPROBE(const uint64_t et3 = rr_stamp();)

    // store the image: 16-byte chunks (buffer stores: chunks past the window's span are dropped,
    // every thread issues the same W / 16 / NT stores), then the bytes of a partial last chunk
    {
        const rsrc_t RS = make_rsrc(out + w0, (uint32_t)span & ~15u);
        const u32x4 *src4 = reinterpret_cast<const u32x4 *>(img4);
#pragma unroll
        for (uint32_t k = 0; k < W / 16 / NT; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(src4[tid + k * NT], RS, (int)((tid + k * NT) * 16), 0, 2 /* nt */);
        const uint32_t full = (uint32_t)(span >> 4), tail = (uint32_t)(span & 15);
        const rsrc_t RT = make_rsrc(out + w0 + 16ull * full, tail);
        __builtin_amdgcn_raw_buffer_store_b8(img[(16u * full + (tid & 15u)) & (W - 1)], RT, (int)tid, 0, 0);
    }
    EPROBE(const uint64_t et4 = rr_stamp();
           if (tid == 0 && g_eprobe) {
               uint64_t *o = g_eprobe + (uint64_t)blockIdx.x * EPROBE_WORDS;
               o[0] = et1 - et0; o[1] = (et2 - et1) - etk; o[2] = etk; o[3] = et3 - et2; o[4] = et4 - et3;
               o[5] = et4 - et0; o[6] = vend - v0; o[7] = ent; o[8] = npc;
               o[9] = tw1; o[10] = tsc; o[11] = twr; o[12] = tw2;
           })
}

// ---- small batches: the whole encode in one launch --------------------------------------
// serObject runs once per evicted key on the main thread (rock.c:691, from the <= 64-pick loop
// at rock_hotkey.c:347).  A batch of at most SMALL_N values whose output is at most
// SMALL_BYTES (data_cap) is encoded by ONE workgroup in ONE launch: sizes per value
// (encode_size, E1's rule and statuses), an in-block scan for the offsets, the capacity cut
// (E3's), each value written by its lane into a zeroed LDS image (serObject's layout, E4's
// bytes), the image stored with 16-byte stores (the output may be pinned host memory mapped
// into the device: rr_encode_batch_host), the totals.  Same offsets, bytes and totals as the
// pipeline.
__device__ __forceinline__ void img_le(uint8_t *img, uint64_t p, uint64_t v, uint32_t nb) {
    for (uint32_t i = 0; i < nb; ++i) img[p + i] = (uint8_t)(v >> (8 * i));
}
__device__ __forceinline__ void img_copy(uint8_t *img, uint64_t p, const uint8_t *__restrict__ src, uint64_t len) {
    for (uint64_t i = 0; i < len; ++i) img[p + i] = src[i];
}
// serObject's bytes of one encodable value (rock_serdes.c:512-535) at image offset p
__device__ void emit_value_small(uint8_t *img, uint64_t p, const uint4 &x, const rr_elem *__restrict__ elems,
                                 const uint8_t *__restrict__ arena) {
    const uint32_t type = x.x & 0xFF, enc = (x.x >> 8) & 0xFF, ne = x.z;
    const rr_elem *el = elems + x.w;
    img_le(img, p, type | ((uint64_t)(x.y & RR_LRU_MASK) << 8), 5);   // serObjectType + lru
    p += 5;
    switch (type) {
        case RR_TYPE_STRING: {                                         // serString :114-128
            const ElemV e = get_elem(el);
            img[p++] = (uint8_t)enc;
            if (enc == RR_ENC_INT) img_le(img, p, e.data, 8);
            else img_copy(img, p, arena + e.data, e.len);
            return;
        }
        case RR_TYPE_HASH_ZIPLIST:                                     // serHash :314-331
        case RR_TYPE_ZSET_ZIPLIST: {                                   // serZset :417-428
            const ElemV e = get_elem(el);
            img_le(img, p, e.len, 8);
            img_copy(img, p + 8, arena + e.data, e.len);
            return;
        }
        case RR_TYPE_LIST_QUICKLIST:                                   // serList :162-188
            for (uint32_t k = 0; k < ne; ++k) {
                const ElemV e = get_elem(el + k);
                if (e.kind == RR_K_INT) {   // sdsll2str
                    const uint32_t l = dec_write(img + p + 4, (int64_t)e.data);
                    img_le(img, p, l, 4);
                    p += 4 + l;
                } else {
                    img_le(img, p, e.len, 4);
                    img_copy(img, p + 4, arena + e.data, e.len);
                    p += 4 + e.len;
                }
            }
            return;
        case RR_TYPE_SET_INTSET:                                       // serSet :217-233
            img_le(img, p, enc | ((uint64_t)ne << 32), 8);
            p += 8;
            for (uint32_t k = 0; k < ne; ++k, p += enc) img_le(img, p, get_elem(el + k).data, enc);
            return;
        default: {                                                     // HT set / hash :234-245, :332-346; skiplist :429-446
            img_le(img, p, type == RR_TYPE_SET_HT ? ne : ne / 2, 8);
            p += 8;
            for (uint32_t k = 0; k < ne; ++k) {
                const ElemV e = get_elem(el + k);
                if (type == RR_TYPE_ZSET_SKIPLIST && (k & 1)) { img_le(img, p, e.data, 8); p += 8; continue; }
                img_le(img, p, e.len, 8);
                img_copy(img, p + 8, arena + e.data, e.len);
                p += 8 + e.len;
            }
            return;
        }
    }
}

// encode_size with the whole wave on one value (its elements one per lane): the same size,
// payload and status
__device__ uint64_t encode_size_wave(uint32_t type, uint32_t enc, uint32_t vstatus, uint64_t eb, uint64_t n,
                                     const rr_elem *elems, uint64_t ecap, uint64_t acap, uint32_t &st, uint64_t &pay) {
    const bool multi = (type == RR_TYPE_LIST_QUICKLIST || type == RR_TYPE_SET_HT || type == RR_TYPE_HASH_HT ||
                        type == RR_TYPE_ZSET_SKIPLIST || (type == RR_TYPE_SET_INTSET && (enc == 2 || enc == 4 || enc == 8))) &&
                       vstatus == RR_OK && eb + n <= ecap &&
                       !((type == RR_TYPE_HASH_HT || type == RR_TYPE_ZSET_SKIPLIST) && (n & 1));
    if (!multi) return encode_size(type, enc, vstatus, eb, n, elems, ecap, acap, st, pay);
    uint64_t sz = 0, p = 0;
    bool bad = false;
    for (uint64_t i = lane_id(); i < n; i += RR_WAVE) {
        const ElemCost c = elem_cost(type, enc, i, get_elem(elems + eb + i), acap);
        sz += c.bytes;
        p += c.pay;
        bad |= c.bad;
    }
    sz = wave_sum_fast(sz) + (type == RR_TYPE_LIST_QUICKLIST ? 5 : 13);
    p = wave_sum_fast(p);
    if (__ballot(bad)) { st = RR_E_ENCODE; pay = 0; return 0; }
    st = RR_OK;
    pay = p;
    return sz;
}

// The same bytes with the whole wave on one value (the per-key calls, n <= SMALL_GW): lane 0
// writes the header, the elements go one per lane — sizes, a wave scan for their offsets, each
// lane its element's fields and payload — and a single string / ziplist payload is copied by
// all lanes.
__device__ void emit_value_wave(uint8_t *img, uint64_t p, const uint4 &x, const rr_elem *__restrict__ elems,
                                const uint8_t *__restrict__ arena) {
    const uint32_t lane = lane_id();
    const uint32_t type = x.x & 0xFF, enc = (x.x >> 8) & 0xFF, ne = x.z;
    const rr_elem *el = elems + x.w;
    if (lane == 0) img_le(img, p, type | ((uint64_t)(x.y & RR_LRU_MASK) << 8), 5);   // serObjectType + lru
    p += 5;
    if (type == RR_TYPE_STRING || type == RR_TYPE_HASH_ZIPLIST || type == RR_TYPE_ZSET_ZIPLIST) {
        const ElemV e = get_elem(el);
        const bool str = type == RR_TYPE_STRING;
        if (lane == 0) {
            if (str) img[p] = (uint8_t)enc;
            else img_le(img, p, e.len, 8);
            if (str && enc == RR_ENC_INT) img_le(img, p + 1, e.data, 8);
        }
        if (!(str && enc == RR_ENC_INT)) {
            const uint64_t q = p + (str ? 1 : 8);
            for (uint64_t i = lane; i < e.len; i += RR_WAVE) img[q + i] = arena[e.data + i];
        }
        return;
    }
    const bool list = type == RR_TYPE_LIST_QUICKLIST, is = type == RR_TYPE_SET_INTSET;
    if (lane == 0 && !list) img_le(img, p, is ? (enc | ((uint64_t)ne << 32)) : type == RR_TYPE_SET_HT ? ne : ne / 2, 8);
    if (!list) p += 8;
    for (uint32_t b = 0; b < ne; b += RR_WAVE) {
        const uint32_t k = b + lane;
        const bool act = k < ne;
        const ElemV e = act ? get_elem(el + k) : ElemV{0, 0, 0};
        // this element's bytes (serList :162-188, serSet :217-245, serHash :332-346, serZset :429-446)
        uint32_t sz = 0;
        if (act) {
            if (list) sz = 4 + (e.kind == RR_K_INT ? sdec_len((int64_t)e.data) : e.len);
            else if (is) sz = enc;
            else if (type == RR_TYPE_ZSET_SKIPLIST && (k & 1)) sz = 8;
            else sz = 8 + e.len;
        }
        const uint32_t incl = wave_incl_scan_u32(sz);
        const uint64_t q = p + incl - sz;
        if (act) {
            if (list && e.kind == RR_K_INT) {
                const uint32_t l = dec_write(img + q + 4, (int64_t)e.data);
                img_le(img, q, l, 4);
            } else if (list) {
                img_le(img, q, e.len, 4);
                img_copy(img, q + 4, arena + e.data, e.len);
            } else if (is || (type == RR_TYPE_ZSET_SKIPLIST && (k & 1))) {
                img_le(img, q, e.data, sz);
            } else {
                img_le(img, q, e.len, 8);
                img_copy(img, q + 8, arena + e.data, e.len);
            }
        }
        p += (uint32_t)__builtin_amdgcn_readlane((int)incl, RR_WAVE - 1);
    }
}

__global__ __launch_bounds__(SMALL_NT) void encode_small_kernel(const rr_value *__restrict__ values,
                                                                const rr_elem *__restrict__ elems, uint64_t ecap,
                                                                const uint8_t *__restrict__ arena, uint64_t acap,
                                                                uint64_t n, uint8_t *__restrict__ out, uint64_t cap,
                                                                uint64_t *__restrict__ offsets, rr_totals *tot,
                                                                uint32_t *done, uint32_t seq) {
    __shared__ __attribute__((aligned(16))) uint8_t img[SMALL_BYTES + 16];
    __shared__ uint64_t wsum[SMALL_NT / RR_WAVE], red[3][SMALL_NT / RR_WAVE];
    __shared__ u32x4 ein[SMALL_EIN / 16];
    __shared__ uint64_t s_at[SMALL_GW];   // (the wave path: each value's image offset, ~0 = not written)
    __shared__ uint64_t s_sz[SMALL_GW], s_pv[SMALL_GW];   // (the wave path: sizes, payloads, statuses)
    __shared__ uint32_t s_st[SMALL_GW];
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid / RR_WAVE;
    // The inputs into LDS first when they fit SMALL_EIN (the per-key calls): one 16-byte load per
    // thread, all in flight, instead of the emission's dependent loads — over PCIe when the inputs
    // are the host entry point's mapped staging.  (Nothing read past the arena's end.)
    {
        static_assert(SMALL_EIN / 16 <= SMALL_NT, "one granule per thread");
        const uint64_t gv = n, ge = ecap, ga = (acap + 15) / 16;
        if ((gv + ge + ga) * 16 <= SMALL_EIN && ((uintptr_t)values & 15) == 0 && ((uintptr_t)elems & 15) == 0 &&
            ((uintptr_t)arena & 15) == 0) {   // (uniform)
            const uint64_t g = tid;
            if (g < gv + ge + ga) {
                u32x4 x;
                if (g < gv) {
                    x = reinterpret_cast<const u32x4 *>(values)[g];
                } else if (g < gv + ge) {
                    x = reinterpret_cast<const u32x4 *>(elems)[g - gv];
                } else {
                    const uint64_t k = g - gv - ge;
                    if (16 * k + 16 <= acap) {
                        x = reinterpret_cast<const u32x4 *>(arena)[k];
                    } else {   // the last, partial granule
                        uint8_t b[16] = {};
                        for (uint32_t i = 0; i < acap - 16 * k; ++i) b[i] = arena[16 * k + i];
                        __builtin_memcpy(&x, b, 16);
                    }
                }
                ein[g] = x;
            }
            values = reinterpret_cast<const rr_value *>(ein);
            elems = reinterpret_cast<const rr_elem *>(ein + gv);
            arena = reinterpret_cast<const uint8_t *>(ein + gv + ge);
            __syncthreads();
        }
    }
    const uint64_t v0 = (uint64_t)tid * SMALL_VPT;
    const bool wave_path = n <= SMALL_GW;   // (uniform)
    if (wave_path) {
        // the few values' sizes with a wave on each (its elements one per lane)
        for (uint32_t v = wave; v < n; v += SMALL_NT / RR_WAVE) {
            const uint4 xv = reinterpret_cast<const uint4 *>(values)[v];
            uint32_t st;
            uint64_t pv;
            const uint64_t sz = encode_size_wave(xv.x & 0xFF, (xv.x >> 8) & 0xFF, xv.x >> 16, xv.w, xv.z, elems, ecap, acap,
                                                 st, pv);
            if (lane == 0) { s_sz[v] = sz; s_pv[v] = pv; s_st[v] = st; }
        }
        __syncthreads();
    }
    uint4 x[SMALL_VPT];
    uint64_t sz[SMALL_VPT], pv[SMALL_VPT], sum = 0, bad = 0, pay = 0, nel = 0;
#pragma unroll
    for (uint32_t j = 0; j < SMALL_VPT; ++j) {
        sz[j] = pv[j] = 0;
        x[j] = make_uint4(0, 0, 0, 0);
        if (v0 + j < n) {
            x[j] = reinterpret_cast<const uint4 *>(values)[v0 + j];
            uint32_t st;
            if (wave_path) {
                sz[j] = s_sz[v0 + j];
                pv[j] = s_pv[v0 + j];
                st = s_st[v0 + j];
            } else {
                sz[j] = encode_size(x[j].x & 0xFF, (x[j].x >> 8) & 0xFF, x[j].x >> 16, x[j].w, x[j].z, elems, ecap, acap, st,
                                    pv[j]);
            }
            bad += st != RR_OK ? 1u : 0u;
            nel += x[j].z;
        }
        sum += sz[j];
    }
    uint64_t total;
    uint64_t a = block_excl_scan<SMALL_NT>(sum, wsum, total);
    const uint64_t lim = total < cap ? total : cap;   // (cap <= SMALL_BYTES: rr_small_encode_fits)
    for (uint32_t k = tid; k < (lim + 31) / 16; k += SMALL_NT) reinterpret_cast<uint4 *>(img)[k] = make_uint4(0, 0, 0, 0);
    __syncthreads();
#pragma unroll 1
    for (uint32_t j = 0; j < SMALL_VPT; ++j) {
        if (v0 + j < n) {
            offsets[v0 + j] = a;
            const uint64_t b = a + sz[j];
            const bool emit = !(b > cap && sz[j]) && sz[j];
            if (b > cap && sz[j]) { bad += 1; }                     // past data_cap: not written (E3)
            else pay += pv[j];
            if (wave_path) s_at[v0 + j] = emit ? a : ~0ull;
            else if (emit) emit_value_small(img, a, x[j], elems, arena);
            a = b;
        }
    }
    // (LDS-only barriers after the offsets stores: __syncthreads() would wait for their
    // acknowledgements, a PCIe round trip when they go to the host entry point's mapped staging)
    if (wave_path) {
        lds_barrier();
        for (uint32_t v = wave; v < n; v += SMALL_NT / RR_WAVE)
            if (s_at[v] != ~0ull) emit_value_wave(img, s_at[v], reinterpret_cast<const uint4 *>(values)[v], elems, arena);
    }
    if (tid == 0) offsets[n] = total;
    bad = wave_sum_fast(bad);
    pay = wave_sum_fast(pay);
    nel = wave_sum_fast(nel);
    if (lane == 0) { red[0][wave] = bad; red[1][wave] = pay; red[2][wave] = nel; }
    lds_barrier();
    // the image out: 16-byte stores, bytes at a partial end (as E4)
    const uint32_t full = (uint32_t)(lim >> 4);
    for (uint32_t c = tid; c < full; c += SMALL_NT) reinterpret_cast<uint4 *>(out)[c] = reinterpret_cast<const uint4 *>(img)[c];
    if (tid < (lim & 15)) out[16ull * full + tid] = img[16u * full + tid];
    if (tid == 0) {
        uint64_t tb = 0, tp = 0, tn = 0;
        for (uint32_t w = 0; w < SMALL_NT / RR_WAVE; ++w) { tb += red[0][w]; tp += red[1][w]; tn += red[2][w]; }
        tot->n_bad = tb;
        tot->payload = tp;
        tot->n_elems = tn;
        tot->bytes = total;
    }
    signal_done(done, seq);
}

}  // namespace

extern "C" int rr_small_decode_fits(uint64_t n, uint64_t data_cap) {
    return n <= SMALL_N && data_cap <= SMALL_BYTES && (n <= SMALL_GW || data_cap <= n * SMALL_LANE_BYTES);
}
extern "C" hipError_t rr_launch_decode_small(const uint8_t *blob, const uint64_t *offsets, uint64_t n, rr_value *values,
                                             rr_elem *elems, uint64_t elem_cap, uint8_t *arena, uint64_t data_cap,
                                             rr_totals *totals, uint32_t *done, uint32_t seq, hipStream_t stream) {
    hipLaunchKernelGGL(decode_small_kernel, dim3(1), dim3(SMALL_NT), 0, stream, blob, offsets, n, values, elems, elem_cap,
                       arena, data_cap, totals, done, seq);
    return hipGetLastError();
}

// ---- the pipelined host encode: which arena bytes a chunk of values reads ----------------
// The largest end (data + len) of the STR / ZLRAW descriptors of the values the encode will read
// (status RR_OK, descriptors inside elem_cap: encode_size's conditions), clamped to arena_cap:
// each of NEED_BLOCKS workgroups stores its part's maximum into a word of mapped host memory,
// and the host lets the chunk's encode start once that much of the arena has been uploaded.
__global__ __launch_bounds__(1024) void arena_need_kernel(const rr_value *__restrict__ values, uint64_t n,
                                                          const rr_elem *__restrict__ elems, uint64_t ecap,
                                                          uint64_t acap, uint64_t *need) {
    __shared__ uint64_t wm[16];
    uint64_t m = 0;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 x = reinterpret_cast<const uint4 *>(values)[v];
        const uint64_t eb = x.w, ne = x.z;
        if ((x.x >> 16) != RR_OK || eb + ne > ecap) continue;
        for (uint64_t k = 0; k < ne; ++k) {
            const uint4 d = reinterpret_cast<const uint4 *>(elems + eb)[k];
            const uint32_t kind = d.w & 0xFF;
            if (kind == RR_K_STR || kind == RR_K_ZLRAW) {
                const uint64_t end = ((uint64_t)d.x | ((uint64_t)d.y << 32)) + d.z;
                m = end > m ? end : m;
            }
        }
    }
    for (int o = RR_WAVE / 2; o > 0; o >>= 1) {
        const uint64_t y = __shfl_xor(m, o, RR_WAVE);
        m = y > m ? y : m;
    }
    if (lane_id() == 0) wm[threadIdx.x / RR_WAVE] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t w = 0; w < blockDim.x / RR_WAVE; ++w) m = wm[w] > m ? wm[w] : m;
        need[blockIdx.x] = m < acap ? m : acap;
    }
}
extern "C" hipError_t rr_launch_arena_need(const rr_value *values, uint64_t n, const rr_elem *elems, uint64_t elem_cap,
                                           uint64_t arena_cap, uint64_t *need, hipStream_t stream) {
    hipLaunchKernelGGL(arena_need_kernel, dim3(RR_NEED_BLOCKS), dim3(1024), 0, stream, values, n, elems, elem_cap, arena_cap,
                       need);
    return hipGetLastError();
}

extern "C" int rr_small_encode_fits(uint64_t n, uint64_t data_cap) {
    return n > 0 && n <= SMALL_N && data_cap <= SMALL_BYTES && (n <= SMALL_GW || data_cap <= n * SMALL_LANE_BYTES);
}
extern "C" hipError_t rr_launch_encode_small(const rr_value *values, const rr_elem *elems, uint64_t elem_cap,
                                             const uint8_t *arena, uint64_t arena_cap, uint64_t n, uint8_t *out,
                                             uint64_t cap, uint64_t *offsets, rr_totals *totals, uint32_t *done,
                                             uint32_t seq, hipStream_t stream) {
    hipLaunchKernelGGL(encode_small_kernel, dim3(1), dim3(SMALL_NT), 0, stream, values, elems, elem_cap, arena, arena_cap,
                       n, out, cap, offsets, totals, done, seq);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------- launch
#ifndef RR_DEC_W
#define RR_DEC_W 73728
#endif
#ifndef RR_DEC_SLACK
#define RR_DEC_SLACK 4096
#endif
#ifndef RR_DEC_NW
#define RR_DEC_NW 8
#endif
constexpr uint32_t DEC_W = RR_DEC_W, DEC_NW = RR_DEC_NW;
// (values per sort chunk: one per thread, the chunk's slot scan)
#define DECODE_KERNEL decode_kernel<RR_DEC_W, RR_DEC_SLACK, RR_DEC_NW, RR_DEC_NW * RR_WAVE>
#define DECODE_ONE decode_kernel<RR_DEC_W, RR_DEC_SLACK, RR_DEC_NW, RR_DEC_NW * RR_WAVE, true>
// (RR_DEC_ONE=0 in the environment: the two-launch form for every batch — A/B runs only)
static bool dec_one(void) {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("RR_DEC_ONE");
        v = !(e && e[0] == '0');
    }
    return v != 0;
}


// Resident workgroup count for a persistent launch: occupancy query minus one block per CU
// (the API over-reports by one for SGPR-heavy kernels, MI355X_MICROARCH.md §Residency).
template <typename K>
static uint32_t resident_grid(K kernel, int block, bool margin = true) {
    int dev = 0, cus = 0, occ = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, block, 0) != hipSuccess || occ < 1) occ = 1;
    if (margin && occ > 1) occ -= 1;
    if (cus < 1) cus = 1;
    return (uint32_t)(cus * occ);
}

static uint64_t scan_tiles(uint64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }

// windows: sized from data_cap (>= offsets[n], host-known without a sync); windows past
// offsets[n] own no values and copy nothing
// The window size of a call: the batch cut into whole generations of the resident windows (two
// per CU), each window as close to DEC_W as that allows — so the last generation is not a
// partial one that leaves most CUs idle (config 4 at 1M values: 14 generations of 69.4 KiB
// windows instead of 13.2 of 72 KiB), and a small batch spreads over every CU instead of a
// few full windows (config 1 at 100K values: 512 windows of 13.7 KiB instead of 98).
constexpr uint64_t DEC_WMIN = 1024;
// Per-device launch facts: the calling thread's current device, which every entry
// point of rr_api.c sets to its context's device first; one slot per device id, filled by
// whichever thread gets there first (racing threads store the same value)
constexpr int RR_MAX_DEV = 64;
static uint32_t dev_cache(uint32_t (&cache)[RR_MAX_DEV], uint32_t (*query)(void)) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    uint32_t *slot = &cache[(uint32_t)dev % RR_MAX_DEV];
    uint32_t v = __atomic_load_n(slot, __ATOMIC_RELAXED);
    if (!v) {
        v = query();
        __atomic_store_n(slot, v, __ATOMIC_RELAXED);
    }
    return v;
}
static uint32_t q_dec_slots(void) { return resident_grid(DECODE_KERNEL, DEC_NW * RR_WAVE, false); }
static uint32_t q_cus(void) {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
    return c > 0 ? (uint32_t)c : 1u;
}
static uint32_t g_dec_slots[RR_MAX_DEV], g_cus[RR_MAX_DEV];
static uint32_t dec_slots(void) { return dev_cache(g_dec_slots, q_dec_slots); }
static uint32_t dev_cus(void) { return dev_cache(g_cus, q_cus); }
static uint32_t dec_win(uint64_t data_cap) {
    const uint64_t slots = dec_slots();
    const uint64_t per_gen = slots * DEC_W, gens = (data_cap + per_gen - 1) / per_gen;
    uint64_t w = gens ? (data_cap + gens * slots - 1) / (gens * slots) : DEC_WMIN;
    w = (w + 15) & ~15ull;
    return (uint32_t)(w < DEC_WMIN ? DEC_WMIN : w > DEC_W ? DEC_W : w);
}
static uint64_t dec_windows(uint64_t data_cap) { return data_cap / dec_win(data_cap) + 1; }

// Decode scratch (uint64 words): [HDR] [reservations u32, n] [first_val u32, nwin + 1]
// [first_off, nwin + 1] [class bytes, n].  The window and group sums are in a buffer of their
// own (rr_decode_sums_words), zero between calls; count_kernel's block 0 zeroes the totals.
// Launches: count_kernel, decode_kernel.  (Round 3 ran a look-back scan of the
// reservations between the two — 15.4 us on config 4 — and a fourth kernel for the fixup and
// the totals fold — 5.6 us.  Measured dead ends, in git history: a fused single-pass decode
// with a window-level look-back, 0.401 vs 0.353 ms — the look-back waits ~5 us per window
// generation; count + scan in one launch with an in-kernel look-back, +40 us.)
static uint64_t dec_groups(uint64_t nw) { return nw / WGROUP + 1; }
extern "C" uint64_t rr_decode_scratch_words(uint64_t data_cap, uint64_t n) {
    const uint64_t nw = dec_windows(data_cap);
    return RR_SCRATCH_HDR + (n + 2) / 2 + (nw + 2) / 2 + (nw + 1) + (n + 7) / 8 + 2;
}
// The sums (one half of the context's double buffer): [window sums, nwin] [group sums, nwin / WGROUP + 1],
// or the one-launch form's words (one_words(nwin) <= this)
extern "C" uint64_t rr_decode_sums_words(uint64_t data_cap) {
    const uint64_t nw = dec_windows(data_cap), two = nw + dec_groups(nw);
    return two > one_words(nw) ? two : one_words(nw);
}

extern "C" hipError_t rr_launch_decode(const uint8_t *blob, const uint64_t *offsets, uint64_t n, rr_value *values,
                                       rr_elem *elems, uint64_t elem_cap, uint8_t *arena, uint64_t *scratch,
                                       uint64_t *sums, uint64_t *zero, uint64_t nzero, uint64_t data_cap,
                                       rr_totals *totals, hipStream_t stream, int first_only) {
    uint32_t win = dec_win(data_cap), nw = (uint32_t)(data_cap / win + 1);
    // A small batch that fits one window per CU, at most a sort chunk (512 values) a window, gets
    // one window per CU instead of two: config 1 at 100K values 22.0 -> 19.1 us, config 2 / 4 at
    // 30K values -16 % / -10 %; at 200K config-1 values (781 a window) two per CU stay faster
    // (profiles/r5_small_windows_ab.txt).  Fewer windows than dec_windows(data_cap): the scratch
    // and the sums sized from data_cap still cover them.
    const uint64_t cus = dev_cus();
    if (data_cap <= cus * DEC_W && n <= cus * DEC_NW * RR_WAVE) {
        uint64_t w = ((data_cap + cus - 1) / cus + 15) & ~15ull;
        w = w < DEC_WMIN ? DEC_WMIN : w;
        if (w > win) {
            win = (uint32_t)w;
            nw = (uint32_t)(data_cap / win + 1);
        }
    }
    // A batch of one generation of windows: one launch (decode_kernel's ONE form) instead of
    // count_kernel + decode_kernel.  (The debug hook that withholds the second launch keeps the
    // two-launch form, which it tests.)
    uint64_t *wtot = sums;
    uint64_t *gtot = wtot + nw;
    uint32_t *counts = reinterpret_cast<uint32_t *>(scratch + RR_SCRATCH_HDR);
    uint32_t *first_val = counts + ((n + 2) & ~1ull);
    uint64_t *first_off = reinterpret_cast<uint64_t *>(first_val + ((nw + 2) & ~1u));
    uint8_t *cls = reinterpret_cast<uint8_t *>(first_off + nw + 1);
    if (first_only != 1 && nw <= dec_slots() && nw <= DEC_NW * RR_WAVE && dec_one()) {   // (a look-back thread per earlier window)
        hipLaunchKernelGGL((DECODE_ONE), dim3(nw), dim3(DEC_NW * RR_WAVE), 0, stream, blob, data_cap, offsets, n,
                           nullptr, nullptr, cls, counts, nullptr, nullptr, values, elems, elem_cap, arena, nw, win,
                           totals, sums, zero, nzero, (uint32_t)(first_only == 2));
        return hipGetLastError();
    }
    if (data_cap < (1ull << 32))
        hipLaunchKernelGGL(count_kernel<true>, dim3((uint32_t)((n + 1 + 255) / 256)), dim3(256), 0, stream, blob, offsets, n,
                           first_val, first_off, nw, win, counts, cls, wtot, gtot, zero, nzero, totals);
    else
        hipLaunchKernelGGL(count_kernel<false>, dim3((uint32_t)((n + 1 + 255) / 256)), dim3(256), 0, stream, blob, offsets,
                           n, first_val, first_off, nw, win, counts, cls, wtot, gtot, zero, nzero, totals);
    if (first_only == 1) return hipGetLastError();
    hipLaunchKernelGGL((DECODE_KERNEL), dim3(nw), dim3(DEC_NW * RR_WAVE), 0, stream, blob, data_cap, offsets, n,
                       first_val, first_off, cls, counts, wtot, gtot, values, elems, elem_cap, arena, nw, win, totals,
                       nullptr, nullptr, 0, 0u);
    return hipGetLastError();
}

// Encode scratch (uint64 words): [HDR] [error word] [tile stats, 3 per 256 values, twice]
// [block sums, t] [group sums, t / WGROUP + 1] [first value per output window u32, nwin+1].
// E1's block 0 zeroes the error word and the totals.  The group sums are in the context's
// zero-between-calls buffer (rr_encode_sums_words): E4's block 0 zeroes them (E3 read them).
#ifndef RR_ENC_W
#define RR_ENC_W 16384
#endif
#ifndef RR_ENC_RCAP   // payload runs queued per window (LDS: 12 bytes each)
#define RR_ENC_RCAP 416   // (6 emit workgroups per CU: 26.6 KB of LDS each)
#endif
constexpr uint32_t ENC_W = RR_ENC_W, ENC_NT = 256, ENC_RCAP = RR_ENC_RCAP;
static uint64_t enc_windows(uint64_t data_cap) { return data_cap / ENC_W + 1; }

extern "C" uint64_t rr_encode_scratch_words(uint64_t n, uint64_t data_cap) {
    const uint64_t t = (n + 255) / 256, nw = enc_windows(data_cap);
    return RR_SCRATCH_HDR + 1 + 6 * t + t + (nw + 2) / 2 + 2;
}

extern "C" uint64_t rr_encode_sums_words(uint64_t n) { return (n + 255) / 256 / WGROUP + 1; }

extern "C" hipError_t rr_launch_encode(const rr_value *values, const rr_elem *elems, uint64_t elem_cap,
                                       const uint8_t *arena, uint64_t arena_cap, uint64_t n, uint8_t *out,
                                       uint64_t cap, uint64_t *offsets, uint64_t *scratch, uint64_t *sums,
                                       rr_totals *totals, hipStream_t stream, int first_only) {
    if (n == 0) {
        hipError_t e = hipMemsetAsync(offsets, 0, sizeof(uint64_t), stream);
        if (e == hipSuccess && totals) e = hipMemsetAsync(totals, 0, sizeof(rr_totals), stream);
        return e;
    }
    const uint32_t t = (uint32_t)((n + 255) / 256);
    const uint64_t nw = enc_windows(cap);
    uint64_t *err = scratch + RR_SCRATCH_HDR;   // device error word (no look-back left to set it)
    uint64_t *stats = err + 1;
    uint64_t *btot = stats + 6 * (uint64_t)t, *gtot = sums;
    uint32_t *fv = reinterpret_cast<uint32_t *>(btot + t);
    hipLaunchKernelGGL((enc_size_kernel<256, ENC_SIZE_U>), dim3(t), dim3(256), 0, stream, values, elems, n, elem_cap,
                       arena_cap, offsets, stats, btot, gtot, err, 1u, totals);
    if (first_only) return hipGetLastError();
    hipLaunchKernelGGL(enc_index_kernel<ENC_W>, dim3(t), dim3(256), 0, stream, values, elems, n, elem_cap, arena_cap,
                       offsets, btot, gtot, cap, fv, nw, stats + 3 * (uint64_t)t);
    hipLaunchKernelGGL((enc_emit_kernel<ENC_W, ENC_NT, ENC_RCAP>), dim3((uint32_t)nw), dim3(ENC_NT), 0, stream,
                       values, elems, arena, n, out, cap, offsets, fv, stats, 2 * t, totals, err, gtot, t / WGROUP + 1);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------- shards
// Multi-GPU sharding (rr_shard.c): values are independent, so a batch splits
// into contiguous value ranges balanced by bytes, shard k starting at the first value whose
// first byte is at or after k * total / g.  Three small kernels serve rr_shard.c:

// plan[4k..4k+3] = {v0, v1, b0, b1} of shard k (thread k: two lower-bound searches)
__global__ __launch_bounds__(64) void shard_plan_kernel(const uint64_t *__restrict__ offsets, uint64_t n, uint32_t g,
                                                        uint64_t *__restrict__ plan) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= g) return;
    const uint64_t total = offsets[n];
    uint64_t cut[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const uint32_t kk = k + e;
        if (kk == 0) { cut[e] = 0; continue; }
        if (kk == g) { cut[e] = n; continue; }
        const uint64_t target = (uint64_t)(((unsigned __int128)total * kk) / g);
        uint64_t lo = 0, hi = n;   // first v in [0, n) with offsets[v] >= target, else n
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (offsets[mid] < target) lo = mid + 1;
            else hi = mid;
        }
        cut[e] = lo;
    }
    plan[4 * (uint64_t)k + 0] = cut[0];
    plan[4 * (uint64_t)k + 1] = cut[1];
    plan[4 * (uint64_t)k + 2] = offsets[cut[0]];
    plan[4 * (uint64_t)k + 3] = offsets[cut[1]];
}

// words[0, n) = 0 (the graph-captured decode's sums, re-zeroed at every replay: a captured
// hipMemsetAsync measured as not re-running on replay on this stack, tools/graph_diag.py)
__global__ __launch_bounds__(256) void zero_words_kernel(uint64_t *__restrict__ words, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        words[i] = 0;
}
extern "C" hipError_t rr_launch_zero_words(uint64_t *words, uint64_t n, hipStream_t stream) {
    if (!n) return hipSuccess;
    const uint64_t b = (n + 255) / 256;
    hipLaunchKernelGGL(zero_words_kernel, dim3((uint32_t)(b < 256 ? b : 256)), dim3(256), 0, stream, words, n);
    return hipGetLastError();
}

// offsets[i] -= sub (a received shard's offsets, relative to its first byte)
__global__ __launch_bounds__(256) void offsets_rebase_kernel(uint64_t *__restrict__ offs, uint64_t count, uint64_t sub) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) offs[i] -= sub;
}

// A decoded shard placed in the whole batch: elem_base += elem_add; the arena offsets of STR /
// ZLRAW descriptors += byte_add (the arena mirrors the blob buffer, so a shard's arena is the
// whole arena's slice at the shard's first byte).  The zero-filled slots of a malformed value
// (kind STR, data 0, len 0 — no real string starts at byte 0 of a value) stay zero.
__global__ __launch_bounds__(256) void flat_rebase_kernel(rr_value *__restrict__ values, uint64_t n,
                                                          rr_elem *__restrict__ elems, uint64_t ne,
                                                          uint64_t elem_add, uint64_t byte_add) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n || i < ne; i += stride) {
        if (i < n) {
            uint4 v = reinterpret_cast<uint4 *>(values)[i];
            v.w += (uint32_t)elem_add;
            reinterpret_cast<uint4 *>(values)[i] = v;
        }
        if (i < ne) {
            uint4 e = reinterpret_cast<uint4 *>(elems)[i];
            const uint32_t kind = e.w & 0xFF;
            const uint64_t d = (uint64_t)e.x | ((uint64_t)e.y << 32);
            if ((kind == RR_K_STR || kind == RR_K_ZLRAW) && (d | e.z) != 0) {
                const uint64_t d2 = d + byte_add;
                e.x = (uint32_t)d2;
                e.y = (uint32_t)(d2 >> 32);
                reinterpret_cast<uint4 *>(elems)[i] = e;
            }
        }
    }
}

extern "C" hipError_t rr_launch_shard_plan(const uint64_t *offsets, uint64_t n, uint32_t g, uint64_t *plan,
                                           hipStream_t stream) {
    hipLaunchKernelGGL(shard_plan_kernel, dim3((g + 63) / 64), dim3(64), 0, stream, offsets, n, g, plan);
    return hipGetLastError();
}
extern "C" hipError_t rr_launch_offsets_rebase(uint64_t *offs, uint64_t count, uint64_t sub, hipStream_t stream) {
    if (count == 0 || sub == 0) return hipSuccess;
    hipLaunchKernelGGL(offsets_rebase_kernel, dim3((uint32_t)((count + 255) / 256)), dim3(256), 0, stream, offs, count,
                       sub);
    return hipGetLastError();
}
extern "C" hipError_t rr_launch_flat_rebase(rr_value *values, uint64_t n, rr_elem *elems, uint64_t ne, uint64_t elem_add,
                                            uint64_t byte_add, hipStream_t stream) {
    const uint64_t m = n > ne ? n : ne;
    if (m == 0 || (elem_add == 0 && byte_add == 0)) return hipSuccess;
    uint64_t blocks = (m + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(flat_rebase_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, values, n, elems, ne, elem_add,
                       byte_add);
    return hipGetLastError();
}

// ---- streaming device copy: the roofline anchor (SURVEY.md §8d "a measured device copy-kernel
// bandwidth on the box") -----------------------------------------------------------------------
// The same bytes-per-lane shape the decode's window copy uses: 16-byte buffer loads, COPY_U of
// them in flight per lane before any store, nontemporal 16-byte stores; a workgroup per
// COPY_U * 256 * 16 bytes (≫ 256 CUs' worth of workgroups), blocks dealt over the XCDs in
// order.  Bytes past the end read as zeros and their stores are dropped (buffer range), so
// there is no tail branch.  Used by bench.py as `copy_ref`; no part of the serdes path.
//
// Shapes (rr_copy_shape, tools/time_copy.py): U 16-byte loads in flight per lane, NT threads, a
// workgroup per U * NT * 16 bytes (one pass) or a resident grid striding over the buffer, and
// nontemporal (aux 2) or default-policy stores.
template <uint32_t U, uint32_t NT, bool NTS, bool NTL = false>
__global__ __launch_bounds__(NT) void copy_kernel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                  uint64_t bytes) {
    constexpr uint64_t TILE = (uint64_t)U * NT * 16;
    for (uint64_t base = (uint64_t)blockIdx.x * TILE; base < bytes; base += (uint64_t)gridDim.x * TILE) {
        const uint64_t left = bytes - base;
        const uint32_t span = left < TILE ? (uint32_t)left : (uint32_t)TILE;
        const rsrc_t RS = make_rsrc(src + base, span), RD = make_rsrc(dst + base, span);
        u32x4 x[U];
#pragma unroll
        for (uint32_t k = 0; k < U; ++k)
            x[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(RS, (int)((threadIdx.x + k * NT) * 16), 0,
                                                                                 NTL ? 2 : 0));
#pragma unroll
        for (uint32_t k = 0; k < U; ++k)
            __builtin_amdgcn_raw_buffer_store_b128(x[k], RD, (int)((threadIdx.x + k * NT) * 16), 0, NTS ? 2 : 0);
    }
}

template <uint32_t U, uint32_t NT, bool NTS, bool NTL = false>
static hipError_t launch_copy_shape(uint8_t *dst, const uint8_t *src, uint64_t bytes, uint32_t grid, hipStream_t stream) {
    const uint64_t tiles = (bytes + (uint64_t)U * NT * 16 - 1) / ((uint64_t)U * NT * 16);
    if (grid == 0 || grid > tiles) grid = (uint32_t)tiles;
    hipLaunchKernelGGL((copy_kernel<U, NT, NTS, NTL>), dim3(grid), dim3(NT), 0, stream, src, dst, bytes);
    return hipGetLastError();
}

// shape: 0 = the default below; 1-8 = the alternatives timed by tools/time_copy.py (diagnostics).
// Measured (497 MB, read + write bytes): 4 granules per thread with nontemporal loads and stores
// 6.36 TB/s, 1 per thread 6.30, nontemporal stores only 5.85-5.89 (2 or 4 per thread), 8 per
// thread (round 3's) 5.56, a resident-size grid 5.72.
extern "C" hipError_t rr_launch_copy_shape(uint8_t *dst, const uint8_t *src, uint64_t bytes, int shape,
                                           hipStream_t stream) {
    if (bytes == 0) return hipSuccess;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    switch (shape) {
        case 1: return launch_copy_shape<8, 256, true>(dst, src, bytes, 0, stream);   // (round 3's)
        case 2: return launch_copy_shape<4, 256, true>(dst, src, bytes, 0, stream);
        case 3: return launch_copy_shape<2, 256, true>(dst, src, bytes, 0, stream);
        case 4: return launch_copy_shape<1, 256, true>(dst, src, bytes, 0, stream);
        case 5: return launch_copy_shape<4, 256, true, true>(dst, src, bytes, 0, stream);
        case 6: return launch_copy_shape<2, 512, true>(dst, src, bytes, 0, stream);
        case 7: return launch_copy_shape<4, 1024, true>(dst, src, bytes, 0, stream);
        case 8: return launch_copy_shape<4, 256, true>(dst, src, bytes, (uint32_t)cus * 16, stream);
        default: return launch_copy_shape<4, 256, true, true>(dst, src, bytes, 0, stream);   // (= 5: 6.36 TB/s)
    }
}

extern "C" hipError_t rr_launch_copy(uint8_t *dst, const uint8_t *src, uint64_t bytes, hipStream_t stream) {
    return rr_launch_copy_shape(dst, src, bytes, 0, stream);
}

// ---- the look-back scan for other launchers (rr_snappy.hip) --------------------------------
// x[0..n) -> exclusive prefix in place, x[n] = total; lb (rr_scan_words(n) words) must be zero
// and x[n] must be 0 beforehand (the caller's first kernel does both, as count_kernel does).
extern "C" uint64_t rr_scan_words(uint64_t n) {
    const uint64_t st = scan_tiles(n);
    return 1 + st + (st + LB_GROUP - 1) / LB_GROUP;
}
extern "C" hipError_t rr_launch_scan_u64(uint64_t *x, uint64_t n, uint64_t *lb, uint64_t *err, hipStream_t stream) {
    const uint32_t st = (uint32_t)scan_tiles(n);
    if (st) hipLaunchKernelGGL(scan_kernel, dim3(st), dim3(256), 0, stream, x, n, lb, st, err);
    return hipGetLastError();
}
