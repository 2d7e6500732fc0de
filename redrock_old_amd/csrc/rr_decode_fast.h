// rr_decode_fast.h — the fast decode path for one LDS-staged window.
//
// The exact parser (parse_value in rr_kernels.hip) maps one lane to one value and walks it
// twice (count, emit).  Lanes of a wave hold values of different types, so a wave executes
// the union of every type's loop, and the List emission runs string2ll byte by byte: on the
// mixed batch that cost ~5 ms per 1M values.  The fast path restructures the work:
//   walk   lane = value; ONE unified step loop for all types (loop count = max elements over
//          the lanes, not the sum over types), one LDS latency per element, records every
//          element's position into an LDS list {pos:16 | owner lane:6 | index:10};
//   emit   lane = element record: decode the descriptor from the staged bytes (string2ll of
//          list entries from registers, ziplist entry headers, scores, intset members) and
//          store it at elem_base(owner) + index.
// The walk validates with exactly the checks of rock_serdes.c/ziplist.c that the exact parser
// applies; any value it cannot accept (malformed, >1023 elements, too many records) sends the
// whole window to the exact parser, which assigns the reference's per-value status codes.
#pragma once
#include "rr_device.h"

namespace rr {

typedef const __attribute__((address_space(3))) uint32_t *lds_u32p;

// 4 / 8 bytes at any byte offset of the stage: aligned dword reads + alignbyte (the reads of
// one field are independent, one LDS latency).
__device__ __forceinline__ uint32_t s8(lds_cptr S, uint32_t p) { return S[p]; }
__device__ __forceinline__ uint32_t s32(lds_cptr S, uint32_t p) {
    lds_u32p W = (lds_u32p)S;
    const uint32_t a = p >> 2, sh = p & 3;
    const uint32_t w0 = W[a], w1 = W[a + 1];
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
}
__device__ __forceinline__ uint64_t s64(lds_cptr S, uint32_t p) {
    lds_u32p W = (lds_u32p)S;
    const uint32_t a = p >> 2, sh = p & 3;
    const uint32_t w0 = W[a], w1 = W[a + 1], w2 = W[a + 2];
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}

// zipTryEncoding (ziplist.c:480) + string2ll (util.c:360): an entry of 1..31 bytes is an
// integer iff it is "0" or [-]?[1-9][0-9]* within int64.  A 20-digit magnitude is always
// >= 1e19 > 2^63, so anything longer than 20 bytes fails; up to 19 digits cannot overflow
// uint64 while accumulating.  Bytes come from registers (6 dword reads), no per-byte LDS trip.
__device__ __forceinline__ bool lds_try_int(lds_cptr S, uint32_t d, uint32_t len, int64_t &out) {
    if (len == 0 || len > 20) return false;
    lds_u32p W = (lds_u32p)S;
    const uint32_t a = d >> 2, sh = d & 3;
    uint32_t w[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) w[i] = W[a + i];
    uint32_t b[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) b[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
    const uint32_t c0 = b[0] & 0xFF;
    if (len == 1 && c0 == '0') { out = 0; return true; }
    const uint32_t neg = c0 == '-' ? 1u : 0u;
    const uint32_t nd = len - neg;
    if (nd == 0 || nd > 19) return false;
    bool ok = true;
    uint64_t v = 0;
#pragma unroll
    for (uint32_t j = 0; j < 20; ++j) {
        const uint32_t c = (b[j >> 2] >> (8 * (j & 3))) & 0xFF;
        if (j >= neg && j < len) {
            const bool lead = j == neg;
            ok &= lead ? (c >= '1' && c <= '9') : (c >= '0' && c <= '9');
            v = v * 10 + (c - '0');
        }
    }
    if (!ok) return false;
    if (neg) {
        if (v > (1ull << 63)) return false;
        out = (int64_t)(0ull - v);
    } else {
        if (v > 0x7FFFFFFFFFFFFFFFull) return false;
        out = (int64_t)v;
    }
    return true;
}

struct WalkOut {
    uint32_t n;      // descriptors of this lane's value
    uint32_t enc;    // record enc byte
    bool fail;       // fast path cannot take this value
};

constexpr uint32_t REC_KMAX = 1024;

// Unified walker.  vb/len: the lane's value in the stage; recs/ecap: the record list; nrec:
// wave-uniform running record count (updated).  Inactive lanes pass active = false.
__device__ __forceinline__ WalkOut fast_walk(lds_cptr S, bool active, uint32_t vb, uint32_t len, uint32_t *recs_ptr,
                                             uint32_t ecap, uint32_t &nrec) {
    __attribute__((address_space(3))) uint32_t *recs = (__attribute__((address_space(3))) uint32_t *)recs_ptr;
    const uint32_t lane = lane_id();
    WalkOut o{0, 0, false};
    uint32_t type = 0xFF;
    bool walking = false;
    uint32_t p = 0, end = vb + len, zl0 = 0, zlL = 0, prev_raw = 0, last = 0, nint = 0;
    uint64_t cnt = 0;
    // records emitted before the loop (String element, ziplist ZLRAW)
    bool pre = false;
    uint32_t prepos = 0;
    if (active) {
        if (len < 5) o.fail = true;
        else {
            type = s8(S, vb);
            switch (type) {
                case RR_TYPE_STRING: {
                    if (len < 6) { o.fail = true; break; }
                    const uint32_t enc = s8(S, vb + 5);
                    o.enc = enc;
                    if (enc == RR_ENC_INT) o.fail = len != 14;
                    else if (enc == RR_ENC_RAW) o.fail = false;
                    else if (enc == RR_ENC_EMBSTR) o.fail = len - 6 > RR_EMBSTR_SIZE_LIMIT;
                    else o.fail = true;
                    if (!o.fail) { pre = true; prepos = vb; o.n = 1; }
                    break;
                }
                case RR_TYPE_SET_INTSET: {
                    if (len < 13) { o.fail = true; break; }
                    const uint32_t w = s32(S, vb + 5), c = s32(S, vb + 9);
                    if ((w != 2 && w != 4 && w != 8) || (uint64_t)(len - 13) != (uint64_t)w * c) { o.fail = true; break; }
                    o.enc = w;
                    nint = c;
                    p = vb + 13;
                    walking = true;
                    break;
                }
                case RR_TYPE_LIST_QUICKLIST:
                    p = vb + 5;
                    walking = true;
                    break;
                case RR_TYPE_SET_HT:
                case RR_TYPE_HASH_HT:
                case RR_TYPE_ZSET_SKIPLIST:
                    if (len < 13) { o.fail = true; break; }
                    cnt = s64(S, vb + 5);
                    p = vb + 13;
                    walking = true;
                    break;
                case RR_TYPE_HASH_ZIPLIST:
                case RR_TYPE_ZSET_ZIPLIST: {
                    if (len < 13) { o.fail = true; break; }
                    const uint64_t L = s64(S, vb + 5);
                    if ((uint64_t)(len - 13) != L || L < 11) { o.fail = true; break; }
                    zl0 = vb + 13;
                    zlL = len - 13;
                    if (s32(S, zl0) != zlL) { o.fail = true; break; }
                    pre = true;
                    prepos = zl0;
                    o.n = 1;
                    p = zl0 + 10;
                    last = zl0 + 10;
                    walking = true;
                    break;
                }
                default:
                    o.fail = true;
            }
        }
    }
    {   // pre-loop records
        const uint64_t m = __ballot(pre);
        const uint32_t idx = nrec + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (pre && idx < ecap) recs[idx] = prepos | (lane << 16);
        nrec += (uint32_t)__builtin_popcountll(m);
    }
    while (__ballot(walking)) {
        bool emit = false;
        uint32_t rpos = p;
        uint32_t k = o.n;
        if (walking) {
            switch (type) {
                case RR_TYPE_SET_INTSET:
                    if (k < nint) { rpos = p + k * o.enc; emit = true; ++o.n; }
                    else walking = false;
                    break;
                case RR_TYPE_LIST_QUICKLIST:
                    if (p == end) { walking = false; break; }
                    if (end - p < 4) { o.fail = true; break; }
                    {
                        const uint32_t L = s32(S, p);
                        if (L > end - p - 4) { o.fail = true; break; }
                        emit = true;
                        ++o.n;
                        p += 4 + L;
                    }
                    break;
                case RR_TYPE_SET_HT:
                case RR_TYPE_HASH_HT:
                    if (p == end) { walking = false; break; }
                    if (end - p < 8) { o.fail = true; break; }
                    {
                        const uint64_t L = s64(S, p);
                        if (L > (uint64_t)(end - p - 8)) { o.fail = true; break; }
                        emit = true;
                        ++o.n;
                        p += 8 + (uint32_t)L;
                    }
                    break;
                case RR_TYPE_ZSET_SKIPLIST:
                    if ((k & 1) == 0) {
                        if (p == end) { walking = false; break; }
                        if ((uint64_t)(k >> 1) == cnt) { o.fail = true; break; }   // bytes after the last node
                        if (end - p < 8) { o.fail = true; break; }
                        const uint64_t L = s64(S, p);
                        if (L > (uint64_t)(end - p - 8)) { o.fail = true; break; }
                        emit = true;
                        ++o.n;
                        p += 8 + (uint32_t)L;
                    } else {
                        if (end - p < 8) { o.fail = true; break; }
                        emit = true;
                        ++o.n;
                        p += 8;
                    }
                    break;
                default: {   // ziplist entry, ziplist.c:300-447
                    const uint32_t zend = zl0 + zlL;
                    if (p >= zend) { o.fail = true; break; }
                    const uint32_t b0 = s8(S, p);
                    if (b0 == 0xFF) { walking = false; break; }
                    uint32_t pl, pls;
                    if (b0 < 254) { pl = b0; pls = 1; }
                    else {
                        if (p + 5 > zend - 1) { o.fail = true; break; }
                        pl = s32(S, p + 1);
                        pls = 5;
                    }
                    if (pl != prev_raw) { o.fail = true; break; }
                    const uint32_t q = p + pls;
                    if (q >= zend - 1) { o.fail = true; break; }
                    const uint32_t enc = s8(S, q);
                    uint32_t e;
                    if (enc < 0xC0) {
                        const uint32_t cls = enc & 0xC0;
                        uint32_t ls, sl;
                        if (cls == 0x00) { ls = 1; sl = enc & 0x3F; }
                        else if (cls == 0x40) {
                            if (q + 2 > zend - 1) { o.fail = true; break; }
                            ls = 2;
                            sl = ((enc & 0x3F) << 8) | s8(S, q + 1);
                        } else {
                            if (q + 5 > zend - 1) { o.fail = true; break; }
                            ls = 5;
                            sl = __builtin_bswap32(s32(S, q + 1));
                        }
                        const uint64_t e64 = (uint64_t)q + ls + sl;
                        if (e64 > zend - 1) { o.fail = true; break; }
                        e = (uint32_t)e64;
                    } else {
                        uint32_t isz;
                        if (enc == 0xFE) isz = 1;
                        else if (enc == 0xC0) isz = 2;
                        else if (enc == 0xF0) isz = 3;
                        else if (enc == 0xD0) isz = 4;
                        else if (enc == 0xE0) isz = 8;
                        else if (enc >= 0xF1 && enc <= 0xFD) isz = 0;
                        else { o.fail = true; break; }
                        e = q + 1 + isz;
                        if (e > zend - 1) { o.fail = true; break; }
                    }
                    emit = true;
                    ++o.n;
                    prev_raw = e - p;
                    last = p;
                    p = e;
                    break;
                }
            }
            if (o.fail) walking = false;
            if (emit && k >= REC_KMAX) { o.fail = true; walking = false; emit = false; }
        }
        const uint64_t m = __ballot(emit);
        const uint32_t idx = nrec + (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (emit && idx < ecap) recs[idx] = rpos | (lane << 16) | (k << 22);
        nrec += (uint32_t)__builtin_popcountll(m);
    }
    // end-of-value checks (rock_serdes.c counts; ziplist header fields)
    if (active && !o.fail) {
        switch (type) {
            case RR_TYPE_SET_HT: o.fail = (uint64_t)o.n != cnt; break;
            case RR_TYPE_HASH_HT: o.fail = (o.n & 1) || (uint64_t)(o.n >> 1) != cnt; break;
            case RR_TYPE_ZSET_SKIPLIST: o.fail = (o.n & 1) || (uint64_t)(o.n >> 1) != cnt; break;
            case RR_TYPE_HASH_ZIPLIST:
            case RR_TYPE_ZSET_ZIPLIST: {
                const uint32_t entries = o.n - 1;
                const uint32_t zllen = s8(S, zl0 + 8) | (s8(S, zl0 + 9) << 8);
                o.fail = p != zl0 + zlL - 1 || (zllen != 0xFFFF && zllen != entries) ||
                         s32(S, zl0 + 4) != last - zl0 || (entries & 1);
                break;
            }
            default:
                break;
        }
    }
    return o;
}

// Descriptor for record (pos, k) of a value of `type` at stage offset vb (batch offset of a
// stage position x is sbase + x).  Adds payload bytes to pay.
__device__ __forceinline__ void fast_emit(lds_cptr S, uint64_t sbase, uint32_t type, uint32_t enc, uint32_t vb,
                                          uint32_t len, uint32_t pos, uint32_t k, uint4 &w, uint64_t &pay) {
    uint64_t data = 0;
    uint32_t elen = 0, kind = RR_K_STR, zenc = 0;
    switch (type) {
        case RR_TYPE_STRING:
            if (enc == RR_ENC_INT) { data = s64(S, vb + 6); kind = RR_K_INT; }
            else { data = sbase + vb + 6; elen = len - 6; pay += elen; }
            break;
        case RR_TYPE_LIST_QUICKLIST: {
            const uint32_t L = s32(S, pos);
            int64_t iv;
            if (lds_try_int(S, pos + 4, L, iv)) { data = (uint64_t)iv; kind = RR_K_INT; }
            else { data = sbase + pos + 4; elen = L; pay += L; }
            break;
        }
        case RR_TYPE_SET_INTSET: {
            if (enc == 2) data = (uint64_t)(int64_t)(int16_t)(s32(S, pos) & 0xFFFF);
            else if (enc == 4) data = (uint64_t)(int64_t)(int32_t)s32(S, pos);
            else data = s64(S, pos);
            kind = RR_K_INT;
            break;
        }
        case RR_TYPE_SET_HT:
        case RR_TYPE_HASH_HT:
            elen = (uint32_t)s64(S, pos);
            data = sbase + pos + 8;
            pay += elen;
            break;
        case RR_TYPE_ZSET_SKIPLIST:
            if (k & 1) { data = s64(S, pos); kind = RR_K_SCORE; }
            else { elen = (uint32_t)s64(S, pos); data = sbase + pos + 8; pay += elen; }
            break;
        default:   // ziplists
            if (k == 0) { data = sbase + pos; elen = len - 13; kind = RR_K_ZLRAW; pay += elen; }
            else {
                const uint32_t b0 = s8(S, pos);
                const uint32_t q = pos + (b0 < 254 ? 1u : 5u);
                const uint32_t e = s8(S, q);
                if (e < 0xC0) {
                    const uint32_t cls = e & 0xC0;
                    uint32_t ls, sl;
                    if (cls == 0x00) { ls = 1; sl = e & 0x3F; }
                    else if (cls == 0x40) { ls = 2; sl = ((e & 0x3F) << 8) | s8(S, q + 1); }
                    else { ls = 5; sl = __builtin_bswap32(s32(S, q + 1)); }
                    data = sbase + q + ls;
                    elen = sl;
                    zenc = cls;
                } else {
                    int64_t v;
                    const uint32_t x = q + 1;
                    if (e >= 0xF1 && e <= 0xFD) v = (int64_t)(e & 0x0F) - 1;
                    else if (e == 0xFE) v = (int8_t)s8(S, x);
                    else if (e == 0xC0) v = (int16_t)(s32(S, x) & 0xFFFF);
                    else if (e == 0xF0) v = ((int32_t)(s32(S, x) << 8)) >> 8;
                    else if (e == 0xD0) v = (int32_t)s32(S, x);
                    else v = (int64_t)s64(S, x);
                    data = (uint64_t)v;
                    kind = RR_K_INT;
                    zenc = e;
                }
            }
            break;
    }
    w.x = (uint32_t)data;
    w.y = (uint32_t)(data >> 32);
    w.z = elen;
    w.w = kind | (zenc << 8);
}

}  // namespace rr
