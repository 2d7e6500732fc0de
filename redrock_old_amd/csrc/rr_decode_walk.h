// rr_decode_walk.h — fused walk + emit of one chunk of <= 64 values straight from global memory.
//
// Why not LDS: staging a window big enough to give every lane of a wave a value (~32 KB of
// mixed values) caps a CU at ~4 waves, and the walk/emit loops are then latency-exposed
// (measured: 80% of wave cycles in s_waitcnt, 2 ms per 1M values).  Here each wave copies its
// window to the arena with plain streaming loads and then walks its values from the same bytes
// (L2/MALL-hot: they were just loaded), so occupancy is set by registers alone.
//
// lane = value.  A header read (32 bytes at the value) classifies it and emits what needs no
// walk (String descriptor, ziplist ZLRAW).  Then ONE unified step loop for all types: each step
// reads 32 bytes at the lane's cursor (3 dwordx4 loads, one memory latency) — enough for any
// element header of any type plus a List entry's 20 digits or a ziplist int64 — decodes the
// element, writes its descriptor to elem_base + k (elem_base comes from the reservation scan,
// so no second pass) and advances.  The checks are exactly the exact parser's (rock_serdes.c /
// ziplist.c asserts); a value the walk rejects, or whose element count differs from its
// reservation, sends the whole chunk to the exact parser, which rewrites every slot of it.
#pragma once
#include "rr_decode_fast.h"

namespace rr {

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));

// bytes [p, p+32) of the blob buffer (readable for cap bytes) into 8 dwords.
__device__ __forceinline__ void g_read8(const uint8_t *__restrict__ blob, uint64_t cap, uint64_t p, uint32_t (&o)[8]) {
    const uint64_t a = p & ~3ull;
    const uint32_t sh = (uint32_t)(p & 3);
    if (a + 48 <= cap) {
        const u32x4u *q = reinterpret_cast<const u32x4u *>(blob + a);
        const u32x4u w0 = q[0], w1 = q[1], w2 = q[2];
        const uint32_t w[9] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x};
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
    } else {   // the last bytes of the buffer: byte loads, zeros past its end
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t q = p + 4 * i + j;
                x |= (q < cap ? (uint32_t)blob[q] : 0u) << (8 * j);
            }
            o[i] = x;
        }
    }
}

struct ChunkOut {
    uint32_t n, enc, type, lru;
    bool fail;
    uint64_t pay;
};

__device__ __forceinline__ void put_desc(rr_elem *e, uint64_t data, uint32_t len, uint32_t kind, uint32_t zenc) {
    uint4 w;
    w.x = (uint32_t)data;
    w.y = (uint32_t)(data >> 32);
    w.z = len;
    w.w = kind | (zenc << 8);
    *reinterpret_cast<uint4 *>(e) = w;
}

// write: the value's reserved slots [eb, eb + r) fit the descriptor array.
__device__ __forceinline__ ChunkOut walk_value(const uint8_t *__restrict__ blob, uint64_t cap_bytes, bool active,
                                               uint64_t o_lo, uint64_t o_hi, rr_elem *__restrict__ elems,
                                               uint64_t eb, uint64_t r, bool write) {
    ChunkOut o{0, 0, 0xFF, 0, false, 0};
    const uint64_t len = o_hi - o_lo;
    uint64_t p = 0, end = o_hi, zl0 = 0, zlL = 0, last = 0, cnt = 0;
    uint32_t prev_raw = 0, nint = 0, type = 0xFF;
    bool walking = false;
    if (active) {
        uint32_t h[8];
        g_read8(blob, cap_bytes, o_lo, h);
        type = h[0] & 0xFF;
        o.lru = __builtin_amdgcn_alignbyte(h[1], h[0], 1) & RR_LRU_MASK;
        const uint32_t f5 = __builtin_amdgcn_alignbyte(h[2], h[1], 1);   // bytes 5..8
        const uint32_t f9 = __builtin_amdgcn_alignbyte(h[3], h[2], 1);   // bytes 9..12
        const uint64_t u5 = (uint64_t)f5 | ((uint64_t)f9 << 32);         // u64 at 5
        if (len < 5) { o.fail = true; type = 0xFF; }
        else switch (type) {
            case RR_TYPE_STRING: {
                if (len < 6) { o.fail = true; break; }
                const uint32_t enc = f5 & 0xFF;
                o.enc = enc;
                if (enc == RR_ENC_INT) {
                    if (len != 14) { o.fail = true; break; }
                    const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(h[2], h[1], 2) |
                                       ((uint64_t)__builtin_amdgcn_alignbyte(h[3], h[2], 2) << 32);
                    if (write && r >= 1) put_desc(elems + eb, v, 0, RR_K_INT, 0);
                } else if (enc == RR_ENC_RAW || (enc == RR_ENC_EMBSTR && len - 6 <= RR_EMBSTR_SIZE_LIMIT)) {
                    if (write && r >= 1) put_desc(elems + eb, o_lo + 6, (uint32_t)(len - 6), RR_K_STR, 0);
                    o.pay = len - 6;
                } else { o.fail = true; break; }
                o.n = 1;
                break;
            }
            case RR_TYPE_SET_INTSET:
                if (len < 13 || (f5 != 2 && f5 != 4 && f5 != 8) || len - 13 != (uint64_t)f5 * f9) { o.fail = true; break; }
                o.enc = f5;
                nint = f9;
                p = o_lo + 13;
                walking = true;
                break;
            case RR_TYPE_LIST_QUICKLIST:
                p = o_lo + 5;
                walking = true;
                break;
            case RR_TYPE_SET_HT:
            case RR_TYPE_HASH_HT:
            case RR_TYPE_ZSET_SKIPLIST:
                if (len < 13) { o.fail = true; break; }
                cnt = u5;
                p = o_lo + 13;
                walking = true;
                break;
            case RR_TYPE_HASH_ZIPLIST:
            case RR_TYPE_ZSET_ZIPLIST: {
                if (len < 13 || len - 13 != u5 || u5 < 11) { o.fail = true; break; }
                zl0 = o_lo + 13;
                zlL = u5;
                const uint32_t zlbytes = __builtin_amdgcn_alignbyte(h[4], h[3], 1);   // bytes 13..16
                if (zlbytes != zlL) { o.fail = true; break; }
                if (write && r >= 1) put_desc(elems + eb, zl0, (uint32_t)zlL, RR_K_ZLRAW, 0);
                o.pay = zlL;
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
    while (__ballot(walking)) {
        if (walking) {
            const uint32_t k = o.n;
            uint32_t b[8];
            g_read8(blob, cap_bytes, p, b);
            const uint64_t u0 = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
            bool emit = false;
            uint64_t data = 0;
            uint32_t elen = 0, kind = RR_K_STR, zenc = 0;
            switch (type) {
                case RR_TYPE_SET_INTSET:
                    if (k >= nint) { walking = false; break; }
                    data = o.enc == 2 ? (uint64_t)(int64_t)(int16_t)(b[0] & 0xFFFF)
                         : o.enc == 4 ? (uint64_t)(int64_t)(int32_t)b[0] : u0;
                    kind = RR_K_INT;
                    emit = true;
                    p += o.enc;
                    break;
                case RR_TYPE_LIST_QUICKLIST: {
                    if (p == end) { walking = false; break; }
                    if (end - p < 4 || b[0] > end - p - 4) { o.fail = true; break; }
                    const uint32_t d[5] = {b[1], b[2], b[3], b[4], b[5]};
                    int64_t iv;
                    if (regs_try_int(d, b[0], iv)) { data = (uint64_t)iv; kind = RR_K_INT; }
                    else { data = p + 4; elen = b[0]; o.pay += elen; }
                    emit = true;
                    p += 4 + b[0];
                    break;
                }
                case RR_TYPE_SET_HT:
                case RR_TYPE_HASH_HT:
                    if (p == end) { walking = false; break; }
                    if (end - p < 8 || u0 > end - p - 8) { o.fail = true; break; }
                    data = p + 8;
                    elen = b[0];
                    o.pay += elen;
                    emit = true;
                    p += 8 + b[0];
                    break;
                case RR_TYPE_ZSET_SKIPLIST:
                    if ((k & 1) == 0) {
                        if (p == end) { walking = false; break; }
                        if ((uint64_t)(k >> 1) == cnt) { o.fail = true; break; }   // bytes after the last node
                        if (end - p < 8 || u0 > end - p - 8) { o.fail = true; break; }
                        data = p + 8;
                        elen = b[0];
                        o.pay += elen;
                        p += 8 + b[0];
                    } else {
                        if (end - p < 8) { o.fail = true; break; }
                        data = u0;
                        kind = RR_K_SCORE;
                        p += 8;
                    }
                    emit = true;
                    break;
                default: {   // ziplist entry, ziplist.c:300-447
                    const uint64_t zend = zl0 + zlL;
                    if (p >= zend) { o.fail = true; break; }
                    const uint32_t b0 = b[0] & 0xFF;
                    if (b0 == 0xFF) { walking = false; break; }
                    const bool big = b0 >= 254;
                    if (big && p + 5 > zend - 1) { o.fail = true; break; }
                    const uint32_t pl = big ? __builtin_amdgcn_alignbyte(b[1], b[0], 1) : b0;
                    if (pl != prev_raw) { o.fail = true; break; }
                    const uint32_t qo = big ? 5u : 1u;
                    const uint64_t q = p + qo;
                    if (q >= zend - 1) { o.fail = true; break; }
                    const uint32_t e = byte_at(b, qo);
                    uint64_t en;
                    if (e < 0xC0) {
                        const uint32_t cls = e & 0xC0;
                        uint32_t ls, sl;
                        if (cls == 0x00) { ls = 1; sl = e & 0x3F; }
                        else if (cls == 0x40) {
                            if (q + 2 > zend - 1) { o.fail = true; break; }
                            ls = 2;
                            sl = ((e & 0x3F) << 8) | byte_at(b, qo + 1);
                        } else {
                            if (q + 5 > zend - 1) { o.fail = true; break; }
                            ls = 5;
                            sl = __builtin_bswap32(dword_at(b, qo + 1));
                        }
                        en = q + ls + sl;
                        if (en > zend - 1) { o.fail = true; break; }
                        data = q + ls;
                        elen = sl;
                        zenc = cls;
                    } else {
                        uint32_t isz;
                        if (e == 0xFE) isz = 1;
                        else if (e == 0xC0) isz = 2;
                        else if (e == 0xF0) isz = 3;
                        else if (e == 0xD0) isz = 4;
                        else if (e == 0xE0) isz = 8;
                        else if (e >= 0xF1 && e <= 0xFD) isz = 0;
                        else { o.fail = true; break; }
                        en = q + 1 + isz;
                        if (en > zend - 1) { o.fail = true; break; }
                        const uint32_t lo = dword_at(b, qo + 1), hi = dword_at(b, qo + 5);
                        int64_t v;
                        if (isz == 0) v = (int64_t)(e & 0x0F) - 1;
                        else if (isz == 1) v = (int8_t)(lo & 0xFF);
                        else if (isz == 2) v = (int16_t)(lo & 0xFFFF);
                        else if (isz == 3) v = ((int32_t)(lo << 8)) >> 8;
                        else if (isz == 4) v = (int32_t)lo;
                        else v = (int64_t)((uint64_t)lo | ((uint64_t)hi << 32));
                        data = (uint64_t)v;
                        kind = RR_K_INT;
                        zenc = e;
                    }
                    emit = true;
                    prev_raw = (uint32_t)(en - p);
                    last = p;
                    p = en;
                    break;
                }
            }
            if (o.fail) walking = false;
            if (emit) {
                if (write && k < r) put_desc(elems + eb + k, data, elen, kind, zenc);
                ++o.n;
                if (o.n > r) { o.fail = true; walking = false; }   // more elements than reserved
            }
        }
    }
    if (active && !o.fail) {
        switch (type) {
            case RR_TYPE_SET_HT: o.fail = (uint64_t)o.n != cnt; break;
            case RR_TYPE_HASH_HT:
            case RR_TYPE_ZSET_SKIPLIST: o.fail = (o.n & 1) || (uint64_t)(o.n >> 1) != cnt; break;
            case RR_TYPE_HASH_ZIPLIST:
            case RR_TYPE_ZSET_ZIPLIST: {
                uint32_t z[8];
                g_read8(blob, cap_bytes, zl0, z);   // zlbytes, zltail, zllen
                const uint32_t entries = o.n - 1;
                const uint32_t zllen = z[2] & 0xFFFF;
                o.fail = p != zl0 + zlL - 1 || (zllen != 0xFFFF && zllen != entries) ||
                         (uint64_t)z[1] != last - zl0 || (entries & 1);
                break;
            }
            default:
                break;
        }
    }
    o.type = type;
    return o;
}

}  // namespace rr
