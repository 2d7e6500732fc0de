// rr_decode_fast.h — the fast decode path for one LDS-staged window chunk (<= 64 values).
//
// The exact parser (parse_value in rr_kernels.hip) maps one lane to one value and walks it
// twice (count, emit); lanes of a wave hold values of different types, so a wave executes the
// union of every type's loop, each with several dependent LDS reads per element.  The fast
// path restructures the work:
//   walk   lane = value; ONE unified step loop for all types (loop count = the most elements
//          of any lane, not the sum over types).  Every step reads the same 12 bytes at the
//          lane's cursor (one LDS round trip: 4 aligned ds_read_b32 + alignbyte) and decodes the
//          element header of whichever type from registers; the element's position is appended
//          to an LDS record list {pos:16 | owner lane:6 | index:10}.
//   emit   lane = record: one 32-byte read at the record (9 ds_read_b32) holds everything a
//          descriptor needs (list length + up to 20 digits for string2ll, ziplist entry header +
//          int64, HT/skiplist length, score, intset member); decoded from registers and stored
//          at elem_base(owner) + index.
// The walk applies exactly the checks of rock_serdes.c / ziplist.c that the exact parser does;
// any value it cannot take (malformed, > 1023 elements, record overflow) sends the chunk to
// the exact parser, which assigns the reference's per-value status codes.
#pragma once
#include "rr_device.h"

namespace rr {

typedef const __attribute__((address_space(3))) uint32_t *lds_u32p;
typedef __attribute__((address_space(3))) uint32_t *lds_u32w;

__device__ __forceinline__ uint32_t s8(lds_cptr S, uint32_t p) { return S[p]; }
__device__ __forceinline__ uint32_t s32(lds_cptr S, uint32_t p) {
    lds_u32p W = (lds_u32p)S;
    const uint32_t a = p >> 2, sh = p & 3;
    return __builtin_amdgcn_alignbyte(W[a + 1], W[a], sh);
}

// bytes [p, p + 4*N) of the stage into N dwords (N+1 aligned reads, one LDS latency)
template <int N>
__device__ __forceinline__ void s_read(lds_cptr S, uint32_t p, uint32_t (&o)[N]) {
    lds_u32p W = (lds_u32p)S;
    const uint32_t a = p >> 2, sh = p & 3;
    uint32_t w[N + 1];
#pragma unroll
    for (int i = 0; i <= N; ++i) w[i] = W[a + i];
#pragma unroll
    for (int i = 0; i < N; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}

// byte j of a dword array (j a compile-time or small runtime index)
template <int N>
__device__ __forceinline__ uint32_t byte_at(const uint32_t (&b)[N], uint32_t j) {
    uint32_t w = b[0];
#pragma unroll
    for (int i = 1; i < N; ++i) w = (j >> 2) == (uint32_t)i ? b[i] : w;
    return (w >> (8 * (j & 3))) & 0xFF;
}
// 4 bytes starting at byte j (j <= 4*(N-1))
template <int N>
__device__ __forceinline__ uint32_t dword_at(const uint32_t (&b)[N], uint32_t j) {
    uint32_t lo = b[0], hi = b[1];
#pragma unroll
    for (int i = 1; i < N - 1; ++i) {
        lo = (j >> 2) == (uint32_t)i ? b[i] : lo;
        hi = (j >> 2) == (uint32_t)i ? b[i + 1] : hi;
    }
    return __builtin_amdgcn_alignbyte(hi, lo, j & 3);
}

// zipTryEncoding (ziplist.c:480) + string2ll (util.c:360) over bytes d[0, len) given as 5
// dwords: an entry of 1..31 bytes is an integer iff it is "0" or [-]?[1-9][0-9]* within int64.
// A 20-digit magnitude is always >= 1e19 > 2^63, so more than 20 bytes fails; up to 19 digits
// cannot overflow uint64 while accumulating.
__device__ __forceinline__ bool regs_try_int(const uint32_t (&b)[5], uint32_t len, int64_t &out) {
    if (len == 0 || len > 20) return false;
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
            ok &= j == neg ? (c - '1' <= 8u) : (c - '0' <= 9u);
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

// Records are written at their DESTINATION slot: value's slot base rb (= its elem_base minus
// the chunk's) + element index.  Emission then walks the slots in order, so consecutive lanes
// store consecutive descriptors (coalesced) and a 64-slot round spans only a few values.
// Slots past the value's reservation r are not written (the value then fails anyway).
__device__ __forceinline__ void rec_put(lds_u32w recs, bool emit, uint32_t rb, uint32_t k, uint32_t r, uint32_t rec) {
    if (emit && k < r) recs[rb + k] = rec;
}

// Walk classes (one per lane, fixed for the walk)
constexpr uint32_t WC_NONE = 0, WC_LIST = 1, WC_HT = 2, WC_SL = 3, WC_ZL = 4, WC_IS = 5;

// Unified walker.  vb/len: the lane's value in the stage; recs: the wave's slot table; rb/r:
// the lane's slot base and reservation.  Inactive lanes pass active = false.
//
// The step is straight-line select arithmetic: every class's element size and validity are
// computed from the same 12 bytes and the lane's class picks its own (v_cndmask), so a wave
// whose lanes hold different types runs ~one step's worth of instructions per step instead of
// the sum of every type's branches (a switch here compiled to ~870 instructions per step).
__device__ __forceinline__ WalkOut fast_walk(lds_cptr S, bool active, uint32_t vb, uint32_t len, lds_u32w recs,
                                             uint32_t rb, uint32_t r) {
    const uint32_t lane = lane_id();
    WalkOut o{0, 0, false};
    uint32_t cls = WC_NONE, p = vb, end = vb + len, zl0 = 0, zend = 0, prev_raw = 0, last = 0, nint = 0, w = 0;
    uint64_t cnt = 0;
    bool pre = false;
    uint32_t prepos = 0;
    if (active) {
        uint32_t h[4];   // header: type, lru, enc / count fields (bytes vb .. vb+15)
        s_read<4>(S, vb, h);
        const uint32_t type = len >= 5 ? (h[0] & 0xFF) : 0xFFu;
        const uint32_t f5 = __builtin_amdgcn_alignbyte(h[2], h[1], 1);   // bytes 5..8
        const uint32_t f9 = __builtin_amdgcn_alignbyte(h[3], h[2], 1);   // bytes 9..12
        const uint64_t u5 = (uint64_t)f5 | ((uint64_t)f9 << 32);
        if (type == RR_TYPE_STRING) {
            const uint32_t enc = f5 & 0xFF;
            o.enc = enc;
            o.fail = len < 6 || !(enc == RR_ENC_RAW || (enc == RR_ENC_INT && len == 14) ||
                                  (enc == RR_ENC_EMBSTR && len - 6 <= RR_EMBSTR_SIZE_LIMIT));
            pre = !o.fail;
            prepos = vb;
            o.n = pre ? 1 : 0;
        } else if (type == RR_TYPE_SET_INTSET) {
            o.fail = len < 13 || (f5 != 2 && f5 != 4 && f5 != 8) || (uint64_t)(len - 13) != (uint64_t)f5 * f9;
            o.enc = f5;
            w = f5;
            nint = f9;
            cls = o.fail ? WC_NONE : WC_IS;
            p = vb + 13;
        } else if (type == RR_TYPE_LIST_QUICKLIST) {
            cls = WC_LIST;
            p = vb + 5;
        } else if (type == RR_TYPE_SET_HT || type == RR_TYPE_HASH_HT || type == RR_TYPE_ZSET_SKIPLIST) {
            o.fail = len < 13;
            cnt = u5;
            cls = o.fail ? WC_NONE : (type == RR_TYPE_ZSET_SKIPLIST ? WC_SL : WC_HT);
            p = vb + 13;
        } else if (type == RR_TYPE_HASH_ZIPLIST || type == RR_TYPE_ZSET_ZIPLIST) {
            zl0 = vb + 13;
            const uint32_t zlbytes = __builtin_amdgcn_alignbyte(h[4 - 1], h[3], 1);   // bytes 13..16 (h[3] bytes 12..15)
            (void)zlbytes;
            o.fail = len < 13 || (uint64_t)(len - 13) != u5 || u5 < 11 || s32(S, zl0) != len - 13;
            zend = vb + len;
            pre = !o.fail;
            prepos = zl0;
            o.n = pre ? 1 : 0;
            cls = o.fail ? WC_NONE : WC_ZL;
            p = zl0 + 10;
            last = zl0 + 10;
        } else {
            o.fail = true;
        }
    }
    rec_put(recs, pre, rb, 0, r, prepos | (lane << 16));
    bool walking = cls != WC_NONE;
    while (__ballot(walking)) {
        uint32_t b[3];   // bytes p .. p+11: every element header of every class fits
        s_read<3>(S, p, b);
        const uint32_t k = o.n;
        const uint32_t L32 = b[0];
        const uint64_t L64 = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
        const uint32_t rem = end - p;
        // ---- LIST: u32 length + bytes
        const bool chain_end = p == end;
        const bool l_bad = rem < 4 || L32 > rem - 4;
        // ---- HT / skiplist member: u64 length + bytes; skiplist score: 8 bytes
        const bool h_bad = rem < 8 || L64 > (uint64_t)(rem - 8);
        const bool sl_score = (k & 1) != 0;
        const bool sl_extra = !sl_score && (uint64_t)(k >> 1) == cnt;   // bytes after the last node
        // ---- ziplist entry (ziplist.c:300-447)
        const uint32_t b0 = L32 & 0xFF;
        const bool z_end = b0 == 0xFF;
        const bool big = b0 >= 254;
        const uint32_t pl = big ? __builtin_amdgcn_alignbyte(b[1], b[0], 1) : b0;
        const uint32_t pls = big ? 5u : 1u;
        const uint32_t qe = big ? __builtin_amdgcn_alignbyte(b[2], b[1], 1) : __builtin_amdgcn_alignbyte(b[1], b[0], 1);
        const uint32_t qe4 = big ? ((b[2] >> 8) & 0xFF) : ((b[1] >> 8) & 0xFF);
        const uint32_t enc = qe & 0xFF;
        const bool zstr = enc < 0xC0;
        const uint32_t scls = enc >> 6;
        const uint32_t ls = scls == 0 ? 1u : (scls == 1 ? 2u : 5u);
        const uint32_t sl = scls == 0 ? (enc & 0x3F)
                          : scls == 1 ? (((enc & 0x3F) << 8) | ((qe >> 8) & 0xFF))
                                      : ((((qe >> 8) & 0xFF) << 24) | (((qe >> 16) & 0xFF) << 16) |
                                         (((qe >> 24) & 0xFF) << 8) | qe4);
        const bool imm = enc >= 0xF1 && enc <= 0xFD;
        const uint32_t isz = enc == 0xFE ? 1u : enc == 0xC0 ? 2u : enc == 0xF0 ? 3u : enc == 0xD0 ? 4u : enc == 0xE0 ? 8u : 0u;
        const bool int_ok = imm || enc == 0xFE || enc == 0xC0 || enc == 0xF0 || enc == 0xD0 || enc == 0xE0;
        const uint64_t q = (uint64_t)p + pls;
        const uint64_t zsize = zstr ? (uint64_t)pls + ls + sl : (uint64_t)pls + 1 + isz;
        const bool z_bad = p >= zend || (big && p + 5 > zend - 1) || pl != prev_raw || q >= zend - 1 ||
                           (zstr && scls == 1 && q + 2 > zend - 1) || (zstr && scls >= 2 && q + 5 > zend - 1) ||
                           (!zstr && !int_ok) || (uint64_t)p + zsize > zend - 1;
        // ---- pick this lane's class
        bool at_end, bad;
        uint32_t size;
        if (cls == WC_LIST) { at_end = chain_end; bad = l_bad; size = 4 + L32; }
        else if (cls == WC_HT) { at_end = chain_end; bad = h_bad; size = 8 + L32; }
        else if (cls == WC_SL) {
            at_end = !sl_score && chain_end;
            bad = sl_score ? rem < 8 : (sl_extra || h_bad);
            size = sl_score ? 8u : 8 + L32;
        } else if (cls == WC_ZL) {
            at_end = p < zend && z_end;
            bad = z_bad;
            size = (uint32_t)zsize;
        } else {   // WC_IS
            at_end = k >= nint;
            bad = false;
            size = w;
        }
        const bool emit = walking && !at_end && !bad;
        o.fail |= walking && !at_end && bad;
        rec_put(recs, emit, rb, k, r, p | (lane << 16) | (k << 22));
        if (emit) {
            prev_raw = size;
            last = p;
            p += size;
            o.n = k + 1;
        }
        walking = emit && o.n <= r && k + 1 < REC_KMAX;
        o.fail |= emit && (o.n > r || k + 1 >= REC_KMAX);
    }
    // end-of-value checks (rock_serdes.c counts; ziplist header fields)
    if (active && !o.fail) {
        if (cls == WC_HT) {
            const uint32_t type = s8(S, vb);
            o.fail = type == RR_TYPE_SET_HT ? (uint64_t)o.n != cnt : ((o.n & 1) || (uint64_t)(o.n >> 1) != cnt);
        } else if (cls == WC_SL) {
            o.fail = (o.n & 1) || (uint64_t)(o.n >> 1) != cnt;
        } else if (cls == WC_ZL) {
            uint32_t z[3];
            s_read<3>(S, zl0, z);   // zlbytes, zltail, zllen
            const uint32_t entries = o.n - 1;
            const uint32_t zllen = z[2] & 0xFFFF;
            o.fail = p != zend - 1 || (zllen != 0xFFFF && zllen != entries) || z[1] != last - zl0 || (entries & 1);
        }
    }
    return o;
}

// Descriptor for record (pos, k) of a value of `type` at stage offset vb (batch offset of a
// stage position x is sbase + x).  Adds payload bytes to pay.
__device__ __forceinline__ void fast_emit(lds_cptr S, uint64_t sbase, uint32_t type, uint32_t enc, uint32_t vb,
                                          uint32_t len, uint32_t pos, uint32_t k, uint4 &w, uint64_t &pay) {
    uint32_t b[8];   // bytes pos .. pos+31
    s_read<8>(S, pos, b);
    uint64_t data = 0;
    uint32_t elen = 0, kind = RR_K_STR, zenc = 0;
    switch (type) {
        case RR_TYPE_STRING:   // pos == vb
            if (enc == RR_ENC_INT) {
                data = (uint64_t)__builtin_amdgcn_alignbyte(b[2], b[1], 2) |
                       ((uint64_t)__builtin_amdgcn_alignbyte(b[3], b[2], 2) << 32);
                kind = RR_K_INT;
            } else { data = sbase + vb + 6; elen = len - 6; pay += elen; }
            break;
        case RR_TYPE_LIST_QUICKLIST: {
            const uint32_t L = b[0];
            const uint32_t d[5] = {b[1], b[2], b[3], b[4], b[5]};
            int64_t iv;
            if (regs_try_int(d, L, iv)) { data = (uint64_t)iv; kind = RR_K_INT; }
            else { data = sbase + pos + 4; elen = L; pay += L; }
            break;
        }
        case RR_TYPE_SET_INTSET:
            if (enc == 2) data = (uint64_t)(int64_t)(int16_t)(b[0] & 0xFFFF);
            else if (enc == 4) data = (uint64_t)(int64_t)(int32_t)b[0];
            else data = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
            kind = RR_K_INT;
            break;
        case RR_TYPE_SET_HT:
        case RR_TYPE_HASH_HT:
            elen = b[0];
            data = sbase + pos + 8;
            pay += elen;
            break;
        case RR_TYPE_ZSET_SKIPLIST:
            if (k & 1) { data = (uint64_t)b[0] | ((uint64_t)b[1] << 32); kind = RR_K_SCORE; }
            else { elen = b[0]; data = sbase + pos + 8; pay += elen; }
            break;
        default:   // ziplists
            if (k == 0) { data = sbase + pos; elen = len - 13; kind = RR_K_ZLRAW; pay += elen; }
            else {
                // entry header: prevlen 1 byte (enc at +1) or 5 bytes (enc at +5); every field is
                // extracted with static byte offsets from the 32 bytes read (no indexed arrays)
                const bool big = (b[0] & 0xFF) >= 254;
                const uint32_t qo = big ? 5u : 1u;
                const uint32_t e = big ? ((b[1] >> 8) & 0xFF) : ((b[0] >> 8) & 0xFF);
                const uint32_t x1 = big ? ((b[1] >> 16) & 0xFF) : ((b[0] >> 16) & 0xFF);   // byte qo+1
                const uint32_t lo = big ? __builtin_amdgcn_alignbyte(b[2], b[1], 2)
                                        : __builtin_amdgcn_alignbyte(b[1], b[0], 2);        // bytes qo+1..qo+4
                const uint32_t hi = big ? __builtin_amdgcn_alignbyte(b[3], b[2], 2)
                                        : __builtin_amdgcn_alignbyte(b[2], b[1], 2);        // bytes qo+5..qo+8
                if (e < 0xC0) {
                    const uint32_t cls = e & 0xC0;
                    uint32_t ls, sl;
                    if (cls == 0x00) { ls = 1; sl = e & 0x3F; }
                    else if (cls == 0x40) { ls = 2; sl = ((e & 0x3F) << 8) | x1; }
                    else { ls = 5; sl = __builtin_bswap32(lo); }
                    data = sbase + pos + qo + ls;
                    elen = sl;
                    zenc = cls;
                } else {
                    int64_t v;
                    if (e >= 0xF1 && e <= 0xFD) v = (int64_t)(e & 0x0F) - 1;
                    else if (e == 0xFE) v = (int8_t)(lo & 0xFF);
                    else if (e == 0xC0) v = (int16_t)(lo & 0xFFFF);
                    else if (e == 0xF0) v = ((int32_t)(lo << 8)) >> 8;
                    else if (e == 0xD0) v = (int32_t)lo;
                    else v = (int64_t)((uint64_t)lo | ((uint64_t)hi << 32));
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
