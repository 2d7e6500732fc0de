// rr_decode_class.h — type-homogeneous decode of one batch of <= 64 values (lane = value).
//
// The count kernel files every value under a CLASS (one per walk shape, header already checked)
// and the decode kernel sorts each tile of values by class, so a wave only ever runs one
// class's loop: a step costs that class's few instructions, not the union over every type a
// mixed wave would hold (a mixed walk measured ~200 wave-instructions per step, ~60 % of
// them branch/exec-mask SALU).
//
// Bytes come from the workgroup's LDS-staged byte window (LdsSrc), or, for a window whose
// values run too far past it, from global memory through a buffer descriptor (GlbSrc:
// window-relative 32-bit offsets; a read past the blob buffer returns zeros instead of
// faulting).  Either way every step reads a fixed 8-28 bytes at its cursor.
//
// Each routine applies the checks of rock_serdes.c / ziplist.c that the exact parser
// (parse_value) applies; a lane whose value fails any of them reports `fail`, and the caller
// re-runs that value through the exact parser, which assigns the reference's status code and
// zero-fills the value's slots.  Descriptors are stored as they are found (slot eb + k), only
// while k < reservation and the value's slots fit the caller's capacity.
#pragma once
#include "rr_device.h"

namespace rr {

// value classes (count_kernel -> decode sort); the decode kernel runs them heaviest first
constexpr uint32_t C_STR = 0, C_IS = 1, C_LIST = 2, C_HT = 3, C_SL = 4, C_ZL = 5, C_EXACT = 6, C_N = 7;

typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const uint8_t *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)bytes, 0x00020000);
}

// bytes [p, p + 4N) of the tile (tile-relative p) into N dwords; reads past the descriptor's
// range give zero bytes
template <int N>
__device__ __forceinline__ void gread(rsrc_t R, uint32_t p, uint32_t (&o)[N]) {
    constexpr int D = N + 1;
    uint32_t w[D];
    const uint32_t a = p & ~3u, sh = p & 3u;
#pragma unroll
    for (int i = 0; i < D; i += 4) {
        if (D - i >= 4) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(R, (int)(a + 4 * i), 0, 0);
            w[i] = v[0]; w[i + 1] = v[1]; w[i + 2] = v[2]; w[i + 3] = v[3];
        } else if (D - i == 3) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b96(R, (int)(a + 4 * i), 0, 0);
            w[i] = v[0]; w[i + 1] = v[1]; w[i + 2] = v[2];
        } else if (D - i == 2) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(R, (int)(a + 4 * i), 0, 0);
            w[i] = v[0]; w[i + 1] = v[1];
        } else {
            w[i] = __builtin_amdgcn_raw_buffer_load_b32(R, (int)(a + 4 * i), 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
}

// Byte sources for the walks.  p is relative to the source's base; get<N> returns bytes
// [p, p + 4N) as N dwords (N+1 aligned reads + alignbyte).
struct GlbSrc {   // global memory through a buffer descriptor: reads past its range give zeros
    rsrc_t R;
    template <int N>
    __device__ __forceinline__ void get(uint32_t p, uint32_t (&o)[N]) const { gread<N>(R, p, o); }
};
struct LdsSrc {   // the workgroup's staged window; reads may run up to 64 bytes past it
    lds_cptr S;
    template <int N>
    __device__ __forceinline__ void get(uint32_t p, uint32_t (&o)[N]) const {
        const __attribute__((address_space(3))) uint32_t *W = (const __attribute__((address_space(3))) uint32_t *)S;
        const uint32_t a = p >> 2, sh = p & 3;
        uint32_t w[N + 1];
#pragma unroll
        for (int i = 0; i <= N; ++i) w[i] = W[a + i];
#pragma unroll
        for (int i = 0; i < N; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
    }
};

__device__ __forceinline__ uint32_t ab(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }

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

__device__ __forceinline__ void put_desc(rr_elem *e, uint64_t data, uint32_t len, uint32_t kind, uint32_t zenc) {
    uint4 w;
    w.x = (uint32_t)data;
    w.y = (uint32_t)(data >> 32);
    w.z = len;
    w.w = kind | (zenc << 8);
    *reinterpret_cast<uint4 *>(e) = w;
}

__device__ __forceinline__ void put_value(rr_value *v, uint32_t type, uint32_t enc, uint32_t status, uint32_t lru,
                                          uint32_t n, uint32_t eb) {
    uint4 w;
    w.x = type | (enc << 8) | (status << 16);
    w.y = lru & RR_LRU_MASK;
    w.z = n;
    w.w = eb;
    *reinterpret_cast<uint4 *>(v) = w;
}

// One lane's value in a batch.  q: tile-relative offset of the blob, L: its length; B: batch
// offset of tile byte 0 (descriptor data = B + tile position, the mirror-arena offset);
// eb / r: slot base and reservation; ok: the reservation fits the caller's capacity.
struct Lane {
    uint32_t q, L;
    uint64_t B;
    rr_elem *el;       // elems + eb
    uint32_t r;
    bool ok;
};

// header bytes 0..15 of the value: type | lru (bytes 1..4) | byte 5 | bytes 5..8 | bytes 9..12
struct Head {
    uint32_t h[4];
    __device__ __forceinline__ uint32_t type() const { return h[0] & 0xFF; }
    __device__ __forceinline__ uint32_t lru() const { return ab(h[1], h[0], 1); }
    __device__ __forceinline__ uint32_t b5() const { return (h[1] >> 8) & 0xFF; }
    __device__ __forceinline__ uint32_t f5() const { return ab(h[2], h[1], 1); }
    __device__ __forceinline__ uint32_t f9() const { return ab(h[3], h[2], 1); }
    __device__ __forceinline__ uint64_t u5() const { return (uint64_t)f5() | ((uint64_t)f9() << 32); }
};

// ---- String (rock_serdes.c:114-158): enc INT -> inline i64, RAW/EMBSTR -> bytes 6..L
__device__ __forceinline__ void do_string(const Head &H, const Lane &l, uint64_t &pay) {
    if (H.b5() == RR_ENC_INT) {
        if (l.ok) put_desc(l.el, (uint64_t)ab(H.h[2], H.h[1], 2) | ((uint64_t)ab(H.h[3], H.h[2], 2) << 32), 0, RR_K_INT, 0);
    } else {
        if (l.ok) put_desc(l.el, l.B + l.q + 6, l.L - 6, RR_K_STR, 0);
        pay += l.L - 6;
    }
}

// ---- intset (rock_serdes.c:217-245, intset.c:45-52): fixed-width members, no walk
template <class Src>
__device__ __forceinline__ void do_intset(const Src &R, const Head &H, const Lane &l) {
    const uint32_t w = H.f5(), cnt = H.f9();
    if (!l.ok) return;
    uint32_t p = l.q + 13;
    for (uint32_t k = 0; k < cnt; ++k, p += w) {
        uint32_t x[2];
        R.template get<2>(p, x);
        const int64_t v = w == 2 ? (int64_t)(int16_t)(x[0] & 0xFFFF)
                        : w == 4 ? (int64_t)(int32_t)x[0] : (int64_t)((uint64_t)x[0] | ((uint64_t)x[1] << 32));
        put_desc(l.el + k, (uint64_t)v, 0, RR_K_INT, 0);
    }
}

// ---- List (rock_serdes.c:162-214): {u32 len, bytes}* to the end; integer-looking entries
// become INT (quicklistPushTail re-encodes them, ziplist.c:480)
template <class Src>
__device__ __forceinline__ bool do_list(const Src &R, const Lane &l, uint32_t &n, uint64_t &pay) {
    uint32_t p = l.q + 5, k = 0;
    const uint32_t end = l.q + l.L;
    bool fail = false;
    while (p != end) {
        uint32_t b[6];   // len + 20 bytes
        R.template get<6>(p, b);
        const uint32_t rem = end - p, len = b[0];
        if (rem < 4 || len > rem - 4 || k >= l.r) { fail = true; break; }
        const uint32_t d[5] = {b[1], b[2], b[3], b[4], b[5]};
        int64_t iv;
        if (regs_try_int(d, len, iv)) {
            if (l.ok) put_desc(l.el + k, (uint64_t)iv, 0, RR_K_INT, 0);
        } else {
            if (l.ok) put_desc(l.el + k, l.B + p + 4, len, RR_K_STR, 0);
            pay += len;
        }
        ++k;
        p += 4 + len;
    }
    n = k;
    return fail || k != l.r;
}

// ---- Set / Hash hash tables (rock_serdes.c:248-311, :349-414): u64 count, {u64 len, bytes}*
template <class Src>
__device__ __forceinline__ bool do_ht(const Src &R, const Head &H, const Lane &l, uint32_t &n, uint64_t &pay) {
    const uint64_t cnt = H.u5();
    uint32_t p = l.q + 13, k = 0;
    const uint32_t end = l.q + l.L;
    bool fail = false;
    while (p != end) {
        uint32_t b[2];
        R.template get<2>(p, b);
        const uint32_t rem = end - p;
        if (rem < 8 || b[1] != 0 || b[0] > rem - 8 || k >= l.r) { fail = true; break; }
        if (l.ok) put_desc(l.el + k, l.B + p + 8, b[0], RR_K_STR, 0);
        pay += b[0];
        ++k;
        p += 8 + b[0];
    }
    n = k;
    const bool cnt_ok = H.type() == RR_TYPE_SET_HT ? (uint64_t)k == cnt : ((k & 1) == 0 && (uint64_t)(k >> 1) == cnt);
    return fail || !cnt_ok || k != l.r;
}

// ---- ZSet skiplist (rock_serdes.c:448-508): u64 count, {u64 len, member, f64 score}*
template <class Src>
__device__ __forceinline__ bool do_skiplist(const Src &R, const Head &H, const Lane &l, uint32_t &n, uint64_t &pay) {
    const uint64_t cnt = H.u5();
    uint32_t p = l.q + 13, k = 0;
    const uint32_t end = l.q + l.L;
    bool fail = false;
    while (p != end) {
        uint32_t b[2];
        R.template get<2>(p, b);
        const uint32_t rem = end - p;
        if (rem < 8 || k >= l.r) { fail = true; break; }
        if (k & 1) {
            if (l.ok) put_desc(l.el + k, (uint64_t)b[0] | ((uint64_t)b[1] << 32), 0, RR_K_SCORE, 0);
            p += 8;
        } else {
            if (b[1] != 0 || b[0] > rem - 8) { fail = true; break; }
            if (l.ok) put_desc(l.el + k, l.B + p + 8, b[0], RR_K_STR, 0);
            pay += b[0];
            p += 8 + b[0];
        }
        ++k;
    }
    n = k;
    return fail || (k & 1) || (uint64_t)(k >> 1) != cnt || k != l.r;
}

// ---- Hash / ZSet ziplists (rock_serdes.c:314-346, :417-446; ziplist.c:300-447): element 0
// is the raw ziplist, then one descriptor per entry
template <class Src>
__device__ __forceinline__ bool do_ziplist(const Src &R, const Lane &l, uint32_t &n, uint64_t &pay) {
    const uint32_t zl0 = l.q + 13, zend = l.q + l.L, zlast = zend - 1;   // zlast: the 0xFF byte
    uint32_t z[3];
    R.template get<3>(zl0, z);   // zlbytes, zltail, zllen
    if (l.ok) put_desc(l.el, l.B + zl0, l.L - 13, RR_K_ZLRAW, 0);
    pay += l.L - 13;
    uint32_t p = zl0 + 10, prev_raw = 0, last = zl0 + 10, k = 1;
    bool fail = false;
    for (;;) {
        uint32_t b[4];   // prevlen (1 or 5) + encoding + up to 9 more bytes
        R.template get<4>(p, b);
        const uint32_t b0 = b[0] & 0xFF;
        if (p >= zend) { fail = true; break; }
        if (b0 == 0xFF) break;
        // every field of the entry header from registers, as selects (no per-encoding branches)
        const bool big = b0 >= 254;
        const uint32_t pl = big ? ab(b[1], b[0], 1) : b0;
        const uint32_t qp = p + (big ? 5u : 1u);
        const uint32_t e = big ? (b[1] >> 8) & 0xFF : (b[0] >> 8) & 0xFF;
        const uint32_t x1 = big ? (b[1] >> 16) & 0xFF : (b[0] >> 16) & 0xFF;
        const uint32_t lo = big ? ab(b[2], b[1], 2) : ab(b[1], b[0], 2);   // bytes after the encoding byte
        const uint32_t hi = big ? ab(b[3], b[2], 2) : ab(b[2], b[1], 2);
        const bool zstr = e < 0xC0;
        const uint32_t scls = e >> 6;   // string length class 0 / 1 / 2
        const uint32_t ls = scls == 0 ? 1u : scls == 1 ? 2u : 5u;
        const uint32_t sl = scls == 0 ? (e & 0x3F) : scls == 1 ? (((e & 0x3F) << 8) | x1) : __builtin_bswap32(lo);
        const bool imm = e - 0xF1u <= 0xFDu - 0xF1u;
        const uint32_t isz = e == 0xFE ? 1u : e == 0xC0 ? 2u : e == 0xF0 ? 3u : e == 0xD0 ? 4u : e == 0xE0 ? 8u : 0u;
        const int64_t i8 = (int8_t)(lo & 0xFF), i16 = (int16_t)(lo & 0xFFFF), i24 = ((int32_t)(lo << 8)) >> 8;
        const int64_t i32 = (int32_t)lo, i64 = (int64_t)((uint64_t)lo | ((uint64_t)hi << 32));
        const int64_t iv = imm ? (int64_t)(e & 0x0F) - 1 : isz == 1 ? i8 : isz == 2 ? i16 : isz == 3 ? i24 : isz == 4 ? i32 : i64;
        const uint64_t endp = zstr ? (uint64_t)qp + ls + sl : (uint64_t)qp + 1 + isz;
        const bool bad = (big && p + 5 > zlast) || pl != prev_raw || qp >= zlast || k >= l.r ||
                         (!zstr && !imm && isz == 0) || (zstr && qp + ls > zlast) || endp > zlast;
        if (bad) { fail = true; break; }
        if (l.ok) put_desc(l.el + k, zstr ? l.B + qp + ls : (uint64_t)iv, zstr ? sl : 0, zstr ? RR_K_STR : RR_K_INT,
                           zstr ? (e & 0xC0) : e);
        prev_raw = (uint32_t)endp - p;
        last = p;
        p = (uint32_t)endp;
        ++k;
    }
    n = k;
    const uint32_t entries = k - 1, zllen = z[2] & 0xFFFF;
    return fail || p != zlast || (zllen != 0xFFFF && zllen != entries) || z[1] != last - zl0 || (entries & 1) ||
           k != l.r;
}

}  // namespace rr
