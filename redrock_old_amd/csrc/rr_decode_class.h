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

// value classes (count_kernel -> decode sort); the decode kernel runs them heaviest first.
// Sets and hashes are separate classes so a batch knows wave-uniformly which members are keys.
constexpr uint32_t C_STR = 0, C_IS = 1, C_LIST = 2, C_HT = 3, C_SL = 4, C_ZL = 5, C_EXACT = 6, C_HH = 7, C_N = 8;

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

// Byte sources for the walks.  p is relative to the source's base.  fetch<N>(p) issues the
// N+1 aligned dword reads covering bytes [p, p + 4N) and returns them raw; Raw::align turns
// them into N dwords.  The walks fetch the NEXT cursor's bytes and align them only at the top
// of the next step, so the read's latency overlaps the current step's checks and stores (an
// align right after the read would make the compiler wait for it there).
template <int N>
struct Raw {
    uint32_t w[N + 1];
    uint32_t sh;
    __device__ __forceinline__ void align(uint32_t (&o)[N]) const {
#pragma unroll
        for (int i = 0; i < N; ++i) o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
    }
};

struct GlbSrc {   // global memory through a buffer descriptor: reads past its range give zeros
    rsrc_t R;
    template <int N>
    __device__ __forceinline__ Raw<N> fetch(uint32_t p) const {
        constexpr int D = N + 1;
        Raw<N> r;
        const uint32_t a = p & ~3u;
        r.sh = p & 3u;
#pragma unroll
        for (int i = 0; i < D; i += 4) {
            if (D - i >= 4) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(R, (int)(a + 4 * i), 0, 0);
                r.w[i] = v[0]; r.w[i + 1] = v[1]; r.w[i + 2] = v[2]; r.w[i + 3] = v[3];
            } else if (D - i == 3) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b96(R, (int)(a + 4 * i), 0, 0);
                r.w[i] = v[0]; r.w[i + 1] = v[1]; r.w[i + 2] = v[2];
            } else if (D - i == 2) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(R, (int)(a + 4 * i), 0, 0);
                r.w[i] = v[0]; r.w[i + 1] = v[1];
            } else {
                r.w[i] = __builtin_amdgcn_raw_buffer_load_b32(R, (int)(a + 4 * i), 0, 0);
            }
        }
        return r;
    }
    template <int N>
    __device__ __forceinline__ void get(uint32_t p, uint32_t (&o)[N]) const { fetch<N>(p).align(o); }
    // the chain steps' reads: the dword / the byte at p (an aligned pair + alignbyte here)
    __device__ __forceinline__ uint32_t u32(uint32_t p) const { uint32_t x[1]; get<1>(p, x); return x[0]; }
    __device__ __forceinline__ uint32_t u8(uint32_t p) const { return u32(p) & 0xFF; }
    __device__ __forceinline__ uint32_t u8b(uint32_t p) const { return u8(p); }
};
struct LdsSrc {   // the workgroup's staged window; reads may run up to 64 bytes past it
    lds_cptr S;
    template <int N>
    __device__ __forceinline__ Raw<N> fetch(uint32_t p) const {
        const __attribute__((address_space(3))) uint32_t *W = (const __attribute__((address_space(3))) uint32_t *)S;
        Raw<N> r;
        const uint32_t a = p >> 2;
        r.sh = p & 3;
#pragma unroll
        for (int i = 0; i <= N; ++i) r.w[i] = W[a + i];
        return r;
    }
    template <int N>
    __device__ __forceinline__ void get(uint32_t p, uint32_t (&o)[N]) const { fetch<N>(p).align(o); }
    // the chain steps' reads: the dword at p from the aligned pair + alignbyte.  (An unaligned
    // ds_read_b32 — gfx950 serves it — measured slower on every walk: ZL batches 16.7K -> 22.4K
    // cycles, cfg 4 0.353 -> 0.392 ms; the LDS splits it.)
    __device__ __forceinline__ uint32_t u32(uint32_t p) const { uint32_t x[1]; get<1>(p, x); return x[0]; }
    __device__ __forceinline__ uint32_t u8(uint32_t p) const { return u32(p) & 0xFF; }
    // the byte at p by a byte read (ds_read_u8: any address, no align step)
    __device__ __forceinline__ uint32_t u8b(uint32_t p) const { return S[p]; }
};

__device__ __forceinline__ uint32_t ab(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }

// zipTryEncoding (ziplist.c:480) + string2ll (util.c:360) over bytes d[0, len) given as 5
// dwords: an entry of 1..31 bytes is an integer iff it is "0" or [-]?[1-9][0-9]* within int64.
// A 20-digit magnitude is always >= 1e19 > 2^63, so more than 20 bytes fails; up to 19 digits
// cannot overflow uint64.
//
// Straight-line SWAR (selects only, so a wave pays one pass whatever mix of lengths its lanes
// hold): the digit check runs four bytes at a time; the digits are turned into values 0-9 by
// one subtraction per dword and RIGHT-aligned in a 20-byte field (a funnel shift by 20 - len
// bytes: dwords by three conditional moves, bytes by alignbyte), which leaves leading zeros and
// pushes the bytes past the entry out; each dword then converts as 4 digits with two multiply-
// add steps (pairs, then the two pairs), and five 4-digit chunks combine with two 64-bit MADs.
__device__ __forceinline__ uint32_t swar4(uint32_t x) {   // bytes d0..d3 (d0 most significant) -> value
    const uint32_t t = x * 10u + (x >> 8);                  // bytes 0 / 2: 10*d0+d1, 10*d2+d3
    return __umul24(t & 0xFFu, 100u) + ((t >> 16) & 0xFFu);
}
__device__ __forceinline__ bool regs_try_int(const uint32_t (&b)[5], uint32_t len, int64_t &out) {
    const uint32_t c0 = b[0] & 0xFF;
    const uint32_t neg = c0 == '-' ? 1u : 0u;
    // digit check of bytes [neg, len) four at a time (SWAR, VALU only): a byte is a digit iff
    // its high nibble is 3 and its low nibble + 6 does not carry into bit 4
    uint32_t nondig = 0;
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) {
        const uint32_t x = b[k];
        const uint32_t nd = ((x & 0xF0F0F0F0u) ^ 0x30303030u) | (((x & 0x0F0F0F0Fu) + 0x06060606u) & 0x10101010u);
        const uint32_t cnt = len > 4 * k + 4 ? 4u : len > 4 * k ? len - 4 * k : 0u;
        uint32_t m = cnt ? 0xFFFFFFFFu >> (32 - 8 * cnt) : 0u;
        if (k == 0) m &= neg ? 0xFFFFFF00u : 0xFFFFFFFFu;
        nondig |= nd & m;
    }
    // digit values: '-' becomes a leading 0; borrows of non-digit bytes past the entry only run
    // upward, into bytes the shift drops
    uint32_t x[5];
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) x[k] = b[k];
    x[0] = neg ? (x[0] & 0xFFFFFF00u) | 0x30u : x[0];
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) x[k] -= 0x30303030u;
    // right-align: byte i -> byte i + s, s = 20 - len (len > 20 never passes the checks)
    const uint32_t s = len <= 20 ? 20 - len : 0;
    const uint32_t q = s >> 2, r = s & 3;
    if (q & 1) { x[4] = x[3]; x[3] = x[2]; x[2] = x[1]; x[1] = x[0]; x[0] = 0; }
    if (q & 2) { x[4] = x[2]; x[3] = x[1]; x[2] = x[0]; x[1] = 0; x[0] = 0; }
    if (q & 4) { x[4] = x[0]; x[3] = 0; x[2] = 0; x[1] = 0; x[0] = 0; }
    uint32_t y[5];
#pragma unroll
    for (uint32_t k = 0; k < 5; ++k) {
        const uint32_t lo = k ? x[k - 1] : 0u;
        y[k] = r ? __builtin_amdgcn_alignbyte(x[k], lo, 4 - r) : x[k];
    }
    const uint32_t h8 = __umul24(swar4(y[0]), 10000u) + swar4(y[1]);   // < 1e8
    const uint32_t m8 = __umul24(swar4(y[2]), 10000u) + swar4(y[3]);
    const uint64_t v16 = (uint64_t)h8 * 100000000ull + m8;              // < 1e16
    const uint64_t v = (uint64_t)(uint32_t)v16 * 10000ull + swar4(y[4]) + ((uint64_t)((uint32_t)(v16 >> 32) * 10000u) << 32);
    const uint32_t c1 = (b[0] >> 8) & 0xFF;
    const uint32_t dfirst = (neg ? c1 : c0) - '0';
    const uint32_t nd = len - neg;
    const bool zero = len == 1 && c0 == '0';
    const bool ok = zero | ((nondig == 0) & (dfirst - 1u <= 8u) & (len <= 20) & (nd - 1u <= 18u) &
                           (v <= 0x7FFFFFFFFFFFFFFFull + neg));
    out = zero ? 0 : neg ? (int64_t)(0ull - v) : (int64_t)v;
    return ok;
}

// Descriptor stores go through a buffer descriptor over the window's slot range: a slot
// offset of NOSLOT (lanes whose value does not fit the caller's capacity) is out of range and
// the hardware drops the store, so no store needs a branch.
constexpr uint32_t NOSLOT = 0xFFFFFFF0u;
__device__ __forceinline__ void put_desc(rsrc_t E, uint32_t off, uint64_t data, uint32_t len, uint32_t kind,
                                         uint32_t zenc) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u w;
    w.x = (uint32_t)data;
    w.y = (uint32_t)(data >> 32);
    w.z = len;
    w.w = kind | (zenc << 8);
#if defined(RR_ABLATE) && RR_ABLATE == 4   // timing-only builds (tools/): no descriptor stores
    asm volatile("" ::"v"(w.x), "v"(w.y), "v"(w.z), "v"(w.w), "v"(off));
#else
    __builtin_amdgcn_raw_buffer_store_b128(w, E, (int)off, 0, 0);   // (nontemporal: cfg 3 0.45 -> 0.73 ms, the L2 combines them)
#endif
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

// One lane's value in a batch.  q: source-relative offset of the blob, L: its length; B: batch
// offset of source byte 0 (descriptor data = B + source position, the mirror-arena offset);
// r: its reservation; ok: the reservation fits the caller's capacity.
struct Lane {
    uint32_t q, L;
    uint64_t B;
    rsrc_t E;          // descriptors of the window
    uint32_t so;       // byte offset of slot eb in E
    uint32_t r;
    bool ok;
    // byte offset of the value's slot k, or NOSLOT when its slots do not fit
    __device__ __forceinline__ uint32_t slot(uint32_t k) const { return ok ? so + 16 * k : NOSLOT; }
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
        put_desc(l.E, l.slot(0), (uint64_t)ab(H.h[2], H.h[1], 2) | ((uint64_t)ab(H.h[3], H.h[2], 2) << 32), 0, RR_K_INT, 0);
    } else {
        put_desc(l.E, l.slot(0), l.B + l.q + 6, l.L - 6, RR_K_STR, 0);
        pay += l.L - 6;
    }
}

// The walks run the whole wave in lock-step: every lane executes every step, a lane that is
// done or failed is masked by selects (its cursor frozen, its descriptor store sent to NOSLOT),
// and the loop exits when a ballot finds no lane still walking.  Divergent per-lane loop exits
// instead cost ~10 exec-mask SALU instructions per step, half of all issued instructions.
//
// They are also software-pipelined: a step computes the next cursor from the bytes it holds
// and issues the read there BEFORE its checks and descriptor store, so the read's latency
// overlaps them.  The loop body is two steps with the raw read buffers swapping roles
// (ping-pong): one step per iteration needs a register copy of the in-flight buffer at the
// back-edge, and the compiler waits for the read to land before that copy.
#define RR_PINGPONG(RA, RB, STEP)  \
    for (;;) {                     \
        if (STEP(RA, RB)) break;   \
        if (STEP(RB, RA)) break;   \
    }

// ---- duplicate keys of hash tables (desSet's dictAdd keeps the first copy, rock_serdes.c:297;
// desHash asserts there is none, :399-400).  The walk fingerprints every key member (set members,
// hash fields) of a value with at most HT_FP_KEYS keys into 16 bits and keeps them in a packed
// register shift register (no LDS: the stage fills it); a repeated fingerprint, or a value with
// more keys, goes on the fixup list, where fixup_kernel compares the actual bytes.
// A member's fingerprint hashes its length and the 8 bytes that end it.  For a member shorter
// than 8 bytes those include the tail of its own length field — a function of the length — so
// equal members always hash equal, and the bytes come with the read of the next length field.
constexpr uint32_t HT_FP_KEYS = 16;
__device__ __forceinline__ uint32_t member_fp16(uint32_t len, uint32_t lo, uint32_t hi) {
    uint32_t h = (lo ^ __builtin_amdgcn_alignbit(hi, hi, 13) ^ len) * 0x9E3779B1u;
    h = (h ^ hi ^ (h >> 15)) * 0x85EBCA6Bu;
    h = (h >> 16) ^ (h & 0xFFFFu);
    return h == 0xFFFFu ? 0xFFFEu : h;   // 0xFFFF marks an empty slot
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// ---- Set / Hash hash tables (rock_serdes.c:248-311, :349-414): u64 count, {u64 len, bytes}*
// Every step reads 16 bytes at p - 8: the 8 bytes ending the previous member (its fingerprint)
// and this member's length field.  HASH is wave-uniform (sets and hashes are separate classes),
// so a hash batch skips the fingerprint work on the steps that end a value, not a field.
template <class Src>
__device__ __forceinline__ bool do_ht(const Src &R, const Head &H, const Lane &l, bool active, uint32_t &n,
                                      uint64_t &pay, bool &fix, const bool hash) {
    const uint64_t cnt = H.u5();
    const bool chk = active && cnt <= HT_FP_KEYS;
    bool dupfp = active && cnt > HT_FP_KEYS;
    uint32_t p = l.q + 13, k = 0, it = 0, plen = 0;
    const uint32_t end = l.q + l.L;
    bool fail = false, live = active;
    uint32_t fpr[HT_FP_KEYS / 2];
#pragma unroll
    for (uint32_t j = 0; j < HT_FP_KEYS / 2; ++j) fpr[j] = 0xFFFFFFFFu;
    Raw<4> ra = R.template fetch<4>(p - 8), rb;
    auto step = [&](const Raw<4> &cur, Raw<4> &nxt) __attribute__((always_inline)) {
        uint32_t b[4];
        cur.align(b);
        const uint32_t rem = end - p;
        const uint64_t nx = (uint64_t)p + 8 + b[2];
        const uint32_t pn = ((nx < end) & (b[3] == 0)) ? (uint32_t)nx : end;
        nxt = R.template fetch<4>((live ? pn : p) - 8);
        __builtin_amdgcn_sched_barrier(0);   // keep the read ahead of the checks and the store
        const bool done = p == end;
        const bool bad = (rem < 8) | (b[3] != 0) | (b[2] > rem - 8) | (k >= l.r);
        const bool emit = live & !done & !bad;
        fail |= live & !done & bad;
        put_desc(l.E, emit ? l.slot(k) : NOSLOT, l.B + p + 8, b[2], RR_K_STR, 0);
        pay += emit ? b[2] : 0;
        // the member before p (member it - 1 of every live lane) is a key: fingerprint it, test
        // it against the earlier keys, shift it in (lanes that stopped walking no longer care)
        if (it > 0 && (!hash || (it & 1))) {
            const uint32_t f = member_fp16(plen, b[0], b[1]);
            const uint32_t pat = f | (f << 16);
            u16x2 m = __builtin_bit_cast(u16x2, fpr[0] ^ pat);
#pragma unroll
            for (uint32_t j = 1; j < HT_FP_KEYS / 2; ++j)
                m = __builtin_elementwise_min(m, __builtin_bit_cast(u16x2, fpr[j] ^ pat));
            dupfp |= chk & live & ((m.x == 0) | (m.y == 0));
#pragma unroll
            for (uint32_t j = HT_FP_KEYS / 2 - 1; j > 0; --j) fpr[j] = __builtin_amdgcn_alignbit(fpr[j], fpr[j - 1], 16);
            fpr[0] = (fpr[0] << 16) | f;
        }
        plen = b[2];
        ++it;
        k += emit;
        p = emit ? pn : p;
        live = emit;
        return __ballot(live) == 0;
    };
    RR_PINGPONG(ra, rb, step)
    n = k;
    const bool cnt_ok = !hash ? (uint64_t)k == cnt : ((k & 1) == 0 && (uint64_t)(k >> 1) == cnt);
    fix = dupfp && k >= (hash ? 4u : 2u);
    return fail || !cnt_ok || k != l.r;
}

// ---- grouped walks ---------------------------------------------------------------------
// A batch of cnt values gives each value G = 64 / cnt lanes (G <= GMAX, uniform per batch;
// lane g of its group).  Every lane of a group walks the value's chain — the length fields, a
// read and an add per element, the same LDS address for the whole group — and the per-element
// work that does not feed the chain (integer parse, descriptor store, score checks) is split:
// lane g takes elements g, g + G, g + 2G, ...  A walk step costs ~4 cycles per wave-instruction
// whatever the number of active lanes, so with ~20 Lists or ~4 skiplists per window this cuts
// the wave-instructions of a batch 2-8x.  Every lane of a group sees every element, so checks
// over the whole value (counts, fingerprints, score order) come out the same on all of them;
// the group's lane 0 records the value.
constexpr uint32_t GMAX = 16;

// One verdict for a grouped value: any lane's failure fails the whole group
__device__ __forceinline__ bool group_any(bool x, uint32_t G, uint32_t g) {
    const uint32_t base = lane_id() - g;
    const uint64_t gm = (G >= 64 ? ~0ull : ((1ull << G) - 1)) << base;
    return (__ballot(x) & gm) != 0;
}

// ---- List (rock_serdes.c:162-214), grouped: {u32 len, bytes}* to the end.  The chain takes
// exactly the value's reservation of elements (count_kernel counted the ones that parse) with
// no checks — a read and an add per element, the position clamped to the value; each lane then
// checks its own elements' length fields (and that the last one ends the value) and stores
// them.  The verdicts are those of one walk to the end.
// Software-pipelined with the group size a compile-time constant: round r + 1's G chain steps are
// issued in the same basic block as round r's element decode (string2ll, checks, descriptor
// store), so the decode fills the chain's LDS-latency gaps (as do_ziplist_bp; LIST batch 17.3K
// -> 12.1K cycles).  The last round walks one wasted chain (clamped at the value's end).
template <uint32_t G, class Src>
__device__ __forceinline__ bool do_list_bp(const Src &R, const Lane &l, bool active, uint32_t g, uint32_t &n,
                                           uint64_t &pay) {
    const uint32_t end = l.q + l.L, r = active ? l.r : 0u;
    uint32_t p = l.q + 5;
    bool fail = active && r == 0 && p != end;
    auto chain = [&](uint32_t &mp) __attribute__((always_inline)) {
        mp = l.q;
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) {
            const uint32_t x = R.u32(p);
            const uint32_t rem = end - p;
            mp = j == g ? p : mp;
            p = min(p + 4 + min(x, rem), end);
        }
    };
    auto decode = [&](uint32_t mk, uint32_t mp) __attribute__((always_inline)) {
        const bool mine = mk < r;
        uint32_t b[6];
        R.template get<6>(mp, b);
        const uint32_t ml = b[0], rem = end - mp;
        const bool bad = (rem < 4) | (ml > rem - 4) | ((mk + 1 == r) & (mp + 4 + ml != end));
        fail |= mine & bad;
        const uint32_t d[5] = {b[1], b[2], b[3], b[4], b[5]};
        int64_t iv;
        const bool isint = regs_try_int(d, ml, iv);
        const bool st = mine & !bad;
        put_desc(l.E, st ? l.slot(mk) : NOSLOT, isint ? (uint64_t)iv : l.B + mp + 4, isint ? 0 : ml,
                 isint ? RR_K_INT : RR_K_STR, 0);
        pay += st && !isint ? ml : 0;
    };
    uint32_t mpA;
    chain(mpA);
    for (uint32_t rounds = 0;; ++rounds) {
        uint32_t mpB;
        chain(mpB);                     // round + 1's chain ...
        decode(rounds * G + g, mpA);    // ... beside round's element decode
        if (__ballot((rounds + 1) * G < r) == 0) break;
        mpA = mpB;
    }
    n = r;
    return group_any(fail, G, g);
}

// ---- Set / Hash hash tables, grouped.  The chain steps read only the u64 length fields (every
// lane of the group walks the same chain: a read, three checks and an add per member); lane g
// takes members g, g + G, ...: once per G chain steps it stores its member's descriptor and,
// for a key member, fingerprints it from the 8 bytes that end it (as do_ht).  The walk takes
// exactly the value's reservation of members and then must stand at the value's end (the
// verdicts of do_ht's walk to the end).  The duplicate test runs once per value after the
// walk: each lane compares the keys it holds with those of every other lane of its group
// (rotations by d = 1 .. G-1, one shuffle per round of keys) and its own.  A lane keeps the
// keys of its first HT_G_ROUNDS rounds, which covers HT_FP_KEYS keys when G >= HT_FP_KEYS /
// HT_G_ROUNDS lanes hold keys (a hash's keys are its even members: G >= 8; a set: G >= 4 —
// below that the batch runs do_ht).
constexpr uint32_t HT_G_ROUNDS = 4;
__device__ __forceinline__ uint32_t ht_group_min(bool hash) { return hash ? 2 * HT_FP_KEYS / HT_G_ROUNDS : HT_FP_KEYS / HT_G_ROUNDS; }
template <class Src>
__device__ __forceinline__ bool do_ht_g(const Src &R, const Head &H, const Lane &l, bool active, uint32_t G,
                                        uint32_t g, uint32_t &n, uint64_t &pay, bool &fix, const bool hash) {
    const uint64_t cnt = H.u5();
    const bool chk = active && cnt <= HT_FP_KEYS;
    const uint32_t end = l.q + l.L, r = active ? l.r : 0u;
    uint32_t p = l.q + 13;
    bool fail = active && r == 0 && p != end;   // an empty table is its 13-byte header
    uint32_t fps[HT_G_ROUNDS];
#pragma unroll
    for (uint32_t q = 0; q < HT_G_ROUNDS; ++q) fps[q] = 0xFFFFFFFFu;
    uint32_t rounds = 0;   // (wave-uniform)
    for (;; ++rounds) {
        // G chain steps with no checks: p only moves forward and stays <= end, a member whose
        // length does not fit is caught by its own lane below (and fails the whole value)
        uint32_t mp = l.q;
        for (uint32_t j = 0; j < G; ++j) {
            const uint32_t x = R.u32(p);
            const uint32_t rem = end - p;
            mp = j == g ? p : mp;
            p = min(p + 8 + min(x, rem), end);
        }
        // my member (index mk): its length field's checks, the descriptor, the fingerprint
        const uint32_t mk = rounds * G + g;
        const bool mine = mk < r;
        uint32_t x[2];
        R.template get<2>(mp, x);
        const uint32_t ml = x[0], rem = end - mp;
        const bool bad = (rem < 8) | (x[1] != 0) | (ml > rem - 8) | ((mk + 1 == r) & (mp + 8 + ml != end));
        fail |= mine & bad;
        put_desc(l.E, (mine & !bad) ? l.slot(mk) : NOSLOT, l.B + mp + 8, ml, RR_K_STR, 0);
        pay += (mine & !bad) ? ml : 0;
        uint32_t t[2];
        R.template get<2>((mine & !bad) ? mp + ml : l.q, t);   // bytes [mp + 8 + ml - 8, mp + 8 + ml): the member's last 8
        const bool key = mine & (!hash | ((mk & 1) == 0));
        const uint32_t f = key ? member_fp16(ml, t[0], t[1]) : 0xFFFFFFFFu;
#pragma unroll
        for (uint32_t q = 0; q < HT_G_ROUNDS; ++q) fps[q] = rounds == q ? f : fps[q];
        if (__ballot((rounds + 1) * G < r) == 0) break;
    }
    // duplicate keys: each key packed with its group's id (lane / G; G is a power of two <= 16
    // here, so a group never straddles a 16-lane DPP row), non-keys get values no key can have
    // and no other slot shares; then my keys against each other and against those of the lanes
    // d = 1 .. G-1 away in my row (DPP row rotations: no LDS round trips), so an equal pair is
    // a repeated fingerprint within one value
    const uint32_t RU = rounds + 1 < HT_G_ROUNDS ? rounds + 1 : HT_G_ROUNDS;   // rounds holding keys
    const uint32_t base = lane_id() - g;
    const uint32_t gid = lane_id() / G;
    uint32_t fpp[HT_G_ROUNDS];
#pragma unroll
    for (uint32_t q = 0; q < HT_G_ROUNDS; ++q)
        fpp[q] = fps[q] != 0xFFFFFFFFu ? (gid << 16) | fps[q] : 0xFFFF0000u | (lane_id() << 2) | q;
    bool dup = false;
#pragma unroll
    for (uint32_t a = 0; a < HT_G_ROUNDS; ++a)
#pragma unroll
        for (uint32_t b = a + 1; b < HT_G_ROUNDS; ++b) dup |= fpp[a] == fpp[b];
    // A hash's keys are its even members and G is even, so only even lanes hold keys: an odd
    // rotation pairs keys with non-keys and is skipped.  The fillers (top half 0xFFFF, unique per
    // lane and round) match nothing, so the rounds past RU need no mask in the compares.
#define RR_HT_ROT(D)                                                                                   \
    if ((D) < G && (!hash || ((D) & 1) == 0)) {                                                        \
        _Pragma("unroll") for (uint32_t q = 0; q < HT_G_ROUNDS; ++q) {                                 \
            if (q < RU) {                                                                              \
                const uint32_t x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)fpp[q], 0x120 + (D), 0xF, 0xF, false); \
                _Pragma("unroll") for (uint32_t qq = 0; qq < HT_G_ROUNDS; ++qq) dup |= fpp[qq] == x;   \
            }                                                                                          \
        }                                                                                              \
    }
    RR_HT_ROT(1) RR_HT_ROT(2) RR_HT_ROT(3) RR_HT_ROT(4) RR_HT_ROT(5) RR_HT_ROT(6) RR_HT_ROT(7)
    RR_HT_ROT(8) RR_HT_ROT(9) RR_HT_ROT(10) RR_HT_ROT(11) RR_HT_ROT(12) RR_HT_ROT(13) RR_HT_ROT(14) RR_HT_ROT(15)
#undef RR_HT_ROT
    const uint64_t gm = (G >= 64 ? ~0ull : ((1ull << G) - 1)) << base;
    const bool gfail = (__ballot(fail) & gm) != 0;
    const bool dupg = (__ballot(dup & chk) & gm) != 0;
    n = r;
    const bool cnt_ok = !hash ? (uint64_t)r == cnt : ((r & 1) == 0 && (uint64_t)(r >> 1) == cnt);
    fix = active && (cnt > HT_FP_KEYS || (chk && dupg)) && r >= (hash ? 4u : 2u);
    return gfail || !cnt_ok;
}

// ---- ZSet skiplist, grouped: the chain takes the reservation's pairs with no checks (a read
// and an add per pair: {u64 l, member, f64 score}); each lane then checks its pairs' length
// fields and scores — the order / NaN check (see do_skiplist) against the previous pair's
// score, from the lane before it or, for a round's first pair, from the previous round's last
template <class Src>
__device__ __forceinline__ bool do_skiplist_g(const Src &R, const Head &H, const Lane &l, bool active, uint32_t G,
                                              uint32_t g, uint32_t &n, uint64_t &pay) {
    const uint64_t cnt = H.u5();
    const uint32_t end = l.q + l.L, r = active ? l.r : 0u, np = r >> 1;   // np: pairs
    uint32_t p = l.q + 13;
    bool fail = active && ((r & 1) || (uint64_t)np != cnt || (np == 0 && p != end));
    const uint32_t base = lane_id() - g;
    uint32_t clo = 0, chi = 0;   // the previous round's last score
    for (uint32_t rounds = 0;; ++rounds) {
        uint32_t mp = l.q;
        for (uint32_t j = 0; j < G; ++j) {
            const uint32_t x = R.u32(p);
            const uint32_t rem = end - p;
            mp = j == g ? p : mp;
            p = min(p + 16 + min(x, rem), end);
        }
        const uint32_t mk = rounds * G + g;
        const bool mine = mk < np;
        uint32_t a[2], c[2];
        R.template get<2>(mp, a);
        const uint32_t ml = a[0], rem = end - mp;
        const bool bad1 = (rem < 16) | (a[1] != 0) | (ml > rem - 16) | ((mk + 1 == np) & (mp + 16 + ml != end));
        R.template get<2>((mine & !bad1) ? mp + 8 + ml : l.q, c);
        const double sc = __longlong_as_double((long long)((uint64_t)c[0] | ((uint64_t)c[1] << 32)));
        const uint32_t plo = wave_from_prev(c[0]), phi = wave_from_prev(c[1]);   // (lane g - 1; g = 0 uses clo / chi)
        const double prev = __longlong_as_double((long long)(g ? ((uint64_t)plo | ((uint64_t)phi << 32))
                                                               : ((uint64_t)clo | ((uint64_t)chi << 32))));
        clo = (uint32_t)__shfl((int)c[0], (int)(base + G - 1), RR_WAVE);
        chi = (uint32_t)__shfl((int)c[1], (int)(base + G - 1), RR_WAVE);
        // strictly below the previous score (pair 0: not NaN)
        const bool order = mk == 0 ? !(sc != sc) : sc < prev;
        const bool bad = bad1 | !order;
        fail |= mine & bad;
        const bool st = mine & !bad;
        put_desc(l.E, st ? l.slot(2 * mk) : NOSLOT, l.B + mp + 8, ml, RR_K_STR, 0);
        put_desc(l.E, st ? l.slot(2 * mk + 1) : NOSLOT, (uint64_t)c[0] | ((uint64_t)c[1] << 32), 0, RR_K_SCORE, 0);
        pay += st ? ml : 0;
        if (__ballot((rounds + 1) * G < np) == 0) break;
    }
    n = r;
    return group_any(fail, G, g);
}

// ---- intset, grouped: members at fixed positions, lane g takes members g, g + G, ...; the
// width (2 / 4 / 8, per lane) is a bit-field width, not a branch
template <class Src>
__device__ __forceinline__ void do_intset_g(const Src &R, const Head &H, const Lane &l, bool active, uint32_t G,
                                            uint32_t g) {
    const uint32_t w = H.f5(), cnt = active && l.ok ? H.f9() : 0;
    for (uint32_t k0 = 0; __ballot(k0 + g < cnt) != 0; k0 += G) {
        const uint32_t k = k0 + g;
        const bool live = k < cnt;
        uint32_t x[2];
        R.template get<2>(l.q + 13 + (live ? w * k : 0u), x);
        const uint32_t lo = w == 2 ? (uint32_t)__builtin_amdgcn_sbfe((int)x[0], 0, 16) : x[0];
        const uint32_t hi = w == 8 ? x[1] : (uint32_t)((int32_t)lo >> 31);
        put_desc(l.E, live ? l.so + 16 * k : NOSLOT, (uint64_t)lo | ((uint64_t)hi << 32), 0, RR_K_INT, 0);
    }
}

// ---- Hash / ZSet ziplists (rock_serdes.c:314-346, :417-446; ziplist.c:300-447): element 0
// is the raw ziplist, then one descriptor per entry.  Grouped on ONE backward chain: a backward
// step needs only the prevlen field (ziplist.c:300-330: 1 byte, or 0xFE + u32; an entry's
// prevlen is the size of the entry before it), so the chain costs a few instructions per entry;
// all the per-entry work — the encoding, the length / integer fields, the checks, the descriptor
// store — is done off the chain, lane g of the value's G-lane group taking entries N-1-g,
// N-1-g-G, ...  The checks are those of one forward walk (ziplist.c:300-447): the entries tile
// [10, zlbytes-1) exactly (each entry, decoded from its own header, ends where the next one
// starts; the last ends at the 0xFF byte, entry 0 starts right after the header with prevlen 0),
// zltail is the last entry, zllen entries, an even count of them.  A ziplist whose zllen
// saturated (0xFFFF) goes to the exact parser.
// Software-pipelined with the group size a compile-time constant: a round's G backward chain
// steps are straight-line code, and the chain of round r + 1 (which needs only the positions) is
// issued in the same basic block as the entry decode of round r (which needs nothing of the next
// chain), so the decode's instructions fill the chain's LDS-latency gaps instead of following
// them (ZL batch 18.5K -> 16.7K cycles).  The last round walks one wasted chain (clamped at entry
// 0).  (Measured dead ends: two lanes per value walking from both ends, 2 or 4 entries per lane
// per round, R rounds of the chain blocked into registers before R decodes.)
template <uint32_t G, class Src>
__device__ __forceinline__ bool do_ziplist_bp(const Src &R, const Lane &l, bool active, uint32_t g, uint32_t &n,
                                              uint64_t &pay) {
    const uint32_t zl0 = l.q + 13, zend = l.q + l.L, zlast = zend - 1;   // zlast: the 0xFF byte
    const uint32_t first = zl0 + 10;                                     // entry 0
    uint32_t z[3];
    R.template get<3>(zl0, z);   // zlbytes, zltail, zllen
    const uint32_t N = active && (z[2] & 0xFFFF) != 0xFFFF ? z[2] & 0xFFFF : 0u;
    const uint32_t endbyte = R.template fetch<1>(zlast).w[0];   // (aligned dword holding zlast)
    put_desc(l.E, active && g == 0 ? l.slot(0) : NOSLOT, l.B + zl0, l.L - 13, RR_K_ZLRAW, 0);
    pay += active && g == 0 ? l.L - 13 : 0;
    bool fail = active && (z[2] & 0xFFFF) == 0xFFFF;   // saturated count: the exact parser walks it
    uint32_t p = zl0 + z[1];
    p = p < first ? first : p > zlast ? zlast : p;
    uint32_t expect = zlast;   // where the entry at p must end
    // one round's chain: G backward steps; this lane keeps step g's entry (mp) and its end (me)
    auto chain = [&](uint32_t &mp, uint32_t &me) __attribute__((always_inline)) {
        mp = first;
        me = zlast;
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) {
            // prevlen: its first byte by a byte read, the u32 of a 5-byte prevlen by a dword
            // read issued beside it (off the common path's dependency chain; an aligned pair +
            // alignbyte measured ZL batch 16.9K vs 16.3K cycles)
            const uint32_t b0 = R.u8b(p);
            const uint32_t pb = R.u32(p + 1);
            const uint32_t pl = b0 >= 254 ? pb : b0;
            const uint32_t pn = p - min(pl, p - first);
            mp = j == g ? p : mp;
            me = j == g ? expect : me;
            expect = p;
            p = pn;
        }
    };
    // the entry decode and its checks (index idx = N-1-mk)
    auto decode = [&](uint32_t mk, uint32_t mp, uint32_t me) __attribute__((always_inline)) {
        const bool mine = mk < N;
        const uint32_t idx = N - 1 - mk;
        uint32_t b[4];
        R.template get<4>(mp, b);
        const uint32_t b0 = b[0] & 0xFF;
        const bool big = b0 >= 254;
        const uint32_t pl = big ? ab(b[1], b[0], 1) : b0;
        const uint32_t qp = mp + (big ? 5u : 1u);
        const uint32_t e = big ? (b[1] >> 8) & 0xFF : (b[0] >> 8) & 0xFF;
        const uint32_t x1 = big ? (b[1] >> 16) & 0xFF : (b[0] >> 16) & 0xFF;
        const uint32_t lo = big ? ab(b[2], b[1], 2) : ab(b[1], b[0], 2);
        const uint32_t hi = big ? ab(b[3], b[2], 2) : ab(b[2], b[1], 2);
        const bool zstr = e < 0xC0;
        const uint32_t scls = e >> 6;
        const uint32_t ls = 1 + scls + 2 * (scls >> 1);
        const uint32_t sl1 = scls == 0 ? (e & 0x3F) : (((e & 0x3F) << 8) | x1);
        const uint32_t sl = scls >= 2 ? __builtin_bswap32(lo) : sl1;
        const bool imm = e - 0xF1u <= 0xFDu - 0xF1u;
        const uint32_t isz = (e & 0x0F) == 0 && e >= 0xC0 ? (0x3842u >> (4 * ((e >> 4) & 3))) & 0xF
                                                           : (uint32_t)(e == 0xFE);
        const uint64_t endp = (uint64_t)qp + (zstr ? ls + sl : 1 + isz);
        const bool bad = (mp < first) | (mp >= zlast) | (b0 == 0xFF) | (big & (mp + 5 > zlast)) | (qp >= zlast) |
                         (idx + 1 >= l.r) | (!zstr & !imm & (isz == 0)) | (zstr & (qp + ls > zlast)) |
                         (endp != (uint64_t)me) | (idx == 0 ? ((mp != first) | (pl != 0)) : (pl > mp - first));
        fail |= mine & bad;
        const uint32_t sh = (32 - 8 * isz) & 31;
        const int64_t v32 = (int32_t)(lo << sh) >> sh;
        const int64_t iv = isz == 8 ? (int64_t)((uint64_t)lo | ((uint64_t)hi << 32)) : imm ? (int64_t)(e & 0x0F) - 1 : v32;
        put_desc(l.E, (mine & !bad) ? l.slot(idx + 1) : NOSLOT, zstr ? l.B + qp + ls : (uint64_t)iv, zstr ? sl : 0,
                 zstr ? RR_K_STR : RR_K_INT, zstr ? (e & 0xC0) : e);
    };
    uint32_t mpA, meA;
    chain(mpA, meA);
    for (uint32_t rounds = 0;; ++rounds) {
        uint32_t mpB, meB;
        chain(mpB, meB);   // round + 1's chain ...
        decode(rounds * G + g, mpA, meA);   // ... beside round's decode
        if (__ballot((rounds + 1) * G < N) == 0) break;
        mpA = mpB;
        meA = meB;
    }
    const uint32_t base = lane_id() - g;
    const uint64_t gm = (G >= 64 ? ~0ull : ((1ull << G) - 1)) << base;
    const bool gfail = (__ballot(fail) & gm) != 0;
    const uint32_t zllen = z[2] & 0xFFFF;
    const bool ok = !gfail && (zllen & 1) == 0 && (endbyte >> (8 * (zlast & 3)) & 0xFF) == 0xFF &&
                    (zllen > 0 || (z[1] == 10 && first == zlast));
    n = 1 + zllen;
    return !ok || n != l.r;
}

}  // namespace rr
