// rr_snappy.hip — snappy raw-format compression / decompression of RocksDB data blocks on
// gfx950 (include/rr_snappy.h).
//
// One wave per block for both directions: snappy's format is a chain (every tag's size decides
// where the next one starts; the compressor's hash table is updated probe by probe), so a block
// is a serial walk, and the wave's 64 lanes work inside each step — the copy of a literal or a
// back-reference, the extension of a match, the staging of the block into LDS.  Parallelism
// comes from many blocks in flight.
//
//   snz_len_kernel    thread per block: the varint32 length preamble -> out_offs[i] (then the
//                     engine's look-back scan turns the lengths into packed offsets)
//   snz_dec_kernel    wave per block: the compressed bytes through a 1 KiB register window
//                     (16 B per lane, uniform tag parsing by readlane), the output assembled
//                     in LDS and written out once; a block longer than the LDS window is
//                     decompressed straight into global memory (copies then read their
//                     sources back through the L2 after the wave's stores drained)
//   snz_comp_kernel   wave per block: snappy 1.1.8's CompressFragment (oracle/rr_snappy.c
//                     cites the lines) on a uniform control path, with the fragment and its
//                     16K-entry hash table in LDS; output to a per-block slot
//   snz_pack_kernel   wave per block: slots -> packed output
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rr_kernels.h"
#include "../../include/rr_snappy.h"

namespace {

constexpr uint32_t WAVE = 64;
constexpr uint32_t FRAG = 1u << 16;        // snappy kBlockSize (snappy.h:197-198)
constexpr uint32_t TAB_MIN = 1u << 8;      // kMinHashTableSize
constexpr uint32_t TAB_MAX = 1u << 14;     // kMaxHashTableSize
constexpr uint32_t MARGIN = 15;            // kInputMarginBytes
// LDS window per wave (the block decompressed in place in it): RocksDB blocks are cut at ~16 KiB
// (block_size, rocksdbapi.cc:77) plus at most one entry; 18 KiB holds those up to a 2 KiB last
// entry with 8 waves per CU (20 KiB: 7 waves, 11 % slower on config 4; 17.5 KiB: 9 waves, +3 %
// more but 1.5 KiB of room), and a longer block decompresses straight into global memory
#ifndef RR_SNZ_DEC_WIN
#define RR_SNZ_DEC_WIN 18432
#endif
constexpr uint32_t SNZ_DEC_WIN = RR_SNZ_DEC_WIN;
// staged fragment bytes per wave; 0 (default): the compressor reads its input in place through
// the buffer resource, so a wave holds only the 32 KiB hash table (5 waves per CU instead of 3;
// 18432 measured configs 4 / 3 5 % slower, config 2 +33 %: profiles/r5_snappy_compress_literal_ab.txt)
#ifndef RR_SNZ_FRAG
#define RR_SNZ_FRAG 0
#endif
constexpr uint32_t SNZ_FRAG_LDS = RR_SNZ_FRAG;
// the decompressor's tag chain through speculative tag sizes at 64 * RR_SNZ_SPEC positions (1,
// 2 or 4 a lane; a readlane a tag); 0: one LDS read a tag
#ifndef RR_SNZ_SPEC
#define RR_SNZ_SPEC 1
#endif

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
// LDS pointers kept in address space 3, so accesses compile to ds_* (a generic pointer gives flat_*
// instructions, whose waits also drain every outstanding global store of the wave)
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ rsrc_t mkr(const void *base, uint64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)(bytes < 0x7FFFFFF0ull ? bytes : 0x7FFFFFF0ull),
                                             0x00020000);
}
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// ---- decompression ------------------------------------------------------------------------
#ifdef RR_PROBE
// Decompress probe (diagnostics; tools/probe_snappy.py): cycles (s_memtime) per phase summed over
// the call's LDS-path blocks: stage, A (tag chain), B (tag decode + checks), literals,
// back-references, output; [6] blocks, [7] batches, [8] tags
__device__ unsigned long long g_snz_probe[9];
extern "C" int rr_snz_probe_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_snz_probe), sizeof(g_snz_probe)) == hipSuccess ? 0 : -1;
}
extern "C" int rr_snz_probe_reset() {
    static const unsigned long long z[9] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_snz_probe), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
__device__ __forceinline__ uint64_t snz_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define SNZP(...) __VA_ARGS__
#else
#define SNZP(...)
#endif
__global__ __launch_bounds__(256) void snz_len_kernel(const uint8_t *__restrict__ in,
                                                      const uint64_t *__restrict__ in_offs, uint64_t n,
                                                      uint64_t *__restrict__ out_offs, uint8_t *__restrict__ status,
                                                      uint64_t *__restrict__ lb, uint32_t lbw) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < lbw) lb[i] = 0;
    if (i < n) {
        const uint64_t c0 = in_offs[i], c1 = in_offs[i + 1];
        uint32_t v = 0, shift = 0;
        bool ok = false;
        for (uint64_t k = c0; k < c1 && shift < 32; ++k, shift += 7) {   // ReadUncompressedLength
            const uint32_t c = in[k], val = c & 0x7F;
            if (shift == 28 && val >= 16) break;
            v |= val << shift;
            if (c < 128) { ok = true; break; }
        }
        out_offs[i] = ok ? v : 0;
        status[i] = ok ? RR_SNAPPY_OK : RR_SNAPPY_E_HEADER;
    } else if (i == n) {
        out_offs[n] = 0;
    }
}

// The compressed block through a register window: lane l holds bytes [wb + 16 l, wb + 16 l + 16)
// of the block's buffer resource (positions q relative to it), 1 KiB in all.  (A second KiB
// loaded ahead, the window sliding by 1 KiB as the parse passes it, measured 17 % slower.)
struct Win {
    rsrc_t R;
    uint32_t wb;
    uint32_t x[4];
    static constexpr uint32_t SPAN = 1024;
    __device__ __forceinline__ void load(uint32_t at) {
        wb = at & ~15u;
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(R, (int)(wb + 16 * lane_id()), 0, 0);
        x[0] = v[0]; x[1] = v[1]; x[2] = v[2]; x[3] = v[3];
    }
    // keep p (+ 8 bytes) inside the window
    __device__ __forceinline__ void track(uint32_t p) {
        if (p + 8 > wb + SPAN) load(p);
    }
    // the aligned dword at q (q - wb < SPAN, q % 4 == 0), uniform
    __device__ __forceinline__ uint32_t dw(uint32_t q) const {
        const uint32_t r = q - wb, k = (r >> 2) & 3;
        const uint32_t v = k == 0 ? x[0] : k == 1 ? x[1] : k == 2 ? x[2] : x[3];
        return rdl(v, r >> 4);
    }
    // 5+ bytes starting at q (uniform), low byte first
    __device__ __forceinline__ uint64_t bytes(uint32_t q) const {
        const uint32_t a = q & ~3u;
        const uint64_t v = (uint64_t)dw(a) | ((uint64_t)dw(a + 4) << 32);
        return v >> (8 * (q & 3));
    }
};

__device__ __forceinline__ void wait_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// wave64 inclusive scan (u32) in DPP: row shifts within each 16-lane row, then the rows' last
// lanes carried up by row_bcast:15 / row_bcast:31 (as rr_device.h's wave_incl_scan_u32)
__device__ __forceinline__ uint32_t scan_u32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

// lane mod off for off <= 64: (lane + 0.5) / off is at least 1 / 129 away from an integer, far
// beyond v_rcp_f32's error, so the truncated product is the exact quotient
__device__ __forceinline__ uint32_t lane_mod(uint32_t lane, uint32_t off) {
    const uint32_t k = (uint32_t)(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)off));
    return lane - k * off;
}

// wave64 max (u32): the DPP scan's shape with max, read at the last lane
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
    return rdl(x, WAVE - 1);
}

// Byte copies inside the LDS window, a lane each (lanes with `mine`): l bytes from s to d, 16 a
// round (five aligned source dwords, realigned, then the bytes), every lane's reads of a round
// before its writes.  The caller guarantees no copy of the set reads bytes another one writes.
__device__ __forceinline__ void lane_copies(lds_u8 *win, bool mine, uint32_t s, uint32_t d, uint32_t l) {
    lds_u32 *win32 = (lds_u32 *)win;
    for (uint32_t r = 0; __ballot(mine && r < l); r += 16) {
        const bool a = mine && r < l;
        const uint32_t q = s + r, qa = a ? q >> 2 : 0u, sh = q & 3;
        const uint32_t x0 = win32[qa], x1 = win32[qa + 1], x2 = win32[qa + 2], x3 = win32[qa + 3], x4 = win32[qa + 4];
        const uint32_t w[4] = {__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                               __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
        const uint32_t nb = a ? (l - r < 16 ? l - r : 16u) : 0u;
        // destination-aligned: up to 3 head bytes, whole dwords (the stream realigned by the head),
        // up to 3 tail bytes — at most 10 LDS writes instead of 16 byte writes
        const uint32_t dst = d + r, h0 = (4u - (dst & 3)) & 3, h = h0 < nb ? h0 : nb;
        const uint32_t fd = (nb - h) >> 2, tl = (nb - h) & 3;
#pragma unroll
        for (uint32_t i = 0; i < 3; ++i)
            if (i < h) win[dst + i] = (uint8_t)(w[0] >> (8 * i));
        lds_u32 *dd = (lds_u32 *)(win + ((dst + h) & ~3u));
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (k < fd) dd[k] = __builtin_amdgcn_alignbyte(k + 1 < 4 ? w[k + 1] : 0u, w[k], h);
        const uint32_t lo = fd == 0 ? w[0] : fd == 1 ? w[1] : fd == 2 ? w[2] : w[3];
        const uint32_t hi = fd == 0 ? w[1] : fd == 1 ? w[2] : fd == 2 ? w[3] : 0u;
        const uint32_t T = __builtin_amdgcn_alignbyte(hi, lo, h);
#pragma unroll
        for (uint32_t i = 0; i < 3; ++i)
            if (i < tl) win[dst + h + 4 * fd + i] = (uint8_t)(T >> (8 * i));
    }
}

// Tag decoding shared by both paths (snappy.cc:808 DecompressAllTags, oracle/rr_snappy.c):
// t holds the 5+ bytes from the tag on (uniform).  Literals: hdr = 1 + extra length bytes,
// len = the literal's bytes; copies: hdr = 1 + offset bytes, len / off of the back-reference.
struct Tag {
    uint32_t hdr, len, off;
    bool lit;
};
__device__ __forceinline__ Tag decode_tag(uint64_t t) {
    const uint32_t c = (uint32_t)t & 0xFF, ty = c & 3, v = (uint32_t)(t >> 8);
    Tag g;
    g.lit = ty == 0;
    if (g.lit) {
        g.len = (c >> 2) + 1;
        g.hdr = 1;
        g.off = 0;
        if (g.len >= 61) {
            const uint32_t nb = g.len - 60;
            g.len = (nb == 4 ? v : v & ((1u << (8 * nb)) - 1)) + 1;   // (0: 2^32 wrapped)
            g.hdr += nb;
        }
    } else {
        const uint32_t nb = ty == 1 ? 1u : ty == 2 ? 2u : 4u;
        g.hdr = 1 + nb;
        g.len = ty == 1 ? 4 + ((c >> 2) & 7) : (c >> 2) + 1;
        g.off = ty == 1 ? ((c >> 5) << 8) | (v & 0xFF) : ty == 2 ? v & 0xFFFF : v;
    }
    return g;
}

// A block whose output fits the LDS window, decompressed in place: the compressed bytes staged
// at the window's end with every load in flight (one round trip), the output assembled from the
// window's start, every later read from LDS.  Two phases per batch of up to 64 tags:
//   A. the tag chain, serially and lean: each tag's size from its first bytes (one LDS read and a
//      dozen scalar instructions), its start written into lane k of a VGPR;
//   B. the batch's 64 tags decoded at once, one per lane (VALU), their output positions by a
//      wave scan, every check of the serial decoder per lane (the first failing tag's verdict is
//      the block's); then the literals copied, then the back-references in stream order (a
//      back-reference reads only output before its own position: earlier literals and earlier
//      back-references).
// Each tag's writes stay below the compressed bytes not yet read — a literal's destination at
// least 8 bytes below its source, a back-reference's end below the next tag — else the block
// bails out (*bail) to the global path.
//   R: the block's dwords from its 4-aligned base, s0 + clen bytes (s0: the block's first byte);
//   returns the status (RR_SNAPPY_*) with the output in win[0, expected).
__device__ uint32_t dec_block_lds(rsrc_t R, uint32_t s0, uint32_t clen, uint32_t expected, lds_u8 *win, uint32_t wcap,
                                  bool &bail) {
    lds_u32 *win32 = (lds_u32 *)win;
    typedef __attribute__((address_space(3))) u32x4_t lds_u32x4;
    const uint32_t lane = lane_id(), end = s0 + clen, ng = (end + 15) >> 4;
    const uint32_t D = wcap + 16 - 16 * ng;   // (the allocation's last 16 bytes: reads past the end)
    SNZP(uint64_t pt = snz_stamp(), pa = 0, pb = 0, pl = 0, pc = 0, nbat = 0, ntag = 0; const uint64_t p0 = pt;)
    {
        constexpr uint32_t SG = (SNZ_DEC_WIN + 16) / 16 / WAVE + 1;
        u32x4_t g[SG];
#pragma unroll
        for (uint32_t j = 0; j < SG; ++j) g[j] = __builtin_amdgcn_raw_buffer_load_b128(R, (int)(16 * (lane + WAVE * j)), 0, 0);
        lds_u32x4 *d4 = (lds_u32x4 *)(win + D);
#pragma unroll
        for (uint32_t j = 0; j < SG; ++j)
            if (lane + WAVE * j < ng) d4[lane + WAVE * j] = g[j];
    }
    // 8 bytes at LDS address a (uniform; two dwords, in SGPRs)
    auto rd8 = [&](uint32_t a) __attribute__((always_inline)) -> uint64_t {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)win32[a >> 2]);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)win32[(a >> 2) + 1]);
        return (((uint64_t)hi << 32) | lo) >> (8 * (a & 3));
    };
    uint32_t p = s0;
    {
        uint64_t t = rd8(D + p);
        while (t & 0x80) { ++p; t >>= 8; }   // the preamble (validated by snz_len_kernel: <= 5 bytes)
        ++p;
    }
    uint32_t pos = 0;
    SNZP(uint64_t pst; { const uint64_t t = snz_stamp(); pst = t - p0; pt = t; })
    while (p < end) {
        // A. up to 64 tag starts.  The size a tag would have at each of the 64 * PP positions from
        //    p on (PP a lane, speculatively: one LDS round trip and a few VALU ops), then the chain
        //    through them by readlanes — a few cycles a tag instead of an LDS round trip; a tag
        //    that lands past those positions (a long literal) starts the next round.
        uint32_t tp = 0, nt = 0;
#if RR_SNZ_SPEC
        constexpr uint32_t PP = RR_SNZ_SPEC;   // positions a lane
        static_assert(PP == 1 || PP == 2 || PP == 4, "positions a lane");
        do {
            const uint32_t wp = p, ab = (D + wp) & ~3u, bo = ((D + wp) & 3u) + PP * lane;
            const uint32_t di = (ab >> 2) + (bo >> 2), bs = bo & 3;
            const uint32_t w0 = win32[di], w1 = win32[di + 1], w2 = PP > 1 ? win32[di + 2] : 0u;   // (one position: 8 bytes hold it)
            const uint64_t x01 = ((uint64_t)w1 << 32) | w0, x12 = ((uint64_t)w2 << 32) | w1;
            uint32_t sp[(PP + 1) / 2];
#pragma unroll
            for (uint32_t j = 0; j < PP; ++j) {
                if (PP <= 2) {   // (32-bit: the tag byte and the 4 bytes after it by alignbyte, len - 1)
                    const uint32_t o = bs + j;   // (0 .. 4)
                    const uint32_t c = (o < 4 ? __builtin_amdgcn_alignbyte(w1, w0, o) : w1) & 0xFF, ty = c & 3, c6 = (c >> 2) + 1;
                    const uint32_t v = o < 3 ? __builtin_amdgcn_alignbyte(w1, w0, o + 1) : o == 3 ? w1 : __builtin_amdgcn_alignbyte(w2, w1, 1);
                    const uint32_t q = wp + PP * lane + j, nb = c6 > 60 ? c6 - 60 : 0u;
                    const uint32_t lm1 = nb ? (nb == 4 ? v : v & ((1u << (8 * nb)) - 1)) : c6 - 1;
                    const uint32_t lsz = q >= end ? 1u : lm1 >= end - q - 1 ? end - q + 1 : 2 + nb + lm1;   // (past the end: phase B's TRUNC)
                    const uint32_t sz = ty == 0 ? lsz : ty == 1 ? 2u : ty == 2 ? 3u : 5u;
                    if (PP == 1) sp[0] = sz;
                    else if (j & 1) sp[j >> 1] |= sz << 16;
                    else sp[j >> 1] = sz & 0xFFFF;
                    continue;
                }
                const uint32_t o = bs + j;   // (0 .. 6: the position's bytes from the lane's three dwords)
                const uint64_t t = o < 4 ? x01 >> (8 * o) : x12 >> (8 * (o - 4));
                const uint32_t q = wp + PP * lane + j, c = (uint32_t)t & 0xFF, ty = c & 3, c6 = (c >> 2) + 1;
                const uint32_t nb = c6 > 60 ? c6 - 60 : 0u, v = (uint32_t)(t >> 8);
                const uint64_t len = nb ? (uint64_t)(nb == 4 ? v : v & ((1u << (8 * nb)) - 1)) + 1 : c6;
                const uint32_t rem = q < end ? end - q : 0u;
                const uint32_t lsz = len >= rem ? rem + 1 : (uint32_t)(1 + nb + len);   // (past the end: phase B's TRUNC)
                const uint32_t sz = ty == 0 ? lsz : ty == 1 ? 2u : ty == 2 ? 3u : 5u;
                if (PP == 1) sp[0] = sz;
                else if (j & 1) sp[j >> 1] |= sz << 16;
                else sp[j >> 1] = sz & 0xFFFF;
            }
            // (sizes past 16 bits only on the last tag: rem + 1 <= the block's bytes < 2^16, or
            //  a literal as long as the rest, which ends the block's chain either way)
            do {
                const uint32_t r = p - wp, l = r / PP, j = r % PP;
                uint32_t v = sp[0];
#pragma unroll
                for (uint32_t k = 1; k < (PP + 1) / 2; ++k) v = (j >> 1) == k ? sp[k] : v;
                const uint32_t pair = rdl(v, l);
                const uint32_t sz = PP == 1 ? pair : (j & 1) ? pair >> 16 : pair & 0xFFFF;
                tp = lane == nt ? p : tp;
                ++nt;
                p += sz;
            } while (nt < WAVE && p < end && p - wp < PP * WAVE);
        } while (nt < WAVE && p < end);
#else
        do {
            const uint64_t t = rd8(D + p);
            const uint32_t c = (uint32_t)t & 0xFF, ty = c & 3, c6 = (c >> 2) + 1;
            uint32_t sz;
            if (ty == 0) {
                const uint32_t nb = c6 > 60 ? c6 - 60 : 0u;
                const uint64_t len = nb ? ((t >> 8) & ((1ull << (8 * nb)) - 1)) + 1 : c6;
                sz = len > end - p ? end - p + 1 : (uint32_t)(1 + nb + len);   // (past the end: phase B's TRUNC)
            } else {
                sz = ty == 1 ? 2u : ty == 2 ? 3u : 5u;
            }
            tp = lane == nt ? p : tp;
            ++nt;
            p += sz;
        } while (nt < WAVE && p < end);
#endif
        SNZP({ const uint64_t t = snz_stamp(); pa += t - pt; pt = t; ++nbat; ntag += nt; })
        // B. the batch's tags, one per lane
        const bool act = lane < nt;
        const uint32_t a = D + (act ? tp : 0);
        const uint32_t lo = win32[a >> 2], hi = win32[(a >> 2) + 1], sh = a & 3;
        const uint32_t b0 = __builtin_amdgcn_alignbyte(hi, lo, sh);
        const uint32_t v = sh == 3 ? hi : __builtin_amdgcn_alignbyte(hi, lo, sh + 1);   // the 4 bytes after the tag byte
        const uint32_t c = b0 & 0xFF, ty = c & 3, c6 = (c >> 2) + 1;
        const bool lit = ty == 0;
        const uint32_t nb = lit ? (c6 > 60 ? c6 - 60 : 0u) : ty == 3 ? 4u : ty;
        const uint32_t vv = nb >= 4 ? v : v & ((1u << (8 * nb)) - 1);
        const uint32_t len = lit ? (nb ? vv + 1 : c6) : ty == 1 ? 4 + ((c >> 2) & 7) : c6;   // (0: 2^32 wrapped)
        const uint32_t off = ty == 1 ? ((c >> 5) << 8) | vv : vv;
        const uint32_t tq = tp + 1 + nb;   // the literal's bytes / the next tag
        const uint32_t tpn = lit ? tq + len : tq;
        // output positions: the exclusive scan of the lengths (each clamped past `expected`: a
        // longer one fails its check whatever the scan says)
        const uint32_t ol = act ? (len < expected + 1 ? len : expected + 1) : 0u;
        const uint32_t tpos = pos + scan_u32(ol) - ol;
        // the serial decoder's checks, in its order (0 = none, 4 = bail out)
        uint32_t code = 0;
        if (act) {
            if (tq > end) code = RR_SNAPPY_E_TRUNC;
            else if (lit) code = len == 0 || len > end - tq ? RR_SNAPPY_E_TRUNC : len > expected - tpos ? RR_SNAPPY_E_OVERFLOW
                                 : D + tq < tpos + 8 ? 0xFFu : 0u;
            else code = off == 0 || off > tpos ? RR_SNAPPY_E_OFFSET : len > expected - tpos ? RR_SNAPPY_E_OVERFLOW
                        : tpos + len > D + tpn ? 0xFFu : 0u;
        }
        const uint64_t badm = __ballot(code != 0);
        SNZP({ const uint64_t t = snz_stamp(); pb += t - pt; pt = t; })
        if (badm) {
            const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)code, (int)__builtin_ctzll(badm));
            if (f == 0xFFu) bail = true;
            return f == 0xFFu ? RR_SNAPPY_OK : f;
        }
        // the literals.  When every literal destination of the batch (and the up to 3 bytes a
        // long literal's last dword spills past its end) lies below every literal source (the
        // usual case: the compressed bytes sit at the window's end, far above the output), the
        // literals longer than 64 bytes go first, one after the other by the whole wave, then the
        // others together, a lane each (exact bytes: they land after any spill into them, and no
        // copy reads what another writes); otherwise all of them one after the other
        const bool islit = act && lit;
        uint64_t m = __ballot(islit);
        const bool par = m && wave_max_u32(islit ? tpos + len + 4 : 0u) <= ~wave_max_u32(islit ? ~(D + tq) : 0u);
        if (par) m = __ballot(islit && len > WAVE);
        while (m) {
            const int k = (int)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t dpos = (uint32_t)__builtin_amdgcn_readlane((int)tpos, k);
            const uint32_t src = D + (uint32_t)__builtin_amdgcn_readlane((int)tq, k);
            const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)len, k);
            if (l <= WAVE) {
                const uint8_t x = lane < l ? win[src + lane] : 0;
                if (lane < l) win[dpos + lane] = x;
            } else {
                // bytes to a 4-aligned destination, then 16 bytes per lane from five aligned
                // source dwords (the last dword may spill up to 3 bytes past the literal, below
                // its source: overwritten by a later element before anything reads them); the
                // head bytes are read with the first chunk and written with it (one LDS round trip)
                const uint32_t h = (4u - (dpos & 3)) & 3;
                const uint8_t hx = lane < h ? win[src + lane] : 0;
                const uint32_t d0 = dpos + h, q0 = src + h, body = l - h, a0 = q0 & ~3u, s3 = q0 & 3;
                uint32_t i = 0;
                do {   // (body > 60: at least one chunk)
                    const uint32_t k4 = i + 16 * lane, sa = k4 < body ? (a0 + k4) >> 2 : 0u;   // (idle lanes: word 0)
                    const uint32_t x0 = win32[sa], x1 = win32[sa + 1], x2 = win32[sa + 2], x3 = win32[sa + 3], x4 = win32[sa + 4];
                    if (i == 0 && lane < h) win[dpos + lane] = hx;
                    lds_u32 *w = win32 + ((d0 + k4) >> 2);
                    if (k4 < body) w[0] = __builtin_amdgcn_alignbyte(x1, x0, s3);
                    if (k4 + 4 < body) w[1] = __builtin_amdgcn_alignbyte(x2, x1, s3);
                    if (k4 + 8 < body) w[2] = __builtin_amdgcn_alignbyte(x3, x2, s3);
                    if (k4 + 12 < body) w[3] = __builtin_amdgcn_alignbyte(x4, x3, s3);
                    i += 16 * WAVE;
                } while (i < body);
            }
        }
        if (par) lane_copies(win, islit && len <= WAVE, D + tq, tpos, len);
        SNZP({ const uint64_t t = snz_stamp(); pl += t - pt; pt = t; })
        // the back-references: those that do not overlap themselves and read only output before
        // the batch's first back-reference (final once the literals are in) together, a lane
        // each; then the others in stream order: out[pos + j] = out[pos - off + j % off]
        const bool iscop = act && !lit;
        m = __ballot(iscop);
        if (m) {
            const uint32_t c0 = rdl(tpos, (uint32_t)__builtin_ctzll(m));
            const bool indep = iscop && off >= len && tpos - off + len <= c0;
            lane_copies(win, indep, tpos - off, tpos, len);
            m = __ballot(iscop && !indep);
        }
        while (m) {
            const int k = (int)__builtin_ctzll(m);
            m &= m - 1;
            const uint32_t dpos = (uint32_t)__builtin_amdgcn_readlane((int)tpos, k);
            const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)off, k);
            const uint32_t l = (uint32_t)__builtin_amdgcn_readlane((int)len, k);
            const uint32_t j = o < l ? lane_mod(lane, o) : lane;
            const uint8_t x = lane < l ? win[dpos - o + j] : 0;
            if (lane < l) win[dpos + lane] = x;
        }
        pos = (uint32_t)__builtin_amdgcn_readlane((int)(tpos + ol), (int)(nt - 1));
        SNZP({ const uint64_t t = snz_stamp(); pc += t - pt; pt = t; })
    }
    SNZP(if (lane == 0) {
        atomicAdd(&g_snz_probe[0], (unsigned long long)pst); atomicAdd(&g_snz_probe[1], (unsigned long long)pa);
        atomicAdd(&g_snz_probe[2], (unsigned long long)pb); atomicAdd(&g_snz_probe[3], (unsigned long long)pl);
        atomicAdd(&g_snz_probe[4], (unsigned long long)pc); atomicAdd(&g_snz_probe[6], 1ull);
        atomicAdd(&g_snz_probe[7], (unsigned long long)nbat); atomicAdd(&g_snz_probe[8], (unsigned long long)ntag);
    })
    return pos == expected ? RR_SNAPPY_OK : RR_SNAPPY_E_LENGTH;
}

// A block past the LDS window (or one that bailed out of it): the compressed bytes through a
// register window, the output straight into global memory (a back-reference reads its source
// back through the L2 once the wave's earlier stores have drained).
__device__ uint32_t dec_block_global(rsrc_t R, uint32_t s0, uint32_t clen, uint32_t expected, rsrc_t Ro) {
    const uint32_t lane = lane_id(), end = s0 + clen;
    Win W;
    W.R = R;
    W.load(s0);
    uint32_t p = s0;
    while (W.bytes(p) & 0x80) ++p;   // the preamble (already validated)
    ++p;
    uint32_t pos = 0;
    while (p < end) {
        W.track(p);
        const Tag g = decode_tag(W.bytes(p));
        if (p + g.hdr > end) return RR_SNAPPY_E_TRUNC;
        p += g.hdr;
        if (g.lit) {
            if (g.len == 0 || g.len > end - p) return RR_SNAPPY_E_TRUNC;
            if (g.len > expected - pos) return RR_SNAPPY_E_OVERFLOW;
            for (uint32_t i = 0; i < g.len; i += WAVE) {
                const uint32_t k = i + lane;
                if (k < g.len)
                    __builtin_amdgcn_raw_buffer_store_b8(__builtin_amdgcn_raw_buffer_load_b8(R, (int)(p + k), 0, 0), Ro,
                                                         (int)(pos + k), 0, 0);
            }
            p += g.len;
        } else {
            if (g.off == 0 || g.off > pos) return RR_SNAPPY_E_OFFSET;
            if (g.len > expected - pos) return RR_SNAPPY_E_OVERFLOW;
            uint32_t j = lane;
            if (g.off < g.len) j = lane_mod(lane, g.off);
            wait_stores();   // the wave's earlier output has reached the L2
            const uint8_t x = lane < g.len ? __builtin_amdgcn_raw_buffer_load_b8(Ro, (int)(pos - g.off + j), 0, 17) : 0;
            if (lane < g.len) __builtin_amdgcn_raw_buffer_store_b8(x, Ro, (int)(pos + lane), 0, 0);
        }
        pos += g.len;
    }
    return pos == expected ? RR_SNAPPY_OK : RR_SNAPPY_E_LENGTH;
}

__global__ __launch_bounds__(WAVE) void snz_dec_kernel(const uint8_t *__restrict__ in, uint64_t in_cap,
                                                       const uint64_t *__restrict__ in_offs, uint64_t n,
                                                       uint8_t *__restrict__ out, uint64_t out_cap,
                                                       const uint64_t *__restrict__ out_offs,
                                                       uint8_t *__restrict__ status, uint32_t wcap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    lds_u8 *win = (lds_u8 *)smem;
    lds_u32 *win32 = (lds_u32 *)win;
    const uint32_t lane = lane_id();
    for (uint64_t b = blockIdx.x; b < n; b += gridDim.x) {
        if (status[b] != RR_SNAPPY_OK) continue;   // (the preamble did not parse)
        const uint64_t o0 = out_offs[b], o1 = out_offs[b + 1];
        if (o1 > out_cap) {
            if (lane == 0) status[b] = RR_SNAPPY_E_CAPACITY;
            continue;
        }
        const uint32_t expected = (uint32_t)(o1 - o0);
        const uint64_t c0 = in_offs[b], clen = in_offs[b + 1] - c0;
        const uint32_t s0 = (uint32_t)(c0 & 3);
        const uint64_t base = c0 - s0;   // (whole dwords: the buffer's padding, not past it)
        uint8_t *gout = out + o0;
        const rsrc_t Ro = mkr(gout, expected);
        uint32_t st = RR_SNAPPY_OK;
        bool bail = !(expected <= wcap && ((s0 + clen + 15) & ~15ull) <= wcap);
        if (!bail) {
            const uint64_t span = (s0 + clen + 15) & ~15ull;
            st = dec_block_lds(mkr(in + base, span < in_cap - base ? span : in_cap - base), s0, (uint32_t)clen, expected,
                               win, wcap, bail);
            SNZP(const uint64_t po0 = snz_stamp();)
            if (!bail && st == RR_SNAPPY_OK) {   // LDS -> output: bytes to a 4-aligned address, 16 B per lane, bytes
                const uint32_t g0 = (uint32_t)((uintptr_t)gout & 3), hh = min((4u - g0) & 3, expected);
                const uint32_t t0 = hh + ((expected - hh) & ~3u);
                if (lane < hh) __builtin_amdgcn_raw_buffer_store_b8(win[lane], Ro, (int)lane, 0, 0);
                // five LDS dwords -> four output dwords, one dwordx4 store (output dword-aligned);
                // the last partial group of dwords one at a time
                const uint32_t sh = hh & 3, t16 = hh + ((t0 - hh) & ~15u);
                for (uint32_t j = hh + 16 * lane; j < t16; j += 16 * WAVE) {
                    const uint32_t a = j >> 2;
                    const uint32_t w0 = win32[a], w1 = win32[a + 1], w2 = win32[a + 2], w3 = win32[a + 3], w4 = win32[a + 4];
                    const u32x4_t v = {__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                                       __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
                    __builtin_amdgcn_raw_buffer_store_b128(v, Ro, (int)j, 0, 0);
                }
                for (uint32_t j = t16 + 4 * lane; j < t0; j += 4 * WAVE) {
                    const uint32_t a = j >> 2;
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_alignbyte(win32[a + 1], win32[a], j & 3), Ro, (int)j, 0, 0);
                }
                if (t0 + lane < expected) __builtin_amdgcn_raw_buffer_store_b8(win[t0 + lane], Ro, (int)(t0 + lane), 0, 0);
            }
            SNZP(if (lane == 0) atomicAdd(&g_snz_probe[5], (unsigned long long)(snz_stamp() - po0));)
        }
        if (bail) st = dec_block_global(mkr(in + base, in_cap - base), s0, (uint32_t)clen, expected, Ro);
        if (lane == 0) status[b] = (uint8_t)st;
    }
}

// ---- compression (snappy 1.1.8 CompressFragment; oracle/rr_snappy.c) ------------------------
__device__ __forceinline__ uint32_t log2floor(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }
__device__ __forceinline__ uint32_t table_size(uint32_t fn) {   // CalculateTableSize, snappy.cc:442-455
    return fn > TAB_MAX ? TAB_MAX : fn < TAB_MIN ? TAB_MIN : 2u << log2floor(fn - 1);
}
__device__ __forceinline__ uint32_t hash32(uint32_t v, uint32_t shift) { return (v * 0x1e35a7bdu) >> shift; }

// The fragment's bytes: staged in LDS (ib, at ib[sh + k]) or, when it does not fit, read from
// global memory through the block's buffer resource (at R[g + k]).
struct Frag {
    const lds_u8 *ib;    // LDS stage
    rsrc_t R;
    uint32_t sh, g;
    bool lds;
    __device__ __forceinline__ uint32_t ld32(uint32_t k) const {   // 4 bytes at k, uniform
        if (lds) {
            const uint32_t q = sh + k, a = q & ~3u;
            const uint32_t lo = *reinterpret_cast<const lds_u32 *>(ib + a);
            const uint32_t hi = *reinterpret_cast<const lds_u32 *>(ib + a + 4);
            return __builtin_amdgcn_alignbyte(hi, lo, q & 3);
        }
        const uint32_t q = g + k, a = q & ~3u;
        const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(R, (int)a, 0, 0);
        const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(R, (int)a + 4, 0, 0);
        return __builtin_amdgcn_alignbyte(hi, lo, q & 3);
    }
    __device__ __forceinline__ uint32_t byte(uint32_t k) const {   // per lane
        if (lds) return ib[sh + k];
        return __builtin_amdgcn_raw_buffer_load_b8(R, (int)(g + k), 0, 0);
    }
};

// Output slot writer: uniform op, lanes store bytes.
struct Out {
    rsrc_t R;
    uint32_t op;
    uint32_t mis;   // the slot's address mod 4 (its base is any byte)
    __device__ __forceinline__ void put(uint32_t nbytes, uint64_t v) {   // up to 8 bytes, lanes < nbytes
        const uint32_t l = lane_id();
        if (l < nbytes) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> (8 * l)), R, (int)(op + l), 0, 0);
        op += nbytes;
    }
    __device__ __forceinline__ void literal(const Frag &F, uint32_t from, uint32_t len) {   // EmitLiteral
        const uint32_t n1 = len - 1;
        if (n1 < 60) {
            put(1, n1 << 2);
        } else {
            const uint32_t count = (log2floor(n1) >> 3) + 1;
            put(1 + count, (uint64_t)((59 + count) << 2) | ((uint64_t)n1 << 8));
        }
        // the bytes: a head up to the first 4-aligned destination byte and a tail of < 4 as
        // bytes, the body as aligned destination dwords, 4 a lane a round (1 KiB a wave: one
        // load round trip per KiB instead of one per 64 bytes — an incompressible block is
        // nearly all literal), each from two aligned source loads and an alignbyte
        // (a literal of <= 64 bytes: one byte a lane, one round trip)
        const uint32_t l = lane_id();
        if (len <= WAVE) {
            if (l < len) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)F.byte(from + l), R, (int)(op + l), 0, 0);
            op += len;
            return;
        }
        const uint32_t h = (4u - ((mis + op) & 3u)) & 3u;
        const uint32_t nd = (len - h) >> 2, s = from + h, d = op + h, t = h + 4 * nd;
        // head and tail bytes loaded with the first round's dwords (stores before a load would
        // make its wait cover them too), stored after it
        const uint32_t hb = l < h ? F.byte(from + l) : 0u, tb = l < len - t ? F.byte(from + t + l) : 0u;
        for (uint32_t i = 0; i < nd; i += 4 * WAVE) {
            uint32_t v[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t k = i + j * WAVE + l;
                v[j] = k < nd ? F.ld32(s + 4 * k) : 0u;
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t k = i + j * WAVE + l;
                if (k < nd) __builtin_amdgcn_raw_buffer_store_b32(v[j], R, (int)(d + 4 * k), 0, 0);
            }
        }
        if (l < h) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)hb, R, (int)(op + l), 0, 0);
        if (l < len - t) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)tb, R, (int)(op + t + l), 0, 0);
        op += len;
    }
    __device__ __forceinline__ void copy64(uint32_t offset, uint32_t len, bool allow_short) {   // EmitCopyAtMost64
        if (allow_short && len < 12 && offset < 2048)
            put(2, (uint64_t)(1 + ((len - 4) << 2) + ((offset >> 3) & 0xe0)) | ((uint64_t)(offset & 0xFF) << 8));
        else
            put(3, (uint64_t)(2 + ((len - 1) << 2)) | ((uint64_t)(offset & 0xFFFF) << 8));
    }
    __device__ __forceinline__ void copy(uint32_t offset, uint32_t len) {   // EmitCopy
        if (len < 12) { copy64(offset, len, true); return; }
        while (len >= 68) { copy64(offset, 64, false); len -= 64; }
        if (len > 64) { copy64(offset, 60, false); len -= 60; }
        copy64(offset, len, true);
    }
};

// The compressor's hash table (CompressFragment's `table`, snappy.cc:468-486): ts u16 entries,
// all zero at the fragment's start, table[h] = the last position stored under hash h.
// RR_SNZ_SPARSE = 0 (the default): that dense array, 2 * ts bytes of LDS (32 KiB for a 16 KiB
// block: 5 waves per CU).  Otherwise the same map as an open-addressing table of RR_SNZ_SPARSE u32
// entries ((h + 1) << 16 | position, 0 empty; linear probing from h's low bits): a fragment stores
// only as many hashes as its probes touch — a few hundred for an incompressible 16 KiB block — so
// 16 KiB of LDS holds it and a CU runs twice the waves.  Lookups return what the dense array would
// (0 for a hash never stored); a fragment that would fill more than 3/4 of the entries is
// abandoned (its block goes to a second pass with the dense array), so every output byte is the
// dense compressor's (the snappy suite is bit-exact either way).  Measured, round 6
// (profiles/r6_snappy_sparse_ab.txt): incompressible config 2 247 -> 358 GB/s (4096 entries) /
// 450 (2048), but config 4 33.1 -> 17.9 / 23.9 and config 3 13.9 -> 10.0 / 12.4 GB/s — their
// repeated ziplist fields make copies, each copy restarts the probe schedule at stride 1, so a
// block's table fills (the dense second pass then redoes it) and the probe loops and CAS inserts
// cost more than the doubled occupancy wins.  Not the default.
#ifndef RR_SNZ_SPARSE
#define RR_SNZ_SPARSE 0
#endif
constexpr uint32_t SPT = RR_SNZ_SPARSE, SPT_LIMIT = SPT - SPT / 4;
template <bool SPARSE>
struct HTab {
    lds_u16 *d;   // dense
    lds_u32 *t;   // sparse
    __device__ __forceinline__ uint32_t get(uint32_t h) const {
        if (!SPARSE) return d[h];
        uint32_t i = h & (SPT - 1);
        const uint32_t key = h + 1;
        for (;;) {
            const uint32_t e = t[i];
            if (e == 0) return 0u;
            if ((e >> 16) == key) return e & 0xFFFFu;
            i = (i + 1) & (SPT - 1);
        }
    }
    // table[h] = pos; 1 when this claimed an empty entry.  Lanes storing together hold distinct
    // hashes (the round's last writer of each), or all the same (the uniform steps)
    __device__ __forceinline__ uint32_t put(uint32_t h, uint32_t pos) {
        if (!SPARSE) { d[h] = (uint16_t)pos; return 0u; }
        const uint32_t key = h + 1, nv = (key << 16) | pos;
        uint32_t i = h & (SPT - 1);
        for (;;) {
            const uint32_t e = t[i];
            if (e == 0) {
                uint32_t exp = 0;
                if (__atomic_compare_exchange_n(&t[i], &exp, nv, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) return 1u;
                if ((exp >> 16) == key) { t[i] = nv; return 0u; }   // (a lane of the same store got there first)
            } else if ((e >> 16) == key) {
                t[i] = nv;
                return 0u;
            }
            i = (i + 1) & (SPT - 1);
        }
    }
};

// FindMatchLength: bytes equal at a + i and b + i, for b + i < lim; 64 lanes a step
__device__ __forceinline__ uint32_t match_len(const Frag &F, uint32_t a, uint32_t b, uint32_t lim) {
    const uint32_t l = lane_id();
    for (uint32_t m = 0;; m += WAVE) {
        const uint32_t k = m + l;
        const bool stop = b + k >= lim || F.byte(a + k) != F.byte(b + k);
        const uint64_t bal = __ballot(stop);
        if (bal) return m + (uint32_t)__builtin_ctzll(bal);
    }
}

#ifndef RR_SNZ_K   // most probes a compressor step-1 round evaluates at once (1: the serial loop)
#define RR_SNZ_K 16
#endif
template <bool SPARSE>
__device__ bool compress_fragment(const Frag &F, uint32_t fn, HTab<SPARSE> table, uint32_t ts, Out &O) {
    const uint32_t shift = 32 - log2floor(ts);
    uint32_t ip = 0, next_emit = 0, used = 0;   // used: sparse entries claimed
    auto claimed = [&](uint32_t c) __attribute__((always_inline)) {
        if (SPARSE) used += (uint32_t)__popcll(__ballot(c != 0));
        return SPARSE && used > SPT_LIMIT;
    };
    if (fn >= MARGIN) {
        const uint32_t ip_limit = fn - MARGIN;
        uint32_t next_hash = hash32(F.ld32(++ip), shift);
        for (;;) {
            uint32_t cand;
#if RR_SNZ_K > 1
            // step 1, RR_SNZ_K probes at once: lane j takes the j-th probe the scan would make
            // from here if none before it matched (the skip schedule is known in advance); its
            // candidate is the last earlier lane's position with the same hash, else the table.
            // The first lane that matches (or whose next position passes ip_limit) is where the
            // serial loop stops; the table gets exactly the updates the serial loop makes up to
            // there, the last lane of each hash writing.
            (void)next_hash;
            {
                const uint32_t lane = lane_id();
                uint32_t P0 = ip, S0 = 32, K = RR_SNZ_K < 16 ? RR_SNZ_K : 16;   // (doubling up to RR_SNZ_K while nothing matches)
                for (;;) {
                    uint32_t P = P0, S = S0;
                    if (S0 + K <= 64) {   // the stride is 1 for the whole round (the common case)
                        P = P0 + lane;
                        S = S0 + lane;
                    } else {
                        for (uint32_t t = 0; t + 1 < K; ++t) {
                            const uint32_t B = S >> 5;
                            P = t < lane ? P + B : P;
                            S = t < lane ? S + B : S;
                        }
                    }
                    const uint32_t B = S >> 5, Pn = P + B;
                    const bool act = lane < K;
                    const bool valid = act & (Pn <= ip_limit);
                    const uint32_t x = F.ld32(act ? P : 0);
                    const uint32_t H = hash32(x, shift);
                    int prev = -1;
#if RR_SNZ_K == 16
                    // (one 16-lane DPP row: lane j sees lane j - r by a row shift, no LDS round trip)
                    // (farthest first, so the nearest equal lane is the last to write prev: no
                    // "not found yet" test in the chain)
                    // (H + 1 is never 0, so lanes shifted in from outside the row read 0 by
                    // bound_ctrl and the row shift folds into the compare: v_cmp_eq_u32_dpp)
                    const uint32_t H1 = H + 1;
#define SNZ_ROW_SHR(r) { \
        const uint32_t hk = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)H1, 0x110 + (r), 0xF, 0xF, true); \
        prev = hk == H1 ? (int)lane - (r) : prev; }
                    SNZ_ROW_SHR(15) SNZ_ROW_SHR(14) SNZ_ROW_SHR(13) SNZ_ROW_SHR(12) SNZ_ROW_SHR(11)
                    SNZ_ROW_SHR(10) SNZ_ROW_SHR(9) SNZ_ROW_SHR(8) SNZ_ROW_SHR(7) SNZ_ROW_SHR(6)
                    SNZ_ROW_SHR(5) SNZ_ROW_SHR(4) SNZ_ROW_SHR(3) SNZ_ROW_SHR(2) SNZ_ROW_SHR(1)
#undef SNZ_ROW_SHR
#else
                    for (uint32_t r = 1; r < K; ++r) {
                        const uint32_t hk = (uint32_t)__shfl((int)H, (int)((lane - r) & (WAVE - 1)), WAVE);
                        prev = (prev < 0 && lane >= r && hk == H) ? (int)(lane - r) : prev;
                    }
#endif
                    const uint32_t Pp = (uint32_t)__shfl((int)P, prev < 0 ? (int)lane : prev, WAVE);
                    const uint32_t c = prev >= 0 ? Pp : table.get(act ? H : 0);
                    const bool m = valid && x == F.ld32(c);
                    const uint64_t stop = __ballot(act && (!valid || m));
                    const uint32_t sl = stop ? (uint32_t)__builtin_ctzll(stop) : K;
                    const bool hit = sl < K && ((__ballot(m) >> sl) & 1);
                    const bool commit = act && (lane < sl || (hit && lane == sl));
                    // the table gets each hash's last committing lane: every committing lane
                    // with an earlier same-hash lane tells that lane it was overwritten — a
                    // forward permute through the LDS crossbar, no LDS memory (a lane no one
                    // writes reads 0: tools/micro/permute_probe.hip); the others send to lane
                    // 63, which no round uses (K < 64).  (A 256-byte mark array in LDS held
                    // the compressor at 4 waves per CU: 29.9 -> 30.5 GB/s on config 4.)
                    const bool tell = commit && prev >= 0;
                    const int over = __builtin_amdgcn_ds_permute((tell ? prev : (int)WAVE - 1) * 4, tell ? 1 : 0);
                    uint32_t cl = 0;
                    if (commit && !over) cl = table.put(H, P);
                    if (claimed(cl)) return false;
                    if (sl < K) {
                        if (!hit) goto remainder;
                        ip = rdl(P, sl);
                        cand = rdl(c, sl);
                        break;
                    }
                    P0 = rdl(Pn, K - 1);
                    S0 = rdl(S + B, K - 1);
                    K = K < RR_SNZ_K ? 2 * K : K;
                }
            }
#else
            uint32_t skip = 32, next_ip = ip;
            for (;;) {   // step 1: probe for a 4-byte match
                ip = next_ip;
                const uint32_t h = next_hash;
                const uint32_t between = skip >> 5;
                skip += between;
                next_ip = ip + between;
                if (next_ip > ip_limit) goto remainder;
                next_hash = hash32(F.ld32(next_ip), shift);
                cand = table.get(h);
                if (claimed(table.put(h, ip))) return false;
                if (F.ld32(ip) == F.ld32(cand)) break;
            }
#endif
            O.literal(F, next_emit, ip - next_emit);   // step 2
            uint32_t cur, cbytes;
            do {   // step 3: copies while the next position matches again
                const uint32_t b0 = ip;
                const uint32_t matched = 4 + match_len(F, cand + 4, ip + 4, fn);
                ip += matched;
                O.copy(b0 - cand, matched);
                next_emit = ip;
                if (ip >= ip_limit) goto remainder;
                const uint32_t prev = F.ld32(ip - 1);
                if (claimed(table.put(hash32(prev, shift), ip - 1))) return false;
                cur = F.ld32(ip);
                const uint32_t ch = hash32(cur, shift);
                cand = table.get(ch);
                cbytes = F.ld32(cand);
                if (claimed(table.put(ch, ip))) return false;
            } while (cur == cbytes);
            next_hash = hash32(F.ld32(ip + 1), shift);
            ++ip;
        }
    }
remainder:
    if (next_emit < fn) O.literal(F, next_emit, fn - next_emit);
    return true;
}

// SPARSE: the first pass (sparse tables; a block whose fragment overflows its table gets size
// RR_SNZ_REDO); !SPARSE after it: the dense pass over the blocks marked RR_SNZ_REDO only
// (SPT == 0: the dense pass over every block, the one pass)
constexpr uint64_t RR_SNZ_REDO = ~0ull;
template <bool SPARSE>
__global__ __launch_bounds__(WAVE) void snz_comp_kernel(const uint8_t *__restrict__ in, uint64_t in_cap,
                                                        const uint64_t *__restrict__ in_offs, uint64_t n,
                                                        uint8_t *__restrict__ slots,
                                                        const uint64_t *__restrict__ slot_offs,
                                                        uint64_t *__restrict__ sizes, uint32_t fcap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    HTab<SPARSE> table{(lds_u16 *)sm, (lds_u32 *)sm};
    lds_u8 *ib = (lds_u8 *)sm + (SPARSE ? 4 * SPT : 2 * TAB_MAX);
    const uint32_t lane = lane_id();
    for (uint64_t b = blockIdx.x; b < n; b += gridDim.x) {
        if (!SPARSE && SPT != 0 && sizes[b] != RR_SNZ_REDO) continue;   // (the dense pass: marked blocks only)
        const uint64_t c0 = in_offs[b], len = in_offs[b + 1] - c0;
        const uint32_t s0 = (uint32_t)(c0 & 3);
        Frag F;
        F.R = mkr(in + (c0 - s0), in_cap - (c0 - s0));
        F.ib = ib;
        Out O;
        O.R = mkr(slots + slot_offs[b], slot_offs[b + 1] - slot_offs[b]);
        O.op = 0;
        O.mis = (uint32_t)((uintptr_t)(slots + slot_offs[b]) & 3u);
        {   // varint32 length
            uint32_t v = (uint32_t)len, nb = 1;
            uint64_t enc = 0;
            for (uint32_t k = 0; k < 5; ++k) {
                const uint32_t more = v >= 128;
                enc |= (uint64_t)((v & 0x7F) | (more << 7)) << (8 * k);
                if (!more) { nb = k + 1; break; }
                v >>= 7;
            }
            O.put(nb, enc);
        }
        for (uint64_t f = 0; f < len; f += FRAG) {
            const uint32_t fn = (uint32_t)(len - f < FRAG ? len - f : FRAG);
            const uint32_t ts = table_size(fn);
            if (SPARSE) for (uint32_t k = lane; k < SPT; k += WAVE) table.t[k] = 0;
            else for (uint32_t k = lane; k < ts / 2; k += WAVE) ((lds_u32 *)table.d)[k] = 0;
            F.g = s0 + (uint32_t)f;
            F.sh = (uint32_t)((c0 + f) & 15);
            F.lds = F.sh + fn + 8 <= fcap;
            if (F.lds) {   // aligned granules covering the fragment (+ pad), source alignment kept:
                           // every granule's load in flight at once, then the LDS stores
                constexpr uint32_t SG = SNZ_FRAG_LDS ? (SNZ_FRAG_LDS + 15) / 16 / WAVE + 1 : 1;
                const uint64_t ab = (c0 + f) & ~15ull;
                const rsrc_t RS = mkr(in + ab, in_cap - ab);
                const uint32_t ng = (F.sh + fn + 8 + 15) / 16;
                u32x4_t v[SG];
#pragma unroll
                for (uint32_t k = 0; k < SG; ++k) {
                    const uint32_t q = lane + k * WAVE;
                    v[k] = q < ng ? __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(RS, (int)(16 * q), 0, 0))
                                  : u32x4_t{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (uint32_t k = 0; k < SG; ++k) {
                    const uint32_t q = lane + k * WAVE;
                    if (q < ng) reinterpret_cast<__attribute__((address_space(3))) u32x4_t *>(ib)[q] = v[k];
                }
            }
            if (!compress_fragment<SPARSE>(F, fn, table, ts, O)) {
                O.op = ~0u;   // (abandoned: the dense pass redoes the whole block)
                break;
            }
        }
        if (lane == 0) sizes[b] = O.op == ~0u ? RR_SNZ_REDO : O.op;
    }
}

// A wave per block, four blocks a workgroup.  The packed destination is split at its 16-byte
// boundaries: the head and tail (< 16 bytes each) a byte a lane, the body as aligned 16-byte
// stores from unaligned 16-byte loads of the slot (gfx950 serves an unaligned global load),
// PACK_U loads a lane in flight before their stores.  (Round 5 and before: a byte a lane,
// ~0.9 TB/s of copy; config 2's blocks barely compress, so that was a quarter of its call.)
constexpr uint32_t PACK_WPB = 4, PACK_U = 4;
typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));
__global__ __launch_bounds__(PACK_WPB * WAVE) void snz_pack_kernel(const uint8_t *__restrict__ slots,
                                                                   const uint64_t *__restrict__ slot_offs, uint64_t n,
                                                                   uint8_t *__restrict__ out,
                                                                   const uint64_t *__restrict__ out_offs) {
    const uint32_t lane = lane_id();
    const uint64_t step = (uint64_t)gridDim.x * PACK_WPB;
    for (uint64_t b = (uint64_t)blockIdx.x * PACK_WPB + threadIdx.x / WAVE; b < n; b += step) {
        const uint64_t o0 = out_offs[b], len = out_offs[b + 1] - o0;
        const uint8_t *s = slots + slot_offs[b];
        uint8_t *d = out + o0;
        const uint64_t h0 = (16 - (o0 & 15)) & 15, h = h0 < len ? h0 : len;
        const uint64_t body = (len - h) & ~15ull, t0 = h + body;
        if (lane < h) d[lane] = s[lane];
        if (lane < len - t0) d[t0 + lane] = s[t0 + lane];
        const u32x4_ua *sv = reinterpret_cast<const u32x4_ua *>(s + h);
        u32x4_t *dv = reinterpret_cast<u32x4_t *>(d + h);
        const uint64_t nv = body >> 4;
        for (uint64_t k0 = 0; k0 < nv; k0 += PACK_U * WAVE) {
            u32x4_t v[PACK_U];
#pragma unroll
            for (uint32_t u = 0; u < PACK_U; ++u) {
                const uint64_t k = k0 + u * WAVE + lane;
                if (k < nv) v[u] = sv[k];
            }
#pragma unroll
            for (uint32_t u = 0; u < PACK_U; ++u) {
                const uint64_t k = k0 + u * WAVE + lane;
                if (k < nv) dv[k] = v[u];
            }
        }
    }
}

__global__ __launch_bounds__(256) void snz_bound_kernel(const uint64_t *__restrict__ in_offs, uint64_t n,
                                                        uint64_t *__restrict__ slot_offs, uint64_t *__restrict__ lb,
                                                        uint32_t lbw) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < lbw) lb[i] = 0;
    if (i < n) {
        const uint64_t len = in_offs[i + 1] - in_offs[i];
        slot_offs[i] = 32 + len + len / 6;   // MaxCompressedLength
    } else if (i == n) {
        slot_offs[n] = 0;
    }
}

__global__ __launch_bounds__(256) void snz_sizes_kernel(uint64_t *__restrict__ sizes, uint64_t n,
                                                        uint64_t *__restrict__ lb, uint32_t lbw) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < lbw) lb[i] = 0;
    if (i == n) sizes[n] = 0;
}

uint32_t grid_for(uint64_t n, uint32_t cap) { return (uint32_t)(n < cap ? (n ? n : 1) : cap); }

}  // namespace


extern "C" uint64_t rr_snappy_scratch_words(uint64_t n, uint64_t slot_bytes) {
    return rr_scan_words(n) + 1 + (n + 1) + (slot_bytes + 7) / 8 + 2;
}

// decompression: 3 launches (length preambles, scan, blocks)
extern "C" hipError_t rr_launch_snappy_decompress(const uint8_t *in, uint64_t in_cap, const uint64_t *in_offs, uint64_t n, uint8_t *out,
                                                  uint64_t out_cap, uint64_t *out_offs, uint8_t *status,
                                                  uint64_t *scratch, hipStream_t stream) {
    const uint64_t lbw = rr_scan_words(n);
    uint64_t *lb = scratch, *err = scratch + lbw;
    const uint64_t m = (n + 1 > lbw ? n + 1 : lbw);
    hipLaunchKernelGGL(snz_len_kernel, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, stream, in, in_offs, n, out_offs,
                       status, lb, (uint32_t)lbw);
    hipError_t e = rr_launch_scan_u64(out_offs, n, lb, err, stream);
    if (e != hipSuccess || n == 0) return e != hipSuccess ? e : hipGetLastError();
    hipLaunchKernelGGL(snz_dec_kernel, dim3(grid_for(n, 1u << 20)), dim3(WAVE), SNZ_DEC_WIN + 48, stream, in, in_cap, in_offs, n, out,
                       out_cap, (const uint64_t *)out_offs, status, SNZ_DEC_WIN);
    return hipGetLastError();
}

// compression: bounds + scan -> per-block slots in scratch, blocks, sizes + scan, pack
extern "C" hipError_t rr_launch_snappy_compress(const uint8_t *in, uint64_t in_cap, const uint64_t *in_offs, uint64_t n, uint8_t *out,
                                                uint64_t *out_offs, uint64_t *scratch, uint64_t slot_bytes,
                                                hipStream_t stream) {
    const uint64_t lbw = rr_scan_words(n);
    uint64_t *lb = scratch, *err = scratch + lbw, *slot_offs = err + 1;
    uint8_t *slots = reinterpret_cast<uint8_t *>(slot_offs + n + 1);
    (void)slot_bytes;
    const uint64_t m = (n + 1 > lbw ? n + 1 : lbw);
    const dim3 g((uint32_t)((m + 255) / 256));
    hipLaunchKernelGGL(snz_bound_kernel, g, dim3(256), 0, stream, in_offs, n, slot_offs, lb, (uint32_t)lbw);
    hipError_t e = rr_launch_scan_u64(slot_offs, n, lb, err, stream);
    if (e != hipSuccess) return e;
    if (n && SPT != 0) {   // sparse tables (RR_SNZ_SPARSE), then the dense pass over the blocks they could not hold
        hipLaunchKernelGGL(snz_comp_kernel<true>, dim3(grid_for(n, 1u << 20)), dim3(WAVE), 4 * SPT + SNZ_FRAG_LDS, stream, in,
                           in_cap, in_offs, n, slots, (const uint64_t *)slot_offs, out_offs, SNZ_FRAG_LDS);
        hipLaunchKernelGGL(snz_comp_kernel<false>, dim3(grid_for(n, 2048)), dim3(WAVE), 2 * TAB_MAX + SNZ_FRAG_LDS, stream, in,
                           in_cap, in_offs, n, slots, (const uint64_t *)slot_offs, out_offs, SNZ_FRAG_LDS);
    } else if (n) {
        const uint32_t smem = 2 * TAB_MAX + SNZ_FRAG_LDS;   // (5 waves per CU at the default fragment size)
        hipLaunchKernelGGL(snz_comp_kernel<false>, dim3(grid_for(n, 1u << 20)), dim3(WAVE), smem, stream, in, in_cap, in_offs, n, slots,
                           (const uint64_t *)slot_offs, out_offs, SNZ_FRAG_LDS);
    }
    hipLaunchKernelGGL(snz_sizes_kernel, g, dim3(256), 0, stream, out_offs, n, lb, (uint32_t)lbw);
    e = rr_launch_scan_u64(out_offs, n, lb, err, stream);
    if (e != hipSuccess || n == 0) return e != hipSuccess ? e : hipGetLastError();
    hipLaunchKernelGGL(snz_pack_kernel, dim3(grid_for((n + PACK_WPB - 1) / PACK_WPB, 1u << 20)), dim3(PACK_WPB * WAVE), 0, stream, slots,
                       (const uint64_t *)slot_offs, n, out, (const uint64_t *)out_offs);
    return hipGetLastError();
}
