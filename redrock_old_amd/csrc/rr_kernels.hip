// rr_kernels.hip — CDNA4 (gfx950) decode and encode kernels for RedRock value blobs.
//
// Decode (blob batch -> flat batch): memset + count / scan / decode / finalize launches.
//   count: thread per value, descriptor reservation + walk class; scan: reservations ->
//   elem_base; decode: workgroup per 64 KiB blob window, streams the window into the MIRROR
//   arena (every payload lands at its blob offset) and into LDS, sorts the window's values by
//   class, walks + emits single-class 64-value batches (lane = value).  Details at K1-K4.
// Encode (flat batch -> blob batch): memset + size / scan / index / emit / finalize launches.
//   size: thread per value; scan: sizes -> offsets; index: first value of each 16 KiB output
//   window; emit: workgroup per output window builds the window's bytes in LDS
//   (element-parallel tasks, aligned stores) and stores it coalesced.  Details at E1-E5.
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

// Batch totals: every tile stores its partials {bad, payload, count} with plain stores into
// its own slot; a one-workgroup finalize kernel folds them after the main launch.  (A single
// returning atomic per tile on one word serialises at ~88/us — measured 2.8 ms at 121K tiles.)
__device__ __forceinline__ void tile_stats(uint64_t *stats, uint32_t tile, uint64_t bad, uint64_t pay, uint64_t cnt) {
    if (lane_id() == 0) {
        stats[3 * (uint64_t)tile + 0] = bad;
        stats[3 * (uint64_t)tile + 1] = pay;
        stats[3 * (uint64_t)tile + 2] = cnt;
    }
}

// mode 0 (decode): bytes = offsets[n]; mode 1 (encode): bytes = inclusive prefix of the last
// tile.  Many blocks (one CU reads ~60 GB/s: a single-block fold of 121K tiles took 56 us),
// each folding a slice and adding into *out, which the launcher zeroes first.
// (nblocks: how many of the grid's blocks fold — the decode's post kernel folds in block 0 alone:
// ~500 blocks each adding into the same three words serialised at the memory side)
__device__ __forceinline__ void fold_totals(const uint64_t *__restrict__ stats, uint64_t *state, uint32_t ntiles,
                                            const uint64_t *__restrict__ offsets, uint64_t n, int mode, rr_totals *out,
                                            const uint64_t *__restrict__ extra, uint64_t *err,
                                            uint32_t nblocks = 0xFFFFFFFFu) {
    __shared__ uint64_t red[3][4];
    uint64_t b = 0, p = 0, c = 0;
    const uint32_t nbk = gridDim.x < nblocks ? gridDim.x : nblocks;
    if (blockIdx.x >= nbk) return;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += nbk * blockDim.x) {
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
        if (blockIdx.x == 0) {
            if (extra) {   // decode: {bad, payload} changes of the fixup pass
                atomicAdd((unsigned long long *)&out->n_bad, (unsigned long long)extra[0]);
                atomicAdd((unsigned long long *)&out->payload, (unsigned long long)extra[1]);
            }
            if (mode == 2) {   // decode: descriptor slots = scanned total, bytes = offsets[n]
                out->bytes = offsets[n];
                atomicAdd((unsigned long long *)&out->n_elems, (unsigned long long)state[0]);
            } else
                out->bytes = mode == 0 ? offsets[n] : (ntiles ? (lb_load(&state[ntiles - 1]) & LB_VAL) : 0);
            if (err && lb_load(err)) out->bytes = ~0ull;   // device-side failure: outputs invalid
        }
    }
}

__global__ __launch_bounds__(256) void finalize_kernel(const uint64_t *__restrict__ stats, uint64_t *state,
                                                       uint32_t ntiles, const uint64_t *__restrict__ offsets,
                                                       uint64_t n, int mode, rr_totals *out,
                                                       const uint64_t *__restrict__ extra, uint64_t *err) {
    fold_totals(stats, state, ntiles, offsets, n, mode, out, extra, err);
}

// (the totals were zeroed by the pipeline's first kernel)
static hipError_t launch_finalize(const uint64_t *stats, uint64_t *state, uint32_t ntiles, const uint64_t *offsets,
                                  uint64_t n, int mode, rr_totals *out, hipStream_t stream, uint64_t *err,
                                  const uint64_t *extra = nullptr) {
    uint32_t blocks = (ntiles + 255) / 256;
    if (blocks > 512) blocks = 512;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(finalize_kernel, dim3(blocks), dim3(256), 0, stream, stats, state, ntiles, offsets, n, mode, out,
                       extra, err);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------- decode
// Four launches, no inter-workgroup waits except the scan's look-back:
//   K1 count_kernel   thread per value: its descriptor reservation (rr_format.h) and its walk
//                     class (rr_decode_class.h; header checks done here);
//   K2 scan_kernel    exclusive scan of the reservations -> elem_base of every value;
//   K3 decode_kernel  workgroup per tile of DEC_T values: streams the tile's bytes into the
//                     mirror arena, sorts the tile's values by class in LDS, then its waves take
//                     64-value single-class batches (heaviest class first) and walk + emit them
//                     from L2-hot global memory;
//   K4 finalize       totals.

// ---- K1: reservation + class per value ------------------------------------------------
// reserve(i) = the descriptor slots value i owns (rr_format.h): header fields only, plus the
// length chain of a List.  Equal to the decoded count for every valid blob.
__device__ __forceinline__ uint64_t zl_walk_count_g(const uint8_t *zl, uint64_t L) {
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

__device__ __forceinline__ uint64_t reserve_g(const uint8_t *b, uint64_t L) {
    if (L < 5) return 0;
    const uint32_t t = b[0];
    if (t == RR_TYPE_STRING) return L >= 6 ? 1 : 0;
    if (t == RR_TYPE_LIST_QUICKLIST) {
        uint64_t p = 5, n = 0;
        while (p < L) {
            if (L - p < 4) break;
            const uint64_t l = ld_u32(b + p);
            if (l > L - p - 4) break;
            ++n;
            p += 4 + l;
        }
        return n;
    }
    if (L < 13) return 0;
    switch (t) {
        case RR_TYPE_SET_INTSET: {
            const uint64_t w = ld_u32(b + 5), c = ld_u32(b + 9);
            return ((w == 2 || w == 4 || w == 8) && L - 13 == w * c) ? c : 0;
        }
        case RR_TYPE_SET_HT: { const uint64_t c = ld_u64(b + 5), m = (L - 13) / 8; return c < m ? c : m; }
        case RR_TYPE_HASH_HT: { const uint64_t c = ld_u64(b + 5), m = (L - 13) / 8; return c > m / 2 ? m : 2 * c; }
        case RR_TYPE_ZSET_SKIPLIST: { const uint64_t c = ld_u64(b + 5), m = (L - 13) / 16; return 2 * (c < m ? c : m); }
        case RR_TYPE_HASH_ZIPLIST:
        case RR_TYPE_ZSET_ZIPLIST: {
            const uint64_t Lz = ld_u64(b + 5);
            if (Lz != L - 13 || Lz < 11) return 0;
            const uint64_t zllen = ld_u16(b + 21);
            if (zllen != 0xFFFF) { const uint64_t m = (Lz - 11) / 2; return 1 + (zllen < m ? zllen : m); }
            return 1 + zl_walk_count_g(b + 13, Lz);
        }
        default:
            return 0;
    }
}

// The class of a value: which single-class walk decodes it.  Every check that needs only the
// header is made here; values failing one (and unknown types) go to the exact parser.
__device__ __forceinline__ uint32_t classify_g(const uint8_t *b, uint64_t L) {
    if (L < 5) return C_EXACT;
    switch (b[0]) {
        case RR_TYPE_STRING: {
            if (L < 6) return C_EXACT;
            const uint32_t enc = b[5];
            const uint64_t rest = L - 6;
            if (enc == RR_ENC_INT) return rest == 8 ? C_STR : C_EXACT;
            if (enc == RR_ENC_EMBSTR) return rest <= RR_EMBSTR_SIZE_LIMIT ? C_STR : C_EXACT;
            if (enc == RR_ENC_RAW) return rest <= 0xFFFFFFFFull ? C_STR : C_EXACT;
            return C_EXACT;
        }
        case RR_TYPE_LIST_QUICKLIST:
            return C_LIST;
        case RR_TYPE_SET_INTSET: {
            if (L < 13) return C_EXACT;
            const uint64_t w = ld_u32(b + 5), c = ld_u32(b + 9);
            return ((w == 2 || w == 4 || w == 8) && L - 13 == w * c) ? C_IS : C_EXACT;
        }
        case RR_TYPE_SET_HT:
            return L < 13 ? C_EXACT : C_HT;
        case RR_TYPE_HASH_HT:
            return L < 13 ? C_EXACT : C_HH;
        case RR_TYPE_ZSET_SKIPLIST:
            return L < 13 ? C_EXACT : C_SL;
        case RR_TYPE_HASH_ZIPLIST:
        case RR_TYPE_ZSET_ZIPLIST: {
            if (L < 24) return C_EXACT;   // 13-byte header + the 11-byte empty ziplist
            const uint64_t Lz = ld_u64(b + 5);
            return (Lz == L - 13 && ld_u32(b + 13) == Lz) ? C_ZL : C_EXACT;
        }
        default:
            return C_EXACT;
    }
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
// dword at byte p of the value b (p + 4 <= its length): aligned loads only
__device__ __forceinline__ uint32_t ld_u32_al(const uint8_t *b, uint64_t p) {
    const uintptr_t x = reinterpret_cast<uintptr_t>(b) + p;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(x & ~(uintptr_t)3);
    const uint32_t s = (uint32_t)x & 3;
    const uint32_t lo = w[0], hi = s ? w[1] : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}

typedef uint32_t u32_ua __attribute__((aligned(1)));   // unaligned dword (one global_load_dword)
#ifndef RR_COUNT_UA   // 1: count_kernel's List chain reads each length field with one unaligned load
#define RR_COUNT_UA 1     // (count 54.6 -> 52.5 us)
#endif
#ifndef RR_COUNT_HOIST   // 1: count_kernel issues its offsets loads together, the header loads next
#define RR_COUNT_HOIST 1
#endif
// reserve_g + classify_g from the header dwords (same results, byte for byte)
__device__ __forceinline__ void reserve_classify(const uint8_t *b, uint64_t L, const uint32_t (&d)[6],
                                                 uint64_t &r, uint32_t &c) {
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
            uint64_t p = 5, n = 0;
#ifdef RR_COUNT_NOLIST   // timing-only builds (tools/): no list walk (wrong reservations)
            p = L;
#endif
            while (p < L) {
                if (L - p < 4) break;
#if RR_COUNT_UA   // one unaligned dword load (gfx950 serves it from one line) instead of an aligned pair
                const uint64_t l = *reinterpret_cast<const u32_ua *>(b + p);
#else
                const uint64_t l = ld_u32_al(b, p);
#endif
                if (l > L - p - 4) break;
                ++n;
                p += 4 + l;
            }
            r = n;
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
// totals: later kernels of the same stream use them, so no separate memset launch is needed.
__device__ __forceinline__ void zero_call_words(uint64_t *words, uint32_t nwords, rr_totals *tot) {
    if (blockIdx.x != 0) return;
    for (uint32_t k = threadIdx.x; k < nwords; k += blockDim.x) words[k] = 0;
    if (tot && threadIdx.x < 4) reinterpret_cast<uint64_t *>(tot)[threadIdx.x] = 0;
}

__global__ __launch_bounds__(256) void count_kernel(const uint8_t *__restrict__ blob,
                                                    const uint64_t *__restrict__ offsets, uint64_t n,
                                                    uint32_t *__restrict__ first_val, uint32_t nwin, uint32_t win,
                                                    uint64_t *__restrict__ counts, uint8_t *__restrict__ cls,
                                                    uint64_t *zero_words, uint32_t nzero, rr_totals *tot) {
    zero_call_words(zero_words, nzero, tot);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    if (i == n) counts[n] = 0;   // (the scan writes the total here when there are values)
#if RR_COUNT_HOIST
    // the three offsets in one round trip (loads at clamped indices, no guard branch whose join
    // made the compiler wait for the first two before issuing the third), the header granules
    // in the next, issued before the first_val stores
    const uint64_t o_hi = offsets[i];
    const uint64_t o_lo = offsets[i ? i - 1 : 0];
    const uint64_t b1 = offsets[i < n ? i + 1 : n];
    uint32_t d[6];
    if (i < n) head24(blob, o_hi, b1, d);
    const uint64_t w_lo = i == 0 ? 0 : o_lo / win + 1;
#else
    const uint64_t o_hi = offsets[i];
    const uint64_t w_lo = i == 0 ? 0 : offsets[i - 1] / win + 1;
#endif
    // first_val[w] = first value whose first byte is at or after w*win (windows past the
    // last value start, and the sentinel nwin, get n)
    const uint64_t w_hi = i == n ? nwin : o_hi / win;
    for (uint64_t w = w_lo; w <= w_hi && w <= nwin; ++w) first_val[w] = (uint32_t)i;
    if (i < n) {
#if !RR_COUNT_HOIST
        const uint64_t b1 = offsets[i + 1];
#endif
#ifdef RR_COUNT_BYTES   // the byte-load formulation (diagnostics)
        counts[i] = reserve_g(blob + o_hi, b1 - o_hi);
        cls[i] = (uint8_t)classify_g(blob + o_hi, b1 - o_hi);
#else
#if !RR_COUNT_HOIST
        uint32_t d[6];
        head24(blob, o_hi, b1, d);
#endif
        uint64_t r;
        uint32_t c;
        reserve_classify(blob + o_hi, b1 - o_hi, d, r, c);
        counts[i] = r;
        cls[i] = (uint8_t)c;
#endif
    }
}

// ---- K1+K2 in one launch: count_scan_kernel -----------------------------------------------
// count_kernel's per-value work, then the block's exclusive scan, then a decoupled look-back
// between the 256-value blocks (blockIdx order, two-level groups, rr_device.h): the block writes
// elem_base straight away.  The look-back's round trips (a few us under load) sit at the end of
// each block and are hidden by the other resident blocks of the CU, so the separate scan launch
// (its own look-back, the counts written and read again) goes away.  (A look-back that never
// resolves — a block dispatched out of order behind a full machine — sets the call's error word
// after the bounded wait: the host sees RR_API_EDEVICE, never a hang.)
constexpr uint32_t CS_NT = 256;
__global__ __launch_bounds__(CS_NT) void count_scan_kernel(const uint8_t *__restrict__ blob,
                                                          const uint64_t *__restrict__ offsets, uint64_t n,
                                                          uint32_t *__restrict__ first_val, uint32_t nwin, uint32_t win,
                                                          uint64_t *__restrict__ ebase, uint8_t *__restrict__ cls,
                                                          uint64_t *lb_state, uint64_t *lb_groups, uint32_t ntiles,
                                                          uint64_t *err, rr_totals *tot) {
    zero_call_words(nullptr, 0, tot);
    __shared__ uint64_t wsum[CS_NT / RR_WAVE];
    __shared__ uint64_t sh_pre;
    const uint32_t tile = blockIdx.x, tid = threadIdx.x, lane = lane_id(), wave = tid / RR_WAVE;
    const uint64_t i = (uint64_t)tile * CS_NT + tid;
    uint64_t r = 0;
    if (i <= n) {
        const uint64_t o_hi = offsets[i];
        const uint64_t w_lo = i == 0 ? 0 : offsets[i - 1] / win + 1;
        const uint64_t w_hi = i == n ? nwin : o_hi / win;
        for (uint64_t w = w_lo; w <= w_hi && w <= nwin; ++w) first_val[w] = (uint32_t)i;
        if (i < n) {
            const uint64_t b1 = offsets[i + 1];
            uint32_t d[6];
            head24(blob, o_hi, b1, d);
            uint32_t c;
            reserve_classify(blob + o_hi, b1 - o_hi, d, r, c);
            cls[i] = (uint8_t)c;
        }
    }
    const uint64_t incl = wave_incl_scan(r);
    if (lane == RR_WAVE - 1) wsum[wave] = incl;
    __syncthreads();
    uint64_t wpre = 0, agg = 0;
#pragma unroll
    for (uint32_t k = 0; k < CS_NT / RR_WAVE; ++k) {
        wpre += k < wave ? wsum[k] : 0;
        agg += wsum[k];
    }
    if (wave == 0) {
        const uint64_t pre = lookback(lb_state, lb_groups, tile, ntiles, agg, err);
        if (lane == 0) sh_pre = pre;
    }
    __syncthreads();
    const uint64_t pre = sh_pre;
    if (i < n) ebase[i] = pre + wpre + incl - r;
    if (tile == ntiles - 1 && tid == CS_NT - 1) ebase[n] = pre + agg;   // the call's descriptor total
}

// ---- K2: exclusive scan of the reservations -> elem_base -------------------------------
// 4096 values per 256-thread workgroup, tile ids from an atomic ticket (so a tile only waits
// on tiles already running), decoupled look-back between tiles (two-level, rr_device.h).
#ifndef RR_SCAN_PT
#define RR_SCAN_PT 16
#endif
constexpr uint32_t SCAN_PER_THREAD = RR_SCAN_PT;
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

// ---- K3: tiles: mirror copy + class sort + single-class batches ------------------------
// The exact parser, lane = value v (from global memory): the reference's status codes for
// malformed values, zero-filled slots, capacity handling.
// per-value contribution to the window totals (returned by value: accumulators passed by
// reference were merged into one dynamically-addressed update and spilled to scratch)
struct Acc {
    uint32_t bad;
    uint64_t pay;
};

#ifdef RR_DEC_NOINL
#define RR_COLD __noinline__
#else
#define RR_COLD __forceinline__
#endif
// Values whose descriptors need a whole-value pass the walks cannot make (duplicate keys of a
// hash table, re-sorting a skiplist) are queued for fixup_kernel: fix[0] counts them, their
// indices follow the FIX_HDR header words (capacity n: a value is queued at most once).
constexpr uint32_t FIX_HDR = 4;   // [0] queued, [1] error word, [2] bad delta, [3] payload delta
__device__ __forceinline__ void queue_fixup(uint64_t *fix, uint64_t v) {
    const uint64_t i = atomicAdd((unsigned long long *)fix, 1ull);
    reinterpret_cast<uint32_t *>(fix + FIX_HDR)[i] = (uint32_t)v;
}

// (eb, r: the value's first descriptor slot and its reservation)
__device__ RR_COLD Acc exact_value(const uint8_t *__restrict__ blob, uint64_t v,
                                           const uint64_t *__restrict__ offsets, uint64_t eb, uint64_t r,
                                           rr_value *__restrict__ values, rr_elem *__restrict__ elems, uint64_t cap,
                                           uint64_t *fix) {
    uint64_t pay = 0;
    const uint64_t o_lo = offsets[v], o_hi = offsets[v + 1];
    const uint8_t *b = blob + o_lo;
    Parsed pr = parse_value<false, const uint8_t *>(b, o_lo, o_hi - o_lo, nullptr);
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
        Parsed e = parse_value<true, const uint8_t *>(b, o_lo, o_hi - o_lo, elems + eb);
        pay += e.payload;
        const uint32_t t = ld_u8(b);
        const uint64_t keys = t == RR_TYPE_HASH_HT ? ne / 2 : ne;
        if (((t == RR_TYPE_SET_HT || t == RR_TYPE_HASH_HT) && keys >= 2) || e.unsorted) queue_fixup(fix, v);
    }
    const uint32_t len = (uint32_t)(o_hi - o_lo);
    put_value(values + v, len ? ld_u8(b) : 0, pr.enc, status, len >= 5 ? ld_u32(b + 1) : 0, (uint32_t)ne,
              (uint32_t)eb);
    return Acc{status != RR_OK ? 1u : 0u, pay};
}

// ziplists: 1 = grouped walks on one backward prevlen chain (do_ziplist_bg, RR_ZL_VPB values
// per batch), 0 = two lanes per value walking from both ends (do_ziplist, DEC_BL / 2 values)
#ifndef RR_ZL_BACK
#define RR_ZL_BACK 1
#endif
#ifndef RR_ZL_VPB
#define RR_ZL_VPB 16
#endif
#ifndef RR_ZL_PIPE   // 1: ziplist batches run do_ziplist_bp (compile-time group size, pipelined rounds)
#define RR_ZL_PIPE 1
#endif
#if RR_ZL_BACK
constexpr uint32_t ZL_VPB = RR_ZL_VPB;
#endif
// hash tables: 1 = grouped walks (do_ht_g) whenever the batch gives a value enough lanes to
// hold its keys, with RR_HH_VPB hashes / RR_HT_VPB sets per batch; 0 = lane per value (do_ht)
#ifndef RR_HT_GROUPED
#define RR_HT_GROUPED 1
#endif
#ifndef RR_HH_VPB
#define RR_HH_VPB 8
#endif
#ifndef RR_HT_VPB
#define RR_HT_VPB 16
#endif
#ifndef RR_LIST_PIPE   // 1: List batches run do_list_bp (compile-time group size, pipelined rounds)
#define RR_LIST_PIPE 1     // (LIST batch 17.3K -> 12.1K cycles with 16 Lists per batch)
#endif
#ifndef RR_LIST_VPB   // Lists per batch (grouped: fewer Lists per batch, more lanes per List)
#if RR_LIST_PIPE
#define RR_LIST_VPB 16
#else
#define RR_LIST_VPB 64
#endif
#endif
// class batch order: heaviest walks first (longest-job-first over the window's waves)
#ifndef RR_DEC_ORDER
#define RR_DEC_ORDER C_ZL, C_SL, C_HH, C_HT, C_LIST, C_EXACT, C_IS, C_STR
#endif
__constant__ uint32_t CLASS_ORDER[C_N] = {RR_DEC_ORDER};
// the class of batch-order slot k from registers (a select chain over the compile-time order:
// no constant-memory load on each batch's path)
__device__ __forceinline__ uint32_t class_at(uint32_t k) {
    constexpr uint32_t ord[C_N] = {RR_DEC_ORDER};
    uint32_t c = ord[0];
#pragma unroll
    for (uint32_t i = 1; i < C_N; ++i) c = k == i ? ord[i] : c;
    return c;
}
#ifndef RR_DEC_BREG   // 1: the batch loop keeps the chunk's batch prefixes in registers
#define RR_DEC_BREG 0   // (measured: decode_kernel -2.6 % in one trace, calls mixed, cfg 3 +1.5 %)
#endif

// One single-class batch: lane < cnt decodes value v (byte offsets relative to the source,
// whose byte 0 is batch offset B).
// One single-class batch, run by the whole wave: lane < cnt (active) decodes value v (byte
// offsets relative to the source, whose byte 0 is batch offset B).  The walks run the wave in
// lock-step (rr_decode_class.h); values they reject, and the EXACT class, go to the exact
// parser lane by lane.
// G lanes per value (grouped walks, rr_decode_class.h), this lane being lane g of its group;
// the group's lane 0 records the value (or runs the exact parser), every lane returns the
// payload of the elements it stored.
// (eb_v, r_v: value v's first descriptor slot and its reservation, for active lanes)
template <class Src>
__device__ __forceinline__ Acc run_batch(const Src &src, uint32_t c, bool active, uint64_t v, uint32_t G, uint32_t g,
                                         uint64_t B, rsrc_t E,
                                         uint64_t eb0, const uint8_t *__restrict__ blob,
                                         const uint64_t *__restrict__ offsets, uint64_t eb_v, uint64_t r_v,
                                         rr_value *__restrict__ values, rr_elem *__restrict__ elems, uint64_t cap,
                                         uint64_t *fix) {
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
        } else if (c == C_LIST) {
#if RR_LIST_PIPE   // grouped, software-pipelined (G a power of two)
            if (G >= 16) fail = do_list_bp<16>(src, l, active, g, ne, vp);
            else if (G >= 8) fail = do_list_bp<8>(src, l, active, g, ne, vp);
            else if (G >= 4) fail = do_list_bp<4>(src, l, active, g, ne, vp);
            else if (G >= 2) fail = do_list_bp<2>(src, l, active, g, ne, vp);
            else fail = do_list_bp<1>(src, l, active, g, ne, vp);
#else
            fail = do_list_g(src, l, active, G, g, ne, vp);
#endif
        } else if (c == C_HT || c == C_HH) {   // grouped (G > 1) or lane per value (do_ht)
            if (G > 1) fail = do_ht_g(src, H, l, active, G, g, ne, vp, fixup, c == C_HH);
            else fail = do_ht(src, H, l, active, ne, vp, fixup, c == C_HH);
        } else if (c == C_SL) {
            fail = do_skiplist_g(src, H, l, active, G, g, ne, vp);
        } else {
#if RR_ZL_BACK && RR_ZL_PIPE   // C_ZL: grouped, software-pipelined (G a power of two >= 4)
            if (G >= 16) fail = do_ziplist_bp<16>(src, l, active, g, ne, vp);
            else if (G >= 8) fail = do_ziplist_bp<8>(src, l, active, g, ne, vp);
            else fail = do_ziplist_bp<4>(src, l, active, g, ne, vp);
#elif RR_ZL_BACK   // C_ZL: grouped, one backward prevlen chain per value
            fail = do_ziplist_bg(src, l, active, G, g, ne, vp);
#else            // C_ZL: G == 2, lane 1 of the pair walks backward
            fail = do_ziplist(src, l, active, g != 0, ne, vp);
#endif
        }
        exact = fail;
        if (active && !fail) {
            if (g == 0) {
                if (fixup && l.ok) queue_fixup(fix, v);
                put_value(values + v, H.type(), enc, l.ok ? RR_OK : RR_E_CAPACITY, H.lru(), ne, (uint32_t)eb);
                acc.bad = l.ok ? 0u : 1u;
            }
            acc.pay = l.ok ? vp : 0;
        }
        active &= g == 0;   // the exact parser runs once per value, on the group's lane 0
    }
    if (active && exact) acc = exact_value(blob, v, offsets, eb_v, r_v, values, elems, cap, fix);
    return acc;
}

// the unstaged (global-memory) instantiation: cold path, kept out of line in RR_DEC_NOINL
// builds so the hot staged code stays small
__device__ RR_COLD Acc run_batch_g(const GlbSrc &src, uint32_t c, bool active, uint64_t v, uint32_t G, uint32_t g,
                                   uint64_t B, rsrc_t E, uint64_t eb0, const uint8_t *__restrict__ blob,
                                   const uint64_t *__restrict__ offsets, uint64_t eb_v, uint64_t r_v,
                                   rr_value *__restrict__ values, rr_elem *__restrict__ elems, uint64_t cap,
                                   uint64_t *fix) {
    return run_batch(src, c, active, v, G, g, B, E, eb0, blob, offsets, eb_v, r_v, values, elems, cap, fix);
}

// Workgroup per byte WINDOW of W bytes: window t owns the values whose first byte lies in
// [t*W, (t+1)*W) (first_val from K1).  The workgroup
//   1. streams the window into the mirror arena and, from the same loads, stages the bytes of
//      its values (the window + the tail of its last value, up to SLACK more) into LDS;
//   2. per chunk of <= PMAX of its values: counting-sorts them by class in LDS;
//   3. its waves take single-class batches of <= 64 values, heaviest class first, and walk +
//      emit them from LDS (from global memory when the values did not fit the stage).
// Probe build (make VARIANT=probe EXTRA=-DRR_PROBE, tools/probe_decode.py): per-window phase
// cycles and per-class batch cycles / counts / lanes into a buffer set by rr_probe_set
// (PROBE_WORDS u64 per window).  Diagnostics only; the product build has none of it.
#ifdef RR_PROBE
constexpr uint32_t PROBE_WORDS = 32;
__device__ uint64_t *g_probe;
extern "C" int rr_probe_set(void *p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_probe), &p, sizeof(p)) == hipSuccess ? 0 : -1; }
#define PROBE(...) __VA_ARGS__
#else
#define PROBE(...)
#endif

// lanes per walk batch: a class's values in a chunk are cut into batches of at most DEC_BL, so
// a class with few values per window can still spread over several waves
#ifndef RR_DEC_BL
#define RR_DEC_BL 64
#endif
constexpr uint32_t DEC_BL = RR_DEC_BL;
static_assert(DEC_BL >= 2 && DEC_BL <= RR_WAVE && DEC_BL % 2 == 0, "batch lanes");
// values per batch of a class (a class with more values in the chunk gets several batches)
__device__ __forceinline__ uint32_t class_vpb(uint32_t c) {
#if RR_ZL_BACK
    if (c == C_ZL) return ZL_VPB;
#else
    if (c == C_ZL) return DEC_BL / 2;   // two lanes each
#endif
#if RR_HT_GROUPED
    if (c == C_HH) return RR_HH_VPB;
    if (c == C_HT) return RR_HT_VPB;
#endif
    if (c == C_LIST) return RR_LIST_VPB;
    return DEC_BL;
}
// 1: the mirror-arena copy is written by waves that ran out of walk batches (step 4), not
// during staging
#ifndef RR_DEC_LATECOPY
#define RR_DEC_LATECOPY 0
#endif
#ifndef RR_DEC_PF   // persistent workgroups, next window's arena copy overlapped with the walks
#define RR_DEC_PF 0
#endif
#ifndef RR_DEC_OVL   // the window's loads in flight under the class sort (fused copy builds)
#define RR_DEC_OVL 1
#endif
#if RR_DEC_LATECOPY   // (the overlap applies to the fused copy)
#undef RR_DEC_OVL
#define RR_DEC_OVL 0
#endif
#ifndef RR_DEC_OVL_K  // granules (16 B) per thread loaded before the sort (the rest after it)
#define RR_DEC_OVL_K 9
#endif
// 1: the window's loads, arena stores and stage writes go through buffer resources with no
// exec-mask branches (out-of-range loads read zeros, out-of-range stores are dropped, unstaged
// granules are written to a dummy LDS slot), and the workgroup's barriers order LDS only.
// The branch joins of the guarded copy made the compiler's wait-count pass wait for each
// store's acknowledgement before the next store, and the conditional loads made the sort's
// first barrier wait for all of them (vmcnt(0)).
#ifndef RR_DEC_BFREE
#define RR_DEC_BFREE 1
#endif
#ifndef RR_DEC_BALANCE   // 1: a class's values split evenly over its batches
#define RR_DEC_BALANCE 0
#endif
#ifndef RR_DEC_PRIO   // wave priority during the walks (0: none; see the batch loop)
#define RR_DEC_PRIO 0
#endif
#ifndef RR_DEC_KE   // window granules per thread loaded before the class bytes (the rest after)
#define RR_DEC_KE 2
#endif
#if RR_DEC_BFREE
#define DEC_SYNC() lds_barrier()
#else
#define DEC_SYNC() __syncthreads()
#endif
#ifndef RR_DEC_EARLY  // late-copy builds: write the arena copy from the stage before the walks, not after
#define RR_DEC_EARLY 0
#endif
#ifndef RR_DEC_GLDS   // late-copy staging by global_load_lds (LDS-DMA) instead of register loads
#define RR_DEC_GLDS 0
#endif
#ifndef RR_DEC_SU   // 16-byte staging loads in flight per thread (late-copy staging)
#define RR_DEC_SU 4
#endif
#if RR_DEC_LATECOPY
#define PROBE_OR_LATE(...) __VA_ARGS__
#else
#define PROBE_OR_LATE(...)
#endif
// Two 512-thread workgroups per CU = 4 waves per SIMD, so at most 128 VGPRs: the allocator is
// told so (left to itself it takes 137 for the hash-table walk and the CU holds one workgroup).
#ifndef RR_DEC_WPE
#define RR_DEC_WPE 4
#endif
#ifndef RR_DEC_EBPF   // 1: the window's elem_base words touched under the sort (cache-warm batch loads)
#define RR_DEC_EBPF 0
#endif
#ifndef RR_DEC_ATOT   // 1: decode_kernel adds its windows' totals atomically (no fold in decode_post)
#define RR_DEC_ATOT 1
#endif
#if RR_DEC_WPE > 0
#define DEC_WPE_ATTR __attribute__((amdgpu_waves_per_eu(RR_DEC_WPE)))
#else
#define DEC_WPE_ATTR
#endif
template <uint32_t W, uint32_t SLACK, uint32_t NW, uint32_t PMAX>
__global__ __launch_bounds__(NW * RR_WAVE) DEC_WPE_ATTR void decode_kernel(const uint8_t *__restrict__ blob, uint64_t data_cap,
                                                              const uint64_t *__restrict__ offsets, uint64_t n,
                                                              const uint32_t *__restrict__ first_val,
                                                              const uint8_t *__restrict__ cls,
                                                              const uint64_t *__restrict__ ebase,
                                                              rr_value *__restrict__ values,
                                                              rr_elem *__restrict__ elems, uint64_t elem_cap,
                                                              uint8_t *__restrict__ arena, uint64_t *__restrict__ stats,
                                                              uint64_t *fix, uint32_t nwin, rr_totals *tot) {
    constexpr uint32_t NT = NW * RR_WAVE, STAGE = W + SLACK;
    static_assert(PMAX % NT == 0 && W % 16 == 0 && SLACK % 16 == 0, "tile shape");
#ifndef RR_DEC_LDSPAD   // diagnostics: extra LDS per workgroup (e.g. to hold one workgroup per CU)
#define RR_DEC_LDSPAD 0
#endif
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE + 64 + RR_DEC_LDSPAD];
    __shared__ uint16_t perm[PMAX];
    __shared__ uint32_t ccount[C_N], cbase[C_N], ccur[C_N], bpre[C_N + 1];
    __shared__ uint32_t next_batch;
    __shared__ uint32_t next_copy;   // (late-copy and persistent builds)
    (void)next_copy;
    __shared__ uint64_t red[2][NW];
    PROBE(__shared__ uint64_t prb[PROBE_WORDS]; uint64_t pt0 = __builtin_amdgcn_s_memtime(), pt1 = 0, pt2 = 0;
          if (threadIdx.x < PROBE_WORDS) prb[threadIdx.x] = 0;)
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid / RR_WAVE;
#if RR_DEC_PF
    // persistent: this workgroup's windows blockIdx.x, + gridDim.x, ...; while a window's longest
    // walks run, the waves with no batch left copy the NEXT window to the arena (global ->
    // global), which also leaves its bytes in the L2 for that window's LDS stage
    for (uint32_t tile = blockIdx.x, it = 0; tile < nwin; tile += gridDim.x, ++it) {
    if (it) DEC_SYNC();   // the previous window is done with the LDS
    if (tid == 0) next_copy = 0;
    PROBE(pt0 = __builtin_amdgcn_s_memtime(); if (threadIdx.x < PROBE_WORDS) prb[threadIdx.x] = 0;)
#else
    {
    const uint32_t tile = blockIdx.x, it = 0;
    (void)nwin;
    (void)it;
#endif
    const uint64_t padded = (offsets[n] + 15) & ~15ull;
    const uint64_t W0 = (uint64_t)tile * W;
    const uint64_t W1 = W0 + W < padded ? W0 + W : padded;
    // the arena copy starts at the call's first value (a call over a slice of a larger buffer —
    // the chunks of rr_decode_batch_host — copies only its own bytes); the stage always lies
    // past it (S0 >= offsets[v_lo] >= offsets[0])
    const uint64_t A0 = W0 > (offsets[0] & ~15ull) ? W0 : (offsets[0] & ~15ull);
#if RR_DEC_OVL && RR_DEC_BFREE
    // the window's own granules [A0, W1) first: their range needs only offsets[0] and
    // offsets[n], not first_val -> offsets, so the loads go out at the window's start; the
    // stage's tail [W1, ov_e) (the last values' bytes past the window) follows the sort.  The
    // arena gets [A0, W1) (stores past it are dropped); g = A0 / 16 + tid + k * NT is at byte
    // offset 16 (tid + k NT)
    constexpr uint32_t KM = W / 16 / NT;   // granules per thread of a whole window
    static_assert(W % (16 * NT) == 0, "window granules per thread");
    const uint64_t ov_a = A0 >> 4, ov_w1 = W1 >> 4;
    const uint32_t ov_mb = ov_w1 > ov_a ? (uint32_t)((ov_w1 - ov_a) * 16) : 0u;
    const rsrc_t ov_RM = make_rsrc(blob + A0, ov_mb);
    const rsrc_t ov_RA = make_rsrc(arena + A0, ov_mb);
    // KE granules per thread go out before the first_val -> offsets / class-byte loads, the rest
    // after the class bytes: the sort waits (vmcnt, in issue order) for the class bytes and
    // therefore for the early granules only
    constexpr uint32_t KE = RR_DEC_KE < KM ? RR_DEC_KE : KM;
    u32x4 ov_m[KM];
#pragma unroll
    for (uint32_t k = 0; k < KE; ++k)
        ov_m[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ov_RM, (int)((tid + k * NT) * 16), 0, 0));
#endif
    const uint64_t v_lo = first_val[tile], v_hi = first_val[tile + 1];
    uint64_t S0 = W0, S1 = W0;
    if (v_hi > v_lo) {
        S0 = offsets[v_lo] & ~15ull;
        S1 = (offsets[v_hi] + 15) & ~15ull;
    }
    const bool staged = S1 - S0 <= STAGE;
    const uint64_t cap = elem_cap < 0xFFFFFFFFull ? elem_cap : 0xFFFFFFFFull;   // elem_base is 32-bit

    // the first chunk's class bytes, loaded before the copy so their latency hides under it
    uint32_t cls0[PMAX / NT];
#pragma unroll
    for (uint32_t j = 0; j < PMAX / NT; ++j) {
        const uint64_t v = v_lo + j * NT + tid;
        cls0[j] = v < v_hi ? (uint32_t)cls[v] : C_N;
    }
#if RR_DEC_EBPF
    // the first chunk's elem_base words touched now, in flight under the sort (into this CU's
    // L1 and the L2), so each batch's per-value elem_base loads hit the cache instead of memory
    uint32_t ebpf = 0;
#pragma unroll
    for (uint32_t j = 0; j < PMAX / NT; ++j) {
        const uint64_t v = v_lo + j * NT + tid;
        ebpf |= (uint32_t)ebase[v < v_hi ? v : v_lo];
    }
#endif
#if RR_DEC_OVL && RR_DEC_BFREE
#pragma unroll
    for (uint32_t k = KE; k < KM; ++k)
        ov_m[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ov_RM, (int)((tid + k * NT) * 16), 0, 0));
    // the stage's tail [W1, S1): at most SLACK bytes, KT granules per thread, also in flight
    // under the sort
    constexpr uint32_t KT = (SLACK / 16 + NT - 1) / NT;
    const uint64_t ov_t0 = ov_w1 > ov_a ? ov_w1 : ov_a;
    const uint64_t ov_te = (staged && S1 > W1 ? S1 : W1) >> 4;
    const rsrc_t ov_RT = make_rsrc(blob + ov_t0 * 16, ov_te > ov_t0 ? (uint32_t)((ov_te - ov_t0) * 16) : 0u);
    u32x4 ov_t[KT];
#pragma unroll
    for (uint32_t k = 0; k < KT; ++k)
        ov_t[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ov_RT, (int)((tid + k * NT) * 16), 0, 0));
#endif

#if RR_DEC_LATECOPY
    // 1. value bytes -> LDS only; the window's arena copy is written in step 4 by waves that
    //    have run out of batches, overlapping the longest walks
    if (tid == 0) next_copy = 0;
#if RR_DEC_GLDS
    // every stage load in flight at once, straight to LDS (no VGPRs): wave w fills the 1 KiB
    // blocks w, w + NW, ... (lane-linear: lane l's 16 bytes land at block + 16 l)
    if (staged) {
        const uint64_t cs0 = S0 >> 4, cs1 = S1 >> 4;
        const uint32_t nblk = (uint32_t)((cs1 - cs0 + RR_WAVE - 1) / RR_WAVE);
        for (uint32_t b = wave; b < nblk; b += NW) {
            const uint64_t g = cs0 + (uint64_t)b * RR_WAVE + lane;
            if (g < cs1)
                __builtin_amdgcn_global_load_lds((const void *)(blob + g * 16),
                                                 (__attribute__((address_space(3))) void *)(stage + b * 16 * RR_WAVE),
                                                 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#else
    if (staged) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(blob);
        u32x4 *lds = reinterpret_cast<u32x4 *>(stage);
        const uint64_t cs0 = S0 >> 4, cs1 = S1 >> 4;
        uint64_t c = cs0 + tid;
        for (; c + (RR_DEC_SU - 1) * NT < cs1; c += RR_DEC_SU * NT) {
            u32x4 x[RR_DEC_SU];
#pragma unroll
            for (int k = 0; k < RR_DEC_SU; ++k) x[k] = src[c + k * NT];
#pragma unroll
            for (int k = 0; k < RR_DEC_SU; ++k) lds[c + k * NT - cs0] = x[k];
        }
        for (; c < cs1; c += NT) lds[c - cs0] = src[c];
    }
#endif
#else
#if RR_DEC_OVL
    // 1''. the common case (the window and its values' tail fit RR_DEC_OVL_K granules per
    //      thread): the loads are issued here and land while the class sort below runs; the
    //      arena stores and the LDS stage writes follow the sort (plain loads survive its
    //      barriers).  The sort reads no global memory, so none of its waits drain them.
    const uint64_t eb0 = ebase[v_lo], eb1 = ebase[v_hi];
    const uint64_t ov_s0 = S0 >> 4, ov_e = (staged && S1 > W1 ? S1 : W1) >> 4;
    const bool ovl = !(RR_DEC_PF && it > 0);
#if RR_DEC_BFREE
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    lds_u32x4 *ov_lds = (lds_u32x4 *)(__attribute__((address_space(3))) uint8_t *)stage;
    // granule g's stage slot, or the dummy slot just past the stage (reads past the stage see
    // garbage there, which the walks never use: every read is checked against its value's end)
    auto ov_slot = [&](uint64_t g) __attribute__((always_inline)) -> uint32_t {
        return (staged & (g >= ov_s0) & (g < ov_e)) ? (uint32_t)(g - ov_s0) : STAGE / 16;
    };
    auto ov_finish = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t k = 0; k < KM; ++k) {
#ifndef RR_ABLATE_NOCOPY
            __builtin_amdgcn_raw_buffer_store_b128(ov_m[k], ov_RA, (int)((tid + k * NT) * 16), 0, 2 /* nt */);
#endif
            ov_lds[ov_slot(ov_a + tid + (uint64_t)k * NT)] = ov_m[k];
        }
        // the stage's tail [W1, ov_e): LDS only
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k) ov_lds[ov_slot(ov_t0 + tid + (uint64_t)k * NT)] = ov_t[k];
    };
    if (ovl) {
    } else
#else
    const uint64_t ov_w1 = W1 >> 4;
    u32x4 ov_x[RR_DEC_OVL_K];
    if (ovl) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(blob);
#pragma unroll
        for (int k = 0; k < RR_DEC_OVL_K; ++k) {
            const uint64_t g = (A0 >> 4) + tid + (uint64_t)k * NT;
            ov_x[k] = g < ov_e ? src[g] : u32x4{0u, 0u, 0u, 0u};
        }
    }
    auto ov_finish = [&]() __attribute__((always_inline)) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(blob);
        u32x4 *dst = reinterpret_cast<u32x4 *>(arena);
        u32x4 *lds = reinterpret_cast<u32x4 *>(stage);
#pragma unroll
        for (int k = 0; k < RR_DEC_OVL_K; ++k) {
            const uint64_t g = (A0 >> 4) + tid + (uint64_t)k * NT;
#ifndef RR_ABLATE_NOCOPY
            if (g < ov_w1) __builtin_nontemporal_store(ov_x[k], dst + g);
#endif
            if (staged && g >= ov_s0 && g < ov_e) lds[g - ov_s0] = ov_x[k];
        }
        // the rest of the window (beyond the prefetched granules), loaded now
        uint64_t c = (A0 >> 4) + tid + (uint64_t)RR_DEC_OVL_K * NT;
        for (; c + 3 * NT < ov_e; c += 4 * NT) {
            u32x4 x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = src[c + k * NT];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t cc = c + k * NT;
#ifndef RR_ABLATE_NOCOPY
                if (cc < ov_w1) __builtin_nontemporal_store(x[k], dst + cc);
#endif
                if (staged && cc >= ov_s0) lds[cc - ov_s0] = x[k];
            }
        }
        for (; c < ov_e; c += NT) {
            const u32x4 x = src[c];
#ifndef RR_ABLATE_NOCOPY
            if (c < ov_w1) __builtin_nontemporal_store(x, dst + c);
#endif
            if (staged && c >= ov_s0) lds[c - ov_s0] = x;
        }
    };
    if (ovl) {
    } else
#endif   // RR_DEC_BFREE
#endif
    if (RR_DEC_PF && it > 0) {
        // 1'. the arena copy was made during the previous window: value bytes -> LDS only
        //     (L2-hot: that copy just read them)
        if (staged) {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(blob);
            u32x4 *lds = reinterpret_cast<u32x4 *>(stage);
            const uint64_t cs0 = S0 >> 4, cs1 = S1 >> 4;
            uint64_t c = cs0 + tid;
            for (; c + 3 * NT < cs1; c += 4 * NT) {
                u32x4 x[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) x[k] = src[c + k * NT];
#pragma unroll
                for (int k = 0; k < 4; ++k) lds[c + k * NT - cs0] = x[k];
            }
            for (; c < cs1; c += NT) lds[c - cs0] = src[c];
        }
    } else
    // 1. window -> arena, value bytes -> LDS (one load feeds both)
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(blob);
        u32x4 *dst = reinterpret_cast<u32x4 *>(arena);
        u32x4 *lds = reinterpret_cast<u32x4 *>(stage);
        const uint64_t cw1 = W1 >> 4, cs0 = S0 >> 4;
        const uint64_t ce = (staged && S1 > W1 ? S1 : W1) >> 4;
        uint64_t c = (A0 >> 4) + tid;
        for (; c + 3 * NT < ce; c += 4 * NT) {
            u32x4 x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) x[k] = src[c + k * NT];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t cc = c + k * NT;
#ifndef RR_ABLATE_NOCOPY   // timing-only builds (tools/)
                if (cc < cw1) __builtin_nontemporal_store(x[k], dst + cc);
#endif
                if (staged && cc >= cs0) lds[cc - cs0] = x[k];
            }
        }
        for (; c < ce; c += NT) {
            const u32x4 x = src[c];
#ifndef RR_ABLATE_NOCOPY
            if (c < cw1) __builtin_nontemporal_store(x, dst + c);
#endif
            if (staged && c >= cs0) lds[c - cs0] = x;
        }
    }
#endif
#if RR_DEC_LATECOPY && RR_DEC_EARLY
    // 1b. the window's arena copy straight from the LDS stage (bytes before S0, and windows
    //     that are not staged, from global memory), before the walks start
    __syncthreads();   // the stage is complete
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(blob);
        u32x4 *dst = reinterpret_cast<u32x4 *>(arena);
        const u32x4 *lds = reinterpret_cast<const u32x4 *>(stage);
        const uint64_t cw0 = W0 >> 4, cw1 = W1 >> 4, cs0 = S0 >> 4, cs1 = staged ? S1 >> 4 : cs0;
        for (uint64_t g = cw0 + tid; g < cw1; g += NT) {
            const u32x4 x = g >= cs0 && g < cs1 ? lds[g - cs0] : src[g];
#ifndef RR_ABLATE_NOCOPY
            __builtin_nontemporal_store(x, dst + g);
#endif
        }
    }
#endif
    // values that do not fit the stage are read from global memory; if even their 32-bit
    // window-relative byte or slot offsets could overflow, the exact parser takes them
#if !RR_DEC_OVL
    const uint64_t eb0 = ebase[v_lo], eb1 = ebase[v_hi];
#endif
    const bool far = (!staged && S1 - S0 > 0xFFFFFF00ull) || (eb1 - eb0) * 16 >= NOSLOT;
    const LdsSrc lsrc{(lds_cptr)stage};
    const GlbSrc gsrc{make_rsrc(blob + S0, (uint32_t)(data_cap - S0 < 0xFFFFFFFFull ? data_cap - S0 : 0xFFFFFFFFull))};
    // the window's descriptor slots [eb0, eb1), cut at the capacity
    const uint64_t ecut = eb1 < cap ? eb1 : cap;
    const rsrc_t E = make_rsrc(reinterpret_cast<const uint8_t *>(elems + eb0),
                               far || ecut <= eb0 ? 0u : (uint32_t)((ecut - eb0) * 16));

    uint64_t bad = 0, pay = 0;
#ifdef RR_ABLATE   // timing-only builds (tools/): 1 = copy + stage only, 2 = + class sort, no batches
    const uint64_t v_end = RR_ABLATE == 1 ? v_lo : v_hi;
#else
    const uint64_t v_end = v_hi;
#endif
    // 2. counting sort of a chunk of values by class (ballot per class, one LDS atomic per
    //    class per wave-round) into perm, class bases and batch prefixes
    auto sort_chunk = [&](uint64_t c0) __attribute__((always_inline)) {
        const uint32_t nv = (uint32_t)(v_hi - c0 < PMAX ? v_hi - c0 : PMAX);
        if (tid < C_N) { ccount[tid] = 0; ccur[tid] = 0; }
        if (tid == 0) next_batch = 0;
        DEC_SYNC();   // also: the previous chunk's batches are done
        PROBE(if (c0 == v_lo) pt1 = __builtin_amdgcn_s_memtime();)
        uint32_t myc[PMAX / NT];
#pragma unroll
        for (uint32_t j = 0; j < PMAX / NT; ++j) {
            const uint32_t i = j * NT + tid;
            const uint32_t ci = c0 == v_lo ? cls0[j] : i < nv ? (uint32_t)cls[c0 + i] : C_N;
            myc[j] = i < nv ? (far ? C_EXACT : ci) : C_N;
            if (j * NT + wave * RR_WAVE >= nv) continue;   // (wave-uniform) no values in this round
#pragma unroll
            for (uint32_t c = 0; c < C_N; ++c) {
                const uint64_t m = __ballot(myc[j] == c);
                if (m && lane == 0) atomicAdd(&ccount[c], (uint32_t)__popcll(m));
            }
        }
        DEC_SYNC();
        if (tid == 0) {
            uint32_t s = 0, bs = 0;
            for (uint32_t k = 0; k < C_N; ++k) {
                const uint32_t c = CLASS_ORDER[k];
                const uint32_t vpb = class_vpb(c);
                cbase[c] = s;
                bpre[k] = bs;
                s += ccount[c];
                bs += (ccount[c] + vpb - 1) / vpb;
            }
            bpre[C_N] = bs;
        }
        DEC_SYNC();
#pragma unroll
        for (uint32_t j = 0; j < PMAX / NT; ++j) {
            const uint32_t i = j * NT + tid;
            if (j * NT + wave * RR_WAVE >= nv) continue;
#pragma unroll
            for (uint32_t c = 0; c < C_N; ++c) {
                const uint64_t m = __ballot(myc[j] == c);
                if (m) {
                    uint32_t at = 0;
                    if (lane == 0) at = atomicAdd(&ccur[c], (uint32_t)__popcll(m));
                    at = __builtin_amdgcn_readfirstlane(at);   // (lane 0 took the atomic)
                    if (myc[j] == c) perm[cbase[c] + at + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint16_t)i;
                }
            }
        }
    };
    if (v_end > v_lo) sort_chunk(v_lo);   // (with the window's loads still in flight)
#if RR_DEC_OVL
    if (ovl) ov_finish();   // they have landed under the sort
#if RR_DEC_EBPF
    asm volatile("" ::"v"(ebpf));   // (landed with the window's loads: keeps the touch alive)
#endif
#endif
    for (uint64_t c0 = v_lo; c0 < v_end; c0 += PMAX) {
        if (c0 != v_lo) {
            DEC_SYNC();   // every wave is done with the previous chunk's batches
            sort_chunk(c0);
        }
        DEC_SYNC();   // the stage and the chunk's sort are complete

        PROBE(if (c0 == v_lo) pt2 = __builtin_amdgcn_s_memtime();)
        // 3. single-class batches, taken dynamically by the waves
#if defined(RR_ABLATE) && RR_ABLATE == 2
        const uint32_t nb = 0;
#else
        const uint32_t nb = bpre[C_N];
#endif
#if RR_DEC_BREG   // the chunk's batch prefixes, read once (wave-uniform)
        uint32_t bp[C_N + 1];
#pragma unroll
        for (uint32_t k = 0; k <= C_N; ++k) bp[k] = __builtin_amdgcn_readfirstlane(bpre[k]);
#endif
        for (;;) {
            uint32_t bi = 0;
            if (lane == 0) bi = atomicAdd(&next_batch, 1u);
            bi = __builtin_amdgcn_readfirstlane(bi);
            if (bi >= nb) break;
#if RR_DEC_BREG
            uint32_t k = 0, bk = bp[0];
#pragma unroll
            for (uint32_t i = 1; i < C_N; ++i) {
                const bool ge = bi >= bp[i];
                k = ge ? i : k;
                bk = ge ? bp[i] : bk;
            }
            const uint32_t c = class_at(k);
#define BPRE_K bk
#else
            uint32_t k = 0;
            while (bi >= bpre[k + 1]) ++k;
            const uint32_t c = CLASS_ORDER[k];
#define BPRE_K bpre[k]
#endif
#if RR_DEC_BALANCE   // the class's values split evenly over its batches (same batch count)
            const uint32_t vpb0 = class_vpb(c), nbc = (ccount[c] + vpb0 - 1) / vpb0;
            const uint32_t vpb = (ccount[c] + nbc - 1) / nbc;
#else
            const uint32_t vpb = class_vpb(c);
#endif
            const uint32_t first = cbase[c] + (bi - BPRE_K) * vpb;
            const uint32_t cnt = min(ccount[c] - (bi - BPRE_K) * vpb, vpb);
#undef BPRE_K
#ifdef RR_SKIP_CLASSES   // timing-only builds (tools/): skip the batches of these classes
            if ((RR_SKIP_CLASSES >> c) & 1) continue;
#endif
            PROBE(const uint64_t tb0 = __builtin_amdgcn_s_memtime();)
#if RR_DEC_PRIO == 1   // the long chained classes issue ahead of the other waves of their SIMD
            if (c == C_HH || c == C_ZL || c == C_LIST || c == C_HT) __builtin_amdgcn_s_setprio(2);
#elif RR_DEC_PRIO == 2   // every walk ahead of the copy / sort phases of the other workgroup
            __builtin_amdgcn_s_setprio(1);
#endif
            // lanes per value: ziplists 2 (two-ended walk), chained classes 64 / cnt (grouped walks)
            const bool grouped = c == C_LIST || c == C_SL || c == C_IS || (RR_ZL_BACK && c == C_ZL);
            const uint32_t Gw = max(1u, min(GMAX, (uint32_t)RR_WAVE / cnt));
#if RR_HT_GROUPED   // grouped hash-table walks when a value gets lanes enough for its keys
            const bool htg = (c == C_HT || c == C_HH) && Gw >= ht_group_min(c == C_HH);
#else
            const bool htg = false;
#endif
            // (hash tables: a power of two, so a value's lanes lie in one DPP row, do_ht_g)
            const uint32_t Gh = 1u << (31 - __builtin_clz(Gw));
            const bool pow2 = htg || (RR_ZL_PIPE && c == C_ZL) || (RR_LIST_PIPE && c == C_LIST);   // (ziplists: G 4, 8 or 16)
            const uint32_t G = __builtin_amdgcn_readfirstlane((c == C_ZL && !RR_ZL_BACK) ? 2u : pow2 ? Gh : grouped ? Gw : 1u);
            const uint32_t li = lane / G, g = lane - li * G;   // the value's index in the batch
            const bool active = li < cnt;
            const uint64_t v = c0 + (active ? perm[first + li] : 0u);
            uint64_t eb_v = eb0, r_v = 0;
            if (active) { eb_v = ebase[v]; r_v = ebase[v + 1] - eb_v; }
#ifndef RR_DEC_NOGLOBAL
            const Acc a = staged ? run_batch(lsrc, c, active, v, G, g, S0, E, eb0, blob, offsets, eb_v, r_v, values, elems,
                                             cap, fix)
                                 : run_batch_g(gsrc, c, active, v, G, g, S0, E, eb0, blob, offsets, eb_v, r_v, values,
                                               elems, cap, fix);
#else   // timing-only builds (tools/): no unstaged walks (wrong for windows that overflow the stage)
            const Acc a = run_batch(lsrc, c, active, v, G, g, S0, E, eb0, blob, offsets, eb_v, r_v, values, elems, cap, fix);
            (void)gsrc;
#endif
#if RR_DEC_PRIO
            __builtin_amdgcn_s_setprio(0);
#endif
            bad += a.bad;
            pay += a.pay;
            PROBE(if (lane == 0) {
                atomicAdd((unsigned long long *)&prb[3 + c], (unsigned long long)(__builtin_amdgcn_s_memtime() - tb0));
                atomicAdd((unsigned long long *)&prb[3 + C_N + c], 1ull);
                atomicAdd((unsigned long long *)&prb[3 + 2 * C_N + c], (unsigned long long)cnt);
            })
        }
    }
#if RR_DEC_PF
    {   // 4'. the next window's mirror-arena copy, 4 KiB tasks taken by waves with no batch left
        const uint32_t ntile = tile + gridDim.x;
        const uint64_t nW0 = (uint64_t)ntile * W, nW1 = nW0 + W < padded ? nW0 + W : padded;
        if (ntile < nwin && nW1 > nW0) {
            if (v_end == v_lo) DEC_SYNC();   // (no chunk ran: order next_copy's reset)
            const uint64_t cw0 = nW0 >> 4, cw1 = nW1 >> 4;
            constexpr uint32_t TASK = 4 * RR_WAVE;   // 16-byte granules per task
            const uint32_t ntask = (uint32_t)((cw1 - cw0 + TASK - 1) / TASK);
            // buffer resources over the next window: no exec-mask branches around the stores
            const rsrc_t RL = make_rsrc(blob + nW0, (uint32_t)(nW1 - nW0));
            const rsrc_t RA = make_rsrc(arena + nW0, (uint32_t)(nW1 - nW0));
            for (;;) {
                uint32_t ti = 0;
                if (lane == 0) ti = atomicAdd(&next_copy, 1u);
                ti = __builtin_amdgcn_readfirstlane(ti);
                if (ti >= ntask) break;
                u32x4 x[4];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    x[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         RL, (int)((ti * TASK + lane + k * RR_WAVE) * 16), 0, 0));
#pragma unroll
                for (int k = 0; k < 4; ++k) {
#ifndef RR_ABLATE_NOCOPY
                    __builtin_amdgcn_raw_buffer_store_b128(x[k], RA, (int)((ti * TASK + lane + k * RR_WAVE) * 16), 0, 2);
#endif
                }
            }
        }
    }
#endif
#if RR_DEC_LATECOPY && !RR_DEC_EARLY
    // 4. the window's mirror-arena copy in 4 KiB tasks, taken by each wave as soon as it has no
    //    batch left (from the LDS stage where the window's bytes are staged, else from global)
    {
        if (v_end == v_lo) __syncthreads();   // (no chunk ran: order next_copy's reset)
        const u32x4 *src = reinterpret_cast<const u32x4 *>(blob);
        u32x4 *dst = reinterpret_cast<u32x4 *>(arena);
        const u32x4 *lds = reinterpret_cast<const u32x4 *>(stage);
        const uint64_t cw0 = W0 >> 4, cw1 = W1 >> 4, cs0 = S0 >> 4, cs1 = staged ? S1 >> 4 : cs0;
        constexpr uint32_t TASK = 4 * RR_WAVE;   // 16-byte granules per task
        const uint32_t ntask = (uint32_t)((cw1 - cw0 + TASK - 1) / TASK);
        for (;;) {
            uint32_t ti = 0;
            if (lane == 0) ti = atomicAdd(&next_copy, 1u);
            ti = __builtin_amdgcn_readfirstlane(ti);
            if (ti >= ntask) break;
            const uint64_t g0 = cw0 + (uint64_t)ti * TASK + lane;
            u32x4 x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t g = g0 + k * RR_WAVE;
                if (g < cw1) x[k] = g >= cs0 && g < cs1 ? lds[g - cs0] : src[g];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t g = g0 + k * RR_WAVE;
                if (g < cw1) __builtin_nontemporal_store(x[k], dst + g);
            }
        }
    }
#endif
    bad = wave_sum_fast(bad);
    pay = wave_sum_fast(pay);
    if (lane == 0) { red[0][wave] = bad; red[1][wave] = pay; }
    DEC_SYNC();
    if (tid == 0) {
        uint64_t tb = 0, tp = 0;
        for (uint32_t w = 0; w < NW; ++w) { tb += red[0][w]; tp += red[1][w]; }
#if RR_DEC_ATOT
        // the window's {bad, payload} straight into the call's totals (zeroed by count_kernel):
        // two non-returning atomics per window, ~7K per call spread over the kernel, so
        // decode_post has no fold to do (7.3 -> 5.6 us)
        (void)stats;
        if (tot && tb) atomicAdd((unsigned long long *)&tot->n_bad, (unsigned long long)tb);
        if (tot && tp) atomicAdd((unsigned long long *)&tot->payload, (unsigned long long)tp);
#else
        (void)tot;
        stats[3 * (uint64_t)tile + 0] = tb;
        stats[3 * (uint64_t)tile + 1] = tp;
        stats[3 * (uint64_t)tile + 2] = 0;
#endif
        PROBE(prb[0] = pt1 - pt0; prb[1] = pt2 - pt1; prb[2] = __builtin_amdgcn_s_memtime() - pt2; prb[28] = v_hi - v_lo;
              prb[29] = staged; if (g_probe) for (uint32_t i = 0; i < PROBE_WORDS; ++i) g_probe[(uint64_t)tile * PROBE_WORDS + i] = prb[i];)
    }
    }   // window
}

// ---- fused decode: one pass over the windows -------------------------------------------
// decode_fused_kernel replaces count_kernel + scan_kernel + decode_kernel: a window classifies
// and reserves its own values from its LDS stage (pass A, thread per value; a List walks its
// length chain in LDS), publishes the window's descriptor total right away, sorts its values by
// class and lays out their window-relative slot offsets while the earlier windows' totals come
// in, then resolves its first slot by a decoupled look-back over the windows (rr_device.h) and
// walks + emits the single-class batches as decode_kernel does.  No value header is read from
// global memory twice.  dec_index_kernel before it only reads the offsets (the first value of
// every window) and zeroes the call's words.

// reserve_classify over a byte source (the LDS stage, or global memory through a buffer
// resource for a window whose values overflow the stage): same results, byte for byte
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {   // a wave-uniform 64-bit value into SGPRs
    return (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)x) |
           ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32);
}

template <class Src>
__device__ __forceinline__ void classify_reserve_src(const Src &S, uint32_t q, uint64_t L, const uint8_t *b_glb,
                                                     uint32_t &c, uint64_t &r) {
    r = 0;
    c = C_EXACT;
    if (L < 5) return;
    uint32_t d[6];
    S.template get<6>(q, d);
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
        case RR_TYPE_LIST_QUICKLIST: {   // the length chain (the count the walk will take)
            c = C_LIST;
            uint64_t p = 5, n = 0;
            while (p < L) {
                if (L - p < 4) break;
                uint32_t x[1];
                S.template get<1>(q + (uint32_t)p, x);
                const uint64_t l = x[0];
                if (l > L - p - 4) break;
                ++n;
                p += 4 + l;
            }
            r = n;
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
            r = 1 + zl_walk_count_g(b_glb + 13, Lz);   // (a saturated count: rare, from global memory)
            return;
        }
        default:
            return;
    }
}

// zeroes the call's words (window look-back state, fixup header, totals) and finds the first
// value of every window from the offsets alone
__global__ __launch_bounds__(256) void dec_index_kernel(const uint64_t *__restrict__ offsets, uint64_t n,
                                                        uint32_t *__restrict__ first_val, uint32_t nwin, uint32_t win,
                                                        uint64_t *zero_words, uint32_t nzero, rr_totals *tot) {
    zero_call_words(zero_words, nzero, tot);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const uint64_t o_hi = offsets[i];
    const uint64_t w_lo = i == 0 ? 0 : offsets[i - 1] / win + 1;
    const uint64_t w_hi = i == n ? nwin : o_hi / win;
    for (uint64_t w = w_lo; w <= w_hi && w <= nwin; ++w) first_val[w] = (uint32_t)i;
}

template <uint32_t W, uint32_t SLACK, uint32_t NW, uint32_t PMAX>
__global__ __launch_bounds__(NW * RR_WAVE) DEC_WPE_ATTR void decode_fused_kernel(
    const uint8_t *__restrict__ blob, uint64_t data_cap, const uint64_t *__restrict__ offsets, uint64_t n,
    const uint32_t *__restrict__ first_val, uint8_t *__restrict__ cls, uint32_t *__restrict__ cnt,
    rr_value *__restrict__ values, rr_elem *__restrict__ elems, uint64_t elem_cap, uint8_t *__restrict__ arena,
    uint64_t *__restrict__ stats, uint64_t *fix, uint32_t nwin, uint64_t *lb_state, uint64_t *lb_groups,
    uint64_t *total) {
    constexpr uint32_t NT = NW * RR_WAVE, STAGE = W + SLACK;
    // a chunk of values is one pass-A round: thread i holds value i of every chunk, so the class
    // and reservation it wrote for a later chunk are its own writes when it reads them back
    static_assert(PMAX == NT && W % 16 == 0 && SLACK % 16 == 0, "tile shape");
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE + 64];
    __shared__ uint16_t perm[PMAX];
    __shared__ uint32_t eloc[PMAX + 1];   // window-relative first slot of the chunk's values
    __shared__ uint32_t ccount[C_N], cbase[C_N], ccur[C_N], bpre[C_N + 1];
    __shared__ uint32_t next_batch;
    __shared__ uint64_t red[2][NW];
    __shared__ uint64_t sh_eb0;
    PROBE(__shared__ uint64_t prb[PROBE_WORDS]; uint64_t pt0 = __builtin_amdgcn_s_memtime(), pt1 = 0, pt2 = 0;
          if (threadIdx.x < PROBE_WORDS) prb[threadIdx.x] = 0;)
    const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid / RR_WAVE;
    const uint32_t tile = blockIdx.x;
    const uint64_t padded = (offsets[n] + 15) & ~15ull;
    const uint64_t W0 = (uint64_t)tile * W;
    const uint64_t W1 = W0 + W < padded ? W0 + W : padded;
    const uint64_t A0 = W0 > (offsets[0] & ~15ull) ? W0 : (offsets[0] & ~15ull);
    // 1. the window's loads (as decode_kernel: buffer resources, no exec-mask branches)
    constexpr uint32_t KM = W / 16 / NT;
    static_assert(W % (16 * NT) == 0, "window granules per thread");
    const uint64_t ov_a = A0 >> 4, ov_w1 = W1 >> 4;
    const uint32_t ov_mb = ov_w1 > ov_a ? (uint32_t)((ov_w1 - ov_a) * 16) : 0u;
    const rsrc_t ov_RM = make_rsrc(blob + A0, ov_mb);
    const rsrc_t ov_RA = make_rsrc(arena + A0, ov_mb);
    u32x4 ov_m[KM];
#pragma unroll
    for (uint32_t k = 0; k < KM; ++k)
        ov_m[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ov_RM, (int)((tid + k * NT) * 16), 0, 0));
    const uint64_t v_lo = first_val[tile], v_hi = first_val[tile + 1];
    uint64_t S0 = W0, S1 = W0;
    if (v_hi > v_lo) {
        S0 = offsets[v_lo] & ~15ull;
        S1 = (offsets[v_hi] + 15) & ~15ull;
    }
    const bool staged = S1 - S0 <= STAGE;
    const uint64_t cap = elem_cap < 0xFFFFFFFFull ? elem_cap : 0xFFFFFFFFull;   // elem_base is 32-bit
    constexpr uint32_t KT = (SLACK / 16 + NT - 1) / NT;
    const uint64_t ov_t0 = ov_w1 > ov_a ? ov_w1 : ov_a;
    const uint64_t ov_te = (staged && S1 > W1 ? S1 : W1) >> 4;
    const rsrc_t ov_RT = make_rsrc(blob + ov_t0 * 16, ov_te > ov_t0 ? (uint32_t)((ov_te - ov_t0) * 16) : 0u);
    u32x4 ov_t[KT];
#pragma unroll
    for (uint32_t k = 0; k < KT; ++k)
        ov_t[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ov_RT, (int)((tid + k * NT) * 16), 0, 0));
    // the window's first values' offsets, loaded while the window lands
    const uint64_t v0 = v_lo + tid;
    uint64_t o0 = 0, o1 = 0;
    if (v0 < v_hi) { o0 = offsets[v0]; o1 = offsets[v0 + 1]; }
    // 2. window -> arena (nontemporal), value bytes -> the LDS stage
    {
        const uint64_t ov_s0 = S0 >> 4;
        typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
        lds_u32x4 *ov_lds = (lds_u32x4 *)(__attribute__((address_space(3))) uint8_t *)stage;
        auto ov_slot = [&](uint64_t g) __attribute__((always_inline)) -> uint32_t {
            return (staged & (g >= ov_s0) & (g < ov_te)) ? (uint32_t)(g - ov_s0) : STAGE / 16;
        };
#pragma unroll
        for (uint32_t k = 0; k < KM; ++k) {
            __builtin_amdgcn_raw_buffer_store_b128(ov_m[k], ov_RA, (int)((tid + k * NT) * 16), 0, 2 /* nt */);
            ov_lds[ov_slot(ov_a + tid + (uint64_t)k * NT)] = ov_m[k];
        }
#pragma unroll
        for (uint32_t k = 0; k < KT; ++k) ov_lds[ov_slot(ov_t0 + tid + (uint64_t)k * NT)] = ov_t[k];
    }
    const bool far = !staged && S1 - S0 > 0xFFFFFF00ull;
    const LdsSrc lsrc{(lds_cptr)stage};
    const GlbSrc gsrc{make_rsrc(blob + S0, (uint32_t)(data_cap - S0 < 0xFFFFFFFFull ? data_cap - S0 : 0xFFFFFFFFull))};
    DEC_SYNC();   // the stage is complete
    PROBE(pt1 = __builtin_amdgcn_s_memtime();)

    // 3. pass A: class and reservation of every value of the window (thread per value); the
    //    first chunk's stay in registers, later chunks' go to cls / cnt for the same thread
    uint32_t c_first = C_N;
    uint64_t r_first = 0, agg = 0;
    for (uint64_t r0 = v_lo; r0 < v_hi; r0 += NT) {
        const uint64_t v = r0 + tid;
        uint32_t c = C_N;
        uint64_t r = 0;
        if (v < v_hi) {
            const uint64_t o = r0 == v_lo ? o0 : offsets[v], o_end = r0 == v_lo ? o1 : offsets[v + 1];
            const uint64_t L = o_end - o;
            if (far) {
                c = C_EXACT;
                r = reserve_g(blob + o, L);
            } else if (staged) {
                classify_reserve_src(lsrc, (uint32_t)(o - S0), L, blob + o, c, r);
            } else {
                classify_reserve_src(gsrc, (uint32_t)(o - S0), L, blob + o, c, r);
            }
            r = r < 0xFFFFFFFFull ? r : 0xFFFFFFFFull;
            if (r0 == v_lo) { c_first = c; r_first = r; }
        }
        agg += r;
    }
    // (a later chunk classifies its values again in step 4: a class written to global memory
    // here and read back there could come from a stale line of the CU's L1, which the other
    // workgroup on the CU may have filled; only multi-chunk windows pay this)
    (void)cls; (void)cnt;
    agg = wave_sum(agg);
    if (lane == 0) red[0][wave] = agg;
    DEC_SYNC();
    agg = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) agg += red[0][w];
    agg = rfl64(agg);
#ifdef RR_FUSED_NOLB   // timing-only builds (tools/): no look-back (every window's first slot is 0: wrong)
    const bool nolb = true;
#else
    const bool nolb = false;
#endif
    if (wave == 0 && !nolb) lb_publish(lb_state, lb_groups, tile, agg);   // the window's total, as early as possible
    // a window whose descriptor byte offsets overflow the 32-bit slot resource: exact parser
    const bool far2 = far || agg * 16 >= NOSLOT;
    PROBE(pt2 = __builtin_amdgcn_s_memtime();)

    uint64_t bad = 0, pay = 0;
    bool have_eb0 = false;
    uint64_t eb0 = 0;
    uint32_t run = 0;   // window-relative slots of the earlier chunks
    for (uint64_t c0 = v_lo; c0 < v_hi; c0 += PMAX) {
        const uint32_t nv = (uint32_t)(v_hi - c0 < PMAX ? v_hi - c0 : PMAX);
        if (tid < C_N) { ccount[tid] = 0; ccur[tid] = 0; }
        if (tid == 0) next_batch = 0;
        DEC_SYNC();   // (also: every wave is done with the previous chunk's batches)
        // 4. counting sort of the chunk by class + its window-relative slot offsets
        const uint64_t v = c0 + tid;
        const bool in = tid < nv;
        uint32_t myc = C_N, myr = 0;
        if (in) {
            if (c0 == v_lo) { myc = c_first; myr = (uint32_t)r_first; }
            else {
                const uint64_t o = offsets[v], L = offsets[v + 1] - o;
                uint64_t r = 0;
                if (far) { myc = C_EXACT; r = reserve_g(blob + o, L); }
                else if (staged) classify_reserve_src(lsrc, (uint32_t)(o - S0), L, blob + o, myc, r);
                else classify_reserve_src(gsrc, (uint32_t)(o - S0), L, blob + o, myc, r);
                myr = (uint32_t)(r < 0xFFFFFFFFull ? r : 0xFFFFFFFFull);
            }
            myc = far2 ? C_EXACT : myc;
        }
        if (wave * RR_WAVE < nv) {
#pragma unroll
            for (uint32_t c = 0; c < C_N; ++c) {
                const uint64_t m = __ballot(myc == c);
                if (m && lane == 0) atomicAdd(&ccount[c], (uint32_t)__popcll(m));
            }
        }
        const uint64_t incl = wave_incl_scan((uint64_t)myr);
        if (lane == RR_WAVE - 1) red[1][wave] = incl;
        DEC_SYNC();
        uint64_t wpre = 0, ctot = 0;
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) {
            const uint64_t x = red[1][w];
            wpre += w < wave ? x : 0;
            ctot += x;
        }
        ctot = rfl64(ctot);
        if (in) eloc[tid] = run + (uint32_t)(wpre + incl - myr);
        if (tid == 0) {
            eloc[nv] = run + (uint32_t)ctot;
            uint32_t s = 0, bs = 0;
            for (uint32_t k = 0; k < C_N; ++k) {
                const uint32_t c = CLASS_ORDER[k];
                const uint32_t vpb = class_vpb(c);
                cbase[c] = s;
                bpre[k] = bs;
                s += ccount[c];
                bs += (ccount[c] + vpb - 1) / vpb;
            }
            bpre[C_N] = bs;
        }
        run += (uint32_t)ctot;
        DEC_SYNC();
        if (wave * RR_WAVE < nv) {
#pragma unroll
            for (uint32_t c = 0; c < C_N; ++c) {
                const uint64_t m = __ballot(myc == c);
                if (m) {
                    uint32_t at = 0;
                    if (lane == 0) at = atomicAdd(&ccur[c], (uint32_t)__popcll(m));
                    at = __builtin_amdgcn_readfirstlane(at);   // (lane 0 took the atomic)
                    if (myc == c) perm[cbase[c] + at + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint16_t)tid;
                }
            }
        }
        // 5. the window's first slot: the look-back over the earlier windows' totals (resolved
        //    once, by wave 0, after the first chunk's sort — their totals had time to arrive)
        if (!have_eb0) {
            if (nolb) { if (tid == 0) sh_eb0 = 0; }
            else if (wave == 0) {
                const uint64_t pre = lb_resolve(lb_state, lb_groups, tile, nwin, agg, fix + 1);
                if (lane == 0) {
                    sh_eb0 = pre;
                    if (tile == nwin - 1) *total = pre + agg;
                }
            }
            have_eb0 = true;
        }
        DEC_SYNC();   // the chunk's sort, its slot offsets and the window's first slot are complete
        eb0 = rfl64(sh_eb0);
        // the window's descriptor slots [eb0, eb0 + agg), cut at the capacity
        const uint64_t eb1 = eb0 + agg;
        const uint64_t ecut = eb1 < cap ? eb1 : cap;
        const rsrc_t E = make_rsrc(reinterpret_cast<const uint8_t *>(elems + eb0),
                                   far2 || ecut <= eb0 ? 0u : (uint32_t)((ecut - eb0) * 16));
        // 6. single-class batches, taken dynamically by the waves
        const uint32_t nb = __builtin_amdgcn_readfirstlane(bpre[C_N]);
        for (;;) {
            uint32_t bi = 0;
            if (lane == 0) bi = atomicAdd(&next_batch, 1u);
            bi = __builtin_amdgcn_readfirstlane(bi);
            if (bi >= nb) break;
            uint32_t k = 0;
            while (bi >= bpre[k + 1]) ++k;
            const uint32_t c = CLASS_ORDER[k];
            const uint32_t vpb = class_vpb(c);
            const uint32_t first = cbase[c] + (bi - bpre[k]) * vpb;
            const uint32_t bcnt = min(ccount[c] - (bi - bpre[k]) * vpb, vpb);
            PROBE(const uint64_t tb0 = __builtin_amdgcn_s_memtime();)
            const bool grouped = c == C_LIST || c == C_SL || c == C_IS || (RR_ZL_BACK && c == C_ZL);
            const uint32_t Gw = max(1u, min(GMAX, (uint32_t)RR_WAVE / bcnt));
#if RR_HT_GROUPED
            const bool htg = (c == C_HT || c == C_HH) && Gw >= ht_group_min(c == C_HH);
#else
            const bool htg = false;
#endif
            const uint32_t Gh = 1u << (31 - __builtin_clz(Gw));
            const bool pow2 = htg || (RR_ZL_PIPE && c == C_ZL) || (RR_LIST_PIPE && c == C_LIST);   // (ziplists: G 4, 8 or 16)
            const uint32_t G = __builtin_amdgcn_readfirstlane((c == C_ZL && !RR_ZL_BACK) ? 2u : pow2 ? Gh : grouped ? Gw : 1u);
            const uint32_t li = lane / G, g = lane - li * G;
            const bool active = li < bcnt;
            const uint32_t pi = active ? perm[first + li] : 0u;
            const uint64_t vv = c0 + pi;
            const uint64_t eb_v = eb0 + eloc[pi], r_v = active ? eloc[pi + 1] - eloc[pi] : 0;
            const Acc a = staged ? run_batch(lsrc, c, active, vv, G, g, S0, E, eb0, blob, offsets, eb_v, r_v, values,
                                             elems, cap, fix)
                                 : run_batch_g(gsrc, c, active, vv, G, g, S0, E, eb0, blob, offsets, eb_v, r_v, values,
                                               elems, cap, fix);
            bad += a.bad;
            pay += a.pay;
            PROBE(if (lane == 0) {
                atomicAdd((unsigned long long *)&prb[3 + c], (unsigned long long)(__builtin_amdgcn_s_memtime() - tb0));
                atomicAdd((unsigned long long *)&prb[3 + C_N + c], 1ull);
                atomicAdd((unsigned long long *)&prb[3 + 2 * C_N + c], (unsigned long long)bcnt);
            })
        }
    }
    if (v_hi == v_lo && wave == 0 && !nolb) {   // a window with no values still takes part in the look-back
        const uint64_t pre = lb_resolve(lb_state, lb_groups, tile, nwin, agg, fix + 1);
        if (lane == 0 && tile == nwin - 1) *total = pre + agg;
    }
    bad = wave_sum_fast(bad);
    pay = wave_sum_fast(pay);
    if (lane == 0) { red[0][wave] = bad; red[1][wave] = pay; }
    DEC_SYNC();
    if (tid == 0) {
        uint64_t tb = 0, tp = 0;
        for (uint32_t w = 0; w < NW; ++w) { tb += red[0][w]; tp += red[1][w]; }
        stats[3 * (uint64_t)tile + 0] = tb;
        stats[3 * (uint64_t)tile + 1] = tp;
        stats[3 * (uint64_t)tile + 2] = 0;
        PROBE(prb[0] = pt1 - pt0; prb[1] = pt2 - pt1; prb[2] = __builtin_amdgcn_s_memtime() - pt2; prb[28] = v_hi - v_lo;
              prb[29] = staged; if (g_probe) for (uint32_t i = 0; i < PROBE_WORDS; ++i) g_probe[(uint64_t)tile * PROBE_WORDS + i] = prb[i];)
    }
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

#ifndef RR_SCAN_DPP   // 1: block_excl_scan's wave scan in DPP (u32) when no lane's value reaches 2^26
#define RR_SCAN_DPP 1
#endif
template <uint32_t NT>
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t x, uint64_t *wsum, uint64_t &total) {
#if RR_SCAN_DPP   // (64 lanes below 2^26 each: the wave's sum fits 32 bits; else the u64 shuffles)
    const uint64_t incl = __ballot(x >= (1ull << 26)) == 0 ? (uint64_t)wave_incl_scan_u32((uint32_t)x) : wave_incl_scan(x);
#else
    const uint64_t incl = wave_incl_scan(x);
#endif
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

// ---- K4: fixup of queued values ----------------------------------------------------------
// A workgroup per queued value (atomic ticket over the list the walks filled):
//   SET_HT / HASH_HT  exact duplicate-key test — fingerprints of (length, first and last 8
//                     bytes) in an LDS open-addressing table, byte comparison on a fingerprint
//                     match; a value with more keys than fit runs in several passes, each over
//                     one residue class of the fingerprints.  A hash with a repeated field gets
//                     RR_E_DUP (desHash's serverAssert, rock_serdes.c:399-400); a set keeps the
//                     first copy of each member (desSet's dictAdd, :297): later copies are marked
//                     and the descriptors compacted in place, the freed tail slots zeroed.
//   ZSET_SKIPLIST     pairs re-sorted in place into serZset's order (descending score, then
//                     member, equal keys in blob order — the skiplist desZset builds, t_zset.c:
//                     132-180) by a bitonic network over the descriptor pairs in global memory.
// Totals changes go to fix[2] (bad values) / fix[3] (payload, two's complement), folded by the
// finalize kernel.  Only values the walks could not clear arrive here: none in a batch of
// serObject output whose hash tables hold at most HT_FP_KEYS keys, barring 16-bit fingerprint
// collisions.
constexpr uint32_t FIX_NT = 256, FIX_TAB = 8192, FIX_TAB_BITS = 13, FIX_PASS_KEYS = 2048;
#ifndef RR_POST_FOLD_BLOCKS   // blocks of the decode's post kernel that fold the window totals
#define RR_POST_FOLD_BLOCKS 32
#endif

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

__device__ void fix_sort_skiplist(const uint8_t *__restrict__ blob, rr_elem *__restrict__ el, uint32_t np) {
    uint4 *P = reinterpret_cast<uint4 *>(el);   // pair i = P[2i] (member), P[2i + 1] (score)
    uint32_t m = 1;
    while (m < np) m <<= 1;
    // bitonic network with every comparator ascending (first step of each merge compares
    // mirrored positions): positions >= np act as +infinity and are never touched
    for (uint32_t k = 2; k <= m; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < m / 2; t += FIX_NT) {
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

__device__ __forceinline__ void fixup_values(const uint8_t *__restrict__ blob, uint64_t *fix,
                                             rr_value *__restrict__ values, rr_elem *__restrict__ elems,
                                             rr_totals *out) {
    __shared__ unsigned long long tab[FIX_TAB];
    __shared__ uint64_t wsum[FIX_NT / RR_WAVE];
    __shared__ uint32_t sh_flag;   // bit 0: a duplicate key, bit 1: a pass overflowed the table
    const uint32_t tid = threadIdx.x;
    const uint64_t nq = fix[0];
    const uint32_t *list = reinterpret_cast<const uint32_t *>(fix + FIX_HDR);
    // queued values are rare (none in serObject output with small hash tables): a static
    // stride over the queue, no ticket atomics on an empty one
    for (uint64_t t = blockIdx.x; t < nq; t += gridDim.x) {
        if (tid == 0) sh_flag = 0;
        __syncthreads();
        const uint32_t v = list[t];
        const uint4 rv = reinterpret_cast<const uint4 *>(values)[v];
        const uint32_t type = rv.x & 0xFF, n = rv.z;
        rr_elem *el = elems + rv.w;
        if (type == RR_TYPE_ZSET_SKIPLIST) {
            fix_sort_skiplist(blob, el, n / 2);
        } else {
            const uint32_t per = type == RR_TYPE_SET_HT ? 1 : 2, nk = n / per;
            uint32_t K = (nk + FIX_PASS_KEYS - 1) / FIX_PASS_KEYS;
            for (;;) {
                for (uint32_t r = 0; r < K; ++r) {
                    for (uint32_t j = tid; j < FIX_TAB; j += FIX_NT) tab[j] = 0;
                    __syncthreads();
                    for (uint32_t i = tid; i < nk; i += FIX_NT) {
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
                                    atomicOr(&sh_flag, 1u);
                                    break;
                                }
                            }
                            h = (h + 1) & (FIX_TAB - 1);
                            if (++probes == FIX_TAB) { atomicOr(&sh_flag, 2u); break; }
                        }
                    }
                    __syncthreads();
                    if (sh_flag & 2) break;
                }
                if (!(sh_flag & 2)) break;
                K *= 2;   // a residue class overflowed the table: finer classes (marks stay valid)
                __syncthreads();
                if (tid == 0) sh_flag &= ~2u;
                __syncthreads();
            }
            if (sh_flag & 1) {
                // compact the kept descriptors forward (a chunk is read before it is written,
                // and writes never pass the chunk's own positions), zero the freed tail
                uint64_t kept = 0, dropped = 0;
                for (uint32_t c0 = 0; c0 < n; c0 += FIX_NT) {
                    const uint32_t i = c0 + tid;
                    uint4 d = make_uint4(0, 0, 0, 0);
                    if (i < n) d = reinterpret_cast<const uint4 *>(el)[i];
                    const bool keep = i < n && (per == 2 || (d.w >> 16) == 0);
                    uint64_t tot;
                    const uint64_t pos = block_excl_scan<FIX_NT>(keep ? 1u : 0u, wsum, tot);
                    dropped += i < n && !keep ? d.z : 0;
                    __syncthreads();
                    if (keep && per == 1) reinterpret_cast<uint4 *>(el)[kept + pos] = d;
                    if (per == 2 && i < n) dropped += d.z;   // a hash with a repeated field loses all
                    kept += tot;
                    __syncthreads();
                }
                const uint32_t nk2 = per == 2 ? 0u : (uint32_t)kept;
                for (uint32_t i = nk2 + tid; i < n; i += FIX_NT) reinterpret_cast<uint4 *>(el)[i] = make_uint4(0, 0, 0, 0);
                dropped = wave_sum(dropped);
                if (lane_id() == 0 && dropped && out)
                    atomicAdd((unsigned long long *)&out->payload, (unsigned long long)(0ull - dropped));
                if (tid == 0) {
                    uint4 w = rv;
                    w.z = nk2;
                    if (per == 2) {
                        w.x = (rv.x & 0xFFFFu) | ((uint32_t)RR_E_DUP << 16);
                        if (out) atomicAdd((unsigned long long *)&out->n_bad, 1ull);
                    }
                    reinterpret_cast<uint4 *>(values)[v] = w;
                }
            }
        }
        __syncthreads();
    }
}

// ---- K4: the decode's last kernel: the fixup pass over the queued values (their totals
// changes added straight into the zeroed totals), then the fold of the windows' totals
__global__ __launch_bounds__(FIX_NT) void decode_post_kernel(const uint8_t *__restrict__ blob, uint64_t *fix,
                                                             rr_value *__restrict__ values,
                                                             rr_elem *__restrict__ elems,
                                                             const uint64_t *__restrict__ stats, uint64_t *state,
                                                             uint32_t ntiles, const uint64_t *__restrict__ offsets,
                                                             uint64_t n, rr_totals *out) {
    fixup_values(blob, fix, values, elems, out);
#if RR_DEC_ATOT   // (block 0 only: the bytes, the descriptor total and the error word)
    if (out) fold_totals(stats, state, 0, offsets, n, 2, out, nullptr, fix + 1, 1);
#else
    if (out) fold_totals(stats, state, ntiles, offsets, n, 2, out, nullptr, fix + 1, RR_POST_FOLD_BLOCKS);
#endif
}

// ---------------------------------------------------------------------------------------- encode
__device__ __forceinline__ bool fits_width(int64_t x, uint32_t w) {
    if (w == 8) return true;
    if (w == 4) return x >= INT32_MIN && x <= INT32_MAX;
    return x >= INT16_MIN && x <= INT16_MAX;
}


// Decimal digits of an unsigned magnitude (sdsll2str's length without the sign): compares,
// no divisions.
__device__ __forceinline__ uint32_t udigits(uint64_t v) {
    uint32_t l = 1;
    uint64_t p = 10;
#pragma unroll
    for (int k = 1; k < 20; ++k) {
        l += v >= p ? 1u : 0u;
        p = k < 19 ? p * 10 : p;
    }
    return l;
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

// Encode runs as five launches (one memset, no inter-workgroup waits beyond the scan's
// look-back):
//   E1 enc_size_kernel  workgroup per 256 values, element-parallel: blob size (0 for an
//                       unencodable value) into offsets[v], per-tile {bad, payload, descriptors};
//   E2 scan_kernel      in-place exclusive scan -> offsets[0..n];
//   E3 enc_index_kernel thread per value: first value of every W-byte output window, and the
//                       values that would cross data_cap (RR_E_CAPACITY, payload taken back);
//   E4 enc_emit_kernel  workgroup per W-byte output window: builds the window's bytes in an
//                       LDS image (headers and length fields by element-parallel tasks,
//                       payloads by 64-byte copy pieces), then stores it with 16-byte
//                       coalesced stores;
//   E5 finalize         totals.
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
// two block-wide exclusive scans sharing one barrier (ws: [2][NT / RR_WAVE])
#ifndef RR_ENC_SIZE_DPP   // 1: E1's per-round wave scans in DPP (u32) when no lane's cost reaches 2^26
#define RR_ENC_SIZE_DPP 1
#endif
template <uint32_t NT>
__device__ __forceinline__ void block_excl_scan2(uint64_t x, uint64_t y, uint64_t (*ws)[NT / RR_WAVE], uint64_t &ex,
                                                 uint64_t &ey, uint64_t &tx, uint64_t &ty) {
#if RR_ENC_SIZE_DPP   // (64 lanes below 2^26 each: the wave's sums fit 32 bits; else the u64 shuffles)
    const bool small = __ballot((x | y) >= (1ull << 26)) == 0;
    const uint64_t ix = small ? (uint64_t)wave_incl_scan_u32((uint32_t)x) : wave_incl_scan(x);
    const uint64_t iy = small ? (uint64_t)wave_incl_scan_u32((uint32_t)y) : wave_incl_scan(y);
#else
    const uint64_t ix = wave_incl_scan(x), iy = wave_incl_scan(y);
#endif
    const uint32_t wv = threadIdx.x / RR_WAVE;
    if (lane_id() == RR_WAVE - 1) { ws[0][wv] = ix; ws[1][wv] = iy; }
    lds_barrier();
    uint64_t px = 0, py = 0, sx = 0, sy = 0;
#pragma unroll
    for (uint32_t k = 0; k < NT / RR_WAVE; ++k) {
        const uint64_t a = ws[0][k], b = ws[1][k];
        px += k < wv ? a : 0;
        py += k < wv ? b : 0;
        sx += a;
        sy += b;
    }
    ex = px + ix - x;
    ey = py + iy - y;
    tx = sx;
    ty = sy;
}

#ifndef RR_ENC_SIZE_U   // task rounds whose descriptors are loaded together
#define RR_ENC_SIZE_U 2
#endif
#ifndef RR_ENC_SHORT   // values with at most this many tasks are costed by their own lane
#define RR_ENC_SHORT 4
#endif
constexpr uint32_t ENC_SHORT = RR_ENC_SHORT;
#ifndef RR_ENC_SIZE_PF   // descriptor lines of a long value prefetched by E1 before its task rounds
#define RR_ENC_SIZE_PF 0
#endif
#ifndef RR_ENC_SIZE_SEG   // 1: E1 sums a value's task costs by wave-segmented LDS atomics (no per-round barrier)
#define RR_ENC_SIZE_SEG 1
#endif
#ifndef RR_ENC_SIZE_MAP   // 1: E1 maps tasks to values through an LDS map (blocks of <= ENC_MAPCAP tasks)
#define RR_ENC_SIZE_MAP 1
#endif
constexpr uint32_t ENC_MAPCAP = 4096;
// Task -> value map of a round of NT values (the value's index at each of its tasks, u8), from
// the task bases: the value with tasks writes its index at its first task (the head), then a
// running max fills the runs — heads increase along the map, so the zeros between them (the map
// was zeroed beforehand, ordered by a barrier) never win: 16 positions a thread, the carry across
// threads by a DPP max scan and the waves' maxima in LDS.  Returns whether the round's tt tasks
// fit the map (block-uniform); ends with an LDS barrier either way.
// The last j in [0, NT) with tb[j] <= t, for a non-decreasing tb[0..NT] with tb[0] <= t: two
// rounds of independent LDS reads instead of log2(NT) dependent ones — the 16 bucket heads
// tb[16k] (compared all at once), then the 16 entries of the chosen bucket (four 16-byte reads).
template <uint32_t NT>
__device__ __forceinline__ uint32_t search_last_le(const uint32_t *tb, uint32_t t) {
    static_assert(NT == 256, "16 buckets of 16");
    uint32_t b = 0;
#pragma unroll
    for (uint32_t k = 1; k < 16; ++k) b += tb[16 * k] <= t ? 1u : 0u;
    const uint4 *q = reinterpret_cast<const uint4 *>(tb + 16 * b);
    uint32_t c = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint4 x = q[k];
        c += (x.x <= t ? 1u : 0u) + (x.y <= t ? 1u : 0u) + (x.z <= t ? 1u : 0u) + (x.w <= t ? 1u : 0u);
    }
    return 16 * b + c - 1;
}
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
#ifndef RR_ENC_SIZE_WPE   // waves per SIMD E1 is built for (0: the compiler's choice)
#define RR_ENC_SIZE_WPE 0
#endif
#if RR_ENC_SIZE_WPE > 0
#define ENC_SIZE_WPE_ATTR __attribute__((amdgpu_waves_per_eu(RR_ENC_SIZE_WPE)))
#else
#define ENC_SIZE_WPE_ATTR
#endif
template <uint32_t NT, uint32_t U>
__global__ __launch_bounds__(NT) ENC_SIZE_WPE_ATTR void enc_size_kernel(const rr_value *__restrict__ values,
                                                      const rr_elem *__restrict__ elems, uint64_t n,
                                                      uint64_t ecap, uint64_t acap,
                                                      uint64_t *__restrict__ sizes, uint64_t *__restrict__ stats,
                                                      uint64_t *zero_words, uint32_t nzero, rr_totals *tot) {
    zero_call_words(zero_words, nzero, tot);
    __shared__ uint32_t tb[NT + 1];                  // first task of each value
    __shared__ uint32_t s_el[NT], s_te[NT], s_bad[NT];
    __shared__ uint64_t s_b0[NT], s_b1[NT], s_p0[NT], s_p1[NT];   // byte / payload scans at the first task, after the last
    __shared__ uint64_t ws0[NT / RR_WAVE], ws[2][2][NT / RR_WAVE];
    __shared__ uint64_t red[3][NT / RR_WAVE];
#if RR_ENC_SIZE_MAP
    // task -> value map of the block when it has at most ENC_MAPCAP tasks (build_task_map): one
    // LDS read per task instead of a binary search of the task bases
    __shared__ __attribute__((aligned(16))) uint8_t tmap[ENC_MAPCAP];
    __shared__ uint32_t wmax[NT / RR_WAVE];
    reinterpret_cast<uint4 *>(tmap)[threadIdx.x] = make_uint4(0, 0, 0, 0);   // (ordered before the
                                                                             // heads by the scan's barrier)
#endif
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
#if RR_ENC_SIZE_PF
    // a long value's lane requests the first RR_ENC_SIZE_PF 64-byte lines of its descriptors
    // while the short values' lanes load theirs, so the task rounds' loads later hit the L2
    // (the OR keeps the loads; it is consumed once, after the rounds)
    uint32_t pfacc = 0;
    if (ntask > ENC_SHORT) {
        const uint32_t *d = reinterpret_cast<const uint32_t *>(elems + eb);
        const uint32_t lines = (uint32_t)((ne + 3) / 4);   // 4 descriptors per 64-byte line
#pragma unroll
        for (uint32_t k = 0; k < RR_ENC_SIZE_PF; ++k) pfacc |= d[16 * (k < lines ? k : lines - 1)];
    }
#endif
    s_el[tid] = (uint32_t)eb;
    s_te[tid] = type | (enc << 8);
    s_bad[tid] = bad;
    s_b0[tid] = s_p0[tid] = 0;
    s_b1[tid] = sh_b;
    s_p1[tid] = sh_p;
    uint64_t TT;
    const uint32_t base = (uint32_t)block_excl_scan<NT>(ntask, ws0, TT);
    tb[tid] = base;
    if (tid == NT - 1) tb[NT] = base + ntask;
#if RR_ENC_SIZE_MAP
    const bool usemap = build_task_map<NT>(tmap, wmax, base, ntask, TT);
#else
    lds_barrier();
#endif
    auto fetch = [&](uint64_t t, uint32_t &pj, ElemV &pe) {
        pj = 0;
        pe = ElemV{0, 0, 0};
        if (t < TT) {
            uint32_t lo = 0;
#if RR_ENC_SIZE_MAP
            if (usemap) lo = tmap[t];
            else
#endif
#pragma unroll
            for (uint32_t s = NT / 2; s > 0; s >>= 1)
                if (tb[lo + s] <= t) lo += s;
            pj = lo;
            pe = get_elem(elems + s_el[lo] + (uint32_t)(t - tb[lo]));
        }
    };
    uint64_t runb = 0, runp = 0;
    uint32_t par = 0;
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
            uint32_t k = 0;
            if (act) {
                k = (uint32_t)(t - tb[j[u]]);
                const uint32_t te = s_te[j[u]];
                c = task_cost(te & 0xFF, te >> 8, k, e[u], acap);
            }
#if RR_ENC_SIZE_SEG
            // wave-segmented sums, no block barrier per round: a wave's tasks run over a few
            // values in order; each value's run in the wave adds (inclusive scan at its last
            // task) - (exclusive scan at its first task) to the value's sums with two LDS atomics
            (void)k;
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
            (void)par; (void)runb; (void)runp; (void)ws;
#else
            uint64_t exb, exp, tb_, tp_;
            block_excl_scan2<NT>(c.bytes, c.pay, ws[par], exb, exp, tb_, tp_);
            par ^= 1;
            if (act) {
                if (k == 0) { s_b0[j[u]] = runb + exb; s_p0[j[u]] = runp + exp; }
                if (t + 1 == tb[j[u] + 1]) { s_b1[j[u]] = runb + exb + c.bytes; s_p1[j[u]] = runp + exp + c.pay; }
                if (c.bad) s_bad[j[u]] = 1;
            }
            runb += tb_;
            runp += tp_;
#endif
        }
    }
    lds_barrier();
#if RR_ENC_SIZE_PF
    asm volatile("" ::"v"(pfacc));
#endif
    uint64_t size = 0, pay = 0;
    if (v < n) {
        bad = s_bad[tid];
        size = bad ? 0 : hdr + (s_b1[tid] - s_b0[tid]);
        pay = bad ? 0 : s_p1[tid] - s_p0[tid];
        sizes[v] = size;
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
}

// ---- E3: window index + capacity check ---------------------------------------------------
// fv[w] = the value holding output byte w*W (values of size 0 hold none).  A value whose end
// passes data_cap is not written (rock_serdes has no such case: sds grows; the batch API
// bounds the output): it counts as bad and its payload is taken back out of the totals
// (stored as a two's-complement negative, folded by the same modular sum).
#ifndef RR_ENC_FOLD4   // 1: E4's block 0 folds the tile totals (no finalize launch)
#define RR_ENC_FOLD4 1   // (encode cfg 4 -1 %, cfg 2 / 3 within noise)
#endif
#ifndef RR_ENC_ATOT   // 1: E3 adds the totals atomically and sets the bytes (no finalize launch)
#define RR_ENC_ATOT 0   // (measured: encode +7 %: 11.7K same-address atomics inside a 5 us kernel serialize)
#endif
template <uint32_t W>
__global__ __launch_bounds__(256) void enc_index_kernel(const rr_value *__restrict__ values,
                                                        const rr_elem *__restrict__ elems, uint64_t n,
                                                        uint64_t ecap, uint64_t acap,
                                                        const uint64_t *__restrict__ offsets, uint64_t cap,
                                                        uint32_t *__restrict__ fv, uint64_t nwin,
                                                        uint64_t *__restrict__ stats, rr_totals *tot,
                                                        uint64_t *err) {
    __shared__ uint64_t red[2][4];
    const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t bad = 0, pay = 0;
    if (v < n) {
        const uint64_t a = offsets[v], b = offsets[v + 1];
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
#if RR_ENC_ATOT
        // this block's totals and E1's for the same 256 values straight into the call's totals
        // (zeroed by E1's block 0, a kernel earlier): {bad, payload, descriptors}, no finalize
        // launch; the last value's thread sets the bytes (or the device-failure mark)
        (void)stats;
        s += stats[-3 * (int64_t)gridDim.x + 3 * (int64_t)blockIdx.x + threadIdx.x];   // (E1's tile stats)
        unsigned long long *f = reinterpret_cast<unsigned long long *>(tot);
        if (tot && s) atomicAdd(threadIdx.x == 0 ? &f[2] : threadIdx.x == 1 ? &f[3] : &f[0], (unsigned long long)s);
#else
        (void)tot;
        (void)err;
        stats[3 * (uint64_t)blockIdx.x + threadIdx.x] = s;
#endif
    }
#if RR_ENC_ATOT
    if (tot && v + 1 == n) tot->bytes = lb_load(err) ? ~0ull : offsets[n];
#endif
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
#else
#define EPROBE(...)
#endif

#ifndef RR_ENC_TPF
#define RR_ENC_TPF 1
#endif
#ifndef RR_ENC_ROT   // 1: the granule copies' store order rotated per lane group (LDS bank spread)
#define RR_ENC_ROT 0   // (measured: within noise, cfg 2 / 3 +1-2 %)
#endif
#ifndef RR_ENC_SEARCH2   // 1: E4's task -> value search in two rounds of independent LDS reads
#define RR_ENC_SEARCH2 0   // (measured: E4 343.6 -> 365 us: more LDS instructions in an issue-bound kernel)
#endif
#ifndef RR_ENC_EMIT_MAP   // 1: E4 maps tasks to values through an LDS map (build_task_map)
#define RR_ENC_EMIT_MAP 0   // (measured: E4 +2 %, its 4 KiB more LDS per workgroup)
#endif

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

// The window image: byte writes at absolute output positions, clipped to [w0, w0 + span).
// Naturally aligned LDS stores only: a misaligned ds_write costs ~7 aligned ones on gfx950
// (tools/micro/lds_align.hip: misaligned b32/b64/b128 all ~0.45 ms vs 0.06-0.10 ms aligned).
// lds_put writes the low nb (<= 8) bytes of v at image offset d: ascending alignment steps
// (1, 2, 4), then descending sizes (8, 4, 2, 1); every store lands on its natural alignment.
__device__ __forceinline__ void lds_put(uint8_t *img, uint32_t d, uint64_t v, uint32_t nb) {
    uint32_t r = nb;
    if ((d & 1) && r >= 1) { img[d] = (uint8_t)v; v >>= 8; d += 1; r -= 1; }
    if ((d & 2) && r >= 2) { *reinterpret_cast<uint16_t *>(img + d) = (uint16_t)v; v >>= 16; d += 2; r -= 2; }
    if ((d & 4) && r >= 4) { *reinterpret_cast<uint32_t *>(img + d) = (uint32_t)v; v >>= 32; d += 4; r -= 4; }
    if (r & 8) { *reinterpret_cast<uint64_t *>(img + d) = v; return; }
    if (r & 4) { *reinterpret_cast<uint32_t *>(img + d) = (uint32_t)v; v >>= 32; d += 4; }
    if (r & 2) { *reinterpret_cast<uint16_t *>(img + d) = (uint16_t)v; v >>= 16; d += 2; }
    if (r & 1) img[d] = (uint8_t)v;
}

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

#ifndef RR_ENC_OR   // 1: fields OR-ed into the zeroed image (one or two aligned 64-bit LDS atomics)
#define RR_ENC_OR 1
#endif
#ifndef RR_ENC_ALIGNED   // 1: granule copies for pieces aligned with their image offset mod 16
#define RR_ENC_ALIGNED 1
#endif
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
    __device__ __forceinline__ void put(uint64_t pos, uint32_t b) const {
        const uint64_t d = pos - w0;
        if (d < span) img[d] = (uint8_t)b;
    }
    // little-endian field of nb (<= 8) bytes
    __device__ __forceinline__ void field(uint64_t pos, uint64_t v, uint32_t nb) const {
        const uint64_t d = pos - w0;
#if RR_ENC_OR
        if (d < span && d + nb <= span) lds_or(img, (uint32_t)d, v, nb);
#else
        if (d < span && d + nb <= span) lds_put(img, (uint32_t)d, v, nb);
#endif
        else
            for (uint32_t i = 0; i < nb; ++i) put(pos + i, (uint32_t)(v >> (8 * i)) & 0xFF);
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


template <uint32_t W, uint32_t NT, uint32_t RCAP>
#ifdef RR_ENC_NVGPR   // (tuning: a hard VGPR budget for the emit kernel)
#define ENC_NVGPR_ATTR __attribute__((amdgpu_num_vgpr(RR_ENC_NVGPR)))
#else
#define ENC_NVGPR_ATTR
#endif
#ifndef RR_ENC_WPE   // waves per SIMD the emit kernel is built for
#define RR_ENC_WPE 6      // (74 VGPRs, no spills; 5: E4 345 us, 6: 307 us)
#endif
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(RR_ENC_WPE))) ENC_NVGPR_ATTR void enc_emit_kernel(const rr_value *__restrict__ values,
                                                      const rr_elem *__restrict__ elems,
                                                      const uint8_t *__restrict__ arena, uint64_t n,
                                                      uint8_t *__restrict__ out, uint64_t cap,
                                                      const uint64_t *__restrict__ offsets,
                                                      const uint32_t *__restrict__ fv,
                                                      const uint64_t *__restrict__ stats, uint32_t ntiles,
                                                      rr_totals *tot, uint64_t *err) {
    static_assert(W <= 65536 && W % 64 == 0, "image offsets are 16-bit, pieces 64-byte blocks");
#if RR_ENC_FOLD4
    // block 0 folds E1's and E3's tile totals into the call's totals before its window (the
    // finalize launch's work, hidden under the other windows)
    if (tot) fold_totals(stats, nullptr, ntiles, offsets, n, 0, tot, nullptr, err, 1);
#else
    (void)stats; (void)ntiles; (void)tot; (void)err;
#endif
    static_assert(RCAP >= 2 && W / 64 + RCAP < 65536, "run piece bases are 16-bit");
    constexpr uint32_t RTOP = 1u << (31 - __builtin_clz(RCAP - 1));   // largest power of two < RCAP
    __shared__ uint4 img4[W / 16];
    __shared__ uint64_t rq_a[RCAP];        // run: arena offset | length << 40
    __shared__ uint32_t rq_dp[RCAP];       // run: image offset | first piece (pieces of earlier runs) << 16
    __shared__ __attribute__((aligned(16))) uint32_t tb[NT + 1];   // task base of each value of the round
    __shared__ uint64_t sv_pos[NT];        // output position of the value's first task, less the
                                           // element-byte scan there once its first task is costed
    __shared__ uint32_t sv_el[NT];         // elem_base
    __shared__ uint32_t sv_te[NT];         // type | enc << 8
    __shared__ uint64_t wsum[2][NT / RR_WAVE];
    __shared__ uint64_t sh_nrp;            // runs reserved | pieces reserved << 32
    __shared__ uint32_t sh_pend;           // pieces of the queued runs, when the queue overflowed
    __shared__ uint32_t sh_unal;           // some queued run is not aligned with its image offset mod 16
#if RR_ENC_EMIT_MAP   // task -> value map of a value round (build_task_map)
    __shared__ __attribute__((aligned(16))) uint8_t tmap[ENC_MAPCAP];
    __shared__ uint32_t wmax[NT / RR_WAVE];
#endif
    uint8_t *img = reinterpret_cast<uint8_t *>(img4);
    const uint32_t tid = threadIdx.x;
    const uint64_t total = offsets[n];
    const uint64_t lim = total < cap ? total : cap;
    const uint64_t w0 = (uint64_t)blockIdx.x * W;
    if (w0 >= lim) return;
    EPROBE(uint64_t et0 = rr_stamp(), etk = 0, ent = 0, tf = 0, tsc = 0, twr = 0, tw1 = 0, tw2 = 0;)
    const uint64_t span = lim - w0 < W ? lim - w0 : W;
    const Img I{img, w0, span};
#pragma unroll
    for (uint32_t k = tid; k < W / 16; k += NT) img4[k] = make_uint4(0, 0, 0, 0);
    if (tid == 0) { sh_nrp = 0; sh_pend = 0xFFFFFFFFu; sh_unal = 0; }
    const uint64_t v0 = fv[blockIdx.x];
    const uint64_t vend = w0 + W < total ? (uint64_t)fv[blockIdx.x + 1] + 1 : n;
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
        const uint32_t np = queued ? ((dst + l - 1) >> 6) - (dst >> 6) + 1 : 0;
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
#if RR_ENC_ALIGNED
            if ((reinterpret_cast<uintptr_t>(arena) + src - dst) & 15) sh_unal = 1;
#endif
        } else {   // queue full (rare; keeps the kernel small): byte copy
            if (queued && r == RCAP) sh_pend = p0;
            for (uint32_t i = 0; i < l; ++i) img[dst + i] = arena[src + i];
        }
    };

    for (uint64_t vb = v0; vb < vend; vb += NT) {
        const uint64_t v = vb + tid;
        uint32_t tasks = 0;
#if RR_ENC_EMIT_MAP   // (the previous round's last reads of the map are behind its closing barrier)
        reinterpret_cast<uint4 *>(tmap)[tid] = make_uint4(0, 0, 0, 0);
#endif
        if (v < vend) {
            const uint64_t a = offsets[v], b = offsets[v + 1];
            const uint4 x = reinterpret_cast<const uint4 *>(values)[v];
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
                    if (nb) I.field(a + 5 * f, f == 0 ? (type | ((uint64_t)(x.y & RR_LRU_MASK) << 8)) : fv8, nb);
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
#if RR_ENC_EMIT_MAP
        const bool usemap = build_task_map<NT>(tmap, wmax, base, tasks, tt);
#else
        lds_barrier();
#endif
        EPROBE(const uint64_t eth = rr_stamp(); ent += tt;)
        uint64_t run = 0;   // element bytes of the earlier task rounds
        // task rounds in groups of TPF: every round's descriptor is loaded up front, so a
        // group costs one memory round trip
        auto fetch = [&](uint64_t t, uint32_t &pj, ElemV &pe) {
            pj = 0;
            pe = ElemV{0, 0, 0};
            if (t < tt) {
                // last value j with tb[j] <= t
                uint32_t lo = 0;
#if RR_ENC_EMIT_MAP
                if (usemap) lo = tmap[t];
                else
#endif
#if RR_ENC_SEARCH2
                lo = search_last_le<NT>(tb, (uint32_t)t);
#else
#pragma unroll
                for (uint32_t s = NT / 2; s > 0; s >>= 1)
                    if (tb[lo + s] <= t) lo += s;
#endif
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
                if (fnb) I.field(p, fval, fnb);
                EPROBE(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const uint64_t rw1 = rr_stamp(); tw1 += rw1 - rs1;)
                if (type == RR_TYPE_LIST_QUICKLIST && !pay) I.decimal(p + 4, (int64_t)e.data, (uint32_t)(es - 4));
                EPROBE(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const uint64_t rw2 = rr_stamp(); tw2 += rw2 - rw1;)
                ppos = p + hdr;
            }
            payload(pay, ppos, e.data, e.len);
            run += rt;
            EPROBE(asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); const uint64_t rs2 = rr_stamp(); twr += rs2 - rs1;)
        };
        // task rounds in groups of four: the group's descriptors are loaded up front, so a
        // group costs one memory round trip
#if RR_ENC_TPF == 1
        for (uint64_t g0 = 0; g0 < tt; g0 += NT) {
            uint32_t j0;
            ElemV e0;
            fetch(g0 + tid, j0, e0);
            round(g0, j0, e0);
        }
#else
        for (uint64_t g0 = 0; g0 < tt; g0 += 4 * NT) {
            uint32_t j0, j1, j2, j3;
            ElemV e0, e1, e2, e3;
            fetch(g0 + tid, j0, e0);
            fetch(g0 + NT + tid, j1, e1);
            fetch(g0 + 2 * NT + tid, j2, e2);
            fetch(g0 + 3 * NT + tid, j3, e3);
            EPROBE(asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); tf += rr_stamp() - eth;)
            round(g0, j0, e0);
            if (g0 + NT < tt) round(g0 + NT, j1, e1);
            if (g0 + 2 * NT < tt) round(g0 + 2 * NT, j2, e2);
            if (g0 + 3 * NT < tt) round(g0 + 3 * NT, j3, e3);
        }
#endif
        lds_barrier();
        EPROBE(const uint64_t ett = rr_stamp(); etk += ett - eth;)
    }
    EPROBE(const uint64_t et2 = rr_stamp();)

    // payload pieces: piece b of the window -> its run (last run whose first piece <= b) ->
    // the run's k-th 64-byte image block
    const uint32_t nr = (uint32_t)sh_nrp < RCAP ? (uint32_t)sh_nrp : RCAP;
    const uint32_t npc = sh_pend != 0xFFFFFFFFu ? sh_pend : (uint32_t)(sh_nrp >> 32);
    auto piece = [&](uint32_t b, uint64_t &ps, uint32_t &pd, uint32_t &pl) {
        uint32_t lo = 0;   // (steps from the largest power of two below RCAP: every index reachable)
#if RR_ENC_SEARCH2
        // the last queued run whose first piece <= b, in three rounds of seven independent LDS
        // reads (stride 64, 8, 1) instead of nine dependent ones: rq_dp[i] < (b + 1) << 16 is a
        // prefix-true predicate over the runs [0, nr)
        static_assert(RCAP == 512, "three levels of 8");
        (void)RTOP;
        const uint32_t key = (b + 1) << 16;
#pragma unroll
        for (uint32_t st = 64; st > 0; st >>= 3) {
            uint32_t c = 0;
#pragma unroll
            for (uint32_t k = 1; k < 8; ++k) {
                const uint32_t i = lo + k * st;
                c += (i < nr && rq_dp[i < RCAP ? i : RCAP - 1] < key) ? 1u : 0u;
            }
            lo += c * st;
        }
#else
#pragma unroll
        for (uint32_t s = RTOP; s > 0; s >>= 1)
            if (lo + s < nr && (rq_dp[lo + s] >> 16) <= b) lo += s;
#endif
        const uint64_t a = rq_a[lo];
        const uint32_t dp = rq_dp[lo], dst = dp & 0xFFFF, l = (uint32_t)(a >> 40), k = b - (dp >> 16);
        const uint32_t d0 = k == 0 ? dst : ((dst >> 6) + k) << 6;
        const uint32_t e1 = (((dst >> 6) + k + 1) << 6), e = e1 < dst + l ? e1 : dst + l;
        ps = (a & JQ_SRC) + (d0 - dst);
        pd = d0;
        pl = e > d0 ? e - d0 : 0;   // (inside one 64-byte block by construction)
    };
#if RR_ENC_ALIGNED
    // Every run aligned with its image offset mod 16 (any arena that keeps the blob layout, the
    // decode's mirror arena included): pieces move whole granules (RR_AL_LOAD / RR_AL_STORE).
    // A window with any other run takes the byte plan below for all its pieces.
    if (sh_unal == 0) {
        for (uint32_t j = tid; j < npc; j += 2 * NT) {
            const bool two = j + NT < npc;
            uint64_t s0, s1 = 0;
            uint32_t d0, l0, d1 = 0, l1 = 0;
            piece(j, s0, d0, l0);
            if (two) piece(j + NT, s1, d1, l1);
#if RR_ENC_ROT
            const uint32_t rot = (lane_id() >> 2) & 3;
#else
            const uint32_t rot = 0;
#endif
            RR_AL_LOAD(xa, s0, d0, l0, rot)
            RR_AL_LOAD(xb, s1, d1, l1, rot)
            RR_AL_STORE(xa, d0, l0, rot)
            RR_AL_STORE(xb, d1, l1, rot)
        }
    } else
#endif
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

    // store the image: 16-byte chunks, bytes at a partial end
    u32x4 *dst4 = reinterpret_cast<u32x4 *>(out + w0);
    const u32x4 *src4 = reinterpret_cast<const u32x4 *>(img4);
    const uint32_t full = (uint32_t)(span >> 4);
    for (uint32_t c = tid; c < full; c += NT) __builtin_nontemporal_store(src4[c], dst4 + c);
    const uint32_t tail = (uint32_t)(span & 15);
    if (tid < tail) out[w0 + 16ull * full + tid] = img[16u * full + tid];
    EPROBE(const uint64_t et4 = rr_stamp();
           if (tid == 0 && g_eprobe) {
               uint64_t *o = g_eprobe + (uint64_t)blockIdx.x * EPROBE_WORDS;
               o[0] = et1 - et0; o[1] = (et2 - et1) - etk; o[2] = etk; o[3] = et3 - et2; o[4] = et4 - et3;
               o[5] = et4 - et0; o[6] = vend - v0; o[7] = ent; o[8] = npc;
               o[9] = tw1; o[10] = tsc; o[11] = twr; o[12] = tw2;
           })
}

}  // namespace

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
#ifndef RR_DEC_PMAX
#define RR_DEC_PMAX 1024
#endif
constexpr uint32_t DEC_W = RR_DEC_W, DEC_NW = RR_DEC_NW;
#define DECODE_KERNEL decode_kernel<RR_DEC_W, RR_DEC_SLACK, RR_DEC_NW, RR_DEC_PMAX>

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
static uint64_t dec_windows(uint64_t data_cap) { return data_cap / DEC_W + 1; }

#ifndef RR_DEC_FUSED   // 1: dec_index_kernel + decode_fused_kernel; 0: count + scan + decode_kernel
#define RR_DEC_FUSED 0
#endif
#if RR_DEC_FUSED
// the fused kernel's chunk is one pass-A round of the workgroup's threads
#undef RR_DEC_PMAX
#define RR_DEC_PMAX (RR_DEC_NW * RR_WAVE)
#define DECODE_FUSED_KERNEL decode_fused_kernel<RR_DEC_W, RR_DEC_SLACK, RR_DEC_NW, RR_DEC_PMAX>
// Decode scratch (uint64 words): [HDR] [window look-back: state nwin, groups] [descriptor total,
// 1] [fixup header, then its u32 list of up to n values] [window stats, 3 per window] [first_val
// u32, nwin+1] [reservations u32, n] [class bytes, n].  dec_index_kernel zeroes the look-back
// words, the total and the fixup header.
extern "C" uint64_t rr_decode_scratch_words(uint64_t data_cap, uint64_t n) {
    const uint64_t nw = dec_windows(data_cap);
    return RR_SCRATCH_HDR + nw + (nw + LB_GROUP - 1) / LB_GROUP + FIX_HDR + (n + 2) / 2 + 1 + 3 * nw + (nw + 2) / 2 +
           (n + 2) / 2 + (n + 7) / 8 + 2;
}

extern "C" hipError_t rr_launch_decode(const uint8_t *blob, const uint64_t *offsets, uint64_t n, rr_value *values,
                                       rr_elem *elems, uint64_t elem_cap, uint8_t *arena, uint64_t *scratch,
                                       uint64_t data_cap, rr_totals *totals, hipStream_t stream) {
    const uint32_t nw = (uint32_t)dec_windows(data_cap);
    uint64_t *lb_state = scratch + RR_SCRATCH_HDR;
    uint64_t *lb_groups = lb_state + nw;
    const uint64_t lb_words = nw + (nw + LB_GROUP - 1) / LB_GROUP;
    uint64_t *total = lb_state + lb_words;
    uint64_t *fix = total + 1;                           // header words, then the u32 list
    uint64_t *stats = fix + FIX_HDR + (n + 2) / 2;
    uint32_t *first_val = reinterpret_cast<uint32_t *>(stats + 3 * (uint64_t)nw);
    uint32_t *cnt = first_val + ((nw + 2) & ~1u);
    uint8_t *cls = reinterpret_cast<uint8_t *>(cnt + ((n + 2) & ~1ull));
    hipLaunchKernelGGL(dec_index_kernel, dim3((uint32_t)((n + 1 + 255) / 256)), dim3(256), 0, stream, offsets, n,
                       first_val, nw, DEC_W, lb_state, (uint32_t)(lb_words + 1 + FIX_HDR), totals);
    hipLaunchKernelGGL((DECODE_FUSED_KERNEL), dim3(nw), dim3(DEC_NW * RR_WAVE), 0, stream, blob, data_cap, offsets, n,
                       first_val, cls, cnt, values, elems, elem_cap, arena, stats, fix, nw, lb_state, lb_groups, total);
    static uint32_t post_grid = 0;
    if (!post_grid) post_grid = resident_grid(decode_post_kernel, FIX_NT, false);
    hipLaunchKernelGGL(decode_post_kernel, dim3(post_grid), dim3(FIX_NT), 0, stream, blob, fix, values, elems, stats,
                       total, nw, offsets, n, totals);
    return hipGetLastError();
}
#else
// Decode scratch (uint64 words): [HDR] [scan: ticket, look-back state + groups] [fixup header,
// then its u32 list of up to n values] [counts -> elem_base, n+1] [window stats, 3 per window]
// [first_val u32, nwin+1] [class bytes, n].  The look-back words and the fixup header are
// zeroed by one memset per call.
#ifndef RR_COUNT_SCAN   // 1: count_scan_kernel (one launch); 0: count_kernel + scan_kernel
#define RR_COUNT_SCAN 0     // (measured: the 3.9K in-kernel look-backs cost +40 us on cfg 4, +50 on cfg 2)
#endif
static uint32_t cs_tiles(uint64_t n) { return (uint32_t)((n + 1 + CS_NT - 1) / CS_NT); }
// look-back words of the reservation scan: count_scan_kernel's 256-value blocks, or scan_kernel's
// ticket + 4096-value tiles
static uint64_t dec_lb_words(uint64_t n) {
#if RR_COUNT_SCAN
    const uint64_t t = cs_tiles(n);
    return t + (t + LB_GROUP - 1) / LB_GROUP;
#else
    const uint64_t st = scan_tiles(n);
    return 1 + st + (st + LB_GROUP - 1) / LB_GROUP;
#endif
}
extern "C" uint64_t rr_decode_scratch_words(uint64_t data_cap, uint64_t n) {
    const uint64_t nw = dec_windows(data_cap);
    return RR_SCRATCH_HDR + dec_lb_words(n) + FIX_HDR + (n + 2) / 2 + (n + 1) + 3 * nw + (nw + 2) / 2 + (n + 7) / 8 + 2;
}

extern "C" hipError_t rr_launch_decode(const uint8_t *blob, const uint64_t *offsets, uint64_t n, rr_value *values,
                                       rr_elem *elems, uint64_t elem_cap, uint8_t *arena, uint64_t *scratch,
                                       uint64_t data_cap, rr_totals *totals, hipStream_t stream) {
    const uint32_t st = (uint32_t)scan_tiles(n), nw = (uint32_t)dec_windows(data_cap);
    (void)st;
    uint64_t *lb = scratch + RR_SCRATCH_HDR;
    const uint64_t lb_words = dec_lb_words(n);
    uint64_t *fix = lb + lb_words;                      // header words, then the u32 list
    uint64_t *counts = fix + FIX_HDR + (n + 2) / 2;
    uint64_t *stats = counts + n + 1;
    uint32_t *first_val = reinterpret_cast<uint32_t *>(stats + 3 * (uint64_t)nw);
    uint8_t *cls = reinterpret_cast<uint8_t *>(first_val + ((nw + 2) & ~1u));
#if RR_COUNT_SCAN   // reservations, classes and elem_base in one launch (count_scan_kernel), after one
                    // memset of its look-back words and the fixup header (contiguous: scratch layout)
    {
        const uint32_t nb = cs_tiles(n);
        if (hipMemsetAsync(lb, 0, (lb_words + FIX_HDR) * sizeof(uint64_t), stream) != hipSuccess) return hipGetLastError();
        hipLaunchKernelGGL(count_scan_kernel, dim3(nb), dim3(CS_NT), 0, stream, blob, offsets, n, first_val, nw, DEC_W,
                           counts, cls, lb, lb + nb, nb, fix + 1, totals);
    }
#else
    hipLaunchKernelGGL(count_kernel, dim3((uint32_t)((n + 1 + 255) / 256)), dim3(256), 0, stream, blob, offsets, n,
                       first_val, nw, DEC_W, counts, cls, lb, (uint32_t)(lb_words + FIX_HDR), totals);
    if (st) hipLaunchKernelGGL(scan_kernel, dim3(st), dim3(256), 0, stream, counts, n, lb, st, fix + 1);
#endif
#if RR_DEC_PF
    static uint32_t dec_grid = 0;
    if (!dec_grid) dec_grid = resident_grid(DECODE_KERNEL, DEC_NW * RR_WAVE, false);
    const uint32_t grid = nw < dec_grid ? nw : dec_grid;
#else
    const uint32_t grid = nw;
#endif
    hipLaunchKernelGGL((DECODE_KERNEL), dim3(grid), dim3(DEC_NW * RR_WAVE), 0, stream, blob, data_cap, offsets, n,
                       first_val, cls, counts, values, elems, elem_cap, arena, stats, fix, nw, totals);
    static uint32_t post_grid = 0;
#ifdef RR_POST_GRID   // (tuning: a fixed post grid instead of the resident one)
    if (!post_grid) post_grid = RR_POST_GRID;
#else
    if (!post_grid) post_grid = resident_grid(decode_post_kernel, FIX_NT, false);
#endif
    hipLaunchKernelGGL(decode_post_kernel, dim3(post_grid), dim3(FIX_NT), 0, stream, blob, fix, values, elems, stats,
                       counts + n, nw, offsets, n, totals);
    return hipGetLastError();
}

#endif   // RR_DEC_FUSED

// Encode scratch (uint64 words): [HDR] [scan: ticket, look-back state + groups]
// [tile stats, 3 per 256 values, twice] [first value per output window u32, nwin+1].
#ifndef RR_ENC_W
#define RR_ENC_W 16384
#endif
#ifndef RR_ENC_RCAP   // payload runs queued per window (LDS: 12 bytes each)
#define RR_ENC_RCAP 416   // (6 emit workgroups per CU: 26.6 KB of LDS each)
#endif
constexpr uint32_t ENC_W = RR_ENC_W, ENC_NT = 256, ENC_RCAP = RR_ENC_RCAP;
static uint64_t enc_windows(uint64_t data_cap) { return data_cap / ENC_W + 1; }

extern "C" uint64_t rr_encode_scratch_words(uint64_t n, uint64_t data_cap) {
    const uint64_t st = scan_tiles(n), t = (n + 255) / 256, nw = enc_windows(data_cap);
    return RR_SCRATCH_HDR + 1 + st + (st + LB_GROUP - 1) / LB_GROUP + 1 + 6 * t + (nw + 2) / 2 + 2;
}

extern "C" hipError_t rr_launch_encode(const rr_value *values, const rr_elem *elems, uint64_t elem_cap,
                                       const uint8_t *arena, uint64_t arena_cap, uint64_t n, uint8_t *out,
                                       uint64_t cap, uint64_t *offsets, uint64_t *scratch, rr_totals *totals,
                                       hipStream_t stream) {
    hipError_t e;
    if (n == 0) {
        e = hipMemsetAsync(offsets, 0, sizeof(uint64_t), stream);
        if (e == hipSuccess && totals) e = hipMemsetAsync(totals, 0, sizeof(rr_totals), stream);
        return e;
    }
    const uint32_t st = (uint32_t)scan_tiles(n), t = (uint32_t)((n + 255) / 256);
    const uint64_t nw = enc_windows(cap);
    uint64_t *lb = scratch + RR_SCRATCH_HDR;
    const uint64_t lb_words = 1 + st + (st + LB_GROUP - 1) / LB_GROUP;
    uint64_t *err = lb + lb_words;   // device error word (look-back timeout)
    uint64_t *stats = err + 1;
    uint32_t *fv = reinterpret_cast<uint32_t *>(stats + 6 * (uint64_t)t);
    hipLaunchKernelGGL((enc_size_kernel<256, RR_ENC_SIZE_U>), dim3(t), dim3(256), 0, stream, values, elems, n, elem_cap, arena_cap, offsets,
                       stats, lb, (uint32_t)(lb_words + 1), totals);
    hipLaunchKernelGGL(scan_kernel, dim3(st), dim3(256), 0, stream, offsets, n, lb, st, err);
    hipLaunchKernelGGL(enc_index_kernel<ENC_W>, dim3(t), dim3(256), 0, stream, values, elems, n, elem_cap, arena_cap,
                       offsets, cap, fv, nw, stats + 3 * (uint64_t)t, totals, err);
    hipLaunchKernelGGL((enc_emit_kernel<ENC_W, ENC_NT, ENC_RCAP>), dim3((uint32_t)nw), dim3(ENC_NT), 0, stream,
                       values, elems, arena, n, out, cap, offsets, fv, stats, 2 * t, RR_ENC_FOLD4 ? totals : nullptr,
                       err);
    e = hipGetLastError();
#if !RR_ENC_ATOT && !RR_ENC_FOLD4
    if (e == hipSuccess && totals) e = launch_finalize(stats, lb, 2 * t, offsets, n, 0, totals, stream, err);
#endif
    return e;
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
constexpr uint32_t COPY_U = 8, COPY_NT = 256;
__global__ __launch_bounds__(COPY_NT) void copy_kernel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                       uint64_t bytes) {
    const uint64_t base = (uint64_t)blockIdx.x * (COPY_U * COPY_NT * 16);
    const uint64_t left = bytes - base;
    const uint32_t span = left < COPY_U * COPY_NT * 16 ? (uint32_t)left : COPY_U * COPY_NT * 16;
    const rsrc_t RS = make_rsrc(src + base, span), RD = make_rsrc(dst + base, span);
    u32x4 x[COPY_U];
#pragma unroll
    for (uint32_t k = 0; k < COPY_U; ++k)
        x[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(RS, (int)((threadIdx.x + k * COPY_NT) * 16), 0, 0));
#pragma unroll
    for (uint32_t k = 0; k < COPY_U; ++k)
        __builtin_amdgcn_raw_buffer_store_b128(x[k], RD, (int)((threadIdx.x + k * COPY_NT) * 16), 0, 2 /* nt */);
}

extern "C" hipError_t rr_launch_copy(uint8_t *dst, const uint8_t *src, uint64_t bytes, hipStream_t stream) {
    if (bytes == 0) return hipSuccess;
    const uint64_t blocks = (bytes + COPY_U * COPY_NT * 16 - 1) / (COPY_U * COPY_NT * 16);
    hipLaunchKernelGGL(copy_kernel, dim3((uint32_t)blocks), dim3(COPY_NT), 0, stream, src, dst, bytes);
    return hipGetLastError();
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
