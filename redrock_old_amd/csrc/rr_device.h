// rr_device.h — device-side building blocks shared by the decode and encode kernels:
// unaligned little-endian loads, strict integer parse / decimal render (util.c, sds.c),
// wave64 scans and the decoupled look-back used for output offsets.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rr_format.h"

#define RR_WAVE 64

namespace rr {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Byte-composed little-endian loads.  Templated on the pointer type so the same parser runs
// on LDS-staged bytes (address_space(3): ds_read_u8, ~100-cycle latency) and on global memory
// (fallback for windows whose values do not fit the stage).  The byte loads of one field are
// independent, so a field costs one memory latency, not four.
typedef const __attribute__((address_space(3))) uint8_t *lds_cptr;

template <typename P>
__device__ __forceinline__ uint32_t ld_u8(P p) { return p[0]; }
template <typename P>
__device__ __forceinline__ uint32_t ld_u16(P p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
template <typename P>
__device__ __forceinline__ uint32_t ld_u32(P p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
template <typename P>
__device__ __forceinline__ uint64_t ld_u64(P p) { return (uint64_t)ld_u32(p) | ((uint64_t)ld_u32(p + 4) << 32); }

// util.c:360-424 string2ll, restricted by zipTryEncoding (ziplist.c:480): 1 <= len < 32.
template <typename P>
__device__ __forceinline__ bool zip_try_int(P s, uint32_t len, int64_t &out) {
    if (len == 0 || len >= 32) return false;
    uint32_t c0 = ld_u8(s);
    if (len == 1 && c0 == '0') { out = 0; return true; }
    uint32_t i = 0;
    bool neg = false;
    if (c0 == '-') {
        neg = true;
        i = 1;
        if (len == 1) return false;
    }
    uint32_t c = ld_u8(s + i);
    if (c < '1' || c > '9') return false;
    uint64_t v = c - '0';
    ++i;
    for (; i < len; ++i) {
        c = ld_u8(s + i);
        if (c < '0' || c > '9') return false;
        if (v > (~0ull / 10)) return false;
        v *= 10;
        if (v > (~0ull - (c - '0'))) return false;
        v += c - '0';
    }
    if (neg) {
        if (v > (1ull << 63)) return false;
        out = (int64_t)(0ull - v);
    } else {
        if (v > 0x7FFFFFFFFFFFFFFFull) return false;
        out = (int64_t)v;
    }
    return true;
}

// Length of sdsll2str(v) (sds.c:450-479).
__device__ __forceinline__ uint32_t dec_len(int64_t value) {
    uint64_t v = value < 0 ? 0ull - (uint64_t)value : (uint64_t)value;
    uint32_t l = 1;
    while (v >= 10) { v /= 10; ++l; }
    return l + (value < 0 ? 1u : 0u);
}
// Writes sdsll2str(v) at d (byte stores), returns length.
__device__ __forceinline__ uint32_t dec_write(uint8_t *d, int64_t value) {
    uint32_t l = dec_len(value);
    uint64_t v = value < 0 ? 0ull - (uint64_t)value : (uint64_t)value;
    uint32_t p = l;
    do { d[--p] = (uint8_t)('0' + (v % 10)); v /= 10; } while (v);
    if (value < 0) d[0] = '-';
    return l;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup-scope fence for all
// memory: it makes every wave wait for the acknowledgement of its outstanding global stores
// (s_waitcnt vmcnt(0)), ~1-2 us behind a burst of streaming stores.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Wave64 inclusive scan (u64) with shuffles.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
    uint32_t lane = lane_id();
#pragma unroll
    for (int d = 1; d < RR_WAVE; d <<= 1) {
        uint64_t y = __shfl_up(x, d, RR_WAVE);
        if (lane >= (uint32_t)d) x += y;
    }
    return x;
}
// Wave64 inclusive scans (u32) in DPP: four row shifts scan each row of 16 lanes, then
// row_bcast:15 / row_bcast:31 carry each row's last lane into the rows above it — six VALU ops,
// no LDS round trips (the shuffle form above is twelve ds_bpermute round trips for a u64).
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_max_u32(uint32_t x) {   // (same shape, max)
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
    return x;
}
// the value of lane - 1 (lane 0: 0) / lane + 1 (lane 63: 0) by a whole-wave DPP shift
__device__ __forceinline__ uint32_t wave_from_prev(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, false);   // wave_shr:1
}
__device__ __forceinline__ uint32_t wave_from_next(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false);   // wave_shl:1
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
    for (int d = RR_WAVE / 2; d > 0; d >>= 1) x += __shfl_xor(x, d, RR_WAVE);
    return x;
}
// wave_sum (every lane active) by the DPP scan and one readlane when no lane reaches 2^26 (the
// sum then fits 32 bits): six VALU ops instead of twelve ds_bpermute round trips
__device__ __forceinline__ uint64_t wave_sum_fast(uint64_t x) {
    if (__ballot(x >= (1ull << 26)) == 0)
        return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32((uint32_t)x), RR_WAVE - 1);
    return wave_sum(x);
}
// inclusive scan (every lane active): DPP u32 when no lane reaches 2^26, else the shuffles
__device__ __forceinline__ uint64_t wave_incl_scan_fast(uint64_t x) {
    return __ballot(x >= (1ull << 26)) == 0 ? (uint64_t)wave_incl_scan_u32((uint32_t)x) : wave_incl_scan(x);
}

// ---- decoupled look-back (single-pass scan across wave tiles) ---------------------------
// One 8-byte word per tile: bits 62-63 flag (0 empty, 1 aggregate, 2 inclusive prefix),
// bits 0-61 value.  The word is the data (a self-contained granule written by one relaxed
// agent-scope store = sc1), so no separate flag and no fence are needed
// (cdna_hip_programming.md §6 Guideline 16, R2).  Words are zeroed by a hipMemsetAsync
// before every launch.  Tile ids are handed out in launch order by an atomic counter, so a
// tile only waits on tiles whose waves are already resident.
constexpr uint64_t LB_AGG = 1ull << 62;
constexpr uint64_t LB_INC = 2ull << 62;
constexpr uint64_t LB_VAL = (1ull << 62) - 1;

__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Two-level look-back.  Tiles are grouped by 64 (LB_GROUP); besides its own word every tile
// adds (1 << 48) | aggregate to its group word with one non-returning atomic, so a group word
// says both how many of its tiles have published and their total.  A tile's exclusive prefix
// is then found in ~2-3 round trips whatever the number of tiles in flight: one sweep of the
// (up to 63) earlier tiles of its own group, then sweeps over 64 earlier groups at a time,
// each lane reading a group word and the word of that group's last tile (an inclusive prefix
// there ends the walk).  With thousands of concurrent tiles a flat 64-tile look-back needs
// ~tiles/64 round trips per tile (measured: 3.9 ms for 121K tiles); this needs ~3.
constexpr uint32_t LB_GROUP = 64;
constexpr uint64_t GRP_ONE = 1ull << 48;
constexpr uint64_t GRP_VAL = GRP_ONE - 1;

// A wait that never ends (a tile that never publishes: a hardware or scheduling fault) is cut
// after 2^24 sleeps: the call's error word *err is set and the prefix returned is 0 — the host
// sees rr_totals.bytes == UINT64_MAX (rr_serdes.h) instead of silently wrong offsets.
// The look-back in two halves, so a tile can publish its aggregate as soon as it knows it and
// resolve its prefix later (other work in between): lb_publish by one wave, lb_resolve by one
// whole wave (it also publishes the inclusive prefix).
__device__ __forceinline__ void lb_publish(uint64_t *state, uint64_t *groups, uint32_t tile, uint64_t agg) {
    if (lane_id() == 0) {
        lb_store(&state[tile], (tile == 0 ? LB_INC : LB_AGG) | agg);
        atomicAdd((unsigned long long *)&groups[tile / LB_GROUP], (unsigned long long)(GRP_ONE | agg));
    }
}
__device__ __forceinline__ uint64_t lb_resolve(uint64_t *state, uint64_t *groups, uint32_t tile, uint32_t ntiles,
                                               uint64_t agg, uint64_t *err);
__device__ __forceinline__ uint64_t lookback(uint64_t *state, uint64_t *groups, uint32_t tile, uint32_t ntiles,
                                             uint64_t agg, uint64_t *err) {
    lb_publish(state, groups, tile, agg);
    return lb_resolve(state, groups, tile, ntiles, agg, err);
}
__device__ __forceinline__ uint64_t lb_resolve(uint64_t *state, uint64_t *groups, uint32_t tile, uint32_t ntiles,
                                               uint64_t agg, uint64_t *err) {
    const uint32_t lane = lane_id();
    const uint32_t g = tile / LB_GROUP, p = tile % LB_GROUP;
    if (tile == 0) return 0;
    uint64_t excl = 0;
    uint32_t spins = 0;
    // phase 1: earlier tiles of the same group
    if (p) {
        for (;;) {
            uint64_t s = lane < p ? lb_load(&state[tile - 1 - lane]) : LB_INC;
            uint64_t flag = s >> 62;
            uint64_t inc = __ballot(lane < p && flag == 2);
            uint64_t empty = __ballot(lane < p && flag == 0);
            uint32_t first = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
            uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1);
            if (empty & upto) {
                if (++spins > (1u << 24)) { lb_store(err, 1); return 0; }   // bounded: never hang the GPU
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl = wave_sum_fast(lane < p && lane <= first ? (s & LB_VAL) : 0);
            if (first < 64) goto done;
            break;
        }
    }
    // phase 2: whole earlier groups, 64 per sweep
    for (int64_t gg = (int64_t)g - 1;;) {
        const int64_t k = gg - (int64_t)lane;
        uint64_t last = LB_INC, grp = 0;
        bool complete = true;
        if (k >= 0) {
            last = lb_load(&state[(uint64_t)k * LB_GROUP + LB_GROUP - 1]);
            grp = lb_load(&groups[k]);
            uint64_t members = (uint64_t)ntiles - (uint64_t)k * LB_GROUP;
            if (members > LB_GROUP) members = LB_GROUP;
            complete = (grp >> 48) == members;
        }
        const bool is_inc = (last >> 62) == 2;
        uint64_t inc = __ballot(is_inc);
        uint32_t first = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
        uint64_t upto_excl = first >= 64 ? ~0ull : ((1ull << first) - 1);   // lanes before the INC lane
        uint64_t incomplete = __ballot(!complete);
        if (incomplete & upto_excl) {
            if (++spins > (1u << 24)) { lb_store(err, 1); return 0; }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        uint64_t v = 0;
        if (lane < first) v = grp & GRP_VAL;
        else if (lane == first) v = last & LB_VAL;
        excl += wave_sum_fast(v);
        if (first < 64) break;
        gg -= RR_WAVE;
    }
done:
    if (lane == 0) lb_store(&state[tile], LB_INC | (excl + agg));
    return excl;
}

__device__ __forceinline__ uint32_t next_tile(uint64_t *counter) {
    uint32_t t = 0;
    if (lane_id() == 0) t = (uint32_t)atomicAdd((unsigned long long *)counter, 1ull);
    return __builtin_amdgcn_readfirstlane(t);
}

}  // namespace rr
