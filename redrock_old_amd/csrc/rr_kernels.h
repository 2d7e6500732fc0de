/* rr_kernels.h — launch entry points of rr_kernels.hip, called by the C host layer (rr_api.c). */
#ifndef RR_KERNELS_H
#define RR_KERNELS_H

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "../../include/rr_format.h"
#include "../../include/rr_serdes.h"

/* scratch layout (uint64 words): [0] tile counter, [1] done counter, [2] byte total,
 * [8 .. 8+64) 16 shards x {bad, payload, elems, -}, then one look-back word per tile
 * (decode: per byte window, followed by the u32 first-value table of the windows). */
#define RR_SCRATCH_HDR 72

#ifdef __cplusplus
extern "C" {
#endif

/* sums: rr_decode_sums_words(data_cap) words, zero on entry (count_kernel adds the window and
 * group sums into them, decode_kernel reads them; a batch of one window generation runs
 * decode_kernel's one-launch form alone, which keeps its look-back and end words there and leaves
 * them zero); zero / nzero: words the call zeroes on the way (the other half of the context's
 * double buffer).  first_only (test hooks): 1 launch only count_kernel (the two-launch form);
 * 2 the one-launch form sums every earlier window itself (its look-back's help path). */
hipError_t rr_launch_decode(const uint8_t *blob, const uint64_t *offsets, uint64_t n, rr_value *values,
                            rr_elem *elems, uint64_t elem_cap, uint8_t *arena, uint64_t *scratch, uint64_t *sums,
                            uint64_t *zero, uint64_t nzero, uint64_t data_cap, rr_totals *totals, hipStream_t stream,
                            int first_only);
uint64_t rr_decode_sums_words(uint64_t data_cap);
hipError_t rr_launch_zero_words(uint64_t *words, uint64_t n, hipStream_t stream);
hipError_t rr_launch_encode(const rr_value *values, const rr_elem *elems, uint64_t elem_cap, const uint8_t *arena,
                            uint64_t arena_cap, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *offsets,
                            uint64_t *scratch, uint64_t *sums, rr_totals *totals, hipStream_t stream, int first_only);
uint64_t rr_encode_sums_words(uint64_t n);
uint64_t rr_decode_scratch_words(uint64_t data_cap, uint64_t n);
uint64_t rr_scan_words(uint64_t n);
hipError_t rr_launch_scan_u64(uint64_t *x, uint64_t n, uint64_t *lb, uint64_t *err, hipStream_t stream);
uint64_t rr_snappy_scratch_words(uint64_t n, uint64_t slot_bytes);
hipError_t rr_launch_snappy_decompress(const uint8_t *in, uint64_t in_cap, const uint64_t *in_offs, uint64_t n, uint8_t *out,
                                       uint64_t out_cap, uint64_t *out_offs, uint8_t *status, uint64_t *scratch,
                                       hipStream_t stream);
hipError_t rr_launch_snappy_compress(const uint8_t *in, uint64_t in_cap, const uint64_t *in_offs, uint64_t n, uint8_t *out,
                                     uint64_t *out_offs, uint64_t *scratch, uint64_t slot_bytes, hipStream_t stream);
hipError_t rr_launch_shard_plan(const uint64_t *offsets, uint64_t n, uint32_t g, uint64_t *plan, hipStream_t stream);
hipError_t rr_launch_offsets_rebase(uint64_t *offs, uint64_t count, uint64_t sub, hipStream_t stream);
hipError_t rr_launch_flat_rebase(rr_value *values, uint64_t n, rr_elem *elems, uint64_t ne, uint64_t elem_add,
                                 uint64_t byte_add, hipStream_t stream);
uint64_t rr_encode_scratch_words(uint64_t n, uint64_t data_cap);
hipError_t rr_launch_copy(uint8_t *dst, const uint8_t *src, uint64_t bytes, hipStream_t stream);
hipError_t rr_launch_copy_shape(uint8_t *dst, const uint8_t *src, uint64_t bytes, int shape, hipStream_t stream);
/* the pipelined host encode: the end of the arena bytes the valid values [0, n) read, as
 * RR_NEED_BLOCKS partial maxima into mapped host words */
#define RR_NEED_BLOCKS 32
hipError_t rr_launch_arena_need(const rr_value *values, uint64_t n, const rr_elem *elems, uint64_t elem_cap,
                                uint64_t arena_cap, uint64_t *need, hipStream_t stream);
/* small batches (one workgroup, one launch): whether a batch qualifies, and the launches; a
 * non-NULL done (host-mapped) receives seq once every result is visible to the host */
int rr_small_decode_fits(uint64_t n, uint64_t data_cap);
int rr_small_encode_fits(uint64_t n, uint64_t data_cap);
hipError_t rr_launch_decode_small(const uint8_t *blob, const uint64_t *offsets, uint64_t n, rr_value *values,
                                  rr_elem *elems, uint64_t elem_cap, uint8_t *arena, uint64_t data_cap, rr_totals *totals,
                                  uint32_t *done, uint32_t seq, hipStream_t stream);
hipError_t rr_launch_encode_small(const rr_value *values, const rr_elem *elems, uint64_t elem_cap, const uint8_t *arena,
                                  uint64_t arena_cap, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *offsets,
                                  rr_totals *totals, uint32_t *done, uint32_t seq, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif
