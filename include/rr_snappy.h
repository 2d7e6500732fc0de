/*
 * rr_snappy.h — GPU block compression of RocksDB data blocks.
 *
 * RedRock stores the serialized values in RocksDB (rocksdbapi.cc:133-168), whose block-based
 * tables compress every data block (block_size = ROCKDB_BLOCK_SIZE << 10 = 16 KiB,
 * rocksdbapi.cc:77,142) with the default compressor, snappy (options.compression is left at
 * its default, rocksdbapi.cc:159-161; the reference vendors snappy 1.1.8, deps/snappy).  These
 * calls compress / decompress a batch of such blocks on the GPU in snappy's raw format — the
 * bytes RocksDB's Snappy_Compress / Snappy_Uncompress write and read:
 *
 *   rr_snappy_compress_batch    block i -> snappy::RawCompress(block i), byte-identical to the
 *                               v1.1.8 compressor (varint32 length, 64 KiB fragments, the
 *                               hash-table match finder with its skip heuristic);
 *   rr_snappy_decompress_batch  block i -> snappy::RawUncompress(block i) with its validation;
 *                               a block it would reject gets a nonzero status instead.
 *
 * Conventions as rr_serdes.h: device pointers, the caller's stream, no host synchronisation in
 * the device entry points (a context's scratch grows between calls, not under capture).
 */
#ifndef RR_SNAPPY_H
#define RR_SNAPPY_H

#include <stdint.h>
#include "rr_serdes.h"

#ifdef __cplusplus
extern "C" {
#endif

/* per-block decompression status (0 = OK); every nonzero one is a `false` from snappy */
#define RR_SNAPPY_OK          0
#define RR_SNAPPY_E_HEADER    1   /* bad varint32 length preamble (snappy.cc:779-800) */
#define RR_SNAPPY_E_TRUNC     2   /* a tag, its extra bytes or a literal runs past the block */
#define RR_SNAPPY_E_OFFSET    3   /* copy offset 0 or before the start of the output (AppendFromSelf) */
#define RR_SNAPPY_E_OVERFLOW  4   /* more output than the preamble announced (Append / AppendFromSelf) */
#define RR_SNAPPY_E_LENGTH    5   /* less output than the preamble announced (CheckLength) */
#define RR_SNAPPY_E_CAPACITY  6   /* the block's output does not fit out->data_cap (batch API only) */

/* snappy::MaxCompressedLength (snappy.cc:98-118): 32 + n + n / 6 */
uint64_t rr_snappy_max_compressed_length(uint64_t n);
/* out->data_cap rr_snappy_compress_batch needs for n blocks of data_bytes in all: the sum of
 * the per-block bounds can not exceed 32 n + data_bytes + data_bytes / 6 (+ 16) */
uint64_t rr_snappy_compress_bound(uint64_t n, uint64_t data_bytes);

/* Both directions: in->data 16-byte aligned, in->data_cap a multiple of 16 covering every block
 * (the kernels read whole dwords up to it, never past it).
 * Compress in's n blocks (in->offsets[n+1]) into out->data, packed:
 * block i's compressed bytes at [out->offsets[i], out->offsets[i+1]).  out->data_cap must be at
 * least rr_snappy_compress_bound(n, in->data_cap): no block can then run out of room.  The
 * context's scratch holds per-block output slots (about 1.17x the input). */
int rr_snappy_compress_batch(rr_ctx *ctx, const rr_blob_batch *in, rr_blob_batch *out, void *stream);

/* Decompress in's n snappy blocks into out->data, packed in block order by the lengths their
 * preambles announce (out->offsets[n+1] written by the call); status[i] (device, n bytes) is
 * RR_SNAPPY_OK or an RR_SNAPPY_E_* code, and a failed block's output bytes are unspecified.
 * out->data_cap bounds the output: a block past it gets RR_SNAPPY_E_CAPACITY. */
int rr_snappy_decompress_batch(rr_ctx *ctx, const rr_blob_batch *in, rr_blob_batch *out, uint8_t *status,
                               void *stream);

/* Host-pointer forms (stage through the context's device buffers; synchronous).
 * compress: out_cap >= rr_snappy_compress_bound(n, offsets[n]); out_offsets[n+1] written.
 * decompress: out_offsets[n+1] and status[n] written; returns RR_API_EINVAL if out_cap is
 * smaller than the sum of the announced lengths (nothing is decompressed then). */
int rr_snappy_compress_batch_host(rr_ctx *ctx, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                                  uint8_t *out, uint64_t out_cap, uint64_t *out_offsets);
int rr_snappy_decompress_batch_host(rr_ctx *ctx, const uint8_t *data, const uint64_t *offsets, uint64_t n,
                                    uint8_t *out, uint64_t out_cap, uint64_t *out_offsets, uint8_t *status);

#ifdef __cplusplus
}
#endif
#endif
