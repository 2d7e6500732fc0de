/* rr_snappy.h — TEST INFRASTRUCTURE: CPU restatement of snappy's raw block format (rr_snappy.c).
 * Status codes match include/rr_snappy_gpu.h. */
#ifndef RR_ORACLE_SNAPPY_H
#define RR_ORACLE_SNAPPY_H
#include <stdint.h>

#define RRS_OK          0
#define RRS_E_HEADER    1   /* bad varint32 length preamble */
#define RRS_E_TRUNC     2   /* a tag, its extra bytes or a literal runs past the input */
#define RRS_E_OFFSET    3   /* copy offset 0 or before the start of the output */
#define RRS_E_OVERFLOW  4   /* more output than the preamble announced */
#define RRS_E_LENGTH    5   /* less output than the preamble announced */
#define RRS_E_CAPACITY  6   /* preamble length larger than the caller's output slot */

uint64_t rrs_max_compressed(uint64_t n);
uint64_t rrs_compress(const uint8_t *in, uint64_t n, uint8_t *out);
int rrs_uncompressed_length(const uint8_t *in, uint64_t n, uint32_t *len, uint32_t *hdr);
int rrs_uncompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_len);
void rrs_compress_batch(const uint8_t *in, const uint64_t *offs, uint64_t n, uint8_t *out, const uint64_t *slot,
                        uint64_t *sizes, int nthreads);
void rrs_uncompress_batch(const uint8_t *in, const uint64_t *offs, uint64_t n, uint8_t *out,
                          const uint64_t *out_offs, uint8_t *status, int nthreads);
#endif
