/*
 * rr_host.h — the engine's host codec: RedRock value blobs <-> the flat form of rr_format.h on
 * the calling CPU thread, one value at a time (row f1's single-value path).
 *
 * RedRock calls its codec one key at a time: desObject per rock-thread restore job
 * (rock.c:468, :552-575) and per key in the BGSAVE / AOF-rewrite child (rock.c:538), serObject
 * per evicted key on the main thread (rock.c:691 via rock_hotkey.c:348/:431).  A GPU call costs a
 * launch and a PCIe round trip (~15 µs) where one value needs ~0.1 µs of CPU, so the compat shim
 * (rock_serdes_compat.c) runs those calls here and sends only batches above its measured
 * crossover to the GPU entry points of rr_serdes.h.  The GPU entry points never fall back to this
 * codec: it is a routing target chosen by the caller, by batch size.
 *
 * Contract: the records, descriptors, statuses, totals, offsets and bytes of rr_decode_batch /
 * rr_encode_batch for the same input (tests/test_host_codec.py holds it to the oracle on the
 * golden fixtures, every synthetic config and the structured fuzz corpus; the GPU suite holds the
 * GPU to the same oracle).  Plain C, no HIP: usable in a fork child that must not touch the HIP
 * runtime its parent initialised (rock.c:527-550).  Thread-safe: no global state.
 */
#ifndef RR_HOST_H
#define RR_HOST_H

#include <stdint.h>

#include "rr_format.h"
#include "rr_serdes.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Descriptor slots blob [b, b + len) owns in a batch (rr_format.h): from its header fields (and
 * a List's length chain), equal to its descriptor count when it is valid. */
uint64_t rr_host_reserve(const uint8_t *b, uint64_t len);

/* desObject (rock_serdes.c:538-564) for one blob, into the flat form.  STR / ZLRAW descriptors
 * hold `base` + the payload's offset in the blob (base = the blob's offset in its batch, the
 * arena mirror of rr_format.h; 0 to index the blob itself).  Writes v->type, enc, status, lru
 * and n_elems (not elem_base) and el[0 .. n_elems).  `cap` slots are available at el: a valid
 * value that needs more returns RR_E_CAPACITY; *need (may be NULL) = the slots the value owns
 * (a SET_HT keeps one per blob member, duplicates included) — call again with that many.
 * Returns v->status. */
int rr_host_decode_value(const uint8_t *blob, uint64_t len, uint64_t base, rr_value *v, rr_elem *el,
                         uint64_t cap, uint64_t *need);

/* The status and record (type, enc, status, lru, n_elems) rr_host_decode_value gives, without
 * its descriptors: a Hash / ZSet ziplist is walked for its verdict only (a caller keeping the raw
 * ziplist, as desObject does, needs no entry descriptors).  Returns v->status. */
int rr_host_check_value(const uint8_t *blob, uint64_t len, rr_value *v);

/* rr_decode_batch_host's contract on the CPU: elem_base = the reservations' prefix, a malformed
 * value's slots zero-filled, RR_E_CAPACITY past elem_cap, totals; arena (may be NULL) receives
 * the byte mirror of data.  Always RR_API_OK (RR_API_EINVAL for a NULL pointer). */
int rr_host_decode_batch(const uint8_t *data, const uint64_t *offsets, uint64_t n, rr_value *values,
                         rr_elem *elems, uint64_t elem_cap, uint8_t *arena, rr_totals *totals);

/* serObject's size for one flat value (rock_serdes.c:512-535): RR_OK and the blob's byte count,
 * or RR_E_ENCODE and 0 for a value the encoder cannot write (the rules of rr_encode_batch,
 * rr_serdes.h).  elems is the batch's descriptor array, elem_cap its length; arena_cap bounds the
 * payload references (UINT64_MAX with arena == NULL below). */
int rr_host_encode_size(const rr_value *v, const rr_elem *elems, uint64_t elem_cap, uint64_t arena_cap,
                        uint64_t *size);

/* Writes the blob of one value whose rr_host_encode_size was RR_OK, at out.  Payload bytes are
 * read at arena + descriptor.data; with arena == NULL a descriptor's data is the payload's host
 * address (the compat shim describes live robj strings that way instead of copying them). */
void rr_host_encode_value(const rr_value *v, const rr_elem *elems, const uint8_t *arena, uint8_t *out);

/* rr_encode_batch_host's contract on the CPU (offsets[0..n], data, totals; values past data_cap
 * counted bad and not written). */
int rr_host_encode_batch(const rr_value *values, const rr_elem *elems, uint64_t elem_cap, const uint8_t *arena,
                         uint64_t arena_cap, uint64_t n, uint8_t *data, uint64_t data_cap, uint64_t *offsets,
                         rr_totals *totals);

#ifdef __cplusplus
}
#endif
#endif
