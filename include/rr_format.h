/*
 * rr_format.h — the RedRock value-blob format and the flat decoded form.
 *
 * Blob format (what RedRock's src/rock_serdes.c writes into RocksDB):
 *   every blob = u8 type (rock.h:50-63) | u32 lru (host LE, rock_serdes.c:514-518) | body
 * Bodies per type (all multi-byte fields native little-endian, no varints):
 *   STRING          u8 enc (OBJ_ENCODING_RAW 0 / INT 1 / EMBSTR 8) | RAW,EMBSTR: bytes to end;
 *                   INT: i64                                              (rock_serdes.c:114-158)
 *   LIST_QUICKLIST  ({u32 len, u8[len]})* to end, no count; integer entries rendered as
 *                   decimal by sdsll2str                                  (rock_serdes.c:162-214)
 *   SET_INTSET      u32 enc∈{2,4,8} | u32 n | n*enc bytes LE ints         (rock_serdes.c:220-226)
 *   SET_HT          u64 n | ({u64 len, u8[len]})*                         (rock_serdes.c:227-239)
 *   HASH_ZIPLIST    u64 L | u8[L] raw ziplist (field,value entries)       (rock_serdes.c:317-320)
 *   HASH_HT         u64 n | ({u64 fl, f, u64 vl, v})*                     (rock_serdes.c:322-339)
 *   ZSET_ZIPLIST    u64 L | u8[L] raw ziplist (member,score entries)      (rock_serdes.c:420-423)
 *   ZSET_SKIPLIST   u64 n | ({u64 l, ele, f64 score})* tail->head          (rock_serdes.c:425-440)
 *
 * Flat decoded form (device resident, produced by decode, consumed by encode):
 *   rr_value[n]     one 16-byte record per value
 *   rr_elem[m]      16-byte element descriptors, values own [elem_base, elem_base+n_elems)
 *   arena           payload bytes.  Decode lays the arena out as a MIRROR of the blob buffer:
 *                   a payload byte found at blob offset o is stored at arena offset o.  This
 *                   keeps every copy 16-byte congruent (aligned dwordx4 loads and stores) and
 *                   needs no prefix scan for arena offsets.  Encode accepts any arena layout.
 *
 * Element layout per type:
 *   STRING          1 elem: STR{arena off, len} (RAW/EMBSTR) or INT{i64} (INT)
 *   LIST_QUICKLIST  1 elem per entry: INT{v} when the entry passes zipTryEncoding
 *                   (ziplist.c:480: 1<=len<32 and string2ll, util.c:360) — exactly what
 *                   desList's quicklistPushTail stores — else STR
 *   SET_INTSET      n INT elems; rr_value.enc = intset width
 *   SET_HT          STR elems in blob order, later duplicates of a member dropped (desSet's
 *                   dictAdd keeps the first and ignores the rest, rock_serdes.c:297); the
 *                   value still owns one slot per blob member, the unused tail is zero
 *   HASH_ZIPLIST    ZLRAW{arena off, L} then one elem per ziplist entry (STR or INT,
 *   ZSET_ZIPLIST    zenc = the entry's encoding byte); encode only needs ZLRAW
 *   HASH_HT         2n STR elems: field, value, field, value, ... (duplicate field: RR_E_DUP)
 *   ZSET_SKIPLIST   2n elems: STR member, SCORE{f64 bits}, ... in the order serZset writes
 *                   the skiplist desZset builds: descending (score, member) (zslInsert,
 *                   t_zset.c:132-180, then the tail->head walk rock_serdes.c:430-440), equal
 *                   keys in blob order.  A blob serZset wrote is already in that order.
 */
#ifndef RR_FORMAT_H
#define RR_FORMAT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* On-disk type tags, rock.h:50-63 */
#define RR_TYPE_STRING          0
#define RR_TYPE_SET_HT          2
#define RR_TYPE_HASH_HT         4
#define RR_TYPE_ZSET_SKIPLIST   5
#define RR_TYPE_SET_INTSET      11
#define RR_TYPE_ZSET_ZIPLIST    12
#define RR_TYPE_HASH_ZIPLIST    13
#define RR_TYPE_LIST_QUICKLIST  14

/* String encodings as stored in the enc byte, server.h:575-583 */
#define RR_ENC_RAW     0
#define RR_ENC_INT     1
#define RR_ENC_EMBSTR  8
#define RR_EMBSTR_SIZE_LIMIT 44   /* rock_serdes.c:132 */

#define RR_LRU_MASK 0xFFFFFFu     /* robj.lru is a 24-bit bitfield, server.h:592-599 */

/* Element kinds */
#define RR_K_STR    0
#define RR_K_INT    1
#define RR_K_SCORE  2
#define RR_K_ZLRAW  3

/* Per-value decode status (0 = OK).  Codes 1-7, 9, 13 and 14 are the reference's own
 * serverAssert/serverPanic sites; the compat shim turns any nonzero status into abort().
 * Codes marked [stricter] reject blobs the reference would load into a broken object (it
 * never validates those bytes); see DESIGN.md "Deviations" for the full table.
 * When one blob has several defects the engine reports the structural one (SHORT / TRUNC /
 * COUNT) before DUP / NAN; the reference may hit a different assert first — either way the
 * value is rejected. */
#define RR_OK               0
#define RR_E_SHORT          1   /* blob shorter than its fixed header (rock_serdes.c:134,192,249,350,449,539-542) */
#define RR_E_TYPE           2   /* unknown type tag (rock_serdes.c:561) */
#define RR_E_STR_ENC        3   /* string enc not RAW/INT/EMBSTR (rock_serdes.c:148) */
#define RR_E_STR_INTLEN     4   /* INT string payload != 8 bytes (rock_serdes.c:145) */
#define RR_E_EMBSTR_LEN     5   /* EMBSTR longer than 44 (rock_serdes.c:152) */
#define RR_E_TRUNC          6   /* a length field runs past the blob (rock_serdes.c:202-206,288-295,...) */
#define RR_E_COUNT          7   /* element count disagrees with the header (rock_serdes.c:303,404,501) */
#define RR_E_INTSET         8   /* contents length != width*count (rock_serdes.c:274); [stricter]
                                   also width not 2/4/8 and the u32 wrap of width*count */
#define RR_E_ZL_LEN         9   /* ziplist byte count != remaining blob (rock_serdes.c:360,459) */
#define RR_E_ZL_CORRUPT     10  /* [stricter] ziplist entries / zltail / zllen / odd pair count do
                                   not parse by ziplist.c:300-447 (the reference copies them blind) */
#define RR_E_CAPACITY       11  /* output descriptor / byte capacity exceeded (batch API only) */
#define RR_E_ENCODE         12  /* flat value cannot be encoded (bad kind / missing ZLRAW / status
                                   != 0 / descriptor or payload outside the caller's buffers) */
#define RR_E_DUP            13  /* HASH_HT duplicate field: dictAdd != DICT_OK, rock_serdes.c:399-400 */
#define RR_E_NAN            14  /* ZSET_SKIPLIST NaN score: zslInsert serverAssert(!isnan(score)),
                                   t_zset.c:137 reached from rock_serdes.c:498 */
#define RR_N_STATUS         15

typedef struct rr_value {   /* 16 bytes */
    uint8_t  type;          /* RR_TYPE_* */
    uint8_t  enc;           /* STRING: RR_ENC_*; SET_INTSET: width 2/4/8; else 0 */
    uint16_t status;        /* RR_OK or RR_E_* (decode) */
    uint32_t lru;           /* low 24 bits of the stored u32 (robj.lru bitfield) */
    uint32_t n_elems;
    uint32_t elem_base;
} rr_value;

typedef struct rr_elem {    /* 16 bytes */
    uint64_t data;          /* STR/ZLRAW: arena byte offset; INT: int64; SCORE: f64 bits */
    uint32_t len;           /* STR/ZLRAW: byte length; else 0 */
    uint8_t  kind;          /* RR_K_* */
    uint8_t  zenc;          /* ziplist entries: the entry encoding byte; else 0 */
    uint16_t rsv;
} rr_elem;

#ifdef __cplusplus
}
#endif
#endif
