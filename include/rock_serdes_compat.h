/*
 * rock_serdes_compat.h — RedRock's legacy serdes entry points (src/rock_serdes.h:47-49) on
 * the MI355X engine, for a build inside a Redis tree.
 *
 * The bodies are redrock_old_amd/compat/rock_serdes_compat.c.  They need Redis's robj / sds /
 * dict / quicklist / intset / skiplist (server.h), so this header declares them only when
 * compiled inside a RedRock tree: -DRR_REDIS_TREE, after #include "server.h".
 *
 *   desObject / desString   the blob goes through rr_decode_batch_host (the GPU decode), the
 *                           robj is built on the host from the flat records — heap objects
 *                           cannot be built on the device;
 *   serObject               the robj is flattened on the host, rr_encode_batch_host writes
 *                           the blob (the GPU encode), returned as a fresh zmalloc'd sds;
 *   any nonzero per-value status, and any engine error, ends in serverPanic() — the
 *   reference aborts through serverAssert/serverPanic on the same inputs (rock_serdes.c).
 *
 * One value per call pays a kernel launch; the batch forms below are what the RedRock call
 * sites should use: the rock thread's restore queue (rock.c:302-383, one key per RockJob
 * today, server.h:1013-1019) and the fork child's snapshot loads (rock.c:527-540) restore
 * many keys per call, and the evictor (rock_hotkey.c:315-455) dumps many victims per call.
 * INTEGRATION.md shows the patches.
 */
#ifndef ROCK_SERDES_COMPAT_H
#define ROCK_SERDES_COMPAT_H

#include "rr_serdes.h"
#include "rr_rdb.h"

#ifdef RR_REDIS_TREE
/* rock_serdes.h:47 declares 2 args; the definition (rock_serdes.c:133) takes the lru too, and
 * that is the one provided (nothing outside rock_serdes.c calls it). */
robj *desString(char *s, size_t len, uint32_t lru);
sds serObject(robj *o);                 /* rock_serdes.h:48, rock_serdes.c:512 */
robj *desObject(void *buf, size_t len); /* rock_serdes.h:49, rock_serdes.c:538 */

/* Batch forms: n blobs -> n robj (out[i] == desObject(bufs[i], lens[i])), n robj -> n sds
 * (out[i] == serObject(objs[i])), one engine call each. */
void rr_compat_des_batch(void *const *bufs, const size_t *lens, size_t n, robj **out);
void rr_compat_ser_batch(robj *const *objs, size_t n, sds *out);

/* Row f4 (rr_rdb.h): the fork child's batch restore.  k keys of database dbid, held in the
 * parent's RocksDB snapshot, requested over the child's pipes (rock_rdb.c:240-267) in one FLAT
 * request: the parent's service (rr_rdb_serve) decodes them on its GPU and the robj are built
 * here from the records — out[i] == loadValFromRockForRdb(dbid, keys[i]) (rock.c:527-550).
 * The child never touches the GPU. */
void rr_compat_rdb_load_batch(int fd_req, int fd_resp, int dbid, sds *keys, size_t k, robj **out);

/* GPU the calling thread's engine context is created on (default 0; set before first use). */
void rr_compat_set_device(int device);

/* rock_serdes.h:51-55: the debug round trips of `ROCK testserdes*` (rock.c:170-184), over the
 * engine, logging through serverLog as the reference's do (rock_serdes.c:626-901). */
void _test_ser_des_string(void);
void _test_ser_des_list(void);
void _test_ser_des_set(void);
void _test_ser_des_hash(void);
void _test_ser_des_zset(void);

/* Fork children (rock.c:527-550).  A process that has used the engine opens, right before each
 * fork (pthread_atfork), a connection of the child's own with a decode service thread behind
 * it; desObject in the child sends its blobs there over a socket and builds the robj from the
 * flat records that come back, never touching the HIP runtime.  The service ends when the
 * child closes its end (exit, kill) and closes its own end when a request fails, so a child
 * never reads another child's reply and never waits on a dead service.
 * rr_compat_service_start opens this process's own connection (0 or -1);
 * rr_compat_test_as_child(1) makes this process route desObject as a child would;
 * rr_compat_test_send_only writes one FLAT request and returns without its reply (a child
 * killed mid-call); rr_compat_test_drop_services shuts every live service end down (tests). */
int rr_compat_service_start(void);
void rr_compat_test_as_child(int on);
int rr_compat_test_send_only(const void *blob, size_t len);
void rr_compat_test_drop_services(void);
#endif

#endif
