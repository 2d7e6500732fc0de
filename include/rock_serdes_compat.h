/*
 * rock_serdes_compat.h — the legacy single-value signatures of RedRock's serdes
 * (src/rock_serdes.h:47-49), kept for a drop-in build inside a Redis tree.
 *
 * These need Redis's robj/sds types (server.h), so they are only declared when the file is
 * compiled inside a RedRock tree (-DRR_REDIS_TREE, after #include "server.h").  Their bodies
 * flatten an robj into the rr_format.h form, run a batch of one through rr_serdes.h and turn
 * any nonzero per-value status into serverPanic() — the reference's abort-on-malformed
 * semantics (rock_serdes.c asserts).  Status: SURVEY.md §8f row f1 ("next"); see
 * INTEGRATION.md for the patch to rock.c (:468, :538, :691) that switches callers to the
 * batch entry points instead.
 */
#ifndef ROCK_SERDES_COMPAT_H
#define ROCK_SERDES_COMPAT_H

#include "rr_serdes.h"

#ifdef RR_REDIS_TREE
/* rock_serdes.h:47 declares 2 args; the definition (rock_serdes.c:133) takes the lru too. */
robj *desString(char *s, size_t len);
sds serObject(robj *o);                 /* rock_serdes.h:48, rock_serdes.c:512 */
robj *desObject(void *buf, size_t len); /* rock_serdes.h:49, rock_serdes.c:538 */
#endif

#endif
