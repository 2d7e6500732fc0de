/*
 * server.h — a minimal model of the Redis API that redrock_old_amd/compat/rock_serdes_compat.c
 * uses, for the shim's unit test only (TEST INFRASTRUCTURE: never linked into the engine).
 * Inside a real RedRock tree the shim includes the tree's own server.h instead.
 *
 * Names, types and signatures follow the reference: robj (server.h:586-599), object
 * constructors (object.c:41-258), sds (sds.c:89-170), dict (dict.h:141-147, dict.c:111-597),
 * quicklist (quicklist.h:90-166), intset (intset.h:35-39), zskiplist/zset (server.h:866-885,
 * t_zset.c:132), ziplistBlobLen (ziplist.c:1186), ll2string (util.h:54).  The behaviour is
 * simplified where the shim cannot tell: a dict iterates in insertion order, a skiplist is a
 * sorted doubly linked list, a quicklist is one array.  serverPanic / serverAssert jump back
 * into the test (mr_panic_jmp) instead of exiting, so a test can observe an abort.
 */
#ifndef MINIREDIS_SERVER_H
#define MINIREDIS_SERVER_H

#include <setjmp.h>
#include <stddef.h>
#include <stdint.h>

typedef char *sds;
extern const char *SDS_NOINIT;   /* sds.h:37: sdsnewlen leaves the buffer uninitialised */
sds sdsnewlen(const void *init, size_t initlen);
size_t sdslen(const sds s);
void sdsfree(sds s);

void *zmalloc(size_t size);
void *zrealloc(void *ptr, size_t size);
void zfree(void *ptr);

#define OBJ_STRING 0
#define OBJ_LIST 1
#define OBJ_SET 2
#define OBJ_ZSET 3
#define OBJ_HASH 4
#define OBJ_ENCODING_RAW 0
#define OBJ_ENCODING_INT 1
#define OBJ_ENCODING_HT 2
#define OBJ_ENCODING_ZIPLIST 5
#define OBJ_ENCODING_INTSET 6
#define OBJ_ENCODING_SKIPLIST 7
#define OBJ_ENCODING_EMBSTR 8
#define OBJ_ENCODING_QUICKLIST 9
#define LRU_BITS 24
typedef struct redisObject {
    unsigned type : 4;
    unsigned encoding : 4;
    unsigned lru : LRU_BITS;
    int refcount;
    void *ptr;
} robj;

/* dict */
#define DICT_OK 0
#define DICT_ERR 1
#define DICT_HT_INITIAL_SIZE 4
typedef struct dictType { int unused; } dictType;
typedef struct dictEntry { void *key; union { void *val; } v; } dictEntry;
typedef struct dict { dictEntry *ents; unsigned long used, cap; dictType *type; } dict;
typedef struct dictIterator { dict *d; unsigned long i; } dictIterator;
#define dictGetKey(he) ((he)->key)
#define dictGetVal(he) ((he)->v.val)
#define dictSize(d) ((d)->used)
extern dictType setDictType, hashDictType, zsetDictType;
dict *dictCreate(dictType *type, void *privDataPtr);
int dictExpand(dict *d, unsigned long size);
int dictAdd(dict *d, void *key, void *val);
dictEntry *dictFind(dict *d, const void *key);
dictIterator *dictGetIterator(dict *d);
dictEntry *dictNext(dictIterator *iter);
void dictReleaseIterator(dictIterator *iter);

/* quicklist */
typedef struct quicklist quicklist;
typedef struct quicklistIter quicklistIter;
typedef struct quicklistEntry {
    const quicklist *quicklist;
    void *node;
    unsigned char *zi;
    unsigned char *value;
    long long longval;
    unsigned int sz;
    int offset;
} quicklistEntry;
#define AL_START_HEAD 0
void quicklistSetOptions(quicklist *ql, int fill, int depth);
int quicklistPushTail(quicklist *ql, void *value, size_t sz);
quicklistIter *quicklistGetIterator(const quicklist *ql, int direction);
int quicklistNext(quicklistIter *iter, quicklistEntry *entry);
void quicklistReleaseIterator(quicklistIter *iter);

/* intset */
typedef struct intset { uint32_t encoding; uint32_t length; int8_t contents[]; } intset;

/* sorted set */
typedef struct zskiplistNode {
    sds ele;
    double score;
    struct zskiplistNode *backward, *forward;
} zskiplistNode;
typedef struct zskiplist { zskiplistNode *header, *tail; unsigned long length; int level; } zskiplist;
typedef struct zset { dict *dict; zskiplist *zsl; } zset;
zskiplistNode *zslInsert(zskiplist *zsl, double score, sds ele);

size_t ziplistBlobLen(unsigned char *zl);
int ll2string(char *s, size_t len, long long value);

robj *createObject(int type, void *ptr);
robj *createRawStringObject(const char *ptr, size_t len);
robj *createEmbeddedStringObject(const char *ptr, size_t len);
robj *createStringObjectFromLongLongForValue(long long value);
robj *createQuicklistObject(void);
robj *createSetObject(void);
robj *createIntsetObject(void);
robj *createZsetObject(void);
void decrRefCount(robj *o);

sds sdsfromlonglong(long long value);

/* server.h:1059 keyspace of one database (the model keeps only its main dict) */
typedef struct redisDb { dict *dict; } redisDb;
struct redisServer { int list_max_ziplist_size; int list_compress_depth; redisDb *db; };
extern struct redisServer server;
void mr_init_db(void);   /* server.db[0] with an empty keyspace dict */

/* serverLog levels, server.h:344-347; the model appends every line to mr_log (and stdout) */
#define LL_DEBUG 0
#define LL_VERBOSE 1
#define LL_NOTICE 2
#define LL_WARNING 3
extern char *mr_log;       /* all lines logged so far, '\n'-separated */
extern size_t mr_log_len;
void mr_log_reset(void);
void serverLog(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

extern jmp_buf *mr_panic_jmp;
extern char mr_panic_msg[256];
__attribute__((noreturn)) void _serverPanic(const char *file, int line, const char *msg, ...);
__attribute__((noreturn)) void _serverAssert(const char *estr, const char *file, int line);
#define serverPanic(...) _serverPanic(__FILE__, __LINE__, __VA_ARGS__)
#define serverAssert(_e) ((_e) ? (void)0 : _serverAssert(#_e, __FILE__, __LINE__))

#endif
