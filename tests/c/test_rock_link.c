/*
 * test_rock_link.c — the drop-in link check of the legacy boundary: a
 * translation unit that sees the serdes functions exactly as rock.c does, through the
 * prototypes of rock_serdes.h:47-55 (the two-argument desString included, which nothing calls),
 * linked against the shim (redrock_old_amd/compat/rock_serdes_compat.c), the minimal Redis model
 * and librr_serdes.so.  It runs rock.c's call set: rockCommand's `ROCK testserdes*` hooks
 * (rock.c:170-184) on live keys of db 0, desObject (rock.c:468, :538) and serObject (:691).
 * TEST INFRASTRUCTURE.  Exit status 0 when every logged result is the expected one.
 */
#include <stdio.h>
#include <string.h>

#include "server.h"   /* (the Redis tree's server.h in RedRock) */

/* rock_serdes.h:47-55, as rock.c includes them */
robj *desString(char *s, size_t len);
sds serObject(robj *o);
robj *desObject(void *buf, size_t len);
void _test_ser_des_string(void);
void _test_ser_des_list(void);
void _test_ser_des_set(void);
void _test_ser_des_hash(void);
void _test_ser_des_zset(void);

static int fails;
#define EXPECT(line) do { if (!strstr(mr_log ? mr_log : "", line)) { fails++; printf("FAIL: log lacks \"%s\"\n", line); } } while (0)

static void set_key(const char *name, robj *o) {
    sds key = sdsnewlen(name, strlen(name));
    dictEntry *de = dictFind(server.db[0].dict, key);
    if (de) { decrRefCount(dictGetVal(de)); de->v.val = o; sdsfree(key); }
    else dictAdd(server.db[0].dict, key, o);
}

int main(void) {
    mr_init_db();
    robj *(*des_string_as_rock_c_sees_it)(char *, size_t) = desString;   /* linked, not called */
    if (!des_string_as_rock_c_sees_it) fails++;

    /* ROCK testserdesstr: the three literal strings through serObject + desString */
    mr_log_reset();
    _test_ser_des_string();
    EXPECT("1 round trip ok, blob len = 14");
    EXPECT("2 round trip ok, blob len = 9");
    EXPECT("3 round trip ok, blob len = 66");

    /* ROCK testserdeslist: key abc holds a quicklist */
    robj *list = createQuicklistObject();
    sds e0 = sdsnewlen("hello", 5), e1 = sdsfromlonglong(42);
    quicklistPushTail(list->ptr, e0, sdslen(e0));
    quicklistPushTail(list->ptr, e1, sdslen(e1));
    sdsfree(e0); sdsfree(e1);
    set_key("abc", list);
    mr_log_reset();
    _test_ser_des_list();
    EXPECT("index = 0, entry sz = 5, entry val = hello");
    EXPECT("index = 1, entry long value = 42");
    EXPECT("index = 0, entry sz = 3, entry val = xxx");
    EXPECT("index = 1, entry long value = -1234567");

    /* ROCK testserdeshash: key abc holds an HT hash */
    robj *hash = createObject(OBJ_HASH, dictCreate(&hashDictType, NULL));
    hash->encoding = OBJ_ENCODING_HT;
    dictAdd(hash->ptr, sdsnewlen("f1", 2), sdsnewlen("v1", 2));
    dictAdd(hash->ptr, sdsnewlen("f2", 2), sdsnewlen("value-two", 9));
    set_key("abc", hash);
    mr_log_reset();
    _test_ser_des_hash();
    EXPECT("des encoding = ht");
    EXPECT("no = 0, field = f1, val = v1");
    EXPECT("no = 1, field = f2, val = value-two");

    /* ROCK testserdeszset: key abc holds a skiplist zset */
    robj *zs = createZsetObject();
    zset *z = zs->ptr;
    const char *mem[3] = {"a", "b", "c"};
    const double sc[3] = {1.5, -2.0, 7.0};
    for (int i = 0; i < 3; i++) {
        sds m = sdsnewlen(mem[i], 1);
        zskiplistNode *zn = zslInsert(z->zsl, sc[i], m);
        dictAdd(z->dict, m, &zn->score);
    }
    set_key("abc", zs);
    mr_log_reset();
    _test_ser_des_zset();
    EXPECT("des encoding = skiplist");
    EXPECT("zset skiplist i = 0, key = c, score = 7.000000");
    EXPECT("zset skiplist i = 2, key = b, score = -2.000000");

    /* ROCK testserdesset: key def holds an HT set (and abc is not a set: the hook only logs) */
    robj *set = createSetObject();
    dictAdd(set->ptr, sdsnewlen("m1", 2), NULL);
    dictAdd(set->ptr, sdsnewlen("", 0), NULL);
    set_key("def", set);
    mr_log_reset();
    _test_ser_des_set();
    EXPECT("set ht, key = m1, val is null");
    EXPECT("set ht, key = , val is null");
    mr_log_reset();
    _test_ser_des_list();   /* abc is a zset now */
    EXPECT("val type or encoding not correct!");

    /* rock.c:691 / :468: serObject, then desObject of the blob */
    sds blob = serObject(set);
    robj *back = desObject(blob, sdslen(blob));
    if (back->type != OBJ_SET || back->encoding != OBJ_ENCODING_HT || dictSize((dict *)back->ptr) != 2) {
        fails++;
        printf("FAIL: desObject(serObject(set))\n");
    }
    decrRefCount(back);
    sdsfree(blob);
    printf("rock.c link set: %d failures\n", fails);
    return fails ? 1 : 0;
}
