/*
 * test_compat.c — unit test of the legacy-signature shim (redrock_old_amd/compat/
 * rock_serdes_compat.c) through desObject / desString / serObject and the batch forms, over the
 * golden fixtures (tests/golden/kat.json, K1-K9 + edge cases + the reference's test shapes;
 * written into fixtures.h by tests/test_compat.py), linked with the minimal Redis model
 * (tests/c/miniredis) and the engine library.
 *
 * Every fixture, on each route:  status != 0 -> desObject must panic (the reference's
 *                                serverAssert site);
 *                                status == 0 -> serObject(desObject(b)) must be the blob serObject
 *                                writes for the object desObject built (the fixture's
 *                                "reencoded", lru masked to 24 bits), and desString must keep the
 *                                caller's lru.
 *   host   (CPU suite)  the host codec route (the default for one value); the batch forms; the
 *                       fork-child route in-process and through a real fork (the child decodes on
 *                       its own CPU; forced onto the GPU route it must refuse, not touch HIP).
 *   gpu    (GPU suite)  the host checks, then the same fixtures through the GPU route: every
 *                       object equal to the host route's, every blob equal; a fork after the
 *                       parent used the GPU.
 * Exit status 0 when every check passes.
 */
#include <stdio.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "server.h"
#include "rock_serdes_compat.h"
#include "fixtures.h"

static int fails;
#define CHECK(c, ...) do { if (!(c)) { fails++; printf("FAIL %s: ", fx ? fx->name : "-"); printf(__VA_ARGS__); printf("\n"); } } while (0)

/* Structural equality of two objects of the minimal Redis model. */
static int sds_eq(sds a, sds b) { return sdslen(a) == sdslen(b) && !memcmp(a, b, sdslen(a)); }
static int dict_eq(dict *a, dict *b, int vals) {
    if (dictSize(a) != dictSize(b)) return 0;
    dictIterator *it = dictGetIterator(a);
    dictEntry *e;
    int ok = 1;
    while (ok && (e = dictNext(it))) {
        dictEntry *f = dictFind(b, dictGetKey(e));
        ok = f && (!vals || sds_eq(dictGetVal(e), dictGetVal(f)));
    }
    dictReleaseIterator(it);
    return ok;
}
static int obj_eq(robj *a, robj *b) {
    if (a->type != b->type || a->encoding != b->encoding || a->lru != b->lru) return 0;
    switch (a->encoding) {
        case OBJ_ENCODING_INT: return a->ptr == b->ptr;
        case OBJ_ENCODING_RAW:
        case OBJ_ENCODING_EMBSTR: return sds_eq(a->ptr, b->ptr);
        case OBJ_ENCODING_ZIPLIST: {
            const size_t l = ziplistBlobLen(a->ptr);
            return l == ziplistBlobLen(b->ptr) && !memcmp(a->ptr, b->ptr, l);
        }
        case OBJ_ENCODING_INTSET: {
            const intset *x = a->ptr, *y = b->ptr;
            return x->encoding == y->encoding && x->length == y->length &&
                   !memcmp(x->contents, y->contents, (size_t)x->encoding * x->length);
        }
        case OBJ_ENCODING_QUICKLIST: {
            quicklistIter *i = quicklistGetIterator(a->ptr, AL_START_HEAD), *j = quicklistGetIterator(b->ptr, AL_START_HEAD);
            quicklistEntry x, y;
            int ok = 1, nx, ny;
            while (ok && (nx = quicklistNext(i, &x)) & (ny = quicklistNext(j, &y)))
                ok = (x.value == NULL) == (y.value == NULL) &&
                     (x.value ? x.sz == y.sz && !memcmp(x.value, y.value, x.sz) : x.longval == y.longval);
            ok = ok && !nx && !ny;
            quicklistReleaseIterator(i);
            quicklistReleaseIterator(j);
            return ok;
        }
        case OBJ_ENCODING_HT: return dict_eq(a->ptr, b->ptr, a->type == OBJ_HASH);
        case OBJ_ENCODING_SKIPLIST: {
            const zset *x = a->ptr, *y = b->ptr;
            if (x->zsl->length != y->zsl->length || !dict_eq(x->dict, y->dict, 0)) return 0;
            for (zskiplistNode *n = x->zsl->header, *m = y->zsl->header; n || m; n = n->forward, m = m->forward)
                if (!n || !m || n->score != m->score || !sds_eq(n->ele, m->ele)) return 0;
            return 1;
        }
        default: return 0;
    }
}

static void *bufs[N_FIXTURES];
static size_t lens[N_FIXTURES], nok;
static const fixture_t *okfx[N_FIXTURES];

/* every fixture through the one-value signatures on the current route; returns the panics */
static int one_value_route(const char *route, robj **keep) {
    int panics = 0;
    const fixture_t *fx = NULL;
    nok = 0;
    for (int i = 0; i < N_FIXTURES; i++) {
        fx = &FIXTURES[i];
        jmp_buf jb;
        mr_panic_jmp = &jb;
        robj *volatile o = NULL;
        if (setjmp(jb) == 0) {
            o = desObject((void *)fx->blob, fx->len);
        } else {
            CHECK(fx->status != 0, "%s: desObject panicked on a valid blob: %s", route, mr_panic_msg);
            if (fx->status) panics++;
            continue;
        }
        mr_panic_jmp = NULL;
        CHECK(fx->status == 0, "%s: desObject accepted a blob the reference rejects (status %d)", route, fx->status);
        if (fx->status) continue;
        sds s = serObject(o);
        CHECK(sdslen(s) == fx->out_len && !memcmp(s, fx->out, fx->out_len),
              "%s: serObject(desObject(b)) differs (%zu vs %zu bytes)", route, sdslen(s), fx->out_len);
        if (fx->blob[0] == 0) {   /* String: desString keeps the caller's lru */
            robj *o2 = desString((char *)fx->blob, fx->len, 77);
            CHECK(o2->lru == 77 && o2->type == OBJ_STRING && o2->encoding == o->encoding, "%s: desString", route);
            decrRefCount(o2);
        }
        sdsfree(s);
        if (keep) keep[nok] = o;
        else decrRefCount(o);
        bufs[nok] = (void *)fx->blob;
        lens[nok] = fx->len;
        okfx[nok++] = fx;
    }
    mr_panic_jmp = NULL;
    return panics;
}

/* the batch forms on the current route: every valid fixture in one call each way */
static void batch_route(const char *route) {
    robj *objs[N_FIXTURES];
    sds outs[N_FIXTURES];
    const fixture_t *fx = NULL;
    rr_compat_des_batch(bufs, lens, nok, objs);
    rr_compat_ser_batch(objs, nok, outs);
    for (size_t i = 0; i < nok; i++) {
        fx = okfx[i];
        CHECK(sdslen(outs[i]) == fx->out_len && !memcmp(outs[i], fx->out, fx->out_len), "%s: batch round trip differs", route);
        sdsfree(outs[i]);
        decrRefCount(objs[i]);
    }
}

/* a real fork (rock.c:536-538) after the parent decoded the valid fixtures (pobj): the child's
 * desObject (default route) must build the same objects on its own CPU; the child leaves with
 * _exit (it never touches the HIP runtime, not even through exit handlers) */
static void forked_child_route(robj **pobj, int parent_used_gpu) {
    const fixture_t *fx = NULL;
    fflush(stdout);
    const pid_t pid = fork();
    if (pid == 0) {
        int bad = 0;
        rr_compat_set_route(RR_COMPAT_ROUTE_AUTO);
        for (size_t i = 0; i < nok; i++) {
            robj *o = desObject(bufs[i], lens[i]);
            if (!obj_eq(o, pobj[i])) bad++;
            sds s = serObject(o);
            if (sdslen(s) != okfx[i]->out_len || memcmp(s, okfx[i]->out, okfx[i]->out_len)) bad++;
            sdsfree(s);
            decrRefCount(o);
        }
        _exit(bad ? 1 : 0);
    }
    int wst = -1;
    CHECK(pid > 0 && waitpid(pid, &wst, 0) == pid, "fork / waitpid");
    CHECK(WIFEXITED(wst) && WEXITSTATUS(wst) == 0, "forked child: decode differs (wait status %d)", wst);

    /* forced onto the GPU route, the child of a parent whose HIP runtime is up must refuse (panic,
     * exit 3) rather than touch it */
    if (!parent_used_gpu) return;
    const pid_t pc = fork();
    if (pc == 0) {
        rr_compat_set_route(RR_COMPAT_ROUTE_GPU);
        jmp_buf jb;
        mr_panic_jmp = &jb;
        if (setjmp(jb) == 0) {
            (void)desObject(bufs[0], lens[0]);
            _exit(5);
        }
        _exit(strstr(mr_panic_msg, "fork child") ? 3 : 4);
    }
    CHECK(pc > 0 && waitpid(pc, &wst, 0) == pc && WIFEXITED(wst) && WEXITSTATUS(wst) == 3,
          "child forced onto the GPU route: expected a refusal (exit 3), wait status %d", wst);
}

int main(int argc, char **argv) {
    setvbuf(stdout, NULL, _IONBF, 0);   /* (a crash keeps what was printed) */
    const int gpu = argc > 1 && !strcmp(argv[1], "gpu");
    const fixture_t *fx = NULL;
    robj *hobj[N_FIXTURES];

    /* the host route: one value per call (RedRock's call sites), the batch forms */
    rr_compat_set_route(RR_COMPAT_ROUTE_HOST);
    const int panics = one_value_route("host", hobj);
    const size_t nvalid = nok;
    batch_route("host");

    /* the fork-child route in-process: desObject on the host, the GPU route refused */
    rr_compat_test_as_child(1);
    rr_compat_set_route(RR_COMPAT_ROUTE_AUTO);
    const int child_panics = one_value_route("child", NULL);
    CHECK(child_panics == panics && nok == nvalid, "child route rejected %d malformed blobs, parent %d", child_panics,
          panics);
    {
        rr_compat_set_route(RR_COMPAT_ROUTE_GPU);
        jmp_buf jb;
        mr_panic_jmp = &jb;
        volatile int refused = 0;
        if (setjmp(jb) == 0) (void)desObject(bufs[0], lens[0]);
        else refused = strstr(mr_panic_msg, "fork child") != NULL;
        mr_panic_jmp = NULL;
        CHECK(refused, "the engine must refuse a child: %s", mr_panic_msg);
        CHECK(rr_compat_in_flight() == 0, "a refused call left %d engine calls in flight", rr_compat_in_flight());
    }
    rr_compat_test_as_child(0);

    int gpu_checked = 0;
    if (gpu) {   /* the GPU route: the same verdicts, the same objects, the same blobs */
        rr_compat_set_route(RR_COMPAT_ROUTE_GPU);
        robj *gobj[N_FIXTURES];
        const int gpanics = one_value_route("gpu", gobj);
        CHECK(gpanics == panics && nok == nvalid, "gpu route rejected %d malformed blobs, host %d", gpanics, panics);
        for (size_t i = 0; i < nok; i++) {
            fx = okfx[i];
            CHECK(obj_eq(gobj[i], hobj[i]), "gpu route's object differs from the host route's");
            decrRefCount(gobj[i]);
            gpu_checked++;
        }
        batch_route("gpu");
        CHECK(rr_compat_in_flight() == 0, "%d engine calls still in flight", rr_compat_in_flight());
    }
    fx = NULL;
    forked_child_route(hobj, gpu);   /* (after the GPU route: the parent's HIP runtime is up) */
    for (size_t i = 0; i < nvalid; i++) decrRefCount(hobj[i]);
    printf("compat shim: %zu fixtures round-tripped, %d rejected with a panic (host route, batch, child route)%s%s; "
           "%d failures\n", nvalid, panics, gpu ? ", gpu route objects equal: " : "", gpu ? (gpu_checked ? "yes" : "no") : "",
           fails);
    return fails ? 1 : 0;
}
