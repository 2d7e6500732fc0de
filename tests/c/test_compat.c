/*
 * test_compat.c — unit test of the legacy-signature shim (redrock_old_amd/compat/
 * rock_serdes_compat.c) through desObject / desString / serObject and the batch forms,
 * over the golden fixtures (tests/golden/kat.json, K1-K9 + edge cases; written into
 * fixtures.h by tests/test_compat.py).  Links the engine library (the decode / encode run on
 * the GPU) and the minimal Redis model (tests/c/miniredis).
 *
 * Every fixture:  status != 0  -> desObject must panic (the reference's serverAssert site);
 *                 status == 0  -> serObject(desObject(b)) must be the blob serObject writes for
 *                                 the object desObject built (the fixture's "reencoded", lru
 *                                 masked to 24 bits), and desString must keep the caller's lru.
 * Then the fork-child route: in-process (rr_compat_test_as_child) and through real forks — a
 * child that decodes every valid fixture through the parent's decode service, a child killed
 * between its request and the reply followed by one that must get its own reply, and a child
 * whose service was shut down, which must panic rather than wait.
 * Exit status 0 when every check passes.
 */
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "server.h"
#include "rock_serdes_compat.h"
#include "fixtures.h"

static int fails;
#define CHECK(c, ...) do { if (!(c)) { fails++; printf("FAIL %s: ", fx->name); printf(__VA_ARGS__); printf("\n"); } } while (0)

/* Structural equality of two objects of the minimal Redis model (no serObject: a fork child
 * must not touch the GPU the parent's encode would use). */
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

int main(void) {
    setvbuf(stdout, NULL, _IONBF, 0);   /* (a crash keeps what was printed) */
    int checked = 0, panics = 0;
    robj *objs[N_FIXTURES];
    void *bufs[N_FIXTURES];
    size_t lens[N_FIXTURES], nok = 0;
    const fixture_t *okfx[N_FIXTURES];
    for (int i = 0; i < N_FIXTURES; i++) {
        const fixture_t *fx = &FIXTURES[i];
        jmp_buf jb;
        mr_panic_jmp = &jb;
        robj *volatile o = NULL;
        if (setjmp(jb) == 0) {
            o = desObject((void *)fx->blob, fx->len);
        } else {
            CHECK(fx->status != 0, "desObject panicked on a valid blob: %s", mr_panic_msg);
            if (fx->status) panics++;
            continue;
        }
        CHECK(fx->status == 0, "desObject accepted a blob the reference rejects (status %d)", fx->status);
        if (fx->status) continue;
        sds s = serObject(o);
        CHECK(sdslen(s) == fx->out_len && !memcmp(s, fx->out, fx->out_len), "serObject(desObject(b)) differs (%zu vs %zu bytes)",
              sdslen(s), fx->out_len);
        if (fx->blob[0] == 0) {   /* String: desString keeps the caller's lru */
            robj *o2 = desString((char *)fx->blob, fx->len, 77);
            CHECK(o2->lru == 77 && o2->type == OBJ_STRING && o2->encoding == o->encoding, "desString");
            decrRefCount(o2);
        }
        sdsfree(s);
        decrRefCount(o);
        bufs[nok] = (void *)fx->blob;
        lens[nok] = fx->len;
        okfx[nok++] = fx;
        checked++;
    }
    /* the batch forms: every valid fixture in one decode call and one encode call */
    mr_panic_jmp = NULL;
    rr_compat_des_batch(bufs, lens, nok, objs);
    sds outs[N_FIXTURES];
    rr_compat_ser_batch(objs, nok, outs);
    for (size_t i = 0; i < nok; i++) {
        const fixture_t *fx = okfx[i];
        CHECK(sdslen(outs[i]) == fx->out_len && !memcmp(outs[i], fx->out, fx->out_len), "batch round trip differs");
        sdsfree(outs[i]);
        decrRefCount(objs[i]);
    }
    /* a fork child's route (rock.c:538): desObject through the parent's decode service thread
     * (the process routes as a child; the service decodes on the GPU), then the objects compared
     * through serObject back in parent mode; the engine itself must refuse child use */
    const fixture_t *fx = NULL;
    CHECK(rr_compat_service_start() == 0, "decode service start");
    rr_compat_test_as_child(1);
    rr_compat_des_batch(bufs, lens, nok, objs);
    int child_panics = 0;
    for (int i = 0; i < N_FIXTURES; i++) {
        if (!FIXTURES[i].status) continue;
        jmp_buf jb;
        mr_panic_jmp = &jb;
        if (setjmp(jb) == 0) (void)desObject((void *)FIXTURES[i].blob, FIXTURES[i].len);
        else child_panics++;
    }
    {
        jmp_buf jb;
        mr_panic_jmp = &jb;
        volatile int refused = 0;
        if (setjmp(jb) == 0) (void)serObject(objs[0]);
        else refused = strstr(mr_panic_msg, "fork child") != NULL;
        CHECK(refused, "serObject in a child must refuse the GPU: %s", mr_panic_msg);
        mr_panic_jmp = NULL;
    }
    rr_compat_test_as_child(0);
    rr_compat_ser_batch(objs, nok, outs);
    for (size_t i = 0; i < nok; i++) {
        fx = okfx[i];
        CHECK(sdslen(outs[i]) == fx->out_len && !memcmp(outs[i], fx->out, fx->out_len), "child-route round trip differs");
        sdsfree(outs[i]);
        decrRefCount(objs[i]);
    }
    fx = &FIXTURES[0];
    CHECK(child_panics == panics, "child route rejected %d malformed blobs, parent %d", child_panics, panics);

    /* a real fork (rock.c:536-538): the parent decodes every valid fixture on its GPU (its engine
     * context exists), then forks; the child's desObject goes through the parent's decode
     * service and must build the same objects.  The child leaves with _exit: it never touches
     * the HIP runtime, not even through exit handlers. */
    robj *pobj[N_FIXTURES];
    for (size_t i = 0; i < nok; i++) pobj[i] = desObject(bufs[i], lens[i]);
    fflush(stdout);
    const pid_t pid = fork();
    if (pid == 0) {
        int bad = 0;
        for (size_t i = 0; i < nok; i++) {
            robj *o = desObject(bufs[i], lens[i]);
            if (!obj_eq(o, pobj[i])) bad++;
            decrRefCount(o);
        }
        _exit(bad ? 1 : 0);
    }
    int wst = -1;
    CHECK(pid > 0 && waitpid(pid, &wst, 0) == pid, "fork / waitpid");
    CHECK(WIFEXITED(wst) && WEXITSTATUS(wst) == 0, "forked child: decode differs or failed (wait status %d)", wst);

    /* a child killed between its request and the reply (killRDBChild): the next child must get
     * its own reply, not the dead child's (every fork has its own connection) */
    const size_t ia = 0, ib = nok - 1;
    const pid_t pa = fork();
    if (pa == 0) _exit(rr_compat_test_send_only(bufs[ia], lens[ia]) == 0 ? 0 : 2);
    CHECK(pa > 0 && waitpid(pa, &wst, 0) == pa && WIFEXITED(wst) && WEXITSTATUS(wst) == 0, "request-only child");
    const pid_t pb = fork();
    if (pb == 0) {
        robj *o = desObject(bufs[ib], lens[ib]);
        _exit(obj_eq(o, pobj[ib]) ? 0 : 1);
    }
    CHECK(pb > 0 && waitpid(pb, &wst, 0) == pb && WIFEXITED(wst) && WEXITSTATUS(wst) == 0,
          "child after a killed child: wrong object (a stale reply?), status %d", wst);

    /* the parent's service ends while a child is about to call: the child must fail (panic,
     * exit 3), not wait forever; an alarm turns a hang into a failure */
    int sync_fd[2];
    CHECK(pipe(sync_fd) == 0, "pipe");
    const pid_t pc = fork();
    if (pc == 0) {
        char c;
        close(sync_fd[1]);
        signal(SIGPIPE, SIG_IGN);   /* as Redis runs (server.c setupSignalHandlers) */
        alarm(20);
        if (read(sync_fd[0], &c, 1) != 1) _exit(4);
        jmp_buf jb;
        mr_panic_jmp = &jb;
        if (setjmp(jb) == 0) {
            (void)desObject(bufs[ia], lens[ia]);
            _exit(5);   /* decoded through a service that was shut down */
        }
        _exit(3);
    }
    close(sync_fd[0]);
    rr_compat_test_drop_services();
    CHECK(write(sync_fd[1], "x", 1) == 1, "sync write");
    close(sync_fd[1]);
    CHECK(pc > 0 && waitpid(pc, &wst, 0) == pc && WIFEXITED(wst) && WEXITSTATUS(wst) == 3,
          "child of a dead service: expected a panic (exit 3), wait status %d", wst);

    for (size_t i = 0; i < nok; i++) decrRefCount(pobj[i]);
    printf("compat shim: %d fixtures round-tripped, %d rejected with a panic, batch of %zu, child route %zu + %d, "
           "forked children 4; %d failures\n", checked, panics, nok, nok, child_panics, fails);
    return fails ? 1 : 0;
}
