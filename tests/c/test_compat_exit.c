/*
 * test_compat_exit.c — the compat shim at process exit, with threads the shim does not own still
 * calling it (RedRock's rock thread, rock.c:615, is never joined and loops on desObject,
 * rock.c:552-596).  Deterministic: the window the exit must survive is held open by a test hook.
 *
 *   thread A  decodes one value on the GPU route and ends; its engine context's teardown (the
 *             shim destroys a thread's context when the thread ends) is held inside the engine
 *             for 400 ms by rr_compat_test_hold_teardown;
 *   thread B  loops desObject on the GPU route, forever;
 *   main      once A's teardown is being held and B has made 20 calls, calls exit(0).
 *
 * The shim's exit handler must wait for A's teardown and for B's call in flight, and park B's
 * next call, before the HIP runtime's own teardown runs: the process exits 0 and prints the
 * state it exited in.  (Round 5's compat test died with SIGSEGV at exit twice: a thread inside
 * the runtime while it was torn down)
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "server.h"
#include "rock_serdes_compat.h"

/* K1 of SURVEY.md §8c (String INT 134123) and a List, both valid */
static const unsigned char k1[] = {0x00, 0, 0, 0, 0, 0x01, 0xEB, 0x0B, 0x02, 0, 0, 0, 0, 0};
static const unsigned char k4[] = {0x0E, 0, 0, 0, 0, 3, 0, 0, 0, 'x', 'x', 'x', 8, 0, 0, 0,
                                   '-', '1', '2', '3', '4', '5', '6', '7'};
static int b_calls;

static void *thread_a(void *arg) {
    (void)arg;
    decrRefCount(desObject((void *)k1, sizeof k1));
    rr_compat_test_hold_teardown(400);
    return NULL;   /* -> the held teardown of this thread's context */
}

static void *thread_b(void *arg) {
    (void)arg;
    for (;;) {
        decrRefCount(desObject((void *)k4, sizeof k4));
        __atomic_add_fetch(&b_calls, 1, __ATOMIC_SEQ_CST);
    }
    return NULL;
}

int main(void) {
    setvbuf(stdout, NULL, _IONBF, 0);
    rr_compat_set_route(RR_COMPAT_ROUTE_GPU);
    decrRefCount(desObject((void *)k1, sizeof k1));   /* the owner's context and exit handler */
    pthread_t a, b;
    if (pthread_create(&a, NULL, thread_a, NULL) || pthread_create(&b, NULL, thread_b, NULL)) return 2;
    const struct timespec ms = {0, 1000000};
    for (int i = 0; !(rr_compat_test_holding() && __atomic_load_n(&b_calls, __ATOMIC_SEQ_CST) >= 20); i++) {
        if (i > 30000) {
            printf("setup timed out: holding %d, thread B calls %d\n", rr_compat_test_holding(), b_calls);
            return 3;
        }
        nanosleep(&ms, NULL);
    }
    printf("exit: thread A's teardown held, thread B at %d calls, %d engine calls in flight\n",
           __atomic_load_n(&b_calls, __ATOMIC_SEQ_CST), rr_compat_in_flight());
    exit(0);
}
