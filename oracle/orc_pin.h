/*
 * orc_pin.h — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * Worker thread t of a timed CPU run is pinned to the t-th CPU of
 * ORC_CPUS (a comma-separated list: bench.py passes the least busy CPUs of
 * the mask, one per physical core) or else of the process's affinity mask,
 * so a 16-thread run on a 16-CPU share of a large host keeps one worker per
 * CPU instead of migrating between them (the CPU baseline moved
 * 15-25 % between repetitions).  ORC_PIN=0 in the environment turns it off.
 * Must be included before any system header that reads _GNU_SOURCE.
 */
#ifndef WG_ORC_PIN_H
#define WG_ORC_PIN_H

#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>

/* The idx-th CPU of ORC_CPUS (read at every call: bench.py re-picks the
 * quietest CPUs before each timed repetition), else of the affinity mask;
 * -1 when pinning is off or nothing is known. */
static int orc_pin_cpu(int idx) {
    const char *e = getenv("ORC_PIN");
    if (e && e[0] == '0')
        return -1;
    const char *l = getenv("ORC_CPUS");
    if (l && *l) {
        int list[1024], n = 0;
        while (*l && n < 1024) {
            char *end = NULL;
            const long c = strtol(l, &end, 10);
            if (end == l)
                break;
            if (c >= 0 && c < CPU_SETSIZE)
                list[n++] = (int)c;
            l = *end == ',' ? end + 1 : end;
        }
        if (n > 0)
            return list[idx % n];
    }
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) != 0)
        return -1;
    const int n = CPU_COUNT(&set);
    if (n <= 0)
        return -1;
    for (int c = 0, k = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &set) && k++ == idx % n)
            return c;
    return -1;
}

/* A one-thread timed run goes to a pinned worker too when bench.py names
 * the CPUs (ORC_CPUS set, pinning on): run on the calling thread it could
 * migrate between cores of different speed from repetition to repetition
 * (round 4's bimodal 1-core leg).  Without ORC_CPUS (tests) one thread runs
 * on the caller. */
static inline int orc_pin_single(void) {
    const char *e = getenv("ORC_PIN");
    const char *l = getenv("ORC_CPUS");
    return !(e && e[0] == '0') && l && *l;
}

/* Start worker idx on its CPU.  The CPU is set in the creation attributes,
 * never on the running thread by its handle: a worker that has already
 * finished carries TID 0 in its handle, and sched_setaffinity(0) pins the
 * CALLER — the timing thread then ended up on one CPU and every later
 * repetition with it (16 workers on one core: a 64-B verify baseline of 2.1
 * instead of 21.6 GiB/s).  A CPU the attributes cannot take: unpinned. */
static inline int orc_spawn(pthread_t *tid, int idx, void *(*fn)(void *), void *arg) {
    pthread_attr_t a;
    pthread_attr_init(&a);
    const int c = orc_pin_cpu(idx);
    if (c >= 0) {
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(c, &one);
        (void)pthread_attr_setaffinity_np(&a, sizeof one, &one);
    }
    int rc = pthread_create(tid, &a, fn, arg);
    pthread_attr_destroy(&a);
    if (rc != 0)
        rc = pthread_create(tid, NULL, fn, arg);
    return rc;
}

#endif
