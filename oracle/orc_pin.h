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

static int orc_pin_cpus[1024];
static int orc_pin_n = -1;
static pthread_once_t orc_pin_once = PTHREAD_ONCE_INIT;

static void orc_pin_init(void) {
    const char *e = getenv("ORC_PIN");
    orc_pin_n = 0;
    if (e && e[0] == '0')
        return;
    const char *l = getenv("ORC_CPUS");
    if (l && *l) {
        while (*l && orc_pin_n < 1024) {
            char *end = NULL;
            const long c = strtol(l, &end, 10);
            if (end == l)
                break;
            if (c >= 0 && c < CPU_SETSIZE)
                orc_pin_cpus[orc_pin_n++] = (int)c;
            l = *end == ',' ? end + 1 : end;
        }
        if (orc_pin_n > 0)
            return;
    }
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) != 0)
        return;
    for (int c = 0; c < CPU_SETSIZE && orc_pin_n < 1024; c++)
        if (CPU_ISSET(c, &set))
            orc_pin_cpus[orc_pin_n++] = c;
}

/* Pin thread `t` (worker index idx) to one CPU of the affinity mask. */
static inline void orc_pin_thread(pthread_t t, int idx) {
    pthread_once(&orc_pin_once, orc_pin_init);
    if (orc_pin_n <= 0)
        return;
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(orc_pin_cpus[idx % orc_pin_n], &one);
    (void)pthread_setaffinity_np(t, sizeof one, &one);
}

#endif
