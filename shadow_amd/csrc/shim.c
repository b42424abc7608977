/*
 * Weak stand-ins for the Shadow symbols the drop-in imports (shd_topology.h).
 * Inside Shadow the simulator's strong definitions replace every one of these:
 *   address_*           /root/reference/src/main/routing/shd-address.c:101-144
 *   random_nextDouble   /root/reference/src/main/utility/shd-random.c:30-41 (libc rand_r)
 *   worker_updateMinTimeJump  /root/reference/src/main/core/shd-worker.c:384-387
 * Standalone (tests, bench, INTEGRATION.md examples) they provide a minimal
 * Address/Random and record the min-latency upcall.
 */
#include <arpa/inet.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/shd_topology.h"

#define WEAK __attribute__((weak))

struct _Address {
    uint32_t ip; /* network order, as shd-address.c:16 */
    char ipString[INET6_ADDRSTRLEN + 1];
    char* name;
    char* idString;
};

struct _Random {
    unsigned int seedState;
    unsigned int initialSeed;
};

WEAK Address* shdtop_address_new(uint32_t networkIP, const gchar* name) {
    Address* a = (Address*)calloc(1, sizeof(Address));
    a->ip = networkIP;
    if (!inet_ntop(AF_INET, &a->ip, a->ipString, sizeof a->ipString)) strcpy(a->ipString, "NULL");
    a->name = strdup(name ? name : "host");
    size_t n = strlen(a->name) + strlen(a->ipString) + 32;
    a->idString = (char*)malloc(n);
    snprintf(a->idString, n, "%s-%s (eth,mac=0)", a->name, a->ipString);
    return a;
}

WEAK void shdtop_address_free(Address* a) {
    if (!a) return;
    free(a->name);
    free(a->idString);
    free(a);
}

WEAK uint32_t address_toNetworkIP(Address* a) { return a->ip; }
WEAK const gchar* address_toHostIPString(Address* a) { return a->ipString; }
WEAK const gchar* address_toString(Address* a) { return a->idString; }

/* shd-address.c:137-144 */
WEAK uint32_t address_stringToIP(const gchar* ipString) {
    struct in_addr inaddr;
    if (ipString && 1 == inet_pton(AF_INET, ipString, &inaddr)) return inaddr.s_addr;
    return INADDR_NONE;
}

WEAK Random* shdtop_random_new(unsigned int seed) {
    Random* r = (Random*)calloc(1, sizeof(Random));
    r->seedState = seed;
    r->initialSeed = seed;
    return r;
}
WEAK void shdtop_random_free(Random* r) { free(r); }

/* shd-random.c:30-41: rand_r() / RAND_MAX */
WEAK gdouble random_nextDouble(Random* r) {
    int v = rand_r(&r->seedState);
    return (gdouble)(((gdouble)v) / ((gdouble)RAND_MAX));
}

static double g_last_jump = 0.0;
static uint64_t g_jump_calls = 0;
/* the first kJumpHistory upcall values, in call order (standalone tests) */
#define kJumpHistory 4096
static double g_jump_hist[kJumpHistory];
static pthread_mutex_t g_jump_mu = PTHREAD_MUTEX_INITIALIZER;

/* shd-worker.c:384-387 -> shd-slave.c:365-372 (slave lock) -> shd-master.c:133-144 */
WEAK void worker_updateMinTimeJump(gdouble minPathLatency) {
    uint64_t bits;
    memcpy(&bits, &minPathLatency, sizeof bits);
    pthread_mutex_lock(&g_jump_mu);
    if (g_jump_calls < kJumpHistory) g_jump_hist[g_jump_calls] = minPathLatency;
    __atomic_store_n((uint64_t*)&g_last_jump, bits, __ATOMIC_SEQ_CST);
    __atomic_add_fetch(&g_jump_calls, 1, __ATOMIC_SEQ_CST);
    pthread_mutex_unlock(&g_jump_mu);
}

/* copies up to n recorded upcall values; returns how many were recorded in all */
WEAK uint64_t shdtop_min_time_jump_history(gdouble* out, uint64_t n) {
    pthread_mutex_lock(&g_jump_mu);
    uint64_t k = g_jump_calls;
    for (uint64_t i = 0; i < n && i < k && i < kJumpHistory; ++i) out[i] = g_jump_hist[i];
    pthread_mutex_unlock(&g_jump_mu);
    return k;
}

WEAK gdouble shdtop_last_min_time_jump(void) {
    uint64_t b = __atomic_load_n((uint64_t*)&g_last_jump, __ATOMIC_SEQ_CST);
    double d;
    memcpy(&d, &b, sizeof d);
    return d;
}
WEAK uint64_t shdtop_min_time_jump_calls(void) { return __atomic_load_n(&g_jump_calls, __ATOMIC_SEQ_CST); }
WEAK void shdtop_reset_min_time_jump(void) {
    pthread_mutex_lock(&g_jump_mu);
    g_last_jump = 0.0;
    __atomic_store_n(&g_jump_calls, 0, __ATOMIC_SEQ_CST);
    pthread_mutex_unlock(&g_jump_mu);
}
