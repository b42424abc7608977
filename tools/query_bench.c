/*
 * Per-packet consumer of the drop-in: worker_sendPacket
 * (/root/reference/src/main/core/shd-worker.c:216-271) asks
 * topology_getReliability then topology_getLatency for every packet and turns
 * the latency into a delay of ceil(lat * 1e6) ns (:247). This times that pair of
 * calls from P threads after the first query has computed the table on the GPU.
 *
 * usage: query_bench <graphml> <hosts> <queries per thread> <threads>
 * build: gcc -O2 -pthread tools/query_bench.c -Iinclude -Lshadow_amd -lshdtopology \
 *            -Wl,-rpath,$PWD/shadow_amd -lm -o tools/query_bench
 */
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "shd_topology.h"

static Topology* g_top;
static Address** g_addr;
static int g_hosts;
static long g_q;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void* worker(void* arg) {
    unsigned seed = (unsigned)(size_t)arg;
    unsigned long long acc = 0;
    for (long i = 0; i < g_q; ++i) {
        Address* s = g_addr[rand_r(&seed) % g_hosts];
        Address* d = g_addr[rand_r(&seed) % g_hosts];
        double rel = topology_getReliability(g_top, s, d);
        double lat = topology_getLatency(g_top, s, d);
        if (rel >= 0) acc += (unsigned long long)ceil(lat * 1000000.0); /* SIMTIME_ONE_MILLISECOND */
    }
    return (void*)(size_t)acc;
}

int main(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "usage: %s graphml hosts queries threads\n", argv[0]); return 2; }
    g_hosts = atoi(argv[2]);
    g_q = atol(argv[3]);
    int P = atoi(argv[4]);
    g_top = topology_new(argv[1]);
    if (!g_top) return 1;
    g_addr = calloc(g_hosts, sizeof *g_addr);
    for (int i = 0; i < g_hosts; ++i) {
        char name[32];
        snprintf(name, sizeof name, "h%d", i);
        const unsigned a = 11u << 24 | (unsigned)(i + 1);  /* 11.0.0.0 + i + 1, as Shadow's DNS assigns */
        const uint32_t ip = (uint32_t)((a >> 24) | ((a >> 8) & 0xff00) | ((a << 8) & 0xff0000) | (a << 24));
        g_addr[i] = shdtop_address_new(ip, name);
        Random* r = shdtop_random_new((unsigned)i + 1);
        topology_attach(g_top, g_addr[i], r, NULL, NULL, NULL, NULL, NULL);
        shdtop_random_free(r);
    }
    double t0 = now();
    double first = topology_getLatency(g_top, g_addr[0], g_addr[g_hosts - 1]);  /* computes the table */
    double t1 = now();
    pthread_t th[256];
    for (int p = 0; p < P; ++p) pthread_create(&th[p], NULL, worker, (void*)(size_t)(p + 1));
    unsigned long long sum = 0;
    for (int p = 0; p < P; ++p) { void* r; pthread_join(th[p], &r); sum += (unsigned long long)(size_t)r; }
    double t2 = now();
    printf("{\"hosts\": %d, \"threads\": %d, \"table_ms\": %.1f, \"first_latency\": %.17g, "
           "\"packets_per_s\": %.4g, \"delay_checksum\": %llu}\n",
           g_hosts, P, (t1 - t0) * 1e3, first, (double)g_q * P / (t2 - t1), sum);
    topology_free(g_top);
    return 0;
}
