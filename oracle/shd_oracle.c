/*
 * shd_oracle.c — CPU restatement of Shadow's topology-routing path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (shadow_amd/) links, loads or
 * calls this file.  It is used by tests/ (as the parity checker),
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, nowhere else.
 *
 * It restates, in plain C99 with its own data structures (no code shared with
 * the product), the behaviour of /root/reference at v0:
 *
 *   orc_is_complete        src/main/routing/shd-topology.c:129-230 (_topology_isComplete)
 *   orc_get_eid            igraph_get_eid as called at shd-topology.c:189,643-645
 *   orc_lookup_path        shd-topology.c:941-979 (_topology_lookupPath, complete branch)
 *   orc_dijkstra           igraph_get_shortest_paths_dijkstra as called at shd-topology.c:868
 *                          (igraph >= 0.7: dist init -1, binary 2-way heap of -dist,
 *                          strict '<' improvement, parent edge recorded, early exit once
 *                          every distinct target is popped, mode OUT)
 *   orc_epilogue           shd-topology.c:663-773 (_topology_computeSourcePathsHelper)
 *                          incl. _topology_getEdgeHelper :636-661
 *   orc_routes             shd-topology.c:775-939 (_topology_computeSourcePaths) for many
 *                          sources: Dijkstra, then the epilogue for every target, in
 *                          target order, plus the running row minimum of :602-606
 *   orc_window_ns          shd-master.c:118-144 (minimum time jump -> round window)
 *
 * igraph is a third-party library absent from /root/reference and from this
 * image (version unpinned: cmake/FindIGRAPH.cmake:12-49). Its Dijkstra is
 * restated from its published algorithm; its heap order among EQUAL-distance
 * tight predecessors is NOT pinned by any reference test, so the canonical rule
 * (orc_canonical_pred: smallest-distance tight predecessor as igraph's strict
 * '<' gives, then minimum index; bitwise tightness) stands in for it there.
 * Pinning: tests/test_oracle.py checks this file against the reference's own
 * test-config topologies (known answers), the bundled topologies (direct-edge
 * tables generated independently in numpy), and networkx/scipy shortest paths.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct orc_graph {
    int32_t V;
    int64_t E;
    int directed;
    int32_t *efrom, *eto;
    double *elat, *eloss, *vloss;
    /* incidence lists for mode OUT (undirected: every incident edge; a self-loop
     * appears twice, as igraph_incident does) sorted by (neighbour, edge id) */
    int64_t* iptr;
    int64_t* iedge;
    /* sorted (key, edge) index for get_eid */
    uint64_t* ekey;
    int64_t* eidx;
} orc_graph;

static uint64_t pair_key(const orc_graph* g, int32_t u, int32_t v) {
    if (!g->directed && u > v) { int32_t t = u; u = v; v = t; }
    return ((uint64_t)(uint32_t)u << 32) | (uint32_t)v;
}

static const orc_graph* g_sort_graph; /* qsort context */
static int32_t g_sort_vertex;

static int32_t other_end(const orc_graph* g, int64_t e, int32_t v) { return g->efrom[e] == v ? g->eto[e] : g->efrom[e]; }

static int cmp_inc(const void* a, const void* b) {
    int64_t ea = *(const int64_t*)a, eb = *(const int64_t*)b;
    int32_t na = other_end(g_sort_graph, ea, g_sort_vertex), nb = other_end(g_sort_graph, eb, g_sort_vertex);
    if (na != nb) return na < nb ? -1 : 1;
    return ea < eb ? -1 : (ea > eb ? 1 : 0);
}

typedef struct { uint64_t k; int64_t e; } KE;
static int cmp_ke(const void* a, const void* b) {
    const KE* x = (const KE*)a;
    const KE* y = (const KE*)b;
    if (x->k != y->k) return x->k < y->k ? -1 : 1;
    return x->e < y->e ? -1 : (x->e > y->e ? 1 : 0);
}

void orc_graph_free(orc_graph* g) {
    if (!g) return;
    free(g->efrom); free(g->eto); free(g->elat); free(g->eloss); free(g->vloss);
    free(g->iptr); free(g->iedge); free(g->ekey); free(g->eidx);
    free(g);
}

orc_graph* orc_graph_new(int32_t V, int64_t E, int directed, const int32_t* efrom, const int32_t* eto,
                         const double* elat, const double* eloss, const double* vloss) {
    orc_graph* g = (orc_graph*)calloc(1, sizeof(orc_graph));
    if (!g) return NULL;
    g->V = V; g->E = E; g->directed = directed ? 1 : 0;
    g->efrom = (int32_t*)malloc(sizeof(int32_t) * (size_t)(E + 1));
    g->eto = (int32_t*)malloc(sizeof(int32_t) * (size_t)(E + 1));
    g->elat = (double*)malloc(sizeof(double) * (size_t)(E + 1));
    g->eloss = (double*)malloc(sizeof(double) * (size_t)(E + 1));
    g->vloss = (double*)malloc(sizeof(double) * (size_t)(V + 1));
    for (int64_t e = 0; e < E; ++e) {
        if (efrom[e] < 0 || efrom[e] >= V || eto[e] < 0 || eto[e] >= V) { orc_graph_free(g); return NULL; }
        g->efrom[e] = efrom[e]; g->eto[e] = eto[e]; g->elat[e] = elat[e]; g->eloss[e] = eloss ? eloss[e] : 0.0;
    }
    for (int32_t v = 0; v < V; ++v) g->vloss[v] = vloss ? vloss[v] : 0.0;
    /* incidence lists */
    g->iptr = (int64_t*)calloc((size_t)V + 1, sizeof(int64_t));
    for (int64_t e = 0; e < E; ++e) {
        g->iptr[g->efrom[e] + 1]++;
        if (!g->directed) g->iptr[g->eto[e] + 1]++;
    }
    for (int32_t v = 0; v < V; ++v) g->iptr[v + 1] += g->iptr[v];
    g->iedge = (int64_t*)malloc(sizeof(int64_t) * (size_t)(g->iptr[V] + 1));
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(V + 1));
    memcpy(fill, g->iptr, sizeof(int64_t) * (size_t)V);
    for (int64_t e = 0; e < E; ++e) {
        g->iedge[fill[g->efrom[e]]++] = e;
        if (!g->directed) g->iedge[fill[g->eto[e]]++] = e;
    }
    free(fill);
    g_sort_graph = g;
    for (int32_t v = 0; v < V; ++v) {
        g_sort_vertex = v;
        qsort(g->iedge + g->iptr[v], (size_t)(g->iptr[v + 1] - g->iptr[v]), sizeof(int64_t), cmp_inc);
    }
    /* get_eid index */
    KE* ke = (KE*)malloc(sizeof(KE) * (size_t)(E + 1));
    for (int64_t e = 0; e < E; ++e) { ke[e].k = pair_key(g, g->efrom[e], g->eto[e]); ke[e].e = e; }
    qsort(ke, (size_t)E, sizeof(KE), cmp_ke);
    g->ekey = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(E + 1));
    g->eidx = (int64_t*)malloc(sizeof(int64_t) * (size_t)(E + 1));
    for (int64_t e = 0; e < E; ++e) { g->ekey[e] = ke[e].k; g->eidx[e] = ke[e].e; }
    free(ke);
    return g;
}

/* igraph_get_eid(graph, &eid, from, to, directed=TRUE, error=TRUE): the edge
 * joining from->to (either orientation when undirected). With parallel edges
 * igraph's choice is unpinned; the lowest edge id is used. */
int64_t orc_get_eid(const orc_graph* g, int32_t u, int32_t v) {
    if (u < 0 || v < 0 || u >= g->V || v >= g->V) return -1;
    uint64_t k = pair_key(g, u, v);
    int64_t lo = 0, hi = g->E;
    while (lo < hi) {
        int64_t mid = lo + (hi - lo) / 2;
        if (g->ekey[mid] < k) lo = mid + 1; else hi = mid;
    }
    if (lo < g->E && g->ekey[lo] == k) return g->eidx[lo];
    return -1;
}

/* _topology_isComplete (:129-230) */
int orc_is_complete(const orc_graph* g) {
    for (int32_t v = 0; v < g->V; ++v) {
        int64_t ecount = g->iptr[v + 1] - g->iptr[v];
        if (!g->directed && orc_get_eid(g, v, v) >= 0) ecount -= 1; /* :187-199 */
        if (ecount < g->V) return 0;                               /* :201 */
    }
    return 1;
}

/* _topology_getEdgeHelper (:636-661) */
static int edge_helper(const orc_graph* g, int32_t from, int32_t to, double* lat, double* rel) {
    int64_t e = orc_get_eid(g, from, to);
    if (e < 0) return -1;
    if (lat) *lat = g->elat[e];
    if (rel) *rel = 1.0f - g->eloss[e]; /* float literal promoted: 1.0 - p in double */
    return 0;
}

/* _topology_lookupPath (:941-979). Returns 0 on success. */
int orc_lookup_path(const orc_graph* g, int32_t s, int32_t t, double* lat, double* rel) {
    double totalLatency = 0.0, totalReliability = 1.0;
    double edgeLatency = 0.0, edgeReliability = 1.0;
    totalReliability *= (1.0f - g->vloss[s]);
    totalReliability *= (1.0f - g->vloss[t]);
    if (edge_helper(g, s, t, &edgeLatency, &edgeReliability)) return -1;
    totalLatency += edgeLatency;
    totalReliability *= edgeReliability;
    *lat = totalLatency;
    *rel = totalReliability;
    return 0;
}

/* _topology_computeSourcePathsHelper (:663-773): path = igraph vertex list,
 * path[0] == s when nv > 1, path[nv-1] = destination. Returns 0 on success. */
int orc_epilogue(const orc_graph* g, int32_t s, const int32_t* path, int32_t nv, double* lat, double* rel) {
    double totalLatency = 0.0;
    double totalReliability = 1.0;
    int32_t d;
    totalReliability *= (1.0f - g->vloss[s]); /* :694 */
    if (nv == 0) {                             /* :698-702 */
        totalLatency = 1.0;
        d = s;
    } else {
        d = path[nv - 1];
        if ((s != d) || (s == d && nv > 2)) totalReliability *= (1.0f - g->vloss[d]); /* :709-711 */
        int32_t start = nv == 1 ? 0 : 1;
        int32_t from = s;
        for (int32_t i = start; i < nv; ++i) {
            int32_t to = path[i];
            double el = 0, er = 0;
            if (edge_helper(g, from, to, &el, &er)) return -1; /* :733-739 */
            totalLatency += el;                                /* :742 */
            totalReliability *= er;                            /* :743 */
            from = to;
        }
    }
    (void)d;
    if (totalLatency == 0.0) totalLatency = 1.0; /* :760-765 */
    *lat = totalLatency;
    *rel = totalReliability;
    return 0;
}

/* ---- igraph_2wheap restatement: max-heap on -dist with a position index ---- */
typedef struct {
    double* val;
    int32_t* id;
    int32_t* pos; /* vertex -> heap slot + 1 (0: not in heap) */
    int32_t n;
} Heap;

static void hswap(Heap* h, int32_t a, int32_t b) {
    double tv = h->val[a]; h->val[a] = h->val[b]; h->val[b] = tv;
    int32_t ti = h->id[a]; h->id[a] = h->id[b]; h->id[b] = ti;
    h->pos[h->id[a]] = a + 1;
    h->pos[h->id[b]] = b + 1;
}
static void hshift_up(Heap* h, int32_t e) {
    while (e > 0) {
        int32_t p = (e + 1) / 2 - 1;
        if (h->val[e] < h->val[p]) break; /* igraph_i_2wheap_shift_up: swaps on >= */
        hswap(h, e, p);
        e = p;
    }
}
static void hsink(Heap* h, int32_t e) {
    for (;;) {
        int32_t l = 2 * e + 1, r = 2 * e + 2;
        if (l >= h->n) break;
        int32_t c = (r >= h->n || h->val[l] >= h->val[r]) ? l : r;
        if (h->val[e] < h->val[c]) { hswap(h, e, c); e = c; } else break;
    }
}
static void hpush(Heap* h, int32_t v, double x) {
    h->val[h->n] = x; h->id[h->n] = v; h->pos[v] = h->n + 1; h->n++;
    hshift_up(h, h->n - 1);
}
static int32_t hpop(Heap* h, double* x) {
    int32_t v = h->id[0];
    *x = h->val[0];
    hswap(h, 0, h->n - 1);
    h->n--;
    h->pos[v] = 0;
    hsink(h, 0);
    return v;
}
static void hmodify(Heap* h, int32_t v, double x) {
    int32_t p = h->pos[v] - 1;
    h->val[p] = x;
    hsink(h, p);
    hshift_up(h, p);
}

/* Dijkstra as igraph >= 0.7 runs it (call :868). dist[v] = -1 where unreached
 * when the search stopped; parent_edge[v] = edge id or -1. */
int orc_dijkstra(const orc_graph* g, int32_t s, const int32_t* targets, int32_t nT, double* dist,
                 int64_t* parent_edge) {
    const int32_t V = g->V;
    Heap h;
    h.val = (double*)malloc(sizeof(double) * (size_t)(V + 1));
    h.id = (int32_t*)malloc(sizeof(int32_t) * (size_t)(V + 1));
    h.pos = (int32_t*)calloc((size_t)V + 1, sizeof(int32_t));
    h.n = 0;
    uint8_t* is_target = (uint8_t*)calloc((size_t)V + 1, 1);
    int32_t to_reach = 0;
    for (int32_t i = 0; i < nT; ++i)
        if (!is_target[targets[i]]) { is_target[targets[i]] = 1; to_reach++; }
    for (int32_t v = 0; v < V; ++v) { dist[v] = -1.0; parent_edge[v] = -1; }
    dist[s] = 0.0;
    hpush(&h, s, -0.0);
    while (h.n > 0 && to_reach > 0) {
        double negd;
        int32_t u = hpop(&h, &negd);
        double mindist = -negd;
        if (is_target[u]) { is_target[u] = 0; to_reach--; }
        for (int64_t p = g->iptr[u]; p < g->iptr[u + 1]; ++p) {
            int64_t e = g->iedge[p];
            int32_t to = other_end(g, e, u);
            double alt = mindist + g->elat[e];
            double cur = dist[to];
            if (cur < 0) {
                dist[to] = alt; parent_edge[to] = e; hpush(&h, to, -alt);
            } else if (alt < cur) {
                dist[to] = alt; parent_edge[to] = e; hmodify(&h, to, -alt);
            }
        }
    }
    free(h.val); free(h.id); free(h.pos); free(is_target);
    return 0;
}

/* Full (no early exit) distances, for the canonical predecessor rule. */
int orc_dijkstra_all(const orc_graph* g, int32_t s, double* dist, int64_t* parent_edge) {
    int32_t* all = (int32_t*)malloc(sizeof(int32_t) * (size_t)(g->V + 1));
    for (int32_t v = 0; v < g->V; ++v) all[v] = v;
    int rc = orc_dijkstra(g, s, all, g->V, dist, parent_edge);
    free(all);
    return rc;
}

/* Canonical predecessor among the u with an edge u->v such that
 * fl(dist[u] + latency) == dist[v] bitwise ("tight"): the smallest dist[u],
 * then the minimum index u. igraph's strict-'<' Dijkstra keeps the first tight
 * relaxation in heap pop order, i.e. the tight u with the smallest distance
 * (orc_dijkstra: 'alt < cur'); only equal-distance ties depend on its heap
 * order, and those take the minimum index here. ntight[v] = number of
 * distinct tight u (1 along a whole chain = unique shortest path). */
int orc_canonical_pred(const orc_graph* g, const double* dist, int32_t s, int32_t* pred, int32_t* ntight) {
    for (int32_t v = 0; v < g->V; ++v) { pred[v] = -1; if (ntight) ntight[v] = 0; }
    if (!g->directed) {
        /* incidence lists are sorted by neighbour id: parallel edges are adjacent */
        for (int32_t v = 0; v < g->V; ++v) {
            if (v == s || dist[v] < 0) continue;
            int32_t lastu = -1;
            for (int64_t p = g->iptr[v]; p < g->iptr[v + 1]; ++p) {
                int64_t e = g->iedge[p];
                int32_t u = other_end(g, e, v);
                if (u == v || u == lastu || dist[u] < 0) continue;
                if (!(dist[u] + g->elat[e] == dist[v])) continue;
                lastu = u;
                if (ntight) ntight[v]++;
                if (pred[v] < 0 || dist[u] < dist[pred[v]] || (dist[u] == dist[pred[v]] && u < pred[v])) pred[v] = u;
            }
        }
    } else {
        /* edges in (from,to) key order: parallel edges of one pair are adjacent */
        int32_t lastu = -1, lastv = -1;
        for (int64_t k = 0; k < g->E; ++k) {
            int64_t e = g->eidx[k];
            int32_t u = g->efrom[e], v = g->eto[e];
            if (u == v || v == s || dist[u] < 0 || dist[v] < 0) continue;
            if (!(dist[u] + g->elat[e] == dist[v])) continue;
            if (u == lastu && v == lastv) continue;
            lastu = u; lastv = v;
            if (ntight) ntight[v]++;
            if (pred[v] < 0 || dist[u] < dist[pred[v]] || (dist[u] == dist[pred[v]] && u < pred[v])) pred[v] = u;
        }
    }
    return 0;
}

/* igraph's vertex list [s, ..., t] from parent edges; returns nv (0 if t
 * unreached). buf must hold V entries. */
static int32_t path_from_parents(const orc_graph* g, int32_t s, int32_t t, const int64_t* parent_edge,
                                 const double* dist, int32_t* buf) {
    if (dist[t] < 0) return 0;
    int32_t n = 0, v = t;
    while (parent_edge[v] >= 0) { ++n; v = other_end(g, parent_edge[v], v); }
    if (v != s) return 0;
    int32_t nv = n + 1;
    buf[n] = t;
    v = t;
    int32_t k = n;
    while (parent_edge[v] >= 0) { v = other_end(g, parent_edge[v], v); buf[--k] = v; }
    return nv;
}

static int32_t path_from_pred(int32_t s, int32_t t, const int32_t* pred, const double* dist, int32_t V,
                              int32_t* buf) {
    if (dist[t] < 0) return 0;
    int32_t n = 0, v = t;
    while (v != s) { if (pred[v] < 0 || n > V) return 0; ++n; v = pred[v]; }
    buf[n] = t;
    v = t;
    int32_t k = n;
    while (v != s) { v = pred[v]; buf[--k] = v; }
    return n + 1;
}

typedef struct {
    const orc_graph* g;
    const int32_t *src, *dst;
    int32_t S, T, mode;
    double *lat, *rel, *row_min;
    int32_t* hops;
    int32_t next;
    pthread_mutex_t mu;
    int rc;
} RoutesJob;

static void routes_row(RoutesJob* J, int32_t i, double* dist, int64_t* pe, int32_t* pred, int32_t* buf) {
    const orc_graph* g = J->g;
    const int32_t s = J->src[i];
    double rowmin = INFINITY;
    int complete = J->mode == 2;
    if (!complete) {
        if (J->mode == 1) {
            orc_dijkstra_all(g, s, dist, pe);
            orc_canonical_pred(g, dist, s, pred, NULL);
        } else {
            orc_dijkstra(g, s, J->dst, J->T, dist, pe);
        }
    }
    for (int32_t j = 0; j < J->T; ++j) {
        const int32_t t = J->dst[j];
        double l = NAN, r = NAN;
        int32_t h = -1;
        if (complete) {
            if (orc_lookup_path(g, s, t, &l, &r) == 0) h = 1; else { l = NAN; r = NAN; }
        } else {
            int32_t nv = J->mode == 1 ? path_from_pred(s, t, pred, dist, g->V, buf)
                                      : path_from_parents(g, s, t, pe, dist, buf);
            if (nv > 0 && orc_epilogue(g, s, buf, nv, &l, &r) == 0) h = nv == 1 ? 1 : nv - 1;
            else { l = NAN; r = NAN; }
        }
        size_t o = (size_t)i * (size_t)J->T + (size_t)j;
        J->lat[o] = l;
        J->rel[o] = r;
        if (J->hops) J->hops[o] = h;
        if (l < rowmin) rowmin = l;
    }
    if (J->row_min) J->row_min[i] = rowmin;
}

static void* routes_worker(void* arg) {
    RoutesJob* J = (RoutesJob*)arg;
    const int32_t V = J->g->V;
    double* dist = (double*)malloc(sizeof(double) * (size_t)(V + 1));
    int64_t* pe = (int64_t*)malloc(sizeof(int64_t) * (size_t)(V + 1));
    int32_t* pred = (int32_t*)malloc(sizeof(int32_t) * (size_t)(V + 1));
    int32_t* buf = (int32_t*)malloc(sizeof(int32_t) * (size_t)(V + 2));
    for (;;) {
        pthread_mutex_lock(&J->mu);
        int32_t i = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (i >= J->S) break;
        routes_row(J, i, dist, pe, pred, buf);
    }
    free(dist); free(pe); free(pred); free(buf);
    return NULL;
}

/* S x T route table as the reference's path cache would hold it after every
 * source row was computed. mode 0: shortest-path branch with igraph-like
 * parents; mode 1: shortest-path branch with canonical predecessors; mode 2:
 * complete branch (direct edge). threads >= 1 (1 = reference-faithful: the
 * reference serialises Dijkstra under graphLock, :859-893). */
int orc_routes(const orc_graph* g, const int32_t* src, int32_t S, const int32_t* dst, int32_t T, int mode,
               double* lat, double* rel, int32_t* hops, double* row_min, int threads) {
    RoutesJob J;
    J.g = g; J.src = src; J.dst = dst; J.S = S; J.T = T; J.mode = mode;
    J.lat = lat; J.rel = rel; J.hops = hops; J.row_min = row_min; J.next = 0; J.rc = 0;
    pthread_mutex_init(&J.mu, NULL);
    if (threads <= 1) {
        routes_worker(&J);
    } else {
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
        for (int k = 0; k < threads; ++k) pthread_create(&th[k], NULL, routes_worker, &J);
        for (int k = 0; k < threads; ++k) pthread_join(th[k], NULL);
        free(th);
    }
    pthread_mutex_destroy(&J.mu);
    return J.rc;
}

/* shd-master.c:133-144 then :118-131: the upcall truncates ms to an integer
 * before scaling to ns; the window is 10 ms when that is 0, floored by the
 * --runahead configuration. */
uint64_t orc_window_ns(double min_path_latency_ms, uint64_t runahead_ns) {
    const uint64_t one_ms = 1000000ull;
    uint64_t next = ((uint64_t)min_path_latency_ms) * one_ms;
    uint64_t w = next > 0 ? next : 10ull * one_ms;
    if (runahead_ns > 0 && w < runahead_ns) w = runahead_ns;
    return w;
}

/* packet delay in ns, shd-worker.c:247 */
uint64_t orc_delay_ns(double latency_ms) { return (uint64_t)ceil(latency_ms * 1000000.0); }
