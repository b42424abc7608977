// CPU model of one k_routes_sssp bucket's relaxation (experiments only, not the
// product): K lanes, near-far windows of width delta, round-synchronous
// expansion of near-pending vertices, two-pass drains -- the schedule of
// routes.hip phase 1 / phase 2 / drain. Counts the memory requests that set the
// kernel's time (head-row reads per arc visit, arc blocks, improvements, drain
// row reads, rounds) under several expansion policies, so policies can be
// compared without GPU time. Distances are checked against a plain Dijkstra.
//
// usage: sim_relax <input.bin> <policy> [hubdeg] [jacobi]   (jacobi 1: every expansion uses the
//   round-start value; 2: only hub expansions do, as a phase-1 snapshot would)
//   policy 0: baseline (every arc of a near vertex, every lane below thr)
//   policy 1: deferred suffix: at each expansion only the arcs that can still
//             produce a near mark (w < thr - min key of the active lanes; arcs
//             sorted by weight) are relaxed; the rest are relaxed once per
//             window, at its close, for the lanes whose key settled in it
//             (they can only produce far marks). Applied to vertices with
//             degree >= hubdeg (0 = all).
//   policy 2: fixed light/heavy split at delta (Meyer-Sanders) for deg >= hubdeg.
//   policy 3: policy 1 with per-lane predicates (the kernel design): only lanes
//             whose key lies in the current window [thr_lo, thr) are active; at an
//             expansion lane l relaxes the arcs with w < thr - key_l (head rows
//             read for w < thr - min key), at the window's close the arcs with
//             w >= thr - key_l; every expanded vertex is marked for the close;
//             arc blocks whose first weight >= delta are never read at an
//             expansion, and the close reads blocks from the first one holding
//             an arc some lane needs.
//   policy 4: relaxed-value memo for vertices of degree >= hubdeg: an expansion
//             relaxes only lanes whose value differs from the one they were last
//             relaxed with, and SPECULATIVELY also the lanes whose finite key is
//             still above the window (far), recording their values too; a hub
//             whose near lanes all match the memo is skipped (no rows read).
//   policy 5: policy 4 without the speculation (memo only).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define K 16

static int32_t V, NB;
static int64_t A;
static int64_t* rowptr;
static int32_t* col;
static double* w;
static uint8_t* pend;  // pendant: never pending
static double delta;
static int32_t* bsrc;  // [NB][K]

static double* dist;
static uint8_t *nflag, *fflag, *dflag;
static int32_t *nlist, *nnext, *flist, *dlist;
static int32_t nn, nnn, nf, nd;
static int policy, hubdeg, jacobi;
static double thr, thr_prev;
static double* memo;  // policy 4/5: [V][K] value each lane was last relaxed with
static double skipped, specimp;

static struct {
    double rounds, drains, expansions, arcvisits, blocks, improvements, drainrows, closerows, closearcs, closeexp;
    double hubexp, hubarcs;
} C;

static void mark_near(int32_t v) {
    if (pend[v]) return;
    if (!nflag[v]) { nflag[v] = 1; nnext[nnn++] = v; }
}
static void mark_far(int32_t v) {
    if (pend[v]) return;
    if (!fflag[v]) { fflag[v] = 1; flist[nf++] = v; }
}
static void mark_def(int32_t v) {
    if (!dflag[v]) { dflag[v] = 1; dlist[nd++] = v; }
}

static inline int is_hub(int32_t u) { return rowptr[u + 1] - rowptr[u] >= hubdeg; }

// relax arcs [a0, a1) of u for lanes in mask with lane-specific minimum weight wmin[l]
static void relax_range(int32_t u, int64_t a0, int64_t a1, const double* du, unsigned mask, const double* wmin) {
    for (int64_t a = a0; a < a1; ++a) {
        const int32_t v = col[a];
        const double wa = w[a];
        C.arcvisits += 1;
        double* dv = dist + (size_t)v * K;
        for (int l = 0; l < K; ++l) {
            if (!(mask >> l & 1u)) continue;
            if (wmin && wa < wmin[l]) continue;
            const double c = du[l] + wa;
            if (c < dv[l]) {
                dv[l] = c;
                C.improvements += 1;
                if (c < thr) mark_near(v); else mark_far(v);
            }
        }
    }
    C.blocks += (double)((a1 - a0 + 7) / 8);
}

static double* snap;  // jacobi snapshot of expanded rows (per round)
// SIM_ORDER: expansion order inside a round. 0 marking order; 1 breadth-first rank from
// the highest-degree vertex, ascending (the GPU's: relabel_bfs numbering, lists built by
// bitmap scans); 2 the same, descending (hubs last); 3 degree ascending
static int sim_order;
static int32_t* bfs_rank;
static int cmp_rank(const void* a, const void* b) {
    const int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    int64_t kx, ky;
    if (sim_order == 3) { kx = rowptr[x + 1] - rowptr[x]; ky = rowptr[y + 1] - rowptr[y]; }
    else { kx = bfs_rank[x]; ky = bfs_rank[y]; if (sim_order == 2) { kx = -kx; ky = -ky; } }
    return kx < ky ? -1 : kx > ky ? 1 : 0;
}

static void expand3(int32_t u, const double* du) {
    unsigned act = 0;
    double kmin = INFINITY, wlo[K], whi[K];
    for (int l = 0; l < K; ++l) {
        wlo[l] = 0.0; whi[l] = -INFINITY;
        if (du[l] >= thr_prev && du[l] < thr) { act |= 1u << l; whi[l] = thr - du[l]; if (du[l] < kmin) kmin = du[l]; }
    }
    const int64_t a0 = rowptr[u], a1 = rowptr[u + 1];
    if (a1 > a0) mark_def(u);
    // blocks whose first weight < delta are listed (read) at every expansion
    int64_t nb = 0;
    for (int64_t b = a0; b < a1; b += 8) if (w[b] < delta) ++nb;
    C.blocks += (double)nb;
    if (!act) return;
    C.expansions += 1;
    const double lim = thr - kmin;
    for (int64_t a = a0; a < a1 && w[a] < lim; ++a) {
        const int32_t v = col[a];
        const double wa = w[a];
        C.arcvisits += 1;
        double* dv = dist + (size_t)v * K;
        for (int l = 0; l < K; ++l) {
            if (!(act >> l & 1u) || !(wa < whi[l])) continue;
            const double c = du[l] + wa;
            if (c < dv[l]) {
                dv[l] = c;
                C.improvements += 1;
                if (c < thr) mark_near(v); else mark_far(v);
            }
        }
    }
    (void)wlo;
}

static void close3(void) {
    for (int32_t i = 0; i < nd; ++i) {
        const int32_t u = dlist[i];
        dflag[u] = 0;
        const double* du = dist + (size_t)u * K;
        C.closerows += 1;
        unsigned m = 0;
        double kmax = -INFINITY, wmin[K];
        for (int l = 0; l < K; ++l)
            if (du[l] >= thr_prev && du[l] < thr) { m |= 1u << l; wmin[l] = thr - du[l]; if (du[l] > kmax) kmax = du[l]; }
        if (!m) continue;
        const double lim = thr - kmax;  // rows needed for w >= lim
        int64_t a = rowptr[u];
        const int64_t a1 = rowptr[u + 1];
        while (a < a1 && w[a] < lim) ++a;
        if (a == a1) continue;
        C.closeexp += 1;
        const int64_t bfirst = rowptr[u] + (a - rowptr[u]) / 8 * 8;
        C.blocks += (double)((a1 - bfirst + 7) / 8);
        const double av0 = C.arcvisits;
        for (; a < a1; ++a) {
            const int32_t v = col[a];
            const double wa = w[a];
            C.arcvisits += 1;
            double* dv = dist + (size_t)v * K;
            for (int l = 0; l < K; ++l) {
                if (!(m >> l & 1u) || wa < wmin[l]) continue;
                const double c = du[l] + wa;
                if (c < dv[l]) {
                    dv[l] = c;
                    C.improvements += 1;
                    if (c < thr) { fprintf(stderr, "close near mark\n"); exit(3); }
                    mark_far(v);
                }
            }
        }
        C.closearcs += C.arcvisits - av0;
    }
    nd = 0;
}

static void expand4(int32_t u, const double* din) {
    double du[K];
    memcpy(du, din, sizeof du);
    const int hub = is_hub(u);
    double* mu = memo + (size_t)u * K;
    unsigned act = 0, spec = 0;
    for (int l = 0; l < K; ++l) {
        if (!(du[l] < INFINITY)) continue;
        if (hub && du[l] == mu[l]) continue;
        if (du[l] < thr) act |= 1u << l;
        else if (hub && policy == 4) spec |= 1u << l;
    }
    if (!act) { if (hub) skipped += 1; return; }
    C.expansions += 1;
    if (hub) {
        C.hubexp += 1;
        for (int l = 0; l < K; ++l) if ((act | spec) >> l & 1u) mu[l] = du[l];
    }
    const double av0 = C.arcvisits, im0 = C.improvements;
    relax_range(u, rowptr[u], rowptr[u + 1], du, act | spec, NULL);
    if (hub) C.hubarcs += C.arcvisits - av0;
    (void)im0;
}

static void expand(int32_t u, const double* din) {
    if (policy == 3) { expand3(u, din); return; }
    if (policy >= 4) { expand4(u, din); return; }
    double du[K];
    memcpy(du, din, sizeof du);
    unsigned act = 0;
    double kmin = INFINITY;
    for (int l = 0; l < K; ++l)
        if (du[l] < thr) { act |= 1u << l; if (du[l] < kmin) kmin = du[l]; }
    if (!act) return;
    C.expansions += 1;
    const int64_t a0 = rowptr[u], a1 = rowptr[u + 1];
    const int hub = is_hub(u);
    if (hub) C.hubexp += 1;
    const double av0 = C.arcvisits;
    if (policy == 1 && hub) {
        // arcs sorted by weight: prefix w < thr - kmin can produce near marks
        const double lim = thr - kmin;
        int64_t a = a0;
        while (a < a1 && w[a] < lim) ++a;
        relax_range(u, a0, a, du, act, NULL);
        if (a < a1) mark_def(u);
    } else if (policy == 2 && hub) {
        int64_t a = a0;
        while (a < a1 && w[a] < delta) ++a;
        relax_range(u, a0, a, du, act, NULL);
        if (a < a1) mark_def(u);
    } else {
        relax_range(u, a0, a1, du, act, NULL);
    }
    if (hub) C.hubarcs += C.arcvisits - av0;
}

// window close: deferred arcs for the lanes whose key settled in [thr_prev, thr)
static void close_window(void) {
    for (int32_t i = 0; i < nd; ++i) {
        const int32_t u = dlist[i];
        dflag[u] = 0;
        double du[K], wmin[K];
        memcpy(du, dist + (size_t)u * K, sizeof du);
        C.closerows += 1;
        unsigned m = 0;
        double lmin = INFINITY;
        for (int l = 0; l < K; ++l)
            if (du[l] >= thr_prev && du[l] < thr) {
                m |= 1u << l;
                wmin[l] = policy == 1 ? thr - du[l] : delta;
                if (wmin[l] < lmin) lmin = wmin[l];
            }
        if (!m) continue;
        int64_t a = rowptr[u];
        while (a < rowptr[u + 1] && w[a] < lmin) ++a;
        C.closeexp += 1;
        const double av0 = C.arcvisits;
        relax_range(u, a, rowptr[u + 1], du, m, wmin);
        C.closearcs += C.arcvisits - av0;
    }
    nd = 0;
}

static int drain(void) {
    C.drains += 1;
    const double thr_old = thr;
    thr = thr_old + delta;
    for (int pass = 0; pass < 2; ++pass) {
        int moved = 0, farf = 0;
        double minfar = INFINITY;
        const int32_t n = nf;
        nf = 0;
        static int32_t* tmp;
        if (!tmp) tmp = malloc(sizeof(int32_t) * (size_t)V);
        memcpy(tmp, flist, sizeof(int32_t) * (size_t)n);
        for (int32_t i = 0; i < n; ++i) fflag[tmp[i]] = 0;
        for (int32_t i = 0; i < n; ++i) {
            const int32_t v = tmp[i];
            C.drainrows += 1;
            const double* dv = dist + (size_t)v * K;
            int now = 0, keep = 0;
            for (int l = 0; l < K; ++l) {
                const double key = dv[l];
                if (key >= thr_old && key < thr) now = 1;
                if (key >= thr && key < INFINITY) { keep = 1; if (key < minfar) minfar = key; }
            }
            if (now) { mark_near(v); moved = 1; }
            if (keep) { mark_far(v); farf = 1; }
        }
        if (moved) return 1;
        if (!farf) return 0;
        thr = minfar + delta;
    }
    return 1;
}

static void run_bucket(const int32_t* src) {
    for (size_t i = 0; i < (size_t)V * K; ++i) dist[i] = INFINITY;
    if (memo) for (size_t i = 0; i < (size_t)V * K; ++i) memo[i] = NAN;
    nnn = nf = nd = 0;
    thr = delta;
    thr_prev = policy == 3 ? -INFINITY : 0.0;
    for (int l = 0; l < K; ++l) {
        const int32_t s = src[l];
        if (s < 0) continue;
        dist[(size_t)s * K + l] = 0.0;
        if (!pend[s]) mark_near(s);
        else {
            for (int64_t a = rowptr[s]; a < rowptr[s + 1]; ++a) {
                double* d = dist + (size_t)col[a] * K + l;
                if (w[a] < *d) { *d = w[a]; if (w[a] < thr) mark_near(col[a]); else mark_far(col[a]); }
            }
        }
    }
    for (;;) {
        // take the near set
        nn = nnn;
        int32_t* t = nlist; nlist = nnext; nnext = t;
        nnn = 0;
        for (int32_t i = 0; i < nn; ++i) nflag[nlist[i]] = 0;
        if (nn == 0) {
            if (policy == 3) close3();
            else if (policy) close_window();
            const double tp = thr;
            if (nnn > 0) {  // (close passes never mark near)
                fprintf(stderr, "close produced near marks\n");
                exit(2);
            }
            if (!drain()) break;
            thr_prev = tp;
            continue;
        }
        C.rounds += 1;
        if (sim_order) qsort(nlist, (size_t)nn, sizeof(int32_t), cmp_rank);
        if (jacobi) {
            for (int32_t i = 0; i < nn; ++i) memcpy(snap + (size_t)i * K, dist + (size_t)nlist[i] * K, K * 8);
        }
        for (int32_t i = 0; i < nn; ++i)
            expand(nlist[i], (jacobi == 1 || (jacobi == 2 && is_hub(nlist[i]))) ? snap + (size_t)i * K
                                                                                 : dist + (size_t)nlist[i] * K);
    }
}

// plain Dijkstra for checking one lane
static int check_lane(int32_t s, int l) {
    double* d = malloc(sizeof(double) * (size_t)V);
    int32_t* heap = malloc(sizeof(int32_t) * (size_t)(A + V + 1));
    double* hk = malloc(sizeof(double) * (size_t)(A + V + 1));
    int64_t hn = 0;
    for (int32_t v = 0; v < V; ++v) d[v] = INFINITY;
    d[s] = 0;
    heap[0] = s; hk[0] = 0; hn = 1;
    while (hn) {
        int32_t u = heap[0];
        double ku = hk[0];
        --hn;
        if (hn) {
            int32_t x = heap[hn]; double kx = hk[hn];
            int64_t i = 0;
            for (;;) {
                int64_t c = 2 * i + 1;
                if (c >= hn) break;
                if (c + 1 < hn && hk[c + 1] < hk[c]) ++c;
                if (hk[c] < kx) { heap[i] = heap[c]; hk[i] = hk[c]; i = c; } else break;
            }
            heap[i] = x; hk[i] = kx;
        }
        if (ku > d[u]) continue;
        for (int64_t a = rowptr[u]; a < rowptr[u + 1]; ++a) {
            const double c = ku + w[a];
            const int32_t v = col[a];
            if (c < d[v]) {
                d[v] = c;
                int64_t i = hn++;
                while (i > 0 && hk[(i - 1) / 2] > c) { heap[i] = heap[(i - 1) / 2]; hk[i] = hk[(i - 1) / 2]; i = (i - 1) / 2; }
                heap[i] = v; hk[i] = c;
            }
        }
    }
    int bad = 0;
    for (int32_t v = 0; v < V; ++v)
        if (d[v] != dist[(size_t)v * K + l]) { ++bad; }
    free(d); free(heap); free(hk);
    return bad;
}

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s in.bin policy [hubdeg] [jacobi] [check]\n", argv[0]); return 1; }
    policy = atoi(argv[2]);
    hubdeg = argc > 3 ? atoi(argv[3]) : 0;
    jacobi = argc > 4 ? atoi(argv[4]) : 0;
    const int check = argc > 5 ? atoi(argv[5]) : 0;
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror("open"); return 1; }
    if (fread(&V, 4, 1, f) != 1 || fread(&A, 8, 1, f) != 1 || fread(&delta, 8, 1, f) != 1 || fread(&NB, 4, 1, f) != 1) return 1;
    rowptr = malloc(8 * (size_t)(V + 1));
    col = malloc(4 * (size_t)A);
    w = malloc(8 * (size_t)A);
    pend = malloc((size_t)V);
    bsrc = malloc(4 * (size_t)NB * K);
    if (fread(rowptr, 8, (size_t)V + 1, f) != (size_t)V + 1 || fread(col, 4, (size_t)A, f) != (size_t)A ||
        fread(w, 8, (size_t)A, f) != (size_t)A || fread(pend, 1, (size_t)V, f) != (size_t)V ||
        fread(bsrc, 4, (size_t)NB * K, f) != (size_t)NB * K) { fprintf(stderr, "short read\n"); return 1; }
    fclose(f);
    { const char* d = getenv("SIM_DELTA"); if (d) delta = atof(d); }
    { const char* o = getenv("SIM_ORDER"); sim_order = o ? atoi(o) : 0; }
    if (sim_order == 1 || sim_order == 2) {  // breadth-first ranks from the highest-degree vertex
        bfs_rank = malloc(4 * (size_t)V);
        int32_t* q = malloc(4 * (size_t)V);
        for (int32_t v = 0; v < V; ++v) bfs_rank[v] = -1;
        int32_t hub = 0, qh = 0, qt = 0, next = 0;
        for (int32_t v = 1; v < V; ++v) if (rowptr[v + 1] - rowptr[v] > rowptr[hub + 1] - rowptr[hub]) hub = v;
        for (int32_t r = 0; r < V; ++r) {
            const int32_t root = r == 0 ? hub : r;
            if (bfs_rank[root] >= 0) continue;
            bfs_rank[root] = next++; q[qt++] = root;
            while (qh < qt) {
                const int32_t u = q[qh++];
                for (int64_t a = rowptr[u]; a < rowptr[u + 1]; ++a)
                    if (bfs_rank[col[a]] < 0) { bfs_rank[col[a]] = next++; q[qt++] = col[a]; }
            }
        }
        free(q);
    }
    dist = malloc(sizeof(double) * (size_t)V * K);
    snap = malloc(sizeof(double) * (size_t)V * K);
    if (policy >= 4) memo = malloc(sizeof(double) * (size_t)V * K);
    nflag = calloc((size_t)V, 1); fflag = calloc((size_t)V, 1); dflag = calloc((size_t)V, 1);
    nlist = malloc(4 * (size_t)V); nnext = malloc(4 * (size_t)V); flist = malloc(4 * (size_t)V); dlist = malloc(4 * (size_t)V);
    { const char* x = getenv("SIM_LANES");  /* keep only the first n lanes of each group */
      if (x) { const int nl = atoi(x); for (int32_t b = 0; b < NB; ++b) for (int l = nl; l < K; ++l) bsrc[(size_t)b * K + l] = -1; } }
    for (int32_t b = 0; b < NB; ++b) {
        run_bucket(bsrc + (size_t)b * K);
        if (check && b == 0) {
            int bad = 0;
            for (int l = 0; l < K; l += 5) bad += check_lane(bsrc[l], l);
            printf("check bucket 0: %d wrong distances\n", bad);
        }
    }
    const double n = NB;
    printf("policy %d hubdeg %d jacobi %d delta %.2f buckets %d order %d\n", policy, hubdeg, jacobi, delta, NB, sim_order);
    printf("  rounds %.1f drains %.1f expansions/V %.3f arcvisits/A %.3f blocks %.0f improvements %.0f drainrows %.0f\n",
           C.rounds / n, C.drains / n, C.expansions / n / V, C.arcvisits / n / (double)A, C.blocks / n,
           C.improvements / n, C.drainrows / n);
    printf("  close: rows %.0f expansions %.0f arcs %.0f | hub expansions %.0f hub arc visits %.0f\n", C.closerows / n,
           C.closeexp / n, C.closearcs / n, C.hubexp / n, C.hubarcs / n);
    if (policy >= 4) printf("  memo: skipped hub expansions %.0f per bucket\n", skipped / n);
    // request model: one line per arc visit (head row) + one per 8-arc block + drain/close rows
    const double req = C.arcvisits + C.blocks + C.drainrows + C.closerows;
    printf("  line requests per bucket %.0f (arc rows %.0f blocks %.0f drain %.0f close %.0f) atomics %.0f\n", req / n,
           C.arcvisits / n, C.blocks / n, C.drainrows / n, C.closerows / n, C.improvements / n);
    return 0;
}
