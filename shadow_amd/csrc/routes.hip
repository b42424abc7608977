// MI355X (gfx950) routing engine: the device half of the shdr_* C-ABI.
//
// Replaces, for /root/reference/src/main/routing/shd-topology.c:
//   _topology_computeSourcePaths       :775-939  (igraph Dijkstra call :868)
//   _topology_computeSourcePathsHelper :663-773  (ordered latency/reliability epilogue)
//   _topology_lookupPath               :941-979  (complete-graph direct edge)
//   min tracking of _storePathInCache  :602-613
//
// Design:
//   * CSR graph resident in HBM; dist / predecessor state laid out [V][K]: the K
//     sources of one "bucket" sit in K adjacent lanes, so one arc read serves K
//     sources and a vertex's distances are one contiguous K*8-byte row.
//   * A wave64 is 64/K sub-groups of K lanes; each sub-group works one vertex
//     (phase 1) or one arc chunk (phase 2) at a time.
//   * k_routes_sssp is persistent: one 256-thread workgroup owns one bucket at a
//     time and runs, with only workgroup barriers:
//       near-far (delta-stepping) frontier relaxation over frontier bitmaps,
//       -> canonical predecessor pass (minimum-index tight in-arc, bitwise test),
//       -> fused latency+reliability epilogue walking each (source,target) chain
//          and folding the factors in path order, as the reference does,
//       -> per-source row minimum (scheduler window input).
//   * k_routes_direct is the complete-graph branch: a dense gather.
// No MFMA: this is irregular f64 compare/add work, bound by memory.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "graph.hpp"

namespace shdr {
HostGraph* host_of(shdr_graph* g);
const HostGraph* host_of(const shdr_graph* g);
}  // namespace shdr

#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t _e = (x);                                                           \
        if (_e != hipSuccess) {                                                        \
            shdr::set_error(std::string("HIP: ") + #x + ": " + hipGetErrorString(_e)); \
            return SHDR_EHIP;                                                          \
        }                                                                              \
    } while (0)

namespace {

constexpr int kThreads = 256;   // workgroup size of the persistent SSSP kernel
constexpr int kWaves = kThreads / 64;
constexpr int kChunk = 32;      // arcs per phase-2 work item (splits hub vertices)
constexpr int kStack = 32;      // per-lane LDS stack depth of the epilogue walk
constexpr uint64_t kInfBits = 0x7FF0000000000000ull;

__device__ __forceinline__ uint64_t ld_u64_sc1(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_u32_sc1(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// LDS hand-off between lanes of one wave: order the ds_write before the ds_read.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ double as_f64(uint64_t b) { return __builtin_bit_cast(double, b); }
__device__ __forceinline__ uint64_t as_u64(double d) { return __builtin_bit_cast(uint64_t, d); }

struct DevGraph {
    int32_t V;
    int32_t A;
    const int32_t* rowptr;  // [V+1] out-CSR
    const int32_t* col;     // [A]
    const double* w;        // [A]
    const double* oclat;    // [A] canonical-edge latency of out-arc
    const double* ocrel;    // [A] canonical-edge reliability factor of out-arc
    const int32_t* irowptr; // in-CSR (aliases out-CSR when undirected)
    const int32_t* isrc;    // [A] source vertex of in-arc
    const double* iw;
    const double* iclat;
    const double* icrel;
    const double* vrel;     // [V]
    const double* self_lat; // [V]
    const double* self_rel; // [V]
};

// Per-slot scratch of the persistent kernel (one slot per resident workgroup).
struct SlotWs {
    uint64_t* dist;    // [V*K] f64 bits
    int2* pred;        // [V*K] {pred vertex, in-arc index}
    uint32_t* pend;    // [V] pending-lane mask (K <= 32)
    uint32_t* amask;   // [V] active-lane mask of the current round
    uint64_t* bits;    // [3 * Vw] bitmaps: frontier a, frontier b, far
    int2* items;       // [cap] {vertex, chunk}
};

struct SlotArena {
    char* base;
    size_t stride;
    int64_t item_cap;
    int* err;  // set non-zero by a workgroup that hit a guard (host reports it)
    size_t off_pred, off_pend, off_amask, off_bits, off_items;
    __device__ SlotWs at(int slot) const {
        char* b = base + size_t(slot) * stride;
        SlotWs s;
        s.dist = reinterpret_cast<uint64_t*>(b);
        s.pred = reinterpret_cast<int2*>(b + off_pred);
        s.pend = reinterpret_cast<uint32_t*>(b + off_pend);
        s.amask = reinterpret_cast<uint32_t*>(b + off_amask);
        s.bits = reinterpret_cast<uint64_t*>(b + off_bits);
        s.items = reinterpret_cast<int2*>(b + off_items);
        return s;
    }
};

struct RouteOut {
    double* lat;      // [S*T]
    double* rel;      // [S*T]
    int32_t* hops;    // [S*T] or null
    double* row_min;  // [S] or null
    int32_t T;
};

// ------------------------------------------------------------------ complete branch
// _topology_lookupPath (:941-979): lat = 0.0 + l(s,t); rel = ((1*(1-p_s))*(1-p_t))*(1-pl(s,t)).
// The edge is the canonical (get_eid) one; s==t uses the self-loop. No zero override.
__global__ void __launch_bounds__(256) k_routes_direct(DevGraph g, const int32_t* __restrict__ src,
                                                       const int32_t* __restrict__ dst, int32_t S,
                                                       RouteOut out) {
    const int32_t T = out.T;
    for (int32_t i = blockIdx.y; i < S; i += gridDim.y) {
    const int32_t s = src[i];
    const double rs = g.vrel[s];
    const int32_t a0 = g.rowptr[s], a1 = g.rowptr[s + 1];
    double rmin = __builtin_inf();
    for (int32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < T; j += gridDim.x * blockDim.x) {
        const int32_t t = dst[j];
        double el, er;
        if (s == t) {
            el = g.self_lat[s];
            er = g.self_rel[s];
        } else {
            int32_t lo = a0, hi = a1;  // first arc with col >= t
            while (lo < hi) {
                int32_t mid = (lo + hi) >> 1;
                if (g.col[mid] < t) lo = mid + 1; else hi = mid;
            }
            if (lo < a1 && g.col[lo] == t) { el = g.oclat[lo]; er = g.ocrel[lo]; }
            else { el = __builtin_nan(""); er = __builtin_nan(""); }
        }
        double lat = 0.0, rel = 1.0;
        rel *= rs;
        rel *= g.vrel[t];
        lat += el;
        rel *= er;
        const size_t o = size_t(i) * T + j;
        out.lat[o] = lat;
        out.rel[o] = rel;
        if (out.hops) out.hops[o] = (lat == lat) ? 1 : -1;
        if (lat < rmin) rmin = lat;
    }
    if (out.row_min) {
        // block min, then one CAS-min per block (latencies may be any sign here)
        __shared__ double red[4];
        for (int o = 32; o > 0; o >>= 1) rmin = fmin(rmin, __shfl_xor(rmin, o));
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = rmin;
        __syncthreads();
        if (threadIdx.x == 0) {
            double m = red[0];
            for (int k = 1; k < (int)(blockDim.x >> 6); ++k) m = fmin(m, red[k]);
            unsigned long long* p = reinterpret_cast<unsigned long long*>(out.row_min + i);
            unsigned long long cur = *p;
            while (m < as_f64(cur)) {
                unsigned long long prev = atomicCAS(p, cur, as_u64(m));
                if (prev == cur) break;
                cur = prev;
            }
        }
        __syncthreads();
    }
    }
}

__global__ void k_fill_f64(double* p, size_t n, double v) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) p[i] = v;
}

// ------------------------------------------------------------------ shortest-path branch
template <int K>
struct Lanes {
    static constexpr int G = 64 / K;  // sub-groups per wave
    static constexpr uint32_t kFull = (K == 32) ? 0xFFFFFFFFu : ((1u << K) - 1u);
};

// One workgroup, one bucket of K sources, from empty state to finished rows.
template <int K>
__global__ void __launch_bounds__(kThreads) k_routes_sssp(DevGraph g, SlotArena arena,
                                                          const int32_t* __restrict__ src, int32_t S,
                                                          const int32_t* __restrict__ dst, int32_t nbuckets,
                                                          double delta, RouteOut out, int keep_slots) {
    using L = Lanes<K>;
    constexpr int G = L::G;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int sub = lane / K;    // sub-group within the wave
    const int l = lane % K;      // source lane within the bucket
    const int gsub = wave * G + sub;  // sub-group id within the workgroup
    constexpr int NSUB = kWaves * G;
    const int32_t V = g.V;
    const int32_t Vw = (V + 63) >> 6;

    __shared__ int32_t s_nitems;
    __shared__ int32_t s_far_flag;
    __shared__ unsigned long long s_minfar;
    __shared__ int32_t s_wbuf[kWaves][64];
    __shared__ int32_t s_stack[kStack][kThreads];
    __shared__ double s_rowmin[kWaves][64];

    const int slot = blockIdx.x;
    SlotWs ws = arena.at(slot);
    uint64_t* bitsA = ws.bits;
    uint64_t* bitsB = ws.bits + Vw;
    uint64_t* far = ws.bits + 2 * size_t(Vw);

    for (int32_t b = blockIdx.x; b < nbuckets; b += gridDim.x) {
        const int32_t i0 = b * K;
        const int32_t nsrc = min(K, S - i0);
        // this lane's source vertex (sub-group replicas agree)
        const int32_t my_src = (l < nsrc) ? src[i0 + l] : -1;

        // ---- init: dist = +inf, pend = 0, bitmaps = 0
        {
            const size_t n = size_t(V) * K;
            for (size_t k = tid; k < n; k += kThreads) ws.dist[k] = kInfBits;
            for (int32_t v = tid; v < V; v += kThreads) ws.pend[v] = 0u;
            for (int32_t k = tid; k < 3 * Vw; k += kThreads) ws.bits[k] = 0ull;
        }
        __syncthreads();
        if (tid < nsrc) {
            const int32_t s = src[i0 + tid];
            ws.dist[size_t(s) * K + tid] = as_u64(0.0);
            atomicOr(&ws.pend[s], 1u << tid);
            atomicOr(reinterpret_cast<unsigned long long*>(&bitsA[s >> 6]), 1ull << (s & 63));
        }
        if (tid == 0) s_far_flag = 0;
        __syncthreads();

        uint64_t* cur = bitsA;
        uint64_t* nxt = bitsB;
        double thr = delta;
        bool rescan = false;  // a drained near set was just refilled from far
        // guard: every round settles or defers at least one lane; bound the loop
        const int64_t max_rounds = int64_t(V + 16) * (K + 2) + 4096;
        int64_t rounds = 0;

        for (;;) {
            if (++rounds > max_rounds) {
                if (tid == 0) atomicOr(arena.err, 1);
                break;
            }
            // ================= phase 1: scan frontier, snapshot active lanes, emit items
            if (tid == 0) { s_nitems = 0; s_minfar = kInfBits; }
            __syncthreads();
            for (int32_t base = wave * 64; base < Vw; base += kThreads) {
                const int32_t wi = base + lane;
                uint64_t word = 0;
                if (wi < Vw) {
                    word = ld_u64_sc1(&cur[wi]);
                    if (word) cur[wi] = 0ull;
                }
                while (__any(word != 0)) {
                    int32_t v = -1;
                    if (word) {
                        v = wi * 64 + __builtin_ctzll(word);
                        word &= word - 1;
                    }
                    const unsigned long long bal = __ballot(v >= 0);
                    const int cnt = __popcll(bal);
                    if (v >= 0) {
                        const int pos = __popcll(bal & ((1ull << lane) - 1ull));
                        s_wbuf[wave][pos] = v;
                    }
                    wave_sync();
                    for (int r = 0; r < cnt; r += G) {
                        const int idx = r + sub;
                        const int32_t u = (idx < cnt) ? s_wbuf[wave][idx] : -1;
                        bool act = false, pendl = false;
                        double du = 0.0;
                        uint32_t p = 0;
                        if (u >= 0) {
                            p = ld_u32_sc1(&ws.pend[u]);
                            pendl = (p >> l) & 1u;
                            if (pendl) {
                                du = as_f64(ld_u64_sc1(&ws.dist[size_t(u) * K + l]));
                                act = du < thr;
                            }
                        }
                        const unsigned long long ba = __ballot(act);
                        const unsigned long long bf = __ballot(pendl && !act);
                        const uint32_t m_act = uint32_t(ba >> (sub * K)) & L::kFull;
                        const uint32_t m_far = uint32_t(bf >> (sub * K)) & L::kFull;
                        if (pendl && !act) atomicMin(&s_minfar, as_u64(du));
                        int32_t ibase = 0, nch = 0;
                        if (u >= 0 && l == 0) {
                            if (m_act) {
                                ws.pend[u] = p & ~m_act;
                                ws.amask[u] = m_act;
                                const int32_t deg = g.rowptr[u + 1] - g.rowptr[u];
                                nch = (deg + kChunk - 1) / kChunk;
                                if (nch > 0) ibase = atomicAdd(&s_nitems, nch);
                                if (int64_t(ibase) + nch > arena.item_cap) { atomicOr(arena.err, 2); nch = 0; }
                            }
                            if (m_far) {
                                atomicOr(reinterpret_cast<unsigned long long*>(&far[u >> 6]), 1ull << (u & 63));
                                s_far_flag = 1;
                            }
                        }
                        ibase = __shfl(ibase, sub * K);
                        nch = __shfl(nch, sub * K);
                        for (int32_t c = l; c < nch; c += K) ws.items[ibase + c] = make_int2(u, c);
                    }
                    wave_sync();
                }
            }
            __syncthreads();
            const int32_t nitems = s_nitems;
            if (nitems == 0) {
                if (!s_far_flag) break;  // nothing pending anywhere: bucket done
                __syncthreads();
                // near set drained: refill from far and raise the threshold
                if (rescan) {
                    // the previous pass scanned every pending vertex: jump straight past the min
                    thr = as_f64(s_minfar) + delta;
                } else {
                    thr += delta;
                }
                rescan = true;
                uint64_t* t = cur; cur = far; far = t;  // cur was zeroed during the scan
                __syncthreads();
                if (tid == 0) s_far_flag = 0;
                __syncthreads();
                continue;
            }
            rescan = false;

            // ================= phase 2: relax the arcs of every item
            for (int32_t it = gsub; it < nitems; it += NSUB) {
                const int2 item = ws.items[it];
                const int32_t u = item.x;
                const int32_t a0 = g.rowptr[u] + item.y * kChunk;
                const int32_t a1 = min(g.rowptr[u + 1], a0 + kChunk);
                const uint32_t am = ws.amask[u];
                const bool act = (am >> l) & 1u;
                const double du = as_f64(ld_u64_sc1(&ws.dist[size_t(u) * K + l]));
                for (int32_t a = a0; a < a1; a += 2) {
                    const bool has2 = (a + 1) < a1;
                    const int32_t v0 = g.col[a];
                    const double w0 = g.w[a];
                    const int32_t v1 = has2 ? g.col[a + 1] : v0;
                    const double w1 = has2 ? g.w[a + 1] : w0;
                    uint64_t* p0 = &ws.dist[size_t(v0) * K + l];
                    uint64_t* p1 = &ws.dist[size_t(v1) * K + l];
                    const double o0 = as_f64(*p0);
                    const double o1 = as_f64(*p1);
                    const double c0 = du + w0;
                    const double c1 = du + w1;
                    bool imp0 = false, imp1 = false;
                    if (act && c0 < o0) {
                        const uint64_t prev = atomicMin(reinterpret_cast<unsigned long long*>(p0), as_u64(c0));
                        imp0 = c0 < as_f64(prev);
                    }
                    if (act && has2 && c1 < o1) {
                        const uint64_t prev = atomicMin(reinterpret_cast<unsigned long long*>(p1), as_u64(c1));
                        imp1 = c1 < as_f64(prev);
                    }
                    const uint32_t m0 = uint32_t(__ballot(imp0) >> (sub * K)) & L::kFull;
                    const uint32_t m1 = uint32_t(__ballot(imp1) >> (sub * K)) & L::kFull;
                    if (l == 0 && m0) {
                        atomicOr(&ws.pend[v0], m0);
                        atomicOr(reinterpret_cast<unsigned long long*>(&nxt[v0 >> 6]), 1ull << (v0 & 63));
                    }
                    if (l == 0 && m1) {
                        atomicOr(&ws.pend[v1], m1);
                        atomicOr(reinterpret_cast<unsigned long long*>(&nxt[v1 >> 6]), 1ull << (v1 & 63));
                    }
                }
            }
            __syncthreads();
            uint64_t* t = cur; cur = nxt; nxt = t;  // old cur already zeroed in phase 1
        }
        __syncthreads();

        // ================= predecessor pass: minimum-index tight in-arc, bitwise test
        for (int32_t v = gsub; v < V; v += NSUB) {
            const double dv = as_f64(ld_u64_sc1(&ws.dist[size_t(v) * K + l]));
            int2 pr = make_int2(-1, -1);
            bool need = (dv != __builtin_inf()) && (v != my_src);
            const int32_t p0 = g.irowptr[v], p1 = g.irowptr[v + 1];
            for (int32_t p = p0; p < p1; ++p) {
                if (!__any(need)) break;
                if (need) {
                    const int32_t u = g.isrc[p];
                    const double du = as_f64(ld_u64_sc1(&ws.dist[size_t(u) * K + l]));
                    if (du + g.iw[p] == dv) { pr = make_int2(u, p); need = false; }
                }
            }
            ws.pred[size_t(v) * K + l] = pr;
        }
        __syncthreads();

        // ================= epilogue: ordered walk per (source lane, target)
        const double rs = (my_src >= 0) ? g.vrel[my_src] : 0.0;
        double rowmin = __builtin_inf();
        for (int32_t j = gsub; j < out.T; j += NSUB) {
            const int32_t t = dst[j];
            double lat = __builtin_nan(""), rel = __builtin_nan("");
            int32_t hops = -1;
            if (my_src >= 0) {
                if (t == my_src) {
                    // igraph returns the one-vertex path [s]: the self-loop edge, no dst loss (:709-711)
                    const double sl = g.self_lat[t];
                    if (sl == sl) {
                        lat = 0.0; lat += sl;
                        rel = 1.0; rel *= rs; rel *= g.self_rel[t];
                        hops = 1;
                        if (lat == 0.0) lat = 1.0;
                    }
                } else {
                    const double dt = as_f64(ld_u64_sc1(&ws.dist[size_t(t) * K + l]));
                    if (dt != __builtin_inf()) {
                        // walk back, recording the first kStack in-arcs; count all hops
                        int32_t h = 0, v = t;
                        while (v != my_src) {
                            const int2 pr = ws.pred[size_t(v) * K + l];
                            if (h < kStack) s_stack[h][tid] = pr.y;
                            ++h;
                            v = pr.x;
                            if (v < 0 || h > V) { h = -1; if (v >= 0) atomicOr(arena.err, 4); break; }
                        }
                        if (h > 0) {
                            lat = 0.0;
                            rel = 1.0;
                            rel *= rs;
                            rel *= g.vrel[t];
                            // fold in path order (source side first), kStack hops at a time
                            for (int32_t hi = h; hi > 0; hi -= kStack) {
                                const int32_t lo = max(0, hi - kStack);  // hops [lo, hi) counted from t
                                if (h > kStack) {
                                    int32_t vv = t;
                                    for (int32_t k = 0; k < hi; ++k) {
                                        const int2 pr = ws.pred[size_t(vv) * K + l];
                                        if (k >= lo) s_stack[k - lo][tid] = pr.y;
                                        vv = pr.x;
                                    }
                                    for (int32_t k = hi - lo - 1; k >= 0; --k) {
                                        const int32_t p = s_stack[k][tid];
                                        lat += g.iclat[p];
                                        rel *= g.icrel[p];
                                    }
                                } else {
                                    for (int32_t k = h - 1; k >= 0; --k) {
                                        const int32_t p = s_stack[k][tid];
                                        lat += g.iclat[p];
                                        rel *= g.icrel[p];
                                    }
                                }
                            }
                            if (lat == 0.0) lat = 1.0;  // :760-765
                            hops = h;
                        }
                    }
                }
                const size_t o = size_t(i0 + l) * out.T + j;
                out.lat[o] = lat;
                out.rel[o] = rel;
                if (out.hops) out.hops[o] = hops;
                if (lat < rowmin) rowmin = lat;
            }
        }
        // row minimum per source lane across all sub-groups
        if (out.row_min) {
            s_rowmin[wave][lane] = rowmin;
            __syncthreads();
            if (tid < K) {
                double m = __builtin_inf();
                for (int w2 = 0; w2 < kWaves; ++w2)
                    for (int s2 = 0; s2 < G; ++s2) m = fmin(m, s_rowmin[w2][s2 * K + tid]);
                if (tid < nsrc) out.row_min[i0 + tid] = m;
            }
        }
        __syncthreads();
        if (keep_slots) break;
    }
}

}  // namespace

// ==================================================================== engine
struct shdr_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    shdr::CsrImage csr;
    bool complete = false;
    bool directed = false;
    double delta = 0.0;  // 0 = auto
    // graph buffers
    int32_t *rowptr = nullptr, *col = nullptr, *irowptr = nullptr, *isrc = nullptr;
    double *w = nullptr, *oclat = nullptr, *ocrel = nullptr, *iw = nullptr, *iclat = nullptr, *icrel = nullptr;
    double *vrel = nullptr, *self_lat = nullptr, *self_rel = nullptr;
    // workspace
    char* arena = nullptr;
    size_t arena_bytes = 0;
    int32_t* d_src = nullptr;
    int32_t* d_dst = nullptr;
    size_t cap_src = 0, cap_dst = 0;
    double *d_lat = nullptr, *d_rel = nullptr, *d_rowmin = nullptr;
    int* d_err = nullptr;
    int32_t* d_hops = nullptr;
    size_t cap_out = 0;
    // kept trees
    int kept_K = 0;
    int32_t kept_S = 0;
    size_t kept_stride = 0, kept_off_pred = 0;
    bool kept = false;
    // timing
    hipEvent_t ev[8] = {};
    std::vector<std::string> tnames;
    std::vector<float> tms;
    std::vector<void*> owned;
};

namespace {

template <typename T>
int upload(shdr_engine* e, T** dptr, const std::vector<T>& h) {
    size_t n = std::max<size_t>(h.size(), 1);
    HIPCHK(hipMalloc((void**)dptr, n * sizeof(T)));
    e->owned.push_back(*dptr);
    if (!h.empty()) HIPCHK(hipMemcpy(*dptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return SHDR_OK;
}

int ensure(void** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes && *p) return SHDR_OK;
    if (*p) HIPCHK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIPCHK(hipMalloc(p, std::max<size_t>(bytes, 16)));
    *cap = bytes;
    return SHDR_OK;
}

DevGraph devgraph(const shdr_engine* e) {
    DevGraph g;
    g.V = e->csr.V;
    g.A = int32_t(e->csr.A);
    g.rowptr = e->rowptr; g.col = e->col; g.w = e->w; g.oclat = e->oclat; g.ocrel = e->ocrel;
    if (e->csr.same_in_out) {
        g.irowptr = e->rowptr; g.isrc = e->col; g.iw = e->w; g.iclat = e->oclat; g.icrel = e->ocrel;
    } else {
        g.irowptr = e->irowptr; g.isrc = e->isrc; g.iw = e->iw; g.iclat = e->iclat; g.icrel = e->icrel;
    }
    g.vrel = e->vrel; g.self_lat = e->self_lat; g.self_rel = e->self_rel;
    return g;
}

constexpr int kBucketK = 16;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct ArenaLayout {
    size_t stride, off_pred, off_pend, off_amask, off_bits, off_items;
};

ArenaLayout layout_for(int32_t V, int64_t A, int K) {
    ArenaLayout L;
    size_t o = 0;
    o += align_up(size_t(V) * K * 8, 256);
    L.off_pred = o; o += align_up(size_t(V) * K * 8, 256);
    L.off_pend = o; o += align_up(size_t(V) * 4, 256);
    L.off_amask = o; o += align_up(size_t(V) * 4, 256);
    const size_t Vw = (size_t(V) + 63) / 64;
    L.off_bits = o; o += align_up(3 * Vw * 8, 256);
    L.off_items = o; o += align_up((size_t(V) + size_t(A) / kChunk + 64) * 8, 256);
    L.stride = o;
    return L;
}

int record(shdr_engine* e, int k, bool on) {
    if (on) HIPCHK(hipEventRecord(e->ev[k], e->stream));
    return SHDR_OK;
}

}  // namespace

extern "C" {

int32_t shdr_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

shdr_engine* shdr_engine_create(const shdr_graph* gh, int32_t device) {
    const shdr::HostGraph* hg = shdr::host_of(gh);
    if (!hg) { shdr::set_error("engine_create: NULL graph"); return nullptr; }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        shdr::set_error("engine_create: no HIP device visible (the routing engine has no CPU fallback)");
        return nullptr;
    }
    if (device < 0 || device >= n) { shdr::set_error("engine_create: bad device index"); return nullptr; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { shdr::set_error("engine_create: hipGetDeviceProperties failed"); return nullptr; }
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0) {
        shdr::set_error(std::string("engine_create: device is ") + prop.gcnArchName + ", this build targets gfx950 only");
        return nullptr;
    }
    auto* e = new shdr_engine();
    e->device = device;
    shdr::HostGraph* mg = const_cast<shdr::HostGraph*>(hg);
    if (!mg->checked) mg->check();
    shdr::build_csr(*mg, e->csr);
    if (e->csr.A >= (int64_t(1) << 31)) { shdr::set_error("engine_create: >2^31 arcs"); delete e; return nullptr; }
    e->complete = mg->info.is_complete != 0;
    e->directed = mg->directed;
    auto fail = [&](const char* what) -> shdr_engine* {
        char buf[512];
        shdr_last_error(buf, sizeof buf);
        shdr::set_error(std::string("engine_create: ") + what + ": " + buf);
        shdr_engine_free(e);
        return nullptr;
    };
    if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice");
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    for (auto& ev : e->ev)
        if (hipEventCreate(&ev) != hipSuccess) return fail("event");
    const shdr::CsrImage& c = e->csr;
    std::vector<int32_t> rp32(c.rowptr.begin(), c.rowptr.end());
    if (upload(e, &e->rowptr, rp32) || upload(e, &e->col, c.col) || upload(e, &e->w, c.w) ||
        upload(e, &e->oclat, c.oclat) || upload(e, &e->ocrel, c.ocrel) || upload(e, &e->vrel, c.vrel) ||
        upload(e, &e->self_lat, c.self_lat) || upload(e, &e->self_rel, c.self_rel))
        return fail("upload");
    if (!c.same_in_out) {
        std::vector<int32_t> irp32(c.irowptr.begin(), c.irowptr.end());
        if (upload(e, &e->irowptr, irp32) || upload(e, &e->isrc, c.isrc) || upload(e, &e->iw, c.iw) ||
            upload(e, &e->iclat, c.iclat) || upload(e, &e->icrel, c.icrel))
            return fail("upload in-CSR");
    }
    return e;
}

void shdr_engine_free(shdr_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    for (void* p : e->owned) (void)hipFree(p);
    if (e->arena) (void)(void)hipFree(e->arena);
    if (e->d_src) (void)hipFree(e->d_src);
    if (e->d_dst) (void)hipFree(e->d_dst);
    if (e->d_lat) (void)hipFree(e->d_lat);
    if (e->d_rel) (void)hipFree(e->d_rel);
    if (e->d_rowmin) (void)hipFree(e->d_rowmin);
    if (e->d_hops) (void)hipFree(e->d_hops);
    if (e->d_err) (void)hipFree(e->d_err);
    for (auto& ev : e->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

int shdr_engine_set_delta(shdr_engine* e, double delta) {
    if (!e || !(delta >= 0.0)) { shdr::set_error("set_delta: bad argument"); return SHDR_EINVAL; }
    e->delta = delta;
    return SHDR_OK;
}

int shdr_routes_compute(shdr_engine* e, const int32_t* src, int32_t S, const int32_t* dst, int32_t T,
                        double* lat, double* rel, int32_t* hops, double* row_min, uint32_t flags,
                        void* stream_v) {
    if (!e || S < 0 || T < 0 || (S > 0 && !src) || (T > 0 && !dst) || ((S > 0 && T > 0) && (!lat || !rel))) {
        shdr::set_error("routes_compute: bad arguments");
        return SHDR_EINVAL;
    }
    HIPCHK(hipSetDevice(e->device));
    hipStream_t st = stream_v ? (hipStream_t)stream_v : e->stream;
    const bool dev_out = flags & SHDR_OUT_DEVICE;
    const bool timing = flags & SHDR_TIMING;
    const bool keep = flags & SHDR_KEEP_TREES;
    const int32_t V = e->csr.V;
    for (int32_t i = 0; i < S; ++i)
        if (src[i] < 0 || src[i] >= V) { shdr::set_error("routes_compute: source vertex out of range"); return SHDR_EINVAL; }
    for (int32_t j = 0; j < T; ++j)
        if (dst[j] < 0 || dst[j] >= V) { shdr::set_error("routes_compute: target vertex out of range"); return SHDR_EINVAL; }
    e->tnames.clear();
    e->tms.clear();
    e->kept = false;
    if (S == 0 || T == 0) return SHDR_OK;
    int rc;
    if ((rc = ensure((void**)&e->d_src, &e->cap_src, size_t(S) * 4))) return rc;
    if ((rc = ensure((void**)&e->d_dst, &e->cap_dst, size_t(T) * 4))) return rc;
    HIPCHK(hipMemcpyAsync(e->d_src, src, size_t(S) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->d_dst, dst, size_t(T) * 4, hipMemcpyHostToDevice, st));
    RouteOut o;
    o.T = T;
    const size_t npair = size_t(S) * T;
    if (dev_out) {
        o.lat = lat; o.rel = rel; o.hops = hops; o.row_min = row_min;
    } else {
        size_t cap = e->cap_out;
        if (cap < npair || !e->d_lat) {
            if (e->d_lat) { (void)hipFree(e->d_lat); (void)hipFree(e->d_rel); if (e->d_hops) (void)hipFree(e->d_hops); }
            e->d_lat = e->d_rel = nullptr; e->d_hops = nullptr;
            HIPCHK(hipMalloc((void**)&e->d_lat, npair * 8));
            HIPCHK(hipMalloc((void**)&e->d_rel, npair * 8));
            HIPCHK(hipMalloc((void**)&e->d_hops, npair * 4));
            e->cap_out = npair;
        }
        if (e->d_rowmin) (void)hipFree(e->d_rowmin);
        HIPCHK(hipMalloc((void**)&e->d_rowmin, size_t(S) * 8));
        o.lat = e->d_lat; o.rel = e->d_rel; o.hops = hops ? e->d_hops : nullptr; o.row_min = e->d_rowmin;
    }
    DevGraph g = devgraph(e);
    const bool use_direct = e->complete && !(flags & SHDR_FORCE_SSSP);
    if (use_direct) {
        if (o.row_min) {
            hipLaunchKernelGGL(k_fill_f64, dim3(std::max(1, std::min(1024, (S + 255) / 256))), dim3(256), 0, st,
                               o.row_min, size_t(S), __builtin_inf());
        }
        dim3 grid(std::max(1, std::min((T + 255) / 256, 64)), std::min(S, 65535));
        if ((rc = record(e, 0, timing))) return rc;
        hipLaunchKernelGGL(k_routes_direct, grid, dim3(256), 0, st, g, e->d_src, e->d_dst, S, o);
        HIPCHK(hipGetLastError());
        if ((rc = record(e, 1, timing))) return rc;
    } else {
        constexpr int K = kBucketK;
        const int32_t nb = (S + K - 1) / K;
        ArenaLayout Lh = layout_for(V, e->csr.A, K);
        int dev_cus = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, e->device) == hipSuccess) dev_cus = prop.multiProcessorCount;
        int32_t slots = keep ? nb : std::min<int32_t>(nb, dev_cus * 4);
        // bound the arena to ~40% of free HBM
        size_t freeb = 0, totalb = 0;
        HIPCHK(hipMemGetInfo(&freeb, &totalb));
        const size_t have = e->arena_bytes;
        const size_t budget = (freeb + have) * 2 / 5;
        if (size_t(slots) * Lh.stride > budget) {
            if (keep) { shdr::set_error("routes_compute: KEEP_TREES needs more HBM than available"); return SHDR_ENOMEM; }
            slots = std::max<int32_t>(1, int32_t(budget / Lh.stride));
        }
        const size_t need = size_t(slots) * Lh.stride;
        if (e->arena_bytes < need) {
            if (e->arena) HIPCHK(hipFree(e->arena));
            e->arena = nullptr;
            e->arena_bytes = 0;
            HIPCHK(hipMalloc((void**)&e->arena, need));
            e->arena_bytes = need;
        }
        if (!e->d_err) HIPCHK(hipMalloc((void**)&e->d_err, sizeof(int)));
        HIPCHK(hipMemsetAsync(e->d_err, 0, sizeof(int), st));
        SlotArena ar;
        ar.base = e->arena;
        ar.stride = Lh.stride;
        ar.item_cap = int64_t(V) + e->csr.A / kChunk + 64;
        ar.err = e->d_err;
        ar.off_pred = Lh.off_pred; ar.off_pend = Lh.off_pend; ar.off_amask = Lh.off_amask;
        ar.off_bits = Lh.off_bits; ar.off_items = Lh.off_items;
        double delta = e->delta > 0.0 ? e->delta : std::max(1e-9, 0.5 * e->csr.mean_w);
        if ((rc = record(e, 0, timing))) return rc;
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_routes_sssp<K>), dim3(slots), dim3(kThreads), 0, st, g, ar, e->d_src, S,
                           e->d_dst, nb, delta, o, keep ? 1 : 0);
        HIPCHK(hipGetLastError());
        if ((rc = record(e, 1, timing))) return rc;
        if (keep) {
            e->kept = true;
            e->kept_K = K;
            e->kept_S = S;
            e->kept_stride = Lh.stride;
            e->kept_off_pred = Lh.off_pred;
        }
    }
    if (!dev_out) {
        HIPCHK(hipMemcpyAsync(lat, o.lat, npair * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(rel, o.rel, npair * 8, hipMemcpyDeviceToHost, st));
        if (hops) HIPCHK(hipMemcpyAsync(hops, o.hops, npair * 4, hipMemcpyDeviceToHost, st));
        if (row_min) HIPCHK(hipMemcpyAsync(row_min, o.row_min, size_t(S) * 8, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    if (!use_direct) {
        int herr = 0;
        HIPCHK(hipMemcpy(&herr, e->d_err, sizeof(int), hipMemcpyDeviceToHost));
        if (herr) {
            shdr::set_error("routes_compute: device guard tripped (code " + std::to_string(herr) +
                            ": 1=round limit, 2=work-list overflow, 4=broken predecessor chain)");
            return SHDR_EHIP;
        }
    }
    if (timing) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
        e->tnames.push_back(use_direct ? "k_routes_direct" : "k_routes_sssp");
        e->tms.push_back(ms);
    }
    return SHDR_OK;
}

int shdr_engine_pred_tree(shdr_engine* e, int32_t i, int32_t* pred_vertex, double* dist) {
    if (!e || !e->kept || i < 0 || i >= e->kept_S) { shdr::set_error("pred_tree: no kept tree for that row (use SHDR_KEEP_TREES)"); return SHDR_EINVAL; }
    HIPCHK(hipSetDevice(e->device));
    const int K = e->kept_K;
    const int32_t V = e->csr.V;
    const int32_t b = i / K, l = i % K;
    char* base = e->arena + size_t(b) * e->kept_stride;
    std::vector<uint64_t> drow(size_t(V) * K);
    std::vector<int2> prow(size_t(V) * K);
    if (dist) HIPCHK(hipMemcpy(drow.data(), base, drow.size() * 8, hipMemcpyDeviceToHost));
    if (pred_vertex) HIPCHK(hipMemcpy(prow.data(), base + e->kept_off_pred, prow.size() * 8, hipMemcpyDeviceToHost));
    for (int32_t v = 0; v < V; ++v) {
        if (dist) memcpy(&dist[v], &drow[size_t(v) * K + l], 8);
        if (pred_vertex) pred_vertex[v] = prow[size_t(v) * K + l].x;
    }
    return SHDR_OK;
}

int shdr_engine_timing(shdr_engine* e, int32_t* n, const char** names, float* ms, int32_t cap) {
    if (!e || !n) { shdr::set_error("timing: bad arguments"); return SHDR_EINVAL; }
    int32_t k = int32_t(e->tms.size());
    *n = k;
    for (int32_t i = 0; i < k && i < cap; ++i) {
        if (names) names[i] = e->tnames[i].c_str();
        if (ms) ms[i] = e->tms[i];
    }
    return SHDR_OK;
}

}  // extern "C"
