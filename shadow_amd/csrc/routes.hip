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
#include <array>
#include <initializer_list>
#include <thread>
#include <type_traits>
#include <utility>
#include <unistd.h>
#include <sys/mman.h>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
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

// ---- diagnostic build (make diag: -DSHDR_DIAG): per-phase wall ticks and work
// counters summed over workgroups. Never compiled into the product library.
#ifdef SHDR_DIAG
__device__ unsigned long long g_diag[32];
__device__ unsigned long long g_bticks[2][8192];  // per main-launch bucket: start, duration
#define DIAG_ADD(i, v) atomicAdd(&g_diag[i], (unsigned long long)(v))
#define DIAG_NOW() __builtin_amdgcn_s_memrealtime()
#define DIAG_LOCAL(...) __VA_ARGS__
#define DIAG_SKIP(x) (x)
#else
#ifdef SHDR_SKIP_ONLY  // phase-skip experiments without the counters' overhead
#define DIAG_SKIP(x) (x)
#else
#define DIAG_SKIP(x) false
#endif
#define DIAG_ADD(i, v) do { } while (0)
#define DIAG_NOW() 0ull
#define DIAG_LOCAL(...)
#endif

namespace {

constexpr int kChunk = 8;       // arcs per phase-2 work item (hub vertices span many items)
// A vertex's last arc block with at most kHalf real arcs (a "half block": arcs 0-3,
// the rest padding) is relaxed as one half of a PAIR item: two half blocks of two
// pending vertices share one item's 8 head-row loads. bfirst[v]
// carries the flag in bit 31.
constexpr int kHalf = kChunk / 2;
constexpr uint32_t kHalfBit = 0x80000000u;
// Experiment knobs (hub lag, far-mark rule variants, landmark count, window rule,
// partition regions, arena alignment) are compiled only into the experiments
// flavour (make -C shadow_amd flavor NAME=exp DEFS=-DSHDR_EXPERIMENTS); the product
// library runs the measured defaults with no such branches.
#ifdef SHDR_EXPERIMENTS
constexpr bool kExperiments = true;
#else
constexpr bool kExperiments = false;
#endif
// per-lane LDS stack depth (hop factors) of the epilogue walk; 512-thread
// workgroups take 12 so that two of them (pending bitmaps included) share a CU
constexpr int stack_depth(int NT) { return NT == 512 ? 12 : 14; }
// minimum waves per SIMD the compiler must allow (caps VGPRs at 512 / this):
// 512-thread workgroups are built for two per CU (4 waves per SIMD, 128 VGPRs)
// threads per workgroup of the default variants (K = 16 main, K = 8 tail, K = 32):
// 1024 = 16 waves per CU, 128 VGPRs per lane; 768 = 12 waves, 168 VGPRs
#ifndef SHDR_MAIN_NT
#define SHDR_MAIN_NT 1024
#endif
constexpr int kNT = SHDR_MAIN_NT;
constexpr int min_waves_per_eu(int NT) { return NT == 512 ? 4 : (NT >= 1024 ? 1 : 1024 / NT); }
constexpr int kFlushCap = 256;  // per-wave LDS staging slots for relaxation updates
#ifndef SHDR_FLUSH_AT
#define SHDR_FLUSH_AT 64
#endif
constexpr int kFlushAt = SHDR_FLUSH_AT;  // staged updates that trigger a batch after an item
constexpr uint64_t kInfBits = 0x7FF0000000000000ull;

// Scope of the per-slot state accesses. A slot is owned by ONE workgroup (one CU),
// so workgroup scope suffices and keeps the lines in the XCD's L2 (agent-scope
// atomics and sc1 loads drop them and go to the fabric).
#ifdef SHDR_AGENT_SCOPE
#define SLOT_SCOPE __HIP_MEMORY_SCOPE_AGENT
#else
#define SLOT_SCOPE __HIP_MEMORY_SCOPE_WORKGROUP
#endif
__device__ __forceinline__ uint64_t ld_u64_sc1(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, SLOT_SCOPE);
}
__device__ __forceinline__ uint32_t ld_u32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, SLOT_SCOPE);
}
__device__ __forceinline__ void slot_min(uint64_t* p, uint64_t v) {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, SLOT_SCOPE);
}
// "Kept" loads for software pipelines: a plain load whose value is used on one
// side of a select gets sunk into a branch by the compiler, and an exec-masked
// load makes it wait for EVERY load in flight at the join (s_waitcnt vmcnt(0)),
// which serialises the pipeline. Relaxed atomic loads are never sunk; at
// workgroup scope they are the same global_load instructions.
__device__ __forceinline__ int32_t ldk_i32(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ double ldk_f64(const double* p) {
    return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ int2 ldk_i2(const int2* p) {
    const uint64_t b = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return make_int2(int32_t(uint32_t(b)), int32_t(uint32_t(b >> 32)));
}
__device__ __forceinline__ int4 ldk_i4(const int4* p) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
    const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return make_int4(int32_t(uint32_t(a)), int32_t(uint32_t(a >> 32)), int32_t(uint32_t(b)), int32_t(uint32_t(b >> 32)));
}

// LDS hand-off between lanes of one wave: order the ds_write before the ds_read.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ double as_f64(uint64_t b) { return __builtin_bit_cast(double, b); }
__device__ __forceinline__ uint64_t as_u64(double d) { return __builtin_bit_cast(uint64_t, d); }
// (an integer argument would convert numerically: the round-4 guard record read a
// distance word that way and showed ordinary distances as ~2^62)
template <typename T> uint64_t as_u64(T) = delete;

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
    int32_t lat_is_w;       // w == canonical latency on every arc (bitwise)
    int32_t fold_add;       // SHDR_PATH_JITTER: ocrel/icrel hold per-arc jitter, folded by sum
    const int4* pitems;     // in-CSR items {vertex, first in-arc, count <= kChunk, 1 first | 2 last}
    int32_t npitems;
    const int32_t* pfirst;  // [V+1] first item of each vertex in pitems
    // relaxation arcs packed per 8 into 128-B blocks (one cache line per work item):
    // words 0-3 = col[0..7] (u32 pairs), words 4-11 = w[0..7] (f64 bits), 12-15 unused;
    // a vertex's last block is padded with (itself, +inf). Block nblk is all padding.
    const uint64_t* ablk;
    const int32_t* bfirst;  // [V+1] first block of each vertex
    int32_t nblk;
    // Vertices [vexp, V) never need relaxing: every arc in or out joins the same
    // single neighbour q (pendant vertices; device numbering puts them last), so
    // a path through them returns to q and cannot improve anything
    // (dist[q] + w_in + w_out > dist[q] for positive latencies). They get
    // distances and predecessors like any vertex but never enter a pending set.
    int32_t vexp;
    // Hub lag (hub_blocks > 0, plain workgroups with the near set in LDS): a vertex
    // of >= hub_blocks arc blocks that turns near-pending waits one round (its lag
    // byte, the slot's otherwise unused nflag byte) unless only such vertices are
    // pending. Its value may still improve in that round (a hub is reached from many
    // neighbours, first at non-final values), so its many rows are read fewer times.
    int32_t hub_blocks;
    int32_t far_skip;  // skip far marks the head row shows are redundant (flush, kFarKnown)
    int32_t reach_all;  // strongly connected: every vertex reachable from every source (kNoFill)
};

// Arc block words held by one sub-group lane: word (l & 15), and for K = 8 also word l + 8.
template <int K>
struct ArcWords {
    uint64_t a, b;
};
template <int K>
__device__ __forceinline__ ArcWords<K> load_arcs(const DevGraph& g, int32_t blk, int l) {
    ArcWords<K> x;
    const uint64_t* p = g.ablk + size_t(blk) * 16;
    x.a = p[l & 15];
    if constexpr (K < 16) x.b = p[l + 8]; else x.b = 0;
    return x;
}
// Compile-time loop: f(std::integral_constant<int, i>) for i in [0, N) (DPP lane
// selects are instruction immediates, so the unrolled index must be a constant).
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}
// Lane J of every 16-lane DPP row, broadcast to the whole row (row_newbcast): a VALU
// move, no LDS round trip and no lgkmcnt wait (ds_bpermute costs both). Every lane
// of the wave must be active.
template <int J>
__device__ __forceinline__ uint32_t row_bcast(uint32_t x) {
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x150 + J, 0xF, 0xF, false));
}
template <int J>
__device__ __forceinline__ uint64_t row_bcast64(uint64_t x) {
    return uint64_t(row_bcast<J>(uint32_t(x))) | (uint64_t(row_bcast<J>(uint32_t(x >> 32))) << 32);
}
// Sub-group lane J (< min(K, 16)) broadcast to the K lanes of the sub-group. K = 16
// is one DPP row; K = 8 is half a row (the two halves take lanes J and 8 + J);
// wider sub-groups span rows and go through ds_bpermute.
template <int K, int J>
__device__ __forceinline__ uint64_t sub_lane64(uint64_t x, int lane, int sbase) {
    if constexpr (K == 16) {
        return row_bcast64<J>(x);
    } else if constexpr (K == 8) {
        static_assert(J < 8, "K = 8 sub-group lane");
        const uint64_t a = row_bcast64<J>(x), b = row_bcast64<8 + J>(x);
        return (lane & 8) ? b : a;
    } else {
        return uint64_t(__shfl((long long)x, sbase + J));
    }
}
template <int K, int J>
__device__ __forceinline__ int32_t sub_lane32(int32_t x, int lane, int sbase) {
    if constexpr (K == 16) {
        return int32_t(row_bcast<J>(uint32_t(x)));
    } else if constexpr (K == 8) {
        static_assert(J < 8, "K = 8 sub-group lane");
        const uint32_t a = row_bcast<J>(uint32_t(x)), b = row_bcast<8 + J>(uint32_t(x));
        return int32_t((lane & 8) ? b : a);
    } else {
        return __shfl(x, sbase + J);
    }
}
// Word W (< 16) of the sub-group's arc block, broadcast to its K lanes: for K >= 16
// every DPP row holds the whole block (lane l has word l & 15); for K = 8 words 0-7
// are in .a and 8-15 in .b of the sub-group's own 8 lanes.
template <int K, int W>
__device__ __forceinline__ uint64_t blk_word(const ArcWords<K>& x, int lane, int sbase) {
    if constexpr (K >= 16) return row_bcast64<W>(x.a);
    else return sub_lane64<K, (W & 7)>(W < 8 ? x.a : x.b, lane, sbase);
}
// arc Q (< kChunk) of the sub-group's block: head vertex and weight, broadcast to all K lanes
template <int K, int Q>
__device__ __forceinline__ int32_t arc_col(const ArcWords<K>& x, int lane, int sbase) {
    const uint64_t p = blk_word<K, (Q >> 1)>(x, lane, sbase);
    return int32_t((Q & 1) ? uint32_t(p >> 32) : uint32_t(p));
}
template <int K, int Q>
__device__ __forceinline__ double arc_w(const ArcWords<K>& x, int lane, int sbase) {
    return as_f64(blk_word<K, 4 + Q>(x, lane, sbase));
}

// Per-slot scratch of the persistent kernel (one slot per resident workgroup).
struct SlotWs {
    uint64_t* dist;    // [V*K] f64 bits
    int2* pred;        // [V*K] {pred vertex, in-arc index}
    uint8_t* nflag;    // [V] near-pending byte per vertex (used when the bitmaps do not fit LDS)
    uint8_t* fflag;    // [V] far-pending byte per vertex
    int4* items;       // [cap] {vertex, first arc, arc count, 0}
};

struct SlotArena {
    char* base;
    size_t stride;
    int64_t item_cap;
    int* err;     // set non-zero by a workgroup that hit a guard (host reports it)
    int* ticket;  // next bucket to hand out (dynamic scheduling), one per launch
    size_t off_pred, off_nflag, off_fflag, off_items;
    // Cluster mode (k_routes_sssp<..., CLU = true>): cl workgroups share one bucket
    // and one slot. Per cluster, at cbase + cluster * cstride: a ClusterRec, then
    // per member a private far-set byte array (PM 1; c_far bytes each), the
    // published near bitmaps ([2 parities][cl][c_plane words]), and the work-item
    // lists of members 1..cl-1 (c_items bytes each; member 0 uses the slot's).
    int32_t cl;
    char* cbase;
    size_t cstride, c_off_far, c_far, c_off_plane, c_plane, c_off_items, c_items;
    __device__ SlotWs at(int slot) const {
        char* b = base + size_t(slot) * stride;
        SlotWs s;
        s.dist = reinterpret_cast<uint64_t*>(b);
        s.pred = reinterpret_cast<int2*>(b + off_pred);
        s.nflag = reinterpret_cast<uint8_t*>(b + off_nflag);
        s.fflag = reinterpret_cast<uint8_t*>(b + off_fflag);
        s.items = reinterpret_cast<int4*>(b + off_items);
        return s;
    }
};

struct RouteOut {
    double* lat;      // [S*T]
    double* rel;      // [S*T]
    int32_t* hops;    // [S*T] or null
    double* row_min;  // [S] or null
    int32_t T;
    const int32_t* rowmap;  // processed source i -> output row (null = identity)
    const double* soff;     // per processed source: near/far key offset (null = 0)
    uint32_t* bcost;        // per bucket of this launch: duration in 100 MHz ticks (null = off)
    const int32_t* boff;    // per bucket b of this launch: rows [boff[b], boff[b+1]) (null = K-row buckets)
    int32_t nb;             // buckets of this launch when boff is set
    uint32_t* done;         // per bucket: set (system scope, host-mapped) once its rows are in HBM (null = off)
};

// Per-cluster record: the barrier counter on a line of its own, then the values
// each member publishes before a barrier (double-buffered by barrier parity:
// a member writes buffer p only after every member has passed the barrier that
// followed the last read of p), then the members' per-lane row minima.
struct ClusterVal {
    uint32_t any_near, any_far, moved, pad;
    unsigned long long minfar;
    int32_t bucket, pad2;
};
struct ClusterRec {
    uint32_t arrive;
    uint32_t xcc;  // OR of 1 << (member's XCD): the members must share one L2
    uint32_t pad[30];
    ClusterVal val[2][8];
    unsigned long long rowmin[8][64];
};
constexpr size_t kClusterRecBytes = 8192;
static_assert(sizeof(ClusterRec) <= kClusterRecBytes, "cluster record");
constexpr int kMaxCluster = 8;
// bound of every cross-workgroup spin (cluster barriers): 4 s at 100 MHz
#ifndef SHDR_SPIN_TICKS
#define SHDR_SPIN_TICKS 400000000ull
#endif
constexpr int kAutoCluster = 4;  // largest cluster the automatic rule picks

// First-failure record next to the guard word (err[4] = 1 once taken, err[5..15]
// = the failing site's fields): one confirming run names the bucket, cluster
// member, lane and vertices of the first guard trip instead of only its code.
constexpr int kErrWords = 16;
__device__ __forceinline__ void guard_record(int* err, int code, int f0, int f1, int f2, int f3, int f4, int f5,
                                             int f6, int f7, int f8) {
    atomicOr(err, code);
    if (atomicCAS(err + 4, 0, 1) == 0) {
        const int f[11] = {code, f0, f1, f2, f3, f4, f5, f6, f7, f8, 0};
        for (int i = 0; i < 11; ++i) __hip_atomic_store(err + 5 + i, f[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Order-preserving f64 -> u64 map (for atomicMin over possibly negative keys).
__device__ __forceinline__ uint64_t key_enc(double x) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double key_dec(uint64_t k) {
    return __builtin_bit_cast(double, (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k);
}

// Distance rows without a per-bucket fill. A bucket of parity par stores its
// distances as plain f64 bits lowered with atomicMin (par 0) or as complemented
// bits raised with atomicMax (par 1); either way a row word left by the previous
// bucket (the other parity) decodes as +inf and loses every comparison, so a
// slot's next bucket needs no 128-MB (cfg5) refill of its rows. That holds when
// the previous bucket wrote every (vertex, lane) word: every vertex reachable
// from every source (strongly connected graph) and every lane holding a source;
// otherwise the slot's state byte says "dirty" and the next bucket fills.
// Distances are non-negative, so valid words decode below +inf's bits.
#ifndef SHDR_NOFILL
#define SHDR_NOFILL 1
#endif
constexpr bool kNoFill = SHDR_NOFILL;
__device__ __forceinline__ uint64_t denc(double d, int par) {
    const uint64_t b = __builtin_bit_cast(uint64_t, d);
    return par ? ~b : b;
}
__device__ __forceinline__ double ddec(uint64_t x, int par) {
    const uint64_t y = par ? ~x : x;
    return y < 0x7FF0000000000000ull ? __builtin_bit_cast(double, y) : __builtin_inf();
}

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
// wave-wide inclusive prefix sum
__device__ __forceinline__ int wave_incl_scan(int x, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x;
}

// One workgroup owns one bucket of K sources at a time, from empty state to
// finished rows. NT threads = NT/64 waves = NSUB sub-groups of K lanes; lane l
// of every sub-group serves source lane l of the bucket.
//
// Relaxation is near-far delta-stepping over vertex ROWS. Every lane carries a
// key = dist - off; a vertex is pending "near" once some lane improved to a key
// below the threshold, "far" otherwise. Pending state is ONE bit per vertex
// (LDS bitmaps when they fit, PM 2 / near only PM 1; else slot bytes): relaxing a
// vertex relaxes every lane whose key is below the threshold, so lanes that did
// not change cost compares, not memory operations, and an improvement costs a
// single scattered memory operation (the atomicMin) plus an LDS bit. A lane value
// is never relaxed before its key is below the threshold, and every value is
// relaxed once the threshold passes it (drains re-mark far vertices), which is
// all the argument for the exact distances needs. Rounds are separated by
// workgroup barriers, so pending words are taken without atomics.
//
// CLU (cluster mode, small shards): arena.cl workgroups share one bucket and
// its slot, so a shard with fewer buckets than CUs still fills the chip (the
// relaxation of one bucket is bound by its CU's memory requests, ~40 rounds of
// ~500 us on cfg4, so splitting a round's work over cl CUs divides it). Every
// round ends in a cluster barrier with an agent-scope release/acquire
// (placement-independent: members need not share an XCD, they are only
// mapped to one for L2 affinity). Per round each member publishes its LDS
// near bitmap (marks it made), and relaxes the vertices of the words it owns
// (word w belongs to member w % cl) of the OR of all published bitmaps; far
// sets stay private (each member drains the vertices it marked far); the
// drain's moved / far / minimum-key decisions are reduced over the cluster.
// Distance updates are agent-scope atomics; a row read that misses another
// member's improvement of this round only costs a redundant relaxation (the
// improver marked the vertex, so it is relaxed again next round after the
// barrier's acquire). The predecessor pass (full in-arc list) and the epilogue
// (targets) are split over the members; the leader draws the bucket tickets
// and writes the row minima.
// epilogue: NCH chains per lane, each with a kStack-deep stack of u32 in-arc indices
#ifndef SHDR_NCH
#define SHDR_NCH 2
#endif
// The workgroup's static LDS. It depends on (NT, PM) only, not on the bucket width
// K, so one workgroup can run buckets of two widths in one launch (k_routes_pass:
// the half-width tail buckets, then the full-width ones) over a single allocation.
template <int NT, int PM>
struct Smem {
    static constexpr int NW = NT / 64;
    static constexpr int FC = PM == 1 ? kFlushCap / 2 : kFlushCap;  // staging slots per wave
    static constexpr int NCH = SHDR_NCH;
    static constexpr int kStack = stack_depth(NT) * 2 / NCH;
    // relaxation staging and the epilogue's hop stacks are never live together
    // (PM 1: the stacks live in the dynamic region instead, dead bitmaps by then)
    static constexpr size_t kStageBytes = size_t(NW) * FC * (sizeof(int32_t) + sizeof(double));
    static constexpr size_t kStackBytes = size_t(NCH) * kStack * NT * sizeof(uint32_t);
    static constexpr size_t kPoolBytes = (PM == 1 || kStageBytes > kStackBytes) ? kStageBytes : kStackBytes;
    double pool[kPoolBytes / sizeof(double)];
    unsigned long long rowmin_l[64];  // per source lane, key_enc order
    unsigned long long minfar;
    int32_t vlist[NW][128];  // per-wave vertex lists (compaction, drain)
    int32_t nitems, npairs, anyv, anydef, far_flag, moved, cfail, par, fill, bucket;
};

template <int K, int NT, int PM, bool CLU = false>
__device__ __forceinline__ void sssp_body(const DevGraph& g, const SlotArena& arena, const int32_t* __restrict__ src,
                                          int32_t S, const int32_t* __restrict__ dst, int32_t nbuckets, double delta,
                                          const RouteOut& out, int keep_slots, Smem<NT, PM>& sm) {
    constexpr int G = 64 / K;     // sub-groups per wave
    constexpr int NW = NT / 64;
    constexpr int NSUB = NW * G;
    // pending-set storage (PM): 2 = near and far bitmaps in LDS; 1 = near bitmap in
    // LDS, far set as slot bytes; 0 = both as slot bytes (4 vertices per word)
    constexpr bool NEAR_LDS = PM >= 1, FAR_LDS = PM == 2;
    constexpr int VPWN = NEAR_LDS ? 32 : 4, VPWF = FAR_LDS ? 32 : 4;  // vertices per 32-bit word
    constexpr int FC = Smem<NT, PM>::FC;                                // staging slots per wave
    static_assert(!CLU || NEAR_LDS, "cluster mode publishes the LDS near bitmap");
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int sub = lane / K;    // sub-group within the wave
    const int l = lane % K;      // source lane within the bucket
    const int sbase = sub * K;   // first wave lane of this sub-group
    const int gsub = wave * G + sub;
    const int32_t V = g.V;
    // index helpers; SHDR_BCHK builds (debug flavour only) clamp out-of-range
    // indices to 0 and flag them in the error word instead of faulting
#ifdef SHDR_BCHK
#define SIDX(v, ln) bchk(size_t(v) * K + size_t(ln), size_t(V) * K, 256, (v) >= 0 && (v) < V && (ln) >= 0 && (ln) < K)
#define AIDX(a) bchk(size_t(a), size_t(g.A), 512, true)
#define IIDX(i) bchk(size_t(i), size_t(arena.item_cap), 1024, (i) >= 0)
    auto bchk = [&](size_t i, size_t n, int code, bool ok) -> size_t {
        if (!ok || i >= n) { atomicOr(arena.err, code); return 0; }
        return i;
    };
#else
#define SIDX(v, ln) (size_t(v) * K + (ln))
#define AIDX(a) (a)
#define IIDX(i) (i)
#endif
    // relaxation scans only the words of vertices that can be pending ([0, vexp));
    // the chain pass below uses the same storage over all V
    const int32_t WN = (g.vexp + VPWN - 1) / VPWN, WF = (g.vexp + VPWF - 1) / VPWF;
    const int32_t WNall = (V + VPWN - 1) / VPWN;

    extern __shared__ uint32_t s_dyn[];  // LDS bitmaps: near [WN] (then far [WF]); PM 1: also the hop stacks
    int32_t& s_nitems = sm.nitems;
    int32_t& s_npairs = sm.npairs;  // half-block pairs of this round (relax_items, pair)
    int32_t& s_anyv = sm.anyv;  // phase 1 found a near vertex
    int32_t& s_anydef = sm.anydef;  // phase 1 deferred a hub (hub lag)
    int32_t& s_far_flag = sm.far_flag;
    int32_t& s_moved = sm.moved;
    unsigned long long& s_minfar = sm.minfar;
    auto& s_vlist = sm.vlist;  // [NW][128]
    auto& s_rowmin_l = sm.rowmin_l;  // [64]
    constexpr int NCH = Smem<NT, PM>::NCH;
    constexpr int kStack = Smem<NT, PM>::kStack;
    double* const s_pool = sm.pool;
    double* s_ec = s_pool;                                                   // [NW][FC] candidate
    int32_t* s_ev = reinterpret_cast<int32_t*>(s_pool + NW * FC);             // [NW][FC] (v<<6)|(near<<5)|lane
    uint32_t* s_stack = PM == 1 ? s_dyn : reinterpret_cast<uint32_t*>(s_pool);  // [NCH][kStack][NT] in-arc

    // cluster identity: cid = bucket slot, cr = rank in the cluster. Members of a
    // cluster are blocks b, b+8, ... (dealt to one XCD: L2 affinity only)
    int32_t cl = 1, cr = 0, cid = blockIdx.x;
    if constexpr (CLU) {
        cl = arena.cl;
        const int32_t bid = blockIdx.x;
        if (gridDim.x % (8 * cl) == 0) {
            const int32_t kq = bid >> 3;
            cr = kq % cl;
            cid = (bid & 7) + 8 * (kq / cl);
        } else {
            cr = bid % cl;
            cid = bid / cl;
        }
    }
    const int slot = cid;
    SlotWs ws = arena.at(slot);
    char* const crec_b = CLU ? arena.cbase + size_t(cid) * arena.cstride : nullptr;
    ClusterRec* const crec = reinterpret_cast<ClusterRec*>(crec_b);
    if constexpr (CLU) {
        if (cr > 0) ws.items = reinterpret_cast<int4*>(crec_b + arena.c_off_items + size_t(cr - 1) * arena.c_items);
        if (PM == 1) ws.fflag = reinterpret_cast<uint8_t*>(crec_b + arena.c_off_far + size_t(cr) * arena.c_far);
    }
    // published near bitmap of member r, parity p
    auto plane = [&](int p, int r) -> uint32_t* {
        return reinterpret_cast<uint32_t*>(crec_b + arena.c_off_plane) + (size_t(p) * cl + r) * arena.c_plane;
    };
    // Cluster barrier (every thread calls it): stores and atomics of every wave
    // drained, agent release, one arrival on the monotonic counter, a bounded
    // poll, agent acquire. false = timed out (a member never arrived: the guard
    // word gets 8 and the workgroup leaves the kernel).
    // Once the first barrier has shown every member on one XCD (next_bucket), the
    // members share that XCD's L2: drained stores are already visible to the
    // others there, and the agent release (a write-back of every dirty line of
    // the whole L2, other workgroups' included) is dropped. The acquire stays
    // (members' L1s are private). This relies on every cluster-shared buffer
    // (slot rows, planes, cluster records) being coarse-grained device memory
    // that the XCD's L2 caches: the arena and d_cl come from plain hipMalloc
    // only (arena_alloc, ensure); fine-grained or host-mapped memory would need
    // the release back.
    uint32_t cgen = 0;
    bool c_one_xcd = false;
    DIAG_LOCAL(unsigned long long d_cbn = 0, d_cbt = 0;)
    int32_t& s_cfail = sm.cfail;
    auto cbar = [&]() -> bool {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        ++cgen;
        if (tid == 0) {
            DIAG_LOCAL(const unsigned long long d_cb0 = DIAG_NOW(); ++d_cbn;)
            s_cfail = 0;
            if (!c_one_xcd) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&crec->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t target = cgen * uint32_t(cl);
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(&crec->arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > SHDR_SPIN_TICKS) {
                    atomicOr(arena.err, 8);
                    s_cfail = 1;
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            DIAG_LOCAL(d_cbt += DIAG_NOW() - d_cb0;)
        }
        __syncthreads();
        return s_cfail == 0;
    };
    (void)plane; (void)cbar;
    // this bucket's row encoding parity (denc / ddec): plain workgroups on strongly
    // connected graphs; cluster and kept-tree launches always fill (parity 0). The
    // slot's state byte sits past the pending bytes' last word (nflag[V + 8]).
    const bool nofill_ok = kNoFill && !CLU && !(keep_slots & 1) && g.reach_all;
    int par = 0;
    int32_t& s_par = sm.par;
    int32_t& s_fill = sm.fill;
    uint32_t* near_w = NEAR_LDS ? s_dyn : reinterpret_cast<uint32_t*>(ws.nflag);
    uint32_t* far_w = FAR_LDS ? s_dyn + WNall : reinterpret_cast<uint32_t*>(ws.fflag);

    auto mark = [&](bool is_near, int32_t v) {
        if (is_near) {
            if constexpr (NEAR_LDS) atomicOr(&near_w[v >> 5], 1u << (v & 31));
            else ws.nflag[v] = 1;
        } else {
            if constexpr (FAR_LDS) atomicOr(&far_w[v >> 5], 1u << (v & 31));
            else ws.fflag[v] = 1;
        }
    };
    // take (read and clear) one pending word; bit i <=> vertex wi*VPW + i
    auto take_word = [&](uint32_t* arr, int32_t wi, auto lds) -> uint32_t {
        constexpr bool L = decltype(lds)::value;
        uint32_t x;
        if constexpr (L) x = arr[wi];
        else x = ld_u32(&arr[wi]);
        if (!x) return 0u;
        arr[wi] = 0u;
        if constexpr (L) return x;
        else return ((x & 0xFFu) ? 1u : 0u) | ((x & 0xFF00u) ? 2u : 0u) | ((x & 0xFF0000u) ? 4u : 0u) |
                    ((x & 0xFF000000u) ? 8u : 0u);
    };
    // Wave-level compaction of pending-set words (one word per lane, vpw vertices
    // per word) into a list of vertices, handed to emit() 64 at a time: a batch
    // costs one round of global loads however the set bits spread over the lanes.
    // emit(v) is called by the whole wave, v = -1 on lanes without a vertex.
    auto compact_words = [&](int32_t w0, int32_t nwords, int vpw, auto&& take, auto&& emit) {
        int32_t* wl = s_vlist[wave];
        int cnt = 0;  // wave-uniform
        auto flush_list = [&]() {
            wave_sync();
            for (int e0 = 0; e0 < cnt; e0 += 64) emit(e0 + lane < cnt ? wl[e0 + lane] : -1);
            wave_sync();
            cnt = 0;
        };
        for (int32_t wi = w0 + tid; wi - lane < nwords; wi += NT) {  // wave-uniform trip count
            uint32_t bits = wi < nwords ? take(wi) : 0u;
            while (__any(bits != 0)) {
                const bool has = bits != 0;
                const unsigned long long bal = __ballot(has);
                if (has) {
                    wl[cnt + __popcll(bal & ((1ull << lane) - 1ull))] = wi * vpw + __builtin_ctz(bits);
                    bits &= bits - 1;
                }
                cnt += __popcll(bal);
                if (cnt >= 64) flush_list();
            }
        }
        if (cnt > 0) flush_list();
    };
    // the same over the words map(t), t in [0, ntot) (cluster mode: a member's own words)
    auto compact_map = [&](int32_t ntot, auto&& map, int vpw, auto&& take, auto&& emit) {
        int32_t* wl = s_vlist[wave];
        int cnt = 0;
        auto flush_list = [&]() {
            wave_sync();
            for (int e0 = 0; e0 < cnt; e0 += 64) emit(e0 + lane < cnt ? wl[e0 + lane] : -1);
            wave_sync();
            cnt = 0;
        };
        for (int32_t t = tid; t - lane < ntot; t += NT) {
            const int32_t wi = map(t);
            uint32_t bits = t < ntot ? take(wi) : 0u;
            while (__any(bits != 0)) {
                const bool has = bits != 0;
                const unsigned long long bal = __ballot(has);
                if (has) {
                    wl[cnt + __popcll(bal & ((1ull << lane) - 1ull))] = wi * vpw + __builtin_ctz(bits);
                    bits &= bits - 1;
                }
                cnt += __popcll(bal);
                if (cnt >= 64) flush_list();
            }
        }
        if (cnt > 0) flush_list();
    };
    (void)compact_map;
    // work-item buffer: items [0, nitems) from the bottom, half-block pairs from
    // items[icap - 1] down, items[icap] = the all-padding pair (relax_items)
    const int64_t icap = arena.item_cap - 1;
    // append n items per vertex (wave-wide prefix over the lanes' counts)
    auto append_items = [&](int32_t v, int32_t n, auto&& item_of) {
        const int incl = wave_incl_scan(n, lane);
        const int total = __shfl(incl, 63);
        if (total == 0) return;
        int wbase = 0;
        if (lane == 63) wbase = atomicAdd(&s_nitems, total);
        wbase = __shfl(wbase, 63);
        if (int64_t(wbase) + total > icap) {
            if (lane == 0) atomicOr(arena.err, 2);
            return;
        }
        const int o = wbase + incl - n;
        for (int32_t c = 0; c < n; ++c) ws.items[IIDX(o + c)] = item_of(c);
    };
    // Pair the wave's half blocks (lanes with half set, block hb of vertex v): the lane
    // of even rank among them takes the next one's as b (none: the all-padding block).
    // Called by the whole wave; pairs fill the item buffer from the top down.
    auto append_pairs = [&](int32_t v, bool half, int32_t hb) {
        const unsigned long long hm = __ballot(half);
        if (hm == 0) return;
        const int rank = __popcll(hm & ((1ull << lane) - 1ull));
        const unsigned long long above = lane == 63 ? 0ull : hm & (~0ull << (lane + 1));
        const int partner = above ? __builtin_ctzll(above) : lane;
        const int32_t pv = __shfl(v, partner), pb = __shfl(hb, partner);
        const bool own = half && !(rank & 1);
        const unsigned long long om = __ballot(own);
        const int total = __popcll(om);
        int pbase = 0;
        if (lane == 0) pbase = atomicAdd(&s_npairs, total);
        pbase = __shfl(pbase, 0);
        if (own) {
            const int64_t p = int64_t(pbase) + __popcll(om & ((1ull << lane) - 1ull));
            ws.items[IIDX(icap - 1 - p)] = above ? make_int4(v, hb, pv, pb) : make_int4(v, hb, 0, g.nblk);
        }
    };
    using NearL = std::integral_constant<bool, NEAR_LDS>;
    using FarL = std::integral_constant<bool, FAR_LDS>;
    // Apply staged updates [0, cnt): min into dist, then the vertex's pending bit.
    // Staged candidates carry a flag in bit 63 (distances are >= +0, sign clear):
    // set when the vertex is already in the far set, so a far update needs no mark.
    // Invariant: a vertex with a finite far key in any lane has its far bit (every
    // first far value marks it, and each drain re-marks the far vertices it keeps),
    // so the staging step skips the mark when the head row it read shows one. On
    // PM 1 tables (cfg5) that is a scattered byte store per far event saved.
    constexpr uint64_t kFarKnown = 0x8000000000000000ull;
    auto flush = [&](int cnt) {
        for (int e0 = 0; e0 < cnt; e0 += 64) {
            const int e = e0 + lane;
            if (e < cnt) {
                const int32_t ev = s_ev[wave * FC + e];
                const int32_t vv = ev >> 6, ll = ev & 31;
                const bool nr = ev & 32;
                const uint64_t cb = as_u64(s_ec[wave * FC + e]);
                if constexpr (CLU)  // rows shared with the other members' CUs (always parity 0)
                    __hip_atomic_fetch_min(&ws.dist[SIDX(vv, ll)], cb & ~kFarKnown, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                else if (par)
                    __hip_atomic_fetch_max(&ws.dist[SIDX(vv, ll)], ~(cb & ~kFarKnown), __ATOMIC_RELAXED, SLOT_SCOPE);
                else
                    slot_min(&ws.dist[SIDX(vv, ll)], cb & ~kFarKnown);
                if (vv < g.vexp) {
                    // (cluster mode always marks: the far sets are private to the members)
                    const bool always = kExperiments ? (!g.far_skip || (CLU && g.far_skip != 3)) : CLU;
                    if (nr || !(cb & kFarKnown) || always) mark(nr, vv);
                    if (!nr) s_far_flag = 1;
                }
            }
        }
    };

    // Phase 2 of a round: relax the arcs of items g0, g0 + gstride, ... of the
    // bucket's list (n items) at threshold thr, for this lane's key offset off.
    // Software pipeline over this sub-group's items: iteration k issues the dist
    // rows of item k+1, the arc data of item k+2 and the descriptor of item k+3,
    // then compares item k. Loads are unconditional (padding arcs read a valid row
    // with weight +inf) so the vmcnt waits count them statically. Improvements are
    // staged in LDS and applied in batches of >= 64, so the wait for a row seldom
    // covers an atomic. Arc broadcasts within a sub-group are DPP row moves
    // (sub_lane / blk_word): no LDS round trip sits between an arc block's arrival
    // and its row loads.
    //
    // Pair items (pair = true): two half blocks (<= kHalf real arcs each) of two
    // pending vertices a and b in one item {a, block of a, b, block of b}, stored
    // from the top of the item buffer down (pair p at items[icap - 1 - p]). Arc q <
    // kHalf is arc q of a's block, arc q >= kHalf is arc q - kHalf of b's block: the
    // sub-group's lanes load the words of the item's logical block from the two
    // blocks (pair_word), so the arc broadcasts are unchanged; each half compares
    // against its own vertex's row. Eight head-row loads then serve two vertices
    // instead of one plus padding. Past the list a lane reads the all-padding pair
    // at items[icap] (written at bucket start), so the descriptor load needs no select.
    DIAG_LOCAL(unsigned long long d_arcs = 0, d_atom = 0, d_imp = 0, d_ev = 0, d_act = 0, d_rows = 0, d_hubrows = 0;)
    auto relax_items = [&](const int32_t n, const int32_t g0, const int32_t gstride, const double thr, const double off,
                           auto pair) {
        constexpr bool P = decltype(pair)::value;
        using Desc = std::conditional_t<P, int4, int2>;
        const unsigned long long sub_m = (K == 64 ? ~0ull : ((1ull << K) - 1ull)) << sbase;
        const int32_t niters = (n - g0 + gstride - 1) / gstride;
        int32_t witers = max(niters, 0);  // the wave runs the max over its sub-groups
#pragma unroll
        for (int o = K; o < 64; o <<= 1) witers = max(witers, __shfl_xor(witers, o));
        witers = __builtin_amdgcn_readfirstlane(witers);
        // past the list: the all-padding block (vertex 0, weights +inf)
        // (loads are unconditional — an exec-masked load makes the compiler wait
        // for every load in flight at the branch join, serialising the pipeline —
        // and out-of-list lanes select the padding descriptor afterwards)
        // descriptor {vertex, block} (pairs: {vertex a, block a, vertex b, block b})
        auto desc = [&](int32_t k) -> Desc {
            const int32_t it = g0 + k * gstride;
            if constexpr (P) {
                return ws.items[IIDX(it < n ? icap - 1 - it : icap)];
            } else {
                const int2 x = ldk_i2(reinterpret_cast<const int2*>(&ws.items[IIDX(it < n ? it : 0)]));
                return it < n ? x : make_int2(0, g.nblk);
            }
        };
        // logical word W of the item's block: pairs take words 2-3 (columns 4-7) and
        // 8-11 (weights 4-7) from b's block, as its words 0-1 and 4-7
        auto word_ptr = [&](const Desc& d, int W) -> const uint64_t* {
            if constexpr (P) {
                const bool fromb = (0x0F0Cu >> W) & 1u;  // W in {2, 3, 8..11}
                const uint32_t wo = uint32_t(W) - (fromb ? ((W & 8) ? 4u : 2u) : 0u);
                return g.ablk + (size_t(uint32_t(fromb ? d.w : d.y)) << 4) + wo;
            } else {
                return g.ablk + size_t(d.y) * 16 + W;
            }
        };
        auto arcs_of = [&](const Desc& d) -> ArcWords<K> {
            ArcWords<K> x;
            x.a = *word_ptr(d, l & 15);
            if constexpr (K < 16) x.b = *word_ptr(d, l + 8); else x.b = 0;
            return x;
        };
        auto head_row = [&](int32_t v) -> double { return ddec(ld_u64_sc1(&ws.dist[SIDX(v, l)]), par); };
        auto vb_of = [&](const Desc& d) -> int32_t {
            if constexpr (P) return d.z; else return d.x;
        };
        Desc d0 = desc(0), d1 = desc(1), d2 = desc(2), d3;
        ArcWords<K> wd0 = arcs_of(d0), wd1 = arcs_of(d1);
        double du0 = head_row(d0.x), du1 = head_row(d1.x);
        double ub0 = P ? head_row(vb_of(d0)) : 0.0, ub1 = P ? head_row(vb_of(d1)) : 0.0;  // (b's rows: pairs)
        double o0[kChunk];
        sfor<kChunk>([&](auto qc) { o0[qc.value] = head_row(arc_col<K, qc.value>(wd0, lane, sbase)); });
        int cnt = 0;  // staged updates of this wave (uniform)
        for (int32_t k = 0; k < witers; ++k) {
            // ---- issue: rows of item k+1, arc data of item k+2, descriptor of item k+3
            double o1[kChunk];
            sfor<kChunk>([&](auto qc) { o1[qc.value] = head_row(arc_col<K, qc.value>(wd1, lane, sbase)); });
            const ArcWords<K> wd2 = arcs_of(d2);
            const double du2 = head_row(d2.x);
            const double ub2 = P ? head_row(vb_of(d2)) : 0.0;
            d3 = desc(k + 3);
            // ---- compare item k: every lane whose key is below the threshold
            const bool act = du0 - off < thr;
            const bool actb = P ? ub0 - off < thr : act;
            DIAG_LOCAL(if (k * gstride + g0 < n) d_act += act;)
            DIAG_LOCAL(if (l == 0) d_arcs += (k * gstride + g0 < n) ? kChunk : 0;)
            DIAG_LOCAL(if (l == 0 && k * gstride + g0 < n) {
                d_rows += kChunk;  // (padding arcs counted too)
                if (!P && g.rowptr[d0.x + 1] - g.rowptr[d0.x] >= 64) d_hubrows += kChunk;
            })
            sfor<kChunk>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                constexpr bool hb = P && q >= kHalf;  // (pairs: b's half)
                const int32_t vq = arc_col<K, q>(wd0, lane, sbase);
                const double c = (hb ? ub0 : du0) + arc_w<K, q>(wd0, lane, sbase);
                const bool imp = (hb ? actb : act) && (c < o0[q]);
                const unsigned long long bm = __ballot(imp);
                // some lane of the head row holds a finite far key: the vertex is in the far set
                const bool farl = o0[q] < __builtin_inf() && !(o0[q] - off < thr);
                const bool far_known = (kExperiments && g.far_skip == 2) ? farl : (__ballot(farl) & sub_m) != 0;
                if (imp) {
                    const int pos = wave * FC + cnt + __popcll(bm & ((1ull << lane) - 1ull));
                    s_ev[pos] = (vq << 6) | ((c - off < thr) ? 32 : 0) | l;
                    s_ec[pos] = as_f64(as_u64(c) | (far_known ? kFarKnown : 0ull));
                }
                cnt += __popcll(bm);
                DIAG_LOCAL(d_atom += imp; d_imp += imp; if (l == 0 && ((bm >> sbase) & ((K == 64) ? ~0ull : ((1ull << K) - 1ull)))) ++d_ev;)
                if (cnt > FC - 64) {  // staging nearly full: apply now
                    wave_sync();
                    flush(cnt);
                    wave_sync();
                    cnt = 0;
                }
            });
            if (cnt >= kFlushAt) {  // apply a batch (after the next loads were issued)
                wave_sync();
                flush(cnt);
                wave_sync();
                cnt = 0;
            }
            // ---- rotate the pipeline
#pragma unroll
            for (int q = 0; q < kChunk; ++q) o0[q] = o1[q];
            wd0 = wd1; du0 = du1; ub0 = ub1;
            d0 = d1; d1 = d2; d2 = d3;
            wd1 = wd2; du1 = du2; ub1 = ub2;
        }
        wave_sync();
        flush(cnt);
    };

    // Buckets are handed out dynamically (an atomic ticket per workgroup) so that
    // workgroups drawing cheap buckets take more of them; KEEP_TREES launches
    // one workgroup per bucket and keep the bucket -> slot identity.
    int32_t& s_bucket = sm.bucket;
    auto next_bucket = [&](int32_t cur) -> int32_t {
        if (keep_slots & 1) return cur < 0 ? int32_t(blockIdx.x) : nbuckets;
        if constexpr (CLU) {  // the leader draws; the draw travels with a cluster barrier
            const int p = cgen & 1;
            if (tid == 0 && cr == 0) crec->val[p][0].bucket = atomicAdd(arena.ticket, 1);
            if (cur < 0 && tid == 0) {
                uint32_t x;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
                __hip_atomic_fetch_or(&crec->xcc, 1u << (x & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (!cbar()) return nbuckets;
            if (cur < 0) {
                // Members read each other's plain stores and rows through their L2:
                // a cluster spread over two XCDs (private, non-coherent L2s) cannot
                // run. Every member sees the same mask after the barrier, so all
                // leave together and the host recomputes without clusters.
                const uint32_t m = __hip_atomic_load(&crec->xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (m & (m - 1)) {
                    if (tid == 0) atomicOr(arena.err, 16);
                    return nbuckets;
                }
                c_one_xcd = true;
            }
            if (tid == 0) s_bucket = crec->val[p][0].bucket;
            __syncthreads();
            return s_bucket;
        }
        __syncthreads();
        if (tid == 0) s_bucket = atomicAdd(arena.ticket, 1);
        __syncthreads();
        return s_bucket;
    };
#ifdef SHDR_DIAG
    // workgroup start/exit spread of large launches (idle at the end of a launch)
    if (tid == 0 && nbuckets > 300) atomicMax(&g_diag[23], ~(unsigned long long)DIAG_NOW());
    struct ExitStamp {
        int32_t nb; int t;
        __device__ ~ExitStamp() {
            if (t == 0 && nb > 300) {
                const unsigned long long x = DIAG_NOW();
                atomicAdd(&g_diag[20], x); atomicMax(&g_diag[21], x); atomicMax(&g_diag[22], ~x); atomicAdd(&g_diag[24], 1ull);
            }
        }
    } exit_stamp{nbuckets, tid};
#endif
    for (int32_t b = next_bucket(-1); b < nbuckets; b = next_bucket(b)) {
        if (b < 0) {  // (a bucket ticket is never negative)
            if (tid == 0) guard_record(arena.err, 2048, b, cr, nbuckets, 0, 2, 0, 0, 0, 0);
            return;
        }
        const uint64_t tb0 = __builtin_amdgcn_s_memrealtime();
        const int32_t i0 = out.boff ? out.boff[b] : b * K;
        const int32_t nsrc = out.boff ? out.boff[b + 1] - i0 : min(K, S - i0);
        const int32_t my_src = (l < nsrc && i0 >= 0 && i0 + nsrc <= S) ? src[i0 + l] : -1;
        // The bucket record and its sources index everything below: one that is out
        // of range (a launch that read its inputs before they landed) stops the
        // workgroup with guard 64 instead of writing through wild indices. Every
        // member of a cluster reads the same record and leaves together.
        if (__syncthreads_or(nsrc < 1 || nsrc > K || i0 < 0 || i0 + nsrc > S ||
                             (l < nsrc && (my_src < 0 || my_src >= V)))) {
            if (tid == 0) guard_record(arena.err, 64, b, cr, i0, nsrc, S, my_src, 0, 0, 0);
            return;
        }
        // near/far keys are dist - off: lanes whose sources lie at different
        // distances from a common landmark then settle shared vertices together
        const double off = (out.soff && l < nsrc) ? out.soff[i0 + l] : 0.0;
        DIAG_LOCAL(unsigned long long d_t0 = DIAG_NOW(); unsigned long long d_rounds = 0, d_drains = 0,
                   d_scan = 0, d_items = 0, d_walk = 0, d_p1 = 0, d_drow = 0, d_drt = 0, d_hubexp = 0;
                   d_arcs = d_atom = d_imp = d_ev = d_act = d_rows = d_hubrows = 0;)

        // ---- init: this bucket's row encoding (kNoFill); dist = +inf when the
        // slot's rows are not all the previous bucket's (see denc); pending sets
        // empty (byte arrays are consumed back to 0)
        if (tid == 0) {
            ws.items[IIDX(icap)] = make_int4(0, g.nblk, 0, g.nblk);  // the all-padding pair
            const uint8_t st = nofill_ok ? ws.nflag[V + 8] : uint8_t(0);  // 0 dirty, 1 / 2: last bucket's parity + 1
            s_par = st == 1 ? 1 : 0;
            s_fill = st == 0 ? 1 : 0;
        }
        __syncthreads();
        par = s_par;
        {
            const size_t n2 = size_t(V) * K / 2;  // 16-byte stores
            ulonglong2* d2 = reinterpret_cast<ulonglong2*>(ws.dist);
            if (s_fill)  // (a filled slot starts at parity 0)
                for (size_t k = size_t(cr) * NT + tid; k < n2; k += size_t(cl) * NT) d2[k] = make_ulonglong2(kInfBits, kInfBits);
#if defined(SHDR_BCHK) || defined(SHDR_VERIFY)
            // debug flavours: poison the predecessor entries, so a walk that reaches a
            // vertex the predecessor pass never wrote trips the guard (code 32)
            for (size_t k = size_t(cr) * NT + tid; k < size_t(V) * K; k += size_t(cl) * NT) ws.pred[k] = make_int2(-2, -2);
#endif
            if constexpr (NEAR_LDS)
                for (int32_t k = tid; k < (FAR_LDS ? 2 * WNall : WNall); k += NT) s_dyn[k] = 0u;
        }
        // the bucket's clock starts at the smallest lane key (-max offset)
        if (tid == 0) { s_far_flag = 0; s_minfar = key_enc(__builtin_inf()); }
        __syncthreads();
        if (tid < nsrc && out.soff) atomicMin(&s_minfar, key_enc(-out.soff[i0 + tid]));
        __syncthreads();
        double thr = (out.soff ? key_dec(s_minfar) : 0.0) + delta;
        if constexpr (CLU) {  // every member's fill lands before the sources' rows are set
            if (!cbar()) return;
        }
        if (tid < nsrc && cr == 0) {
            const int32_t s = src[i0 + tid];
            const double key0 = out.soff ? -out.soff[i0 + tid] : 0.0;
            ws.dist[SIDX(s, tid)] = denc(0.0, par);
            if (s < g.vexp) {
                mark(key0 < thr, s);
                if (!(key0 < thr)) s_far_flag = 1;
            } else {
                // a pendant source has no pending bit: relax its arcs here (all to one q)
                for (int32_t a = g.rowptr[s]; a < g.rowptr[s + 1]; ++a) {
                    const int32_t q = g.col[a];
                    const double c = g.w[a];
                    if constexpr (CLU)
                        __hip_atomic_fetch_min(&ws.dist[SIDX(q, tid)], as_u64(c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else if (par)
                        __hip_atomic_fetch_max(&ws.dist[SIDX(q, tid)], ~as_u64(c), __ATOMIC_RELAXED, SLOT_SCOPE);
                    else
                        slot_min(&ws.dist[SIDX(q, tid)], as_u64(c));
                    if (q < g.vexp) {
                        mark(c - (out.soff ? out.soff[i0 + tid] : 0.0) < thr, q);
                        if (!(c - (out.soff ? out.soff[i0 + tid] : 0.0) < thr)) s_far_flag = 1;
                    }
                }
            }
        }
        __syncthreads();
        DIAG_LOCAL(unsigned long long d_t1 = DIAG_NOW();)
        const int64_t max_rounds = int64_t(V + 16) * (K + 2) + 4096;
        int64_t rounds = 0;

        for (;;) {
            if (++rounds > max_rounds) {
                if (tid == 0) atomicOr(arena.err, 1);
                break;
            }
            // cluster: publish this member's near marks; the cluster's near / far flags
            bool c_near = true, c_far = false;
            if constexpr (CLU) {
                const int p = cgen & 1;
                uint32_t* pl = plane(p, cr);
                int anyn = 0;
                for (int32_t k = tid; k < WN; k += NT) {
                    const uint32_t x = near_w[k];
                    pl[k] = x;
                    if (x) { near_w[k] = 0u; anyn = 1; }
                }
                anyn = __syncthreads_or(anyn);
                if (tid == 0) { crec->val[p][cr].any_near = uint32_t(anyn); crec->val[p][cr].any_far = uint32_t(s_far_flag); }
                if (!cbar()) return;
                uint32_t an = 0, af = 0;
                for (int r = 0; r < cl; ++r) { an |= crec->val[p][r].any_near; af |= crec->val[p][r].any_far; }
                c_near = an != 0;
                c_far = af != 0;
            }
            // ================= phase 1: near-pending vertices -> arc-chunk items
            DIAG_LOCAL(unsigned long long d_p1s = DIAG_NOW(); ++d_rounds;)
            bool lag = kExperiments && !CLU && NEAR_LDS && g.hub_blocks > 0;
            for (;;) {
                if (tid == 0) { s_nitems = 0; s_npairs = 0; s_anyv = 0; s_anydef = 0; }
                __syncthreads();
                auto emit_items = [&](int32_t v) {
                    int32_t b0 = 0, nb = 0;
                    if (v >= g.vexp) {  // (a pending bit past the expandable range: never set)
                        guard_record(arena.err, 2048, b, cr, v, g.vexp, 0, 0, 0, 0, 0);
                        v = -1;
                    }
                    bool half = false;  // v's last block is a half block (kHalfBit): relaxed in a pair
                    if (v >= 0) {
                        const int32_t f0 = g.bfirst[v];
                        b0 = f0 & int32_t(~kHalfBit);
                        nb = (g.bfirst[v + 1] & int32_t(~kHalfBit)) - b0;
                        half = f0 < 0;
                        if (kExperiments && !CLU && NEAR_LDS && g.hub_blocks > 0 && nb >= g.hub_blocks) {
                            if (lag && !ws.nflag[v]) {  // wait one round: pending again, nothing listed
                                ws.nflag[v] = 1;
                                atomicOr(&near_w[v >> 5], 1u << (v & 31));  // (its word is taken: not seen again this pass)
                                s_anydef = 1;
                                nb = 0;
                            } else if (ws.nflag[v]) {
                                ws.nflag[v] = 0;
                            }
                        }
                        if (nb > 0) s_anyv = 1;
                        half = half && nb > 0;
                        DIAG_LOCAL(if (nb > 0) { ++d_scan; if (g.rowptr[v + 1] - g.rowptr[v] >= 64) ++d_hubexp; })
                    }
                    append_items(v, nb - (half ? 1 : 0), [&](int32_t c) { return make_int4(v, b0 + c, kChunk, 0); });
                    append_pairs(v, half, b0 + nb - 1);
                };
                if constexpr (CLU) {
                    if (c_near) {  // own words (w % cl == cr) of the OR of the published bitmaps
                        const int p = (cgen - 1) & 1;
                        compact_map((WN - cr + cl - 1) / cl, [&](int32_t t) { return t * cl + cr; }, VPWN,
                                    [&](int32_t wi) -> uint32_t {
                                        uint32_t x = 0u;
                                        for (int r = 0; r < cl; ++r) x |= plane(p, r)[wi];
                                        return x;
                                    }, emit_items);
                    }
                } else {
                    compact_words(0, WN, VPWN, [&](int32_t wi) { return take_word(near_w, wi, NearL{}); }, emit_items);
                }
                __syncthreads();
                if (!(lag && s_anyv == 0 && s_anydef != 0)) break;
                lag = false;  // only waiting hubs were pending: list them now
            }
            int32_t nitems = s_nitems, npairs = s_npairs;
            if (int64_t(nitems) + npairs > icap) {  // (bounded by the graph's block count; never taken)
                if (tid == 0) atomicOr(arena.err, 2);
                nitems = npairs = 0;
            }
            DIAG_LOCAL(d_p1 += DIAG_NOW() - d_p1s; if (tid == 0) d_items += nitems;)

            const bool any_near = CLU ? c_near : s_anyv != 0;
            if (!any_near) {
                // ================= drain: near set empty -> raise the threshold
                DIAG_LOCAL(++d_drains; const unsigned long long d_dr0 = DIAG_NOW();)
                if (CLU ? !c_far : !s_far_flag) break;  // nothing pending at all: bucket done
                const double thr_old = thr;
                thr = thr_old + delta;
                bool finished = false;
                for (int pass = 0; pass < 2; ++pass) {
                    __syncthreads();
                    if (tid == 0) { s_moved = 0; s_far_flag = 0; s_minfar = key_enc(__builtin_inf()); }
                    __syncthreads();
                    unsigned long long lane_minfar = key_enc(__builtin_inf());  // smallest kept key seen by this lane
                    for (int32_t wb = wave * 64; wb < WF; wb += NT) {
                        const int32_t wi = wb + lane;
                        uint32_t bits = (wi < WF) ? take_word(far_w, wi, FarL{}) : 0u;
                        while (__any(bits != 0)) {  // 64 far vertices of this wave at a time
                            const bool f = bits != 0;
                            const unsigned long long bal = __ballot(f);
                            if (f) {
                                s_vlist[wave][__popcll(bal & ((1ull << lane) - 1ull))] = wi * VPWF + __builtin_ctz(bits);
                                bits &= bits - 1;
                            }
                            const int cnt = __popcll(bal);
                            wave_sync();
                            // up to kDrainU rows per sub-group in flight (one latency per batch)
#ifndef SHDR_DRAIN_U
#define SHDR_DRAIN_U 8
#endif
                            constexpr int kDrainU = SHDR_DRAIN_U;
                            const unsigned long long sub_mask = (K == 64 ? ~0ull : ((1ull << K) - 1ull)) << sbase;
                            for (int r0 = 0; r0 < cnt; r0 += G * kDrainU) {
                                int32_t uu[kDrainU];
                                double kv[kDrainU];
#pragma unroll
                                for (int u = 0; u < kDrainU; ++u) {
                                    const int idx = r0 + u * G + sub;
                                    uu[u] = (idx < cnt) ? s_vlist[wave][idx] : -1;
                                    const double x = ddec(ld_u64_sc1(&ws.dist[SIDX(max(uu[u], 0), l)]), par);
                                    kv[u] = uu[u] >= 0 ? x : __builtin_inf();
                                }
#pragma unroll
                                for (int u = 0; u < kDrainU; ++u) {
                                    DIAG_LOCAL(if (l == 0 && uu[u] >= 0) ++d_drow;)
                                    const double key = kv[u] - off;
                                    // keys below thr_old were relaxed at their current value
                                    const bool now = uu[u] >= 0 && key >= thr_old && key < thr;
                                    const bool keep = uu[u] >= 0 && key >= thr && key < __builtin_inf();
                                    const unsigned long long bn = __ballot(now) & sub_mask;
                                    const unsigned long long bk = __ballot(keep) & sub_mask;
                                    if (keep) lane_minfar = min(lane_minfar, key_enc(key));
                                    if (l == 0 && uu[u] >= 0) {
                                        if (bn) { mark(true, uu[u]); s_moved = 1; }
                                        if (bk) { mark(false, uu[u]); s_far_flag = 1; }
                                    }
                                }
                            }
                            wave_sync();
                        }
                    }
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) lane_minfar = min(lane_minfar, (unsigned long long)__shfl_xor(lane_minfar, o));
                    if (lane == 0 && lane_minfar != key_enc(__builtin_inf())) atomicMin(&s_minfar, lane_minfar);
                    __syncthreads();
                    int moved = s_moved, farf = s_far_flag;
                    unsigned long long mfar = s_minfar;
                    if constexpr (CLU) {  // the decisions over the cluster
                        const int p = cgen & 1;
                        if (tid == 0) {
                            crec->val[p][cr].moved = uint32_t(s_moved);
                            crec->val[p][cr].any_far = uint32_t(s_far_flag);
                            crec->val[p][cr].minfar = s_minfar;
                        }
                        if (!cbar()) return;
                        moved = 0; farf = 0;
                        for (int r = 0; r < cl; ++r) {
                            moved |= int(crec->val[p][r].moved);
                            farf |= int(crec->val[p][r].any_far);
                            mfar = min(mfar, crec->val[p][r].minfar);
                        }
                    }
                    if (moved) break;
                    if (!farf) { finished = true; break; }
                    thr = key_dec(mfar) + delta;  // first pass saw every far lane: jump past the gap
                }
                __syncthreads();
                DIAG_LOCAL(d_drt += DIAG_NOW() - d_dr0;)
                if (finished) break;
                continue;
            }

            // ================= phase 2: relax the arcs of every item, then every pair
            relax_items(nitems, gsub, NSUB, thr, off, std::false_type{});
            if (npairs > 0) relax_items(npairs, gsub, NSUB, thr, off, std::true_type{});
            __syncthreads();
        }
        // distances are final: drop this CU's L1 copies once, then plain loads are safe
        if constexpr (CLU) {
            if (!cbar()) return;
        } else {
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
        }
#ifdef SHDR_VERIFY
        // verify flavour (never the product): the relaxation's postconditions, checked
        // after it with the product's timing up to here. 128: a pending word left set
        // (this member's near words in LDS, its far words); 512: an arc that still
        // improves its head (dist[h] > fl(dist[v] + w): a relaxation was lost).
        {
            for (int32_t k = tid; k < WNall && NEAR_LDS; k += NT)
                if (near_w[k]) guard_record(arena.err, 128, b, cr, 0, k, int(near_w[k]), rounds, 0, 0, 0);
            const int32_t WFall = FAR_LDS ? WNall : (V + 3) / 4;
            for (int32_t k = tid; k < WFall; k += NT) {
                const uint32_t x = FAR_LDS ? far_w[k] : ld_u32(&far_w[k]);
                if (x) guard_record(arena.err, 128, b, cr, 1, k, int(x), rounds, 0, 0, 0);
            }
            for (int32_t v = cr * NT + tid; v < V; v += cl * NT) {
                for (int32_t ln = 0; ln < nsrc; ++ln) {
                    const double dv = ddec(ld_u64_sc1(&ws.dist[SIDX(v, ln)]), par);
                    if (!(dv < __builtin_inf())) continue;
                    for (int32_t a = g.rowptr[v]; a < g.rowptr[v + 1]; ++a) {
                        const int32_t h = g.col[a];
                        const double c = dv + g.w[a];
                        const double dh = ddec(ld_u64_sc1(&ws.dist[SIDX(h, ln)]), par);
                        if (dh > c)
                            guard_record(arena.err, 512, b, cr, ln, v, h, rounds, int(as_u64(dv) >> 32),
                                         int(as_u64(dh) >> 32), int(as_u64(c) >> 32));
                    }
                }
            }
            __syncthreads();
        }
#endif
        // cluster: the predecessor pass and the epilogue split over cl * NSUB sub-groups
        const int32_t NSUBC = CLU ? cl * NSUB : NSUB;
        const int32_t gsubc = CLU ? cr * NSUB + gsub : gsub;
        DIAG_LOCAL(unsigned long long d_t2 = DIAG_NOW();)

        // ================= predecessor pass: minimum-index tight in-arc, bitwise test
        // The in-CSR is cut into items of <= kChunk in-arcs (static list, graph
        // order); each sub-group owns a contiguous, vertex-aligned range of a list
        // of such items, so a vertex's minimum-index tight arc is found by one
        // sub-group walking its arcs in order. Pipelined like phase 2: rows of item
        // k+1, arc data of item k+2 and the descriptor of item k+3 are in flight
        // while item k is compared.
        //   * full pass: the static list of every vertex's items;
        //   * chain pass (few targets, pending bitmaps in LDS): only the vertices the
        //     epilogue will walk — the targets, then level by level the predecessors
        //     found so far (any lane) — so in-arcs of vertices on no target's chain
        //     are never read.
        // chain pass sets: one bit per vertex, "to do" and "done" (the LDS pending
        // bitmaps, or the slot's pending bytes read as bitmaps; all empty after the
        // relaxation)
        uint32_t* q_todo = near_w;
        uint32_t* q_done = FAR_LDS ? far_w : reinterpret_cast<uint32_t*>(ws.fflag);
        auto mark_todo = [&](int32_t u) {
            const uint32_t bit = 1u << (u & 31);
            if (q_done[u >> 5] & bit) return;
            if constexpr (NEAR_LDS) atomicOr(&q_todo[u >> 5], bit);
            else __hip_atomic_fetch_or(&q_todo[u >> 5], bit, __ATOMIC_RELAXED, SLOT_SCOPE);
        };
        // sub-group gs of ns walks its share of the list
        auto pred_list = [&](const int4* __restrict__ lst, const int32_t n, const bool mark_preds, const int32_t gs,
                             const int32_t ns) {
            auto item = [&](int32_t i) -> int4 { return ldk_i4(&lst[i]); };
            auto vertex_start = [&](int32_t i) {  // first item >= i that opens a vertex
                while (i < n && !(item(i).w & 1)) ++i;
                return i;
            };
            const int32_t lo = vertex_start(int32_t(int64_t(n) * gs / ns));
            const int32_t hi = vertex_start(int32_t(int64_t(n) * (gs + 1) / ns));
            int32_t witers = hi - lo;
#pragma unroll
            for (int o = K; o < 64; o <<= 1) witers = max(witers, __shfl_xor(witers, o));
            witers = __builtin_amdgcn_readfirstlane(witers);
            auto desc = [&](int32_t k) -> int4 {  // unconditional load, then select (see phase 2)
                const int4 x = item(IIDX(max(0, min(lo + k, n - 1))));
                return lo + k < hi ? x : make_int4(0, 0, 0, 0);
            };
            int4 d0 = desc(0), d1 = desc(1), d2 = desc(2), d3;
            // lane q of a sub-group holds in-arc q of the item: source, weight and
            // reliability factor (stored with the predecessor, so the epilogue's
            // walk reads one 16-B entry per hop and no arc array)
            int32_t su0, su1;
            double sw0, sw1, dv0, dv1;
            {
                const int ai = (l < d0.z) ? d0.y + l : 0;
                const int32_t xa = ldk_i32(&g.isrc[AIDX(ai)]);
                const double wa = ldk_f64(&g.iw[AIDX(ai)]);
                su0 = (l < d0.z) ? xa : d0.x;
                sw0 = (l < d0.z) ? wa : __builtin_inf();
                dv0 = ddec(ws.dist[SIDX(d0.x, l)], par);
                const int bi = (l < d1.z) ? d1.y + l : 0;
                const int32_t xb = ldk_i32(&g.isrc[AIDX(bi)]);
                const double wb = ldk_f64(&g.iw[AIDX(bi)]);
                su1 = (l < d1.z) ? xb : d1.x;
                sw1 = (l < d1.z) ? wb : __builtin_inf();
                dv1 = ddec(ws.dist[SIDX(d1.x, l)], par);
            }
            // Tie rule (igraph's strict-'<' Dijkstra keeps the first tight relaxation
            // in pop order, i.e. the tight predecessor with the smallest distance):
            // the tight in-arc with the smallest dist[u], then the lowest in-arc
            // index. Once a lane holds a tight arc (bestd, w_best), an arc whose
            // weight is below w_best - eps (eps >= 2 ulp(dist[v])) cannot be tight
            // with dist[u'] <= bestd, so its row is not needed by that lane: a row
            // load is skipped when every lane of the sub-group can skip it. The
            // state used for item k+1's loads is one item old, which only makes the
            // test more conservative (bestd never grows); at a vertex's first item
            // (d0 or d1 opening a vertex) every real arc is loaded.
            double r0[kChunk];
            sfor<kChunk>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                // a skipped row reads the item's own vertex row instead (already in
                // L1: no new line), and the value is discarded
                const int32_t uq = sub_lane32<K, q>(su0, lane, sbase);
                const double x = ddec(ld_u64_sc1(&ws.dist[SIDX(q < d0.z ? uq : d0.x, l)]), par);
                r0[q] = q < d0.z ? x : __builtin_inf();
            });
            int2 best = make_int2(-1, -1);
            bool need = false;
            double bestd = __builtin_inf(), wthr = -__builtin_inf();
            for (int32_t k = 0; k < witers; ++k) {
                double r1[kChunk];
                const bool fresh = (d0.w & 1) || (d1.w & 1);
                sfor<kChunk>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    const int32_t uq = sub_lane32<K, q>(su1, lane, sbase);
                    const double wq = as_f64(sub_lane64<K, q>(as_u64(sw1), lane, sbase));
                    const bool ld = q < d1.z && (fresh || (need && wq >= wthr));
                    const double x = ddec(ld_u64_sc1(&ws.dist[SIDX(ld ? uq : d1.x, l)]), par);
                    r1[q] = ld ? x : __builtin_inf();
                });
                const int ci = (l < d2.z) ? d2.y + l : 0;
                const int32_t xc = ldk_i32(&g.isrc[AIDX(ci)]);
                const double wc = ldk_f64(&g.iw[AIDX(ci)]);
                const int32_t su2 = (l < d2.z) ? xc : d2.x;
                const double sw2 = (l < d2.z) ? wc : __builtin_inf();
                const double dv2 = ddec(ws.dist[SIDX(d2.x, l)], par);
                d3 = desc(k + 3);
                if (d0.w & 1) {  // first item of vertex d0.x
                    best = make_int2(-1, -1);
                    need = dv0 != __builtin_inf() && d0.x != my_src;
                    bestd = __builtin_inf();
                    wthr = -__builtin_inf();
                }
                sfor<kChunk>([&](auto qc) {
                    constexpr int q = decltype(qc)::value;
                    const double wq = as_f64(sub_lane64<K, q>(as_u64(sw0), lane, sbase));
                    const double c = r0[q] + wq;
                    const int32_t uq = sub_lane32<K, q>(su0, lane, sbase);
                    if (need && c == dv0 && r0[q] < bestd) {
                        best = make_int2(uq, d0.y + q);
                        bestd = r0[q];
                        wthr = wq - dv0 * 0x1p-50;
#ifdef SHDR_TIE_INDEX_ONLY  // experiments only: the round-1 rule (first tight arc in index order)
                        need = false;
#endif
                    }
                });
                if (d0.w & 2) {  // last item of the vertex
                    ws.pred[SIDX(d0.x, l)] = best;
                    if (mark_preds && best.x >= 0) mark_todo(best.x);
                }
#pragma unroll
                for (int q = 0; q < kChunk; ++q) r0[q] = r1[q];
                su0 = su1; sw0 = sw1; dv0 = dv1;
                d0 = d1; d1 = d2; d2 = d3;
                su1 = su2; sw1 = sw2; dv1 = dv2;
            }
        };
        // (cluster mode with the far set in slot bytes, PM 1, always runs the full pass:
        // its chain pass lost level >= 1 vertices in the round-4 build)
        const bool chain_pass = !(keep_slots & 1) && g.pfirst && int64_t(out.T) * 2 <= V && !(CLU && PM == 1);
        const int32_t WQ = (V + 31) / 32;
        if ((keep_slots & 8) || DIAG_SKIP(keep_slots & 2)) {  // distances only: no predecessors
        } else if (!chain_pass) {
            pred_list(g.pitems, g.npitems, false, gsubc, NSUBC);
        } else {
            // cluster: to-do marks are published like the near set; the owner of a
            // word (w % cl) keeps its done bits and expands its to-do vertices
            for (int32_t j = cr * NT + tid; j < out.T; j += cl * NT) mark_todo(dst[j]);
            __syncthreads();  // (cluster: every target's mark lands before the words are published)
            for (;;) {
                if constexpr (CLU) {
                    const int p = cgen & 1;
                    uint32_t* pl = plane(p, cr);
                    int anyt = 0;
                    for (int32_t k = tid; k < WQ; k += NT) {
                        const uint32_t x = q_todo[k];
                        pl[k] = x;
                        if (x) { q_todo[k] = 0u; anyt = 1; }
                    }
                    anyt = __syncthreads_or(anyt);
                    if (tid == 0) crec->val[p][cr].any_near = uint32_t(anyt);
                    if (!cbar()) return;
                    uint32_t an = 0;
                    for (int r = 0; r < cl; ++r) an |= crec->val[p][r].any_near;
                    if (!an) break;
                }
                if (tid == 0) s_nitems = 0;
                __syncthreads();
                // level list: the to-do vertices not yet done
                auto emit_pitems = [&](int32_t v) {
                    int32_t p0 = 0, np = 0;
                    if (v >= V) {  // (a to-do bit past the last vertex: never set)
                        guard_record(arena.err, 2048, b, cr, v, V, 1, 0, 0, 0, 0);
                        v = -1;
                    }
                    if (v >= 0) { p0 = g.pfirst[v]; np = g.pfirst[v + 1] - p0; }
                    append_items(v, np, [&](int32_t c) { return g.pitems[p0 + c]; });
                };
                if constexpr (CLU) {
                    const int p = (cgen - 1) & 1;
                    compact_map((WQ - cr + cl - 1) / cl, [&](int32_t t) { return t * cl + cr; }, 32,
                                [&](int32_t wi) -> uint32_t {
                                    uint32_t x = 0u;
                                    for (int r = 0; r < cl; ++r) x |= plane(p, r)[wi];
                                    const uint32_t bits = x & ~q_done[wi];
                                    q_done[wi] |= bits;
                                    return bits;
                                }, emit_pitems);
                } else {
                    compact_words(0, WQ, 32, [&](int32_t wi) -> uint32_t {
                        uint32_t x;
                        if constexpr (NEAR_LDS) x = q_todo[wi];
                        else x = ld_u32(&q_todo[wi]);  // set by atomics of other waves
                        if (!x) return 0u;
                        q_todo[wi] = 0u;
                        const uint32_t bits = x & ~q_done[wi];
                        q_done[wi] |= bits;
                        return bits;
                    }, emit_pitems);
                }
                __syncthreads();
                const int32_t nl = s_nitems;
                if (!CLU && nl == 0) break;
                // (cluster: a member with an empty level still takes the barriers above)
                if (nl > 0) pred_list(ws.items, nl, true, gsub, NSUB);
                __syncthreads();
            }
            if constexpr (!FAR_LDS)  // give the pending bytes back all-zero
                for (int32_t k = tid; k < WQ; k += NT) q_done[k] = 0u;
        }
        if constexpr (CLU) {  // every member's predecessor entries before the walks
            if (!cbar()) return;
        } else {
            __syncthreads();
        }
        DIAG_LOCAL(unsigned long long d_t3 = DIAG_NOW();)

        // ================= epilogue: ordered walk per (source lane, target)
        // Lane l of a sub-group walks source lane l's chain to the sub-group's
        // target: the K sources of a bucket are grouped to be close, so near the
        // target their chains share vertices and the K predecessor reads of one
        // hop mostly hit the same row.
        if (tid < K) s_rowmin_l[tid] = key_enc(__builtin_inf());
        __syncthreads();
        if (l < nsrc) {
            const int32_t ls = l;
            const int32_t s = src[i0 + ls];
            const int32_t orow = out.rowmap ? out.rowmap[i0 + ls] : i0 + ls;
            double rowmin = __builtin_inf();
            const double rs = g.vrel[s];
            // NCH targets per lane at a time (j, j + NSUB, ...): their chains are walked
            // in lockstep, so each step has NCH independent predecessor loads in flight
            // (the walk is a chain of dependent loads, latency-bound otherwise)
            for (int32_t j0 = gsubc; j0 < out.T && !DIAG_SKIP(keep_slots & 4); j0 += NCH * NSUBC) {
                int32_t tc[NCH], vc[NCH], hc[NCH];
                double dtc[NCH], latc[NCH], relc[NCH];
                bool walk[NCH];
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    const int32_t j = j0 + c * NSUBC;
                    latc[c] = __builtin_nan(""); relc[c] = __builtin_nan("");
                    hc[c] = -1; walk[c] = false; dtc[c] = __builtin_inf();
                    tc[c] = j < out.T ? dst[j] : -1;
                    vc[c] = tc[c];
                    const int32_t t = tc[c];
                    if (t < 0) continue;
                    if (t == s && g.fold_add) {
                        latc[c] = 5.0; relc[c] = 0.0; hc[c] = 0;  // compute-topology-paths.py:24-26
                    } else if (t == s) {
                        // igraph returns the one-vertex path [s]: the self-loop edge, no dst loss (:709-711)
                        const double sl = g.self_lat[t];
                        if (sl == sl) {
                            double lat = 0.0; lat += sl;
                            double rel = 1.0; rel *= rs; rel *= g.self_rel[t];
                            if (lat == 0.0) lat = 1.0;
                            latc[c] = lat; relc[c] = rel; hc[c] = 1;
                        }
                    } else {
                        dtc[c] = ddec(ws.dist[SIDX(t, ls)], par);
                        if (dtc[c] != __builtin_inf()) { walk[c] = true; hc[c] = 0; }
                    }
                }
                // walk back to the source, recording the in-arcs of the first kStack hops
                // (counted from t) in this chain's LDS stack; count all hops
                for (;;) {
                    bool any = false;
#pragma unroll
                    for (int c = 0; c < NCH; ++c) any |= walk[c];
                    if (!any) break;
                    int2 pr[NCH];
#pragma unroll
                    for (int c = 0; c < NCH; ++c) {  // unconditional loads: both chains in flight together
                        const int2 x = ldk_i2(&ws.pred[SIDX(walk[c] ? vc[c] : s, ls)]);
                        pr[c] = walk[c] ? x : make_int2(0, 0);
                    }
#pragma unroll
                    for (int c = 0; c < NCH; ++c) {
                        if (!walk[c]) continue;
                        if (hc[c] < kStack) s_stack[(c * kStack + hc[c]) * NT + tid] = uint32_t(pr[c].y);
                        ++hc[c];
                        const int32_t vfrom = vc[c];
                        vc[c] = pr[c].x;
#if defined(SHDR_BCHK) || defined(SHDR_VERIFY)
                        if (vc[c] == -2) guard_record(arena.err, 32, b, cr, ls, tc[c], vfrom, pr[c].x, pr[c].y, hc[c], 0);
#endif
                        if (vc[c] < 0 || vc[c] >= V || uint32_t(pr[c].y) >= uint32_t(g.A) || hc[c] > V) {
                            // (a broken chain is reported, never followed out of range)
                            if (vc[c] >= 0)
                                guard_record(arena.err, 4, b, cr, ls, tc[c], vfrom, pr[c].x, pr[c].y, hc[c],
                                             int(as_u64(ddec(ws.dist[SIDX(vfrom, ls)], par)) >> 32));
                            hc[c] = -1; walk[c] = false;
                        } else if (vc[c] == s) {
                            walk[c] = false;
                        }
                    }
                }
                // fold in path order (source side first) for the chains that fit their
                // stacks: the factor gathers of all chains are in flight together
                double relf[NCH];
                int32_t kk[NCH];
                bool fast[NCH];
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    fast[c] = tc[c] >= 0 && tc[c] != s && hc[c] > 0 && hc[c] <= kStack;
                    relf[c] = fast[c] ? (g.fold_add ? 0.0 : (1.0 * rs) * g.vrel[tc[c]]) : 0.0;
                    kk[c] = fast[c] ? hc[c] - 1 : -1;
                }
                for (;;) {
                    bool any = false;
#pragma unroll
                    for (int c = 0; c < NCH; ++c) any |= kk[c] >= 0;
                    if (!any) break;
                    double f[NCH][4];
#pragma unroll
                    for (int c = 0; c < NCH; ++c)
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                        {  // unconditional gathers (a finished chain reads factor 0, discarded)
                            const uint32_t ai = kk[c] - u >= 0 ? s_stack[(c * kStack + max(kk[c] - u, 0)) * NT + tid] : 0u;
                            const double x = ldk_f64(&g.icrel[AIDX(ai)]);
                            f[c][u] = kk[c] - u >= 0 ? x : 0.0;
                        }
#pragma unroll
                    for (int c = 0; c < NCH; ++c) {
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (kk[c] - u >= 0) {
                                if (g.fold_add) relf[c] += f[c][u]; else relf[c] *= f[c][u];
                            }
                        kk[c] -= 4;
                    }
                }
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    const int32_t t = tc[c], h = hc[c];
                    if (t < 0 || t == s || h <= 0) continue;
                    uint32_t* stk = s_stack + size_t(c) * kStack * NT + tid;
                    double lat = 0.0;
                    // reliability: ((1 * (1-p_s)) * (1-p_t)) * factors; jitter: 0 + ...
                    double rel = relf[c];
                    if (h > kStack) {
                        // longer than the stack: fold in path order (source side first),
                        // kStack hops at a time, re-walking for each chunk
                        rel = g.fold_add ? 0.0 : (1.0 * rs) * g.vrel[t];
                        for (int32_t hi = h; hi > 0; hi -= kStack) {
                            const int32_t lo = max(0, hi - kStack);  // hops [lo, hi) counted from t
                            if (h > kStack) {
                                int32_t vv = t;
                                for (int32_t k = 0; k < hi; ++k) {
                                    const int2 pr = ws.pred[SIDX(vv, ls)];
                                    if (k >= lo) stk[(k - lo) * NT] = uint32_t(pr.y);
                                    vv = pr.x;
                                }
                            }
                            int32_t k = hi - lo - 1;
                            for (; k >= 3; k -= 4) {
                                const double f0 = g.icrel[AIDX(stk[k * NT])], f1 = g.icrel[AIDX(stk[(k - 1) * NT])];
                                const double f2 = g.icrel[AIDX(stk[(k - 2) * NT])], f3 = g.icrel[AIDX(stk[(k - 3) * NT])];
                                if (g.fold_add) { rel += f0; rel += f1; rel += f2; rel += f3; }
                                else { rel *= f0; rel *= f1; rel *= f2; rel *= f3; }
                            }
                            for (; k >= 0; --k) {
                                const double f = g.icrel[AIDX(stk[k * NT])];
                                if (g.fold_add) rel += f; else rel *= f;
                            }
                        }
                    }
                    if (g.fold_add) rel /= double(h);  // sum(j) / float(len(j))
                    if (!g.lat_is_w) {
                        // multigraph whose parallel edges differ in latency: the
                        // epilogue's canonical latencies are summed in path order
                        // (rare; quadratic re-walk, no stack)
                        for (int32_t k = h - 1; k >= 0; --k) {
                            int32_t vv = t;
                            for (int32_t i = 0; i < k; ++i) vv = ws.pred[SIDX(vv, ls)].x;
                            lat += g.iclat[AIDX(ws.pred[SIDX(vv, ls)].y)];
                        }
                    }
                    // every arc's weight is its canonical edge's latency: the
                    // distance IS the left-to-right latency sum along this chain
                    // (each hop is tight bitwise), so the sum is not redone
                    if (g.lat_is_w) lat = dtc[c];
                    if (lat == 0.0 && !g.fold_add) lat = 1.0;  // :760-765
                    latc[c] = lat; relc[c] = rel;
                    DIAG_LOCAL(d_walk += h;)
                }
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    const int32_t j = j0 + c * NSUBC;
                    if (j >= out.T) continue;
                    const size_t o = size_t(orow) * out.T + j;
                    out.lat[o] = latc[c];
                    out.rel[o] = relc[c];
                    if (out.hops) out.hops[o] = hc[c];
                    if (latc[c] < rowmin) rowmin = latc[c];  // NaN (no path) never counts
                }
            }
            if (rowmin < __builtin_inf()) atomicMin(&s_rowmin_l[ls], key_enc(rowmin));
        }
        __syncthreads();
        if constexpr (CLU) {  // the row minima over the members, written by the leader
            if (tid < K) crec->rowmin[cr][tid] = s_rowmin_l[tid];
            if (!cbar()) return;
            if (cr == 0 && out.row_min && tid < nsrc) {
                unsigned long long m = crec->rowmin[0][tid];
                for (int r = 1; r < cl; ++r) m = min(m, crec->rowmin[r][tid]);
                out.row_min[out.rowmap ? out.rowmap[i0 + tid] : i0 + tid] = key_dec(m);
            }
            if (cr == 0 && out.bcost && tid == 0) out.bcost[b] = uint32_t(__builtin_amdgcn_s_memrealtime() - tb0);
        } else {
            if (out.row_min && tid < nsrc)
                out.row_min[out.rowmap ? out.rowmap[i0 + tid] : i0 + tid] = key_dec(s_rowmin_l[tid]);
            if (out.bcost && tid == 0) out.bcost[b] = uint32_t(__builtin_amdgcn_s_memrealtime() - tb0);
        }
        // the slot's row state for its next bucket: parity + 1 when every (vertex,
        // lane) word was written with this bucket's parity, else 0 (fill next time)
        if (tid == 0 && cr == 0) ws.nflag[V + 8] = (nofill_ok && nsrc == K) ? uint8_t(par + 1) : uint8_t(0);
        if (out.done) {
            // progressive host copy (host outputs): every store of this bucket has
            // landed, the L2 is written back (system-scope release), then the
            // bucket's flag in host memory; the host copies finished rows while the
            // launch runs on
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0 && cr == 0) {
                __threadfence_system();
                __hip_atomic_store(&out.done[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        __syncthreads();
#ifdef SHDR_DIAG
        {
            unsigned long long d_t4 = DIAG_NOW();
            if (tid == 0) {
                DIAG_ADD(0, d_t1 - d_t0); DIAG_ADD(1, d_t2 - d_t1); DIAG_ADD(2, d_p1); DIAG_ADD(3, d_t3 - d_t2);
                DIAG_ADD(4, d_t4 - d_t3); DIAG_ADD(5, d_rounds); DIAG_ADD(6, d_drains); DIAG_ADD(8, d_items);
                DIAG_ADD(13, 1);
            }
            if (tid == 0 && nbuckets > 300 && b < 8192) { g_bticks[0][b] = d_t0; g_bticks[1][b] = d_t4 - d_t0; }
            DIAG_ADD(7, d_scan); DIAG_ADD(9, d_arcs); DIAG_ADD(10, d_atom); DIAG_ADD(11, d_imp); DIAG_ADD(12, d_walk);
            DIAG_ADD(14, d_ev); DIAG_ADD(15, d_drow); DIAG_ADD(17, d_act);
            // per-degree counters (permanent diagnostic output, tools/diag.py): head rows
            // read, of them by vertices of degree >= 64, expansions of such vertices,
            // close rounds and close-round items
            DIAG_ADD(18, d_rows); DIAG_ADD(19, d_hubrows); DIAG_ADD(25, d_hubexp);
            if (tid == 0) DIAG_ADD(16, d_drt);
            // cluster barriers of this member and their ticks (lane 0's arrive-to-acquire)
            if (tid == 0 && CLU) { DIAG_ADD(26, d_cbn); DIAG_ADD(27, d_cbt); d_cbn = d_cbt = 0; }
        }
#endif
    }
}

// The route-table kernel, its half-width tail launch and the landmark pre-pass
// (order_sources) share one body; separate symbols keep them apart in profiles.
template <int K, int NT, int PM, bool CLU = false>
__global__ void __launch_bounds__(NT, min_waves_per_eu(NT)) k_routes_sssp(DevGraph g, SlotArena arena, const int32_t* src,
                                                                  int32_t S, const int32_t* dst, int32_t nbuckets,
                                                                  double delta, RouteOut out, int keep_slots) {
    __shared__ Smem<NT, PM> sm;
    sssp_body<K, NT, PM, CLU>(g, arena, src, S, dst, nbuckets, delta, out, keep_slots, sm);
}
template <int K, int NT, int PM>
__global__ void __launch_bounds__(NT, min_waves_per_eu(NT)) k_routes_sssp_tail(DevGraph g, SlotArena arena, const int32_t* src,
                                                                       int32_t S, const int32_t* dst, int32_t nbuckets,
                                                                       double delta, RouteOut out, int keep_slots) {
    __shared__ Smem<NT, PM> sm;
    sssp_body<K, NT, PM>(g, arena, src, S, dst, nbuckets, delta, out, keep_slots, sm);
}
template <int K, int NT, int PM>
__global__ void __launch_bounds__(NT, min_waves_per_eu(NT)) k_landmarks_sssp(DevGraph g, SlotArena arena, const int32_t* src,
                                                                     int32_t S, const int32_t* dst, int32_t nbuckets,
                                                                     double delta, RouteOut out, int keep_slots) {
    __shared__ Smem<NT, PM> sm;
    sssp_body<K, NT, PM>(g, arena, src, S, dst, nbuckets, delta, out, keep_slots, sm);
}
// One table pass in ONE launch (the default layout when the last wave of full-width
// buckets is at most half full): blocks [0, tail.blocks) first run the partial last
// wave's sources as half-width buckets in their own arena region (their own ticket),
// then every block draws full-width buckets from the main queue. The tail's CU share
// is fixed by block index, not by which of two concurrent launches the hardware
// dispatches first (Tail balancing).
struct TailArgs {
    SlotArena arena;
    const int32_t* src;
    int32_t S, nbuckets, blocks;
    RouteOut out;
};
template <int K, int NT, int PM>
__global__ void __launch_bounds__(NT, min_waves_per_eu(NT)) k_routes_pass(DevGraph g, SlotArena arena, const int32_t* src,
                                                                  int32_t S, const int32_t* dst, int32_t nbuckets,
                                                                  double delta, RouteOut out, int keep_slots,
                                                                  TailArgs tail) {
    __shared__ Smem<NT, PM> sm;
    // Two inlined copies of the full-width body: one after the tail buckets, one for
    // the blocks without tail work. With a single copy behind the tail body, values
    // live across both bodies pushed extra spills into the main body's predecessor
    // and epilogue loops (+1.3 % on cfg5); the blocks that never run tail buckets now
    // get the same code as k_routes_sssp (Register spills).
    if (int32_t(blockIdx.x) >= tail.blocks) {
        sssp_body<K, NT, PM>(g, arena, src, S, dst, nbuckets, delta, out, keep_slots, sm);
        return;
    }
    sssp_body<K / 2, NT, PM>(g, tail.arena, tail.src, tail.S, dst, tail.nbuckets, delta, tail.out, keep_slots, sm);
    sssp_body<K, NT, PM>(g, arena, src, S, dst, nbuckets, delta, out, keep_slots, sm);
}

}  // namespace

// ==================================================================== engine
namespace {
// (bucket width K, workgroup threads) instantiations of k_routes_sssp
struct Variant { int K, NT; };
constexpr Variant kVariants[] = {{8, 256}, {16, 256}, {16, 512}, {32, 512}, {16, kNT}, {8, 512}, {8, kNT}, {32, kNT}};
constexpr int kDefaultVariant = 4;
}  // namespace

struct shdr_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    shdr::CsrImage csr;  // in device numbering (see relabel_bfs)
    // device numbering: newid[caller vertex], oldid[device vertex]; empty = identity
    std::vector<int32_t> newid, oldid;
    std::vector<int32_t> h_msrc, h_mdst;  // caller's src / dst in device numbering
    int32_t vexp = 0;                     // vertices [vexp, V) are pendant (see DevGraph::vexp)
    bool complete = false;
    bool directed = false;
    double delta = 0.0;  // 0 = auto
    double auto_delta = 1.0;  // see auto_delta()
    int variant = kDefaultVariant;
    // graph buffers
    int32_t *rowptr = nullptr, *col = nullptr, *irowptr = nullptr, *isrc = nullptr;
    double *w = nullptr, *oclat = nullptr, *ocrel = nullptr, *iw = nullptr, *iclat = nullptr, *icrel = nullptr;
    double *vrel = nullptr, *self_lat = nullptr, *self_rel = nullptr;
    double *ocjit = nullptr, *icjit = nullptr;  // uploaded on the first SHDR_PATH_JITTER compute
    int4* pitems = nullptr;
    int32_t* pfirst = nullptr;
    int32_t npitems = 0;
    uint64_t *ablk = nullptr, *iablk = nullptr;  // packed arc blocks (out; in when directed)
    int32_t *bfirst = nullptr, *ibfirst = nullptr;
    int32_t nblk = 0, inblk = 0;
    // workspace
    char* arena = nullptr;
    size_t arena_bytes = 0;
    char* arena_raw = nullptr;   // the allocation `arena` is aligned within
    size_t arena_align = 0;      // SHDR_ARENA_ALIGN_MB
    int32_t* d_src = nullptr;
    int32_t* d_dst = nullptr;
    size_t cap_src = 0, cap_dst = 0;
    double *d_lat = nullptr, *d_rel = nullptr, *d_rowmin = nullptr;
    size_t cap_rowmin = 0;
    int* d_err = nullptr;
    int32_t* d_hops = nullptr;
    size_t cap_out = 0, cap_hops = 0;
    // landmark pre-pass (source ordering): distance of every vertex from/to the
    // highest-degree vertex, computed once per engine
    bool lm_ready = false;
    bool lm_pending = false;      // enqueued by engine_create, not yet collected
    hipStream_t lm_stream = nullptr;
    void* d_lm = nullptr;         // landmark vertices, then their [L][V] distance embedding
    size_t cap_lm = 0;
    int lm_count = 0;
    std::vector<double> lm_dist;  // [lm_count][V]
    int32_t* d_rowmap = nullptr;
    double* d_soff = nullptr;
    size_t cap_rowmap = 0, cap_soff = 0;
    std::vector<int32_t> h_src_sorted;
    int32_t last_rows_main = 0;  // rows of the last compute's main launch (the rest ran in the tail launch)
    int last_variant = 0;        // variant of the last compute's main launch
    bool last_partial_first = false;
    int order_mode = 1;  // 0 caller order, 1 landmark grouping, 2 grouping + per-lane key offsets
    int bucket_sort = 1;  // issue full buckets longest-first (landmark spread)
    int pending_lds = 2;  // highest pending-set mode allowed (2 both LDS bitmaps, 1 near only, 0 slot bytes)
    int cus = 256;            // compute units of the device
    int64_t slots_cache[16] = {};
    bool flags_dirty = true;  // slot pending bytes need clearing before the next launch
    // arena regions {byte offset, slot stride, slots} whose flag bytes (pending sets,
    // row state) are known valid: a launch over exactly such a region skips the
    // clear, so its slots keep the row state their last bucket left (kNoFill)
    std::vector<std::array<size_t, 4>> clean_regions;  // {offset, stride, slots, K}
    bool reach_all = false;   // strongly connected graph (DevGraph::reach_all)
    std::vector<int32_t> order_key;  // source list of the cached grouping
    // bucket issue order of the cached grouping: kd groups (full K-groups of kd_perm),
    // position -> group; measured main-launch bucket durations per group (-1 unknown)
    std::vector<int32_t> kd_perm, border;
    std::vector<int32_t> gstart;  // kd group g = kd_perm[gstart[g], gstart[g+1])
    int32_t nsorted = 0;          // groups that take part in the issue-order sort (the rest stay last)
    std::vector<float> gcost;
    int balance = 2;              // 1: balanced bucket layout (whole waves of equal buckets, no tail launch);
                                  // 0: full buckets + tail; 2: balanced only below one half-width wave
    int cur_balance = 0;          // the layout of the compute in progress
    int32_t* d_boff = nullptr;    // bucket row offsets of the processed order (balanced layout,
    size_t cap_boff = 0;          // or K-wide groups with the partial one issued first)
    std::vector<int32_t> h_boff;  // host copy of d_boff
    bool partial_first = false;   // K-wide layout whose partial group is issued first
    int32_t ngroups = 0;
    int cluster = 0;              // SHDR_CLUSTER: workgroups per bucket (0 auto, 1 off, n >= 2 forced)
    bool shared_device = false;   // SHDR_ENGINES_SHARE_DEVICES: no automatic cluster mode
    int cur_cl = 1;               // of the compute in progress
    int far_skip = 1;             // SHDR_FAR_SKIP (DevGraph::far_skip)
    int nofill = 1;               // SHDR_NOFILL (experiments flavour): 0 fills every bucket
    int hub_lag = 0;              // SHDR_HUB_LAG: arc blocks from which a vertex waits a round (DevGraph::hub_blocks; 0 off)
    bool half_pairs = true;       // SHDR_HALF_PAIRS (default 1): half blocks relaxed in pairs (kHalfBit)
    // progressive host copy (host outputs of >= prog_min bytes): rows are written in
    // processing order, each bucket flags its completion in host memory, and the host
    // copies finished rows (pinned staging, then a scatter to the caller's rows)
    // while the launch runs
    int progressive = 1;          // SHDR_PROGRESSIVE
    size_t prog_min = size_t(256) << 20, prog_chunk = size_t(512) << 20;  // bytes per array
    uint32_t* h_done = nullptr;   // pinned, mapped: per main-launch bucket
    size_t cap_done = 0;
    double* h_stage = nullptr;    // pinned staging: [2][chunk rows][T] (cap_stage bytes)
    size_t cap_stage = 0;
    hipStream_t stream3 = nullptr;  // copy stream
    bool last_progressive = false;
    int last_fallback = 0;        // guard code (8 / 16) if the last compute fell back from cluster mode, else 0
    int64_t fallbacks = 0;        // such fallbacks over the engine's life
    std::vector<int32_t> h_perm;  // processed source k -> caller row of the last compute (empty: identity)
    int32_t last_S = 0;
    bool last_reordered = false;
    int tail_cl = 1;             // cluster width of its tail launch (1: none)
    bool cluster_tail = false;    // SHDR_CLUSTER_TAIL: the partial last wave as a cluster launch
    char* d_cl = nullptr;         // cluster records, near-set planes, member scratch
    size_t cap_cl = 0;
    bool costs_fresh = false;
    int profile_order = -1;  // SHDR_PROFILE_ORDER: 1 / 0 measured-duration order for repeated source lists on / off; -1 automatic
    int tail_min_waves = 2;  // full waves of buckets before a half-width tail pays (SHDR_TAIL_MIN_WAVES)
    uint32_t* d_bcost = nullptr;
    size_t cap_bcost = 0;
    int32_t cost_buckets = 0;  // main-launch buckets timed by the last compute
    // kept trees
    int kept_K = 0;
    int32_t kept_S = 0;
    size_t kept_stride = 0, kept_off_pred = 0;
    bool kept = false;
    // timing
    hipEvent_t ev[8] = {};
    hipStream_t stream2 = nullptr;  // concurrent tail launch
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_pass = nullptr;
    bool concurrent_tail = true;
    bool tail_first = true;       // SHDR_TAIL_FIRST (default 1): submit the concurrent tail before the main launch
    // SHDR_PASS (default 1): main rows and tail rows in ONE launch (k_routes_pass) where it
    // is built; 0: the two concurrent launches (tail_first) as in round 5
    bool single_pass = true;
    int last_tail_mode = 0;       // 0 no tail, 1 serial tail launch, 2 concurrent tail launch, 3 single launch
    bool tail_concurrent = false;  // the last compute ran its tail concurrently
    std::vector<std::string> tnames;
    std::vector<float> tms;
    // host phases of the last compute (ms): landmark pre-pass, grouping (incl. the
    // pre-pass), launch (uploads, arena, kernel enqueue), pass wait, exposed D2H, total
    double host_ms[6] = {};
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

DevGraph devgraph(const shdr_engine* e, bool jitter = false) {
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
    g.lat_is_w = e->csr.lat_is_w ? 1 : 0;
    g.fold_add = jitter ? 1 : 0;
    if (jitter) {  // the predecessor entries carry the arc's jitter instead of 1 - loss
        g.ocrel = e->ocjit;
        g.icrel = e->csr.same_in_out ? e->ocjit : e->icjit;
    }
    g.pitems = e->pitems;
    g.npitems = e->npitems;
    g.pfirst = e->pfirst;
    g.ablk = e->ablk; g.bfirst = e->bfirst; g.nblk = e->nblk;
    g.vexp = e->vexp;
    g.hub_blocks = e->hub_lag;
    g.far_skip = e->far_skip;
    g.reach_all = (e->reach_all && e->nofill) ? 1 : 0;
    return g;
}


// One instantiation of k_routes_sssp: (bucket width K, workgroup threads NT,
// pending-set storage PM: 2 both LDS bitmaps, 1 near bitmap in LDS, 0 slot bytes).
template <int K, int NT, int PM>
struct Sssp {
    static hipError_t launch(int slots, size_t dyn, hipStream_t st, const DevGraph& g, const SlotArena& ar,
                             const int32_t* src, int32_t S, const int32_t* dst, int32_t nb, double delta,
                             const RouteOut& o, int keep, int role) {
        auto* fn = role == 2 ? &k_landmarks_sssp<K, NT, PM> : role == 1 ? &k_routes_sssp_tail<K, NT, PM>
                                                                         : &k_routes_sssp<K, NT, PM>;
        if (dyn > 0) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, int(dyn));
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(fn, dim3(slots), dim3(NT), dyn, st, g, ar, src, S, dst, nb, delta, o, keep);
        return hipGetLastError();
    }
    static int occupancy(size_t dyn) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_routes_sssp<K, NT, PM>, NT, dyn) != hipSuccess) return 1;
        return std::max(1, n);
    }
    static size_t static_lds() {
        hipFuncAttributes a{};
        if (hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&k_routes_sssp<K, NT, PM>)) != hipSuccess) return 0;
        return a.sharedSizeBytes;
    }
};

// Cluster-mode instantiation (k_routes_sssp<K, NT, PM, true>): the 1024-thread
// variants with the near set in LDS.
template <int K, int NT, int PM>
struct SsspC {
    // A plain launch on the engine's stream, so it starts only after the
    // stream's earlier copies and memsets (sorted sources, guard word and tickets,
    // zeroed cluster records) have landed. The grid is sized from the occupancy
    // (cluster_slots) so every member can be resident; a member that is not (the
    // device is shared) shows as a barrier timeout and the host recomputes without
    // clusters. Round 3 launched clusters with hipLaunchCooperativeKernel; whether
    // that path waits for the stream's earlier copies and memsets is checked by
    // tools/coop_order.hip, and cooperative launches add no
    // residency guarantee beyond the occupancy answer (MI355X_MICROARCH.md,
    // cooperative launch), so clusters use the plain, stream-ordered launch.
    static hipError_t launch(int grid, size_t dyn, hipStream_t st, const DevGraph& g, const SlotArena& ar,
                             const int32_t* src, int32_t S, const int32_t* dst, int32_t nb, double delta,
                             const RouteOut& o, int keep) {
        auto* fn = &k_routes_sssp<K, NT, PM, true>;
        if (dyn > 0) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, int(dyn));
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(fn, dim3(grid), dim3(NT), dyn, st, g, ar, src, S, dst, nb, delta, o, keep);
        return hipGetLastError();
    }
    static int occupancy(size_t dyn) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_routes_sssp<K, NT, PM, true>, NT, dyn) != hipSuccess) return 0;
        return n;
    }
};
// The single-launch table pass (k_routes_pass): built for the default variant
// (K = 16 buckets with a K = 8 tail, 1024 threads) in every pending mode.
template <int K, int NT, int PM>
struct SsspPass {
    static hipError_t launch(int slots, size_t dyn, hipStream_t st, const DevGraph& g, const SlotArena& ar,
                             const int32_t* src, int32_t S, const int32_t* dst, int32_t nb, double delta,
                             const RouteOut& o, int keep, const TailArgs& ta) {
        auto* fn = &k_routes_pass<K, NT, PM>;
        if (dyn > 0) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, int(dyn));
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(fn, dim3(slots), dim3(NT), dyn, st, g, ar, src, S, dst, nb, delta, o, keep, ta);
        return hipGetLastError();
    }
    static int occupancy(size_t dyn) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_routes_pass<K, NT, PM>, NT, dyn) != hipSuccess) return 0;
        return n;
    }
};
constexpr bool has_pass(int v) { return v == 4; }
template <typename... A>
hipError_t pass_launch(int v, int pm, A&&... a) {
    if (!has_pass(v)) return hipErrorInvalidValue;
#ifdef SHDR_ANALYSIS
    return SsspPass<16, kNT, 1>::launch(std::forward<A>(a)...);
#endif
    return pm == 2 ? SsspPass<16, kNT, 2>::launch(std::forward<A>(a)...)
                   : pm == 1 ? SsspPass<16, kNT, 1>::launch(std::forward<A>(a)...)
                             : SsspPass<16, kNT, 0>::launch(std::forward<A>(a)...);
}
// the single-launch pass runs as many workgroups per CU as the main launch would
bool pass_fits(int v, int pm, size_t dyn, int occ_main) {
    if (!has_pass(v)) return false;
#ifdef SHDR_ANALYSIS
    return SsspPass<16, kNT, 1>::occupancy(dyn) >= occ_main;
#endif
    const int n = pm == 2 ? SsspPass<16, kNT, 2>::occupancy(dyn)
                          : pm == 1 ? SsspPass<16, kNT, 1>::occupancy(dyn) : SsspPass<16, kNT, 0>::occupancy(dyn);
    return n >= occ_main && n > 0;
}

constexpr bool has_cluster(int v) { return v == 4 || v == 6 || v == 7; }
// occupancy of the cluster kernel (0: not built for this variant / mode)
int cluster_occupancy(int v, int pm, size_t dyn) {
    // Both pending sets in LDS (PM 2) only. PM 1 clusters (far set in
    // member-private bytes) returned broken chains and then faulted the GPU in
    // round-3 builds, and the cause is not identified; no
    // BASELINE layout picks them (cfg5 shards stay plain by the wave model), so
    // they are not built into the product's choices. SHDR_EXPERIMENTS builds
    // can still force them (SHDR_CLUSTER_PM1=1) for the investigation.
#ifdef SHDR_EXPERIMENTS
    static const bool allow_pm1 = getenv("SHDR_CLUSTER_PM1") && atoi(getenv("SHDR_CLUSTER_PM1")) != 0;
#else
    constexpr bool allow_pm1 = false;
#endif
    if (!has_cluster(v) || pm < 1 || (pm == 1 && !allow_pm1)) return 0;
#ifdef SHDR_ANALYSIS
    return 0;
#endif
    switch (v) {
        case 4: return pm == 2 ? SsspC<16, kNT, 2>::occupancy(dyn) : SsspC<16, kNT, 1>::occupancy(dyn);
        case 6: return pm == 2 ? SsspC<8, kNT, 2>::occupancy(dyn) : SsspC<8, kNT, 1>::occupancy(dyn);
        default: return pm == 2 ? SsspC<32, kNT, 2>::occupancy(dyn) : SsspC<32, kNT, 1>::occupancy(dyn);
    }
}
template <typename... A>
hipError_t cluster_launch(int v, int pm, A&&... a) {
#ifdef SHDR_ANALYSIS
    return hipErrorInvalidValue;
#endif
    switch (v) {
        case 4: return pm == 2 ? SsspC<16, kNT, 2>::launch(std::forward<A>(a)...) : SsspC<16, kNT, 1>::launch(std::forward<A>(a)...);
        case 6: return pm == 2 ? SsspC<8, kNT, 2>::launch(std::forward<A>(a)...) : SsspC<8, kNT, 1>::launch(std::forward<A>(a)...);
        default: return pm == 2 ? SsspC<32, kNT, 2>::launch(std::forward<A>(a)...) : SsspC<32, kNT, 1>::launch(std::forward<A>(a)...);
    }
}

// PM 1 (near set in LDS, far set in slot bytes) is built for the default
// variant and its tail only; elsewhere it falls back to PM 0.
constexpr bool has_pm1(int v) { return v == 4 || v == 6 || v == 7; }

template <template <int, int, int> class F, typename... A>
auto with_variant(int v, int pm, A&&... a) {
#define SHDR_PMS(K, NT) \
    return pm == 2 ? F<K, NT, 2>::call(std::forward<A>(a)...) : F<K, NT, 0>::call(std::forward<A>(a)...);
#define SHDR_PMS1(K, NT)                                                                                   \
    return pm == 2 ? F<K, NT, 2>::call(std::forward<A>(a)...)                                              \
                   : pm == 1 ? F<K, NT, 1>::call(std::forward<A>(a)...) : F<K, NT, 0>::call(std::forward<A>(a)...);
#ifdef SHDR_ANALYSIS  // tools/spill_map.py --fast: only the cfg5 product instances (never a library)
    if (v == 4) return F<16, kNT, 1>::call(std::forward<A>(a)...);
    return F<8, kNT, 1>::call(std::forward<A>(a)...);
#endif
    switch (v) {
        case 0: SHDR_PMS(8, 256)
        case 1: SHDR_PMS(16, 256)
        case 2: SHDR_PMS(16, 512)
        case 3: SHDR_PMS(32, 512)
        case 4: SHDR_PMS1(16, kNT)
        case 5: SHDR_PMS(8, 512)
        case 6: SHDR_PMS1(8, kNT)
        default: SHDR_PMS1(32, kNT)
    }
#undef SHDR_PMS
#undef SHDR_PMS1
}
template <int K, int NT, int PM>
struct LaunchF { template <typename... A> static hipError_t call(A&&... a) { return Sssp<K, NT, PM>::launch(std::forward<A>(a)...); } };
template <int K, int NT, int PM>
struct OccF { static int call(size_t dyn) { return Sssp<K, NT, PM>::occupancy(dyn); } };
template <int K, int NT, int PM>
struct LdsF { static size_t call() { return Sssp<K, NT, PM>::static_lds(); } };

constexpr size_t kLdsPerCu = 160 * 1024;  // gfx950

// Pending-set storage for this graph and variant: both bitmaps in LDS next to
// the kernel's static LDS if they fit, else the near bitmap alone (sharing its
// region with the epilogue's hop stacks), else slot bytes. -> (mode, dynamic LDS bytes)
struct PendingMode { int pm; size_t dyn; };
PendingMode pending_mode(const shdr_engine* e, int variant) {
    if (e->pending_lds <= 0) return {0, 0};
    const size_t words = size_t((e->csr.V + 31) / 32) * sizeof(uint32_t);
    if (e->pending_lds >= 2 && with_variant<LdsF>(variant, 2) + 2 * words <= kLdsPerCu) return {2, 2 * words};
    if (has_pm1(variant)) {
        const int NT = kVariants[variant].NT;
        const size_t dyn = std::max(words, size_t(stack_depth(NT)) * NT * sizeof(double));
        if (with_variant<LdsF>(variant, 1) + dyn <= kLdsPerCu) return {1, dyn};
    }
    return {0, 0};
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct ArenaLayout {
    size_t stride, off_pred, off_nflag, off_fflag, off_items;
    size_t flags_off, flags_bytes;  // the flag region, zeroed once per compute
};

ArenaLayout layout_for(int32_t V, int64_t A, int K) {
    ArenaLayout L;
    size_t o = 0;
    o += align_up(size_t(V) * K * 8, 256);
    L.off_pred = o; o += align_up(size_t(V) * K * 8, 256);
    L.flags_off = o;
    L.off_nflag = o; o += align_up(size_t(V) + 16, 256);  // per-vertex pending bytes (when not in LDS)
    L.off_fflag = o; o += align_up(size_t(V) + 16, 256);
    L.flags_bytes = o - L.flags_off;
    L.off_items = o; o += align_up((size_t(V) + size_t(A) / kChunk + 64) * 16, 256);
    L.stride = o;
    return L;
}

int record(shdr_engine* e, int k, bool on, hipStream_t st) {
    if (on) HIPCHK(hipEventRecord(e->ev[k], st));
    return SHDR_OK;
}


// Workgroups of variant `var` resident on the whole device at once.
int64_t resident_slots(shdr_engine* e, int var) {
    if (e->slots_cache[var] == 0) {
        const PendingMode pmd = pending_mode(e, var);
        e->slots_cache[var] = int64_t(e->cus) * with_variant<OccF>(var, pmd.pm, pmd.dyn);
#ifdef SHDR_EXPERIMENTS
        // fewer resident workgroups than CUs (what bounds the pass: per-CU or chip-wide request rate)
        if (const char* x = getenv("SHDR_MAX_SLOTS"))
            e->slots_cache[var] = std::max<int64_t>(1, std::min<int64_t>(e->slots_cache[var], atoll(x)));
#endif
    }
    return e->slots_cache[var];
}

// Clusters of cl workgroups resident at once (a multiple of 8 from 8 up, so
// that a cluster's members can be blocks b, b+8, ...), 0 if not built.
int64_t cluster_slots(shdr_engine* e, int var, int cl) {
    const PendingMode pmd = pending_mode(e, var);
    const int64_t wg = int64_t(e->cus) * cluster_occupancy(var, pmd.pm, pmd.dyn);
    int64_t c = wg / std::max(1, cl);
    if (c >= 8) c -= c % 8;
    return c;
}

// Half-width variant with the same workgroup size (tail balancing), or -1.
int tail_variant(int var) {
    const int n = int(sizeof(kVariants) / sizeof(kVariants[0]));
    for (int v = 0; v < n; ++v)
        if (kVariants[v].NT == kVariants[var].NT && 2 * kVariants[v].K == kVariants[var].K) return v;
    return -1;
}

// Launch the shortest-path kernel for S sources (device array src) into o.
// role: 0 route table, 1 its tail launch, 2 landmark pre-pass.
// The device error word and the bucket tickets: [0] guard, [1 + t] ticket t,
// [4..15] the first guard trip's record (guard_record).
int reset_err(shdr_engine* e, hipStream_t st) {
    if (!e->d_err) HIPCHK(hipMalloc((void**)&e->d_err, kErrWords * sizeof(int)));
    HIPCHK(hipMemsetAsync(e->d_err, 0, kErrWords * sizeof(int), st));
    return SHDR_OK;
}

// Grow the slot arena to `bytes` if that stays within ~60% of free HBM.
// -> SHDR_OK, SHDR_ENOMEM (over budget, nothing changed) or an error.
// (Re)allocate the slot arena: `bytes` from a base aligned to arena_align bytes
// (SHDR_ARENA_ALIGN_MB; the allocation is padded by that much).
int arena_alloc(shdr_engine* e, size_t bytes) {
    if (e->arena_raw) HIPCHK(hipFree(e->arena_raw));
    e->arena_raw = nullptr;
    e->arena = nullptr;
    e->arena_bytes = 0;
    const size_t al = e->arena_align;
    HIPCHK(hipMalloc((void**)&e->arena_raw, bytes + al));
    const uintptr_t r = reinterpret_cast<uintptr_t>(e->arena_raw);
    e->arena = al ? reinterpret_cast<char*>((r + al - 1) / al * al) : e->arena_raw;
    e->arena_bytes = bytes;
    e->flags_dirty = true;
    if (getenv("SHDR_VERBOSE"))
        std::fprintf(stderr, "[shdr] arena %.1f GB at %p (raw %p, align %zu MB)\n", double(bytes) / 1e9,
                     static_cast<void*>(e->arena), static_cast<void*>(e->arena_raw), al >> 20);
    return SHDR_OK;
}

int ensure_arena(shdr_engine* e, size_t bytes) {
    if (e->arena_bytes >= bytes) return SHDR_OK;
    size_t freeb = 0, totalb = 0;
    HIPCHK(hipMemGetInfo(&freeb, &totalb));
    if (bytes > (freeb + e->arena_bytes) * 3 / 5) return SHDR_ENOMEM;
    return arena_alloc(e, bytes);
}

// Slots a launch of variant var over S sources uses (before the memory bound).
int32_t launch_slots(shdr_engine* e, int var, int32_t S) {
    const int K = kVariants[var].K;
    return int32_t(std::min<int64_t>((S + K - 1) / K, resident_slots(e, var)));
}

int slot_arena(shdr_engine* e, hipStream_t st, int var, int cl, int32_t slots, int32_t region, size_t region_off,
               int tk, SlotArena& ar);

// Launch the shortest-path kernel for S sources (device array src) into o.
// role: 0 route table, 1 its tail launch, 2 landmark pre-pass. region >= 0: the
// launch uses the arena from byte region_off with `region` slots (the caller
// sized the arena; concurrent launches own disjoint regions) and ticket 1+tk.
int run_sssp(shdr_engine* e, hipStream_t st, const DevGraph& g, const int32_t* src_dev, int32_t S,
             const int32_t* dst_dev, const RouteOut& o, bool keep, int role = 0, int var = -1,
             int32_t region = -1, size_t region_off = 0, int tk = 0, int clv = 0) {
    const int32_t V = e->csr.V;
    if (var < 0) var = e->variant;
    const int K = kVariants[var].K;
    const int32_t nb = o.boff ? o.nb : (S + K - 1) / K;
    ArenaLayout Lh = layout_for(V, e->csr.A, K);
    const PendingMode pmd = pending_mode(e, var);
    const size_t dyn = pmd.dyn;
    // cluster mode: `slots` counts clusters (one bucket slot each), the grid is slots * cl
    const int cl = clv > 0 ? clv : (role == 0 && !keep && region < 0) ? e->cur_cl : 1;
    int32_t slots = cl > 1 ? int32_t(std::min<int64_t>((int64_t(nb) + 7) / 8 * 8, cluster_slots(e, var, cl)))
                           : int32_t(std::min<int64_t>(nb, resident_slots(e, var)));
    if (keep) slots = nb;
    if (region >= 0) slots = region;
    if (region < 0 && e->arena_bytes < size_t(slots) * Lh.stride) {
        // grow the arena, bounded to ~60% of free HBM
        size_t freeb = 0, totalb = 0;
        HIPCHK(hipMemGetInfo(&freeb, &totalb));
        const size_t budget = (freeb + e->arena_bytes) * 3 / 5;
        if (size_t(slots) * Lh.stride > budget) {
            if (keep) { shdr::set_error("routes_compute: KEEP_TREES needs more HBM than available"); return SHDR_ENOMEM; }
            slots = std::max<int32_t>(1, int32_t(budget / Lh.stride));
        }
    }
    const size_t need = size_t(slots) * Lh.stride;
    if (region < 0 && e->arena_bytes < need) {
        int rc;
        if ((rc = arena_alloc(e, need))) return rc;
    }
    SlotArena ar;
    int rc;
    if ((rc = slot_arena(e, st, var, cl, slots, region, region_off, tk, ar))) return rc;
    double delta = e->delta > 0.0 ? e->delta : e->auto_delta;
    const DevGraph& gl = g;
    int kflags = (keep ? 1 : 0) | (role == 2 ? 8 : 0);  // 8: distances only (landmark pre-pass)
#if defined(SHDR_DIAG) || defined(SHDR_SKIP_ONLY)
    if (const char* sk = getenv("SHDR_DIAG_SKIP")) kflags |= atoi(sk) << 1;  // 1: pred pass, 2: epilogue
#endif
    if (cl > 1)
        HIPCHK(cluster_launch(var, pmd.pm, slots * cl, dyn, st, gl, ar, src_dev, S, dst_dev, nb, delta, o, kflags));
    else
        HIPCHK(with_variant<LaunchF>(var, pmd.pm, slots, dyn, st, gl, ar, src_dev, S, dst_dev, nb, delta, o, kflags, role));
    if (keep && role != 2) {
        e->kept = true;
        e->kept_K = K;
        e->kept_S = S;
        e->kept_stride = Lh.stride;
        e->kept_off_pred = Lh.off_pred;
    }
    return SHDR_OK;
}

// One table pass as a single launch (k_routes_pass): the main rows [0, S1) in
// full-width buckets of variant var over `slots` slots from arena offset 0, the
// tail rows [S1, S) in half-width buckets of tail_variant(var) over `tslots` slots
// from offset toff (their own ticket). The caller sized the arena.
int run_pass(shdr_engine* e, hipStream_t st, const DevGraph& g, int var, int32_t S1, int32_t slots, const RouteOut& o,
             int32_t S, int32_t tslots, size_t toff, const RouteOut& o2) {
    const int tvar = tail_variant(var);
    const int K = kVariants[var].K, KT = kVariants[tvar].K;
    const PendingMode pmd = pending_mode(e, var);
    SlotArena am;
    TailArgs ta;
    int rc;
    if ((rc = slot_arena(e, st, var, 1, slots, slots, 0, 0, am))) return rc;
    if ((rc = slot_arena(e, st, tvar, 1, tslots, tslots, toff, 1, ta.arena))) return rc;
    ta.src = e->d_src + S1;
    ta.S = S - S1;
    ta.nbuckets = (ta.S + KT - 1) / KT;
    ta.blocks = std::min(tslots, slots);
    ta.out = o2;
    const int32_t nb = o.boff ? o.nb : (S1 + K - 1) / K;
    const double delta = e->delta > 0.0 ? e->delta : e->auto_delta;
    HIPCHK(pass_launch(var, pmd.pm, slots, pmd.dyn, st, g, am, e->d_src, S1, e->d_dst, nb, delta, o, 0, ta));
    return SHDR_OK;
}

// The slot arena of one launch: `slots` slots of variant var's layout from byte
// region_off (region >= 0) or the whole arena, ticket 1 + tk, cluster records for cl > 1;
// the slots' flag bytes are cleared unless the region is known clean.
int slot_arena(shdr_engine* e, hipStream_t st, int var, int cl, int32_t slots, int32_t region, size_t region_off,
               int tk, SlotArena& ar) {
    const int32_t V = e->csr.V;
    const int K = kVariants[var].K;
    const ArenaLayout Lh = layout_for(V, e->csr.A, K);
    const PendingMode pmd = pending_mode(e, var);
    if (!e->d_err) { shdr::set_error("run_sssp: error word not set up"); return SHDR_EINVAL; }
    ar.base = e->arena + region_off;
    ar.stride = Lh.stride;
    ar.item_cap = int64_t(V) + e->csr.A / kChunk + 64;
    ar.err = e->d_err;
    ar.ticket = e->d_err + 1 + tk;
    ar.off_pred = Lh.off_pred; ar.off_nflag = Lh.off_nflag; ar.off_fflag = Lh.off_fflag;
    ar.off_items = Lh.off_items;
    ar.cl = 1;
    ar.cbase = nullptr;
    ar.cstride = ar.c_off_far = ar.c_far = ar.c_off_plane = ar.c_plane = ar.c_off_items = ar.c_items = 0;
    if (cl > 1) {
        ar.cl = cl;
        ar.c_plane = align_up(size_t((V + 31) / 32), 64);  // near set [0, vexp) and chain-pass to-do [0, V)
        ar.c_far = pmd.pm == 1 ? align_up(size_t(V) + 16, 256) : 0;
        ar.c_items = align_up(size_t(ar.item_cap) * 16, 256);
        ar.c_off_far = kClusterRecBytes;
        ar.c_off_plane = align_up(ar.c_off_far + size_t(cl) * ar.c_far, 256);  // (zeroed per launch up to here)
        ar.c_off_items = align_up(ar.c_off_plane + 2 * size_t(cl) * ar.c_plane * 4, 256);
        ar.cstride = align_up(ar.c_off_items + size_t(cl - 1) * ar.c_items, 4096);
        int rc;
        if ((rc = ensure((void**)&e->d_cl, &e->cap_cl, size_t(slots) * ar.cstride))) return rc;
        ar.cbase = e->d_cl;
        // barrier counters and the private far bytes start at zero (planes are written before read)
        HIPCHK(hipMemset2DAsync(e->d_cl, ar.cstride, 0, ar.c_off_plane, size_t(slots), st));
    }
    // slot pending bytes (used when the LDS bitmaps do not fit) are consumed back to zero by every finished bucket; clear them after a new
    // allocation, a layout change or a tripped guard only
    // (a region launch uses `region` slots from region_off; otherwise every slot of the arena)
    {
        const size_t roff = region >= 0 ? region_off : 0;
        const size_t rslots = region >= 0 ? size_t(slots) : e->arena_bytes / Lh.stride;
        // (the bucket width is part of the key: for tiny V the padded slot strides of
        // two widths coincide, and a wider bucket must not read words a narrower one
        // never wrote as its own parity's rows)
        const std::array<size_t, 4> reg{roff, Lh.stride, rslots, size_t(K)};
        if (e->flags_dirty) {
            e->clean_regions.clear();
            e->flags_dirty = false;
        }
        if (std::find(e->clean_regions.begin(), e->clean_regions.end(), reg) == e->clean_regions.end()) {
            HIPCHK(hipMemset2DAsync(e->arena + roff + Lh.flags_off, Lh.stride, 0, Lh.flags_bytes, rslots, st));
            const size_t lo = roff, hi = roff + rslots * Lh.stride;
            e->clean_regions.erase(std::remove_if(e->clean_regions.begin(), e->clean_regions.end(),
                                                  [&](const std::array<size_t, 4>& r) {
                                                      return r[0] < hi && lo < r[0] + r[2] * r[1];
                                                  }),
                                   e->clean_regions.end());
            e->clean_regions.push_back(reg);
        }
    }
    return SHDR_OK;
}

// Landmark pre-pass + source grouping. Rows of one bucket share every arc read,
// but only lanes whose wavefronts reach a vertex in the same round share the
// row visit (and the coalesced atomic). Sources are embedded by their distances
// to the kLandmarks highest-degree vertices (directed graphs: on the reversed
// graph) — one pre-pass bucket computes all of them — and cut into buckets by recursive
// median splits along the widest coordinate, so each bucket holds sources whose
// distance fields nearly coincide. order_mode 2 additionally shifts each lane's
// near/far key by its distance to the first landmark. Only the schedule
// changes: results are identical for any grouping and offsets.
constexpr int kLandmarks = 4;

// Lanes [0, L) of slot 0's [V][K] distance rows -> [L][V] (the landmark embedding).
// One wave that waits `ticks` of the 100 MHz clock and touches no memory: placed on
// the main launch's stream after the fork, it gives the concurrent tail (submitted
// first on the second stream, behind the fork event) time to be dispatched before the
// main launch takes every CU (SHDR_TAIL_FIRST).
__global__ void __launch_bounds__(64) k_hold(uint32_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void k_lane_extract(const double* __restrict__ rows, int32_t V, int K, int L, double* __restrict__ out) {
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < int64_t(V) * L;
         i += int64_t(gridDim.x) * blockDim.x) {
        const int32_t v = int32_t(i % V), k = int32_t(i / V);
        const double d = rows[size_t(v) * K + k];
        out[i] = (d - d == 0.0) ? d : 0.0;  // unreachable (inf) -> 0
    }
}

// The pre-pass is enqueued when the engine is created (once the CSR and the arc
// blocks are in HBM) and collected at its first use, so its ~0.25 s on cfg5 runs
// under the rest of engine start-up (predecessor items) and under the caller's
// own work; every entry point that touches the arena collects it first.
int landmark_launch(shdr_engine* e, hipStream_t st) {
    const int32_t V = e->csr.V;
    const int K = kVariants[e->variant].K;
    int nl = kLandmarks;
#ifdef SHDR_EXPERIMENTS
    if (const char* x = getenv("SHDR_LANDMARKS")) nl = std::max(1, atoi(x));
#endif
    const int L = std::min<int>(nl, std::min<int>(K, V));
    if (L <= 0) return SHDR_OK;
    // the L highest-degree vertices, degree ties in the caller's numbering (the
    // landmarks do not depend on relabel_bfs)
    std::vector<int32_t> order(static_cast<size_t>(V));
    for (int32_t v = 0; v < V; ++v) order[v] = v;
    auto cid = [&](int32_t v) { return e->oldid.empty() ? v : e->oldid[v]; };
    std::partial_sort(order.begin(), order.begin() + L, order.end(), [&](int32_t a, int32_t b) {
        const int64_t da = e->csr.rowptr[a + 1] - e->csr.rowptr[a], db = e->csr.rowptr[b + 1] - e->csr.rowptr[b];
        return da != db ? da > db : cid(a) < cid(b);
    });
    DevGraph g = devgraph(e);
    if (e->directed) {  // distances TO the landmarks: run on the reversed graph
        std::swap(g.rowptr, g.irowptr); std::swap(g.col, g.isrc); std::swap(g.w, g.iw);
        std::swap(g.oclat, g.iclat); std::swap(g.ocrel, g.icrel);
        g.ablk = e->iablk; g.bfirst = e->ibfirst; g.nblk = e->inblk;
    }
    int rc;
    if ((rc = ensure((void**)&e->d_lm, &e->cap_lm, align_up(size_t(L) * 4, 256) + size_t(L) * V * 8))) return rc;
    HIPCHK(hipMemcpyAsync(e->d_lm, order.data(), size_t(L) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // (order is a temporary)
    RouteOut o{};
    if ((rc = reset_err(e, st))) return rc;
    if ((rc = run_sssp(e, st, g, reinterpret_cast<int32_t*>(e->d_lm), L, nullptr, o, true, 2))) return rc;
    double* emb = reinterpret_cast<double*>(reinterpret_cast<char*>(e->d_lm) + align_up(size_t(L) * 4, 256));
    hipLaunchKernelGGL(k_lane_extract, dim3(1024), dim3(256), 0, st, reinterpret_cast<const double*>(e->arena), V, K, L,
                       emb);
    HIPCHK(hipGetLastError());
    e->lm_count = L;
    e->lm_pending = true;
    e->lm_stream = st;
    return SHDR_OK;
}

// Wait for an enqueued pre-pass and read the embedding back.
int landmark_collect(shdr_engine* e) {
    if (!e->lm_pending) return SHDR_OK;
    e->lm_pending = false;
    const auto tl0 = std::chrono::steady_clock::now();
    struct Stamp {
        shdr_engine* e; std::chrono::steady_clock::time_point t0;
        ~Stamp() { e->host_ms[0] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
    } stamp{e, tl0};
    const int32_t V = e->csr.V, L = e->lm_count;
    HIPCHK(hipStreamSynchronize(e->lm_stream));
    int herr = 0;
    HIPCHK(hipMemcpy(&herr, e->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (herr) {
        shdr::set_error("landmark pre-pass: device guard tripped (code " + std::to_string(herr) + ")");
        return SHDR_EHIP;
    }
    e->lm_dist.resize(size_t(L) * V);
    const char* emb = reinterpret_cast<const char*>(e->d_lm) + align_up(size_t(L) * 4, 256);
    HIPCHK(hipMemcpy(e->lm_dist.data(), emb, e->lm_dist.size() * 8, hipMemcpyDeviceToHost));
    e->lm_ready = true;
    return SHDR_OK;
}

int landmark_prepass(shdr_engine* e, hipStream_t st) {
    if (e->lm_ready) return SHDR_OK;
    int rc;
    if (!e->lm_pending && (rc = landmark_launch(e, st))) return rc;
    return landmark_collect(e);
}

// Recursive median split of the sources of groups [g0, g1) (idx[gstart[g0],
// gstart[g1])) along the widest landmark coordinate: the first ceil((g1-g0)/2)
// groups' sources go left.
void kd_groups(const shdr_engine* e, const int32_t* src, std::vector<int32_t>& idx, const std::vector<int32_t>& gstart,
               size_t g0, size_t g1) {
    if (g1 - g0 <= 1) return;
    const size_t lo = size_t(gstart[g0]), hi = size_t(gstart[g1]);
    const int32_t V = e->csr.V;
    int best = 0;
    double width = -1.0;
    for (int k = 0; k < e->lm_count; ++k) {
        double mn = INFINITY, mx = -INFINITY;
        for (size_t i = lo; i < hi; ++i) {
            const double d = e->lm_dist[size_t(k) * V + src[idx[i]]];
            mn = std::min(mn, d); mx = std::max(mx, d);
        }
        if (mx - mn > width) { width = mx - mn; best = k; }
    }
    const double* col = e->lm_dist.data() + size_t(best) * V;
    std::stable_sort(idx.begin() + lo, idx.begin() + hi,
                     [&](int32_t a, int32_t b) { return col[src[a]] < col[src[b]]; });
    const size_t gm = g0 + (g1 - g0 + 1) / 2;
    kd_groups(e, src, idx, gstart, g0, gm);
    kd_groups(e, src, idx, gstart, gm, g1);
}

// Longest-first issue order: buckets are handed out by ticket, several per
// resident workgroup, so the launch ends when its slowest workgroup does. Before
// any bucket of this source list has been timed, a bucket's cost is predicted by
// how far apart its sources lie (their lanes settle shared vertices in different
// rounds): groups go in decreasing order of their RMS landmark-space spread. Once
// a pass over the same source list has timed its buckets, the order is by
// measured duration (profile-guided LPT). Groups >= nsorted stay last.
std::vector<int32_t> groups_by_spread(const shdr_engine* e, const int32_t* src, const std::vector<int32_t>& perm,
                                      const std::vector<int32_t>& gstart, int32_t nsorted) {
    const int32_t V = e->csr.V;
    const size_t ng = gstart.size() - 1;
    std::vector<double> spread(ng, 0.0);
    for (size_t b = 0; b < ng; ++b) {
        const int32_t a0 = gstart[b], a1 = gstart[b + 1];
        double acc = 0.0;
        for (int k = 0; k < e->lm_count; ++k) {
            const double* col = e->lm_dist.data() + size_t(k) * V;
            double m = 0.0;
            for (int32_t i = a0; i < a1; ++i) m += col[src[perm[i]]];
            m /= std::max(1, a1 - a0);
            for (int32_t i = a0; i < a1; ++i) {
                const double d = col[src[perm[i]]] - m;
                acc += d * d;
            }
        }
        spread[b] = acc;
    }
    std::vector<int32_t> bo(ng);
    for (size_t b = 0; b < ng; ++b) bo[b] = int32_t(b);
    if (e->bucket_sort)
        std::stable_sort(bo.begin(), bo.begin() + nsorted, [&](int32_t a, int32_t b) { return spread[a] > spread[b]; });
    return bo;
}

// Measured order: timed groups by decreasing duration, then the untimed ones
// (a tail launch's) in their previous relative order.
void groups_by_cost(shdr_engine* e) {
    std::vector<int32_t> timed, rest;
    for (int32_t g : e->border) (e->gcost[g] >= 0.f ? timed : rest).push_back(g);
    std::stable_sort(timed.begin(), timed.end(), [&](int32_t a, int32_t b) { return e->gcost[a] > e->gcost[b]; });
    timed.insert(timed.end(), rest.begin(), rest.end());
    e->border.swap(timed);
}

// processed order = the kd groups in border order; bucket b = group border[b]
int apply_order(shdr_engine* e, hipStream_t st, const int32_t* src, int32_t S) {
    std::vector<int32_t> perm(static_cast<size_t>(S));
    std::vector<int32_t> boff(e->border.size() + 1, 0);
    size_t o = 0;
    for (size_t b = 0; b < e->border.size(); ++b) {
        const int32_t g = e->border[b];
        std::copy(e->kd_perm.begin() + e->gstart[g], e->kd_perm.begin() + e->gstart[g + 1], perm.begin() + o);
        o += size_t(e->gstart[g + 1] - e->gstart[g]);
        boff[b + 1] = int32_t(o);
    }
    e->h_boff = boff;
    e->h_perm = perm;
    e->h_src_sorted.resize(size_t(S));
    std::vector<double> soff(static_cast<size_t>(S));
    for (int32_t i = 0; i < S; ++i) {
        e->h_src_sorted[i] = src[perm[i]];
        soff[i] = e->lm_dist[src[perm[i]]];  // landmark 0
    }
    int rc;
    if ((rc = ensure((void**)&e->d_rowmap, &e->cap_rowmap, size_t(S) * 4))) return rc;
    if ((rc = ensure((void**)&e->d_soff, &e->cap_soff, size_t(S) * 8))) return rc;
    if ((rc = ensure((void**)&e->d_boff, &e->cap_boff, boff.size() * 4))) return rc;
    HIPCHK(hipMemcpyAsync(e->d_rowmap, perm.data(), size_t(S) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->d_soff, soff.data(), size_t(S) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->d_boff, boff.data(), boff.size() * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // host vectors above are temporaries
    return SHDR_OK;
}

// Group sizes for S sources. Balanced layout: every wave of the launch full —
// nb = waves x resident slots groups (fewer if S is smaller) of f or f + 1 <= K
// sources, so the last wave is not partial and a small shard (strong scaling:
// 1,250 cfg4 rows on 256 CUs) still occupies every CU. Legacy layout: groups of
// K, the last one partial (its partial wave runs as a concurrent half-width tail).
std::vector<int32_t> group_starts(shdr_engine* e, int32_t S, int K, int32_t* nsorted) {
    std::vector<int32_t> st(1, 0);
    if (e->cur_balance) {
        const int64_t P = e->cur_cl > 1 ? cluster_slots(e, e->variant, e->cur_cl) : resident_slots(e, e->variant);
        const int64_t waves = (S + int64_t(K) * P - 1) / (int64_t(K) * P);
        const int64_t nb = std::min<int64_t>(S, waves * P);
        const int64_t f = S / nb, r = S % nb;
        for (int64_t b = 0; b < nb; ++b) st.push_back(st.back() + int32_t(f + (b < r ? 1 : 0)));
        *nsorted = int32_t(nb);
    } else {
        for (int32_t i = K; i <= S; i += K) st.push_back(i);
        *nsorted = int32_t(st.size() - 1);
        if (st.back() < S) st.push_back(S);
    }
    return st;
}

int order_sources(shdr_engine* e, hipStream_t st, const int32_t* src, int32_t S) {
    const int K = kVariants[e->variant].K;
    if (e->order_mode == 0 || S < 2 * K) return SHDR_OK;
    int rc;
    // the same source list as the last call (e.g. every bench step): reuse its grouping
    const int32_t key_hdr[3] = {S, e->variant,
                                e->order_mode | (e->bucket_sort << 4) | (e->cur_balance << 5) | (e->cur_cl << 8)};
    if (e->order_key.size() == size_t(S) + 3 && std::equal(key_hdr, key_hdr + 3, e->order_key.begin()) &&
        std::equal(src, src + S, e->order_key.begin() + 3)) {
        if (!e->costs_fresh) return SHDR_OK;
        e->costs_fresh = false;
        groups_by_cost(e);
        return apply_order(e, st, src, S);
    }
    if (!e->lm_ready && (rc = landmark_prepass(e, st))) return rc;
    e->kd_perm.resize(static_cast<size_t>(S));
    for (int32_t i = 0; i < S; ++i) e->kd_perm[i] = i;
    e->gstart = group_starts(e, S, K, &e->nsorted);
    e->ngroups = int32_t(e->gstart.size() - 1);
    kd_groups(e, src, e->kd_perm, e->gstart, 0, e->gstart.size() - 1);
    e->border = groups_by_spread(e, src, e->kd_perm, e->gstart, e->nsorted);
    // K-wide layout with a partial last group (S % K != 0): issue that group first.
    // It is the last kd leaf (the extreme sources of the last region along one
    // landmark coordinate) and, issued last, it set a small shard's time: cfg5 over
    // 8 GPUs, part 7: a 10-source bucket started at 201 ms and ran 305 ms while the
    // other parts ended at ~377 ms (diagnostic build, profiles/r02_diag_cfg5_p8.log).
    // Buckets then take explicit row offsets (boff); the tail launch's rows are the
    // last full groups, so its half-width buckets stay aligned to them.
    e->partial_first = !e->cur_balance && e->nsorted < e->ngroups;
    if (e->partial_first) std::rotate(e->border.begin(), e->border.end() - 1, e->border.end());
    e->gcost.assign(e->border.size(), -1.f);
    e->costs_fresh = false;
    e->order_key.clear();
    if ((rc = apply_order(e, st, src, S))) return rc;
    e->order_key.assign(key_hdr, key_hdr + 3);
    e->order_key.insert(e->order_key.end(), src, src + S);
    return SHDR_OK;
}
}  // namespace

// fn(v0, v1) over [0, n) split across up to 16 host threads (engine start-up work
// whose per-vertex pieces write disjoint output)
template <typename F>
static void host_parallel(int32_t n, F&& fn) {
    const int nt = std::max(1, std::min<int>({16, int(std::thread::hardware_concurrency()), (n + 65535) / 65536}));
    if (nt == 1) { fn(0, n); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] { fn(int32_t(int64_t(n) * t / nt), int32_t(int64_t(n) * (t + 1) / nt)); });
    for (auto& x : th) x.join();
}

extern "C" {

int32_t shdr_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// Device numbering: breadth-first from the highest-degree vertex (arcs in either
// direction), unreached vertices appended in index order. Vertices settled in
// the same relaxation rounds then sit close in the [V][K] state and in the arc
// blocks (cfg5: -4.7 % kernel time vs the generator's numbering; a random
// numbering of cfg4 costs +8 %). Each vertex keeps its arc lists in the caller's
// order, so the predecessor pass's minimum-index tie rule and the canonical-edge
// factors pick the same arcs: results do not depend on the numbering.
// Pendant vertices (every arc in or out joins one single neighbour) then move to
// the end, in breadth-first order among themselves: [0, *vexp) are the vertices
// the relaxation may have to expand.
void relabel_bfs(shdr::CsrImage& c, std::vector<int32_t>& newid, std::vector<int32_t>& oldid, int32_t* vexp) {
    const int32_t V = c.V;
    newid.assign(size_t(V), -1);
    oldid.clear();
    oldid.reserve(size_t(V));
    *vexp = V;
    if (V == 0) return;
    int32_t hub = 0;
    auto deg = [&](int32_t v) {
        int64_t d = c.rowptr[v + 1] - c.rowptr[v];
        if (!c.same_in_out) d += c.irowptr[v + 1] - c.irowptr[v];
        return d;
    };
    for (int32_t v = 1; v < V; ++v)
        if (deg(v) > deg(hub)) hub = v;
    auto visit = [&](int32_t v) {
        if (newid[v] < 0) { newid[v] = int32_t(oldid.size()); oldid.push_back(v); }
    };
    visit(hub);
    int32_t low = 0;  // every vertex below it is visited
    for (int32_t next = 0; int32_t(oldid.size()) < V || next < int32_t(oldid.size());) {
        if (next == int32_t(oldid.size())) {  // component exhausted: lowest unvisited vertex
            while (newid[low] >= 0) ++low;
            visit(low);
        }
        const int32_t u = oldid[size_t(next++)];
        for (int64_t a = c.rowptr[u]; a < c.rowptr[u + 1]; ++a) visit(c.col[size_t(a)]);
        if (!c.same_in_out)
            for (int64_t a = c.irowptr[u]; a < c.irowptr[u + 1]; ++a) visit(c.isrc[size_t(a)]);
    }
    {
        auto pendant = [&](int32_t v) {
            int32_t q = -1;
            auto one = [&](int32_t x) {
                if (q < 0) q = x;
                return x == q;
            };
            for (int64_t a = c.rowptr[v]; a < c.rowptr[v + 1]; ++a)
                if (!one(c.col[size_t(a)])) return false;
            if (!c.same_in_out)
                for (int64_t a = c.irowptr[v]; a < c.irowptr[v + 1]; ++a)
                    if (!one(c.isrc[size_t(a)])) return false;
            return true;
        };
        std::vector<int32_t> core, tail;
        core.reserve(size_t(V));
        for (int32_t v : oldid) (pendant(v) ? tail : core).push_back(v);
        *vexp = int32_t(core.size());
        oldid.swap(core);
        oldid.insert(oldid.end(), tail.begin(), tail.end());
        for (int32_t nv = 0; nv < V; ++nv) newid[oldid[size_t(nv)]] = nv;
    }
    auto permute_csr = [&](std::vector<int64_t>& rp, std::vector<int32_t>& cc, std::vector<std::vector<double>*> arrs) {
        std::vector<int64_t> nrp(size_t(V) + 1, 0);
        for (int32_t nv = 0; nv < V; ++nv) nrp[nv + 1] = nrp[nv] + (rp[oldid[nv] + 1] - rp[oldid[nv]]);
        std::vector<int32_t> ncc(cc.size());
        host_parallel(V, [&](int32_t v0, int32_t v1) {
            for (int32_t nv = v0; nv < v1; ++nv) {
                const int64_t o0 = rp[oldid[nv]], n0 = nrp[nv], d = nrp[nv + 1] - n0;
                for (int64_t k = 0; k < d; ++k) ncc[size_t(n0 + k)] = newid[cc[size_t(o0 + k)]];
            }
        });
        for (std::vector<double>* x : arrs) {
            if (x->empty()) continue;
            std::vector<double> y(x->size());
            host_parallel(V, [&](int32_t v0, int32_t v1) {
                for (int32_t nv = v0; nv < v1; ++nv)
                    std::copy(x->begin() + rp[oldid[nv]], x->begin() + rp[oldid[nv] + 1], y.begin() + nrp[nv]);
            });
            x->swap(y);
        }
        rp.swap(nrp);
        cc.swap(ncc);
    };
    permute_csr(c.rowptr, c.col, {&c.w, &c.oclat, &c.ocrel, &c.ocjit});
    if (!c.same_in_out) permute_csr(c.irowptr, c.isrc, {&c.iw, &c.iclat, &c.icrel, &c.icjit});
    for (std::vector<double>* x : {&c.vrel, &c.self_lat, &c.self_rel}) {
        std::vector<double> y(x->size());
        for (int32_t nv = 0; nv < V; ++nv) y[nv] = (*x)[oldid[nv]];
        x->swap(y);
    }
}

// Relaxation window (delta-stepping bucket width): the mean arc weight on graphs
// up to ~1e5 expandable vertices, shrinking beyond:
// delta = mean_w * min(1, (1e5 / vexp)^0.42). Larger graphs re-expand more
// vertices at non-final distances per window (16 lanes whose wavefronts cross a
// vertex in different rounds), so a narrower window wastes fewer arc reads than
// its extra rounds cost. Same-box sweeps (ms per table, tools/ab.py; rule value
// in brackets): cfg4 BA 1e5: 20 / 30 / 40 / 50 -> 78 / 73 / 72 / 74 [50];
// BA 4e5: 30 / 50 -> 508 / 590 [31]; Chung-Lu 3e5 (vexp 2.4e5): 15 / 23 / 30 / 50
// -> 320 / 317 / 310 / 323 [38]; cfg5 Chung-Lu 1e6 (vexp 8e5): 12 / 15 / 20 / 25 /
// 30 / 38 / 50 -> 2332 / 2280 / 2278 / 2283 / 2350 / 2414 / 2584 [25 with a cube
// root]; round 3, one process per setting, 3 reps: 21 / 25 / 30 -> 2190 / 2207 / 2249
// (profiles/r03_delta_sep_ab2.log), hence the 0.42 power (cfg5: 21.1; Chung-Lu 3e5:
// 35; BA 4e5: 28). Results never depend on delta (test_delta_independence).
static double auto_delta(const shdr::CsrImage& c, int32_t vexp) {
    const double mean_w = std::max(1e-9, c.mean_w);
#ifdef SHDR_EXPERIMENTS
    const char* rule = getenv("SHDR_DELTA_RULE");  // 0 = the mean weight
    if (rule && atoi(rule) == 0) return mean_w;
#endif
    if (vexp <= 0) return mean_w;
    return mean_w * std::min(1.0, std::pow(1e5 / double(vexp), 0.42));
}

shdr_engine* shdr_engine_create(const shdr_graph* gh, int32_t device) {
    const shdr::HostGraph* hg = shdr::host_of(gh);
    if (!hg) { shdr::set_error("engine_create: NULL graph"); return nullptr; }
    int n = 0;
    if (const hipError_t he = hipGetDeviceCount(&n); he != hipSuccess || n <= 0) {
        shdr::set_error(std::string("engine_create: no HIP device visible (the routing engine has no CPU fallback; ") +
                        (he != hipSuccess ? hipGetErrorString(he) : "0 devices") + ")");
        return nullptr;
    }
    if (device < 0 || device >= n) { shdr::set_error("engine_create: bad device index"); return nullptr; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { shdr::set_error("engine_create: hipGetDeviceProperties failed"); return nullptr; }
    const int cus = prop.multiProcessorCount;
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0) {
        shdr::set_error(std::string("engine_create: device is ") + prop.gcnArchName + ", this build targets gfx950 only");
        return nullptr;
    }
    auto* e = new shdr_engine();
    e->device = device;
    e->cus = cus;
    // tuning overrides for experiments (results never depend on them)
    if (const char* v = getenv("SHDR_VARIANT")) {
        int x = atoi(v);
        if (x >= 0 && x < int(sizeof(kVariants) / sizeof(kVariants[0]))) e->variant = x;
    }
    if (const char* d = getenv("SHDR_DELTA")) e->delta = std::max(0.0, atof(d));
    if (const char* o = getenv("SHDR_ORDER")) e->order_mode = std::min(2, std::max(0, atoi(o)));
    if (const char* o = getenv("SHDR_BUCKET_SORT")) e->bucket_sort = atoi(o) != 0;
    if (const char* o = getenv("SHDR_PROFILE_ORDER")) e->profile_order = std::min(1, std::max(-1, atoi(o)));
    if (const char* o = getenv("SHDR_TAIL_MIN_WAVES")) e->tail_min_waves = std::max(1, atoi(o));
    if (const char* o = getenv("SHDR_BALANCE")) e->balance = std::min(2, std::max(0, atoi(o)));
    if (const char* o = getenv("SHDR_CLUSTER")) e->cluster = std::min(kMaxCluster, std::max(0, atoi(o)));
    if (const char* o = getenv("SHDR_CLUSTER_TAIL")) e->cluster_tail = atoi(o) != 0;
#ifdef SHDR_EXPERIMENTS
    if (const char* o = getenv("SHDR_HUB_LAG")) e->hub_lag = std::max(0, atoi(o));
    if (const char* o = getenv("SHDR_ARENA_ALIGN_MB")) e->arena_align = size_t(std::max(0, atoi(o))) << 20;
    // 0 always mark, 1 default, 2 lane-local rule, 3 skip inside clusters too (the round-3 rule)
    if (const char* o = getenv("SHDR_FAR_SKIP")) e->far_skip = std::min(3, std::max(0, atoi(o)));
    if (const char* o = getenv("SHDR_NOFILL")) e->nofill = atoi(o) != 0;
#endif
    if (const char* o = getenv("SHDR_PROGRESSIVE")) e->progressive = atoi(o) != 0;
    if (const char* o = getenv("SHDR_PROGRESSIVE_MIN_MB")) e->prog_min = size_t(std::max(0.0, atof(o)) * 1048576.0);
    if (const char* o = getenv("SHDR_PROGRESSIVE_CHUNK_MB"))
        e->prog_chunk = std::max<size_t>(4096, size_t(std::max(0.0, atof(o)) * 1048576.0));
    // engines sharing one device (test switch) cannot count on co-resident clusters
    if (const char* o = getenv("SHDR_ENGINES_SHARE_DEVICES")) e->shared_device = atoi(o) != 0;
    if (const char* p = getenv("SHDR_PENDING_LDS")) e->pending_lds = std::min(2, std::max(0, atoi(p)));
    shdr::HostGraph* mg = const_cast<shdr::HostGraph*>(hg);
    if (!mg->checked) mg->check();
    e->reach_all = mg->info.is_connected != 0;  // strongly connected (HostGraph::check)
    // SHDR_VERBOSE=1: engine start-up phases on stderr
    const bool verbose = getenv("SHDR_VERBOSE") && atoi(getenv("SHDR_VERBOSE")) > 0;
    auto tprev = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!verbose) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[shdr] engine_create %-12s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - tprev).count());
        tprev = now;
    };
    shdr::build_csr(*mg, e->csr);
    phase("csr");
    // every vertex reachable at a finite distance from every source: strongly
    // connected and every relaxation weight finite and non-negative (DevGraph::reach_all)
    for (const double x : e->csr.w)
        if (!(x >= 0.0 && x < INFINITY)) { e->reach_all = false; break; }
    if (e->csr.A >= (int64_t(1) << 31)) { shdr::set_error("engine_create: >2^31 arcs"); delete e; return nullptr; }
    e->complete = mg->info.is_complete != 0;
    e->directed = mg->directed;
    // the complete branch binary-searches the caller-numbered arc lists: keep them
    bool relabel = !e->complete;
    if (const char* r = getenv("SHDR_RELABEL")) relabel = relabel && atoi(r) != 0;  // experiments only
    e->vexp = e->csr.V;
    if (relabel) relabel_bfs(e->csr, e->newid, e->oldid, &e->vexp);
    phase("relabel");
    e->auto_delta = auto_delta(e->csr, e->vexp);
    if (const char* x = getenv("SHDR_PENDANT_SKIP"); x && atoi(x) == 0) e->vexp = e->csr.V;  // experiments only
    auto fail = [&](const char* what) -> shdr_engine* {
        char buf[512];
        shdr_last_error(buf, sizeof buf);
        shdr::set_error(std::string("engine_create: ") + what + ": " + buf);
        shdr_engine_free(e);
        return nullptr;
    };
    if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice");
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    if (hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    if (hipStreamCreateWithFlags(&e->stream3, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    if (hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming) != hipSuccess)
        return fail("event");
    if (const char* c = getenv("SHDR_CONCURRENT_TAIL")) e->concurrent_tail = atoi(c) != 0;
    if (const char* c = getenv("SHDR_TAIL_FIRST")) e->tail_first = atoi(c) != 0;
    if (const char* c = getenv("SHDR_PASS")) e->single_pass = atoi(c) != 0;
    if (const char* c = getenv("SHDR_HALF_PAIRS")) e->half_pairs = atoi(c) != 0;
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
    {
        // packed arc blocks of the out-CSR (and of the in-CSR for the landmark
        // pre-pass on directed graphs, which relaxes the reversed graph); each
        // vertex's arcs in increasing weight (stable; neutral against the caller's
        // order, profiles/r03_defer_ab.log); relaxation order never changes results
        auto pack = [&](const std::vector<int64_t>& rp, const std::vector<int32_t>& cc, const std::vector<double>& ww,
                        uint64_t** dblk, int32_t** dfirst, int32_t* nout) -> bool {
            std::vector<int32_t> first(size_t(c.V) + 1);
            int64_t nb = 0;
            for (int32_t v = 0; v < c.V; ++v) { first[v] = int32_t(nb); nb += (rp[v + 1] - rp[v] + kChunk - 1) / kChunk; }
            if (nb >= (int64_t(1) << 31) - 1) return false;
            first[c.V] = int32_t(nb);
            std::vector<uint64_t> blk(size_t(nb + 1) * 16, 0);
            const uint64_t inf = 0x7FF0000000000000ull;
            auto put = [&](int64_t b, int q, int32_t col, uint64_t wbits) {
                uint64_t* p = blk.data() + size_t(b) * 16;
                p[q >> 1] |= uint64_t(uint32_t(col)) << (32 * (q & 1));
                p[4 + q] = wbits;
            };
            // vertices write disjoint blocks: filled by several host threads
            host_parallel(c.V, [&](int32_t v0, int32_t v1) {
                std::vector<int64_t> ord;
                for (int32_t v = v0; v < v1; ++v) {
                    ord.resize(size_t(rp[v + 1] - rp[v]));
                    for (size_t k = 0; k < ord.size(); ++k) ord[k] = rp[v] + int64_t(k);
                    std::stable_sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) { return ww[size_t(x)] < ww[size_t(y)]; });
                    for (int64_t b = first[v]; b < first[v + 1]; ++b)
                        for (int q = 0; q < kChunk; ++q) {
                            const int64_t k = (b - first[v]) * kChunk + q;
                            if (k < int64_t(ord.size())) {
                                const int64_t a = ord[size_t(k)];
                                uint64_t wb;
                                std::memcpy(&wb, &ww[size_t(a)], 8);
                                put(b, q, cc[size_t(a)], wb);
                            } else {
                                put(b, q, v, inf);
                            }
                        }
                }
            });
            for (int q = 0; q < kChunk; ++q) put(nb, q, 0, inf);
            // bit 31 of first[v]: v's last block holds at most kHalf real arcs (a half
            // block: relaxed paired with another half block)
            if (e->half_pairs)
                for (int32_t v = 0; v < c.V; ++v) {
                    const int64_t r = (rp[v + 1] - rp[v]) % kChunk;
                    if (r >= 1 && r <= kHalf) first[v] |= int32_t(kHalfBit);
                }
            *nout = int32_t(nb);
            return !upload(e, dblk, blk) && !upload(e, dfirst, first);
        };
        phase("upload");
        if (!pack(c.rowptr, c.col, c.w, &e->ablk, &e->bfirst, &e->nblk)) return fail("upload arc blocks");
        if (!c.same_in_out && !pack(c.irowptr, c.isrc, c.iw, &e->iablk, &e->ibfirst, &e->inblk))
            return fail("upload in-arc blocks");
    }
    // the landmark pre-pass (source grouping, partition) runs while the host
    // builds the predecessor items; it is collected at first use
    if (!e->complete && e->csr.V > 0) {
        if (landmark_launch(e, e->stream) != SHDR_OK) {
            // retried at first use when the failure was recoverable (device memory:
            // hipMalloc's error is not sticky); a sticky error (a faulted kernel)
            // fails the engine here instead of surfacing later at a query
            (void)hipGetLastError();
            if (const hipError_t se = hipStreamSynchronize(e->stream); se != hipSuccess) {
                shdr::set_error(std::string("landmark pre-pass: ") + hipGetErrorString(se));
                return fail("device error");
            }
            e->lm_pending = false;
        }
        phase("landmarks enqueued");
    }
    {
        // predecessor-pass items over the in-CSR (== out-CSR when undirected)
        const std::vector<int64_t>& irp = c.same_in_out ? c.rowptr : c.irowptr;
        // one item per kChunk in-arcs, at least one per vertex
        std::vector<int32_t> first(size_t(c.V) + 1);
        int64_t ni = 0;
        for (int32_t v = 0; v < c.V; ++v) {
            first[v] = int32_t(std::min<int64_t>(ni, INT32_MAX));
            ni += std::max<int64_t>(1, (irp[v + 1] - irp[v] + kChunk - 1) / kChunk);
        }
        if (ni >= (int64_t(1) << 31)) return fail("too many predecessor items");
        e->npitems = int32_t(ni);
        first[c.V] = e->npitems;
        std::vector<int4> items(static_cast<size_t>(ni));
        host_parallel(c.V, [&](int32_t v0, int32_t v1) {
            for (int32_t v = v0; v < v1; ++v) {
                const int64_t p0 = irp[v], p1 = irp[v + 1];
                int64_t p = p0;
                int32_t i = first[v];
                do {
                    const int32_t cnt = int32_t(std::min<int64_t>(kChunk, p1 - p));
                    const int fl = (p == p0 ? 1 : 0) | (p + cnt >= p1 ? 2 : 0);
                    items[size_t(i++)] = make_int4(v, int32_t(p), cnt, fl);
                    p += cnt;
                } while (p < p1);
            }
        });
        if (upload(e, &e->pitems, items) || upload(e, &e->pfirst, first)) return fail("upload items");
        phase("blocks+items");
    }
    return e;
}

void shdr_engine_free(shdr_engine* e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->stream2) (void)hipStreamSynchronize(e->stream2);
    if (e->stream3) (void)hipStreamSynchronize(e->stream3);
    for (void* p : e->owned) (void)hipFree(p);
    if (e->arena_raw) (void)hipFree(e->arena_raw);
    if (e->d_src) (void)hipFree(e->d_src);
    if (e->d_dst) (void)hipFree(e->d_dst);
    if (e->d_lat) (void)hipFree(e->d_lat);
    if (e->d_rel) (void)hipFree(e->d_rel);
    if (e->d_rowmin) (void)hipFree(e->d_rowmin);
    if (e->d_hops) (void)hipFree(e->d_hops);
    if (e->d_err) (void)hipFree(e->d_err);
    if (e->d_rowmap) (void)hipFree(e->d_rowmap);
    if (e->d_soff) (void)hipFree(e->d_soff);
    if (e->d_bcost) (void)hipFree(e->d_bcost);
    if (e->d_boff) (void)hipFree(e->d_boff);
    if (e->d_cl) (void)hipFree(e->d_cl);
    if (e->d_lm) (void)hipFree(e->d_lm);
    for (auto& ev : e->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    if (e->stream2) (void)hipStreamDestroy(e->stream2);
    if (e->stream3) (void)hipStreamDestroy(e->stream3);
    if (e->h_done) (void)hipHostFree(e->h_done);
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
    if (e->ev_join) (void)hipEventDestroy(e->ev_join);
    if (e->ev_pass) (void)hipEventDestroy(e->ev_pass);
    delete e;
}

int shdr_engine_set_variant(shdr_engine* e, int32_t variant) {
    if (!e || variant < 0 || variant >= int32_t(sizeof(kVariants) / sizeof(kVariants[0]))) {
        shdr::set_error("set_variant: bad argument");
        return SHDR_EINVAL;
    }
    e->variant = variant;
    return SHDR_OK;
}

int shdr_engine_set_delta(shdr_engine* e, double delta) {
    if (!e || !(delta >= 0.0)) { shdr::set_error("set_delta: bad argument"); return SHDR_EINVAL; }
    e->delta = delta;
    return SHDR_OK;
}

// Touch every page of large host ranges from several threads (MADV_POPULATE_WRITE
// where the kernel has it, else a write of one byte per page read back first, so
// the content is unchanged). Small ranges are left alone.
static void prefault_host(std::initializer_list<std::pair<void*, size_t>> ranges) {
    size_t total = 0;
    for (const auto& r : ranges) total += r.first ? r.second : 0;
    if (total < (size_t(256) << 20)) return;
    const long pg = sysconf(_SC_PAGESIZE) > 0 ? sysconf(_SC_PAGESIZE) : 4096;
    const int nt = std::max(1, std::min<int>(16, int(std::thread::hardware_concurrency())));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (const auto& r : ranges) {
                if (!r.first || !r.second) continue;
                char* b = static_cast<char*>(r.first);
                const size_t chunk = (r.second / nt + pg - 1) / pg * pg;
                char* lo = b + size_t(t) * chunk;
                char* hi = std::min(b + r.second, lo + chunk);
                if (lo >= hi) continue;
                char* alo = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(lo) + pg - 1) / pg * pg);
                // transparent huge pages where the host allows them (2 MB faults, not 4 KB)
                char* hlo = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(lo) + (size_t(2) << 20) - 1) >> 21 << 21);
                char* hhi = reinterpret_cast<char*>(reinterpret_cast<uintptr_t>(hi) >> 21 << 21);
                if (hlo < hhi) (void)madvise(hlo, size_t(hhi - hlo), 14 /* MADV_HUGEPAGE */);
                if (alo < hi && madvise(alo, size_t(hi - alo), 23 /* MADV_POPULATE_WRITE */) == 0) continue;
                for (volatile char* p = lo; p < hi; p += pg) *p = *p;
            }
        });
    for (auto& x : th) x.join();
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
    const int32_t* const src_in = src;
    const int32_t* const dst_in = dst;
    for (int32_t i = 0; i < S; ++i)
        if (src[i] < 0 || src[i] >= V) { shdr::set_error("routes_compute: source vertex out of range"); return SHDR_EINVAL; }
    for (int32_t j = 0; j < T; ++j)
        if (dst[j] < 0 || dst[j] >= V) { shdr::set_error("routes_compute: target vertex out of range"); return SHDR_EINVAL; }
    if (!e->newid.empty()) {  // into device numbering (rows and columns keep the caller's order)
        e->h_msrc.resize(size_t(S));
        e->h_mdst.resize(size_t(T));
        for (int32_t i = 0; i < S; ++i) e->h_msrc[i] = e->newid[src[i]];
        for (int32_t j = 0; j < T; ++j) e->h_mdst[j] = e->newid[dst[j]];
        src = e->h_msrc.data();
        dst = e->h_mdst.data();
    }
    e->tnames.clear();
    e->tms.clear();
    for (double& x : e->host_ms) x = 0.0;
    const auto th0 = std::chrono::steady_clock::now();
    {
        int rc0;
        if (e->lm_pending && (rc0 = landmark_collect(e))) return rc0;  // (it uses the arena)
    }
    auto host_since = [&](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    };
    e->kept = false;
    e->last_fallback = 0;
    e->last_reordered = false;
    e->last_progressive = false;
    e->last_S = S;
    if (S == 0 || T == 0) return SHDR_OK;
    int rc;
    if ((rc = ensure((void**)&e->d_src, &e->cap_src, size_t(S) * 4))) return rc;
    if ((rc = ensure((void**)&e->d_dst, &e->cap_dst, size_t(T) * 4))) return rc;
    HIPCHK(hipMemcpyAsync(e->d_src, src, size_t(S) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->d_dst, dst, size_t(T) * 4, hipMemcpyHostToDevice, st));
    RouteOut o{};
    o.T = T;
    const size_t npair = size_t(S) * T;
    if (dev_out) {
        o.lat = lat; o.rel = rel; o.hops = hops; o.row_min = row_min;
    } else {
        size_t cap = e->cap_out;
        if (cap < npair || !e->d_lat) {
            if (e->d_lat) { (void)hipFree(e->d_lat); (void)hipFree(e->d_rel); }
            e->d_lat = e->d_rel = nullptr;
            HIPCHK(hipMalloc((void**)&e->d_lat, npair * 8));
            HIPCHK(hipMalloc((void**)&e->d_rel, npair * 8));
            e->cap_out = npair;
        }
        if (hops && (rc = ensure((void**)&e->d_hops, &e->cap_hops, npair * 4))) return rc;
        if ((rc = ensure((void**)&e->d_rowmin, &e->cap_rowmin, size_t(S) * 8))) return rc;
        o.lat = e->d_lat; o.rel = e->d_rel; o.hops = hops ? e->d_hops : nullptr; o.row_min = e->d_rowmin;
    }
    const bool jitter = flags & SHDR_PATH_JITTER;
    if (jitter && !e->ocjit) {
        const shdr::CsrImage& c = e->csr;
        if (c.ocjit.size() != size_t(c.A) || (!c.same_in_out && c.icjit.size() != size_t(c.A))) {
            shdr::set_error("routes_compute: SHDR_PATH_JITTER needs a numeric edge attribute 'jitter'");
            return SHDR_EINVAL;
        }
        if (upload(e, &e->ocjit, c.ocjit)) return SHDR_EHIP;
        if (!c.same_in_out && upload(e, &e->icjit, c.icjit)) return SHDR_EHIP;
    }
    DevGraph g = devgraph(e, jitter);
    const bool use_direct = e->complete && !(flags & (SHDR_FORCE_SSSP | SHDR_PATH_JITTER));
    bool prog = false;  // progressive host copy of this compute (below)
    int32_t prog_nb = 0;
    std::vector<int32_t> prog_rows;  // main-launch bucket b = processed rows [prog_rows[b], prog_rows[b+1])
    if (use_direct) {
        if (o.row_min) {
            hipLaunchKernelGGL(k_fill_f64, dim3(std::max(1, std::min(1024, (S + 255) / 256))), dim3(256), 0, st,
                               o.row_min, size_t(S), __builtin_inf());
        }
        dim3 grid(std::max(1, std::min((T + 255) / 256, 64)), std::min(S, 65535));
        if ((rc = record(e, 0, timing, st))) return rc;
        hipLaunchKernelGGL(k_routes_direct, grid, dim3(256), 0, st, g, e->d_src, e->d_dst, S, o);
        HIPCHK(hipGetLastError());
        if ((rc = record(e, 1, timing, st))) return rc;
    } else {
        // Bucket layout. A bucket costs about the same whatever its fill (its
        // rounds and row gathers are set by the graph, not by the lane count), so
        // rows run in full K-wide buckets and the partial last wave in a
        // half-width tail launch (below). A shard smaller than one wave of
        // half-width buckets (strong scaling: cfg4 over 8 GPUs is 1,250 rows for
        // 256 CUs) runs balanced instead: half-width buckets of S/256 sources so
        // that every CU works (cfg4 1,250 rows: 16.8 ms against 18.9 for 157
        // full K=8 buckets and 21.0 for balanced K=16; tools/ab.py, same box).
        struct VarGuard { shdr_engine* e; int v; ~VarGuard() { e->variant = v; } } var_guard{e, e->variant};
        e->cur_cl = 1;
        // Cluster mode (several workgroups per bucket): forced by SHDR_CLUSTER >= 2,
        // or automatic (0) for a shard whose full-width buckets fill at most half of
        // the resident slots (strong scaling: cfg4 over 8 GPUs = 79 buckets on 256
        // CUs): cl = slots / buckets, at most kAutoCluster. With enough buckets
        // plain workgroups win (a cluster's rounds end in cross-CU barriers: cfg5's
        // 6,250-row shard 350 ms plain vs 442 / 411 ms at cl 2 / 4).
        //
        // The automatic width comes from a wave model: a bucket takes about the same
        // time t whatever its fill, a cl-wide cluster runs one in ~ t / (0.7 cl)
        // (measured: cfg4 shards 0.68-0.77, cfg5 6,250-row shard 0.72-0.75), and
        // buckets run in whole waves of the resident slots, so plain ~ ceil(nb /
        // slots) t and cluster ~ ceil(S / (K clusters)) t / (0.7 cl); the smallest
        // wins (cfg4 over 4 GPUs: 157 buckets -> cl 3, 26.0 -> 22.5 ms; cfg5 shards
        // stay plain: 1.53 waves plain against 4-7 waves of clusters).
        int want_cl = e->cluster;
        if (want_cl == 0 && !keep && e->order_mode > 0 && !e->shared_device) {
            want_cl = 1;
            const int K = kVariants[e->variant].K;
            const int64_t nbk = (S + K - 1) / K, slots = resident_slots(e, e->variant);
            const PendingMode pmd = pending_mode(e, e->variant);
            if (nbk >= 8 && slots > 0 && cluster_occupancy(e->variant, pmd.pm, pmd.dyn) > 0) {  // (tiny tables: not worth the barriers)
                double best = double((nbk + slots - 1) / slots);
                for (int c = 2; c <= kAutoCluster; ++c) {
                    const int64_t cs = cluster_slots(e, e->variant, c);
                    if (cs < 1) continue;
                    const double t = double((S + int64_t(K) * cs - 1) / (int64_t(K) * cs)) / (0.7 * c);
                    if (t < best) { best = t; want_cl = c; }
                }
            }
        }
        if (!keep && want_cl >= 2) {
            const PendingMode pmd = pending_mode(e, e->variant);
            if (cluster_occupancy(e->variant, pmd.pm, pmd.dyn) > 0 && cluster_slots(e, e->variant, want_cl) >= 1)
                e->cur_cl = want_cl;
        }
        e->cur_balance = e->balance == 1 || e->cur_cl > 1;
        if (e->cur_cl == 1 && e->balance == 2 && !keep) {
            const int tv = tail_variant(e->variant);
            if (tv >= 0 && int64_t(S) <= int64_t(kVariants[tv].K) * resident_slots(e, tv)) {
                e->variant = tv;
                e->cur_balance = 1;
            }
        }
        // KEEP_TREES rows are read back by processed index: keep the caller's order
        const bool reorder = !keep && e->order_mode > 0 && S >= 2 * kVariants[e->variant].K;
        {
            const auto tg0 = std::chrono::steady_clock::now();
            if (reorder && (rc = order_sources(e, st, src, S))) return rc;
            e->host_ms[1] = host_since(tg0);  // (includes a landmark pre-pass run here, host_ms[0])
        }
        e->last_reordered = reorder;
        const bool balanced = reorder && e->cur_balance;
        if (reorder) {
            HIPCHK(hipMemcpyAsync(e->d_src, e->h_src_sorted.data(), size_t(S) * 4, hipMemcpyHostToDevice, st));
            o.rowmap = e->d_rowmap;
            o.soff = e->order_mode == 2 ? e->d_soff : nullptr;
            if (balanced || e->partial_first) { o.boff = e->d_boff; o.nb = e->ngroups; }
        }
        // Tail balancing: buckets run ~one per resident slot at a time, so S/K
        // buckets leave a last partial wave. With at least two full waves (cfg4:
        // 2 + 113/256, cfg5: 12 + 53/256) and that wave at most half full, its
        // sources go into half-width buckets (K/2) that fill the wave instead, in a
        // concurrent launch (cfg4 -3 %, 7 of 7 same-box pairs; cfg5 -2 %). With a
        // single full wave the half-width buckets' lower row sharing is not
        // repaid (untested).
        int32_t S1 = S;
        int tvar = tail_variant(e->variant);
        e->tail_cl = 1;
        if (reorder && !balanced && tvar >= 0) {
            const int K = kVariants[e->variant].K;
            const int64_t slots = resident_slots(e, e->variant);
            const int64_t nb = (S + K - 1) / K, waves = nb / slots, rem = nb - waves * slots;
            // Cluster tail (SHDR_CLUSTER_TAIL=1, off by default): the last rem <=
            // slots/2 full-width buckets run after the full waves with cl = slots /
            // rem workgroups each (at most kAutoCluster). A cl = 4 bucket takes ~1/3
            // of a plain one, but the launch must wait for the slowest main
            // workgroup (the main launch's exits spread over ~150 ms on cfg5), so it
            // measured slower than the concurrent half-width tail: cfg5 2361 vs 2239
            // ms, 25k / 12.5k-row shards 1247 / 701 vs 1218 / 664 ms, cfg4 73.6 vs
            // 71.3 ms (profiles/r02_cluster_tail_ab.log).
            const PendingMode pmd = pending_mode(e, e->variant);
            const int ct = int(std::min<int64_t>(kAutoCluster, rem > 0 ? slots / rem : 0));
            if (e->cluster_tail && waves >= 1 && ct >= 2 && e->cluster != 1 && !e->shared_device &&
                cluster_occupancy(e->variant, pmd.pm, pmd.dyn) > 0 && cluster_slots(e, e->variant, ct) >= rem) {
                S1 = int32_t(waves * slots * K);
                tvar = e->variant;
                e->tail_cl = ct;
            } else if (waves >= e->tail_min_waves && rem > 0 && 2 * rem <= slots) {
                S1 = int32_t(waves * slots * K);
            }
            if (e->partial_first && S1 < S) {  // the main launch = the first waves * slots groups
                S1 = e->h_boff[size_t(waves * slots)];
                o.nb = int32_t(waves * slots);
            }
        }
        if ((rc = reset_err(e, st))) return rc;
        // Main-launch bucket durations feed the next pass's issue order (same source
        // list). Automatic (-1): on for a main launch of at most 4 waves of buckets,
        // where the last wave's fill is set by a few long buckets (cfg5 shards over 4 / 8
        // GPUs -0.3 to -2.5 %, cfg4 over 4 -0.5 to -3 % on two boxes; 6 waves and more, and
        // the full cfg4 table, neutral; profiles/r04_profile_order_*.log).
        e->cost_buckets = 0;
        const int32_t nb1 = balanced ? e->ngroups : (S1 + kVariants[e->variant].K - 1) / kVariants[e->variant].K;
        const int64_t wslots = e->cur_cl > 1 ? cluster_slots(e, e->variant, e->cur_cl) : resident_slots(e, e->variant);
        if (reorder && (e->profile_order > 0 || (e->profile_order < 0 && wslots > 0 && nb1 <= 4 * wslots))) {
            if ((rc = ensure((void**)&e->d_bcost, &e->cap_bcost, size_t(nb1) * 4))) return rc;
            o.bcost = e->d_bcost;
            e->cost_buckets = nb1;
        }
        // progressive host copy: rows in processing order (the host scatters them to
        // the caller's rows), main-launch buckets flag their completion
        prog = !dev_out && reorder && !keep && !hops && e->progressive && npair * 8 >= e->prog_min &&
               e->h_perm.size() == size_t(S);
        if (prog) {
            prog_nb = o.boff ? o.nb : (S1 + kVariants[e->variant].K - 1) / kVariants[e->variant].K;
            if (e->cap_done < size_t(prog_nb) || !e->h_done) {
                if (e->h_done) HIPCHK(hipHostFree(e->h_done));
                e->h_done = nullptr;
                e->cap_done = 0;
                HIPCHK(hipHostMalloc((void**)&e->h_done, std::max<size_t>(size_t(prog_nb), 1) * 4, hipHostMallocMapped));
                e->cap_done = size_t(prog_nb);
            }
            std::memset(e->h_done, 0, size_t(prog_nb) * 4);
            uint32_t* dptr = nullptr;
            HIPCHK(hipHostGetDevicePointer((void**)&dptr, e->h_done, 0));
            o.done = dptr;
            o.rowmap = nullptr;
            prog_rows.resize(size_t(prog_nb) + 1);
            const int K = kVariants[e->variant].K;
            for (int32_t b = 0; b <= prog_nb; ++b) prog_rows[size_t(b)] = o.boff ? e->h_boff[size_t(b)] : std::min(b * K, S1);
        }
        RouteOut o2 = o;
        o2.bcost = nullptr;
        o2.boff = nullptr;
        o2.done = nullptr;
        o2.rowmap = o.rowmap ? o.rowmap + S1 : nullptr;
        o2.soff = o.soff ? o.soff + S1 : nullptr;
        if (prog) {  // the tail's rows follow the main launch's in processing order
            o2.lat = o.lat + size_t(S1) * T;
            o2.rel = o.rel + size_t(S1) * T;
            if (o2.row_min) o2.row_min = o.row_min + S1;
        }
        // The tail runs CONCURRENTLY on a second stream in its own arena region:
        // its workgroups take the CUs that main workgroups leave as the bucket
        // queue runs dry, instead of waiting for the slowest main workgroup.
        e->tail_concurrent = false;
        e->last_tail_mode = 0;
        if (S1 < S && e->concurrent_tail && e->tail_cl == 1) {
            const ArenaLayout Lm = layout_for(e->csr.V, e->csr.A, kVariants[e->variant].K);
            const ArenaLayout Lt = layout_for(e->csr.V, e->csr.A, kVariants[tvar].K);
            const int32_t sm = launch_slots(e, e->variant, S1), stl = launch_slots(e, tvar, S - S1);
            const size_t off_t = size_t(sm) * Lm.stride, bytes = off_t + size_t(stl) * Lt.stride;
            rc = ensure_arena(e, bytes);
            if (rc && rc != SHDR_ENOMEM) return rc;
            const PendingMode pm_m = pending_mode(e, e->variant), pm_t = pending_mode(e, tvar);
            const bool one = !rc && e->single_pass && !keep && pm_m.pm == pm_t.pm && pm_m.dyn == pm_t.dyn &&
                             stl <= sm && pass_fits(e->variant, pm_m.pm, pm_m.dyn, with_variant<OccF>(e->variant, pm_m.pm, pm_m.dyn));
            if (one) {
                // one launch: blocks [0, stl) run the tail's half-width buckets first
                if ((rc = record(e, 0, timing, st))) return rc;
                if ((rc = run_pass(e, st, g, e->variant, S1, sm, o, S, stl, off_t, o2))) return rc;
                if ((rc = record(e, 1, timing, st))) return rc;
                if ((rc = record(e, 2, timing, st))) return rc;
                if ((rc = record(e, 3, timing, st))) return rc;
                e->tail_concurrent = true;
                e->last_tail_mode = 3;
            } else if (!rc) {
                HIPCHK(hipEventRecord(e->ev_fork, st));
                HIPCHK(hipStreamWaitEvent(e->stream2, e->ev_fork, 0));
                if ((rc = record(e, 0, timing, st))) return rc;
                auto main_launch = [&]() -> int {
                    int r = run_sssp(e, st, g, e->d_src, S1, e->d_dst, o, keep, 0, -1, sm, 0, 0);
                    return r ? r : record(e, 1, timing, st);
                };
                auto tail_launch = [&]() -> int {
                    int r = run_sssp(e, e->stream2, g, e->d_src + S1, S - S1, e->d_dst, o2, false, 1, tvar, stl, off_t, 1);
                    return r ? r : record(e, 2, timing, e->stream2);
                };
                // submission order decides which launch takes the CUs first (SHDR_TAIL_FIRST)
                if (e->tail_first) {
                    if ((rc = tail_launch())) return rc;
                    hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, st, uint32_t(2000));  // 20 us
                    HIPCHK(hipGetLastError());
                    if ((rc = main_launch())) return rc;
                } else {
                    if ((rc = main_launch()) || (rc = tail_launch())) return rc;
                }
                HIPCHK(hipEventRecord(e->ev_join, e->stream2));
                HIPCHK(hipStreamWaitEvent(st, e->ev_join, 0));
                if ((rc = record(e, 3, timing, st))) return rc;
                e->tail_concurrent = true;
                e->last_tail_mode = 2;
            }
            rc = SHDR_OK;
        }
        if (!e->tail_concurrent) {
            if ((rc = record(e, 0, timing, st))) return rc;
            if ((rc = run_sssp(e, st, g, e->d_src, S1, e->d_dst, o, keep))) return rc;
            if ((rc = record(e, 1, timing, st))) return rc;
            if (S1 < S) {
                if ((rc = run_sssp(e, st, g, e->d_src + S1, S - S1, e->d_dst, o2, false, 1, tvar, -1, 0, 1, e->tail_cl)))
                    return rc;
                if ((rc = record(e, 2, timing, st))) return rc;
                e->last_tail_mode = 1;
            }
            if ((rc = record(e, 3, timing, st))) return rc;
        }
        e->last_rows_main = S1;
        e->last_variant = e->variant;
        e->last_partial_first = reorder && !balanced && e->partial_first;
    }
    e->host_ms[2] = host_since(th0);
    e->last_progressive = prog;
    if (prog) {
        // progressive copy (the launch still runs): fault the destination pages in,
        // then copy finished rows as their buckets flag completion
        prefault_host({{lat, npair * 8}, {rel, npair * 8}});
        if (!e->ev_pass) HIPCHK(hipEventCreateWithFlags(&e->ev_pass, hipEventDisableTiming));
        HIPCHK(hipEventRecord(e->ev_pass, st));
        const size_t chunk_rows = std::max<size_t>(1, e->prog_chunk / (size_t(T) * 8));
        // staging for one chunk of lat and one of rel rows; T changes between computes
        // on one engine (drop-in blocks, Python callers), so grow it when this T needs more
        const size_t stage_bytes = 2 * chunk_rows * size_t(T) * 8;
        if (e->h_stage && e->cap_stage < stage_bytes) {
            HIPCHK(hipHostFree(e->h_stage));
            e->h_stage = nullptr;
            e->cap_stage = 0;
        }
        if (!e->h_stage) {
            HIPCHK(hipHostMalloc((void**)&e->h_stage, stage_bytes, hipHostMallocDefault));
            e->cap_stage = stage_bytes;
        }
        const std::vector<int32_t>& perm = e->h_perm;
        const int nth = std::max(1, std::min<int>(16, int(std::thread::hardware_concurrency())));
        auto copy_rows = [&](int32_t r0, int32_t r1) -> int {  // processed rows [r0, r1) -> caller rows
            for (int32_t c0 = r0; c0 < r1; c0 += int32_t(chunk_rows)) {
                const int32_t c1 = std::min<int32_t>(r1, c0 + int32_t(chunk_rows));
                const size_t bytes = size_t(c1 - c0) * T * 8;
                double* sl = e->h_stage;
                double* sr = e->h_stage + chunk_rows * size_t(T);
                HIPCHK(hipMemcpyAsync(sl, o.lat + size_t(c0) * T, bytes, hipMemcpyDeviceToHost, e->stream3));
                HIPCHK(hipMemcpyAsync(sr, o.rel + size_t(c0) * T, bytes, hipMemcpyDeviceToHost, e->stream3));
                HIPCHK(hipStreamSynchronize(e->stream3));
                std::vector<std::thread> th;
                for (int t = 0; t < nth; ++t)
                    th.emplace_back([&, t] {
                        for (int32_t k = c0 + t; k < c1; k += nth) {
                            const size_t dst = size_t(perm[size_t(k)]) * T, src = size_t(k - c0) * T;
                            std::memcpy(lat + dst, sl + src, size_t(T) * 8);
                            std::memcpy(rel + dst, sr + src, size_t(T) * 8);
                        }
                    });
                for (auto& x : th) x.join();
            }
            return SHDR_OK;
        };
        int32_t P = 0, copied = 0;
        const volatile uint32_t* done = e->h_done;
        for (;;) {
            while (P < prog_nb && done[P]) ++P;
            const int32_t ready = prog_rows[size_t(P)];
            if (ready > copied && (size_t(ready - copied) >= chunk_rows || P == prog_nb)) {
                if ((rc = copy_rows(copied, ready))) return rc;
                copied = ready;
            }
            if (P == prog_nb) break;
            const hipError_t q = hipEventQuery(e->ev_pass);
            if (q != hipErrorNotReady) break;  // finished (a guard may have stopped buckets) or failed
            usleep(200);
        }
        HIPCHK(hipEventSynchronize(e->ev_pass));
        e->host_ms[3] = host_since(th0) - e->host_ms[2];
        const auto td0 = std::chrono::steady_clock::now();
        if ((rc = copy_rows(copied, S))) return rc;  // the rest (tail launch rows)
        if (row_min) {
            std::vector<double> rm(static_cast<size_t>(S));
            HIPCHK(hipMemcpyAsync(rm.data(), o.row_min, size_t(S) * 8, hipMemcpyDeviceToHost, e->stream3));
            HIPCHK(hipStreamSynchronize(e->stream3));
            for (int32_t k = 0; k < S; ++k) row_min[perm[size_t(k)]] = rm[size_t(k)];
        }
        e->host_ms[4] = host_since(td0);
    } else if (!dev_out) {
        // Host outputs: fault the destination pages in (16 threads) while the kernels
        // run. A pageable D2H into fresh memory runs at 11 GB/s (the copy faults every
        // page), into faulted memory at 25 GB/s (tools/d2h_bench.py): for cfg5's 40 GB
        // table the drop-in's first query saves ~2 s.
        prefault_host({{lat, npair * 8}, {rel, npair * 8}, {hops, hops ? npair * 4 : 0}});
        if (!e->ev_pass) HIPCHK(hipEventCreateWithFlags(&e->ev_pass, hipEventDisableTiming));
        HIPCHK(hipEventRecord(e->ev_pass, st));
        HIPCHK(hipEventSynchronize(e->ev_pass));
        e->host_ms[3] = host_since(th0) - e->host_ms[2];
        const auto td0 = std::chrono::steady_clock::now();
        HIPCHK(hipMemcpyAsync(lat, o.lat, npair * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(rel, o.rel, npair * 8, hipMemcpyDeviceToHost, st));
        if (hops) HIPCHK(hipMemcpyAsync(hops, o.hops, npair * 4, hipMemcpyDeviceToHost, st));
        if (row_min) HIPCHK(hipMemcpyAsync(row_min, o.row_min, size_t(S) * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        e->host_ms[4] = host_since(td0);
    }
    HIPCHK(hipStreamSynchronize(st));
    if (dev_out) e->host_ms[3] = host_since(th0) - e->host_ms[2];
    if (!use_direct) {
        int herr = 0;
        HIPCHK(hipMemcpy(&herr, e->d_err, sizeof(int), hipMemcpyDeviceToHost));
        if (herr && (e->cur_cl > 1 || e->tail_cl > 1) && (herr & ~(8 | 16)) == 0) {
            // a cluster member never arrived (its workgroups were not all resident:
            // another launch held CUs) or a cluster spanned two XCDs: placement, not
            // results, so recompute with one workgroup per bucket (counted:
            // shdr_engine_last_layout out[6] / out[7]). Any other guard code fails
            // the compute below like in a plain launch: a recompute would hide it.
            std::fprintf(stderr, "[shdr] cluster %s (guard %d): cluster mode off for this engine\n",
                         (herr & 16) ? "members on different XCDs" : "barrier timed out", herr);
            e->cluster = 1;
            e->flags_dirty = true;
            const int rc2 = shdr_routes_compute(e, src_in, S, dst_in, T, lat, rel, hops, row_min, flags, stream_v);
            e->last_fallback = herr;
            ++e->fallbacks;
            return rc2;
        }
        if (herr) {
            e->flags_dirty = true;
            int rec[kErrWords] = {};
            HIPCHK(hipMemcpy(rec, e->d_err, sizeof rec, hipMemcpyDeviceToHost));
            std::string first;
            if (rec[4]) {
                first = "; first trip: code " + std::to_string(rec[5]) + " fields";
                for (int i = 6; i < 15; ++i) first += " " + std::to_string(rec[i]);
            }
            shdr::set_error("routes_compute: device guard tripped (code " + std::to_string(herr) +
                            ": 1=round limit, 2=work-list overflow, 4=broken predecessor chain, "
                            "8=cluster barrier timeout, 16=cluster across XCDs, 32=unwritten predecessor entry, "
                            "64=bucket record or source out of range, 2048=pending vertex or bucket index out of range, "
                            "128/512=SHDR_VERIFY invariant, 256/512/1024=index check of a SHDR_BCHK build" +
                            first + ")");
            return SHDR_EHIP;
        }
        if (e->cost_buckets > 0) {
            std::vector<uint32_t> bc(static_cast<size_t>(e->cost_buckets));
            HIPCHK(hipMemcpy(bc.data(), e->d_bcost, bc.size() * 4, hipMemcpyDeviceToHost));
            for (size_t b = 0; b < bc.size() && b < e->border.size(); ++b) e->gcost[e->border[b]] = float(bc[b]);
            e->costs_fresh = true;
            e->cost_buckets = 0;
        }
    }
    e->host_ms[5] = host_since(th0);
    {
        static const char* const kHost[6] = {"host_landmarks", "host_grouping", "host_launch", "host_pass", "host_d2h",
                                             "host_total"};
        for (int i = 0; i < 6; ++i) { e->tnames.push_back(kHost[i]); e->tms.push_back(float(e->host_ms[i])); }
    }
    if (timing) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, e->ev[0], e->ev[1]));
        // (named like the kernel symbol, as rocprofv3 reports it: the PMC summaries key on it)
        e->tnames.push_back(use_direct ? "k_routes_direct" : e->last_tail_mode == 3 ? "k_routes_pass" : "k_routes_sssp");
        e->tms.push_back(ms);
        if (!use_direct && e->last_rows_main < S && e->last_tail_mode != 3) {
            // concurrent: from the fork (the tail queues behind main for CUs)
            HIPCHK(hipEventElapsedTime(&ms, e->tail_concurrent ? e->ev[0] : e->ev[1], e->ev[2]));
            e->tnames.push_back("k_routes_sssp_tail");
            e->tms.push_back(ms);
        }
        if (!use_direct) {
            HIPCHK(hipEventElapsedTime(&ms, e->ev[0], e->ev[3]));
            e->tnames.push_back("routes_pass");
            e->tms.push_back(ms);
        }
    }
    return SHDR_OK;
}

int shdr_engine_partition(shdr_engine* e, const int32_t* src, int32_t S, int32_t nparts, int32_t* part) {
    if (!e || S < 0 || nparts < 1 || (S > 0 && (!src || !part))) {
        shdr::set_error("engine_partition: bad arguments");
        return SHDR_EINVAL;
    }
    const int32_t V = e->csr.V;
    for (int32_t i = 0; i < S; ++i)
        if (src[i] < 0 || src[i] >= V) { shdr::set_error("engine_partition: source vertex out of range"); return SHDR_EINVAL; }
    std::vector<int32_t> psize(static_cast<size_t>(nparts));
    for (int32_t p = 0; p < nparts; ++p) psize[p] = S / nparts + (p < S % nparts ? 1 : 0);
    if (e->complete || S < 2 * nparts) {  // no landmark embedding (direct-edge branch) or trivial: blocks
        int32_t i = 0;
        for (int32_t p = 0; p < nparts; ++p)
            for (int32_t k = 0; k < psize[p]; ++k) part[i++] = p;
        return SHDR_OK;
    }
    // kd regions of the landmark embedding, m per part, dealt round-robin in kd
    // order: each region is dense (its buckets group as tightly as the whole list's)
    // while every part mixes regions from all over the embedding, so part costs even
    // out (one region per part left the costliest part 1.4x the mean on cfg5 / 8).
    // Regions of at least 256 sources (16 full buckets), at most 16 per part.
    int64_t mmax = 16;
#ifdef SHDR_EXPERIMENTS
    if (const char* x = getenv("SHDR_PART_REGIONS")) mmax = std::max(1, atoi(x));
#endif
    const int32_t m = int32_t(std::max<int64_t>(1, std::min<int64_t>(mmax, int64_t(S) / (int64_t(nparts) * 256))));
    const int32_t R = nparts * m;
    std::vector<int32_t> gstart(size_t(R) + 1, 0);
    for (int32_t r = 0; r < R; ++r) {
        const int32_t p = r % nparts, k = r / nparts;  // region k of part p
        gstart[r + 1] = gstart[r] + psize[p] / m + (k < psize[p] % m ? 1 : 0);
    }
    HIPCHK(hipSetDevice(e->device));
    std::vector<int32_t> msrc(src, src + S);
    int rc;
    if (e->lm_pending && (rc = landmark_collect(e))) return rc;
    if (!e->newid.empty())
        for (int32_t& x : msrc) x = e->newid[x];
    if (!e->lm_ready && (rc = landmark_prepass(e, e->stream))) return rc;
    std::vector<int32_t> idx(static_cast<size_t>(S));
    for (int32_t i = 0; i < S; ++i) idx[i] = i;
    kd_groups(e, msrc.data(), idx, gstart, 0, size_t(R));
    for (int32_t r = 0; r < R; ++r)
        for (int32_t i = gstart[r]; i < gstart[r + 1]; ++i) part[idx[i]] = r % nparts;
    return SHDR_OK;
}

int shdr_engine_pred_tree(shdr_engine* e, int32_t i, int32_t* pred_vertex, double* dist) {
    if (!e || !e->kept || i < 0 || i >= e->kept_S) { shdr::set_error("pred_tree: no kept tree for that row (use SHDR_KEEP_TREES)"); return SHDR_EINVAL; }
    HIPCHK(hipSetDevice(e->device));
    if (e->lm_pending) { const int rc = landmark_collect(e); if (rc) return rc; }
    const int K = e->kept_K;
    const int32_t V = e->csr.V;
    const int32_t b = i / K, l = i % K;
    char* base = e->arena + size_t(b) * e->kept_stride;
    std::vector<uint64_t> drow(size_t(V) * K);
    std::vector<int2> prow(size_t(V) * K);
    if (dist) HIPCHK(hipMemcpy(drow.data(), base, drow.size() * 8, hipMemcpyDeviceToHost));
    if (pred_vertex) HIPCHK(hipMemcpy(prow.data(), base + e->kept_off_pred, prow.size() * sizeof(int2), hipMemcpyDeviceToHost));
    const bool m = !e->oldid.empty();  // report in the caller's numbering
    for (int32_t v = 0; v < V; ++v) {
        const int32_t dv = m ? e->newid[v] : v;
        if (dist) memcpy(&dist[v], &drow[size_t(dv) * K + l], 8);
        if (pred_vertex) {
            const int32_t p = prow[size_t(dv) * K + l].x;
            pred_vertex[v] = (m && p >= 0 && p < V) ? e->oldid[p] : p;
        }
    }
    return SHDR_OK;
}

#ifdef SHDR_DIAG
int shdr_diag_read(unsigned long long* out, int n, int reset) {
    unsigned long long h[32] = {0};
    HIPCHK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_diag), sizeof h));
    for (int i = 0; i < n && i < 32; ++i) out[i] = h[i];
    if (reset) {
        unsigned long long z[32] = {0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_diag), z, sizeof z));
    }
    return SHDR_OK;
}
int shdr_diag_order(shdr_engine* e, int32_t* out, int n) {
    for (int i = 0; i < n && i < int(e->h_src_sorted.size()); ++i) out[i] = e->h_src_sorted[i];
    return int(e->h_src_sorted.size());
}
int shdr_diag_buckets(unsigned long long* start, unsigned long long* dur, int n) {
    static unsigned long long h[2][8192];
    HIPCHK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_bticks), sizeof h));
    for (int i = 0; i < n && i < 8192; ++i) { start[i] = h[0][i]; dur[i] = h[1][i]; }
    return SHDR_OK;
}
#endif

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

int shdr_engine_last_layout(shdr_engine* e, int32_t* out, int32_t n) {
    if (!e || !out || n < 0) { shdr::set_error("last_layout: bad arguments"); return SHDR_EINVAL; }
    const int32_t v[10] = {e->last_variant, e->cur_cl, e->cur_balance, e->last_rows_main, e->tail_cl,
                           e->last_partial_first ? 1 : 0, e->last_fallback, int32_t(std::min<int64_t>(e->fallbacks, INT32_MAX)),
                           e->last_progressive ? 1 : 0, e->last_tail_mode};
    for (int32_t i = 0; i < n && i < 10; ++i) out[i] = v[i];
    return SHDR_OK;
}

int32_t shdr_engine_row_order(shdr_engine* e, int32_t* out, int32_t n) {
    if (!e || n < 0 || (n > 0 && !out)) { shdr::set_error("row_order: bad arguments"); return SHDR_EINVAL; }
    const int32_t S = e->last_S;
    const bool perm = e->last_reordered && e->h_perm.size() == size_t(S);
    for (int32_t k = 0; k < n && k < S; ++k) out[k] = perm ? e->h_perm[size_t(k)] : k;
    return S;
}

}  // extern "C"
