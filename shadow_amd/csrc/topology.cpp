// Drop-in implementation of Shadow's routing API (include/shd_topology.h).
//
// Mirrors /root/reference/src/main/routing/shd-topology.c function by function;
// the difference is WHEN paths are computed and WHERE:
//   * the reference runs one igraph Dijkstra per source on the first cache miss
//     (:775-939), serialised under graphLock (:859-893);
//   * here the first query after attach computes the whole table for every
//     attached source x attached target on the MI355X engine(s) through the
//     shdr_* C-ABI, once, and later queries are lock-free reads.
// What a caller can observe is kept identical:
//   * values: complete graphs use the direct edge (:941-979), others the
//     shortest path + ordered epilogue (:663-773);
//   * the path cache's history: a row (SSSP branch) or pair (complete branch)
//     is "revealed" exactly when the reference would have cached it, and for
//     undirected graphs a miss on (s,d) first answers from a revealed (d,s)
//     (:1001-1004), so the same reversed-path value is returned;
//   * the min-latency upcall (:602-613): worker_updateMinTimeJump is called
//     with the running minimum each time a reveal lowers it.
#include <algorithm>
#include <arpa/inet.h>
#include <chrono>
#include <unistd.h>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/shd_topology.h"
#include "../../include/shdr.h"
#include "graph.hpp"

namespace shdr {
HostGraph* host_of(shdr_graph* g);
}

namespace {

int log_level() {
    static int lvl = [] {
        const char* s = getenv("SHDTOP_LOG");
        return s ? atoi(s) : 1;  // 0 silent, 1 critical/warning, 2 message, 3 info
    }();
    return lvl;
}

void logf(int lvl, const char* tag, const char* fmt, ...) {
    if (lvl > log_level()) return;
    va_list ap;
    va_start(ap, fmt);
    fprintf(stderr, "[shd-topology] %s: ", tag);
    vfprintf(stderr, fmt, ap);
    fputc('\n', stderr);
    va_end(ap);
}
#define critical(...) logf(1, "critical", __VA_ARGS__)
#define warning(...) logf(1, "warning", __VA_ARGS__)
#define message(...) logf(2, "message", __VA_ARGS__)
#define info(...) logf(3, "info", __VA_ARGS__)

// Rows [b * B, b * B + rows) of a table, computed together (one engine pass).
struct Block {
    std::unique_ptr<double[]> lat, rel;  // [rows][n]; written whole by the engine(s), never pre-filled
    std::vector<double> rowMin;
};

// Route table over the attached vertex set of one attach epoch. Its row blocks
// are computed on demand (the block holding a row, the first time a query needs
// one of its rows) and are immutable once published; whole-table mode is one
// block. Block mode (B < n) bounds the host memory of ONE table by the rows
// actually used, as the reference's per-source rows do (shd-topology.c:775-939):
// it is selected when the whole table would exceed a fraction of host RAM. The
// bound is per table: tables of earlier attach epochs keep their computed
// blocks until topology_free, because rows revealed with them keep answering
// from them (the path cache's history), so a run that changes the attached set
// many times after revealing rows holds the sum of those tables' used blocks.
struct Table {
    std::vector<int32_t> srcV, dstV;   // distinct attached vertices: rows (engine-partition order), cols (sorted)
    std::vector<int32_t> rowOf, colOf; // vertex -> row / column index, or -1
    int32_t n = 0;
    int32_t nblk = 0;
    int32_t G = 1;                        // engines a block's rows are split over
    std::vector<int32_t> pstart;          // row offsets of the nblk * G parts (block b = parts [bG, bG + G))
    std::vector<int32_t> rowBlk;          // row -> block
    std::unique_ptr<std::atomic<const Block*>[]> blocks;
    std::vector<std::unique_ptr<Block>> owned;  // (appended under computeLock)
    uint64_t epoch = 0;  // attachEpoch of the attached vertex set it was computed for
    bool ok = false;
    int32_t first_row(int32_t b) const { return pstart[size_t(b) * G]; }
    const Block* block(int32_t row) const { return blocks[size_t(rowBlk[size_t(row)])].load(std::memory_order_acquire); }
};

}  // namespace

namespace {
struct AttachIndex;
// One entry of a source row's reveal history: the tables (attach epochs) the row
// was computed with, newest first. The reference's source cache only ever gains
// entries (g_hash_table_replace per stored target, :575-600), so a pair (s, d)
// is cached iff d was a target of ANY computation of s's row: the union of the
// target sets. Nodes are immutable and live until topology_free.
struct Reveal {
    const Table* t;
    const Reveal* next;
};
struct VipSnapshot {
    uint64_t version;
    std::unordered_map<uint32_t, int32_t> map;
};
constexpr size_t kMaxSnapshots = 64;
// topology_debug_lastComputeTimes slots: engine creation (ms, the call that made
// them), the last block's wall time (ms) and rows, then the first engine's host
// phases of that block (shdr_engine_timing names below)
enum { kTimeCreate = 0, kTimeBlock = 1, kTimeBlockRows = 2, kTimeEngine0 = 3, kTimeEngineN = 6, kTimeSlots = 9 };
const char* const kEngineTimeNames[kTimeEngineN] = {"host_landmarks", "host_grouping", "host_launch",
                                                    "host_pass",      "host_d2h",      "host_total"};
}

struct _Topology {
    shdr_graph* graph = nullptr;
    shdr::HostGraph* hg = nullptr;
    shdr_graph_info info{};

    std::shared_mutex vipLock;  // virtualIPLock (:23-24), taken by attach/detach
    std::unordered_map<uint32_t, int32_t> virtualIP;
    std::vector<int32_t> vertexRefs;  // addresses attached per vertex
    // Queries read an immutable snapshot of virtualIP instead of taking the lock:
    // attach/detach bump vipVersion; the first query that sees a stale snapshot
    // rebuilds it. Snapshots live until topology_free (bounded: after
    // kMaxSnapshots rebuilds, queries fall back to the reader lock).
    std::atomic<uint64_t> vipVersion{0};
    std::atomic<const VipSnapshot*> vipSnap{nullptr};
    std::atomic<bool> snapExhausted{false};  // rebuild budget spent: queries use the reader lock
    std::mutex snapLock;
    std::vector<std::unique_ptr<VipSnapshot>> snapshots;
    std::atomic<uint64_t> attachEpoch{0};  // bumps when the attached vertex set changes (under vipLock)

    std::once_flag attachOnce;
    std::unique_ptr<AttachIndex> attachIndex;
    std::mutex computeLock;
    // the current table, published with release semantics; tables are immutable
    // and kept until topology_free, so readers never take a lock or a refcount
    std::atomic<const Table*> table{nullptr};
    std::vector<std::unique_ptr<Table>> tables;
    std::vector<shdr_engine*> engines;
    bool engineFailed = false;
    // Engines are prepared in the background from topology_new (graph upload,
    // arc blocks, landmark pre-pass), overlapping the hosts' attach calls; the
    // first query that needs a table waits for it (engineLock).
    std::mutex engineLock;
    std::thread enginePrep;

    // path-cache history (:29-31). SSSP branch: per source vertex, the tables the
    // row was revealed with (the reference computes a row over the targets
    // attached at that moment, so (s,d) is a hit only if d was attached at one
    // of those computations); complete branch: one flag per (s,d) pair.
    std::unique_ptr<std::atomic<const Reveal*>[]> revealedRow;
    std::mutex revealLock;  // appends to revealedRow lists
    std::vector<std::unique_ptr<Reveal>> reveals;
    // vertices with a self-loop: the self pair (s, s) of a row from a vertex
    // without one fails igraph_get_eid (:733-739) and is never cached
    std::vector<uint8_t> selfLoop;
    std::unique_ptr<std::atomic<uint64_t>[]> revealedPair;  // one bit per (s, d): V^2 / 8 bytes
    std::mutex minLock;
    double minimumPathLatency = 0.0;  // :30

    std::mutex statLock;
    double shortestPathTotalTime = 0.0;
    unsigned shortestPathCount = 0;
    double lastTimes[kTimeSlots] = {};  // topology_debug_lastComputeTimes
};

namespace {

// Current lock-free snapshot of virtualIP, rebuilding it if an attach/detach
// made it stale; nullptr once the rebuild budget is spent.
const VipSnapshot* vip_snapshot(Topology* top) {
    const uint64_t ver = top->vipVersion.load(std::memory_order_acquire);
    const VipSnapshot* snap = top->vipSnap.load(std::memory_order_acquire);
    if (snap && snap->version == ver) return snap;
    if (top->snapExhausted.load(std::memory_order_relaxed)) return nullptr;
    std::lock_guard<std::mutex> lk(top->snapLock);
    snap = top->vipSnap.load(std::memory_order_acquire);
    if (snap && snap->version == top->vipVersion.load(std::memory_order_acquire)) return snap;
    if (top->snapshots.size() >= kMaxSnapshots) {
        top->snapExhausted.store(true, std::memory_order_relaxed);
        return nullptr;
    }
    auto fresh = std::make_unique<VipSnapshot>();
    {
        std::shared_lock<std::shared_mutex> rl(top->vipLock);
        fresh->version = top->vipVersion.load(std::memory_order_acquire);
        fresh->map = top->virtualIP;
    }
    snap = fresh.get();
    top->snapshots.push_back(std::move(fresh));
    top->vipSnap.store(snap, std::memory_order_release);
    return snap;
}

int32_t vertex_of(Topology* top, Address* a) {
    uint32_t ip = address_toNetworkIP(a);
    std::shared_lock<std::shared_mutex> lk(top->vipLock);
    auto it = top->virtualIP.find(ip);
    return it == top->virtualIP.end() ? -1 : it->second;
}

int num_gpus_wanted() {
    const char* s = getenv("SHDR_NUM_GPUS");
    int n = s ? atoi(s) : 1;
    return n < 1 ? 1 : n;
}

// Test switch: SHDR_ENGINES_SHARE_DEVICES=1 places the SHDR_NUM_GPUS engines
// round-robin on the visible devices (several engines per GPU), so the
// multi-engine row split runs on a one-GPU box. Results never depend on it.
bool engines_share_devices() {
    const char* s = getenv("SHDR_ENGINES_SHARE_DEVICES");
    return s && atoi(s) != 0;
}

// Engines on the visible devices (created once, under engineLock). quiet: the
// background preparation, which leaves a failure to be reported by the query
// that needs the engines.
bool create_engines(Topology* top, bool quiet) {
    std::lock_guard<std::mutex> lk(top->engineLock);
    if (top->engineFailed) return false;
    if (!top->engines.empty()) return true;
    int want = num_gpus_wanted();
    int have = shdr_device_count();
    if (have <= 0) {
        if (quiet) return false;
        critical("no MI355X device visible; the routing engine has no CPU fallback");
        top->engineFailed = true;
        return false;
    }
    if (!engines_share_devices()) want = std::min(want, have);
    auto t0 = std::chrono::steady_clock::now();
    // one engine per device, created concurrently (each its own upload and pre-pass)
    std::vector<shdr_engine*> made(static_cast<size_t>(want), nullptr);
    std::vector<std::string> errs(static_cast<size_t>(want));
    auto make = [&](int k) {
        made[size_t(k)] = shdr_engine_create(top->graph, k % have);
        if (!made[size_t(k)]) {
            char buf[512];
            shdr_last_error(buf, sizeof buf);
            errs[size_t(k)] = buf;
        }
    };
    if (want == 1 || engines_share_devices()) {
        for (int k = 0; k < want; ++k) make(k);
    } else {
        std::vector<std::thread> th;
        for (int k = 0; k < want; ++k) th.emplace_back(make, k);
        for (auto& x : th) x.join();
    }
    // the background (quiet) attempt keeps all engines or none: after any failure the
    // first query tries again and logs what failed
    if (quiet && std::find(made.begin(), made.end(), nullptr) != made.end()) {
        for (auto* m : made)
            if (m) shdr_engine_free(m);
        return false;
    }
    for (int k = 0; k < want; ++k) {
        if (!made[size_t(k)]) {
            if (!quiet) critical("engine on device %d failed: %s", k % have, errs[size_t(k)].c_str());
            for (int j = k + 1; j < want; ++j)
                if (made[size_t(j)]) shdr_engine_free(made[size_t(j)]);
            break;
        }
        top->engines.push_back(made[size_t(k)]);
    }
    if (top->engines.empty()) {
        if (!quiet) top->engineFailed = true;
        return false;
    }
    top->lastTimes[kTimeCreate] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return true;
}

bool ensure_engines(Topology* top) { return create_engines(top, false); }

// Rows per block for an n x n table: SHDR_TABLE_BLOCK_ROWS if set, else the
// whole table unless its 16 n^2 bytes exceed SHDR_TABLE_HOST_FRAC (default 0.5)
// of the host's physical memory, then 4,096-row blocks (one wave of K=16 buckets
// on 256 CUs).
int32_t block_rows_for(int32_t n) {
    if (n <= 0) return 1;
    if (const char* s = getenv("SHDR_TABLE_BLOCK_ROWS")) {
        const long v = atol(s);
        if (v > 0) return int32_t(std::min<long>(v, n));
    }
    double frac = 0.5;
    if (const char* s = getenv("SHDR_TABLE_HOST_FRAC")) frac = atof(s);
    const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
    const double ram = (pages > 0 && psz > 0) ? double(pages) * double(psz) : 0.0;
    if (ram > 0.0 && 16.0 * double(n) * double(n) > frac * ram) return std::min<int32_t>(n, 4096);
    return n;
}

// A new table over the attached vertex set as it is now: rows ordered so that
// every block, and every engine's share of a block, is a spatially coherent part
// of the landmark embedding (shdr_engine_partition over nblk * G parts); no block
// is computed yet (under computeLock).
Table* new_table(Topology* top) {
    std::vector<int32_t> verts;
    uint64_t epoch;
    {
        std::shared_lock<std::shared_mutex> lk(top->vipLock);
        epoch = top->attachEpoch.load(std::memory_order_relaxed);
        verts.reserve(top->virtualIP.size());
        for (auto& kv : top->virtualIP) verts.push_back(kv.second);
    }
    std::sort(verts.begin(), verts.end());
    verts.erase(std::unique(verts.begin(), verts.end()), verts.end());
    if (!ensure_engines(top)) return nullptr;
    auto t = std::make_unique<Table>();
    t->srcV = verts;
    t->dstV = verts;
    t->n = int32_t(verts.size());
    t->epoch = epoch;
    const int32_t n = t->n;
    const int32_t B = block_rows_for(n);
    t->nblk = std::max<int32_t>(1, (n + B - 1) / B);
    t->G = int32_t(top->engines.size());
    const int32_t nparts = t->nblk * t->G;
    std::vector<int32_t> part(size_t(n), 0);
    if (nparts > 1 && n > 0) {
        if (shdr_engine_partition(top->engines[0], verts.data(), n, nparts, part.data()) != SHDR_OK) {
            char buf[512];
            shdr_last_error(buf, sizeof buf);
            critical("row partition failed: %s", buf);
            return nullptr;
        }
        std::vector<int32_t> order(static_cast<size_t>(n));
        for (int32_t i = 0; i < n; ++i) order[size_t(i)] = i;
        std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return part[size_t(a)] < part[size_t(b)]; });
        for (int32_t i = 0; i < n; ++i) t->srcV[size_t(i)] = verts[size_t(order[size_t(i)])];
        std::sort(part.begin(), part.end());
    }
    t->pstart.assign(size_t(nparts) + 1, n);
    for (int32_t p = 0; p < nparts; ++p)  // first row of each part (parts may be empty)
        t->pstart[size_t(p)] = int32_t(std::lower_bound(part.begin(), part.end(), p) - part.begin());
    t->rowBlk.assign(size_t(n), 0);
    for (int32_t b = 0; b < t->nblk; ++b)
        for (int32_t r = t->first_row(b); r < t->first_row(b + 1); ++r) t->rowBlk[size_t(r)] = b;
    t->blocks.reset(new std::atomic<const Block*>[size_t(t->nblk)]);
    for (int32_t b = 0; b < t->nblk; ++b) t->blocks[size_t(b)].store(nullptr, std::memory_order_relaxed);
    t->rowOf.assign(size_t(top->info.vertex_count), -1);
    t->colOf.assign(size_t(top->info.vertex_count), -1);
    for (int32_t i = 0; i < n; ++i) {
        t->rowOf[size_t(t->srcV[size_t(i)])] = i;
        t->colOf[size_t(t->dstV[size_t(i)])] = i;
    }
    t->ok = true;
    Table* raw = t.get();
    top->tables.push_back(std::move(t));
    top->table.store(raw, std::memory_order_release);
    return raw;
}

// Compute block b of t on the engines (each its part of the block's rows, in
// parallel) and publish it (under computeLock).
const Block* compute_block(Topology* top, Table* t, int32_t b) {
    if (const Block* x = t->blocks[size_t(b)].load(std::memory_order_acquire)) return x;
    const int32_t r0 = t->first_row(b), r1 = t->first_row(b + 1);
    const size_t n = size_t(t->n), rows = size_t(r1 - r0);
    auto blk = std::make_unique<Block>();
    blk->lat.reset(new double[std::max<size_t>(rows * n, 1)]);
    blk->rel.reset(new double[std::max<size_t>(rows * n, 1)]);
    blk->rowMin.assign(rows, INFINITY);
    const int G = t->G;
    std::vector<int> rcs(size_t(G), 0);
    std::vector<std::string> errs(static_cast<size_t>(G));
    auto t0 = std::chrono::steady_clock::now();
    auto run = [&](int k) {
        const int32_t a0 = t->pstart[size_t(b) * G + k], a1 = t->pstart[size_t(b) * G + k + 1];
        if (a1 <= a0) return;
        const size_t o = size_t(a0 - r0);
        rcs[size_t(k)] = shdr_routes_compute(top->engines[size_t(k)], t->srcV.data() + a0, a1 - a0, t->dstV.data(),
                                             t->n, blk->lat.get() + o * n, blk->rel.get() + o * n, nullptr,
                                             blk->rowMin.data() + o, 0, nullptr);
        if (rcs[size_t(k)]) { char buf[512]; shdr_last_error(buf, sizeof buf); errs[size_t(k)] = buf; }
    };
    if (G == 1) {
        run(0);
    } else {
        std::vector<std::thread> th;
        for (int k = 0; k < G; ++k) th.emplace_back(run, k);
        for (auto& x : th) x.join();
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int k = 0; k < G; ++k)
        if (rcs[size_t(k)]) { critical("route computation failed on device %d: %s", k, errs[size_t(k)].c_str()); return nullptr; }
    {
        std::lock_guard<std::mutex> lk(top->statLock);
        top->shortestPathTotalTime += secs;
        top->shortestPathCount += top->info.is_complete ? 0u : unsigned(rows);
    }
    top->lastTimes[kTimeBlock] = secs * 1e3;
    top->lastTimes[kTimeBlockRows] = double(rows);
    if (G >= 1) {  // the first engine's host phases (shdr_engine_timing "host_*")
        int32_t nt = 0;
        const char* names[32];
        float ms[32];
        if (shdr_engine_timing(top->engines[0], &nt, names, ms, 32) == SHDR_OK)
            for (int32_t i = 0; i < nt && i < 32; ++i)
                for (int j = 0; j < kTimeEngineN; ++j)
                    if (!strcmp(names[i], kEngineTimeNames[j])) top->lastTimes[kTimeEngine0 + j] = ms[i];
    }
    const Block* raw = blk.get();
    t->owned.push_back(std::move(blk));
    t->blocks[size_t(b)].store(raw, std::memory_order_release);
    message("computed rows %d-%d of a %d x %d route table (block %d of %d) on %d GPU(s) in %f seconds", r0, r1 - 1,
            t->n, t->n, b + 1, t->nblk, G, secs);
    return raw;
}

// The block holding row `row` of t, computed on first use.
const Block* ensure_block(Topology* top, const Table* t, int32_t row) {
    if (const Block* x = t->block(row)) return x;
    std::lock_guard<std::mutex> lk(top->computeLock);
    return compute_block(top, const_cast<Table*>(t), t->rowBlk[size_t(row)]);
}

// A table holding rows sv and dv; with `current`, one computed for the attached
// vertex set as it is now (a miss stores a row over every attached target).
const Table* table_for(Topology* top, int32_t sv, int32_t dv, bool current = false) {
    auto has = [&](const Table* t) {
        return t && t->ok && sv < int32_t(t->rowOf.size()) && dv < int32_t(t->rowOf.size()) && t->rowOf[sv] >= 0 &&
               t->rowOf[dv] >= 0 && (!current || t->epoch == top->attachEpoch.load(std::memory_order_acquire));
    };
    const Table* t = top->table.load(std::memory_order_acquire);
    if (has(t)) return t;
    std::lock_guard<std::mutex> lk(top->computeLock);
    t = top->table.load(std::memory_order_acquire);
    if (has(t)) return t;
    t = new_table(top);
    return has(t) ? t : nullptr;
}

// Running minimum + upcall, _topology_storePathInCache :602-613. The upcall is
// made under minLock: the master keeps the LAST value it receives
// (shd-master.c:135-138 compares ms against ns, so every call wins), and two
// threads upcalling after the lock could deliver a stale larger minimum last.
// The reference re-reads the minimum at call time (:611-612); calling inside
// the lock gives the same guarantee. worker_updateMinTimeJump only takes the
// slave's own mutex (shd-slave.c:365-372) and never calls back here.
void note_min(Topology* top, double lat) {
    std::lock_guard<std::mutex> lk(top->minLock);
    if (top->minimumPathLatency == 0 || lat < top->minimumPathLatency) {
        top->minimumPathLatency = lat;
        worker_updateMinTimeJump(lat);
    }
}

// Record that source row sv was computed with table t (newest first); false if
// t was already in its history (nothing new stored, no new minimum possible).
bool reveal_row(Topology* top, int32_t sv, const Table* t) {
    std::lock_guard<std::mutex> lk(top->revealLock);
    const Reveal* head = top->revealedRow[size_t(sv)].load(std::memory_order_acquire);
    for (const Reveal* r = head; r; r = r->next)
        if (r->t == t) return false;
    auto node = std::make_unique<Reveal>(Reveal{t, head});
    top->revealedRow[size_t(sv)].store(node.get(), std::memory_order_release);
    top->reveals.push_back(std::move(node));
    return true;
}

// _topology_getPathEntry (:982-1044).
bool get_path_entry(Topology* top, Address* srcA, Address* dstA, double* lat, double* rel) {
    int32_t sv, dv;
    {  // _getConnectedVertexIndex (:616-633), both addresses
        const uint32_t sip = address_toNetworkIP(srcA), dip = address_toNetworkIP(dstA);
        auto look = [&](const std::unordered_map<uint32_t, int32_t>& m) {
            auto si = m.find(sip), di = m.find(dip);
            sv = si == m.end() ? -1 : si->second;
            dv = di == m.end() ? -1 : di->second;
        };
        if (const VipSnapshot* snap = vip_snapshot(top)) {
            look(snap->map);
        } else {
            std::shared_lock<std::shared_mutex> lk(top->vipLock);
            look(top->virtualIP);
        }
    }
    if (sv < 0) {
        warning("address %s is not connected to the topology", address_toHostIPString(srcA));
        critical("invalid vertex %d, source address %s is not connected to topology", sv, address_toString(srcA));
        return false;
    }
    if (dv < 0) {
        warning("address %s is not connected to the topology", address_toHostIPString(dstA));
        critical("invalid vertex %d, destination address %s is not connected to topology", dv,
                 address_toString(dstA));
        return false;
    }
    const Table* t = table_for(top, sv, dv);
    auto no_path = [&]() {
        critical("unable to find path between node %s (vertex %d) and node %s (vertex %d)", address_toString(srcA), sv,
                 address_toString(dstA), dv);
        return false;
    };
    if (!t) return no_path();
    const bool complete = top->info.is_complete != 0;
    const bool undirected = top->info.is_directed == 0;
    const size_t V = size_t(top->info.vertex_count);
    int32_t ri = t->rowOf[sv], ci = t->colOf[dv];  // entry answered (row, column of t)
    // cache hit on (s,d)?  else (undirected) on (d,s)?  else compute+store (s,d).
    // SSSP rows: the pair is cached iff row `a` was revealed with a table whose
    // target set held `b` (tables are immutable and live until topology_free).
    // A failed pair is never stored: the self pair of a vertex without a
    // self-loop (get_eid(s, s) fails, :733-739, so _computeSourcePathsHelper
    // returns FALSE before _storePathInCache).
    auto row_has = [&](int32_t a, int32_t b) {
        if (a == b && !top->selfLoop[size_t(a)]) return false;
        for (const Reveal* r = top->revealedRow[size_t(a)].load(std::memory_order_acquire); r; r = r->next)
            if (r->t->colOf[size_t(b)] >= 0) return true;
        return false;
    };
    // complete branch: one bit per (s, d) pair
    auto pair_word = [&](int32_t a, int32_t b) -> std::atomic<uint64_t>& {
        return top->revealedPair[(size_t(a) * V + size_t(b)) >> 6];
    };
    auto pair_bit = [&](int32_t a, int32_t b) { return uint64_t(1) << ((size_t(a) * V + size_t(b)) & 63); };
    auto pair_seen = [&](int32_t a, int32_t b) { return (pair_word(a, b).load(std::memory_order_acquire) & pair_bit(a, b)) != 0; };
    bool hit = complete ? pair_seen(sv, dv) : row_has(sv, dv);
    if (!hit && undirected) {
        bool rhit = complete ? pair_seen(dv, sv) : row_has(dv, sv);
        if (rhit) { ri = t->rowOf[dv]; ci = t->colOf[sv]; hit = true; }
    }
    // a table's rows are computed a block at a time, on first use (values never
    // depend on which table or block answers: same graph, same rows)
    const Block* blk = nullptr;
    if (!hit) {
        // the reference computes and stores here (the whole row over every
        // attached target, :775-939); reveal and feed the min tracker, from a
        // table over the attached set as it is now
        if (t->epoch != top->attachEpoch.load(std::memory_order_acquire)) {
            t = table_for(top, sv, dv, true);
            if (!t) return no_path();
            ri = t->rowOf[sv];
            ci = t->colOf[dv];
        }
        blk = ensure_block(top, t, ri);
        if (!blk) return no_path();
        const size_t o = size_t(ri - t->first_row(t->rowBlk[size_t(ri)]));
        double m;
        bool first;
        bool allSuccess = true;
        if (complete) {
            // _topology_lookupPath (:941-979): a pair without an edge fails before
            // it is stored, so it stays uncached and misses again next time
            m = blk->lat[o * size_t(t->n) + size_t(ci)];
            first = m == m &&
                    (pair_word(sv, dv).fetch_or(pair_bit(sv, dv), std::memory_order_acq_rel) & pair_bit(sv, dv)) == 0;
        } else {
            first = reveal_row(top, sv, t);
            m = blk->rowMin[o];
            // the source is always among the row's targets (:791-797): without a
            // self-loop its self pair fails, the row's allSuccess is FALSE (:910-938),
            // and _topology_getPathEntry skips the re-read and fails the query that
            // triggered the computation (:1018-1035), although the other targets
            // (this pair too, if d != s) were stored
            allSuccess = top->selfLoop[size_t(sv)] != 0;
        }
        if (first && std::isfinite(m)) note_min(top, m);
        if (!allSuccess) return no_path();
    } else {
        blk = ensure_block(top, t, ri);
        if (!blk) return no_path();
    }
    const size_t pi = size_t(ri - t->first_row(t->rowBlk[size_t(ri)])) * size_t(t->n) + size_t(ci);
    const double L = blk->lat[pi];
    if (L != L) {
        critical("unable to find path between node %s (vertex %d) and node %s (vertex %d)", address_toString(srcA), sv,
                 address_toString(dstA), dv);
        return false;
    }
    if (lat) *lat = L;
    if (rel) *rel = blk->rel[pi];
    return true;
}

// ---------------------------------------------------------------- attach (:1071-1258)
// Attachment candidates (_topology_findAttachmentVertex :1174-1258), indexed once
// per topology: the reference scans every vertex per attached host (:1196-1198,
// "@todo: this could be made much more efficient"), which is O(hosts x V) and
// dominates start-up at 50k hosts on 1M vertices. Lists keep vertex-index order,
// so the candidate sets, their usable-IP counts, the longest-prefix scan and the
// uniform pick are exactly the reference's.
struct CandList {
    std::vector<int32_t> v;
    unsigned usable = 0;  // members whose IP is neither INADDR_NONE nor INADDR_ANY
    void add(int32_t x, bool u) { v.push_back(x); usable += u; }
};

struct AttachIndex {
    CandList all;                                       // every "poi" vertex
    std::unordered_map<std::string, CandList> byType;   // ASCII-lowercased type
    std::unordered_map<std::string, CandList> byCode;   // ASCII-lowercased geocode
    std::unordered_map<std::string, CandList> byTypeCode;  // type + '\0' + geocode
    std::unordered_map<uint32_t, CandList> byIP;        // exact vertex IP
    std::vector<uint32_t> ip;                           // per vertex (INADDR_NONE if not a poi)
};

std::string ascii_lower(const char* s) {
    std::string r(s ? s : "");
    for (char& c : r)
        if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');
    return r;
}

const AttachIndex& attach_index(Topology* top) {
    std::call_once(top->attachOnce, [top] {
        auto ix = std::make_unique<AttachIndex>();
        shdr::HostGraph* g = top->hg;
        ix->ip.assign(size_t(g->V), INADDR_NONE);
        for (int32_t v = 0; v < g->V; ++v) {
            if (g->vertex_str("id", v).find("poi") == std::string::npos) continue;  // g_strstr_len(id, "poi")
            const uint32_t vip = address_stringToIP(g->vertex_str("ip", v).c_str());
            const bool usable = vip != INADDR_NONE && vip != INADDR_ANY;
            ix->ip[v] = vip;
            const std::string ty = ascii_lower(g->vertex_str("type", v).c_str());
            const std::string gc = ascii_lower(g->vertex_str("geocode", v).c_str());
            ix->all.add(v, usable);
            ix->byType[ty].add(v, usable);
            ix->byCode[gc].add(v, usable);
            ix->byTypeCode[ty + std::string(1, '\0') + gc].add(v, usable);
            ix->byIP[vip].add(v, usable);
        }
        top->attachIndex = std::move(ix);
    });
    return *top->attachIndex;
}

int32_t find_attachment_vertex(Topology* top, Random* rnd, const char* ipHint, const char* geocodeHint,
                               const char* typeHint) {
    const AttachIndex& ix = attach_index(top);
    static const CandList kEmpty;
    auto get = [](const auto& m, const auto& k) -> const CandList& {
        auto it = m.find(k);
        return it == m.end() ? kEmpty : it->second;
    };
    const uint32_t requestedIP = ipHint ? address_stringToIP(ipHint) : INADDR_NONE;
    // an exact IP match replaces every other filter (:1091-1111)
    const CandList* exact = nullptr;
    if (ipHint && requestedIP != INADDR_NONE && requestedIP != INADDR_ANY) {
        const CandList& e = get(ix.byIP, requestedIP);
        if (!e.v.empty()) exact = &e;
    }
    const CandList* cands;
    if (exact) {
        cands = exact;
    } else {
        const std::string ty = ascii_lower(typeHint), gc = ascii_lower(geocodeHint);
        const CandList& tc = (typeHint && geocodeHint) ? get(ix.byTypeCode, ty + std::string(1, '\0') + gc) : kEmpty;
        const CandList& t = typeHint ? get(ix.byType, ty) : kEmpty;
        const CandList& c = geocodeHint ? get(ix.byCode, gc) : kEmpty;
        cands = !tc.v.empty() ? &tc : !t.v.empty() ? &t : !c.v.empty() ? &c : &ix.all;  // :1206-1218
    }
    if (cands->v.empty()) return -1;
    if (ipHint && cands->usable > 0 && !exact) {  // longest prefix match (:1147-1172)
        uint32_t bestMatch = 0;
        int32_t best = -1;
        for (int32_t v : cands->v) {
            const uint32_t match = ix.ip[v] & requestedIP;
            if (match > bestMatch) { bestMatch = match; best = v; }
        }
        return best;
    }
    const double r = random_nextDouble(rnd);
    const int indexRange = int(cands->v.size()) - 1;
    const int chosen = int(std::round(double(indexRange * r)));
    if (chosen < 0 || chosen > indexRange) return -1;
    return cands->v[size_t(chosen)];
}

}  // namespace

extern "C" {

Topology* topology_new(const gchar* graphPath) {
    if (!graphPath) return nullptr;
    message("reading graphml topology graph at '%s'...", graphPath);
    shdr_graph* g = shdr_graph_load_graphml(graphPath);
    if (!g) {
        char buf[512];
        shdr_last_error(buf, sizeof buf);
        critical("reading graphml topology failed: %s", buf);
        return nullptr;
    }
    auto* top = new Topology();
    top->graph = g;
    top->hg = shdr::host_of(g);
    shdr_graph_check(g, &top->info);
    if (!top->info.is_connected || top->info.cluster_count > 1) {
        critical("topology must be but is not strongly connected");
        topology_free(top);
        return nullptr;
    }
    if (top->info.bad_latency_edges > 0) warning("%lld edges have invalid latency <= 0", (long long)top->info.bad_latency_edges);
    {
        const size_t V = size_t(top->info.vertex_count);
        top->revealedRow.reset(new std::atomic<const Reveal*>[std::max<size_t>(V, 1)]);
        for (size_t v = 0; v < V; ++v) top->revealedRow[v].store(nullptr, std::memory_order_relaxed);
        top->selfLoop.assign(V, 0);
        for (size_t e = 0; e < top->hg->efrom.size(); ++e)
            if (top->hg->efrom[e] == top->hg->eto[e]) top->selfLoop[size_t(top->hg->efrom[e])] = 1;
        if (top->info.is_complete) {
            const size_t words = std::max<size_t>((V * V + 63) / 64, 1);
            top->revealedPair.reset(new std::atomic<uint64_t>[words]);
            for (size_t i = 0; i < words; ++i) top->revealedPair[i].store(0, std::memory_order_relaxed);
        }
    }
    message("topology graph is %s, %s, and strongly connected with %u cluster; %d vertices, %lld edges",
            top->info.is_complete ? "complete" : "incomplete", top->info.is_directed ? "directed" : "undirected",
            (unsigned)top->info.cluster_count, top->info.vertex_count, (long long)top->info.edge_count);
    // the simulator attaches its hosts next: prepare the engines meanwhile
    top->enginePrep = std::thread([top] { create_engines(top, true); });
    return top;
}

void topology_free(Topology* top) {
    if (!top) return;
    {
        std::lock_guard<std::mutex> lk(top->statLock);
        message("path cache cleared, spent %f seconds computing %u shortest paths", top->shortestPathTotalTime,
                top->shortestPathCount);
    }
    if (top->enginePrep.joinable()) top->enginePrep.join();
    for (auto* e : top->engines) shdr_engine_free(e);
    shdr_graph_free(top->graph);
    delete top;
}

void topology_attach(Topology* top, Address* address, Random* randomSourcePool, gchar* ipHint, gchar* geocodeHint,
                     gchar* typeHint, guint64* bwDownOut, guint64* bwUpOut) {
    if (!top || !address) return;
    uint32_t nodeIP = address_toNetworkIP(address);
    int32_t v = find_attachment_vertex(top, randomSourcePool, ipHint, geocodeHint, typeHint);
    if (v < 0) {
        critical("no attachment vertex found for address %s", address_toHostIPString(address));
        return;
    }
    {
        std::unique_lock<std::shared_mutex> lk(top->vipLock);
        if (top->vertexRefs.empty()) top->vertexRefs.assign(size_t(top->hg->V), 0);
        auto it = top->virtualIP.find(nodeIP);
        bool changed = false;  // the set of attached vertices (the targets of a computed row)
        if (it != top->virtualIP.end() && --top->vertexRefs[size_t(it->second)] == 0) changed = true;  // g_hash_table_replace
        if (top->vertexRefs[size_t(v)]++ == 0) changed = true;
        top->virtualIP[nodeIP] = v;
        if (changed) top->attachEpoch.fetch_add(1, std::memory_order_acq_rel);
        top->vipVersion.fetch_add(1, std::memory_order_release);
    }
    if (bwUpOut) *bwUpOut = (guint64)top->hg->vertex_num("bandwidthup", v);
    if (bwDownOut) *bwDownOut = (guint64)top->hg->vertex_num("bandwidthdown", v);
    info("connected address '%s' to point of interest '%s' (ip=%s, geocode=%s, type=%s)",
         address_toHostIPString(address), top->hg->vertex_str("id", v).c_str(),
         top->hg->vertex_str("ip", v).c_str(), top->hg->vertex_str("geocode", v).c_str(),
         top->hg->vertex_str("type", v).c_str());
}

void topology_detach(Topology* top, Address* address) {
    if (!top || !address) return;
    uint32_t ip = address_toNetworkIP(address);
    std::unique_lock<std::shared_mutex> lk(top->vipLock);
    auto it = top->virtualIP.find(ip);
    if (it == top->virtualIP.end()) return;
    if (--top->vertexRefs[size_t(it->second)] == 0) top->attachEpoch.fetch_add(1, std::memory_order_acq_rel);
    top->virtualIP.erase(it);
    top->vipVersion.fetch_add(1, std::memory_order_release);
}

gdouble topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress) {
    double lat = 0;
    if (top && get_path_entry(top, srcAddress, dstAddress, &lat, nullptr)) return lat;
    return -1.0;
}

gdouble topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress) {
    double rel = 0;
    if (top && get_path_entry(top, srcAddress, dstAddress, nullptr, &rel)) return rel;
    return -1.0;
}

gboolean topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress) {
    return topology_getLatency(top, srcAddress, dstAddress) > -1;
}

int topology_debug_isComplete(Topology* top) { return top ? top->info.is_complete : -1; }
int topology_debug_isDirected(Topology* top) { return top ? top->info.is_directed : -1; }
gdouble topology_debug_minimumPathLatency(Topology* top) {
    if (!top) return -1;
    std::lock_guard<std::mutex> lk(top->minLock);
    return top->minimumPathLatency;
}
int32_t topology_debug_vertexOf(Topology* top, Address* address) { return top ? vertex_of(top, address) : -1; }

int topology_debug_lastComputeTimes(Topology* top, double* out, int n) {
    if (!top || !out || n < 0) return -1;
    std::lock_guard<std::mutex> lk(top->computeLock);
    for (int i = 0; i < n && i < kTimeSlots; ++i) out[i] = top->lastTimes[i];
    return kTimeSlots;
}

int topology_debug_tableBlocks(Topology* top, int32_t* rowsPerBlockOut, int32_t* computedOut) {
    if (!top) return -1;
    const Table* t = top->table.load(std::memory_order_acquire);
    if (!t) return 0;
    int32_t c = 0;
    for (int32_t b = 0; b < t->nblk; ++b) c += t->blocks[size_t(b)].load(std::memory_order_acquire) != nullptr;
    if (rowsPerBlockOut) *rowsPerBlockOut = t->nblk > 0 ? t->first_row(1) - t->first_row(0) : 0;
    if (computedOut) *computedOut = c;
    return t->nblk;
}

}  // extern "C"
