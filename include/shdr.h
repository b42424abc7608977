/*
 * shdr.h — thin C-ABI between host code and the MI355X routing engine.
 *
 * Plain pointers and sizes only (no torch, no GLib).  This is the boundary the
 * drop-in (shd_topology.h) calls, and the one a Python/ctypes binding uses in
 * tests and bench.py (INTEGRATION.md shows both bindings).
 *
 * What each entry point replaces in the reference (all paths relative to
 * /root/reference/src/main/routing/shd-topology.c unless stated):
 *
 *   shdr_graph_load_graphml     igraph_read_graph_graphml            :95-123 (call :110)
 *   shdr_graph_check            _topology_checkGraphProperties       :232-320
 *                               _topology_isComplete                 :129-230
 *                               _topology_checkGraphVertices/Edges   :375-474
 *   shdr_graph_get_eid          igraph_get_eid                       :189, :643-645
 *   shdr_engine_create          _topology_extractEdgeWeights         :501-534 (weights -> HBM CSR)
 *   shdr_routes_compute         _topology_computeSourcePaths         :775-939 (Dijkstra call :868)
 *                               _topology_computeSourcePathsHelper   :663-773 (epilogue)
 *                               _topology_lookupPath                 :941-979 (complete branch)
 *                               min tracking in _storePathInCache    :602-613
 *
 * Error convention: functions returning int return 0 on success and a
 * negative SHDR_E* code on failure; shdr_last_error() describes the most
 * recent failure on the calling thread.  There is NO CPU fallback: without a
 * usable gfx950 device shdr_engine_create fails with SHDR_ENODEV.
 */
#ifndef SHDR_H_
#define SHDR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHDR_OK 0
#define SHDR_EINVAL (-1)
#define SHDR_EIO (-2)
#define SHDR_EPARSE (-3)
#define SHDR_ENODEV (-4)
#define SHDR_EHIP (-5)
#define SHDR_ENOMEM (-6)
#define SHDR_ENOPATH (-7)

typedef struct shdr_graph shdr_graph;   /* host-side topology graph */
typedef struct shdr_engine shdr_engine; /* graph resident in one GPU's HBM + workspace */

/* Properties computed by shdr_graph_check (mirrors the Topology fields at
 * shd-topology.c:38-43). */
typedef struct shdr_graph_info {
    int32_t vertex_count;
    int64_t edge_count;
    int32_t is_directed;
    int32_t is_connected;   /* strongly connected (igraph_is_connected STRONG, :241) */
    int32_t cluster_count;  /* strongly connected components (:248) */
    int32_t is_complete;    /* branch selector (:129-230) */
    int64_t self_loops;
    int64_t bad_latency_edges; /* edges with latency <= 0 (:414-419) */
} shdr_graph_info;

/* ---------------- host graph ---------------- */

/* Parse a GraphML file the way igraph's reader indexes it: vertex index = order
 * of first appearance of a node id (in <node> or <edge> elements), edge index =
 * <edge> order; numeric attributes via strtod; missing numeric = NaN, missing
 * string = "". Returns NULL on I/O or parse error (see shdr_last_error). */
shdr_graph* shdr_graph_load_graphml(const char* path);

/* Same, from an in-memory buffer (CDATA topologies in Shadow configs,
 * shd-configuration.c:239-325). */
shdr_graph* shdr_graph_parse_graphml(const char* text, size_t len);

/* Build a graph from plain arrays. vloss may be NULL (all 0); vertex ids become
 * "poi-<index+1>". */
shdr_graph* shdr_graph_from_edges(int32_t vertex_count, int64_t edge_count, int32_t directed,
                                  const int32_t* efrom, const int32_t* eto,
                                  const double* elatency, const double* eloss,
                                  const double* vloss);

/* Synthetic topologies for configs 4-5:
 *   kind 0: Barabasi-Albert, m edges per new vertex (cfg 4: n=1e5, m=3)
 *   kind 1: Chung-Lu power law (exponent ~2.1, mean degree 2m) + spanning tree (cfg 5)
 * plus one self-loop per vertex; latency U(1,100) ms, edge loss U(0,0.01),
 * vertex loss U(0,0.02), self-loop latency U(0.5,5). Deterministic in seed. */
shdr_graph* shdr_graph_generate(int32_t kind, int32_t n, int32_t m, uint64_t seed);

/* Binary image of a parsed graph (endpoints + every attribute column; native
 * byte order). shdr_graph_load_graphml also consults a content-keyed cache of
 * these images when SHDR_GRAPH_CACHE names a directory (SURVEY §8(f) row 4:
 * cfg5-size GraphML takes ~10 s to parse, the image well under 1 s). */
int shdr_graph_save_binary(const shdr_graph* g, const char* path);
shdr_graph* shdr_graph_load_binary(const char* path);

/* The graph as GraphML (nodes in vertex order, edges in edge order, every
 * attribute; numerics as shortest round-trip decimals): loading the file gives
 * back the same graph. Lets synthetic topologies (configs 4-5) go through
 * topology_new like any Shadow topology file. */
int shdr_graph_save_graphml(const shdr_graph* g, const char* path);

void shdr_graph_free(shdr_graph* g);

int shdr_graph_check(shdr_graph* g, shdr_graph_info* info);
int32_t shdr_graph_vertex_count(const shdr_graph* g);
int64_t shdr_graph_edge_count(const shdr_graph* g);
int32_t shdr_graph_is_directed(const shdr_graph* g);

/* Attribute access (VAN/VAS/EAN). Unknown attribute: NaN / "" . */
double shdr_graph_vertex_num(const shdr_graph* g, const char* attr, int32_t v);
const char* shdr_graph_vertex_str(const shdr_graph* g, const char* attr, int32_t v);
double shdr_graph_edge_num(const shdr_graph* g, const char* attr, int64_t e);
int shdr_graph_edge_ends(const shdr_graph* g, int64_t e, int32_t* from, int32_t* to);

/* Export edge arrays (each output may be NULL). */
int shdr_graph_export_edges(const shdr_graph* g, int32_t* efrom, int32_t* eto,
                            double* elatency, double* eloss, double* vloss);

/* Canonical edge between from and to: the lowest edge index joining them
 * (either orientation when undirected). -1 if none. */
int64_t shdr_graph_get_eid(const shdr_graph* g, int32_t from, int32_t to);

/* ---------------- device engine ---------------- */

/* Upload the graph to HBM on `device` (relaxation CSR, reverse CSR, canonical
 * per-arc latency / reliability factors, vertex reliabilities, self-loops).
 * Non-complete graphs are stored in a breadth-first device numbering; every
 * vertex index crossing this API (src, dst, pred_vertex) stays in the graph's
 * own numbering and results do not depend on it.
 * Fails with SHDR_ENODEV when no gfx950 device is visible. */
shdr_engine* shdr_engine_create(const shdr_graph* g, int32_t device);
void shdr_engine_free(shdr_engine* e);

/* flags for shdr_routes_compute */
#define SHDR_OUT_DEVICE 0x1   /* lat/rel/hops/row_min are device pointers on the engine's GPU */
#define SHDR_FORCE_SSSP 0x2   /* run the shortest-path branch even on a complete graph */
#define SHDR_TIMING 0x4       /* record per-kernel HIP-event timings (shdr_engine_timing) */

/* Compute the S x T route table: for every source vertex src[i] and target
 * vertex dst[j], latency (ms) and reliability exactly as the reference stores
 * them in its path cache:
 *   - complete graph: _topology_lookupPath (:941-979), the direct edge;
 *   - otherwise: shortest path (latency-weighted, mode OUT) then the ordered
 *     epilogue of _topology_computeSourcePathsHelper (:663-773).
 * Row-major outputs lat[i*T+j], rel[i*T+j]; hops (may be NULL) = edges on the
 * path; row_min[i] (may be NULL) = min latency over row i (the value the
 * reference's min tracking sees once row i is cached). A pair with no path
 * (missing edge / self-loop) gets lat = NaN.
 * `stream` is a hipStream_t (NULL = the engine's own stream). Blocks until the
 * results are complete. */
int shdr_routes_compute(shdr_engine* e, const int32_t* src, int32_t S,
                        const int32_t* dst, int32_t T,
                        double* lat, double* rel, int32_t* hops, double* row_min,
                        uint32_t flags, void* stream);

/* Source-vertex predecessor tree (in-arc chosen for each vertex) of the last
 * shortest-path compute, for parity tests: pred_vertex[v] = predecessor of v
 * on the path from src[i] (-1 for the source itself), dist[v] its shortest
 * distance; both indexed and valued in the graph's numbering. Only after a
 * compute with SHDR_KEEP_TREES (rows then run in caller order, one bucket per
 * slot, and the trees stay resident until the next compute). */
#define SHDR_KEEP_TREES 0x8
/* Complete-topology metrics (offline precompute; replaces
 * the per-path loop of /root/reference/src/tools/topology/compute-topology-paths.py:19-34):
 * implies SHDR_FORCE_SSSP; lat = the path's latency sum in path order (no
 * zero->1 override), rel = the MEAN per-hop jitter (canonical edges' `jitter`
 * summed in path order, divided by hops); a source paired with itself gets
 * lat 5.0, rel 0.0, hops 0 (the tool's one-vertex-path rule, :24-26). */
#define SHDR_PATH_JITTER 0x10
int shdr_engine_pred_tree(shdr_engine* e, int32_t i, int32_t* pred_vertex, double* dist);

/* Strong-scaling split of a source list over nparts engines or ranks (the
 * reference computes rows one at a time, shd-topology.c:775-939; any split of the
 * rows gives the same table). part[i] in [0, nparts) for src[i]; parts hold
 * S/nparts or S/nparts + 1 sources, each made of compact regions of the
 * landmark embedding the engine groups buckets by (so a shard's buckets are as
 * tight as the whole list's), regions dealt round-robin so parts cost alike.
 * Deterministic: every engine of the same graph, on any GPU, returns the same
 * split. Complete graphs: contiguous blocks. */
int shdr_engine_partition(shdr_engine* e, const int32_t* src, int32_t S, int32_t nparts, int32_t* part);

/* Complete-topology GraphML (the output stage of
 * /root/reference/src/tools/topology/compute-topology-paths.py:120-180).
 * lat / jit: the P x P tables of shdr_routes_compute(e, pois, P, pois, P, ...,
 * SHDR_PATH_JITTER), host memory, row-major. Writes nodes pois[0..P) in that
 * order with every vertex attribute of g, and one undirected edge per pair
 * {i <= j} carrying latency, jitter and packetloss 0.0, taken from row j (the
 * tool runs sources in order and the later source overwrites the pair);
 * latencies <= 0 are replaced by the mean positive self / non-self latency
 * (ensure_nonzero_latency, :96-112); pairs without a path get no edge and
 * SHDR_ENOPATH is returned if that disconnects the result (:171-172). */
int shdr_write_complete_graphml(const shdr_graph* g, const int32_t* pois, int32_t P,
                                const double* lat, const double* jit, const char* path);

/* Timings of the last compute with SHDR_TIMING (milliseconds, HIP events on
 * the compute stream): names[k] / ms[k] for k < *n. */
int shdr_engine_timing(shdr_engine* e, int32_t* n, const char** names, float* ms, int32_t cap);

/* Bucket layout of the last shortest-path compute (schedule only, never results):
 * out[0] kernel variant, out[1] workgroups per bucket of the main launch
 * (cluster width, 1 = plain), out[2] 1 if rows were balanced over whole waves,
 * out[3] rows of the main launch (the rest ran as a tail launch), out[4] tail
 * cluster width, out[5] 1 if a partial group was issued first, out[6] the guard
 * code (8 = cluster barrier timeout, 16 = cluster across XCDs) if the compute fell
 * back from cluster mode and was recomputed with one workgroup per bucket (else 0),
 * out[7] such fallbacks over the engine's life, out[8] 1 if host outputs were
 * copied progressively (finished rows while the launch ran), out[9] how the tail
 * rows ran: 0 no tail, 1 a tail launch after the main launch, 2 a concurrent tail
 * launch on a second stream, 3 one launch whose first workgroups ran the tail's
 * half-width buckets before taking full-width ones (k_routes_pass). Fills min(n, 10). */
int shdr_engine_last_layout(shdr_engine* e, int32_t* out, int32_t n);

/* Processing order of the last shortest-path compute (schedule only): out[k] =
 * the caller's row index (position in src) of the k-th processed source; rows
 * k < last_layout out[3] ran as full-width buckets, the others as the tail's
 * half-width buckets (a tail launch, or the first workgroups of a single launch).
 * Fills min(n, S) and returns S (or a negative SHDR_E* code). */
int32_t shdr_engine_row_order(shdr_engine* e, int32_t* out, int32_t n);

/* Tuning knobs: relaxation bucket width delta in ms (0 = auto: mean arc
 * latency); kernel variant (index into the (sources-per-bucket, threads)
 * table of routes.hip: 0 = (8,256), 1 = (16,256), 2 = (16,512), 3 = (32,512)).
 * Results do not depend on either. */
int shdr_engine_set_delta(shdr_engine* e, double delta);
int shdr_engine_set_variant(shdr_engine* e, int32_t variant);

int32_t shdr_device_count(void);
int shdr_last_error(char* buf, size_t len);
/* "shadow-amd routes <version> (gfx950) kernel <sha>": <sha> is the first 16 hex
 * digits of the SHA-256 of shadow_amd/csrc/routes.hip the library was compiled
 * from (set by shadow_amd/Makefile), so a measurement can be tied to its binary. */
const char* shdr_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SHDR_H_ */
