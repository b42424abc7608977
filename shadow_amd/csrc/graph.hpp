// Host-side topology graph: GraphML ingestion, igraph-equivalent indexing,
// validation and the CSR images uploaded to HBM.
//
// Reference behaviour mirrored here (paths relative to /root/reference):
//   src/main/routing/shd-topology.c:95-123   _topology_loadGraph (igraph_read_graph_graphml)
//   src/main/routing/shd-topology.c:129-230  _topology_isComplete
//   src/main/routing/shd-topology.c:232-320  _topology_checkGraphProperties
//   src/main/routing/shd-topology.c:375-474  _topology_checkGraphVertices/Edges
//   src/main/routing/shd-topology.c:501-534  _topology_extractEdgeWeights
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/shdr.h"

namespace shdr {

struct HostGraph {
    int32_t V = 0;
    int64_t E = 0;
    bool directed = false;

    std::vector<int32_t> efrom, eto;  // edge endpoints, edge index = <edge> order

    // Attributes as igraph's C attribute handler keeps them: numeric (double) or string.
    std::map<std::string, std::vector<double>> vnum, enumr;
    std::map<std::string, std::vector<std::string>> vstr, estr;

    // Derived, built on demand.
    bool checked = false;
    shdr_graph_info info{};
    std::unordered_map<uint64_t, int64_t> canon;  // (u,v) key -> lowest edge index
    bool canon_built = false;

    const std::vector<double>* vnum_ptr(const std::string& a) const {
        auto it = vnum.find(a);
        return it == vnum.end() ? nullptr : &it->second;
    }
    const std::vector<double>* enum_ptr(const std::string& a) const {
        auto it = enumr.find(a);
        return it == enumr.end() ? nullptr : &it->second;
    }
    double vertex_num(const std::string& a, int32_t v) const;
    const std::string& vertex_str(const std::string& a, int32_t v) const;
    double edge_num(const std::string& a, int64_t e) const;

    uint64_t pair_key(int32_t u, int32_t v) const {
        if (!directed && u > v) std::swap(u, v);
        return (uint64_t(uint32_t(u)) << 32) | uint32_t(v);
    }
    void build_canon();
    int64_t get_eid(int32_t u, int32_t v);  // lowest edge index joining u,v; -1 if none

    int check();  // fills info; returns SHDR_OK or error
};

// The device-facing image of a graph (all host vectors, uploaded verbatim).
struct CsrImage {
    int32_t V = 0;
    int64_t A = 0;  // relaxation arcs (self-loops excluded)
    bool directed = false;
    bool same_in_out = false;  // undirected: in-CSR == out-CSR
    // out-CSR, arcs of u sorted by (target, edge index)
    std::vector<int64_t> rowptr;
    std::vector<int32_t> col;
    std::vector<double> w;       // relaxation weight = latency of the arc's own edge
    std::vector<double> oclat;   // latency of canonical edge (u,col)  (get_eid semantics)
    std::vector<double> ocrel;   // 1 - packetloss of canonical edge
    std::vector<double> ocjit;   // jitter of canonical edge (empty if the graph has no edge jitter)
    // in-CSR, in-arcs of v sorted by (source, edge index); empty if same_in_out
    std::vector<int64_t> irowptr;
    std::vector<int32_t> isrc;
    std::vector<double> iw, iclat, icrel, icjit;
    // per vertex
    std::vector<double> vrel;      // 1 - vertex packetloss
    std::vector<double> self_lat;  // canonical self-loop latency or NaN
    std::vector<double> self_rel;  // 1 - its loss or NaN
    double mean_w = 0.0;
    bool lat_is_w = false;  // every arc's weight is bitwise its canonical edge's latency
};

void build_csr(HostGraph& g, CsrImage& out);

HostGraph* parse_graphml(const char* text, size_t len, std::string& err);
HostGraph* generate(int32_t kind, int32_t n, int32_t m, uint64_t seed, std::string& err);

void set_error(const std::string& msg);

}  // namespace shdr
