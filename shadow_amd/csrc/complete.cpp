// GraphML writers. shdr_graph_save_graphml: any graph, lossless (synthetic
// topologies handed to topology_new). shdr_write_complete_graphml: the on-disk
// half of the offline all-sources
// precompute. The shortest-path metrics come from the GPU
// engine (shdr_routes_compute with SHDR_PATH_JITTER); this file turns the P x P
// table into the complete GraphML the simulator's isComplete branch consumes.
//
// Mirrors /root/reference/src/tools/topology/compute-topology-paths.py:
//   node set and attribute copy           main            :153-160
//   one undirected edge per pair, later
//   sources overwrite earlier ones         thread/add_edge :38-44 (nx.Graph)
//   latency / jitter / packetloss 0.0                       :42
//   zero-latency repair                    ensure_nonzero_latency :96-112
//   connectivity assertion                 main            :171-172
// and nx.write_graphml's layout (keys, then nodes, then edges; "d<k>" key ids).
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "graph.hpp"

namespace shdr {
const HostGraph* host_of(const shdr_graph* g);
}

namespace {

void put_xml(std::string& o, const std::string& s) {
    for (char c : s) {
        switch (c) {
            case '&': o += "&amp;"; break;
            case '<': o += "&lt;"; break;
            case '>': o += "&gt;"; break;
            case '"': o += "&quot;"; break;
            case '\'': o += "&apos;"; break;
            default: o += c;
        }
    }
}

// shortest round-trip decimal (what Python's repr of a float guarantees too)
void put_f64(std::string& o, double x) {
    char b[32];
    auto r = std::to_chars(b, b + sizeof b, x);
    o.append(b, r.ptr);
}

struct UnionFind {
    std::vector<int32_t> p;
    explicit UnionFind(int32_t n) : p(size_t(n)) { std::iota(p.begin(), p.end(), 0); }
    int32_t find(int32_t x) {
        while (p[x] != x) x = p[x] = p[p[x]];
        return x;
    }
    void join(int32_t a, int32_t b) { p[find(a)] = find(b); }
};

}  // namespace

extern "C" {

int shdr_write_complete_graphml(const shdr_graph* gh, const int32_t* pois, int32_t P, const double* lat,
                                const double* jit, const char* path) {
    const shdr::HostGraph* g = shdr::host_of(gh);
    if (!g || P < 0 || (P > 0 && (!pois || !lat || !jit)) || !path) {
        shdr::set_error("write_complete_graphml: bad arguments");
        return SHDR_EINVAL;
    }
    {
        std::vector<char> seen(size_t(g->V), 0);
        for (int32_t i = 0; i < P; ++i) {
            if (pois[i] < 0 || pois[i] >= g->V) { shdr::set_error("write_complete_graphml: vertex out of range"); return SHDR_EINVAL; }
            if (seen[pois[i]]++) { shdr::set_error("write_complete_graphml: duplicate vertex in pois"); return SHDR_EINVAL; }
        }
    }
    // value of edge {i, j}: sources run in pois order and nx.Graph.add_edge
    // overwrites, so the later source's row wins: (i <= j) -> row j, column i
    auto at = [&](const double* t, int32_t i, int32_t j) { return t[size_t(j) * size_t(P) + size_t(i)]; };

    // ensure_nonzero_latency: means of the positive self / non-self latencies
    // (summed in edge order), substituted for latencies <= 0
    double intra_sum = 0.0, inter_sum = 0.0;
    int64_t n_intra = 0, n_inter = 0, n_zero = 0;
    UnionFind uf(P);
    for (int32_t i = 0; i < P; ++i)
        for (int32_t j = i; j < P; ++j) {
            const double l = at(lat, i, j);
            if (std::isnan(l)) continue;  // no path: no edge
            if (i != j) uf.join(i, j);
            if (l <= 0.0) ++n_zero;
            else if (i == j) { intra_sum += l; ++n_intra; }
            else { inter_sum += l; ++n_inter; }
        }
    if (n_zero && (!n_intra || !n_inter)) {
        shdr::set_error("write_complete_graphml: zero latencies but no positive mean to replace them with");
        return SHDR_EINVAL;
    }
    const double intra_mean = n_intra ? intra_sum / double(n_intra) : 0.0;
    const double inter_mean = n_inter ? inter_sum / double(n_inter) : 0.0;
    for (int32_t i = 1; i < P; ++i)
        if (uf.find(i) != uf.find(0)) {
            shdr::set_error("write_complete_graphml: the path graph is not connected (unreachable pairs)");
            return SHDR_ENOPATH;
        }

    // keys: vertex attributes (every one the input carries, except the node id), then edge attributes
    struct Key { std::string name; bool numeric; };
    std::vector<Key> vkeys;
    for (const auto& kv : g->vnum) vkeys.push_back({kv.first, true});
    for (const auto& kv : g->vstr)
        if (kv.first != "id") vkeys.push_back({kv.first, false});
    std::sort(vkeys.begin(), vkeys.end(), [](const Key& a, const Key& b) { return a.name < b.name; });

    FILE* f = fopen(path, "wb");
    if (!f) { shdr::set_error(std::string("write_complete_graphml: cannot open ") + path); return SHDR_EIO; }
    std::string head;
    head += "<?xml version='1.0' encoding='utf-8'?>\n"
            "<graphml xmlns=\"http://graphml.graphdrawing.org/xmlns\" "
            "xmlns:xsi=\"http://www.w3.org/2001/XMLSchema-instance\" "
            "xsi:schemaLocation=\"http://graphml.graphdrawing.org/xmlns "
            "http://graphml.graphdrawing.org/xmlns/1.0/graphml.xsd\">\n";
    const size_t nv = vkeys.size();
    for (size_t k = 0; k < nv; ++k) {
        head += "  <key id=\"d" + std::to_string(k) + "\" for=\"node\" attr.name=\"";
        put_xml(head, vkeys[k].name);
        head += vkeys[k].numeric ? "\" attr.type=\"double\" />\n" : "\" attr.type=\"string\" />\n";
    }
    const std::string kl = "d" + std::to_string(nv), kj = "d" + std::to_string(nv + 1), kp = "d" + std::to_string(nv + 2);
    head += "  <key id=\"" + kl + "\" for=\"edge\" attr.name=\"latency\" attr.type=\"double\" />\n";
    head += "  <key id=\"" + kj + "\" for=\"edge\" attr.name=\"jitter\" attr.type=\"double\" />\n";
    head += "  <key id=\"" + kp + "\" for=\"edge\" attr.name=\"packetloss\" attr.type=\"double\" />\n";
    head += "  <graph edgedefault=\"undirected\">\n";
    std::vector<std::string> ids(static_cast<size_t>(P));
    for (int32_t i = 0; i < P; ++i) {
        const int32_t v = pois[i];
        put_xml(ids[i], g->vertex_str("id", v));
        head += "    <node id=\"" + ids[i] + "\">\n";
        for (size_t k = 0; k < nv; ++k) {
            if (vkeys[k].numeric) {
                const double x = g->vnum.at(vkeys[k].name)[v];
                if (std::isnan(x)) continue;  // attribute absent on this vertex
                head += "      <data key=\"d" + std::to_string(k) + "\">";
                put_f64(head, x);
            } else {
                const std::string& x = g->vstr.at(vkeys[k].name)[v];
                if (x.empty()) continue;
                head += "      <data key=\"d" + std::to_string(k) + "\">";
                put_xml(head, x);
            }
            head += "</data>\n";
        }
        head += "    </node>\n";
    }
    bool ok = fwrite(head.data(), 1, head.size(), f) == head.size();
    head.clear();
    head.shrink_to_fit();

    // edges, row-parallel formatting, written in row order
    const int nthreads = std::max(1, std::min<int>(16, int(std::thread::hardware_concurrency())));
    const int32_t rows_per = 32;
    std::vector<std::string> bufs(static_cast<size_t>(nthreads));
    for (int32_t r0 = 0; r0 < P && ok; r0 += rows_per * nthreads) {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; ++t)
            th.emplace_back([&, t] {
                std::string& o = bufs[t];
                o.clear();
                const int32_t lo = r0 + t * rows_per, hi = std::min(P, lo + rows_per);
                for (int32_t i = lo; i < hi; ++i)
                    for (int32_t j = i; j < P; ++j) {
                        double l = at(lat, i, j);
                        if (std::isnan(l)) continue;
                        if (l <= 0.0) l = (i == j) ? intra_mean : inter_mean;
                        o += "    <edge source=\"";
                        o += ids[i];
                        o += "\" target=\"";
                        o += ids[j];
                        o += "\"><data key=\"" + kl + "\">";
                        put_f64(o, l);
                        o += "</data><data key=\"" + kj + "\">";
                        put_f64(o, at(jit, i, j));
                        o += "</data><data key=\"" + kp + "\">0.0</data></edge>\n";
                    }
            });
        for (auto& t : th) t.join();
        for (auto& b : bufs)
            if (ok && !b.empty()) ok = fwrite(b.data(), 1, b.size(), f) == b.size();
    }
    static const char tail[] = "  </graph>\n</graphml>\n";
    if (ok) ok = fwrite(tail, 1, sizeof tail - 1, f) == sizeof tail - 1;
    if (fclose(f) != 0) ok = false;
    if (!ok) { shdr::set_error(std::string("write_complete_graphml: write failed: ") + path); return SHDR_EIO; }
    return SHDR_OK;
}

// The whole graph as GraphML, in the reader's indexing: nodes in vertex order,
// edges in edge order, every vertex / edge attribute column (numeric: shortest
// round-trip decimals, so strtod reads back the same doubles; NaN = absent).
// shdr_graph_load_graphml of the file gives the same graph. Used to hand
// synthetic topologies (configs 4-5) to topology_new like any GraphML.
int shdr_graph_save_graphml(const shdr_graph* gh, const char* path) {
    const shdr::HostGraph* g = shdr::host_of(gh);
    if (!g || !path) { shdr::set_error("save_graphml: bad arguments"); return SHDR_EINVAL; }
    struct Key { std::string name; bool node, numeric; const std::vector<double>* num; const std::vector<std::string>* str; };
    std::vector<Key> keys;
    for (const auto& kv : g->vnum) keys.push_back({kv.first, true, true, &kv.second, nullptr});
    for (const auto& kv : g->vstr)
        if (kv.first != "id") keys.push_back({kv.first, true, false, nullptr, &kv.second});
    for (const auto& kv : g->enumr) keys.push_back({kv.first, false, true, &kv.second, nullptr});
    for (const auto& kv : g->estr) keys.push_back({kv.first, false, false, nullptr, &kv.second});
    // one GraphML key per attribute name and domain: a name held both as a numeric
    // and as a string column cannot be written losslessly
    for (const auto& kv : g->vstr)
        if (g->vnum.count(kv.first)) {
            shdr::set_error("save_graphml: vertex attribute '" + kv.first + "' is both numeric and string");
            return SHDR_EINVAL;
        }
    for (const auto& kv : g->estr)
        if (g->enumr.count(kv.first)) {
            shdr::set_error("save_graphml: edge attribute '" + kv.first + "' is both numeric and string");
            return SHDR_EINVAL;
        }
    const std::vector<std::string>* ids = nullptr;
    if (auto it = g->vstr.find("id"); it != g->vstr.end()) ids = &it->second;
    // vertices without an id get "n<v>", made unique against every id in the graph
    // (a collision would merge two vertices when the file is read back)
    std::unordered_map<int32_t, std::string> fallback_id;
    {
        std::unordered_set<std::string> used;
        if (ids)
            for (const std::string& x : *ids)
                if (!x.empty()) used.insert(x);
        for (int32_t v = 0; v < g->V; ++v) {
            if (ids && !(*ids)[size_t(v)].empty()) continue;
            std::string x = "n" + std::to_string(v);
            while (used.count(x)) x += "_";
            used.insert(x);
            fallback_id.emplace(v, std::move(x));
        }
    }
    FILE* f = fopen(path, "wb");
    if (!f) { shdr::set_error(std::string("save_graphml: cannot open ") + path); return SHDR_EIO; }
    std::string head = "<?xml version='1.0' encoding='utf-8'?>\n<graphml xmlns=\"http://graphml.graphdrawing.org/xmlns\">\n";
    for (size_t k = 0; k < keys.size(); ++k) {
        head += "  <key id=\"d" + std::to_string(k) + "\" for=\"" + (keys[k].node ? "node" : "edge") + "\" attr.name=\"";
        put_xml(head, keys[k].name);
        head += keys[k].numeric ? "\" attr.type=\"double\" />\n" : "\" attr.type=\"string\" />\n";
    }
    head += std::string("  <graph edgedefault=\"") + (g->directed ? "directed" : "undirected") + "\">\n";
    bool ok = fwrite(head.data(), 1, head.size(), f) == head.size();
    auto vid = [&](std::string& o, int32_t v) {
        if (ids && !(*ids)[size_t(v)].empty()) put_xml(o, (*ids)[size_t(v)]);
        else put_xml(o, fallback_id.at(v));
    };
    auto put_data = [&](std::string& o, size_t k, size_t i) {
        const Key& kd = keys[k];
        if (kd.numeric) {
            const double x = (*kd.num)[i];
            if (std::isnan(x)) return;
            o += "<data key=\"d" + std::to_string(k) + "\">";
            put_f64(o, x);
        } else {
            const std::string& x = (*kd.str)[i];
            if (x.empty()) return;
            o += "<data key=\"d" + std::to_string(k) + "\">";
            put_xml(o, x);
        }
        o += "</data>";
    };
    // nodes then edges, formatted in parallel chunks and written in order
    const int nthreads = std::max(1, std::min<int>(16, int(std::thread::hardware_concurrency())));
    auto emit = [&](int64_t n, auto&& one) {
        const int64_t chunk = 65536;
        std::vector<std::string> bufs(static_cast<size_t>(nthreads));
        for (int64_t c0 = 0; c0 < n && ok; c0 += chunk * nthreads) {
            std::vector<std::thread> th;
            for (int t = 0; t < nthreads; ++t)
                th.emplace_back([&, t] {
                    std::string& o = bufs[t];
                    o.clear();
                    const int64_t lo = c0 + t * chunk, hi = std::min(n, lo + chunk);
                    for (int64_t i = lo; i < hi; ++i) one(o, i);
                });
            for (auto& t : th) t.join();
            for (auto& b : bufs)
                if (ok && !b.empty()) ok = fwrite(b.data(), 1, b.size(), f) == b.size();
        }
    };
    emit(g->V, [&](std::string& o, int64_t v) {
        o += "    <node id=\"";
        vid(o, int32_t(v));
        o += "\">";
        for (size_t k = 0; k < keys.size(); ++k)
            if (keys[k].node) put_data(o, k, size_t(v));
        o += "</node>\n";
    });
    emit(g->E, [&](std::string& o, int64_t e) {
        o += "    <edge source=\"";
        vid(o, g->efrom[size_t(e)]);
        o += "\" target=\"";
        vid(o, g->eto[size_t(e)]);
        o += "\">";
        for (size_t k = 0; k < keys.size(); ++k)
            if (!keys[k].node) put_data(o, k, size_t(e));
        o += "</edge>\n";
    });
    static const char tail[] = "  </graph>\n</graphml>\n";
    if (ok) ok = fwrite(tail, 1, sizeof tail - 1, f) == sizeof tail - 1;
    if (fclose(f) != 0) ok = false;
    if (!ok) { shdr::set_error(std::string("save_graphml: write failed: ") + path); return SHDR_EIO; }
    return SHDR_OK;
}

}  // extern "C"
