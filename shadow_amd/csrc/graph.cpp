// Host graph: GraphML reader, validation, canonical-edge index, CSR images,
// synthetic generators and the host half of the shdr_* C-ABI.
//
// The GraphML reader reproduces what igraph_read_graph_graphml (called at
// /root/reference/src/main/routing/shd-topology.c:110) hands to Shadow:
//   * vertex index = order in which a node id is FIRST seen, whether in a <node>
//     element or as an <edge> endpoint (igraph keeps node ids in a trie that
//     assigns the next index on first lookup);
//   * edge index = <edge> element order;
//   * <key attr.type="double|float|int|long"> -> numeric, parsed with strtod;
//     "string" -> string; "boolean" -> numeric 0/1; missing values take the
//     key's <default> or NaN / "";
//   * the node id itself is the vertex attribute "id" (VAS(g,"id",v), :326);
//   * <graph edgedefault="directed"> selects a directed graph.
#include "graph.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <thread>
#include <memory>
#include <unistd.h>
#include <deque>
#include <string_view>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <mutex>
#include <numeric>
#include <sstream>
#include <unordered_set>

namespace shdr {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

static const std::string kEmpty;

double HostGraph::vertex_num(const std::string& a, int32_t v) const {
    auto p = vnum_ptr(a);
    if (!p || v < 0 || v >= V) return std::numeric_limits<double>::quiet_NaN();
    return (*p)[v];
}
const std::string& HostGraph::vertex_str(const std::string& a, int32_t v) const {
    auto it = vstr.find(a);
    if (it == vstr.end() || v < 0 || v >= V) return kEmpty;
    return it->second[v];
}
double HostGraph::edge_num(const std::string& a, int64_t e) const {
    auto p = enum_ptr(a);
    if (!p || e < 0 || e >= E) return std::numeric_limits<double>::quiet_NaN();
    return (*p)[e];
}

void HostGraph::build_canon() {
    // built lazily by the first shdr_graph_get_eid (the engine and the drop-in do
    // not need it: build_csr takes canonical edges from its sorted arc runs)
    if (__atomic_load_n(&canon_built, __ATOMIC_ACQUIRE)) return;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (canon_built) return;
    canon.clear();
    canon.reserve(size_t(E) * 2 + 16);
    for (int64_t e = 0; e < E; ++e) {
        uint64_t k = pair_key(efrom[e], eto[e]);
        auto it = canon.find(k);
        if (it == canon.end()) canon.emplace(k, e);  // keep the lowest index
    }
    __atomic_store_n(&canon_built, true, __ATOMIC_RELEASE);
}

int64_t HostGraph::get_eid(int32_t u, int32_t v) {
    if (u < 0 || v < 0 || u >= V || v >= V) return -1;
    build_canon();
    auto it = canon.find(pair_key(u, v));
    return it == canon.end() ? -1 : it->second;
}

// ---------------------------------------------------------------- validation
// Strong connectivity + SCC count (igraph_is_connected / igraph_clusters STRONG,
// shd-topology.c:241,248), completeness exactly as _topology_isComplete
// (:129-230) and the latency>0 edge check (:414-419).
int HostGraph::check() {
    shdr_graph_info in{};
    in.vertex_count = V;
    in.edge_count = E;
    in.is_directed = directed ? 1 : 0;

    // adjacency (out and, for directed graphs, in) without copies of attributes
    std::vector<int64_t> optr(V + 1, 0), iptr(V + 1, 0);
    for (int64_t e = 0; e < E; ++e) {
        optr[efrom[e] + 1]++;
        iptr[eto[e] + 1]++;
        if (!directed) { optr[eto[e] + 1]++; iptr[efrom[e] + 1]++; }
    }
    for (int32_t v = 0; v < V; ++v) { optr[v + 1] += optr[v]; iptr[v + 1] += iptr[v]; }
    std::vector<int32_t> oadj(optr[V]), iadj(iptr[V]);
    {
        std::vector<int64_t> oc(optr.begin(), optr.end() - 1), ic(iptr.begin(), iptr.end() - 1);
        for (int64_t e = 0; e < E; ++e) {
            int32_t a = efrom[e], b = eto[e];
            oadj[oc[a]++] = b;
            iadj[ic[b]++] = a;
            if (!directed) { oadj[oc[b]++] = a; iadj[ic[a]++] = b; }
        }
    }

    // SCC count: Kosaraju, iterative.
    int32_t scc = 0;
    if (V > 0) {
        std::vector<int32_t> order;
        order.reserve(V);
        std::vector<uint8_t> seen(V, 0);
        std::vector<std::pair<int32_t, int64_t>> st;
        for (int32_t s = 0; s < V; ++s) {
            if (seen[s]) continue;
            seen[s] = 1;
            st.push_back({s, optr[s]});
            while (!st.empty()) {
                auto& top = st.back();
                if (top.second < optr[top.first + 1]) {
                    int32_t w = oadj[top.second++];
                    if (!seen[w]) { seen[w] = 1; st.push_back({w, optr[w]}); }
                } else {
                    order.push_back(top.first);
                    st.pop_back();
                }
            }
        }
        std::vector<int32_t> comp(V, -1);
        std::vector<int32_t> stk;
        for (int32_t k = V - 1; k >= 0; --k) {
            int32_t s = order[k];
            if (comp[s] >= 0) continue;
            comp[s] = scc;
            stk.push_back(s);
            while (!stk.empty()) {
                int32_t x = stk.back();
                stk.pop_back();
                for (int64_t p = iptr[x]; p < iptr[x + 1]; ++p) {
                    int32_t y = iadj[p];
                    if (comp[y] < 0) { comp[y] = scc; stk.push_back(y); }
                }
            }
            ++scc;
        }
    }
    in.cluster_count = scc;
    in.is_connected = (V > 0 && scc == 1) ? 1 : 0;

    // completeness (:167-219): incident count per vertex with igraph_incident
    // semantics (undirected: every incident edge, a self-loop twice; directed:
    // out-edges), minus one if undirected and a self-loop exists (:187-199).
    std::vector<int64_t> cnt(V, 0);
    std::vector<uint8_t> has_loop(V, 0);
    int64_t loops = 0;
    for (int64_t e = 0; e < E; ++e) {
        int32_t a = efrom[e], b = eto[e];
        if (a == b) { has_loop[a] = 1; ++loops; }
        cnt[a]++;
        if (!directed) cnt[b]++;
    }
    bool complete = true;
    for (int32_t v = 0; v < V; ++v) {
        int64_t c = cnt[v];
        if (!directed && has_loop[v]) c -= 1;
        if (c < V) { complete = false; break; }
    }
    in.is_complete = complete ? 1 : 0;
    in.self_loops = loops;

    int64_t bad = 0;
    auto lat = enum_ptr("latency");
    for (int64_t e = 0; e < E; ++e) {
        double l = lat ? (*lat)[e] : std::numeric_limits<double>::quiet_NaN();
        if (l <= 0) ++bad;  // NaN passes, as `latency <= 0` does at :414
    }
    in.bad_latency_edges = bad;
    info = in;
    checked = true;
    return SHDR_OK;
}

// ---------------------------------------------------------------- CSR images
namespace {
// Arcs grouped by a key vertex (counting sort), each group sorted by (other
// vertex, edge index) in parallel; `ptr` = group offsets, `oth` / `eid` = the
// sorted arcs. Canonical edge of (key, other) = the first arc of its run (the
// lowest edge index joining them, igraph_get_eid's choice, :189,:643-645).
// each(f) calls f(k, other, edge) for every arc; a template (not std::function) so the
// two passes over 12 M arcs of a 1M-vertex map inline
template <typename Each>
void group_arcs(int32_t V, int64_t A, Each&& each, std::vector<int64_t>& ptr, std::vector<int32_t>& oth,
                std::vector<int64_t>& eid) {
    ptr.assign(size_t(V) + 1, 0);
    each([&](int32_t k, int32_t, int64_t) { ptr[size_t(k) + 1]++; });
    for (int32_t v = 0; v < V; ++v) ptr[v + 1] += ptr[v];
    oth.resize(size_t(A));
    eid.resize(size_t(A));
    {
        std::vector<int64_t> cur(ptr.begin(), ptr.end() - 1);
        each([&](int32_t k, int32_t o, int64_t e) {
            const int64_t i = cur[size_t(k)]++;
            oth[size_t(i)] = o;
            eid[size_t(i)] = e;
        });
    }
    // rows are already in edge order; sort each by (other, edge) — in parallel
    const int nt = std::max(1, std::min<int>(16, int(std::thread::hardware_concurrency())));
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            std::vector<std::pair<int32_t, int64_t>> tmp;
            const int32_t v0 = int32_t(int64_t(V) * t / nt), v1 = int32_t(int64_t(V) * (t + 1) / nt);
            for (int32_t v = v0; v < v1; ++v) {
                const int64_t a = ptr[v], b = ptr[v + 1];
                bool sorted = true;
                for (int64_t i = a + 1; i < b && sorted; ++i)
                    sorted = oth[size_t(i - 1)] < oth[size_t(i)] || (oth[size_t(i - 1)] == oth[size_t(i)] && eid[size_t(i - 1)] < eid[size_t(i)]);
                if (sorted) continue;
                tmp.clear();
                for (int64_t i = a; i < b; ++i) tmp.emplace_back(oth[size_t(i)], eid[size_t(i)]);
                std::sort(tmp.begin(), tmp.end());
                for (int64_t i = a; i < b; ++i) { oth[size_t(i)] = tmp[size_t(i - a)].first; eid[size_t(i)] = tmp[size_t(i - a)].second; }
            }
        });
    for (auto& x : th) x.join();
}
}  // namespace

void build_csr(HostGraph& g, CsrImage& c) {
    if (!g.checked) g.check();
    const int32_t V = g.V;
    c.V = V;
    c.directed = g.directed;
    c.same_in_out = !g.directed;
    const std::vector<double>* lat = g.enum_ptr("latency");
    const std::vector<double>* elo = g.enum_ptr("packetloss");
    const std::vector<double>* vlo = g.vnum_ptr("packetloss");
    auto L = [&](int64_t e) { return lat ? (*lat)[e] : std::numeric_limits<double>::quiet_NaN(); };
    // (1.0f - EAN(packetloss)) in double arithmetic, :657
    auto R = [&](int64_t e) { return 1.0 - (elo ? (*elo)[e] : std::numeric_limits<double>::quiet_NaN()); };
    // per-hop jitter, summed along paths by the complete-topology precompute
    // (compute-topology-paths.py:30-33); only kept when the graph has it
    const std::vector<double>* ejit = g.enum_ptr("jitter");

    c.vrel.assign(V, 1.0);
    c.self_lat.assign(V, std::numeric_limits<double>::quiet_NaN());
    c.self_rel.assign(V, std::numeric_limits<double>::quiet_NaN());
    for (int32_t v = 0; v < V; ++v) c.vrel[v] = 1.0 - (vlo ? (*vlo)[v] : std::numeric_limits<double>::quiet_NaN());
    int64_t A = 0;
    std::vector<char> has_self(size_t(V), 0);
    for (int64_t e = 0; e < g.E; ++e) {
        const int32_t a = g.efrom[e], b = g.eto[e];
        if (a == b) {  // self-loops never improve a distance; the lowest-index one is kept per vertex
            if (!has_self[a]) { has_self[a] = 1; c.self_lat[a] = L(e); c.self_rel[a] = R(e); }
            continue;
        }
        A += g.directed ? 1 : 2;
    }
    c.A = A;
    // out-CSR sorted by (u, v, e)
    std::vector<int64_t> eid;
    group_arcs(V, A, [&](auto&& f) {
        for (int64_t e = 0; e < g.E; ++e) {
            const int32_t a = g.efrom[e], b = g.eto[e];
            if (a == b) continue;
            f(a, b, e);
            if (!g.directed) f(b, a, e);
        }
    }, c.rowptr, c.col, eid);
    c.w.resize(A);
    c.oclat.resize(A);
    c.ocrel.resize(A);
    c.ocjit.resize(ejit ? A : 0);
    // per-arc values, rows in parallel (a row's canonical edge is the first of its (u, v) run)
    const int nt = std::max(1, std::min<int>(16, int(std::thread::hardware_concurrency())));
    std::vector<double> wpart(size_t(nt), 0.0);
    {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                const int32_t u0 = int32_t(int64_t(V) * t / nt), u1 = int32_t(int64_t(V) * (t + 1) / nt);
                double ws = 0.0;
                int64_t ce = -1;
                for (int32_t u = u0; u < u1; ++u)
                    for (int64_t i = c.rowptr[u]; i < c.rowptr[u + 1]; ++i) {
                        if (i == c.rowptr[u] || c.col[i] != c.col[i - 1]) ce = eid[i];
                        c.w[i] = L(eid[i]);
                        c.oclat[i] = L(ce);
                        c.ocrel[i] = R(ce);
                        if (ejit) c.ocjit[i] = (*ejit)[ce];
                        ws += c.w[i];
                    }
                wpart[size_t(t)] = ws;
            });
        for (auto& x : th) x.join();
    }
    double wsum = 0.0;
    for (double x : wpart) wsum += x;  // (mean_w only sets the relaxation window, never a result)
    int64_t ce = -1;
    c.mean_w = A ? wsum / double(A) : 1.0;
    // multi-edges with different latencies relax with their own weight but the
    // epilogue reads the canonical (get_eid) edge: then the latency must be summed
    c.lat_is_w = A == 0 || std::memcmp(c.w.data(), c.oclat.data(), size_t(A) * sizeof(double)) == 0;
    if (!g.directed) {
        // in-arcs of v == out-arcs of v reversed; canonical edge symmetric.
        c.irowptr.clear(); c.isrc.clear(); c.iw.clear(); c.iclat.clear(); c.icrel.clear(); c.icjit.clear();
        return;
    }
    // in-CSR sorted by (v, u, e)
    group_arcs(V, A, [&](auto&& f) {
        for (int64_t e = 0; e < g.E; ++e) {
            const int32_t a = g.efrom[e], b = g.eto[e];
            if (a != b) f(b, a, e);
        }
    }, c.irowptr, c.isrc, eid);
    c.iw.resize(A);
    c.iclat.resize(A);
    c.icrel.resize(A);
    c.icjit.resize(ejit ? A : 0);
    for (int32_t v = 0; v < V; ++v)
        for (int64_t i = c.irowptr[v]; i < c.irowptr[v + 1]; ++i) {
            if (i == c.irowptr[v] || c.isrc[i] != c.isrc[i - 1]) ce = eid[i];
            c.iw[i] = L(eid[i]);
            c.iclat[i] = L(ce);
            c.icrel[i] = R(ce);
            if (ejit) c.icjit[i] = (*ejit)[ce];
        }
}

// ---------------------------------------------------------------- GraphML
namespace {

struct KeyDef {
    std::string name;
    bool numeric = true;
    bool boolean = false;
    bool for_node = true;  // false: for edge (graph/all keys are ignored except "all")
    bool for_all = false;
    bool has_default = false;
    std::string def;
};

void decode_entities(const char* b, const char* e, std::string& out) {
    out.clear();
    out.reserve(size_t(e - b));
    for (const char* p = b; p < e; ++p) {
        if (*p != '&') { out.push_back(*p); continue; }
        const char* semi = (const char*)memchr(p, ';', size_t(e - p));
        if (!semi) { out.push_back(*p); continue; }
        std::string ent(p + 1, semi);
        if (ent == "lt") out.push_back('<');
        else if (ent == "gt") out.push_back('>');
        else if (ent == "amp") out.push_back('&');
        else if (ent == "quot") out.push_back('"');
        else if (ent == "apos") out.push_back('\'');
        else if (!ent.empty() && ent[0] == '#') {
            unsigned long cp = (ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X'))
                                   ? strtoul(ent.c_str() + 2, nullptr, 16)
                                   : strtoul(ent.c_str() + 1, nullptr, 10);
            if (cp < 0x80) out.push_back(char(cp));
            else if (cp < 0x800) { out.push_back(char(0xC0 | (cp >> 6))); out.push_back(char(0x80 | (cp & 0x3F))); }
            else if (cp < 0x10000) {
                out.push_back(char(0xE0 | (cp >> 12))); out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
                out.push_back(char(0x80 | (cp & 0x3F)));
            } else {
                out.push_back(char(0xF0 | (cp >> 18))); out.push_back(char(0x80 | ((cp >> 12) & 0x3F)));
                out.push_back(char(0x80 | ((cp >> 6) & 0x3F))); out.push_back(char(0x80 | (cp & 0x3F)));
            }
        } else {
            out.append(p, semi + 1);
        }
        p = semi;
    }
}

inline bool is_space(char ch) { return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\r'; }

// One start or end tag as views into the document (no allocation per tag).
struct Tag {
    std::string_view name;  // local name (namespace prefix stripped)
    bool closing = false;
    bool selfclose = false;
    struct Attr { std::string_view name, raw; };  // raw value, entities not decoded
    Attr attrs[16];
    int nattrs = 0;
    const Attr* find(std::string_view k) const {
        for (int i = 0; i < nattrs; ++i)
            if (attrs[i].name == k) return &attrs[i];
        return nullptr;
    }
};

// Attribute value, entity-decoded; returns a view into the document when there
// is nothing to decode, else into `scratch`.
std::string_view attr_value(const Tag::Attr& a, std::string& scratch) {
    if (a.raw.find('&') == std::string_view::npos) return a.raw;
    decode_entities(a.raw.data(), a.raw.data() + a.raw.size(), scratch);
    return scratch;
}

std::string_view local_name(const char* b, const char* e) {
    std::string_view q(b, size_t(e - b));
    const size_t c = q.find(':');
    return c == std::string_view::npos ? q : q.substr(c + 1);
}

// Parses the tag starting at p (p[0]=='<', not a comment/PI/CDATA). Returns
// pointer past '>' or nullptr.
const char* parse_tag(const char* p, const char* end, Tag& t) {
    t.nattrs = 0;
    t.closing = t.selfclose = false;
    ++p;
    if (p < end && *p == '/') { t.closing = true; ++p; }
    const char* nb = p;
    while (p < end && !is_space(*p) && *p != '>' && *p != '/') ++p;
    t.name = local_name(nb, p);
    while (p < end) {
        while (p < end && is_space(*p)) ++p;
        if (p >= end) return nullptr;
        if (*p == '>') return p + 1;
        if (*p == '/') {
            t.selfclose = true;
            ++p;
            while (p < end && *p != '>') ++p;
            return p < end ? p + 1 : nullptr;
        }
        const char* ab = p;
        while (p < end && *p != '=' && !is_space(*p) && *p != '>') ++p;
        Tag::Attr at{local_name(ab, p), std::string_view()};
        while (p < end && is_space(*p)) ++p;
        if (p < end && *p == '=') {
            ++p;
            while (p < end && is_space(*p)) ++p;
            if (p >= end) return nullptr;
            const char q = *p;
            if (q != '"' && q != '\'') return nullptr;
            ++p;
            const char* vb = p;
            p = (const char*)memchr(p, q, size_t(end - p));
            if (!p) return nullptr;
            at.raw = std::string_view(vb, size_t(p - vb));
            ++p;
        }
        if (t.nattrs < 16) t.attrs[t.nattrs++] = at;
    }
    return nullptr;
}

// Node id -> vertex index: open addressing over (hash, view) slots. The ids are
// looked up once per node and twice per edge (10M lookups at cfg5 scale), which
// dominated a node-based std::unordered_map with cache misses.
class IdMap {
  public:
    int32_t find_or_add(std::string_view id, int32_t next) { return find_or_add(id, hash(id), next); }
    int32_t find_or_add(std::string_view id, uint64_t h, int32_t next) {
        if (2 * (n_ + 1) > slots_.size()) grow();
        size_t i = size_t(h) & (slots_.size() - 1);
        for (;;) {
            Slot& s = slots_[i];
            if (s.v < 0) {
                s = Slot{h, id.data(), uint32_t(id.size()), next};
                ++n_;
                return next;
            }
            if (s.h == h && s.len == id.size() && memcmp(s.p, id.data(), id.size()) == 0) return s.v;
            i = (i + 1) & (slots_.size() - 1);
        }
    }

    static uint64_t hash(std::string_view s) {  // FNV-1a, then a finalizer for the low bits
        uint64_t h = 1469598103934665603ull;
        for (char c : s) h = (h ^ uint8_t(c)) * 1099511628211ull;
        h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
        return h;
    }

    void reserve(size_t n) {  // room for n ids without growing
        size_t cap = 1024;
        while (cap < 2 * (n + 1)) cap *= 2;
        while (slots_.size() < cap) grow();
    }
    void prefetch(uint64_t h) const {
        if (!slots_.empty()) __builtin_prefetch(&slots_[size_t(h) & (slots_.size() - 1)]);
    }

  private:
    struct Slot { uint64_t h = 0; const char* p = nullptr; uint32_t len = 0; int32_t v = -1; };
    void grow() {
        std::vector<Slot> old(std::max<size_t>(1024, slots_.size() * 2));
        old.swap(slots_);
        for (const Slot& s : old) {
            if (s.v < 0) continue;
            size_t i = size_t(s.h) & (slots_.size() - 1);
            while (slots_[i].v >= 0) i = (i + 1) & (slots_.size() - 1);
            slots_[i] = s;
        }
    }
    std::vector<Slot> slots_;
    size_t n_ = 0;
};

double parse_numeric(std::string_view s, bool boolean) {
    if (boolean) {
        std::string t;
        for (char ch : s)
            if (!is_space(ch)) t.push_back(char(tolower((unsigned char)ch)));
        if (t == "true" || t == "yes" || t == "1") return 1.0;
        return 0.0;
    }
    if (s.empty()) return 0.0;  // strtod("")
    // strtod stops at the first character that cannot continue a number; text
    // views end at the '<' of the closing tag, so no copy is needed there
    if (s.data()[s.size()] == '<') return strtod(s.data(), nullptr);
    return strtod(std::string(s).c_str(), nullptr);
}

// What the serial reader knows when it reaches the first <node>/<edge> of the
// graph: the key set (declarations precede the graph) and its attribute columns.
struct GraphmlHeader {
    std::vector<KeyDef> keys;
    std::unordered_map<std::string, int> key_index;
    std::vector<int> vcol, ecol;
    size_t nvnum = 0, nvstr = 0, nenum = 0, nestr = 0;
    bool directed = false;
    const char* body = nullptr;  // the first <node>/<edge> start tag
};

}  // namespace

// GraphML -> HostGraph with igraph's reader conventions. Single pass: <data>
// values are converted straight into per-key attribute columns (numeric keys
// parsed in place), node ids are hashed as views into the document. With `hdr`
// set it stops at the graph's first <node>/<edge> and returns nullptr with the
// header filled in (parse_graphml_parallel continues from there).
HostGraph* parse_graphml_serial(const char* text, size_t len, std::string& err, GraphmlHeader* hdr = nullptr) {
    const char* p = text;
    const char* end = text + len;
    std::vector<KeyDef> keys;
    std::unordered_map<std::string, int> key_index;  // key id -> keys[]
    IdMap ids;  // node id -> vertex index (first seen)
    std::deque<std::string> decoded_ids;  // ids that needed entity decoding (stable storage)
    std::vector<std::string_view> id_of;
    // attribute columns, in key declaration order; -1 where a key does not apply
    std::vector<int> vcol, ecol;                       // key -> column slot
    std::vector<std::vector<double>> vnum, enumr;
    std::vector<std::vector<std::string>> vstr, estr;
    std::vector<int32_t> efrom, eto;
    bool in_graph = false, directed = false, seen_graph = false;
    int depth_graph = 0;
    enum Ctx { NONE, NODE, EDGE, KEY } ctx = NONE;
    int32_t cur_v = -1;
    int64_t cur_e = -1;
    int cur_key = -1;  // key of the open <data>/<default>
    int current_keydef = -1;
    bool in_data = false, in_default = false;
    // text of the open <data>: a direct view while it is one plain piece
    const char* text_b = nullptr;
    const char* text_e = nullptr;
    bool text_complex = false;  // CDATA, several pieces or entities: use text_acc
    std::string text_acc, dec, scratch;
    bool columns_ready = false;

    auto node_key = [&](const KeyDef& kd) { return (kd.for_node || kd.for_all) && kd.name != "id"; };
    auto edge_key = [&](const KeyDef& kd) { return !kd.for_node || kd.for_all; };
    auto make_columns = [&] {  // keys precede the graph in GraphML; columns follow the key set
        columns_ready = true;
        vcol.assign(keys.size(), -1);
        ecol.assign(keys.size(), -1);
        for (size_t k = 0; k < keys.size(); ++k) {
            if (node_key(keys[k])) {
                vcol[k] = int(keys[k].numeric ? vnum.size() : vstr.size());
                if (keys[k].numeric) vnum.emplace_back(); else vstr.emplace_back();
            }
            if (edge_key(keys[k])) {
                ecol[k] = int(keys[k].numeric ? enumr.size() : estr.size());
                if (keys[k].numeric) enumr.emplace_back(); else estr.emplace_back();
            }
        }
    };
    const double nan = std::numeric_limits<double>::quiet_NaN();
    auto defaults = [&](bool node) {  // append one element's default values to every column
        for (size_t k = 0; k < keys.size(); ++k) {
            const int c = node ? vcol[k] : ecol[k];
            if (c < 0) continue;
            const KeyDef& kd = keys[k];
            if (kd.numeric) (node ? vnum : enumr)[size_t(c)].push_back(kd.has_default ? parse_numeric(kd.def, kd.boolean) : nan);
            else (node ? vstr : estr)[size_t(c)].push_back(kd.has_default ? kd.def : std::string());
        }
    };
    auto vertex_of = [&](std::string_view id) -> int32_t {
        if (id.data() < text || id.data() >= end) {  // decoded: the map keeps views, give it a stable copy
            decoded_ids.emplace_back(id);
            id = decoded_ids.back();
        }
        const int32_t next = int32_t(id_of.size());
        const int32_t v = ids.find_or_add(id, next);
        if (v == next) {
            id_of.push_back(id);
            defaults(true);
        }
        return v;
    };
    auto text_value = [&]() -> std::string_view {
        if (!text_complex) {
            std::string_view raw = text_b ? std::string_view(text_b, size_t(text_e - text_b)) : std::string_view();
            if (raw.find('&') == std::string_view::npos) return raw;
            text_acc.assign(raw);
        }
        decode_entities(text_acc.data(), text_acc.data() + text_acc.size(), dec);
        return dec;
    };
    auto add_text = [&](const char* b, const char* e) {
        if (b == e) return;
        if (!text_complex && !text_b) { text_b = b; text_e = e; return; }
        if (!text_complex) { text_acc.assign(text_b, text_e); text_complex = true; }
        text_acc.append(b, e);
    };
    auto open_text = [&] { text_b = text_e = nullptr; text_complex = false; text_acc.clear(); };

    Tag t;
    while (p < end) {
        const char* lt = (const char*)memchr(p, '<', size_t(end - p));
        if (!lt) break;
        if (in_data || in_default) add_text(p, lt);
        p = lt;
        if (end - p >= 4 && memcmp(p, "<!--", 4) == 0) {
            const char* q = strstr(p + 4, "-->");
            if (!q || q > end) { err = "unterminated comment"; return nullptr; }
            p = q + 3;
            continue;
        }
        if (end - p >= 9 && memcmp(p, "<![CDATA[", 9) == 0) {
            const char* q = p + 9;
            const char* c = nullptr;
            for (const char* s = q; s + 3 <= end; ++s)
                if (s[0] == ']' && s[1] == ']' && s[2] == '>') { c = s; break; }
            if (!c) { err = "unterminated CDATA"; return nullptr; }
            if (in_data || in_default) {
                // CDATA is literal: protect '&' from entity decoding
                if (!text_complex) { text_acc.assign(text_b ? text_b : q, text_b ? text_e : q); text_complex = true; }
                for (const char* s = q; s < c; ++s) {
                    if (*s == '&') text_acc += "&amp;"; else text_acc.push_back(*s);
                }
            }
            p = c + 3;
            continue;
        }
        if (end - p >= 2 && (p[1] == '?' || p[1] == '!')) {
            const char* q = (const char*)memchr(p, '>', size_t(end - p));
            if (!q) { err = "unterminated declaration"; return nullptr; }
            p = q + 1;
            continue;
        }
        const char* nx = parse_tag(p, end, t);
        if (!nx) { err = "malformed tag"; return nullptr; }
        const std::string_view n = t.name;
        if (hdr && !t.closing && (n == "node" || n == "edge") && in_graph && depth_graph == 1 && !in_data &&
            !in_default && ctx == NONE) {
            hdr->keys = keys;
            hdr->key_index = key_index;
            hdr->vcol = vcol;
            hdr->ecol = ecol;
            hdr->nvnum = vnum.size(); hdr->nvstr = vstr.size(); hdr->nenum = enumr.size(); hdr->nestr = estr.size();
            hdr->directed = directed;
            hdr->body = p;
            return nullptr;
        }
        p = nx;
        if (!t.closing) {
            if (n == "key") {
                KeyDef kd;
                const Tag::Attr* id = t.find("id");
                const Tag::Attr* an = t.find("attr.name");
                const Tag::Attr* at = t.find("attr.type");
                const Tag::Attr* fo = t.find("for");
                if (!id) { err = "key without id"; return nullptr; }
                const std::string idv(attr_value(*id, scratch));
                kd.name = an ? std::string(attr_value(*an, scratch)) : idv;
                const std::string ty = at ? std::string(attr_value(*at, scratch)) : "string";
                kd.numeric = (ty == "double" || ty == "float" || ty == "int" || ty == "long" || ty == "boolean");
                kd.boolean = (ty == "boolean");
                const std::string f = fo ? std::string(attr_value(*fo, scratch)) : "all";
                kd.for_all = (f == "all");
                kd.for_node = (f == "node");
                if (columns_ready) continue;  // a key after graph elements cannot be used (igraph: error)
                auto it = key_index.find(idv);
                if (it != key_index.end()) keys[size_t(it->second)] = kd;  // redefinition: last wins
                else { key_index.emplace(idv, int(keys.size())); keys.push_back(kd); }
                current_keydef = key_index[idv];
                if (!t.selfclose) ctx = KEY;
            } else if (n == "default" && ctx == KEY) {
                in_default = !t.selfclose;
                open_text();
            } else if (n == "graph") {
                ++depth_graph;
                if (!seen_graph && depth_graph == 1) {
                    seen_graph = true;
                    in_graph = true;
                    if (!columns_ready) make_columns();
                    const Tag::Attr* ed = t.find("edgedefault");
                    directed = ed && attr_value(*ed, scratch) == "directed";
                }
                if (t.selfclose) { --depth_graph; if (in_graph) in_graph = false; }
            } else if (n == "node" && in_graph && depth_graph == 1) {
                const Tag::Attr* id = t.find("id");
                if (!id) { err = "node without id"; return nullptr; }
                cur_v = vertex_of(attr_value(*id, scratch));
                ctx = t.selfclose ? NONE : NODE;
            } else if (n == "edge" && in_graph && depth_graph == 1) {
                const Tag::Attr* s = t.find("source");
                const Tag::Attr* d = t.find("target");
                if (!s || !d) { err = "edge without source/target"; return nullptr; }
                const int32_t a = vertex_of(attr_value(*s, scratch));
                const int32_t b = vertex_of(attr_value(*d, scratch));
                efrom.push_back(a);
                eto.push_back(b);
                defaults(false);
                cur_e = int64_t(efrom.size()) - 1;
                ctx = t.selfclose ? NONE : EDGE;
            } else if (n == "data" && (ctx == NODE || ctx == EDGE)) {
                const Tag::Attr* k = t.find("key");
                auto it = k ? key_index.find(std::string(attr_value(*k, scratch))) : key_index.end();
                cur_key = it == key_index.end() ? -1 : it->second;
                open_text();
                in_data = !t.selfclose;
                if (t.selfclose) { in_data = true; goto close_data; }  // empty value
            }
            continue;
        }
        if (n == "data" && in_data) {
        close_data:
            if (cur_key >= 0) {
                const KeyDef& kd = keys[size_t(cur_key)];
                const bool node = ctx == NODE;
                const int c = node ? vcol[size_t(cur_key)] : (ctx == EDGE ? ecol[size_t(cur_key)] : -1);
                if (c >= 0) {
                    const std::string_view val = text_value();
                    if (kd.numeric) (node ? vnum : enumr)[size_t(c)][node ? size_t(cur_v) : size_t(cur_e)] = parse_numeric(val, kd.boolean);
                    else (node ? vstr : estr)[size_t(c)][node ? size_t(cur_v) : size_t(cur_e)] = std::string(val);
                }
            }
            in_data = false;
        } else if (n == "default" && in_default) {
            if (current_keydef >= 0) {
                keys[size_t(current_keydef)].has_default = true;
                keys[size_t(current_keydef)].def = std::string(text_value());
            }
            in_default = false;
        } else if (n == "key") {
            ctx = NONE;
        } else if (n == "node" || n == "edge") {
            ctx = NONE;
        } else if (n == "graph") {
            --depth_graph;
            if (in_graph && depth_graph == 0) in_graph = false;
        }
    }
    if (!seen_graph) { err = "no <graph> element"; return nullptr; }

    auto* g = new HostGraph();
    g->V = int32_t(id_of.size());
    g->E = int64_t(efrom.size());
    g->directed = directed;
    g->efrom = std::move(efrom);
    g->eto = std::move(eto);
    std::vector<std::string>& idcol = g->vstr["id"];
    idcol.reserve(id_of.size());
    for (std::string_view id : id_of) idcol.emplace_back(id);
    for (size_t k = 0; k < keys.size(); ++k) {
        const KeyDef& kd = keys[k];
        if (vcol[k] >= 0) {
            if (kd.numeric) g->vnum[kd.name] = std::move(vnum[size_t(vcol[k])]);
            else g->vstr[kd.name] = std::move(vstr[size_t(vcol[k])]);
        }
        if (ecol[k] >= 0) {
            if (kd.numeric) g->enumr[kd.name] = std::move(enumr[size_t(ecol[k])]);
            else g->estr[kd.name] = std::move(estr[size_t(ecol[k])]);
        }
    }
    return g;
}

namespace {

// One <node>/<edge> of the graph body as a chunk parser saw it, and its <data> values.
struct BodyElem {
    bool edge = false;
    uint32_t d0 = 0, nd = 0;  // its values: Chunk::vals[d0, d0 + nd)
    std::string_view a, b;    // node id / edge source, target
    uint64_t ha = 0, hb = 0;
};
struct BodyVal {
    int key = -1;
    double num = 0.0;
    std::string_view str;  // string keys (a view into the document or Chunk::decoded)
};
struct BodyChunk {
    std::vector<BodyElem> el;
    std::vector<BodyVal> vals;
    std::deque<std::string> decoded;  // entity-decoded ids and values (stable storage)
    bool unsupported = false;         // a construct this path does not take: parse serially
};

// the next "<node" / "<edge" start tag at or after p (nullptr if none before e)
const char* next_element(const char* p, const char* e) {
    while (p < e) {
        const char* lt = static_cast<const char*>(memchr(p, '<', size_t(e - p)));
        if (!lt || e - lt < 6) return nullptr;
        if ((memcmp(lt + 1, "node", 4) == 0 || memcmp(lt + 1, "edge", 4) == 0) &&
            (is_space(lt[5]) || lt[5] == '>' || lt[5] == '/'))
            return lt;
        p = lt + 1;
    }
    return nullptr;
}

// The graph body [b, e) (whole <node>/<edge> elements, no comments, CDATA,
// declarations or nested graphs — the caller checked) as element records.
void parse_body_chunk(const GraphmlHeader& h, const char* b, const char* e, BodyChunk& c) {
    Tag t;
    std::string scratch;
    BodyElem* cur = nullptr;
    auto stable = [&](std::string_view v) -> std::string_view {
        if (v.data() == scratch.data()) { c.decoded.emplace_back(v); return c.decoded.back(); }
        return v;
    };
    auto key_of = [&](std::string_view k) -> int {  // few keys: a linear scan beats hashing a copy
        for (const auto& kv : h.key_index)
            if (kv.first == k) return kv.second;
        return -1;
    };
    const char* p = b;
    while (p < e) {
        const char* lt = static_cast<const char*>(memchr(p, '<', size_t(e - p)));
        if (!lt) break;
        if (e - lt < 2 || lt[1] == '!' || lt[1] == '?') { c.unsupported = true; return; }  // comment, CDATA, declaration
        const char* nx = parse_tag(lt, e, t);
        if (!nx) { c.unsupported = true; return; }
        p = nx;
        const std::string_view n = t.name;
        // prefixed names, nested graphs and late keys: the serial reader's business
        if (n.data() != lt + 1 + (t.closing ? 1 : 0) || n == "graph" || n == "key") { c.unsupported = true; return; }
        if (t.closing) {
            if (n == "node" || n == "edge") cur = nullptr;
            continue;
        }
        if (n == "node" || n == "edge") {
            BodyElem x;
            x.edge = n == "edge";
            x.d0 = uint32_t(c.vals.size());
            if (!x.edge) {
                const Tag::Attr* id = t.find("id");
                if (!id) { c.unsupported = true; return; }  // the serial reader reports it
                x.a = stable(attr_value(*id, scratch));
            } else {
                const Tag::Attr* sa = t.find("source");
                const Tag::Attr* ta = t.find("target");
                if (!sa || !ta) { c.unsupported = true; return; }
                x.a = stable(attr_value(*sa, scratch));
                x.b = stable(attr_value(*ta, scratch));
                x.hb = IdMap::hash(x.b);
            }
            x.ha = IdMap::hash(x.a);
            c.el.push_back(x);
            cur = t.selfclose ? nullptr : &c.el.back();
        } else if (n == "data") {
            std::string_view val;
            if (!t.selfclose) {  // the value is the text up to </data>
                const char* vt = static_cast<const char*>(memchr(p, '<', size_t(e - p)));
                Tag ct;
                const char* cn = vt ? parse_tag(vt, e, ct) : nullptr;
                if (!cn || !ct.closing || ct.name != "data" || ct.name.data() != vt + 2) { c.unsupported = true; return; }
                val = std::string_view(p, size_t(vt - p));
                p = cn;
            }
            if (!cur) continue;  // outside a node/edge: ignored, as the serial reader does
            const Tag::Attr* k = t.find("key");
            const int key = k ? key_of(attr_value(*k, scratch)) : -1;
            if (key < 0) continue;
            const KeyDef& kd = h.keys[size_t(key)];
            BodyVal v;
            v.key = key;
            if (val.find('&') != std::string_view::npos) {
                c.decoded.emplace_back();
                decode_entities(val.data(), val.data() + val.size(), c.decoded.back());
                val = c.decoded.back();
            }
            if (kd.numeric) v.num = parse_numeric(val, kd.boolean);
            else v.str = val;
            c.vals.push_back(v);
            ++cur->nd;
        }
        // any other tag (<desc>, <port>, ...) carries nothing the reader keeps
    }
}

int parse_threads() {
    int nt = std::max(1, std::min<int>(16, int(std::thread::hardware_concurrency())));
    if (const char* x = getenv("OMP_NUM_THREADS")) nt = std::max(1, std::min(nt, atoi(x)));
    return nt;
}

}  // namespace

// Large documents: the serial reader takes the header up to the first
// <node>/<edge>; the body is cut at element starts and parsed by several
// threads into element records (ids hashed, numbers converted); one serial
// merge then assigns vertex indices in document order (igraph's first-seen
// rule) and fills the columns. Anything unusual in the body (comments, CDATA,
// declarations, nested graphs, prefixed names, text-bearing children of
// <data>) sends the document to the serial reader, so results are identical.
// cfg5's 885 MB GraphML: 8.6-10.5 s serial -> 3.3 s with 8 threads (container).
HostGraph* parse_graphml_parallel(const char* text, size_t len, std::string& err, bool* handled) {
    *handled = false;
    const bool tm = getenv("SHDR_PARSE_TIMING") != nullptr;  // phase times on stderr (experiments)
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!tm) return;
        const auto t1 = std::chrono::steady_clock::now();
        fprintf(stderr, "[graphml] %s %.3f s\n", what, std::chrono::duration<double>(t1 - t0).count());
        t0 = t1;
    };
    const char* end = text + len;
    GraphmlHeader h;
    std::string herr;
    if (parse_graphml_serial(text, len, herr, &h) || !h.body) return nullptr;
    lap("header");
    // the body ends at the last </graph>
    const char* bend = nullptr;
    for (const char* q = end - 8; q >= h.body; --q)
        if (*q == '<' && memcmp(q, "</graph", 7) == 0 && (q[7] == '>' || is_space(q[7]))) { bend = q; break; }
    if (!bend) return nullptr;
    lap("checks");
    const int nt = parse_threads();
    std::vector<const char*> cut{h.body};
    for (int i = 1; i < nt; ++i) {
        const char* at = next_element(h.body + size_t(bend - h.body) * size_t(i) / size_t(nt), bend);
        if (at && at > cut.back()) cut.push_back(at);
    }
    cut.push_back(bend);
    std::vector<BodyChunk> ch(cut.size() - 1);
    {
        std::vector<std::thread> th;
        for (size_t i = 0; i < ch.size(); ++i) th.emplace_back([&, i] { parse_body_chunk(h, cut[i], cut[i + 1], ch[i]); });
        for (auto& x : th) x.join();
    }
    lap("chunks");
    for (const auto& c : ch)
        if (c.unsupported) return nullptr;
    // after the body: the rest of the document must be closing tags only
    {
        const char* p = bend;
        Tag t;
        while (p < end) {
            const char* lt = static_cast<const char*>(memchr(p, '<', size_t(end - p)));
            if (!lt) break;
            const char* nx = parse_tag(lt, end, t);
            if (!nx || !t.closing) return nullptr;
            p = nx;
        }
    }
    *handled = true;
    // merge in document order: vertex indices (igraph's first-seen rule) serially,
    // with the hash slots of the next elements prefetched; then the attribute
    // columns in parallel, one column per task, each applying its values in order
    size_t nel = 0, nedge = 0;
    for (const auto& c : ch) {
        nel += c.el.size();
        for (const auto& x : c.el) nedge += x.edge;
    }
    IdMap ids;
    ids.reserve(nel - nedge);
    std::vector<std::string_view> id_of;
    id_of.reserve(nel - nedge);
    std::vector<int32_t> efrom, eto;
    efrom.reserve(nedge);
    eto.reserve(nedge);
    std::vector<std::vector<int64_t>> at(ch.size());  // element -> vertex or edge index
    auto vertex_of = [&](std::string_view id, uint64_t hh) -> int32_t {
        const int32_t next = int32_t(id_of.size());
        const int32_t v = ids.find_or_add(id, hh, next);
        if (v == next) id_of.push_back(id);
        return v;
    };
    constexpr size_t kAhead = 16;
    for (size_t ci = 0; ci < ch.size(); ++ci) {
        const auto& el = ch[ci].el;
        at[ci].resize(el.size());
        for (size_t i = 0; i < el.size(); ++i) {
            if (i + kAhead < el.size()) {
                ids.prefetch(el[i + kAhead].ha);
                if (el[i + kAhead].edge) ids.prefetch(el[i + kAhead].hb);
            }
            const BodyElem& x = el[i];
            if (!x.edge) {
                at[ci][i] = vertex_of(x.a, x.ha);
            } else {
                const int32_t a = vertex_of(x.a, x.ha);
                const int32_t b = vertex_of(x.b, x.hb);
                at[ci][i] = int64_t(efrom.size());
                efrom.push_back(a);
                eto.push_back(b);
            }
        }
    }
    lap("ids");
    const size_t V = id_of.size(), E = efrom.size();
    const double nan = std::numeric_limits<double>::quiet_NaN();
    std::vector<std::vector<double>> vnum(h.nvnum), enumr(h.nenum);
    std::vector<std::vector<std::string>> vstr(h.nvstr), estr(h.nestr);
    {
        std::vector<std::function<void()>> tasks;
        for (size_t k = 0; k < h.keys.size(); ++k) {
            const KeyDef& kd = h.keys[k];
            for (int side = 0; side < 2; ++side) {
                const int cc = side ? h.ecol[k] : h.vcol[k];
                if (cc < 0) continue;
                tasks.push_back([&, k, side, cc] {
                    const bool edge = side == 1;
                    const size_t n = edge ? E : V;
                    std::vector<double>* num = kd.numeric ? &(edge ? enumr : vnum)[size_t(cc)] : nullptr;
                    std::vector<std::string>* str = kd.numeric ? nullptr : &(edge ? estr : vstr)[size_t(cc)];
                    if (num) num->assign(n, kd.has_default ? parse_numeric(kd.def, kd.boolean) : nan);
                    else str->assign(n, kd.has_default ? kd.def : std::string());
                    for (size_t ci = 0; ci < ch.size(); ++ci) {
                        const auto& el = ch[ci].el;
                        for (size_t i = 0; i < el.size(); ++i) {
                            const BodyElem& x = el[i];
                            if (x.edge != edge) continue;
                            for (uint32_t d = 0; d < x.nd; ++d) {
                                const BodyVal& v = ch[ci].vals[x.d0 + d];
                                if (v.key != int(k)) continue;
                                if (num) (*num)[size_t(at[ci][i])] = v.num;
                                else (*str)[size_t(at[ci][i])] = std::string(v.str);
                            }
                        }
                    }
                });
            }
        }
        std::atomic<size_t> next{0};
        std::vector<std::thread> th;
        const size_t nw = std::min<size_t>(tasks.size(), size_t(nt));
        for (size_t w = 0; w < nw; ++w)
            th.emplace_back([&] {
                for (size_t t; (t = next.fetch_add(1)) < tasks.size();) tasks[t]();
            });
        for (auto& x : th) x.join();
    }
    lap("merge");
    auto* g = new HostGraph();
    g->V = int32_t(id_of.size());
    g->E = int64_t(efrom.size());
    g->directed = h.directed;
    g->efrom = std::move(efrom);
    g->eto = std::move(eto);
    std::vector<std::string>& idcol = g->vstr["id"];
    idcol.reserve(id_of.size());
    for (std::string_view id : id_of) idcol.emplace_back(id);
    for (size_t k = 0; k < h.keys.size(); ++k) {
        const KeyDef& kd = h.keys[k];
        if (h.vcol[k] >= 0) {
            if (kd.numeric) g->vnum[kd.name] = std::move(vnum[size_t(h.vcol[k])]);
            else g->vstr[kd.name] = std::move(vstr[size_t(h.vcol[k])]);
        }
        if (h.ecol[k] >= 0) {
            if (kd.numeric) g->enumr[kd.name] = std::move(enumr[size_t(h.ecol[k])]);
            else g->estr[kd.name] = std::move(estr[size_t(h.ecol[k])]);
        }
    }
    (void)err;
    return g;
}

HostGraph* parse_graphml(const char* text, size_t len, std::string& err) {
    const char* mode = getenv("SHDR_GRAPHML_PARALLEL");  // 0: always serial (tests compare the two)
    const bool par = mode ? atoi(mode) != 0 : len >= (size_t(8) << 20);
    if (par && parse_threads() > 1) {
        bool handled = false;
        HostGraph* g = parse_graphml_parallel(text, len, err, &handled);
        if (handled) return g;
    }
    return parse_graphml_serial(text, len, err);
}

// ---------------------------------------------------------------- generators
namespace {
struct Rng {  // xoshiro256** seeded by splitmix64
    uint64_t s[4];
    explicit Rng(uint64_t seed) {
        uint64_t x = seed;
        for (int i = 0; i < 4; ++i) {
            x += 0x9E3779B97F4A7C15ull;
            uint64_t z = x;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            s[i] = z ^ (z >> 31);
        }
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        uint64_t r = rotl(s[1] * 5, 7) * 9;
        uint64_t t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
        s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    double uniform() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
    double uniform(double a, double b) { return a + (b - a) * uniform(); }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};
}  // namespace

HostGraph* generate(int32_t kind, int32_t n, int32_t m, uint64_t seed, std::string& err) {
    if (n < 2 || m < 1 || m >= n) { err = "generate: need n>=2, 1<=m<n"; return nullptr; }
    Rng rng(seed);
    std::vector<int32_t> ef, et;
    if (kind == 0) {
        // Barabasi-Albert: star on m+1 vertices, then every new vertex attaches to
        // m distinct existing vertices chosen proportionally to degree.
        std::vector<int32_t> rep;
        rep.reserve(size_t(2) * size_t(n) * size_t(m));
        for (int32_t i = 1; i <= m; ++i) { ef.push_back(0); et.push_back(i); rep.push_back(0); rep.push_back(i); }
        std::vector<int32_t> chosen;
        for (int32_t v = m + 1; v < n; ++v) {
            chosen.clear();
            while (int32_t(chosen.size()) < m) {
                int32_t t = rep[rng.below(rep.size())];
                if (std::find(chosen.begin(), chosen.end(), t) == chosen.end()) chosen.push_back(t);
            }
            for (int32_t t : chosen) { ef.push_back(v); et.push_back(t); rep.push_back(v); rep.push_back(t); }
        }
    } else if (kind == 1) {
        // Chung-Lu power law (exponent 2.1) with expected total degree 2m per
        // vertex beyond a random recursive spanning tree (connectivity).
        const double gamma = 2.1;
        std::vector<double> wgt(n), cdf(n);
        double sum = 0.0;
        for (int32_t i = 0; i < n; ++i) { wgt[i] = std::pow(double(i) + 10.0, -1.0 / (gamma - 1.0)); sum += wgt[i]; cdf[i] = sum; }
        std::unordered_set<uint64_t> seen;
        seen.reserve(size_t(n) * size_t(m + 2) * 2);
        auto key = [](int32_t a, int32_t b) { if (a > b) std::swap(a, b); return (uint64_t(uint32_t(a)) << 32) | uint32_t(b); };
        // permute vertex labels so hubs are spread over the index space
        std::vector<int32_t> perm(n);
        std::iota(perm.begin(), perm.end(), 0);
        for (int32_t i = n - 1; i > 0; --i) std::swap(perm[i], perm[rng.below(uint64_t(i) + 1)]);
        for (int32_t i = 1; i < n; ++i) {
            int32_t j = int32_t(rng.below(uint64_t(i)));
            int32_t a = perm[i], b = perm[j];
            seen.insert(key(a, b));
            ef.push_back(a); et.push_back(b);
        }
        int64_t target = int64_t(n) * (m - 1);  // tree gives mean degree ~2
        int64_t tries = 0;
        while (int64_t(ef.size()) - (n - 1) < target && tries < target * 20) {
            ++tries;
            double ra = rng.uniform() * sum, rb = rng.uniform() * sum;
            int32_t a = perm[int32_t(std::lower_bound(cdf.begin(), cdf.end(), ra) - cdf.begin())];
            int32_t b = perm[int32_t(std::lower_bound(cdf.begin(), cdf.end(), rb) - cdf.begin())];
            if (a == b) continue;
            if (!seen.insert(key(a, b)).second) continue;
            ef.push_back(a); et.push_back(b);
        }
    } else {
        err = "generate: unknown kind";
        return nullptr;
    }
    auto* g = new HostGraph();
    g->V = n;
    g->directed = false;
    const int64_t Eg = int64_t(ef.size());
    g->E = Eg + n;
    g->efrom = ef;
    g->eto = et;
    auto& lat = g->enumr["latency"];
    auto& jit = g->enumr["jitter"];
    auto& elo = g->enumr["packetloss"];
    lat.resize(g->E); jit.assign(g->E, 0.0); elo.resize(g->E);
    for (int64_t e = 0; e < Eg; ++e) { lat[e] = rng.uniform(1.0, 100.0); elo[e] = rng.uniform(0.0, 0.01); }
    for (int32_t v = 0; v < n; ++v) {
        g->efrom.push_back(v); g->eto.push_back(v);
        lat[Eg + v] = rng.uniform(0.5, 5.0);
        elo[Eg + v] = rng.uniform(0.0, 0.01);
    }
    auto& ids = g->vstr["id"];
    ids.resize(n);
    for (int32_t v = 0; v < n; ++v) ids[v] = "poi-" + std::to_string(v + 1);
    g->vstr["type"].assign(n, "net");
    // a distinct IPv4 per vertex (10.0.0.0/8 by index), so hosts can be placed on
    // chosen vertices through topology_attach's exact-IP hint (shd-topology.c:1091-1111)
    auto& ips = g->vstr["ip"];
    ips.resize(n);
    for (int32_t v = 0; v < n; ++v)
        ips[v] = "10." + std::to_string((v >> 16) & 255) + "." + std::to_string((v >> 8) & 255) + "." + std::to_string(v & 255);
    g->vstr["geocode"].assign(n, "US");
    g->vnum["bandwidthup"].assign(n, 10240.0);
    g->vnum["bandwidthdown"].assign(n, 10240.0);
    g->vnum["asn"].assign(n, 0.0);
    auto& vlo = g->vnum["packetloss"];
    vlo.resize(n);
    for (int32_t v = 0; v < n; ++v) vlo[v] = rng.uniform(0.0, 0.02);
    return g;
}

// ---------------------------------------------------------------- binary graph image
// A parsed graph (endpoints + every attribute column) as one flat file, so a
// topology of cfg5 size (865 MB of GraphML, ~10 s to parse) loads in well under
// a second the next time. Native byte order; the header
// carries a hash of the GraphML it was made from.
namespace {
constexpr char kBinMagic[8] = {'S', 'H', 'D', 'R', 'G', 'R', 'F', '1'};

uint64_t content_hash(const char* p, size_t n) {  // 64-bit multiply-xorshift over 8-byte words
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0xff51afd7ed558ccdull;
        h ^= h >> 32;
    }
    for (; i < n; ++i) h = (h ^ uint8_t(p[i])) * 0x100000001b3ull;
    h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull; h ^= h >> 33;
    return h;
}

struct Writer {
    FILE* f;
    bool ok = true;
    void raw(const void* p, size_t n) { if (ok && n && fwrite(p, 1, n, f) != n) ok = false; }
    template <typename T> void pod(const T& v) { raw(&v, sizeof v); }
    void str(const std::string& s) { pod(uint32_t(s.size())); raw(s.data(), s.size()); }
};
struct Reader {
    const char* p;
    const char* end;
    bool ok = true;
    void raw(void* dst, size_t n) {
        if (!ok || size_t(end - p) < n) { ok = false; return; }
        memcpy(dst, p, n);
        p += n;
    }
    template <typename T> T pod() { T v{}; raw(&v, sizeof v); return v; }
    std::string str() {
        const uint32_t n = pod<uint32_t>();
        if (!ok || size_t(end - p) < n) { ok = false; return {}; }
        std::string s(p, n);
        p += n;
        return s;
    }
};

void write_strcols(Writer& w, const std::map<std::string, std::vector<std::string>>& cols) {
    w.pod(uint32_t(cols.size()));
    for (auto& kv : cols) {
        w.str(kv.first);
        std::vector<uint64_t> off(kv.second.size() + 1, 0);
        for (size_t i = 0; i < kv.second.size(); ++i) off[i + 1] = off[i] + kv.second[i].size();
        w.raw(off.data(), off.size() * 8);
        for (auto& x : kv.second) w.raw(x.data(), x.size());
    }
}
bool read_strcols(Reader& r, std::map<std::string, std::vector<std::string>>& cols, size_t n) {
    const uint32_t nc = r.pod<uint32_t>();
    for (uint32_t c = 0; c < nc && r.ok; ++c) {
        std::string name = r.str();
        std::vector<uint64_t> off(n + 1);
        r.raw(off.data(), off.size() * 8);
        if (!r.ok || off[n] > uint64_t(r.end - r.p)) return false;
        std::vector<std::string>& col = cols[name];
        col.resize(n);
        for (size_t i = 0; i < n; ++i) col[i].assign(r.p + off[i], size_t(off[i + 1] - off[i]));
        r.p += off[n];
    }
    return r.ok;
}
}  // namespace

bool save_binary(const HostGraph& g, const char* path, uint64_t hash) {
    FILE* f = fopen(path, "wb");
    if (!f) { set_error(std::string("save_binary: fopen '") + path + "': " + strerror(errno)); return false; }
    Writer w{f};
    w.raw(kBinMagic, 8);
    w.pod(hash);
    w.pod(g.V);
    w.pod(g.E);
    w.pod(int32_t(g.directed));
    w.raw(g.efrom.data(), size_t(g.E) * 4);
    w.raw(g.eto.data(), size_t(g.E) * 4);
    for (auto* cols : {&g.vnum, &g.enumr}) {
        w.pod(uint32_t(cols->size()));
        for (auto& kv : *cols) { w.str(kv.first); w.raw(kv.second.data(), kv.second.size() * 8); }
    }
    write_strcols(w, g.vstr);
    write_strcols(w, g.estr);
    const bool ok = w.ok && fclose(f) == 0;
    if (!ok) set_error(std::string("save_binary: write to '") + path + "' failed");
    return ok;
}

HostGraph* load_binary(const char* p, size_t n, uint64_t* hash_out, std::string& err) {
    Reader r{p, p + n};
    char magic[8];
    r.raw(magic, 8);
    if (!r.ok || memcmp(magic, kBinMagic, 8) != 0) { err = "not a shdr binary graph"; return nullptr; }
    auto g = std::make_unique<HostGraph>();
    const uint64_t hash = r.pod<uint64_t>();
    g->V = r.pod<int32_t>();
    g->E = r.pod<int64_t>();
    g->directed = r.pod<int32_t>() != 0;
    if (!r.ok || g->V < 0 || g->E < 0 || uint64_t(g->E) * 8 > n) { err = "truncated binary graph"; return nullptr; }
    g->efrom.resize(size_t(g->E));
    g->eto.resize(size_t(g->E));
    r.raw(g->efrom.data(), size_t(g->E) * 4);
    r.raw(g->eto.data(), size_t(g->E) * 4);
    for (int k = 0; k < 2 && r.ok; ++k) {
        auto& cols = k == 0 ? g->vnum : g->enumr;
        const size_t len = k == 0 ? size_t(g->V) : size_t(g->E);
        const uint32_t nc = r.pod<uint32_t>();
        for (uint32_t c = 0; c < nc && r.ok; ++c) {
            std::string name = r.str();
            std::vector<double>& col = cols[name];
            col.resize(len);
            r.raw(col.data(), len * 8);
        }
    }
    if (!r.ok || !read_strcols(r, g->vstr, size_t(g->V)) || !read_strcols(r, g->estr, size_t(g->E))) {
        err = "truncated binary graph";
        return nullptr;
    }
    for (int64_t e = 0; e < g->E; ++e)
        if (g->efrom[e] < 0 || g->efrom[e] >= g->V || g->eto[e] < 0 || g->eto[e] >= g->V) { err = "corrupt binary graph"; return nullptr; }
    if (hash_out) *hash_out = hash;
    return g.release();
}

bool read_file(const char* path, std::string& buf) {
    FILE* f = fopen(path, "rb");
    if (!f) { set_error(std::string("fopen '") + path + "': " + strerror(errno)); return false; }
    buf.clear();
    if (fseek(f, 0, SEEK_END) == 0) {
        const long sz = ftell(f);
        if (sz > 0) buf.resize(size_t(sz));
        rewind(f);
        buf.resize(fread(buf.data(), 1, buf.size(), f));
    }
    char tmp[1 << 16];
    size_t n;
    while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, n);  // non-seekable input
    fclose(f);
    return true;
}

}  // namespace shdr

// ==================================================================== C-ABI
using shdr::HostGraph;
struct shdr_graph { HostGraph g; };

extern "C" {

int shdr_last_error(char* buf, size_t len) {
    if (buf && len) {
        size_t n = std::min(len - 1, shdr::g_last_error.size());
        memcpy(buf, shdr::g_last_error.data(), n);
        buf[n] = 0;
    }
    return int(shdr::g_last_error.size());
}

static shdr_graph* wrap(HostGraph* h) {
    if (!h) return nullptr;
    auto* g = new shdr_graph();
    g->g = std::move(*h);
    delete h;
    return g;
}

shdr_graph* shdr_graph_parse_graphml(const char* text, size_t len) {
    if (!text) { shdr::set_error("parse_graphml: NULL text"); return nullptr; }
    std::string err;
    HostGraph* h = shdr::parse_graphml(text, len, err);
    if (!h) { shdr::set_error("graphml: " + err); return nullptr; }
    return wrap(h);
}

shdr_graph* shdr_graph_load_graphml(const char* path) {
    if (!path) { shdr::set_error("load_graphml: NULL path"); return nullptr; }
    // read eagerly in one piece: Shadow unlinks the file right after topology_new (shd-master.c:210)
    std::string buf;
    if (!shdr::read_file(path, buf)) return nullptr;
    // optional binary cache keyed by the document's content (SHDR_GRAPH_CACHE=<dir>)
    const char* dir = getenv("SHDR_GRAPH_CACHE");
    std::string cpath;
    uint64_t h = 0;
    if (dir && *dir) {
        h = shdr::content_hash(buf.data(), buf.size());
        char name[64];
        snprintf(name, sizeof name, "/%016llx.shdrgraph", (unsigned long long)h);
        cpath = std::string(dir) + name;
        std::string cbuf, err;
        uint64_t ch = 0;
        if (shdr::read_file(cpath.c_str(), cbuf)) {
            HostGraph* hg = shdr::load_binary(cbuf.data(), cbuf.size(), &ch, err);
            if (hg && ch == h) return wrap(hg);
            delete hg;
        }
    }
    shdr_graph* g = shdr_graph_parse_graphml(buf.data(), buf.size());
    if (g && !cpath.empty()) {
        const std::string tmp = cpath + ".tmp" + std::to_string(getpid());
        if (shdr::save_binary(g->g, tmp.c_str(), h)) rename(tmp.c_str(), cpath.c_str());
        else remove(tmp.c_str());
    }
    return g;
}

int shdr_graph_save_binary(const shdr_graph* g, const char* path) {
    if (!g || !path) { shdr::set_error("save_binary: bad arguments"); return SHDR_EINVAL; }
    return shdr::save_binary(g->g, path, 0) ? SHDR_OK : SHDR_EIO;
}

shdr_graph* shdr_graph_load_binary(const char* path) {
    if (!path) { shdr::set_error("load_binary: NULL path"); return nullptr; }
    std::string buf, err;
    if (!shdr::read_file(path, buf)) return nullptr;
    HostGraph* hg = shdr::load_binary(buf.data(), buf.size(), nullptr, err);
    if (!hg) { shdr::set_error("load_binary '" + std::string(path) + "': " + err); return nullptr; }
    return wrap(hg);
}

shdr_graph* shdr_graph_from_edges(int32_t V, int64_t E, int32_t directed, const int32_t* efrom,
                                  const int32_t* eto, const double* elat, const double* eloss,
                                  const double* vloss) {
    if (V < 0 || E < 0 || (E > 0 && (!efrom || !eto || !elat))) { shdr::set_error("from_edges: bad arguments"); return nullptr; }
    auto* h = new HostGraph();
    h->V = V; h->E = E; h->directed = directed != 0;
    h->efrom.assign(efrom, efrom + E);
    h->eto.assign(eto, eto + E);
    for (int64_t e = 0; e < E; ++e)
        if (efrom[e] < 0 || efrom[e] >= V || eto[e] < 0 || eto[e] >= V) { delete h; shdr::set_error("from_edges: endpoint out of range"); return nullptr; }
    h->enumr["latency"].assign(elat, elat + E);
    if (eloss) h->enumr["packetloss"].assign(eloss, eloss + E); else h->enumr["packetloss"].assign(E, 0.0);
    h->enumr["jitter"].assign(E, 0.0);
    if (vloss) h->vnum["packetloss"].assign(vloss, vloss + V); else h->vnum["packetloss"].assign(V, 0.0);
    auto& ids = h->vstr["id"];
    ids.resize(V);
    for (int32_t v = 0; v < V; ++v) ids[v] = "poi-" + std::to_string(v + 1);
    h->vstr["type"].assign(V, "net");
    h->vstr["ip"].assign(V, "0.0.0.0");
    h->vstr["geocode"].assign(V, "US");
    h->vnum["bandwidthup"].assign(V, 10240.0);
    h->vnum["bandwidthdown"].assign(V, 10240.0);
    return wrap(h);
}

shdr_graph* shdr_graph_generate(int32_t kind, int32_t n, int32_t m, uint64_t seed) {
    std::string err;
    HostGraph* h = shdr::generate(kind, n, m, seed, err);
    if (!h) { shdr::set_error(err); return nullptr; }
    return wrap(h);
}

void shdr_graph_free(shdr_graph* g) { delete g; }

int shdr_graph_check(shdr_graph* g, shdr_graph_info* info) {
    if (!g) { shdr::set_error("check: NULL graph"); return SHDR_EINVAL; }
    int rc = g->g.check();
    if (info) *info = g->g.info;
    return rc;
}
int32_t shdr_graph_vertex_count(const shdr_graph* g) { return g ? g->g.V : -1; }
int64_t shdr_graph_edge_count(const shdr_graph* g) { return g ? g->g.E : -1; }
int32_t shdr_graph_is_directed(const shdr_graph* g) { return g ? int32_t(g->g.directed) : -1; }

double shdr_graph_vertex_num(const shdr_graph* g, const char* attr, int32_t v) {
    if (!g || !attr) return std::numeric_limits<double>::quiet_NaN();
    return g->g.vertex_num(attr, v);
}
const char* shdr_graph_vertex_str(const shdr_graph* g, const char* attr, int32_t v) {
    if (!g || !attr) return "";
    return g->g.vertex_str(attr, v).c_str();
}
double shdr_graph_edge_num(const shdr_graph* g, const char* attr, int64_t e) {
    if (!g || !attr) return std::numeric_limits<double>::quiet_NaN();
    return g->g.edge_num(attr, e);
}
int shdr_graph_edge_ends(const shdr_graph* g, int64_t e, int32_t* from, int32_t* to) {
    if (!g || e < 0 || e >= g->g.E) { shdr::set_error("edge_ends: bad edge"); return SHDR_EINVAL; }
    if (from) *from = g->g.efrom[e];
    if (to) *to = g->g.eto[e];
    return SHDR_OK;
}
int shdr_graph_export_edges(const shdr_graph* g, int32_t* efrom, int32_t* eto, double* elat, double* eloss, double* vloss) {
    if (!g) { shdr::set_error("export: NULL graph"); return SHDR_EINVAL; }
    const HostGraph& h = g->g;
    if (efrom) std::copy(h.efrom.begin(), h.efrom.end(), efrom);
    if (eto) std::copy(h.eto.begin(), h.eto.end(), eto);
    for (int64_t e = 0; e < h.E; ++e) {
        if (elat) elat[e] = h.edge_num("latency", e);
        if (eloss) eloss[e] = h.edge_num("packetloss", e);
    }
    if (vloss)
        for (int32_t v = 0; v < h.V; ++v) vloss[v] = h.vertex_num("packetloss", v);
    return SHDR_OK;
}
int64_t shdr_graph_get_eid(const shdr_graph* g, int32_t from, int32_t to) {
    if (!g) return -1;
    return const_cast<shdr_graph*>(g)->g.get_eid(from, to);
}

}  // extern "C"

// internal accessor used by the device engine and the drop-in
namespace shdr {
HostGraph* host_of(shdr_graph* g) { return g ? &g->g : nullptr; }
const HostGraph* host_of(const shdr_graph* g) { return g ? &g->g : nullptr; }
}  // namespace shdr
