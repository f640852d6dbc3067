// nd_order.cpp -- nested-dissection orderings for the sparse LU (the MUMPS
// stand-in of sparse_lu.cpp; the reference's MUMPS orders with METIS or AMD,
// petsc-options-exact:11-35, petsc-options-inexact:105-106).
//
// method 0 (round 3): George's automatic nested dissection -- the separator is
// the smallest level set of a breadth-first level structure with 30-70 % of
// the vertices on each side.  On locally refined FE meshes its separators are
// long and ragged, and the factors grow accordingly.
//
// method 1 (default, round 4): multilevel bisection, the scheme METIS runs for
// its node orderings, written from its published description:
//   * compression: rows with identical closed adjacency (the components of a
//     P2 vector field at one node) are one vertex of weight = their count;
//   * coarsening by heavy-edge matching (visit order a seeded permutation)
//     down to ~120 vertices;
//   * initial bisection of the coarsest graph by greedy graph growing from
//     several seeds, each refined by FM, the smallest cut kept;
//   * uncoarsening with boundary Fiduccia-Mattheyses refinement of the edge cut
//     under a balance bound;
//   * the vertex separator is a minimum vertex cover of the cut edges
//     (Hopcroft-Karp matching + Koenig's theorem), then improved by node FM:
//     a separator vertex moves to one side and pulls its neighbours on the
//     other side into the separator when that shrinks the separator's weight.
// Independent subgraphs are dissected on host threads; every choice depends
// only on the subgraph (seeded permutations, ties by index), so the ordering
// does not depend on the thread count or timing.
#include "nd_order.hpp"

#include <algorithm>
#include <atomic>
#include <climits>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <numeric>
#include <queue>
#include <thread>

#include "amg_host.hpp"

namespace pls {

void sym_graph(const HostCSR &A, std::vector<int64_t> &gp, std::vector<int32_t> &gi, bool skip_zeros) {
    const int64_t n = A.nrows;
    skip_zeros = skip_zeros && A.v.size() == A.ci.size();
    auto edge = [&](int64_t i, int64_t k) { return A.ci[k] != i && !(skip_zeros && A.v[k] == 0.0); };
    std::vector<int64_t> deg(n + 1, 0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (edge(i, k)) {
                ++deg[i + 1];
                ++deg[A.ci[k] + 1];
            }
    for (int64_t i = 0; i < n; ++i) deg[i + 1] += deg[i];
    std::vector<int32_t> tmp(deg[n]);
    std::vector<int64_t> pos(deg.begin(), deg.end() - 1);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k)
            if (edge(i, k)) {
                tmp[pos[i]++] = A.ci[k];
                tmp[pos[A.ci[k]]++] = (int32_t)i;
            }
    gp.assign(n + 1, 0);
    gi.clear();
    gi.reserve(tmp.size());
    for (int64_t i = 0; i < n; ++i) {
        std::sort(tmp.begin() + deg[i], tmp.begin() + deg[i + 1]);
        int32_t last = -1;
        for (int64_t k = deg[i]; k < deg[i + 1]; ++k)
            if (tmp[k] != last) gi.push_back(last = tmp[k]);
        gp[i + 1] = (int64_t)gi.size();
    }
}

namespace {

// ------------------------------------------------ method 0: level sets ---
struct LevelSetDissector {
    const std::vector<int64_t> &gp;
    const std::vector<int32_t> &gi;
    int64_t leaf;
    std::vector<int32_t> stamp, lev;
    int32_t cur = 0;
    std::vector<int32_t> order;
    LevelSetDissector(const std::vector<int64_t> &p, const std::vector<int32_t> &i, int64_t n, int64_t lf)
        : gp(p), gi(i), leaf(lf), stamp(n, 0), lev(n, -1) {}

    int32_t bfs(int32_t s) {
        order.clear();
        order.push_back(s);
        lev[s] = 0;
        int32_t depth = 0;
        for (size_t h = 0; h < order.size(); ++h) {
            const int32_t u = order[h];
            for (int64_t k = gp[u]; k < gp[u + 1]; ++k) {
                const int32_t v = gi[k];
                if (stamp[v] == cur && lev[v] < 0) {
                    lev[v] = lev[u] + 1;
                    depth = std::max(depth, lev[v]);
                    order.push_back(v);
                }
            }
        }
        return depth;
    }
    void clear_lev(const std::vector<int32_t> &set) {
        for (int32_t v : set) lev[v] = -1;
    }

    void run(NDTree &T, std::vector<int32_t> all) {
        struct Work {
            std::vector<int32_t> set;
            int parent, depth;
        };
        std::vector<Work> stack;
        stack.push_back({std::move(all), -1, 0});
        while (!stack.empty()) {
            Work w = std::move(stack.back());
            stack.pop_back();
            const int node = T.add(w.parent, w.depth);
            if ((int64_t)w.set.size() <= leaf) {
                T.piv[node] = std::move(w.set);
                continue;
            }
            ++cur;
            for (int32_t v : w.set) stamp[v] = cur;
            int32_t s = w.set[0];
            for (int sweep = 0; sweep < 2; ++sweep) {
                bfs(s);
                s = order.back();
                clear_lev(order);
            }
            const int32_t depth = bfs(s);
            if (order.size() < w.set.size()) {
                std::vector<int32_t> comp(order), rest;
                for (int32_t v : w.set)
                    if (lev[v] < 0) rest.push_back(v);
                clear_lev(comp);
                stack.push_back({std::move(rest), node, w.depth + 1});
                stack.push_back({std::move(comp), node, w.depth + 1});
                continue;
            }
            if (depth < 2) {
                clear_lev(order);
                T.piv[node] = std::move(w.set);
                continue;
            }
            std::vector<int64_t> cnt(depth + 1, 0);
            for (int32_t v : order) ++cnt[lev[v]];
            const int64_t m = (int64_t)order.size();
            int64_t below = 0, best = -1, best_sz = INT64_MAX, median = -1;
            for (int32_t l = 0; l <= depth; ++l) {
                const int64_t above = m - below - cnt[l];
                if (l >= 1 && l < depth) {
                    if (median < 0 && below + cnt[l] >= m / 2) median = l;
                    if (below >= 3 * m / 10 && above >= 3 * m / 10 && cnt[l] < best_sz) {
                        best = l;
                        best_sz = cnt[l];
                    }
                }
                below += cnt[l];
            }
            const int32_t L = (int32_t)(best >= 0 ? best : (median >= 0 ? median : 1));
            std::vector<int32_t> a, b, sep;
            for (int32_t v : order) (lev[v] < L ? a : lev[v] > L ? b : sep).push_back(v);
            clear_lev(order);
            T.piv[node] = std::move(sep);
            if (!b.empty()) stack.push_back({std::move(b), node, w.depth + 1});
            if (!a.empty()) stack.push_back({std::move(a), node, w.depth + 1});
        }
    }
};

// ------------------------------------------- method 1: multilevel bisection ---
struct WGraph {
    int32_t n = 0;
    std::vector<int64_t> xadj{0};
    std::vector<int32_t> adj, ew, vw;
    int64_t tw = 0;  // total vertex weight
};

struct Rng {  // xorshift64*: seeded from the subgraph, so results do not depend on threads
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {
        if (!s) s = 1;
    }
    uint64_t next() {
        s ^= s >> 12;
        s ^= s << 25;
        s ^= s >> 27;
        return s * 0x2545F4914F6CDD1Dull;
    }
    int32_t below(int32_t m) { return (int32_t)(next() % (uint64_t)m); }
};

void shuffle(std::vector<int32_t> &v, Rng &r) {
    for (int32_t i = (int32_t)v.size() - 1; i > 0; --i) std::swap(v[i], v[r.below(i + 1)]);
}

// heavy-edge matching -> the coarse graph; cmap: fine vertex -> coarse vertex
WGraph coarsen(const WGraph &g, std::vector<int32_t> &cmap, Rng &rng, int32_t maxvw) {
    const int32_t n = g.n;
    std::vector<int32_t> match(n, -1), perm(n);
    std::iota(perm.begin(), perm.end(), 0);
    shuffle(perm, rng);
    for (int32_t u : perm) {
        if (match[u] >= 0) continue;
        int32_t best = -1, bw = -1;
        for (int64_t e = g.xadj[u]; e < g.xadj[u + 1]; ++e) {
            const int32_t v = g.adj[e];
            if (match[v] < 0 && v != u && g.ew[e] > bw && g.vw[u] + g.vw[v] <= maxvw) {
                best = v;
                bw = g.ew[e];
            }
        }
        if (best >= 0) {
            match[u] = best;
            match[best] = u;
        } else {
            match[u] = u;
        }
    }
    cmap.assign(n, -1);
    int32_t cn = 0;
    for (int32_t u = 0; u < n; ++u)
        if (cmap[u] < 0) {
            cmap[u] = cn;
            cmap[match[u]] = cn;
            ++cn;
        }
    WGraph c;
    c.n = cn;
    c.vw.assign(cn, 0);
    c.xadj.assign(cn + 1, 0);
    c.adj.reserve(g.adj.size() / 2 + 16);
    c.ew.reserve(g.adj.size() / 2 + 16);
    std::vector<int32_t> pos(cn, -1);
    std::vector<int32_t> members;
    int32_t ci = 0;
    for (int32_t u = 0; u < n; ++u) {
        if (cmap[u] != ci) continue;  // first member of coarse vertex ci
        members.clear();
        members.push_back(u);
        if (match[u] != u) members.push_back(match[u]);
        const int64_t start = (int64_t)c.adj.size();
        for (int32_t m : members) {
            c.vw[ci] += g.vw[m];
            for (int64_t e = g.xadj[m]; e < g.xadj[m + 1]; ++e) {
                const int32_t cv = cmap[g.adj[e]];
                if (cv == ci) continue;
                if (pos[cv] < 0) {
                    pos[cv] = (int32_t)(c.adj.size() - start);
                    c.adj.push_back(cv);
                    c.ew.push_back(g.ew[e]);
                } else {
                    c.ew[start + pos[cv]] += g.ew[e];
                }
            }
        }
        for (int64_t e = start; e < (int64_t)c.adj.size(); ++e) pos[c.adj[e]] = -1;
        c.xadj[ci + 1] = (int64_t)c.adj.size();
        ++ci;
    }
    c.tw = g.tw;
    return c;
}

// 2-way edge partition state and FM refinement
struct Bisection {
    std::vector<int8_t> where;
    std::vector<int32_t> id, ed;  // weighted internal / external degree
    int64_t w[2] = {0, 0};
    int64_t cut = 0;

    void compute(const WGraph &g) {
        id.assign(g.n, 0);
        ed.assign(g.n, 0);
        w[0] = w[1] = 0;
        cut = 0;
        for (int32_t u = 0; u < g.n; ++u) {
            w[where[u]] += g.vw[u];
            for (int64_t e = g.xadj[u]; e < g.xadj[u + 1]; ++e)
                (where[g.adj[e]] == where[u] ? id[u] : ed[u]) += g.ew[e];
            cut += ed[u];
        }
        cut /= 2;
    }
};

void fm_refine(const WGraph &g, Bisection &b, int64_t maxw, int passes) {
    const int32_t n = g.n;
    const int limit = (int)std::max<int64_t>(25, std::min<int64_t>(150, n / 100));
    std::vector<int32_t> stamp(n, -1);
    struct Mv {
        int32_t v;
    };
    for (int pass = 0; pass < passes; ++pass) {
        std::priority_queue<std::pair<int64_t, int32_t>> heap[2];
        for (int32_t u = 0; u < n; ++u)
            if (b.ed[u] > 0) heap[b.where[u]].push({(int64_t)b.ed[u] - b.id[u], -u});
        std::vector<int32_t> moves;
        int64_t best_cut = b.cut, best_imb = std::max(b.w[0], b.w[1]);
        size_t best_len = 0;
        const int64_t cut0 = b.cut;
        while (true) {
            // the side to move from: the heavier one, unless it has nothing valid
            int from = b.w[0] >= b.w[1] ? 0 : 1;
            int32_t v = -1;
            for (int attempt = 0; attempt < 2 && v < 0; ++attempt, from ^= 1) {
                auto &h = heap[from];
                while (!h.empty()) {
                    const auto [gain, nv] = h.top();
                    const int32_t u = -nv;
                    if (stamp[u] == pass || b.where[u] != from || gain != (int64_t)b.ed[u] - b.id[u]) {
                        h.pop();
                        continue;
                    }
                    if (b.w[from ^ 1] + g.vw[u] > maxw) break;  // would unbalance: try the other side
                    h.pop();
                    v = u;
                    break;
                }
                if (v >= 0) break;
            }
            if (v < 0) break;
            const int f = b.where[v], t = f ^ 1;
            stamp[v] = pass;
            b.cut -= (int64_t)b.ed[v] - b.id[v];
            std::swap(b.id[v], b.ed[v]);
            b.where[v] = (int8_t)t;
            b.w[f] -= g.vw[v];
            b.w[t] += g.vw[v];
            for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; ++e) {
                const int32_t u = g.adj[e];
                if (b.where[u] == t) {
                    b.id[u] += g.ew[e];
                    b.ed[u] -= g.ew[e];
                } else {
                    b.id[u] -= g.ew[e];
                    b.ed[u] += g.ew[e];
                }
                if (stamp[u] != pass && b.ed[u] > 0) heap[b.where[u]].push({(int64_t)b.ed[u] - b.id[u], -u});
            }
            moves.push_back(v);
            const int64_t imb = std::max(b.w[0], b.w[1]);
            if (b.cut < best_cut || (b.cut == best_cut && imb < best_imb)) {
                best_cut = b.cut;
                best_imb = imb;
                best_len = moves.size();
            }
            if (moves.size() - best_len > (size_t)limit) break;
        }
        // roll back past the best prefix
        for (size_t k = moves.size(); k > best_len; --k) {
            const int32_t v = moves[k - 1];
            const int f = b.where[v], t = f ^ 1;
            b.cut -= (int64_t)b.ed[v] - b.id[v];
            std::swap(b.id[v], b.ed[v]);
            b.where[v] = (int8_t)t;
            b.w[f] -= g.vw[v];
            b.w[t] += g.vw[v];
            for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; ++e) {
                const int32_t u = g.adj[e];
                if (b.where[u] == t) {
                    b.id[u] += g.ew[e];
                    b.ed[u] -= g.ew[e];
                } else {
                    b.id[u] -= g.ew[e];
                    b.ed[u] += g.ew[e];
                }
            }
        }
        if (b.cut >= cut0) break;
    }
}

// greedy graph growing from `seed`: side 0 grows until it holds half the weight
void grow(const WGraph &g, int32_t seed, Bisection &b) {
    b.where.assign(g.n, 1);
    std::vector<int64_t> gain(g.n, 0);
    std::priority_queue<std::pair<int64_t, int32_t>> h;
    int64_t w0 = 0;
    const int64_t target = g.tw / 2;
    h.push({0, -seed});
    std::vector<char> in(g.n, 0);
    while (w0 < target) {
        int32_t v = -1;
        while (!h.empty()) {
            const auto [gn, nv] = h.top();
            h.pop();
            const int32_t u = -nv;
            if (!in[u] && gn == gain[u]) {
                v = u;
                break;
            }
        }
        if (v < 0) {  // disconnected: continue from the first vertex not taken
            for (int32_t u = 0; u < g.n; ++u)
                if (!in[u]) {
                    v = u;
                    break;
                }
            if (v < 0) break;
        }
        in[v] = 1;
        b.where[v] = 0;
        w0 += g.vw[v];
        for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; ++e) {
            const int32_t u = g.adj[e];
            if (in[u]) continue;
            gain[u] += 2 * (int64_t)g.ew[e];
            h.push({gain[u], -u});
        }
    }
}

int32_t pseudo_peripheral(const WGraph &g, int32_t s) {
    std::vector<int32_t> lev(g.n, -1), q;
    for (int sweep = 0; sweep < 2; ++sweep) {
        std::fill(lev.begin(), lev.end(), -1);
        q.assign(1, s);
        lev[s] = 0;
        for (size_t h = 0; h < q.size(); ++h)
            for (int64_t e = g.xadj[q[h]]; e < g.xadj[q[h] + 1]; ++e)
                if (lev[g.adj[e]] < 0) {
                    lev[g.adj[e]] = lev[q[h]] + 1;
                    q.push_back(g.adj[e]);
                }
        s = q.back();
    }
    return s;
}

// multilevel edge bisection of g
Bisection ml_bisect(const WGraph &g, const NDOptions &o, Rng &rng) {
    std::vector<WGraph> gs;
    std::vector<std::vector<int32_t>> cmaps;
    const WGraph *cur = &g;
    const int32_t coarsen_to = 120;
    const int32_t maxvw = (int32_t)std::max<int64_t>(1, (int64_t)(1.5 * (double)g.tw / coarsen_to));
    while (cur->n > coarsen_to) {
        std::vector<int32_t> cm;
        WGraph c = coarsen(*cur, cm, rng, maxvw);
        if (c.n > 0.92 * cur->n) break;
        gs.push_back(std::move(c));
        cmaps.push_back(std::move(cm));
        cur = &gs.back();
    }
    const int64_t maxw = (int64_t)(o.imbalance * (double)g.tw / 2.0) + 1;
    // initial bisections of the coarsest graph
    Bisection best;
    int64_t best_key = INT64_MAX;
    for (int s = 0; s < std::max(1, o.seeds); ++s) {
        const int32_t seed = s == 0 ? pseudo_peripheral(*cur, 0) : rng.below(cur->n);
        Bisection b;
        grow(*cur, seed, b);
        b.compute(*cur);
        fm_refine(*cur, b, std::max<int64_t>(maxw, cur->tw / 2 + 1), 4);
        const int64_t key = b.cut * 4 + (std::max(b.w[0], b.w[1]) > maxw ? (int64_t)1 << 40 : 0);
        if (key < best_key) {
            best_key = key;
            best = std::move(b);
        }
    }
    // uncoarsen
    for (int64_t l = (int64_t)gs.size() - 1; l >= 0; --l) {
        const WGraph &fine = l == 0 ? g : gs[l - 1];
        const std::vector<int32_t> &cm = cmaps[l];
        Bisection b;
        b.where.resize(fine.n);
        for (int32_t u = 0; u < fine.n; ++u) b.where[u] = best.where[cm[u]];
        b.compute(fine);
        fm_refine(fine, b, maxw, 6);
        best = std::move(b);
    }
    if (gs.empty()) {
        best.compute(g);
        fm_refine(g, best, maxw, 6);
    }
    return best;
}

// where: 0 / 1 sides, 2 separator.  Minimum vertex cover of the cut edges.
void cover_separator(const WGraph &g, std::vector<int8_t> &where) {
    const int32_t n = g.n;
    std::vector<int32_t> la, lb, idx(n, -1);  // boundary vertices of side 0 / side 1
    for (int32_t u = 0; u < n; ++u) {
        bool bd = false;
        for (int64_t e = g.xadj[u]; e < g.xadj[u + 1] && !bd; ++e) bd = where[g.adj[e]] != where[u];
        if (!bd) continue;
        if (where[u] == 0) {
            idx[u] = (int32_t)la.size();
            la.push_back(u);
        } else {
            idx[u] = (int32_t)lb.size();
            lb.push_back(u);
        }
    }
    if (la.empty()) return;
    const int32_t na = (int32_t)la.size(), nb = (int32_t)lb.size();
    // Hopcroft-Karp on the bipartite graph of cut edges
    std::vector<int32_t> ma(na, -1), mb(nb, -1), dist(na);
    auto nbrs = [&](int32_t a, auto fn) {
        const int32_t u = la[a];
        for (int64_t e = g.xadj[u]; e < g.xadj[u + 1]; ++e)
            if (where[g.adj[e]] == 1) fn(idx[g.adj[e]]);
    };
    const int32_t INF = INT32_MAX;
    auto bfs = [&]() {
        std::vector<int32_t> q;
        bool found = false;
        for (int32_t a = 0; a < na; ++a) {
            if (ma[a] < 0) {
                dist[a] = 0;
                q.push_back(a);
            } else {
                dist[a] = INF;
            }
        }
        for (size_t h = 0; h < q.size(); ++h) {
            const int32_t a = q[h];
            nbrs(a, [&](int32_t bb) {
                const int32_t a2 = mb[bb];
                if (a2 < 0) {
                    found = true;
                } else if (dist[a2] == INF) {
                    dist[a2] = dist[a] + 1;
                    q.push_back(a2);
                }
            });
        }
        return found;
    };
    // iterative DFS along dist layers (a vertex is entered at most once per phase)
    std::vector<int64_t> it(na);
    std::vector<int32_t> seen(na, -1);
    int32_t phase = 0;
    auto dfs = [&](int32_t root) {
        std::vector<int32_t> stack{root};
        seen[root] = phase;
        it[root] = g.xadj[la[root]];
        while (!stack.empty()) {
            const int32_t a = stack.back();
            const int32_t u = la[a];
            bool advanced = false;
            while (it[a] < g.xadj[u + 1]) {
                const int32_t w = g.adj[it[a]++];
                if (where[w] != 1) continue;
                const int32_t bb = idx[w];
                const int32_t a2 = mb[bb];
                if (a2 < 0) {  // augment along the stack
                    int32_t cb = bb;
                    for (int64_t k = (int64_t)stack.size() - 1; k >= 0; --k) {
                        const int32_t ak = stack[k];
                        const int32_t prev = ma[ak];
                        ma[ak] = cb;
                        mb[cb] = ak;
                        cb = prev;
                    }
                    return true;
                }
                if (seen[a2] != phase && dist[a2] == dist[a] + 1) {
                    seen[a2] = phase;
                    it[a2] = g.xadj[la[a2]];
                    stack.push_back(a2);
                    advanced = true;
                    break;
                }
            }
            if (!advanced) stack.pop_back();
        }
        return false;
    };
    while (bfs()) {
        bool any = false;
        for (int32_t a = 0; a < na; ++a)
            if (ma[a] < 0 && seen[a] != phase) any = dfs(a) || any;
        ++phase;
        if (!any) break;  // (cannot happen when bfs found a free vertex; a guard against looping)
    }
    // Koenig: Z = vertices reachable from unmatched side-0 vertices by alternating paths;
    // cover = (A \ Z) u (B n Z)
    std::vector<char> za(na, 0), zb(nb, 0);
    std::vector<int32_t> q;
    for (int32_t a = 0; a < na; ++a)
        if (ma[a] < 0) {
            za[a] = 1;
            q.push_back(a);
        }
    for (size_t h = 0; h < q.size(); ++h)
        nbrs(q[h], [&](int32_t bb) {
            if (zb[bb]) return;
            zb[bb] = 1;
            const int32_t a2 = mb[bb];
            if (a2 >= 0 && !za[a2]) {
                za[a2] = 1;
                q.push_back(a2);
            }
        });
    for (int32_t a = 0; a < na; ++a)
        if (!za[a]) where[la[a]] = 2;
    for (int32_t bb = 0; bb < nb; ++bb)
        if (zb[bb]) where[lb[bb]] = 2;
}

// node FM: move a separator vertex to side `to`, its neighbours on the other
// side enter the separator; accept the best prefix of each pass
void node_refine(const WGraph &g, std::vector<int8_t> &where, int64_t maxw, int passes) {
    const int32_t n = g.n;
    int64_t w[3] = {0, 0, 0};
    for (int32_t u = 0; u < n; ++u) w[where[u]] += g.vw[u];
    std::vector<int32_t> lock(n, -1);
    const int limit = (int)std::max<int64_t>(20, std::min<int64_t>(200, n / 200));
    auto gain = [&](int32_t v, int to) {
        int64_t s = g.vw[v];
        for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; ++e)
            if (where[g.adj[e]] == (to ^ 1)) s -= g.vw[g.adj[e]];
        return s;
    };
    for (int pass = 0; pass < 2 * passes; ++pass) {
        const int lighter = w[0] <= w[1] ? 0 : 1;
        const int to = (pass & 1) ? lighter ^ 1 : lighter;
        const int other = to ^ 1;
        std::priority_queue<std::pair<int64_t, int32_t>> h;
        for (int32_t u = 0; u < n; ++u)
            if (where[u] == 2) h.push({gain(u, to), -u});
        struct Change {
            int32_t v;
            int8_t old;
        };
        std::vector<Change> log;
        std::vector<size_t> mark{0};
        const int64_t sep0 = w[2];
        int64_t best_sep = w[2];
        size_t best_len = 0, nmoves = 0, best_moves = 0;
        while (!h.empty()) {
            const auto [gn, nv] = h.top();
            h.pop();
            const int32_t v = -nv;
            if (where[v] != 2 || lock[v] == pass || gn != gain(v, to)) continue;
            if (w[to] + g.vw[v] > maxw) continue;
            lock[v] = pass;
            log.push_back({v, 2});
            where[v] = (int8_t)to;
            w[2] -= g.vw[v];
            w[to] += g.vw[v];
            for (int64_t e = g.xadj[v]; e < g.xadj[v + 1]; ++e) {
                const int32_t u = g.adj[e];
                if (where[u] != other) continue;
                log.push_back({u, (int8_t)other});
                where[u] = 2;
                w[other] -= g.vw[u];
                w[2] += g.vw[u];
            }
            // gains of separator vertices next to the changed ones
            for (size_t k = log.size(); k-- > 0 && log[k].v != v;) {
                const int32_t u = log[k].v;
                h.push({gain(u, to), -u});
                for (int64_t e = g.xadj[u]; e < g.xadj[u + 1]; ++e)
                    if (where[g.adj[e]] == 2 && lock[g.adj[e]] != pass) h.push({gain(g.adj[e], to), -g.adj[e]});
            }
            ++nmoves;
            if (w[2] < best_sep) {
                best_sep = w[2];
                best_len = log.size();
                best_moves = nmoves;
            }
            if (nmoves - best_moves > (size_t)limit) break;
        }
        for (size_t k = log.size(); k > best_len; --k) {
            const Change &c = log[k - 1];
            w[where[c.v]] -= g.vw[c.v];
            where[c.v] = c.old;
            w[c.old] += g.vw[c.v];
        }
        if (w[2] >= sep0 && (pass & 1)) break;
    }
}

WGraph induced(const WGraph &g, const std::vector<int32_t> &verts, std::vector<int32_t> &loc) {
    WGraph s;
    s.n = (int32_t)verts.size();
    s.vw.resize(s.n);
    s.xadj.assign(s.n + 1, 0);
    for (int32_t i = 0; i < s.n; ++i) loc[verts[i]] = i;
    for (int32_t i = 0; i < s.n; ++i) {
        const int32_t u = verts[i];
        s.vw[i] = g.vw[u];
        s.tw += g.vw[u];
        for (int64_t e = g.xadj[u]; e < g.xadj[u + 1]; ++e) {
            const int32_t l = loc[g.adj[e]];
            if (l >= 0) {
                s.adj.push_back(l);
                s.ew.push_back(g.ew[e]);
            }
        }
        s.xadj[i + 1] = (int64_t)s.adj.size();
    }
    for (int32_t u : verts) loc[u] = -1;
    return s;
}

struct MLDissector {
    const NDOptions &o;
    std::vector<std::vector<int32_t>> members;  // compressed vertex -> original rows
    NDTree &T;
    std::mutex mu;
    MLDissector(const NDOptions &opt, NDTree &t) : o(opt), T(t) {}

    struct Task {
        WGraph g;
        std::vector<int32_t> ids;  // subgraph vertex -> compressed vertex
        int node;
    };

    std::vector<int32_t> rows_of(const std::vector<int32_t> &ids) {
        std::vector<int32_t> r;
        for (int32_t c : ids) r.insert(r.end(), members[c].begin(), members[c].end());
        return r;
    }

    // one task: a leaf, or a separator and two child tasks (A first, then B)
    void process(Task &t, std::vector<Task> &out, std::vector<int32_t> &loc) {
        const WGraph &g = t.g;
        if (g.tw <= o.leaf || g.n <= 2) {
            std::vector<int32_t> r = rows_of(t.ids);
            std::lock_guard<std::mutex> lk(mu);
            T.piv[t.node] = std::move(r);
            return;
        }
        Rng rng((uint64_t)g.n * 1000003ull + (uint64_t)g.tw * 7919ull + (uint64_t)t.ids[0]);
        Bisection b = ml_bisect(g, o, rng);
        std::vector<int8_t> where = b.where;
        cover_separator(g, where);
        const int64_t maxw = (int64_t)(o.imbalance * (double)g.tw / 2.0) + 1;
        if (o.node_passes > 0) node_refine(g, where, maxw, o.node_passes);
        std::vector<int32_t> va, vb, vs;
        for (int32_t u = 0; u < g.n; ++u) (where[u] == 0 ? va : where[u] == 1 ? vb : vs).push_back(u);
        if (va.empty() || vb.empty()) {  // no split found: the set is one front
            std::vector<int32_t> r = rows_of(t.ids);
            std::lock_guard<std::mutex> lk(mu);
            T.piv[t.node] = std::move(r);
            return;
        }
        std::vector<int32_t> sep_ids;
        for (int32_t u : vs) sep_ids.push_back(t.ids[u]);
        std::vector<int32_t> sep_rows = rows_of(sep_ids);
        int na, nb;
        {
            std::lock_guard<std::mutex> lk(mu);
            T.piv[t.node] = std::move(sep_rows);
            const int d = T.depth[t.node] + 1;
            na = T.add(t.node, d);
            nb = T.add(t.node, d);
        }
        for (int side = 0; side < 2; ++side) {
            const std::vector<int32_t> &vv = side == 0 ? va : vb;
            Task c;
            c.g = induced(g, vv, loc);
            c.ids.resize(vv.size());
            for (size_t k = 0; k < vv.size(); ++k) c.ids[k] = t.ids[vv[k]];
            c.node = side == 0 ? na : nb;
            out.push_back(std::move(c));
        }
    }

    void run(Task root, int threads) {
        std::deque<Task> q;
        q.push_back(std::move(root));
        std::mutex qm;
        std::condition_variable cv;
        int busy = 0;
        auto worker = [&]() {
            std::vector<int32_t> loc;
            while (true) {
                Task t;
                {
                    std::unique_lock<std::mutex> lk(qm);
                    cv.wait(lk, [&] { return !q.empty() || busy == 0; });
                    if (q.empty()) return;
                    t = std::move(q.front());
                    q.pop_front();
                    ++busy;
                }
                if ((int32_t)loc.size() < t.g.n) loc.assign(t.g.n, -1);
                std::vector<Task> out;
                process(t, out, loc);
                {
                    std::lock_guard<std::mutex> lk(qm);
                    for (auto &c : out) q.push_back(std::move(c));
                    --busy;
                }
                cv.notify_all();
            }
        };
        std::vector<std::thread> th;
        for (int i = 0; i < std::max(1, threads); ++i) th.emplace_back(worker);
        for (auto &x : th) x.join();
    }
};

}  // namespace

NDTree nested_dissection(const std::vector<int64_t> &gp, const std::vector<int32_t> &gi, int64_t n,
                         const NDOptions &o) {
    NDTree T;
    if (n == 0) {
        T.add(-1, 0);
        return T;
    }
    if (o.method == 0) {
        LevelSetDissector D(gp, gi, n, std::max<int64_t>(1, o.leaf));
        std::vector<int32_t> all(n);
        std::iota(all.begin(), all.end(), 0);
        D.run(T, std::move(all));
        return T;
    }
    MLDissector D(o, T);
    // compression: identical closed adjacency (sorted lists; hash, then compare)
    std::vector<int32_t> comp(n, -1);
    int32_t nc = 0;
    if (o.compress) {
        std::vector<std::pair<uint64_t, int32_t>> key(n);
        for (int64_t i = 0; i < n; ++i) {
            uint64_t h = 1469598103934665603ull;
            bool self = false;
            for (int64_t k = gp[i]; k <= gp[i + 1]; ++k) {
                int32_t v;
                if (k == gp[i + 1]) {
                    if (self) break;
                    v = (int32_t)i;
                } else {
                    v = gi[k];
                    if (!self && v > i) {  // the closed list in ascending order: i goes before v
                        h = (h ^ (uint64_t)i) * 1099511628211ull;
                        self = true;
                    }
                }
                h = (h ^ (uint64_t)v) * 1099511628211ull;
            }
            key[i] = {h, (int32_t)i};
        }
        std::sort(key.begin(), key.end());
        auto same = [&](int32_t a, int32_t b) {  // closed adjacencies equal
            if (gp[a + 1] - gp[a] != gp[b + 1] - gp[b]) return false;
            // N[a] u {a} == N[b] u {b}: b in N[a], a in N[b], the rest equal
            int64_t ka = gp[a], kb = gp[b];
            while (ka < gp[a + 1] || kb < gp[b + 1]) {
                int32_t va = ka < gp[a + 1] ? gi[ka] : INT32_MAX, vb = kb < gp[b + 1] ? gi[kb] : INT32_MAX;
                if (va == b) {
                    ++ka;
                    continue;
                }
                if (vb == a) {
                    ++kb;
                    continue;
                }
                if (va != vb) return false;
                ++ka;
                ++kb;
            }
            return true;
        };
        for (size_t s = 0; s < key.size();) {
            size_t e = s + 1;
            while (e < key.size() && key[e].first == key[s].first) ++e;
            for (size_t a = s; a < e; ++a) {
                const int32_t ia = key[a].second;
                if (comp[ia] >= 0) continue;
                comp[ia] = nc;
                for (size_t b2 = a + 1; b2 < e; ++b2) {
                    const int32_t ib = key[b2].second;
                    if (comp[ib] < 0 && same(ia, ib)) comp[ib] = nc;
                }
                ++nc;
            }
            s = e;
        }
    } else {
        for (int64_t i = 0; i < n; ++i) comp[i] = (int32_t)i;
        nc = (int32_t)n;
    }
    // compressed vertices numbered by their first row (deterministic)
    std::vector<int32_t> first(nc, INT32_MAX);
    for (int64_t i = 0; i < n; ++i) first[comp[i]] = std::min(first[comp[i]], (int32_t)i);
    std::vector<int32_t> byfirst(nc);
    std::iota(byfirst.begin(), byfirst.end(), 0);
    std::sort(byfirst.begin(), byfirst.end(), [&](int32_t a, int32_t b) { return first[a] < first[b]; });
    std::vector<int32_t> renum(nc);
    for (int32_t k = 0; k < nc; ++k) renum[byfirst[k]] = k;
    D.members.assign(nc, {});
    for (int64_t i = 0; i < n; ++i) D.members[renum[comp[i]]].push_back((int32_t)i);
    MLDissector::Task root;
    WGraph &g = root.g;
    g.n = nc;
    g.vw.resize(nc);
    g.xadj.assign(nc + 1, 0);
    {
        std::vector<int32_t> pos(nc, -1);
        for (int32_t c = 0; c < nc; ++c) {
            const int64_t start = (int64_t)g.adj.size();
            g.vw[c] = (int32_t)D.members[c].size();
            g.tw += g.vw[c];
            const int32_t r = D.members[c][0];
            for (int64_t k = gp[r]; k < gp[r + 1]; ++k) {
                const int32_t cv = renum[comp[gi[k]]];
                if (cv == c) continue;
                if (pos[cv] < 0) {
                    pos[cv] = (int32_t)(g.adj.size() - start);
                    g.adj.push_back(cv);
                    g.ew.push_back(1);
                }
            }
            for (int64_t e = start; e < (int64_t)g.adj.size(); ++e) pos[g.adj[e]] = -1;
            g.xadj[c + 1] = (int64_t)g.adj.size();
        }
        // edge weight = product of the endpoints' row counts (edges of the uncompressed graph)
        for (int32_t c = 0; c < nc; ++c)
            for (int64_t e = g.xadj[c]; e < g.xadj[c + 1]; ++e) g.ew[e] = g.vw[c] * g.vw[g.adj[e]];
    }
    root.ids.resize(nc);
    std::iota(root.ids.begin(), root.ids.end(), 0);
    root.node = T.add(-1, 0);
    D.run(std::move(root), o.threads > 0 ? o.threads : amgh::setup_threads());
    return T;
}

}  // namespace pls
