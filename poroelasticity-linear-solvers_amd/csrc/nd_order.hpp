// nd_order.hpp -- fill-reducing nested-dissection orderings of a symmetric
// sparsity graph (host), the assembly tree of the sparse LU (sparse_lu.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace pls {

struct HostCSR;

// the dissection tree: a node's pivots are its separator (or leaf) vertices;
// children in a fixed order (the postorder the LU numbers pivots in)
struct NDTree {
    std::vector<std::vector<int32_t>> piv;  // per node: its vertices
    std::vector<std::vector<int32_t>> ch;   // children (tree order)
    std::vector<int32_t> parent, depth;
    int add(int par, int d) {
        piv.emplace_back();
        ch.emplace_back();
        parent.push_back(par);
        depth.push_back(d);
        if (par >= 0) ch[par].push_back((int)piv.size() - 1);
        return (int)piv.size() - 1;
    }
};

struct NDOptions {
    int64_t leaf = 64;         // a set of at most this many rows is a leaf front
    int method = 1;            // 0: George's level-set separators, 1: multilevel bisection
    double imbalance = 1.10;   // multilevel: heavier side <= imbalance x half the weight
    int seeds = 6;             // multilevel: initial bisections tried on the coarsest graph
    bool compress = true;      // multilevel: rows with identical closed adjacency are one vertex
    int node_passes = 4;       // multilevel: separator (node) FM passes after the vertex cover
    int threads = 0;           // host threads for independent subgraphs (0: setup_threads())
};

// symmetrized adjacency of M's pattern without the diagonal (sorted rows);
// skip_zeros: entries stored with value 0 are not edges (PETSc's MatMatMult
// keeps structural zeros, e.g. in the Schur block selfp -- they add fill
// without adding anything to the factors)
void sym_graph(const HostCSR &A, std::vector<int64_t> &gp, std::vector<int32_t> &gi, bool skip_zeros = false);

// nested dissection of the graph (gp, gi) on n vertices
NDTree nested_dissection(const std::vector<int64_t> &gp, const std::vector<int32_t> &gi, int64_t n,
                         const NDOptions &o);

}  // namespace pls
