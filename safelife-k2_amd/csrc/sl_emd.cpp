// sl_emd.cpp -- host-side earth mover's distance for the episode-end side-effect
// score.
//
// Replaces the third-party call the reference makes at
// /root/reference/safelife/side_effects.py:56, pyemd.emd (pyemd==0.5.1,
// requirements.txt:1; absent from this image), which wraps Pele & Werman's FastEMD
// "emd_hat_gd_metric" for double histograms.  That published algorithm is restated
// here:
//   1. pre-flow: mass present in both histograms at the same bin moves at cost 0
//      (the ground distance is zero on the diagonal);
//   2. fixed-point conversion: masses scaled by 1e6 / max(sum P, sum Q) -- the sums
//      of the histograms as given, before the pre-flow (emd_hat_impl<double> sums
//      POrig / QOrig) -- costs by 1e6 / max(C), both rounded to the nearest integer
//      (floor(x + 0.5));
//   3. the heavier histogram supplies; its excess drains to a threshold node at cost
//      0; the exact integer minimum-cost transport (C is used as given, supply bin
//      first, without transposing when the histograms swap roles);
//   4. the integer optimum scaled back, plus |sum P - sum Q| * extra_mass_penalty
//      (-1: max(C)).
//
// The transport problem is solved exactly by a transportation simplex: a
// north-west-corner spanning tree, block-search pricing over the implicit dense
// cost matrix (costs come from a per-offset table: the reference's ground distance
// depends only on the signed (dy, dx) between two cells), and the classic
// epsilon-perturbation of the supplies (scaled by K = n + 1, +1 per source, +n on
// the last sink) so that no basic flow is ever zero: every pivot strictly lowers the
// cost and the method cannot cycle.  The basis the perturbed problem ends in is
// optimal for the original one; the original flows are recomputed on that tree.
//
// Parity unpinned: no pyemd output exists in this environment to compare with.
// Checked against an exact LP of the same fixed-point problem
// (tests/test_side_effects_cpu.py).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/safelife_hip.h"

namespace {

struct Transport {
    // rows: supply bins; columns: demand bins (+ the threshold node, cost 0)
    int n = 0, m = 0;
    std::vector<int64_t> supply, demand;
    std::vector<int32_t> sy, sx, dy, dx;      // cell coordinates of the bins
    const int64_t *table = nullptr;           // [2H-1][2W-1] fixed-point costs
    int tw = 0, H = 0, W = 0;
    bool threshold = false;                   // last column is the threshold node

    int64_t cost(int i, int j) const {
        if (threshold && j == m - 1) return 0;
        return table[(int64_t)(sy[i] - dy[j] + H - 1) * tw + (sx[i] - dx[j] + W - 1)];
    }
};

struct Basis {
    std::vector<int> r, c;                    // basic cells
    std::vector<int64_t> x;                   // their flows
    std::vector<std::vector<int>> adj;        // node -> incident basic cells
};

// north-west corner rule on (perturbed, hence nondegenerate) supplies and demands:
// n + m - 1 basic cells forming a spanning tree
void northwest(const std::vector<int64_t> &s, const std::vector<int64_t> &d, int n, int m,
               Basis &B) {
    std::vector<int64_t> rs(s), rd(d);
    int i = 0, j = 0;
    while (i < n && j < m) {
        const int64_t f = std::min(rs[i], rd[j]);
        B.r.push_back(i);
        B.c.push_back(j);
        B.x.push_back(f);
        rs[i] -= f;
        rd[j] -= f;
        if (rs[i] == 0 && i < n - 1) i++;
        else j++;
    }
    B.adj.assign(n + m, {});
    for (int k = 0; k < (int)B.r.size(); k++) {
        B.adj[B.r[k]].push_back(k);
        B.adj[n + B.c[k]].push_back(k);
    }
}

// potentials (u_i + v_j = cost on basic cells) and the tree rooted at row 0, in
// breadth-first order
void tree_walk(const Transport &T, const Basis &B, std::vector<int64_t> &pot,
               std::vector<int> &par_cell, std::vector<int> &depth, std::vector<int> &order) {
    std::fill(par_cell.begin(), par_cell.end(), -1);
    std::fill(depth.begin(), depth.end(), -1);
    order.clear();
    order.push_back(0);
    depth[0] = 0;
    pot[0] = 0;
    for (size_t q = 0; q < order.size(); q++) {
        const int u = order[q];
        for (int k : B.adj[u]) {
            const int w = u < T.n ? T.n + B.c[k] : B.r[k];
            if (depth[w] >= 0) continue;
            depth[w] = depth[u] + 1;
            par_cell[w] = k;
            pot[w] = T.cost(B.r[k], B.c[k]) - pot[u];    // row: u_i, column: v_j
            order.push_back(w);
        }
    }
}

// flows of the basis tree for the given supplies / demands (leaf elimination)
void tree_flows(const Transport &T, Basis &B, const std::vector<int64_t> &s,
                const std::vector<int64_t> &d, const std::vector<int> &par_cell,
                const std::vector<int> &order) {
    const int n = T.n;
    std::vector<int64_t> bal(n + T.m);
    for (int i = 0; i < n; i++) bal[i] = s[i];
    for (int j = 0; j < T.m; j++) bal[n + j] = -d[j];
    for (int q = (int)order.size() - 1; q > 0; q--) {    // children before parents
        const int w = order[q], k = par_cell[w];
        const int parent = w < n ? n + B.c[k] : B.r[k];
        // a row sends its net supply to its column parent; a column draws its net
        // demand from its row parent
        B.x[k] = w < n ? bal[w] : -bal[w];
        bal[parent] += bal[w];
        bal[w] = 0;
    }
}

int64_t solve(Transport &T) {
    const int n = T.n, m = T.m, N = n + m;
    const int64_t K = n + 1;
    std::vector<int64_t> ps(n), pd(m);
    for (int i = 0; i < n; i++) ps[i] = K * T.supply[i] + 1;
    for (int j = 0; j < m; j++) pd[j] = K * T.demand[j];
    pd[m - 1] += n;
    Basis B;
    northwest(ps, pd, n, m, B);
    if ((int)B.r.size() != N - 1) return -1;
    std::vector<int64_t> pot(N);
    std::vector<int> par_cell(N), depth(N), order, cyc;
    order.reserve(N);
    const int64_t total = (int64_t)n * m;
    const int64_t block = std::max<int64_t>(64, (int64_t)std::sqrt((double)total));
    int64_t next = 0;                         // pricing resumes where it stopped
    std::vector<int> path_a, path_b;
    for (;;) {
        tree_walk(T, B, pot, par_cell, depth, order);
        // block search: the most negative reduced cost of the first block holding one
        int bi = -1, bj = -1;
        int64_t best = 0, scanned = 0;
        while (scanned < total) {
            const int64_t end = std::min(scanned + block, total);
            for (int64_t q = scanned; q < end; q++) {
                int64_t e = next + q;
                if (e >= total) e -= total;
                const int i = (int)(e / m), j = (int)(e - (int64_t)i * m);
                const int64_t rc = T.cost(i, j) - pot[i] - pot[n + j];
                if (rc < best) {
                    best = rc;
                    bi = i;
                    bj = j;
                }
            }
            scanned = end;
            if (bi >= 0) break;
        }
        if (bi < 0) break;                    // no negative reduced cost: optimal
        next = (next + scanned) % total;
        // the cycle: the tree paths from row bi and column bj up to their common
        // ancestor
        path_a.clear();
        path_b.clear();
        int a = bi, b = n + bj;
        auto up = [&](int &v, std::vector<int> &path) {
            const int k = par_cell[v];
            path.push_back(k);
            v = v < n ? n + B.c[k] : B.r[k];
        };
        while (depth[a] > depth[b]) up(a, path_a);
        while (depth[b] > depth[a]) up(b, path_b);
        while (a != b) {
            up(a, path_a);
            up(b, path_b);
        }
        // from the entering cell's column round to its row: path_b, then path_a
        // reversed; the 1st, 3rd, ... cells lose flow, the others gain it
        cyc.assign(path_b.begin(), path_b.end());
        for (int q = (int)path_a.size() - 1; q >= 0; q--) cyc.push_back(path_a[q]);
        int leave = -1;
        int64_t theta = 0;
        for (size_t q = 0; q < cyc.size(); q += 2)
            if (leave < 0 || B.x[cyc[q]] < theta) {
                theta = B.x[cyc[q]];
                leave = cyc[q];
            }
        for (size_t q = 0; q < cyc.size(); q++) B.x[cyc[q]] += (q & 1) ? theta : -theta;
        // the entering cell takes the leaving cell's slot
        auto drop = [&](int node, int k) {
            auto &v = B.adj[node];
            v.erase(std::find(v.begin(), v.end(), k));
        };
        drop(B.r[leave], leave);
        drop(n + B.c[leave], leave);
        B.r[leave] = bi;
        B.c[leave] = bj;
        B.x[leave] = theta;
        B.adj[bi].push_back(leave);
        B.adj[n + bj].push_back(leave);
    }
    // the optimal tree with the unperturbed supplies and demands
    tree_walk(T, B, pot, par_cell, depth, order);
    tree_flows(T, B, T.supply, T.demand, par_cell, order);
    int64_t cost = 0;
    for (size_t k = 0; k < B.r.size(); k++) {
        if (B.x[k] < 0) return -1;            // cannot happen (see the header)
        cost += B.x[k] * T.cost(B.r[k], B.c[k]);
    }
    return cost;
}

}  // namespace

extern "C" int sl_emd_cells(const double *p, const double *q, const int32_t *ys,
                            const int32_t *xs, int64_t n_cells, const double *cost_table,
                            int H, int W, double extra_mass_penalty, double *out) {
    if (!out || n_cells < 0 || H < 1 || W < 1 ||
        (n_cells > 0 && (!p || !q || !ys || !xs || !cost_table)))
        return SL_EINVAL;
    *out = 0.0;
    if (n_cells == 0) return SL_OK;
    const int tw = 2 * W - 1;
    for (int64_t i = 0; i < n_cells; i++)
        if (ys[i] < 0 || ys[i] >= H || xs[i] < 0 || xs[i] >= W) return SL_EINVAL;
    // 0. mass scale from the histograms as given (FastEMD's emd_hat_impl<double> sums
    //    POrig / QOrig, the caller's histograms, not the pre-flowed ones)
    double sumP = 0.0, sumQ = 0.0;
    for (int64_t i = 0; i < n_cells; i++) {
        sumP += p[i];
        sumQ += q[i];
    }
    // 1. pre-flow at equal bins (emd_hat_gd_metric: metric ground distance)
    std::vector<double> P(p, p + n_cells), Q(q, q + n_cells);
    for (int64_t i = 0; i < n_cells; i++) {
        if (P[i] < Q[i]) {
            Q[i] -= P[i];
            P[i] = 0.0;
        } else {
            P[i] -= Q[i];
            Q[i] = 0.0;
        }
    }
    // 2. fixed point: masses by 1e6 / max original sum, costs by 1e6 / max C over all
    //    pairs; the supply side is chosen on the pre-flowed integer sums (below)
    double maxC = 0.0;
    {
        std::vector<uint8_t> seen((size_t)(2 * H - 1) * tw, 0);   // offsets present
        for (int64_t i = 0; i < n_cells; i++)
            for (int64_t j = 0; j < n_cells; j++) {
                const size_t o = (size_t)(ys[i] - ys[j] + H - 1) * tw + (xs[i] - xs[j] + W - 1);
                if (!seen[o]) {
                    seen[o] = 1;
                    maxC = std::max(maxC, cost_table[o]);
                }
            }
    }
    const double MULT = 1000000.0;
    const double minSum = std::min(sumP, sumQ), maxSum = std::max(sumP, sumQ);
    if (extra_mass_penalty == -1.0) extra_mass_penalty = maxC;
    double dist = 0.0;
    if (maxSum > 0.0 && maxC > 0.0) {
        const double PQnorm = MULT / maxSum, Cnorm = MULT / maxC;
        std::vector<int64_t> itab((size_t)(2 * H - 1) * tw);
        for (size_t o = 0; o < itab.size(); o++)
            itab[o] = (int64_t)std::floor(cost_table[o] * Cnorm + 0.5);
        std::vector<int64_t> iP(n_cells), iQ(n_cells);
        int64_t sP = 0, sQ = 0;
        for (int64_t i = 0; i < n_cells; i++) {
            iP[i] = (int64_t)std::floor(P[i] * PQnorm + 0.5);
            iQ[i] = (int64_t)std::floor(Q[i] * PQnorm + 0.5);
            sP += iP[i];
            sQ += iQ[i];
        }
        // 3. the heavier side supplies (C as given, supply bin first)
        const bool swap = sQ > sP;
        const std::vector<int64_t> &S = swap ? iQ : iP, &D = swap ? iP : iQ;
        Transport T;
        T.table = itab.data();
        T.tw = tw;
        T.H = H;
        T.W = W;
        for (int64_t i = 0; i < n_cells; i++) {
            if (S[i] > 0) {
                T.supply.push_back(S[i]);
                T.sy.push_back(ys[i]);
                T.sx.push_back(xs[i]);
            }
            if (D[i] > 0) {
                T.demand.push_back(D[i]);
                T.dy.push_back(ys[i]);
                T.dx.push_back(xs[i]);
            }
        }
        const int64_t excess = sP > sQ ? sP - sQ : sQ - sP;
        if (excess > 0) {                     // the threshold node absorbs it at cost 0
            T.demand.push_back(excess);
            T.dy.push_back(0);
            T.dx.push_back(0);
            T.threshold = true;
        }
        T.n = (int)T.supply.size();
        T.m = (int)T.demand.size();
        if (T.n > 0 && T.m > 0) {
            const int64_t c = solve(T);
            if (c < 0) return SL_EHIP;
            // 4. back to the caller's units
            dist = (double)c;
            dist = dist / PQnorm;
            dist = dist / Cnorm;
        }
    }
    dist += (maxSum - minSum) * extra_mass_penalty;
    *out = dist;
    return SL_OK;
}
