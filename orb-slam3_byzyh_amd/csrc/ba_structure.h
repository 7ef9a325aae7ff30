// Host side of the local BA solve: g2o's SparseOptimizer::initializeOptimization +
// BlockSolver::buildStructure (g2o/core/block_solver.hpp:91-240) restated for the device layout.
// Pure C++ (no HIP): compiled into liborbgpu.so by csrc/orb_ba.hip and, for timing on the CPU, by
// tools/ba_struct_bench.cpp.
//
// Hessian indices: the free poses in vertex-id order (a pose without edges gets none, like an
// unconnected vertex), then the landmarks in vertex-id order.  Per call the solve needs:
//   land_off / land_edge    landmark -> its edges (edge order), for Hll / b_l
//   landf_off / landf_edge  landmark -> its free-pose edges (pose row ascending), with the pose row
//                           (landf_row) and the landmark (fland) of each, for Z, b_S and x_l
//   pose_off / pose_fl      free pose -> its free edges in landmark order, each with its landmark:
//                           Hpp / b_p, b_S, and the device's search for the landmarks two poses share
//   blk_off                 the upper-triangle S blocks' product-list offsets (block (i, j) lists at
//                           most min(|i|, |j|) products: a pose sees a landmark once)
// The vectors persist between calls (one BaStructure per handle): no allocation in steady state.
#pragma once

#include <algorithm>
#include <cstdint>
#include <numeric>
#include <vector>

#include "orbgpu.h"

namespace orbgpu_ba {

// a free pose's observation: the landmark and the edge
struct LandEdge {
    int32_t l, e;
};
// one product of a Schur block: Z of edge a times Hpl of edge b
struct EdgePair {
    int32_t a, b;
};

struct BaStructure {
    // [0, world) sharding: this rank's landmarks, [l_begin, l_end) of the landmark order
    int nf = 0, nl_all = 0, nl = 0, ne = 0, nfe = 0, nblk = 0;
    bool dup_edge = false;        // two edges between one free pose and one point
    long long n_products = 0;     // blk_off's total (checked against INT32_MAX by the caller)
    const orb_ba_edge_t* ledges = nullptr;  // this rank's edges (the problem's, in place, for one rank)
    std::vector<int32_t> pdeg, qdeg, order, qorder, all_land, pose_h, free_pose, point_l, land_point, lmap;
    std::vector<orb_ba_edge_t> ledges_copy;
    std::vector<int32_t> land_off, land_edge, landf_off, landf_edge, landf_row, fland, pose_off, blk_off, c1, c2;
    std::vector<int32_t> eland, erow;  // per edge: its landmark, its pose row (-1: fixed pose)
    std::vector<LandEdge> pose_fl;
};

// Validated edge references are the caller's job.  Returns false when there is nothing to optimise
// (no edges, or no free vertex): SparseOptimizer::optimize returns -1 there.
inline bool ba_build_structure(const orb_ba_problem_t* pr, int world, int rank, BaStructure& S) {
    const int np = pr->n_poses, nq = pr->n_points, ne_all = pr->n_edges;
    const orb_ba_edge_t* E = pr->edges;
    S.pdeg.assign(np, 0);
    S.qdeg.assign(nq, 0);
    for (int e = 0; e < ne_all; ++e) {
        S.pdeg[E[e].pose]++;
        S.qdeg[E[e].point]++;
    }
    S.order.resize(np);
    std::iota(S.order.begin(), S.order.end(), 0);
    auto by_pose_id = [&](int a, int b) { return pr->pose_id[a] < pr->pose_id[b]; };
    if (!std::is_sorted(S.order.begin(), S.order.end(), by_pose_id)) std::sort(S.order.begin(), S.order.end(), by_pose_id);
    S.pose_h.assign(np, -1);
    S.free_pose.clear();
    for (int i : S.order)
        if (S.pdeg[i] && !pr->pose_fixed[i]) {
            S.pose_h[i] = (int32_t)S.free_pose.size();
            S.free_pose.push_back(i);
        }
    S.qorder.resize(nq);
    std::iota(S.qorder.begin(), S.qorder.end(), 0);
    auto by_point_id = [&](int a, int b) { return pr->point_id[a] < pr->point_id[b]; };
    if (!std::is_sorted(S.qorder.begin(), S.qorder.end(), by_point_id))
        std::sort(S.qorder.begin(), S.qorder.end(), by_point_id);
    S.all_land.clear();
    for (int i : S.qorder)
        if (S.qdeg[i]) S.all_land.push_back(i);
    S.nf = (int)S.free_pose.size();
    S.nl_all = (int)S.all_land.size();
    if (ne_all == 0 || S.nf + S.nl_all == 0) return false;

    // this rank's landmarks: a contiguous range of the landmark order with about 1/world of the edges
    int l_begin = 0, l_end = S.nl_all;
    if (world > 1) {
        std::vector<long long> cum(S.nl_all + 1, 0);
        for (int l = 0; l < S.nl_all; ++l) cum[l + 1] = cum[l] + S.qdeg[S.all_land[l]];
        auto cut = [&](int r) {
            const long long target = cum[S.nl_all] * r / world;
            return (int)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        };
        l_begin = rank == 0 ? 0 : cut(rank);
        l_end = rank == world - 1 ? S.nl_all : cut(rank + 1);
    }
    S.point_l.assign(nq, -1);
    S.land_point.assign(S.all_land.begin() + l_begin, S.all_land.begin() + l_end);
    for (int l = 0; l < (int)S.land_point.size(); ++l) S.point_l[S.land_point[l]] = l;
    S.lmap.clear();
    S.ledges = E;  // one rank: every edge, in place
    if (world > 1) {
        for (int e = 0; e < ne_all; ++e)
            if (S.point_l[E[e].point] >= 0) S.lmap.push_back(e);
        S.ledges_copy.resize(S.lmap.size());
        for (size_t k = 0; k < S.lmap.size(); ++k) S.ledges_copy[k] = E[S.lmap[k]];
        S.ledges = S.ledges_copy.data();
    }
    const orb_ba_edge_t* L = S.ledges;
    const int ne = world > 1 ? (int)S.lmap.size() : ne_all, nl = (int)S.land_point.size(), nf = S.nf;
    S.ne = ne;
    S.nl = nl;

    // landmark -> all edges (edge order), landmark -> free-pose edges, pose -> free edge count
    S.land_off.assign(nl + 1, 0);
    S.landf_off.assign(nl + 1, 0);
    S.pose_off.assign(nf + 1, 0);
    S.eland.resize(ne);
    S.erow.resize(ne);
    // Edges come grouped by map point (LocalBundleAdjustment adds each point's observations in turn,
    // src/Optimizer.cc:1965-2090), so a landmark's counts accumulate in registers over its run of edges
    // instead of a read-modify-write chain through memory per edge.
    {
        const int32_t *pl = S.point_l.data(), *ph = S.pose_h.data();
        int32_t *el = S.eland.data(), *er = S.erow.data(), *lo = S.land_off.data() + 1, *lf = S.landf_off.data() + 1,
                *po = S.pose_off.data() + 1;
        int cur = -1, n_all = 0, n_free = 0;
        for (int e = 0; e < ne; ++e) {
            const int l = pl[L[e].point], r = ph[L[e].pose];
            el[e] = l;
            er[e] = r;
            if (l != cur) {
                if (cur >= 0) {
                    lo[cur] += n_all;
                    lf[cur] += n_free;
                }
                cur = l;
                n_all = n_free = 0;
            }
            ++n_all;
            if (r >= 0) {
                ++n_free;
                po[r]++;
            }
        }
        if (cur >= 0) {
            lo[cur] += n_all;
            lf[cur] += n_free;
        }
    }
    for (int l = 0; l < nl; ++l) {
        S.land_off[l + 1] += S.land_off[l];
        S.landf_off[l + 1] += S.landf_off[l];
    }
    for (int p = 0; p < nf; ++p) S.pose_off[p + 1] += S.pose_off[p];
    const int nfe = S.landf_off[nl];
    S.nfe = nfe;
    S.land_edge.resize(ne);
    S.landf_edge.resize(nfe);
    S.c1.assign(S.land_off.begin(), S.land_off.end() - 1);
    S.c2.assign(S.landf_off.begin(), S.landf_off.end() - 1);
    {  // the cursors of the current landmark's run in registers, as above
        const int32_t *el = S.eland.data(), *er = S.erow.data();
        int32_t *c1 = S.c1.data(), *c2 = S.c2.data(), *le = S.land_edge.data(), *lfe = S.landf_edge.data();
        int cur = -1, k1 = 0, k2 = 0;
        for (int e = 0; e < ne; ++e) {
            const int l = el[e];
            if (l != cur) {
                if (cur >= 0) {
                    c1[cur] = k1;
                    c2[cur] = k2;
                }
                cur = l;
                k1 = c1[l];
                k2 = c2[l];
            }
            le[k1++] = e;
            if (er[e] >= 0) lfe[k2++] = e;
        }
        if (cur >= 0) {
            c1[cur] = k1;
            c2[cur] = k2;
        }
    }
    // each landmark's free edges by pose row, stable (an insertion sort: a landmark has a handful of
    // edges), with their rows and landmarks; then the pose lists in landmark order
    S.fland.resize(nfe);
    S.landf_row.resize(nfe);
    S.pose_fl.resize(nfe);
    S.c1.assign(S.pose_off.begin(), S.pose_off.end() - 1);
    S.dup_edge = false;
    const int32_t* lfo = S.landf_off.data();
    const int32_t* erw = S.erow.data();
    int32_t* fl = S.fland.data();
    int32_t* pc = S.c1.data();
    LandEdge* pfl = S.pose_fl.data();
    for (int l = 0; l < nl; ++l) {
        const int b0 = lfo[l], d = lfo[l + 1] - b0;
        int32_t* e0 = S.landf_edge.data() + b0;
        int32_t* r0 = S.landf_row.data() + b0;
        for (int k = 0; k < d; ++k) r0[k] = erw[e0[k]];
        for (int a = 1; a < d; ++a) {
            const int32_t v = e0[a], key = r0[a];
            int b = a;
            for (; b > 0 && r0[b - 1] > key; --b) {
                e0[b] = e0[b - 1];
                r0[b] = r0[b - 1];
            }
            e0[b] = v;
            r0[b] = key;
        }
        bool dup = false;
        for (int k = 0; k < d; ++k) {
            fl[b0 + k] = l;
            pfl[pc[r0[k]]++] = LandEdge{l, e0[k]};
            dup |= k && r0[k] == r0[k - 1];
        }
        S.dup_edge |= dup;
    }
    // every upper-triangle block of S, row-major (k_ba_schur_pairs / schur_block_ij)
    S.nblk = nf * (nf + 1) / 2;
    S.blk_off.resize(S.nblk + 1);
    long long acc = 0;
    int b = 0;
    for (int i = 0; i < nf; ++i) {
        const int li = S.pose_off[i + 1] - S.pose_off[i];
        for (int j = i; j < nf; ++j, ++b) {
            S.blk_off[b] = (int32_t)std::min<long long>(acc, INT32_MAX);
            acc += std::min(li, S.pose_off[j + 1] - S.pose_off[j]);
        }
    }
    S.blk_off[S.nblk] = (int32_t)std::min<long long>(acc, INT32_MAX);
    S.n_products = acc;
    return true;
}

}  // namespace orbgpu_ba
