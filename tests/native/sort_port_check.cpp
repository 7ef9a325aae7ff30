// Host build of the device-side libstdc++ introsort port (orb-slam3_byzyh_amd/csrc/orb_hd.h):
// for random, tie-heavy (count, UL.x) node arrays, the port must produce exactly the order
// std::sort produces with the reference's compareNodes (src/ORBextractor.cc:676-697, 950).
// Prints "OK <cases>" or the first mismatch.
#include <algorithm>
#include <cstdio>
#include <random>
#include <utility>
#include <vector>

#include "../../orb-slam3_byzyh_amd/csrc/orb_hd.h"

struct Node { int ulx; };

static bool compareNodes(std::pair<int, Node*>& e1, std::pair<int, Node*>& e2) {
    if (e1.first < e2.first) return true;
    if (e1.first > e2.first) return false;
    return e1.second->ulx < e2.second->ulx;
}

// The wave-parallel emulation used on the GPU (k_quadtree, qt_sort): libstdc++'s unguarded Hoare
// partition of [first+1, last) around a[first] expressed through two "stop lists":
//   A = ascending positions with !(a[i] < p), B = descending positions with !(p < a[i]);
//   pairs (A_k, B_k) are swapped while A_k < B_k; with K* the first k where A_k >= B_k (A past its end
//   = +inf, B past its end = -inf) the cut is min(A_K*, B_{K*-1}) (B_{-1} = +inf).
// Checked against orb_unguarded_partition, which test 1 checks against std::sort itself.
template <class T, class Less>
static int stoplist_partition(T* a, int first, int last, Less less) {
    const T p = a[first];
    std::vector<int> A, B;
    for (int i = first + 1; i < last; ++i) if (!less(a[i], p)) A.push_back(i);
    for (int i = last - 1; i > first; --i) if (!less(p, a[i])) B.push_back(i);
    const int lim = (int)std::min(A.size(), B.size());
    int ks = lim;
    for (int k = 0; k < lim; ++k) if (A[k] >= B[k]) { ks = k; break; }
    const long inf = 1L << 40;
    const long ak = ks < (int)A.size() ? A[ks] : inf;
    const long bprev = ks > 0 ? B[ks - 1] : inf;
    for (int k = 0; k < ks; ++k) std::swap(a[A[k]], a[B[k]]);
    return (int)std::min(ak, bprev);
}

int main() {
    std::mt19937 rng(12345);
    {
        int cases = 0;
        for (int n : {17, 18, 19, 33, 40, 100, 500, 1200}) {  // partitions only run on ranges > 16
            for (int rep = 0; rep < 400; ++rep, ++cases) {
                std::vector<int> v(n), w;
                const int kv = 1 + (int)(rng() % (rep % 4 == 0 ? 2 : 20));
                for (int i = 0; i < n; ++i) v[i] = (int)(rng() % kv) * 16 + i % 16;  // payload in low bits
                auto less = [](int x, int y) { return (x >> 4) < (y >> 4); };
                const int mid = n / 2;
                orb_move_median_to_first(v.data(), 0, 1, mid, n - 1, less);
                w = v;
                const int c1 = orb_unguarded_partition(v.data(), 1, n, 0, less);
                const int c2 = stoplist_partition(w.data(), 0, n, less);
                if (c1 != c2 || v != w) { printf("STOPLIST MISMATCH n=%d rep=%d cut %d vs %d\n", n, rep, c1, c2); return 1; }
            }
        }
        printf("stoplist ok %d\n", cases);
    }
    int cases = 0;
    for (int n : {0, 1, 2, 5, 15, 16, 17, 18, 31, 33, 64, 100, 257, 600, 1500, 4000}) {
        for (int rep = 0; rep < 60; ++rep, ++cases) {
            const int kc = 1 + (int)(rng() % (rep % 3 == 0 ? 3 : 12));  // few distinct counts = many ties
            const int kx = 1 + (int)(rng() % (rep % 2 ? 4 : 40));
            std::vector<Node> nodes(n);
            std::vector<int> cnt(n);
            for (int i = 0; i < n; ++i) { nodes[i].ulx = (int)(rng() % kx) * 37; cnt[i] = 2 + (int)(rng() % kc); }
            std::vector<std::pair<int, Node*>> ref;
            for (int i = 0; i < n; ++i) ref.push_back({cnt[i], &nodes[i]});
            std::sort(ref.begin(), ref.end(), compareNodes);
            std::vector<uint16_t> ids(n);
            for (int i = 0; i < n; ++i) ids[i] = (uint16_t)i;
            orb_std_sort(ids.data(), n, [&](uint16_t a, uint16_t b) {
                return cnt[a] < cnt[b] || (cnt[a] == cnt[b] && nodes[a].ulx < nodes[b].ulx);
            });
            for (int i = 0; i < n; ++i)
                if (&nodes[ids[i]] != ref[i].second) {
                    printf("MISMATCH n=%d rep=%d at %d\n", n, rep, i);
                    return 1;
                }
        }
    }
    // adversarial: already sorted / reversed / all equal (exercises median-of-3 and heap fallback)
    for (int mode = 0; mode < 3; ++mode) {
        const int n = 3000;
        std::vector<Node> nodes(n);
        std::vector<int> cnt(n);
        for (int i = 0; i < n; ++i) {
            nodes[i].ulx = mode == 2 ? 0 : (mode == 0 ? i : n - i);
            cnt[i] = 2;
        }
        std::vector<std::pair<int, Node*>> ref;
        for (int i = 0; i < n; ++i) ref.push_back({cnt[i], &nodes[i]});
        std::sort(ref.begin(), ref.end(), compareNodes);
        std::vector<uint16_t> ids(n);
        for (int i = 0; i < n; ++i) ids[i] = (uint16_t)i;
        orb_std_sort(ids.data(), n, [&](uint16_t a, uint16_t b) {
            return cnt[a] < cnt[b] || (cnt[a] == cnt[b] && nodes[a].ulx < nodes[b].ulx);
        });
        for (int i = 0; i < n; ++i)
            if (&nodes[ids[i]] != ref[i].second) { printf("MISMATCH mode=%d at %d\n", mode, i); return 1; }
        ++cases;
    }
    // the depth-limit fallback is std::partial_sort(first, last, last) in libstdc++: check the port
    for (int n : {2, 3, 17, 100, 999}) {
        for (int rep = 0; rep < 20; ++rep, ++cases) {
            std::vector<Node> nodes(n);
            std::vector<int> cnt(n);
            for (int i = 0; i < n; ++i) { nodes[i].ulx = (int)(rng() % 5); cnt[i] = 2 + (int)(rng() % 3); }
            std::vector<std::pair<int, Node*>> ref;
            for (int i = 0; i < n; ++i) ref.push_back({cnt[i], &nodes[i]});
            std::partial_sort(ref.begin(), ref.end(), ref.end(), compareNodes);
            std::vector<uint16_t> ids(n);
            for (int i = 0; i < n; ++i) ids[i] = (uint16_t)i;
            orb_heap_sort(ids.data(), 0, n, [&](uint16_t a, uint16_t b) {
                return cnt[a] < cnt[b] || (cnt[a] == cnt[b] && nodes[a].ulx < nodes[b].ulx);
            });
            for (int i = 0; i < n; ++i)
                if (&nodes[ids[i]] != ref[i].second) { printf("HEAP MISMATCH n=%d at %d\n", n, i); return 1; }
        }
    }
    printf("OK %d\n", cases);
    return 0;
}
