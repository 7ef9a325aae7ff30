// Host/device helpers shared by the HIP kernels and their host-side unit tests.
// Everything here is compiled with -ffp-contract=off on both sides so float results are identical.
#pragma once
#include <stdint.h>

#ifndef ORB_HD
#if defined(__HIPCC__)
#define ORB_HD __host__ __device__
#else
#define ORB_HD
#endif
#endif

// cv::fastAtan2 (OpenCV 4.x atan_f32, baseline build without FMA), degrees in [0, 360).
// Called by IC_Angle, reference src/ORBextractor.cc:137.
ORB_HD static inline float orb_fast_atan2(float y, float x) {
    const float k = (float)(180 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float eps = (float)2.220446049250313080847e-16;  // (float)DBL_EPSILON
    const float ax = x < 0 ? -x : x, ay = y < 0 ? -y : y;
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ---------------------------------------------------------------------------------------------
// Exact port of libstdc++ (GCC 11) std::sort -- __introsort_loop (threshold 16, median-of-3 pivot
// moved to first, unguarded partition, heap-sort fallback at depth 2*lg(n)) followed by
// __final_insertion_sort -- over an array of 16-bit node ids with a caller-supplied "less".
// DistributeOctTree sorts (count, node) pairs with compareNodes (reference src/ORBextractor.cc:
// 676-697, 950), which has ties (equal count and equal UL.x); the resulting order, and hence the
// selected keypoints, depends on this exact algorithm.  Run by ONE lane.
// ---------------------------------------------------------------------------------------------
template <class T, class Less>
ORB_HD static inline void orb_unguarded_linear_insert(T* a, int last, Less less) {
    const T val = a[last];
    int next = last - 1;
    while (less(val, a[next])) { a[last] = a[next]; last = next; --next; }
    a[last] = val;
}

template <class T, class Less>
ORB_HD static inline void orb_insertion_sort(T* a, int first, int last, Less less) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        if (less(a[i], a[first])) {
            const T val = a[i];
            for (int k = i; k > first; --k) a[k] = a[k - 1];
            a[first] = val;
        } else {
            orb_unguarded_linear_insert(a, i, less);
        }
    }
}

template <class T, class Less>
ORB_HD static inline void orb_push_heap(T* a, int first, int hole, int top, T val, Less less) {
    int parent = (hole - 1) / 2;
    while (hole > top && less(a[first + parent], val)) {
        a[first + hole] = a[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[first + hole] = val;
}

template <class T, class Less>
ORB_HD static inline void orb_adjust_heap(T* a, int first, int hole, int len, T val, Less less) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (less(a[first + child], a[first + child - 1])) child--;
        a[first + hole] = a[first + child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        a[first + hole] = a[first + child - 1];
        hole = child - 1;
    }
    orb_push_heap(a, first, hole, top, val, less);
}

template <class T, class Less>
ORB_HD static inline void orb_heap_sort(T* a, int first, int last, Less less) {
    const int len = last - first;
    if (len >= 2) {  // __make_heap
        int parent = (len - 2) / 2;
        while (true) {
            orb_adjust_heap(a, first, parent, len, a[first + parent], less);
            if (parent == 0) break;
            parent--;
        }
    }
    // __heap_select over [first, last, last) adds nothing; then __sort_heap
    while (last - first > 1) {
        --last;
        const T val = a[last];
        a[last] = a[first];
        orb_adjust_heap(a, first, 0, last - first, val, less);
    }
}

template <class T, class Less>
ORB_HD static inline void orb_move_median_to_first(T* a, int result, int x, int y, int z, Less less) {
    int pick;
    if (less(a[x], a[y])) {
        if (less(a[y], a[z])) pick = y;
        else if (less(a[x], a[z])) pick = z;
        else pick = x;
    } else if (less(a[x], a[z])) pick = x;
    else if (less(a[y], a[z])) pick = z;
    else pick = y;
    const T t = a[result]; a[result] = a[pick]; a[pick] = t;
}

template <class T, class Less>
ORB_HD static inline int orb_unguarded_partition(T* a, int first, int last, int pivot, Less less) {
    while (true) {
        while (less(a[first], a[pivot])) ++first;
        --last;
        while (less(a[pivot], a[last])) --last;
        if (!(first < last)) return first;
        const T t = a[first]; a[first] = a[last]; a[last] = t;
        ++first;
    }
}

// `ws` = workspace of kOrbSortStack * 3 ints for the explicit introsort stack (LDS on the device)
constexpr int kOrbSortStack = 40;  // one pending right part per partition level; depth <= 2*lg(n) <= 32

template <class T, class Less>
ORB_HD static inline void orb_std_sort(T* a, int n, Less less, int* ws) {
    if (n <= 1) return;
    int lg = 0;
    for (int m = n; m > 1; m >>= 1) ++lg;
    // __introsort_loop with an explicit stack (the recursion is on the right part, loop on the left)
    struct Range { int first, last, depth; };
    Range* stack = reinterpret_cast<Range*>(ws);
    int sp = 0;
    stack[sp++] = {0, n, 2 * lg};
    while (sp > 0) {
        Range r = stack[--sp];
        int first = r.first, last = r.last, depth = r.depth;
        while (last - first > 16) {
            if (depth == 0) { orb_heap_sort(a, first, last, less); break; }
            --depth;
            const int mid = first + (last - first) / 2;
            orb_move_median_to_first(a, first, first + 1, mid, last - 1, less);
            const int cut = orb_unguarded_partition(a, first + 1, last, first, less);
            // libstdc++ recurses into [cut, last) before continuing with [first, cut).  The two
            // ranges are disjoint, so processing order does not change the result; push the right
            // part and keep looping on the left part.
            stack[sp++] = {cut, last, depth};
            last = cut;
        }
    }
    // __final_insertion_sort
    if (n > 16) {
        orb_insertion_sort(a, 0, 16, less);
        for (int i = 16; i < n; ++i) orb_unguarded_linear_insert(a, i, less);
    } else {
        orb_insertion_sort(a, 0, n, less);
    }
}

template <class T, class Less>
ORB_HD static inline void orb_std_sort(T* a, int n, Less less) {
    int ws[kOrbSortStack * 3];
    orb_std_sort(a, n, less, ws);
}
