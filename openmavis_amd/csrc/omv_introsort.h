// Replica of libstdc++'s std::sort (introsort: median-of-3 quicksort with depth limit 2*lg(n),
// heapsort fallback, final insertion sort with _S_threshold = 16).
//
// Why: ORBextractor::DistributeOctTree sorts (node size, node*) pairs with compareNodes
// (src/ORBextractor.cc:482-494, :629-632), which orders by (size, UL.x) and leaves nodes equal in
// both unordered.  Which of two such nodes is expanded first changes the output, so the device must
// reproduce the exact element moves of the algorithm the reference links against (libstdc++),
// not merely "a" sort.  tests/test_introsort.py checks this replica against std::sort.
//
// Elements are (key1, key2, payload) triples; less(a, b) = (a.k1, a.k2) < (b.k1, b.k2).
#pragma once
#ifdef __HIPCC__
#define OMV_HD __host__ __device__
#else
#define OMV_HD
#endif

namespace omv {

struct SortItem {
    int k1, k2, payload;
};

OMV_HD inline bool item_less(const SortItem &a, const SortItem &b) {
    if (a.k1 < b.k1) return true;
    if (a.k1 > b.k1) return false;
    return a.k2 < b.k2;
}

OMV_HD inline void item_swap(SortItem *a, SortItem *b) {
    SortItem t = *a;
    *a = *b;
    *b = t;
}

OMV_HD inline int floor_log2(int n) {
    int r = 0;
    while (n > 1) n >>= 1, ++r;
    return r;
}

// std::__push_heap
OMV_HD inline void heap_push(SortItem *f, int hole, int top, SortItem v) {
    int parent = (hole - 1) / 2;
    while (hole > top && item_less(f[parent], v)) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = v;
}

// std::__adjust_heap
OMV_HD inline void heap_adjust(SortItem *f, int hole, int len, SortItem v) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (item_less(f[child], f[child - 1])) child--;
        f[hole] = f[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        f[hole] = f[child - 1];
        hole = child - 1;
    }
    heap_push(f, hole, top, v);
}

// std::__partial_sort(first, last, last) == make_heap + sort_heap
OMV_HD inline void heap_sort(SortItem *f, int len) {
    if (len >= 2) {
        for (int parent = (len - 2) / 2;; --parent) {
            heap_adjust(f, parent, len, f[parent]);
            if (parent == 0) break;
        }
    }
    for (int last = len; last > 1;) {
        --last;
        SortItem v = f[last];
        f[last] = f[0];
        heap_adjust(f, 0, last, v);
    }
}

// std::__move_median_to_first
OMV_HD inline void median_to_first(SortItem *res, SortItem *a, SortItem *b, SortItem *c) {
    if (item_less(*a, *b)) {
        if (item_less(*b, *c)) item_swap(res, b);
        else if (item_less(*a, *c)) item_swap(res, c);
        else item_swap(res, a);
    } else if (item_less(*a, *c)) item_swap(res, a);
    else if (item_less(*b, *c)) item_swap(res, c);
    else item_swap(res, b);
}

// std::__unguarded_partition
OMV_HD inline int unguarded_partition(SortItem *arr, int first, int last, int pivot) {
    for (;;) {
        while (item_less(arr[first], arr[pivot])) ++first;
        --last;
        while (item_less(arr[pivot], arr[last])) --last;
        if (!(first < last)) return first;
        item_swap(&arr[first], &arr[last]);
        ++first;
    }
}

// std::__unguarded_linear_insert
OMV_HD inline void unguarded_linear_insert(SortItem *arr, int last) {
    SortItem v = arr[last];
    int next = last - 1;
    while (item_less(v, arr[next])) {
        arr[last] = arr[next];
        last = next;
        --next;
    }
    arr[last] = v;
}

// std::__insertion_sort on [first, last)
OMV_HD inline void insertion_sort(SortItem *arr, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        if (item_less(arr[i], arr[first])) {
            SortItem v = arr[i];
            for (int k = i; k > first; --k) arr[k] = arr[k - 1];
            arr[first] = v;
        } else {
            unguarded_linear_insert(arr, i);
        }
    }
}

// std::sort(arr, arr + n, item_less).  `stack` needs 3*(2*lg(n)+2) ints of scratch (192 always suffice).
OMV_HD inline void libstdcxx_sort(SortItem *arr, int n, int *stack) {
    const int kThreshold = 16;
    if (n <= 1) return;
    // __introsort_loop, made iterative: the reference recursion is on [cut, last) with depth-1,
    // then loops on [first, cut) with the same (already decremented) depth.  The recursion is
    // fully evaluated before the loop continues, so an explicit stack of pending left ranges
    // (processed after the right one completes) reproduces the exact sequence of moves.
    int sp = 0;
    int first = 0, last = n, depth = 2 * floor_log2(n);
    for (;;) {
        while (last - first > kThreshold) {
            if (depth == 0) {
                heap_sort(arr + first, last - first);
                last = first;   // this range is done
                break;
            }
            --depth;
            const int mid = first + (last - first) / 2;
            median_to_first(&arr[first], &arr[first + 1], &arr[mid], &arr[last - 1]);
            const int cut = unguarded_partition(arr, first + 1, last, first);
            // recurse on [cut, last) with `depth`; afterwards continue with [first, cut), `depth`
            stack[sp++] = first;
            stack[sp++] = cut;
            stack[sp++] = depth;
            first = cut;
        }
        if (sp == 0) break;
        depth = stack[--sp];
        last = stack[--sp];
        first = stack[--sp];
    }
    // __final_insertion_sort
    if (n > kThreshold) {
        insertion_sort(arr, 0, kThreshold);
        for (int i = kThreshold; i < n; ++i) unguarded_linear_insert(arr, i);
    } else {
        insertion_sort(arr, 0, n);
    }
}

}  // namespace omv
