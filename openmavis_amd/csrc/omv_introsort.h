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


#ifdef __HIPCC__
// ---- the same sort, data-parallel on the device ----------------------------------------------------
// wave_introsort_loop: __introsort_loop by one wavefront (all 64 lanes, uniform control flow).  The
// sequential __unguarded_partition(first + 1, last, pivot = first) is computed from the original values:
// with LS = ascending positions in [first+1, last) whose item is not < pivot ("left stoppers") and
// RS = descending positions in [first, last) whose item is not > pivot (the pivot itself included), the
// k-th iteration swaps LS[k-1] <-> RS[k-1] while LS[k-1] < RS[k-1]; at the first K with LS[K-1] >= RS[K-1]
// the scan returns min(LS[K-1], RS[K-2]) (a missing LS entry or K = 1 drops that term).  Before the
// crossing neither scan reaches a swapped position, so every stopper is an original one.  The median
// and the (rare) heapsort fallback run on lane 0.
// block_final_insertion_sort: __final_insertion_sort is a stable insertion sort of the whole range, i.e.
// item i goes to rank #{j : (k1, k2, j) < (k1_i, k2_i, i)}; every thread of the block ranks its items.
__device__ __forceinline__ void sort_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LS / RS: scratch of the range's own positions (entries f .. l-1), so disjoint ranges partition concurrently.
__device__ inline int wave_unguarded_partition(SortItem *arr, int f, int l, int *LS, int *RS, int lane) {
    const SortItem p = arr[f];
    const unsigned long long lt = (1ull << lane) - 1ull;
    int nL = 0, nR = 0;
    LS += f, RS += f;
    for (int base = f + 1; base < l; base += 64) {
        const int x = base + lane;
        const bool fl = x < l && !item_less(arr[x], p);
        const unsigned long long m = __ballot(fl);
        if (fl) LS[nL + __popcll(m & lt)] = x;
        nL += __popcll(m);
    }
    for (int base = l - 1; base >= f; base -= 64) {
        const int y = base - lane;
        const bool fl = y >= f && !item_less(p, arr[y]);
        const unsigned long long m = __ballot(fl);
        if (fl) RS[nR + __popcll(m & lt)] = y;
        nR += __popcll(m);
    }
    sort_wave_sync();
    int K = 0;   // crossing iteration, 1-based
    for (int k0 = 0;; k0 += 64) {
        const int k = k0 + lane;
        const int lsv = k < nL ? LS[k] : 0x7fffffff;
        const int rsv = k < nR ? RS[k] : -0x7fffffff;
        const unsigned long long m = __ballot(lsv >= rsv);
        if (m) {
            K = k0 + __ffsll((long long)m);
            break;
        }
    }
    const int cut = min(K - 1 < nL ? LS[K - 1] : 0x7fffffff, K >= 2 ? RS[K - 2] : 0x7fffffff);
    for (int q = lane; q < K - 1; q += 64) {   // disjoint positions: LS[q] < RS[q], both monotone
        const int i = LS[q], j = RS[q];
        const SortItem u = arr[i], v = arr[j];
        arr[i] = v;
        arr[j] = u;
    }
    sort_wave_sync();
    return cut;
}

// `stack`: 3*(2*lg(n)+2) ints; LS, RS: n ints each (LDS).
__device__ inline void wave_introsort_loop(SortItem *arr, int n, int *stack, int *LS, int *RS, int lane) {
    const int kThreshold = 16;
    if (n <= 1) return;
    int sp = 0;
    int first = 0, last = n, depth = 2 * floor_log2(n);
    for (;;) {
        while (last - first > kThreshold) {
            if (depth == 0) {
                if (lane == 0) heap_sort(arr + first, last - first);
                sort_wave_sync();
                last = first;
                break;
            }
            --depth;
            const int mid = first + (last - first) / 2;
            if (lane == 0) median_to_first(&arr[first], &arr[first + 1], &arr[mid], &arr[last - 1]);
            sort_wave_sync();
            const int cut = wave_unguarded_partition(arr, first, last, LS, RS, lane);
            stack[sp] = first, stack[sp + 1] = cut, stack[sp + 2] = depth;   // every lane stores the same value
            sp += 3;
            first = cut;
        }
        if (sp == 0) break;
        sort_wave_sync();
        sp -= 3;
        first = stack[sp], last = stack[sp + 1], depth = stack[sp + 2];
    }
}

// __introsort_loop by all wavefronts of the block: the loop only ever splits a range into two disjoint ranges that it
// then treats independently (each with the depth limit of the split), so the ranges of one recursion depth are
// partitioned concurrently, one range per wavefront, level by level -- the same element moves as the sequential
// loop.  q: 2 * (3 * (n / 17 + 1)) + 2 ints of scratch (two range queues + their counts); LS, RS: n ints each.
__device__ inline int introsort_queue_ints(int n) { return 6 * (n / 17 + 1) + 2; }
__device__ inline void block_introsort_loop(SortItem *arr, int n, int *q, int *LS, int *RS, int tid, int T) {
    const int kThreshold = 16, cap = n / 17 + 1;
    int *cnt = q, *qa = q + 2, *qb = qa + 3 * cap;
    const int lane = tid & 63, wave = tid >> 6, nw = T >> 6;
    if (tid == 0) {
        cnt[0] = n > kThreshold ? 1 : 0, cnt[1] = 0;
        qa[0] = 0, qa[1] = n, qa[2] = 2 * floor_log2(max(n, 1));
    }
    __syncthreads();
    for (int side = 0;; side ^= 1) {
        int *cur = side ? qb : qa, *nxt = side ? qa : qb;
        const int nq = cnt[side];
        if (nq == 0) break;
        for (int r = wave; r < nq; r += nw) {
            const int f = cur[3 * r], l = cur[3 * r + 1];
            int depth = cur[3 * r + 2];
            if (depth == 0) {
                if (lane == 0) heap_sort(arr + f, l - f);
                sort_wave_sync();
                continue;
            }
            --depth;
            const int mid = f + (l - f) / 2;
            if (lane == 0) median_to_first(&arr[f], &arr[f + 1], &arr[mid], &arr[l - 1]);
            sort_wave_sync();
            const int cut = wave_unguarded_partition(arr, f, l, LS, RS, lane);
            if (lane == 0) {
                if (l - cut > kThreshold) {
                    const int k = atomicAdd(&cnt[side ^ 1], 1);
                    nxt[3 * k] = cut, nxt[3 * k + 1] = l, nxt[3 * k + 2] = depth;
                }
                if (cut - f > kThreshold) {
                    const int k = atomicAdd(&cnt[side ^ 1], 1);
                    nxt[3 * k] = f, nxt[3 * k + 1] = cut, nxt[3 * k + 2] = depth;
                }
            }
        }
        __syncthreads();
        if (tid == 0) cnt[side] = 0;
        __syncthreads();
    }
}

// All threads of the block; tmp: n items of scratch.  Requires k1 >= 0, 0 <= k2 < 2^20, n <= 4096.
__device__ inline void block_final_insertion_sort(SortItem *arr, int n, SortItem *tmp, int tid, int T) {
    auto key = [](const SortItem &a, int i) {
        return ((unsigned long long)(unsigned)a.k1 << 32) | ((unsigned long long)(unsigned)a.k2 << 12) | (unsigned)i;
    };
    for (int i = tid; i < n; i += T) {
        const unsigned long long c = key(arr[i], i);
        int r = 0;
        for (int j = 0; j < n; ++j) r += key(arr[j], j) < c ? 1 : 0;
        tmp[r] = arr[i];
    }
    __syncthreads();
    for (int i = tid; i < n; i += T) arr[i] = tmp[i];
    __syncthreads();
}
#endif

}  // namespace omv
