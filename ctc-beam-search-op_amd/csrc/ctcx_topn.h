// ctcx_topn.h — exact, sequential device restatement of the bounded top-N the
// reference uses for its beam (gtl::TopN<BeamEntry*, BeamComparer>, used at
// ctc_ext_beam_search_decoder.h:59, 84-85, 142, 151-155, 192-199, 245-252).
//
// Why it exists: when two beam totals are exactly equal, WHICH entry is the
// bottom (evicted) and the order in which branches are visited next frame
// depend on the heap layout produced by libstdc++'s make_heap / pop_heap /
// sort_heap / introsort.  The fast GPU path (ctcx_decode.hip exact_step)
// replays that heap layout itself, wave-parallel; this literal model, run by
// one lane over LDS arrays, serves the frames the fast path does not model
// (non-finite totals, the beam filling up mid-frame, an entry held twice), the
// unsorted-layout TopN(n) of TopPaths, and std::sort for a frame whose beam
// never overflowed.  Elements are slot ids; the comparator reads each slot's CURRENT
// total (the reference compares through BeamEntry pointers, so an entry
// modified while inside the heap is seen with its new value — e.g. the
// evicted bottom whose total is reset to -inf before the push).
//
// The heap/sort routines follow libstdc++ (bits/stl_heap.h, bits/stl_algo.h,
// unchanged GCC 4.x-13): __adjust_heap, __push_heap, __make_heap, __pop_heap,
// __sort_heap, __introsort_loop (median-of-3 pivot, unguarded partition,
// depth limit 2*floor(log2 n), threshold 16), __final_insertion_sort.
#pragma once

#include <stdint.h>

#include "ctcx_kernels.h"

namespace ctcx {

template <typename T>
struct SlotGreater {
  const CTCX_LDS T* tot;
  __host__ __device__ __forceinline__ bool operator()(int a, int b) const { return tot[a] > tot[b]; }
};

template <class Cmp>
__host__ __device__ void lit_push_heap(CTCX_LDS int* e, int hole, int top, int value, const Cmp& gt) {
  int parent = (hole - 1) / 2;
  while (hole > top && gt(e[parent], value)) {
    e[hole] = e[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  e[hole] = value;
}

template <class Cmp>
__host__ __device__ void lit_adjust_heap(CTCX_LDS int* e, int hole, int len, int value, const Cmp& gt) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (gt(e[second], e[second - 1])) second--;
    e[hole] = e[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    e[hole] = e[second - 1];
    hole = second - 1;
  }
  lit_push_heap(e, hole, top, value, gt);
}

template <class Cmp>
__host__ __device__ void lit_make_heap(CTCX_LDS int* e, int len, const Cmp& gt) {
  if (len < 2) return;
  for (int parent = (len - 2) / 2;; --parent) {
    lit_adjust_heap(e, parent, len, e[parent], gt);
    if (parent == 0) return;
  }
}

// std::pop_heap(e, e + len): the front moves to e[len-1].
template <class Cmp>
__host__ __device__ void lit_pop_heap(CTCX_LDS int* e, int len, const Cmp& gt) {
  if (len > 1) {
    const int value = e[len - 1];
    e[len - 1] = e[0];
    lit_adjust_heap(e, 0, len - 1, value, gt);
  }
}

template <class Cmp>
__host__ __device__ void lit_sort_heap(CTCX_LDS int* e, int len, const Cmp& gt) {
  while (len > 1) {
    lit_pop_heap(e, len, gt);
    --len;
  }
}

template <class Cmp>
__host__ __device__ void lit_insertion_sort(CTCX_LDS int* e, int first, int last, const Cmp& gt) {
  if (first == last) return;
  for (int i = first + 1; i != last; ++i) {
    const int v = e[i];
    if (gt(v, e[first])) {
      for (int k = i; k > first; --k) e[k] = e[k - 1];
      e[first] = v;
    } else {
      int k = i;
      while (gt(v, e[k - 1])) { e[k] = e[k - 1]; --k; }
      e[k] = v;
    }
  }
}

template <class Cmp>
__host__ __device__ void lit_unguarded_insertion_sort(CTCX_LDS int* e, int first, int last, const Cmp& gt) {
  for (int i = first; i != last; ++i) {
    const int v = e[i];
    int k = i;
    while (gt(v, e[k - 1])) { e[k] = e[k - 1]; --k; }
    e[k] = v;
  }
}

template <class Cmp>
__host__ __device__ void lit_move_median_to_first(CTCX_LDS int* e, int result, int a, int b, int c, const Cmp& gt) {
  int pick;
  if (gt(e[a], e[b])) {
    if (gt(e[b], e[c])) pick = b;
    else if (gt(e[a], e[c])) pick = c;
    else pick = a;
  } else if (gt(e[a], e[c])) pick = a;
  else if (gt(e[b], e[c])) pick = c;
  else pick = b;
  const int tmp = e[result]; e[result] = e[pick]; e[pick] = tmp;
}

template <class Cmp>
__host__ __device__ int lit_unguarded_partition(CTCX_LDS int* e, int first, int last, int pivot, const Cmp& gt) {
  while (true) {
    while (gt(e[first], e[pivot])) ++first;
    --last;
    while (gt(e[pivot], e[last])) --last;
    if (!(first < last)) return first;
    const int tmp = e[first]; e[first] = e[last]; e[last] = tmp;
    ++first;
  }
}

// std::sort(e + 0, e + n, gt) — libstdc++ introsort, made iterative.  The
// sub-ranges it sorts are disjoint, so the order in which they are finished
// does not change the result.
template <class Cmp>
__host__ __device__ void lit_sort(CTCX_LDS int* e, int n, const Cmp& gt) {
  if (n <= 1) return;
  int lg = 31 - __builtin_clz((unsigned)n);
  struct Frame { int first, last, depth; };
  Frame stack[64];
  int sp = 0;
  stack[sp++] = Frame{0, n, 2 * lg};
  while (sp > 0) {
    Frame f = stack[--sp];
    int first = f.first, last = f.last, depth = f.depth;
    while (last - first > 16) {
      if (depth == 0) {
        // std::__partial_sort(first, last, last): heap_select + sort_heap
        lit_make_heap(e + first, last - first, gt);
        lit_sort_heap(e + first, last - first, gt);
        break;
      }
      --depth;
      const int mid = first + (last - first) / 2;
      lit_move_median_to_first(e, first, first + 1, mid, last - 1, gt);
      const int cut = lit_unguarded_partition(e, first + 1, last, first, gt);
      stack[sp++] = Frame{cut, last, depth};
      last = cut;
    }
  }
  if (n > 16) {
    lit_insertion_sort(e, 0, 16, gt);
    lit_unguarded_insertion_sort(e, 16, n, gt);
  } else {
    lit_insertion_sort(e, 0, n, gt);
  }
}

// gtl::TopN state over an LDS array of capacity limit+1.
enum { kTopUnordered = 0, kTopBottomKnown = 1, kTopHeap = 2 };

struct LitTop {
  CTCX_LDS int* e;   // capacity limit + 1
  int n;       // elements_.size()
  int limit;
  int state;
  __host__ __device__ int size() const { return n < limit ? n : limit; }
};

template <class Cmp>
__host__ __device__ void lit_top_push(LitTop& h, int v, const Cmp& gt) {
  if (h.limit == 0) return;
  if (h.state != kTopHeap) {
    h.e[h.n++] = v;
    if (h.state != kTopUnordered && !gt(h.e[h.n - 1], h.e[0])) {
      const int tmp = h.e[0]; h.e[0] = h.e[h.n - 1]; h.e[h.n - 1] = tmp;
    }
    if (h.n == h.limit + 1) {
      lit_make_heap(h.e, h.n, gt);
      lit_pop_heap(h.e, h.n, gt);
      h.state = kTopHeap;
    }
  } else if (gt(v, h.e[0])) {
    h.e[h.n - 1] = v;
    lit_pop_heap(h.e, h.n, gt);
  }
}

template <class Cmp>
__host__ __device__ int lit_top_peek_bottom(LitTop& h, const Cmp& gt) {
  if (h.state == kTopUnordered) {
    int m = 0;
    for (int i = 1; i < h.n; ++i)
      if (gt(h.e[m], h.e[i])) m = i;
    if (m != 0) { const int tmp = h.e[0]; h.e[0] = h.e[m]; h.e[m] = tmp; }
    h.state = kTopBottomKnown;
  }
  return h.e[0];
}

// Destructive; leaves the sorted (descending) elements in e[0..return).
template <class Cmp>
__host__ __device__ int lit_top_extract(LitTop& h, const Cmp& gt) {
  int n = h.n;
  if (h.state != kTopHeap) {
    lit_sort(h.e, n, gt);
  } else {
    n -= 1;
    lit_sort_heap(h.e, n, gt);
  }
  return n;
}

}  // namespace ctcx
