// Prefix-on-demand std::sort.  The search loop sorts every candidate change
// of an iteration (processor.cc:840-843, std::sort on the float key) but
// consumes only a prefix.  std::sort is not stable, so the exact order of
// equal keys — which decides the break point — is that of libstdc++'s
// introsort: median-of-three pivot to the front, unguarded Hoare partition,
// recurse right / loop left with depth limit 2*floor(log2 n) falling back to
// heap sort, then one final insertion sort over the whole range
// (bits/stl_algo.h __introsort_loop / __final_insertion_sort).
//
// Partitioning only permutes inside a range, so ranges can be refined in any
// order; and because every element left of a partition cut is <= the pivot
// <= every element right of it, the final insertion sort never moves an
// element across a leaf range — it equals a stable insertion sort of each
// leaf.  Refining leftmost-first and finishing leaves as they are reached
// therefore yields exactly std::sort's permutation, one prefix at a time.
//
// Large ranges are partitioned on the host pool (ParallelPartition): the
// unguarded Hoare partition is a function of two position lists -- the
// left scan's stops L (keys >= pivot, ascending) and the right scan's R
// (keys <= pivot, descending) -- so counting, listing, a binary search for
// the crossing and the swaps all run in parallel and give the same
// permutation and cut as the sequential loop.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "host/thread_pool.h"

namespace gz {

class LazyStdSort {
 public:
  using Elem = std::pair<int, float>;

  LazyStdSort(Elem* a, size_t n) : a_(a) {
    if (n > 1) {
      int lg = 0;
      while ((size_t{2} << lg) <= n) ++lg;
      pending_.push_back(Range{0, n, 2 * lg});
    } else {
      done_ = n;
    }
  }

  // a[0..sorted()) already hold their final std::sort values (or, below a
  // SetPrefix boundary, their final values as a set).
  size_t sorted() const { return done_; }

  // After this, a[0..p) hold the first p values of std::sort's result as a
  // set (in no particular order) and a[p..sorted()) their final values:
  // ranges that lie wholly inside [0, p) are dropped unsorted -- they are
  // leaves of the partition tree whose membership is already final -- and
  // only a range straddling p is refined (partitioned, or finished as a leaf).
  void SetPrefix(size_t p) {
    while (!pending_.empty()) {
      const Range r = pending_.back();
      if (r.hi <= p) {
        pending_.pop_back();
        done_ = r.hi;
        continue;
      }
      if (r.lo >= p) break;
      pending_.pop_back();
      Elem* f = a_ + r.lo;
      Elem* l = a_ + r.hi;
      if (r.hi - r.lo <= kThreshold) {
        InsertionSort(f, l);
        done_ = r.hi;
      } else if (r.depth == 0) {
        HeapSort(f, l);
        done_ = r.hi;
      } else {
        const size_t cut = Cut(f, l);
        pending_.push_back(Range{cut, r.hi, r.depth - 1});
        pending_.push_back(Range{r.lo, cut, r.depth - 1});
      }
    }
    if (done_ < p) done_ = p;
  }

  // After this, a[0..i] hold their final std::sort values.
  void EnsureSorted(size_t i) {
    while (done_ <= i && !pending_.empty()) {
      Range r = pending_.back();
      pending_.pop_back();
      Elem* f = a_ + r.lo;
      Elem* l = a_ + r.hi;
      if (r.hi - r.lo <= kThreshold) {
        InsertionSort(f, l);
        done_ = r.hi;
      } else if (r.depth == 0) {
        HeapSort(f, l);
        done_ = r.hi;
      } else {
        const size_t cut = Cut(f, l);
        pending_.push_back(Range{cut, r.hi, r.depth - 1});
        pending_.push_back(Range{r.lo, cut, r.depth - 1});
      }
    }
  }

 private:
  static constexpr size_t kThreshold = 16;
  // ranges partitioned on the pool: only large frames' (the parallel form
  // does ~3x the sequential work; below this the pool's latency gain is not
  // worth its CPU when several encodes share the pool)
  static constexpr size_t kParallelMin = size_t{1} << 20;
  struct Range {
    size_t lo, hi;
    int depth;
  };

  // One introsort step on [f, l): median-of-3 pivot to the front, unguarded
  // partition; returns the cut (an index of a_).
  size_t Cut(Elem* f, Elem* l) {
    Elem* mid = f + (l - f) / 2;
    MoveMedianToFirst(f, f + 1, mid, l - 1);
    const size_t len = static_cast<size_t>(l - f);
    Elem* c = len >= kParallelMin && len <= 0xffffffffu ? ParallelPartition(f, l)
                                                          : UnguardedPartition(f + 1, l, f);
    return static_cast<size_t>(c - a_);
  }

  // UnguardedPartition(f + 1, l, f) on the pool.  L[k]: the k-th position of
  // [f + 1, l) (ascending) whose key is not below the pivot, R[k]: the k-th
  // (descending) of [f, l) whose key is not above it.  While L[k] < R[k] the
  // sequential loop swaps exactly these pairs (no scan meets a swapped
  // position before the pointers cross); with K the first k where L[k] >=
  // R[k], its last left scan stops at min(L[K], R[K - 1]) -- R[K - 1] now
  // holds an element not below the pivot -- which is the cut.  Positions are
  // u32 (the range is under 2^32): 4 B per entry of L and R at a cut.
  Elem* ParallelPartition(Elem* f, Elem* l) {
    const float pv = f->second;
    const size_t n = static_cast<size_t>(l - f);
    const int chunks = 64;
    const size_t per = (n + chunks - 1) / chunks;
    std::vector<size_t> nl(chunks + 1, 0), nr(chunks + 1, 0);
    ParallelFor(chunks, [&](int c) {
      size_t a = 0, b = 0;
      for (size_t i = c * per; i < std::min(n, (c + 1) * per); ++i) {
        const float k = f[i].second;
        a += (i > 0 && !(k < pv)) ? 1 : 0;
        b += !(pv < k) ? 1 : 0;
      }
      nl[c + 1] = a;
      nr[c + 1] = b;
    });
    for (int c = 0; c < chunks; ++c) {
      nl[c + 1] += nl[c];
      nr[c + 1] += nr[c];
    }
    const size_t cl = nl[chunks], cr = nr[chunks];
    std::vector<uint32_t> L(cl), R(cr);
    ParallelFor(chunks, [&](int c) {
      size_t a = nl[c], b = cr - nr[c];  // R descending: chunk c's last slot
      for (size_t i = c * per; i < std::min(n, (c + 1) * per); ++i) {
        const float k = f[i].second;
        if (i > 0 && !(k < pv)) L[a++] = static_cast<uint32_t>(i);
        if (!(pv < k)) R[--b] = static_cast<uint32_t>(i);
      }
    });
    // K: first k with L[k] >= R[k] (L rises, R falls)
    size_t lo = 0, hi = std::min(cl, cr);
    while (lo < hi) {
      const size_t m = lo + (hi - lo) / 2;
      if (L[m] >= R[m]) hi = m; else lo = m + 1;
    }
    const size_t K = lo;
    const int swap_chunks = static_cast<int>(std::min<size_t>(64, (K + 4095) / 4096));
    if (swap_chunks > 0) {
      const size_t sp = (K + swap_chunks - 1) / swap_chunks;
      ParallelFor(swap_chunks, [&](int c) {
        for (size_t k = c * sp; k < std::min(K, (c + 1) * sp); ++k) std::swap(f[L[k]], f[R[k]]);
      });
    }
    size_t cut = K < cl ? static_cast<size_t>(L[K]) : n;
    if (K > 0) cut = std::min(cut, static_cast<size_t>(R[K - 1]));
    return f + cut;
  }

  static bool Less(const Elem& x, const Elem& y) { return x.second < y.second; }

  static void MoveMedianToFirst(Elem* r, Elem* a, Elem* b, Elem* c) {
    if (Less(*a, *b)) {
      if (Less(*b, *c)) std::swap(*r, *b);
      else if (Less(*a, *c)) std::swap(*r, *c);
      else std::swap(*r, *a);
    } else if (Less(*a, *c)) {
      std::swap(*r, *a);
    } else if (Less(*b, *c)) {
      std::swap(*r, *c);
    } else {
      std::swap(*r, *b);
    }
  }

  static Elem* UnguardedPartition(Elem* f, Elem* l, const Elem* pivot) {
    for (;;) {
      while (Less(*f, *pivot)) ++f;
      --l;
      while (Less(*pivot, *l)) --l;
      if (!(f < l)) return f;
      std::swap(*f, *l);
      ++f;
    }
  }

  static void InsertionSort(Elem* f, Elem* l) {
    if (f == l) return;
    for (Elem* i = f + 1; i != l; ++i) {
      Elem v = *i;
      Elem* j = i;
      while (j != f && Less(v, *(j - 1))) {
        *j = *(j - 1);
        --j;
      }
      *j = v;
    }
  }

  // std::__partial_sort(f, l, l): make_heap + sort_heap (bits/stl_heap.h).
  static void AdjustHeap(Elem* f, ptrdiff_t hole, ptrdiff_t len, Elem v) {
    const ptrdiff_t top = hole;
    ptrdiff_t child = hole;
    while (child < (len - 1) / 2) {
      child = 2 * (child + 1);
      if (Less(f[child], f[child - 1])) child--;
      f[hole] = f[child];
      hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
      child = 2 * (child + 1);
      f[hole] = f[child - 1];
      hole = child - 1;
    }
    ptrdiff_t parent = (hole - 1) / 2;
    while (hole > top && Less(f[parent], v)) {
      f[hole] = f[parent];
      hole = parent;
      parent = (hole - 1) / 2;
    }
    f[hole] = v;
  }

  static void HeapSort(Elem* f, Elem* l) {
    const ptrdiff_t len = l - f;
    if (len >= 2) {
      for (ptrdiff_t parent = (len - 2) / 2;; --parent) {
        AdjustHeap(f, parent, len, f[parent]);
        if (parent == 0) break;
      }
    }
    while (l - f > 1) {
      --l;
      Elem v = *l;
      *l = *f;
      AdjustHeap(f, 0, l - f, v);
    }
  }

  Elem* a_;
  size_t done_ = 0;
  std::vector<Range> pending_;  // back() is the leftmost unfinished range
};

}  // namespace gz
