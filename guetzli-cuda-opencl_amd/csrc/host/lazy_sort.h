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
#pragma once

#include <stddef.h>

#include <utility>
#include <vector>

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
        Elem* mid = f + (l - f) / 2;
        MoveMedianToFirst(f, f + 1, mid, l - 1);
        const size_t cut = static_cast<size_t>(UnguardedPartition(f + 1, l, f) - a_);
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
        Elem* mid = f + (l - f) / 2;
        MoveMedianToFirst(f, f + 1, mid, l - 1);
        const size_t cut = static_cast<size_t>(UnguardedPartition(f + 1, l, f) - a_);
        pending_.push_back(Range{cut, r.hi, r.depth - 1});
        pending_.push_back(Range{r.lo, cut, r.depth - 1});
      }
    }
  }

 private:
  static constexpr size_t kThreshold = 16;
  struct Range {
    size_t lo, hi;
    int depth;
  };

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
