// LazyStdSort must reproduce libstdc++ std::sort's permutation (ties
// included) on every prefix it materialises.
//   lazy_sort_check SEED
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "host/lazy_sort.h"

int main(int argc, char** argv) {
  const unsigned seed = argc > 1 ? atoi(argv[1]) : 1;
  std::mt19937 rng(seed);
  int bad = 0, cases = 0;
  for (int n : {0, 1, 2, 3, 15, 16, 17, 33, 100, 1000, 4097, 100000, 300000, 3000000}) {
    for (int distinct : {1, 2, 7, 100, 1 << 30}) {
      std::vector<std::pair<int, float>> a(n);
      for (int i = 0; i < n; ++i)
        a[i] = {i, static_cast<float>(rng() % static_cast<unsigned>(distinct)) * 0.25f - 3.0f};
      if (distinct == 7 && n > 10) std::sort(a.begin(), a.begin() + n / 2,
          [](const std::pair<int, float>& x, const std::pair<int, float>& y) { return x.second > y.second; });
      auto ref = a;
      std::sort(ref.begin(), ref.end(),
                [](const std::pair<int, float>& x, const std::pair<int, float>& y) { return x.second < y.second; });
      gz::LazyStdSort s(a.data(), a.size());
      const size_t prefix = n ? static_cast<size_t>(rng() % n) : 0;
      s.EnsureSorted(prefix);
      for (size_t i = 0; i < s.sorted() && i < a.size(); ++i)
        if (a[i] != ref[i]) { ++bad; break; }
      s.EnsureSorted(a.size());
      if (a != ref) ++bad;
      ++cases;
      // SetPrefix(p): a[0..p) is std::sort's first p as a multiset, the rest
      // (materialised later) exactly std::sort's
      {
        std::vector<std::pair<int, float>> b(n);
        for (int i = 0; i < n; ++i) b[i] = {i, static_cast<float>(rng() % static_cast<unsigned>(distinct)) * 0.5f};
        auto rb = b;
        std::sort(rb.begin(), rb.end(),
                  [](const std::pair<int, float>& x, const std::pair<int, float>& y) { return x.second < y.second; });
        gz::LazyStdSort t(b.data(), b.size());
        const size_t p = n ? static_cast<size_t>(rng() % (n + 1)) : 0;
        t.SetPrefix(p);
        auto head = std::vector<std::pair<int, float>>(b.begin(), b.begin() + p);
        auto rhead = std::vector<std::pair<int, float>>(rb.begin(), rb.begin() + p);
        std::sort(head.begin(), head.end());
        std::sort(rhead.begin(), rhead.end());
        if (head != rhead || t.sorted() < p) ++bad;
        for (size_t i = p; i < t.sorted() && i < b.size(); ++i)
          if (b[i] != rb[i]) { ++bad; break; }
        if (n) t.EnsureSorted(b.size() - 1);
        for (size_t i = p; i < b.size(); ++i)
          if (b[i] != rb[i]) { ++bad; break; }
        ++cases;
      }
    }
  }
  printf("{\"cases\": %d, \"bad\": %d}\n", cases, bad);
  return bad ? 3 : 0;
}
