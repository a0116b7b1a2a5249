// Host-API matmul timing from C++ on the system HIP runtime (no torch):
// plain and transposed forms alternately, median of 41 calls each.
#include <simd/matrix.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <vector>

template <class F>
double med_us(F &&f) {
  std::vector<double> t;
  for (int i = 0; i < 5; i++) f();
  for (int i = 0; i < 41; i++) {
    auto a = std::chrono::steady_clock::now();
    f();
    auto b = std::chrono::steady_clock::now();
    t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  std::sort(t.begin(), t.end());
  double sum = 0;
  for (double v : t) sum += v;
  std::printf("  [median %.1f mean %.1f max %.1f]", t[t.size() / 2], sum / t.size(), t.back());
  return t[t.size() / 2];
}

int main() {
  const size_t w1 = 256, h1 = 300, w2 = 1000;
  std::vector<float> a(h1 * w1), b(w1 * w2), bt(w2 * w1), c(h1 * w2);
  for (size_t i = 0; i < a.size(); i++) a[i] = std::sin(float(i)) * 10.f;
  for (size_t i = 0; i < b.size(); i++) b[i] = bt[i] = std::sin(float(i)) * 10.f;
  for (int r = 0; r < 3; r++) {
    double nn = med_us([&] { matrix_multiply(1, a.data(), b.data(), w1, h1, w2, w1, c.data()); });
    double nt = med_us([&] {
      matrix_multiply_transposed(1, a.data(), bt.data(), w1, h1, w1, w2, c.data());
    });
    double nt_b = med_us([&] {
      matrix_multiply_transposed(1, a.data(), b.data(), w1, h1, w1, w2, c.data());
    });
    std::printf("nn %.1f nt %.1f nt(b) %.1f us\n", nn, nt, nt_b);
  }
  return 0;
}
