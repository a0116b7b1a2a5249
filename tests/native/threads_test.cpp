// Host API from several threads at once, for the ThreadSanitizer build
// (`make tsan`): every thread mixes convolutions (direct calls and handles),
// matrix, math, wavelet, normalisation and peak calls on its own arrays and
// checks them against values computed before the threads start.  Without a
// GPU (or with VELES_DISABLE_GPU=1) this exercises the host paths and their
// per-thread scratch; with one, the staging arenas, the scratch pool and the
// twiddle cache of the runtime.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include <simd/convolve.h>
#include <simd/detect_peaks.h>
#include <simd/mathfun.h>
#include <simd/matrix.h>
#include <simd/normalize.h>
#include <simd/wavelet.h>

namespace {

std::atomic<int> g_failures{0};

void check(bool ok, const char *what, int thread) {
  if (!ok) {
    std::fprintf(stderr, "thread %d: %s failed\n", thread, what);
    g_failures++;
  }
}

float max_diff(const std::vector<float> &a, const std::vector<float> &b) {
  float m = 0.f;
  for (size_t i = 0; i < a.size(); i++) m = std::fmax(m, std::fabs(a[i] - b[i]));
  return m;
}

void work(int id, int rounds) {
  unsigned seed = 1234u + 77u * id;
  auto rnd = [&] { seed = seed * 1664525u + 1013904223u; return (seed >> 8) * (2.f / 16777216.f) - 1.f; };
  const size_t xl = 3000 + 17 * id, hl = 90 + id, xb = 40000 + 1001 * id, hb = 700 + 3 * id;
  std::vector<float> x(xl), h(hl), xL(xb), hL(hb), a(64 * 96), b(96 * 80), big(200 * 300), v(5000);
  for (auto *vec : {&x, &h, &xL, &hL, &a, &b, &big}) for (auto &e : *vec) e = rnd();
  for (auto &e : v) e = 0.1f + 2.4f * (rnd() + 1.f);
  std::vector<uint8_t> img(64 * 48);
  for (auto &e : img) e = static_cast<uint8_t>((rnd() + 1.f) * 127.f);
  // expected values from the scalar paths, computed by this thread alone
  std::vector<float> conv0(xl + hl - 1), convL0(xb + hb - 1), mm0(64 * 80), add0(big.size()), exp0(v.size()),
      hi0(256), lo0(256), n0(img.size());
  convolve_simd(0, x.data(), xl, h.data(), hl, conv0.data());
  convolve_simd(0, xL.data(), xb, hL.data(), hb, convL0.data());
  matrix_multiply(0, a.data(), b.data(), 96, 64, 80, 96, mm0.data());
  matrix_add(0, big.data(), big.data(), 300, 200, add0.data());
  exp_psv(0, v.data(), v.size(), exp0.data());
  wavelet_apply_na(WAVELET_TYPE_DAUBECHIES, 8, EXTENSION_TYPE_PERIODIC, x.data(), 512, hi0.data(), lo0.data());
  normalize2D(0, img.data(), 64, 64, 48, n0.data(), 64);
  ExtremumPoint *p0 = nullptr;
  size_t np0 = 0;
  detect_peaks(0, xL.data(), xb, kExtremumTypeBoth, &p0, &np0);
  for (int r = 0; r < rounds; r++) {
    std::vector<float> y(conv0.size()), yL(convL0.size()), mm(mm0.size()), add(add0.size()), ex(exp0.size()),
        hi(256), lo(256), nn(n0.size());
    convolve_simd(1, x.data(), xl, h.data(), hl, y.data());
    check(max_diff(y, conv0) < 2e-3f, "convolve_simd small", id);
    convolve_simd(1, xL.data(), xb, hL.data(), hb, yL.data());
    check(max_diff(yL, convL0) < 2e-2f, "convolve_simd large", id);
    ConvolutionHandle ch = convolve_initialize(xb, hb);
    convolve(ch, xL.data(), hL.data(), yL.data());
    convolve_finalize(ch);
    check(max_diff(yL, convL0) < 2e-2f, "convolve handle", id);
    matrix_multiply(1, a.data(), b.data(), 96, 64, 80, 96, mm.data());
    check(max_diff(mm, mm0) < 2e-4f, "matrix_multiply", id);
    matrix_add(1, big.data(), big.data(), 300, 200, add.data());
    check(max_diff(add, add0) == 0.f, "matrix_add", id);
    exp_psv(1, v.data(), v.size(), ex.data());
    float rel = 0.f;
    for (size_t i = 0; i < ex.size(); i++) rel = std::fmax(rel, std::fabs(ex[i] - exp0[i]) / exp0[i]);
    check(rel < 1e-6f, "exp_psv", id);
    wavelet_apply(WAVELET_TYPE_DAUBECHIES, 8, EXTENSION_TYPE_PERIODIC, x.data(), 512, hi.data(), lo.data());
    check(max_diff(hi, hi0) < 1e-5f && max_diff(lo, lo0) < 1e-5f, "wavelet_apply", id);
    normalize2D(1, img.data(), 64, 64, 48, nn.data(), 64);
    check(max_diff(nn, n0) < 1e-6f, "normalize2D", id);
    ExtremumPoint *p1 = nullptr;
    size_t np1 = 0;
    detect_peaks(1, xL.data(), xb, kExtremumTypeBoth, &p1, &np1);
    bool same = np1 == np0;
    for (size_t i = 0; same && i < np0; i++) same = p1[i].position == p0[i].position && p1[i].value == p0[i].value;
    check(same, "detect_peaks", id);
    std::free(p1);
  }
  std::free(p0);
}

}  // namespace

int main(int argc, char **argv) {
  const int nthreads = argc > 1 ? std::atoi(argv[1]) : 8, rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  std::vector<std::thread> threads;
  for (int i = 0; i < nthreads; i++) threads.emplace_back(work, i, rounds);
  for (auto &t : threads) t.join();
  std::printf("%d thread(s) x %d round(s): %d failure(s)\n", nthreads, rounds, g_failures.load());
  return g_failures.load() ? 1 : 0;
}
