// The reference's own benchmark shapes (tests/benchmark.inc users) timed per call through the public C API.
//
// The same source is compiled twice (tools/bench_reference_shapes.py):
//   * against the reference sources (src/*.c, -O2 -march=native; its
//     FFT / overlap-save paths need the external FFTF library, which is not
//     available offline, so those rows are built without them: -DNO_FFT);
//   * against this repo's libvelessimd.so (source-compatible headers).
// Both binaries run on the same host (the GPU box), so the reference's AVX
// code and this library's MFMA / LDS-FFT kernels are timed on identical
// inputs: input[i] = sinf(i) * 10 (reference tests/benchmark.inc:70-72).
// Per-call times include the host<->device staging of the host-pointer API.
// With -DVELES_DEVICE the binary also times device-resident batched calls
// (vs_* API), i.e. the throughput a GPU caller sees.
// Output: one JSON object, microseconds per call.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

extern "C" {
#include <simd/convolve.h>
#include <simd/matrix.h>
#include <simd/memory.h>
#include <simd/wavelet.h>
}
#ifdef VELES_DEVICE
#include <hip/hip_runtime.h>
#include <simd/gpu.h>
extern "C" {
#include <simd/mathfun.h>
}
#endif

namespace {

std::string g_json = "{";
bool g_first = true;

void emit(const std::string &key, double us) {
  char buf[256];
  snprintf(buf, sizeof(buf), "%s\"%s\": %.5f", g_first ? "" : ", ", key.c_str(), us);
  g_json += buf;
  g_first = false;
  fprintf(stderr, "%-48s %12.3f us\n", key.c_str(), us);
}

template <class F>
double time_us(int iters, F &&f) {
  for (int i = 0; i < (iters < 10 ? iters : 10); i++) f();  // warm-up
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; i++) f();
  auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
}

std::vector<float> sig(size_t n) {
  std::vector<float> v(n);
  for (size_t i = 0; i < n; i++) v[i] = sinf(static_cast<float>(i)) * 10.f;
  return v;
}

void conv_rows(int scale) {
  // rows 1-2, 10, 11: brute-force SIMD convolution
  struct S { int x, h, iters; } shapes[] = {{512, 512, 2000}, {1000, 50, 5000}, {200, 50, 5000}};
  for (auto s : shapes) {
    auto x = sig(s.x), h = sig(s.h);
    std::vector<float> y(s.x + s.h - 1);
    const int it = s.iters / scale + 1;
    emit("convolve_simd_" + std::to_string(s.x) + "x" + std::to_string(s.h),
         time_us(it, [&] { convolve_simd(1, x.data(), s.x, h.data(), s.h, y.data()); }));
    emit("convolve_scalar_" + std::to_string(s.x) + "x" + std::to_string(s.h),
         time_us(it / 4 + 1, [&] { convolve_simd(0, x.data(), s.x, h.data(), s.h, y.data()); }));
  }
#ifndef NO_FFT
  // rows 3-5, 7: FFT convolution; rows 8, 9: overlap-save
  struct F { int x, h, iters; } fs[] = {{512, 512, 2000}, {256, 256, 2000}, {128, 128, 2000},
                                          {350, 350, 2000}};
  for (auto s : fs) {
    auto x = sig(s.x), h = sig(s.h);
    std::vector<float> y(s.x + s.h - 1);
    auto hd = convolve_fft_initialize(s.x, s.h);
    emit("convolve_fft_" + std::to_string(s.x) + "x" + std::to_string(s.h),
         time_us(s.iters / scale + 1, [&] { convolve_fft(hd, x.data(), h.data(), y.data()); }));
    convolve_fft_finalize(hd);
  }
  struct O { int x, h, iters; } os[] = {{1000, 50, 2000}, {2000, 950, 1000}, {200, 50, 2000}};
  for (auto s : os) {
    auto x = sig(s.x), h = sig(s.h);
    std::vector<float> y(s.x + s.h - 1);
    auto hd = convolve_overlap_save_initialize(s.x, s.h);
    emit("convolve_overlap_save_" + std::to_string(s.x) + "x" + std::to_string(s.h),
         time_us(s.iters / scale + 1,
                 [&] { convolve_overlap_save(hd, x.data(), h.data(), y.data()); }));
    convolve_overlap_save_finalize(hd);
  }
#endif
}

void matrix_rows(int scale) {
  // rows 12-14: 300x256 . 256x1000 (and the transposed form)
  const int h1 = 300, w1 = 256, w2 = 1000;
  auto a = sig(static_cast<size_t>(h1) * w1), b = sig(static_cast<size_t>(w1) * w2);
  auto bt = sig(static_cast<size_t>(w2) * w1);
  std::vector<float> c(static_cast<size_t>(h1) * w2);
  const int it = 40 / scale + 1;
  emit("matrix_multiply_300x256x1000",
       time_us(it, [&] { matrix_multiply(1, a.data(), b.data(), w1, h1, w2, w1, c.data()); }));
  emit("matrix_multiply_transposed_300x256x1000", time_us(it, [&] {
         matrix_multiply_transposed(1, a.data(), bt.data(), w1, h1, w1, w2, c.data());
       }));
  emit("matrix_multiply_scalar_300x256x1000",
       time_us(2, [&] { matrix_multiply(0, a.data(), b.data(), w1, h1, w2, w1, c.data()); }));
#ifdef VELES_DEVICE
  // the same calls on page-locked operands from vs_host_alloc
  float *pa = static_cast<float *>(vs_host_alloc(a.size() * sizeof(float)));
  float *pb = static_cast<float *>(vs_host_alloc(b.size() * sizeof(float)));
  float *pbt = static_cast<float *>(vs_host_alloc(bt.size() * sizeof(float)));
  float *pc = static_cast<float *>(vs_host_alloc(c.size() * sizeof(float)));
  if (!pa || !pb || !pbt || !pc) return;
  std::copy(a.begin(), a.end(), pa);
  std::copy(b.begin(), b.end(), pb);
  std::copy(bt.begin(), bt.end(), pbt);
  emit("matrix_multiply_pinned_300x256x1000",
       time_us(it * 5, [&] { matrix_multiply(1, pa, pb, w1, h1, w2, w1, pc); }));
  emit("matrix_multiply_transposed_pinned_300x256x1000", time_us(it * 5, [&] {
         matrix_multiply_transposed(1, pa, pbt, w1, h1, w1, w2, pc);
       }));
  vs_host_free(pc);
  vs_host_free(pa);
  vs_host_free(pb);
  vs_host_free(pbt);
#endif
}

void wavelet_rows(int scale) {
  // row 15: wavelet_apply, Daubechies, periodic, length 512
  auto src = sig(512);
  for (int order : {4, 6, 8, 12, 16}) {
    float *prep = wavelet_prepare_array(order, src.data(), src.size());
    float *hi = wavelet_allocate_destination(order, src.size());
    float *lo = wavelet_allocate_destination(order, src.size());
    emit("wavelet_apply_db" + std::to_string(order) + "_512", time_us(20000 / scale + 1, [&] {
           wavelet_apply(WAVELET_TYPE_DAUBECHIES, order, EXTENSION_TYPE_PERIODIC, prep,
                         src.size(), hi, lo);
         }));
    emit("wavelet_apply_na_db" + std::to_string(order) + "_512", time_us(20000 / scale + 1, [&] {
           wavelet_apply_na(WAVELET_TYPE_DAUBECHIES, order, EXTENSION_TYPE_PERIODIC,
                            src.data(), src.size(), hi, lo);
         }));
    free(prep);
    free(hi);
    free(lo);
  }
}

#ifdef VELES_DEVICE
__global__ void empty_kernel() {}

// Where a small host-API call's time goes: an empty launch + event wait
// (the platform floor), a trivial host-API call (staging + dispatch), and
// the device-resident single-signal convolutions (GPU execution latency of
// the kernels themselves, one workgroup each).
void floor_rows() {
  hipStream_t s = nullptr;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  auto wait = [&] {
    hipEventRecord(ev, s);
    while (hipEventQuery(ev) == hipErrorNotReady) {
    }
  };
  emit("floor_empty_launch_and_wait", time_us(20000, [&] {
         hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
         wait();
       }));
  std::vector<float> a(4, 1.f), b(4, 2.f), c(4);
  // sums of host arrays stay on the host at every size; the smallest math
  // call that makes the GPU round trip is pow over 8192 elements
  emit("host_api_matrix_add_2x2",
       time_us(20000, [&] { matrix_add(1, a.data(), b.data(), 2, 2, c.data()); }));
  std::vector<float> a2(16384, 1.f), b2(16384, 2.f), c2(16384);
  emit("host_api_matrix_add_128x128",
       time_us(20000, [&] { matrix_add(1, a2.data(), b2.data(), 128, 128, c2.data()); }));
  emit("floor_host_api_pow_psv_8192",
       time_us(20000, [&] { pow_psv(1, a2.data(), b2.data(), 8192, c2.data()); }));
  {  // the PCIe share of the 300x256 . 256x1000 host call: A and B in, C out
    const size_t in_b = (300 * 256 + 256 * 1000) * sizeof(float), out_b = 300 * 1000 * sizeof(float);
    void *hin = vs_host_alloc(in_b), *hout = vs_host_alloc(out_b), *din = nullptr, *dout = nullptr;
    hipMalloc(&din, in_b);
    hipMalloc(&dout, out_b);
    if (hin && hout && din && dout)
      emit("floor_pcie_pinned_1.33MB_in_1.2MB_out", time_us(500, [&] {
             hipMemcpyAsync(din, hin, in_b, hipMemcpyHostToDevice, s);
             hipMemcpyAsync(hout, dout, out_b, hipMemcpyDeviceToHost, s);
             wait();
           }));
    hipFree(din);
    hipFree(dout);
    vs_host_free(hin);
    vs_host_free(hout);
  }
  for (int algo : {VS_CONV_DIRECT, VS_CONV_FFT}) {
    float *x, *h, *y;
    hipMalloc(&x, 4 * 512);
    hipMalloc(&h, 4 * 512);
    hipMalloc(&y, 4 * 1023);
    hipMemset(x, 0, 4 * 512);
    hipMemset(h, 0, 4 * 512);
    emit(std::string("floor_device_conv_") + (algo == VS_CONV_FFT ? "fft" : "direct") +
             "_512x512_single_call",
         time_us(5000, [&] {
           (void)vs_conv1d(algo, 0, x, 512, 512, h, 512, 0, y, 1023, 1, s);
           wait();
         }));
    hipFree(x);
    hipFree(h);
    hipFree(y);
  }
  hipEventDestroy(ev);
  hipStreamDestroy(s);
}

// Device-resident batched throughput: the same shapes, many signals per
// launch, reported as microseconds per signal (per matrix product).
void device_rows() {
  hipStream_t s = nullptr;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  auto sync_time = [&](int iters, auto &&f) {
    f();
    hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++) f();
    hipStreamSynchronize(s);
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
               .count() / iters;
  };
  struct C { int x, h, algo; const char *name; } cs[] = {
      {512, 512, VS_CONV_DIRECT, "direct"},  {512, 512, VS_CONV_FFT, "fft"},
      {1000, 50, VS_CONV_DIRECT, "direct"},  {1000, 50, VS_CONV_OVERLAP_SAVE, "overlap_save"},
      {2000, 950, VS_CONV_OVERLAP_SAVE, "overlap_save"}, {200, 50, VS_CONV_DIRECT, "direct"}};
  const int batch = 8192;
  for (auto c : cs) {
    float *x, *h, *y;
    const int yl = c.x + c.h - 1;
    hipMalloc(&x, sizeof(float) * c.x * batch);
    hipMalloc(&h, sizeof(float) * c.h);
    hipMalloc(&y, sizeof(float) * yl * batch);
    hipMemset(x, 0, sizeof(float) * c.x * batch);
    hipMemset(h, 0, sizeof(float) * c.h);
    const double us = sync_time(20, [&] {
      (void)vs_conv1d(c.algo, 0, x, c.x, c.x, h, c.h, 0, y, yl, batch, s);
    });
    emit(std::string("device_batched_conv_") + c.name + "_" + std::to_string(c.x) + "x" +
             std::to_string(c.h) + "_per_signal", us / batch);
    hipFree(x);
    hipFree(h);
    hipFree(y);
  }
  {
    const int m = 300, k = 256, n = 1000, batch = 256;
    float *a, *b, *c;
    hipMalloc(&a, sizeof(float) * m * k * batch);
    hipMalloc(&b, sizeof(float) * k * n * batch);
    hipMalloc(&c, sizeof(float) * m * n * batch);
    hipMemset(a, 0, sizeof(float) * m * k * batch);
    hipMemset(b, 0, sizeof(float) * k * n * batch);
    const double us = sync_time(20, [&] {
      vs_sgemm_strided_batched(0, 0, m, n, k, 1.f, a, k, static_cast<int64_t>(m) * k, b, n,
                               static_cast<int64_t>(k) * n, 0.f, c, n,
                               static_cast<int64_t>(m) * n, batch, s);
    });
    emit("device_batched_sgemm_300x256x1000_per_matrix", us / batch);
    hipFree(a);
    hipFree(b);
    hipFree(c);
  }
  for (int order : {4, 8, 16}) {
    const int len = 512, batch = 32768;  // grid.y <= 65535
    float *x, *hi, *lo;
    hipMalloc(&x, sizeof(float) * len * batch);
    hipMalloc(&hi, sizeof(float) * len / 2 * batch);
    hipMalloc(&lo, sizeof(float) * len / 2 * batch);
    hipMemset(x, 0, sizeof(float) * len * batch);
    const double us = sync_time(20, [&] {
      (void)vs_dwt(WAVELET_TYPE_DAUBECHIES, order, EXTENSION_TYPE_PERIODIC, x, len, len, hi, lo,
             len / 2, batch, s);
    });
    emit("device_batched_dwt_db" + std::to_string(order) + "_512_per_signal", us / batch);
    hipFree(x);
    hipFree(hi);
    hipFree(lo);
  }
  hipStreamDestroy(s);
}
#endif

}  // namespace

int main(int argc, char **argv) {
  const int scale = argc > 1 ? std::atoi(argv[1]) : 1;  // divide iteration counts
  conv_rows(scale);
  matrix_rows(scale);
  wavelet_rows(scale);
#ifdef VELES_DEVICE
  floor_rows();
  device_rows();
#endif
  g_json += "}";
  printf("%s\n", g_json.c_str());
  return 0;
}
