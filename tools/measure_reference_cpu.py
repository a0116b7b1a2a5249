#!/usr/bin/env python3
"""Measure the reference library's own CPU code on the BASELINE shapes.

The reference publishes no numbers.  This compiles the
reference sources (read-only mount /root/reference) with its documented
flags (-O2 -march=native, common.ac:267) into a scratch directory and times
  * matrix_multiply(simd=1, ...) at 4096^3 (its AVX GEMM, one core),
  * convolve_simd(simd=1, ...) at x = 2^20, h = 4096 (its brute-force AVX
    convolution; the FFT / overlap-save paths need the external FFTF library,
    which is not available offline -- a stub header satisfies the include,
    those paths are not timed: "parity unpinned").
Results go to bench/reference_cpu_baseline.json, which bench.py divides by.
Only runs where /root/reference exists (the build container).
"""
import json
import os
import subprocess
import sys
import tempfile

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r'''
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
extern "C" {
#include <simd/matrix.h>
#include <simd/memory.h>
#include <simd/convolve.h>
}
int main() {
  const int n = 4096;
  float *a = mallocf((size_t)n * n), *b = mallocf((size_t)n * n), *c = mallocf((size_t)n * n);
  for (size_t i = 0; i < (size_t)n * n; i++) { a[i] = (i % 17) * 0.1f - 0.8f; b[i] = (i % 13) * 0.1f - 0.6f; }
  auto t0 = std::chrono::steady_clock::now();
  matrix_multiply(1, a, b, n, n, n, n, c);
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("{\"sgemm_4096_seconds\": %.4f, \"sgemm_4096_gflops\": %.4f, ", dt, 2.0 * n * n * (double)n / dt / 1e9);
  const int xl = 1 << 20, hl = 4096;
  float *x = mallocf(xl), *h = mallocf(hl), *y = mallocf(xl + hl - 1);
  for (int i = 0; i < xl; i++) x[i] = sinf(i) * 10;
  for (int i = 0; i < hl; i++) h[i] = 1.0f / (i + 1);
  t0 = std::chrono::steady_clock::now();
  convolve_simd(1, x, xl, h, hl, y);
  dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("\"conv_direct_2^20x4096_seconds\": %.4f, \"conv_direct_2^20x4096_msamples_per_s\": %.4f}\n", dt, xl / dt / 1e6);
  return 0;
}
'''

FFTF_STUB = r'''
#pragma once
typedef int FFTFType; typedef int FFTFDirection; typedef int FFTFDimension; typedef int FFTFOptions;
#define FFTF_TYPE_REAL 0
#define FFTF_DIRECTION_FORWARD 0
#define FFTF_DIRECTION_BACKWARD 1
#define FFTF_DIMENSION_1D 1
#define FFTF_NO_OPTIONS 0
typedef void* FFTFInstance;
static inline void *fftf_init(int, int, int, const int *, int, const float *, float *) { return 0; }
static inline void *fftf_init_batch(int, int, int, const int *, int, int, const float *const *, float **) { return 0; }
static inline void fftf_calc(void *) {}
static inline void fftf_destroy(void *) {}
'''


def main():
    if not os.path.isdir(REF):
        print("reference tree not present; nothing to measure")
        return 0
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "fftf"))
        with open(os.path.join(d, "fftf", "api.h"), "w") as f:
            f.write(FFTF_STUB)
        with open(os.path.join(d, "main.cc"), "w") as f:
            f.write(DRIVER)
        flags = ["-O2", "-march=native", "-I" + os.path.join(REF, "inc"), "-I" + REF, "-I" + d]
        objs = []
        for src in ("src/matrix.c", "src/memory.c", "src/convolve.c"):
            o = os.path.join(d, os.path.basename(src) + ".o")
            subprocess.run(["gcc", "-std=gnu99", "-c", os.path.join(REF, src), "-o", o] + flags,
                           check=True)
            objs.append(o)
        exe = os.path.join(d, "refbench")
        subprocess.run(["g++", "-O2", "-march=native", os.path.join(d, "main.cc")] + objs
                       + flags + ["-o", exe, "-lm"], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    res = json.loads(out)
    cpu = subprocess.run(["bash", "-c", "grep -m1 'model name' /proc/cpuinfo | cut -d: -f2"],
                         capture_output=True, text=True).stdout.strip()
    res["source"] = ("reference src/matrix.c + src/convolve.c compiled -O2 -march=native, "
                     f"one core of: {cpu}")
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    with open(os.path.join(REPO, "bench", "reference_cpu_baseline.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
