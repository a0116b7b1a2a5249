// convolve.h / correlate.h (reference src/convolve.c, src/correlate.c).
//
// Handles keep the reference's by-value struct layout; their heap state is a
// small plan record (fft_plan) describing the chosen GPU algorithm.  Operands
// may be host or device pointers; host operands are staged through the
// library stream and the call returns when the result is in place, like the
// reference's synchronous API.  Without a GPU, the FFT / overlap-save handles
// compute the same linear convolution with the host reference FFT.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/convolve.h"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "csrc/api/dispatch.h"
#include "csrc/ref/ref.h"
#include "simd/correlate.h"
#include "simd/gpu.h"

using vs::Staged;

namespace {

struct ConvPlan {
  int algorithm;  // vs_conv_algo actually executed
  size_t x_length, h_length;
  int block;      // transform length (informational)
};

int next_pow2_ge(size_t n) {  // saturates at 2^30 (the handles' int field)
  int p = 1;
  while (static_cast<size_t>(p) < n && p < (1 << 30)) p <<= 1;
  return p;
}

using vs::api::checked_int;

// Long signals in pageable host memory: x goes through the two halves of the
// pinned staging image in pieces, each convolved on its own and its tail of
// hl - 1 samples added to the head of the next piece's result (the
// convolution is linear in x).  While the GPU transfers and convolves one
// piece, the host copies the previous result out and the next piece in; a
// whole-signal call does the three one after the other (120 us per MiB).
// False (nothing done) when pieces do not apply.
bool piped_conv(const char *what, int algo, int reverse, const float *x, size_t xl,
                const float *h, size_t hl, float *result, hipStream_t s, vs_status *status) {
  *status = VS_OK;
  vs::StageImage img;
  // the direct sum with a long filter is bound by the GPU's arithmetic, not by
  // the copies: pieces would only add their overlap (2^24 x 65,536: 43 ms
  // against 33 ms whole)
  if (algo == VS_CONV_DIRECT && hl > 8192) return false;
  if (xl < (size_t{3} << 19) || !vs::is_pageable_host(x) || !vs::is_pageable_host(result) ||
      !vs::stage_image(&img))
    return false;
  const size_t half = img.bytes / 2, half_floats = half / 4;
  if (half_floats < hl + 4096) return false;
  const size_t piece = ((half_floats - hl - 256) / 2) & ~size_t{1023};
  if (piece < 8 * hl || xl < 2 * piece) return false;
  const size_t in_bytes = (piece * 4 + 255) & ~size_t{255};
  vs::DeviceBuffer hdev;
  if ((*status = hdev.alloc(hl * 4, s)) != VS_OK) return true;
  const hipError_t he = hipMemcpyAsync(hdev.get(), h, hl * 4, hipMemcpyHostToDevice, s);
  if (he != hipSuccess) {
    *status = vs::hip_status(he, "hipMemcpyAsync (filter)", __FILE__, __LINE__);
    return true;
  }
  hipEvent_t ev[2] = {nullptr, nullptr};
  if ((*status = vs::stage_half_event(0, &ev[0])) != VS_OK) return true;
  if ((*status = vs::stage_half_event(1, &ev[1])) != VS_OK) return true;
  const size_t pieces = (xl + piece - 1) / piece;
  vs::log(2, "%s: %zu samples in %zu pieces of %zu", what, xl, pieces, piece);
  for (size_t c = 0; c < pieces + 2 && *status == VS_OK; c++) {
    char *in_host = img.host + (c & 1) * half;
    const float *out_host = reinterpret_cast<const float *>(in_host + in_bytes);
    if (c >= 2) {  // retire piece c - 2, which used this half
      const size_t first = (c - 2) * piece, cnt = std::min(piece, xl - first);
      if ((*status = vs::wait_event(ev[c & 1])) != VS_OK) break;
      const size_t overlap = c > 2 ? hl - 1 : 0;
      float *dst = result + first;
      for (size_t i = 0; i < overlap; i++) dst[i] += out_host[i];
      std::memcpy(dst + overlap, out_host + overlap, (cnt + hl - 1 - overlap) * 4);
    }
    if (c < pieces) {
      const size_t first = c * piece, cnt = std::min(piece, xl - first);
      std::memcpy(in_host, x + first, cnt * 4);
      char *in_dev = img.dev + (c & 1) * half;
      float *out_dev = reinterpret_cast<float *>(img.mapped + (c & 1) * half + in_bytes);
      hipError_t e = hipMemcpyAsync(in_dev, in_host, cnt * 4, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) {
        *status = vs_conv1d(algo, reverse, reinterpret_cast<const float *>(in_dev),
                            static_cast<int64_t>(cnt), static_cast<int64_t>(cnt),
                            hdev.as<float>(), checked_int(what, hl), 0, out_dev,
                            static_cast<int64_t>(cnt + hl - 1), 1, s);
        if (*status == VS_OK) e = hipEventRecord(ev[c & 1], s);
      }
      if (e != hipSuccess) *status = vs::hip_status(e, "piped_conv", __FILE__, __LINE__);
    }
  }
  // on an error nothing may still be using the image when the caller goes on
  if (*status != VS_OK) (void)hipStreamSynchronize(s);
  return true;
}

void gpu_conv(const char *what, int algo, int reverse, const float *x, size_t xl,
              const float *h, size_t hl, float *result) {
  const size_t yl = xl + hl - 1;
  // Small direct convolutions run the tap-split kernel (conv.hip), whose
  // workgroups load their input window once with every load in flight:
  // their inputs are read zero-copy from the pinned staging arena (no
  // host->device copy; 512 x 512: one DMA start-up less per call).  Every
  // other path re-reads its inputs and stages them into device memory.
  const bool small_direct = algo == VS_CONV_DIRECT && xl * hl <= (size_t{1} << 20);
  const Staged::Dir in = small_direct ? Staged::kIn : Staged::kInReread;
  vs::api::run_sync(what, [&](hipStream_t s) {
    vs_status piped = VS_OK;
    if (piped_conv(what, algo, reverse, x, xl, h, hl, result, s, &piped)) return piped;
    Staged y(result, yl * 4, Staged::kOut, s);
    Staged xx(x, xl * 4, in, s), hh(h, hl * 4, in, s);
    VS_TRY(y.status());
    VS_TRY(xx.status());
    VS_TRY(hh.status());
    // signals of any length (vs_conv1d cuts rows of 2^29 outputs or more into
    // pieces); only the filter length is bounded
    VS_TRY(vs_conv1d(algo, reverse, xx.dev<float>(), static_cast<int64_t>(xl),
                     static_cast<int64_t>(xl), hh.dev<float>(), checked_int(what, hl),
                     0, y.dev<float>(), static_cast<int64_t>(yl), 1, s));
    return y.finish();
  });
}

// Convolutions (direct calls and handles alike) below this many multiply-adds run the vectorised host
// loops even with simd = 1 when every operand is in host memory: a GPU round
// trip (stage in, launch, stage out, sync) costs 16-18 us on MI355X, the
// host loop 0.02-0.05 ns per MAC (profiles/r3/hostapi).  VELES_HOST_MAX_MACS.
size_t host_max_macs() {
  static const size_t v = [] {
    const char *e = std::getenv("VELES_HOST_MAX_MACS");
    return e && *e ? static_cast<size_t>(std::atoll(e)) : static_cast<size_t>(3) << 18;
  }();
  return v;
}

void run_plan(const char *what, ConvPlan *plan, int reverse, const float *x,
              const float *h, float *result) {
  if (!plan || !x || !h || !result) vs::fatal("%s: invalid arguments", what);
  const bool tiny = plan->x_length * plan->h_length < host_max_macs() &&
                    !vs::api::any_device({x, h, result});
  if (tiny) {  // the direct sum on the host beats a transform and a GPU round trip
    if (reverse) vs::host::correlate_direct(x, plan->x_length, h, plan->h_length, result);
    else vs::host::convolve_direct(x, plan->x_length, h, plan->h_length, result);
  } else if (vs::gpu_available()) {
    gpu_conv(what, plan->algorithm, reverse, x, plan->x_length, h, plan->h_length,
             result);
  } else {
    vs::ref::convolve_fft(x, plan->x_length, h, plan->h_length, reverse, result);
  }
}

ConvPlan *make_plan(int algo, size_t xl, size_t hl) {
  if (xl == 0 || hl == 0) vs::fatal("convolution: empty input");
  auto *p = static_cast<ConvPlan *>(std::malloc(sizeof(ConvPlan)));
  p->algorithm = algo;
  p->x_length = xl;
  p->h_length = hl;
  p->block = algo == VS_CONV_OVERLAP_SAVE
                 ? vs_conv1d_os_block(checked_int("convolution", hl))
                 : next_pow2_ge(xl + hl - 1);
  return p;
}

ConvolutionFFTHandle fft_init(size_t xl, size_t hl, int reverse) {
  ConvolutionFFTHandle h;
  std::memset(&h, 0, sizeof(h));
  ConvPlan *p = make_plan(VS_CONV_FFT, xl, hl);
  h.fft_plan = p;
  h.fft_inverse_plan = p;
  h.M = static_cast<int *>(std::malloc(sizeof(int)));
  *h.M = p->block;
  // the reference's int fields saturate; the plan keeps the exact lengths
  h.x_length = static_cast<int>(std::min<size_t>(xl, INT_MAX));
  h.h_length = checked_int("convolve_fft_initialize", hl);
  h.inputs = nullptr;
  h.reverse = reverse;
  return h;
}

void fft_fini(ConvolutionFFTHandle h) {
  std::free(h.fft_plan);
  std::free(h.M);
}

ConvolutionOverlapSaveHandle os_init(size_t xl, size_t hl, int reverse) {
  // reference src/convolve.c:105: the filter must be shorter than half x.
  if (!(hl < xl / 2) || hl == 0)
    vs::fatal("overlap-save requires 0 < hLength < xLength / 2 (x=%zu h=%zu)", xl, hl);
  ConvolutionOverlapSaveHandle h;
  std::memset(&h, 0, sizeof(h));
  ConvPlan *p = make_plan(VS_CONV_OVERLAP_SAVE, xl, hl);
  h.fft_plan = p;
  h.fft_inverse_plan = p;
  h.x_length = xl;
  h.h_length = hl;
  h.L = static_cast<int *>(std::malloc(sizeof(int)));
  *h.L = p->block;
  h.reverse = reverse;
  return h;
}

void os_fini(ConvolutionOverlapSaveHandle h) {
  std::free(h.fft_plan);
  std::free(h.L);
}

ConvolutionHandle auto_init(size_t xl, size_t hl, int reverse) {
  ConvolutionHandle h;
  std::memset(&h, 0, sizeof(h));
  h.x_length = static_cast<int>(std::min<size_t>(xl, INT_MAX));
  h.h_length = checked_int("convolve_initialize", hl);
  int algo;
  if (vs::gpu_available()) {
    algo = vs_conv1d_select(static_cast<int64_t>(xl), h.h_length, 1);
    if (algo == VS_CONV_OVERLAP_SAVE && !(hl < xl / 2)) algo = VS_CONV_FFT;
    // the brute-force handle has only the int length fields: longer signals
    // take a handle with a plan
    if (algo == VS_CONV_DIRECT && xl > static_cast<size_t>(INT_MAX)) algo = VS_CONV_OVERLAP_SAVE;
  } else {
    // reference heuristic (src/convolve.c:349-363)
    if (xl > hl * 2)
      algo = xl > 200 ? VS_CONV_OVERLAP_SAVE : VS_CONV_DIRECT;
    else
      algo = xl > 350 ? VS_CONV_FFT : VS_CONV_DIRECT;
  }
  vs::log(1, "convolve_initialize(x=%zu, h=%zu): algorithm %d", xl, hl, algo);
  switch (algo) {
    case VS_CONV_OVERLAP_SAVE:
      h.algorithm = kConvolutionAlgorithmOverlapSave;
      h.handle.os = os_init(xl, hl, reverse);
      break;
    case VS_CONV_FFT:
      h.algorithm = kConvolutionAlgorithmFFT;
      h.handle.fft = fft_init(xl, hl, reverse);
      break;
    default:
      h.algorithm = kConvolutionAlgorithmBruteForce;
      break;
  }
  return h;
}

void direct(const char *what, int simd, int reverse, const float *x, size_t xl,
            const float *h, size_t hl, float *result) {
  if (!x || !h || !result || !xl || !hl) vs::fatal("%s: invalid arguments", what);
  const bool tiny = xl * hl < host_max_macs() && !vs::api::any_device({x, h, result});
  if (!tiny && vs::api::use_gpu_simd(simd, what)) {
    gpu_conv(what, VS_CONV_DIRECT, reverse, x, xl, h, hl, result);
  } else if (simd == 0) {  // the scalar reference
    if (reverse) vs::ref::correlate_direct(x, xl, h, hl, result);
    else vs::ref::convolve_direct(x, xl, h, hl, result);
  } else if (reverse) {    // tiny or no GPU: vectorised host loops
    vs::host::correlate_direct(x, xl, h, hl, result);
  } else {
    vs::host::convolve_direct(x, xl, h, hl, result);
  }
}

void auto_run(ConvolutionHandle handle, const float *x, const float *h,
              float *result, int reverse) {
  switch (handle.algorithm) {
    case kConvolutionAlgorithmFFT:
      run_plan("convolve_fft", static_cast<ConvPlan *>(handle.handle.fft.fft_plan),
               handle.handle.fft.reverse, x, h, result);
      break;
    case kConvolutionAlgorithmOverlapSave:
      run_plan("convolve_overlap_save",
               static_cast<ConvPlan *>(handle.handle.os.fft_plan),
               handle.handle.os.reverse, x, h, result);
      break;
    case kConvolutionAlgorithmBruteForce:
      direct(reverse ? "cross_correlate" : "convolve", 1, reverse, x,
             handle.x_length, h, handle.h_length, result);
      break;
  }
}

void auto_fini(ConvolutionHandle handle) {
  switch (handle.algorithm) {
    case kConvolutionAlgorithmFFT:
      fft_fini(handle.handle.fft);
      break;
    case kConvolutionAlgorithmOverlapSave:
      os_fini(handle.handle.os);
      break;
    case kConvolutionAlgorithmBruteForce:
      break;
  }
}

}  // namespace

extern "C" {

/* ------------------------------------------------------------ convolve */
ConvolutionFFTHandle convolve_fft_initialize(size_t xl, size_t hl) {
  return fft_init(xl, hl, 0);
}
void convolve_fft(ConvolutionFFTHandle handle, const float *x, const float *h,
                  float *result) {
  run_plan("convolve_fft", static_cast<ConvPlan *>(handle.fft_plan), handle.reverse,
           x, h, result);
}
void convolve_fft_finalize(ConvolutionFFTHandle handle) { fft_fini(handle); }

ConvolutionOverlapSaveHandle convolve_overlap_save_initialize(size_t xl,
                                                              size_t hl) {
  return os_init(xl, hl, 0);
}
void convolve_overlap_save(ConvolutionOverlapSaveHandle handle, const float *x,
                           const float *h, float *result) {
  run_plan("convolve_overlap_save", static_cast<ConvPlan *>(handle.fft_plan),
           handle.reverse, x, h, result);
}
void convolve_overlap_save_finalize(ConvolutionOverlapSaveHandle handle) {
  os_fini(handle);
}

void convolve_simd(int simd, const float *x, size_t xl, const float *h,
                   size_t hl, float *result) {
  direct("convolve_simd", simd, 0, x, xl, h, hl, result);
}

ConvolutionHandle convolve_initialize(size_t xl, size_t hl) {
  return auto_init(xl, hl, 0);
}
void convolve(ConvolutionHandle handle, const float *x, const float *h,
              float *result) {
  auto_run(handle, x, h, result, 0);
}
void convolve_finalize(ConvolutionHandle handle) { auto_fini(handle); }

/* ----------------------------------------------------------- correlate */
CrossCorrelationFFTHandle cross_correlate_fft_initialize(size_t xl, size_t hl) {
  return fft_init(xl, hl, 1);
}
void cross_correlate_fft(CrossCorrelationFFTHandle handle, const float *x,
                         const float *h, float *result) {
  convolve_fft(handle, x, h, result);
}
void cross_correlate_fft_finalize(CrossCorrelationFFTHandle handle) {
  fft_fini(handle);
}

CrossCorrelationOverlapSaveHandle cross_correlate_overlap_save_initialize(
    size_t xl, size_t hl) {
  return os_init(xl, hl, 1);
}
void cross_correlate_overlap_save(CrossCorrelationOverlapSaveHandle handle,
                                  const float *x, const float *h,
                                  float *result) {
  convolve_overlap_save(handle, x, h, result);
}
void cross_correlate_overlap_save_finalize(
    CrossCorrelationOverlapSaveHandle handle) {
  os_fini(handle);
}

void cross_correlate_simd(int simd, const float *x, size_t xl, const float *h,
                          size_t hl, float *result) {
  direct("cross_correlate_simd", simd, 1, x, xl, h, hl, result);
}

CrossCorrelationHandle cross_correlate_initialize(size_t xl, size_t hl) {
  return auto_init(xl, hl, 1);
}
void cross_correlate(CrossCorrelationHandle handle, const float *x,
                     const float *h, float *result) {
  auto_run(handle, x, h, result, 1);
}
void cross_correlate_finalize(CrossCorrelationHandle handle) {
  auto_fini(handle);
}

}  // extern "C"
