// normalize.h (reference src/normalize.c:445-521).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/normalize.h"

#include "csrc/api/dispatch.h"
#include "csrc/ref/ref.h"
#include "simd/gpu.h"

using vs::Staged;

namespace {
// Host planes / arrays stay on the host even with simd = 1: one or two passes
// over the data cost less than its copy into pinned memory for the GPU
// (normalize2D 2048 x 2048: 0.6 ms on the host, 1.8 ms through the GPU).
constexpr size_t kSmallElems = vs::api::kHostAlways;
bool small(int w, int h, std::initializer_list<const void *> ptrs) {
  return vs::api::host_small(static_cast<size_t>(w) * h, kSmallElems, ptrs);
}

size_t plane_bytes(int stride, int w, int h, size_t elem) {
  return (static_cast<size_t>(h - 1) * stride + w) * elem;
}
}  // namespace

extern "C" {

void minmax2D(int simd, const uint8_t *src, int stride, int w, int h,
              uint8_t *mn, uint8_t *mx) {
  if (!src || w <= 0 || h <= 0 || stride < w)
    vs::fatal("minmax2D: invalid arguments");
  if (!mn && !mx) return;
  if (!vs::api::use_gpu_simd(simd, "minmax2D") || small(w, h, {src})) {
    vs::ref::minmax2d(src, stride, w, h, mn, mx);
    return;
  }
  uint8_t out[2] = {0, 0};
  vs::api::run_sync("minmax2D", [&](hipStream_t s) {
    Staged x(src, plane_bytes(stride, w, h, 1), Staged::kIn, s);
    Staged o(out, 2, Staged::kOut, s);
    VS_TRY(x.status());
    VS_TRY(o.status());
    VS_TRY(vs_minmax2d_u8(x.dev<uint8_t>(), stride, w, h, o.dev<uint8_t>(), s));
    return o.finish();
  });
  if (mn) *mn = out[0];
  if (mx) *mx = out[1];
}

void normalize2D_minmax(int simd, uint8_t mn, uint8_t mx, const uint8_t *src,
                        int sstride, int w, int h, float *dst, int dstride) {
  if (!src || !dst || w <= 0 || h <= 0 || sstride < w || dstride < w || mn > mx)
    vs::fatal("normalize2D_minmax: invalid arguments");
  if (!vs::api::use_gpu_simd(simd, "normalize2D_minmax") || small(w, h, {src, dst})) {
    vs::ref::normalize2d_minmax(mn, mx, src, sstride, w, h, dst, dstride);
    return;
  }
  vs::api::run_sync("normalize2D_minmax", [&](hipStream_t s) {
    // kInOut keeps the row padding of dst untouched.
    Staged o(dst, plane_bytes(dstride, w, h, 4), Staged::kInOut, s);
    Staged x(src, plane_bytes(sstride, w, h, 1), Staged::kIn, s);
    VS_TRY(o.status());
    VS_TRY(x.status());
    VS_TRY(vs_normalize2d_u8(x.dev<uint8_t>(), sstride, w, h, nullptr, mn, mx,
                             o.dev<float>(), dstride, s));
    return o.finish();
  });
}

void normalize2D(int simd, const uint8_t *src, int sstride, int w, int h,
                 float *dst, int dstride) {
  if (!src || !dst || w <= 0 || h <= 0 || sstride < w || dstride < w)
    vs::fatal("normalize2D: invalid arguments");
  if (!vs::api::use_gpu_simd(simd, "normalize2D") || small(w, h, {src, dst})) {
    uint8_t mn, mx;
    vs::ref::minmax2d(src, sstride, w, h, &mn, &mx);
    vs::ref::normalize2d_minmax(mn, mx, src, sstride, w, h, dst, dstride);
    return;
  }
  // Fused on the device: the min/max never leave the GPU.
  vs::api::run_sync("normalize2D", [&](hipStream_t s) {
    Staged o(dst, plane_bytes(dstride, w, h, 4), Staged::kInOut, s);
    Staged x(src, plane_bytes(sstride, w, h, 1), Staged::kIn, s);
    vs::DeviceBuffer mm;
    VS_TRY(o.status());
    VS_TRY(x.status());
    VS_TRY(mm.alloc(2, s));
    VS_TRY(vs_minmax2d_u8(x.dev<uint8_t>(), sstride, w, h, mm.as<uint8_t>(), s));
    VS_TRY(vs_normalize2d_u8(x.dev<uint8_t>(), sstride, w, h, mm.as<uint8_t>(),
                             0, 0, o.dev<float>(), dstride, s));
    return o.finish();
  });
}

void minmax1D(int simd, const float *src, int n, float *mn, float *mx) {
  if (!src || n <= 0) vs::fatal("minmax1D: invalid arguments");
  if (!mn && !mx) return;
  if (!vs::api::use_gpu_simd(simd, "minmax1D") || small(n, 1, {src})) {
    if (simd) vs::host::minmax1d(src, static_cast<size_t>(n), mn, mx);
    else vs::ref::minmax1d(src, n, mn, mx);
    return;
  }
  float out[2] = {0.f, 0.f};
  vs::api::run_sync("minmax1D", [&](hipStream_t s) {
    Staged x(src, static_cast<size_t>(n) * 4, Staged::kIn, s);
    Staged o(out, 8, Staged::kOut, s);
    VS_TRY(x.status());
    VS_TRY(o.status());
    VS_TRY(vs_minmax(x.dev<float>(), n, o.dev<float>(), s));
    return o.finish();
  });
  if (mn) *mn = out[0];
  if (mx) *mx = out[1];
}

}  // extern "C"
