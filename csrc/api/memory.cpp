// memory.h (reference src/memory.c).  Copyright 2026 veles.simd_amd authors.
// Apache-2.0.
#include "simd/memory.h"

#include <cassert>
#include <cstdlib>
#include <cstring>

#include "csrc/api/dispatch.h"
#include "simd/gpu.h"

namespace {
int align_offset(const void *ptr) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
  return (a & 31) ? static_cast<int>(32 - (a % 32)) : 0;
}
}  // namespace

extern "C" {

int align_complement_f32(const float *p) { return align_offset(p) / 4; }
int align_complement_i16(const int16_t *p) { return align_offset(p) / 2; }
int align_complement_u16(const uint16_t *p) { return align_offset(p) / 2; }
int align_complement_i32(const int32_t *p) { return align_offset(p) / 4; }
int align_complement_u32(const uint32_t *p) { return align_offset(p) / 4; }

void *malloc_aligned(size_t size) {
  void *p = nullptr;
  if (posix_memalign(&p, 64, size ? size : 64) != 0) return nullptr;
  return p;
}

void *malloc_aligned_offset(size_t size, int offset) {
  assert(offset >= 0 && offset < 32);
  char *p = static_cast<char *>(malloc_aligned(size + offset));
  return p ? p + offset : nullptr;
}

float *mallocf(size_t length) {
  return static_cast<float *>(malloc_aligned(length * sizeof(float)));
}

void memsetf(float *ptr, float value, size_t length) {
  if (vs::is_device_pointer(ptr)) {
    vs::api::run_sync("memsetf", [&](hipStream_t s) {
      return vs_fill(ptr, value, length, s);
    });
    return;
  }
  for (size_t i = 0; i < length; i++) ptr[i] = value;
}

float *zeropaddingex(const float *ptr, size_t length, size_t *newLength,
                     size_t additionalLength) {
  // 2^(floor(log2 length) + 2): e.g. 100 -> 256, 128 -> 512
  // (reference src/memory.c:129-137).
  size_t nl = length;
  int lg = 2;
  while (nl >>= 1) lg++;
  nl = static_cast<size_t>(1) << lg;
  *newLength = nl;
  float *ret = mallocf(nl + additionalLength);
  if (!ret) return nullptr;
  std::memcpy(ret, ptr, length * sizeof(float));
  memsetf(ret + length, 0.f, nl - length);
  return ret;
}

float *zeropadding(const float *ptr, size_t length, size_t *newLength) {
  return zeropaddingex(ptr, length, newLength, 0);
}

float *rmemcpyf(float *__restrict dest, const float *__restrict src,
                size_t length) {
  if (vs::api::any_device({dest, src})) {
    vs::api::run_sync("rmemcpyf", [&](hipStream_t s) {
      vs::Staged d(dest, length * 4, vs::Staged::kOut, s);
      vs::Staged x(src, length * 4, vs::Staged::kIn, s);
      VS_TRY(d.status());
      VS_TRY(x.status());
      VS_TRY(vs_reverse(x.dev<float>(), d.dev<float>(), length, 0, s));
      return d.finish();
    });
    return dest;
  }
  for (size_t i = 0; i < length; i++) dest[i] = src[length - 1 - i];
  return dest;
}

float *crmemcpyf(float *__restrict dest, const float *__restrict src,
                 size_t length) {
  if (vs::api::any_device({dest, src})) {
    vs::api::run_sync("crmemcpyf", [&](hipStream_t s) {
      vs::Staged d(dest, length * 4, vs::Staged::kOut, s);
      vs::Staged x(src, length * 4, vs::Staged::kIn, s);
      VS_TRY(d.status());
      VS_TRY(x.status());
      VS_TRY(vs_reverse(x.dev<float>(), d.dev<float>(), length, 1, s));
      return d.finish();
    });
    return dest;
  }
  for (size_t i = 0; i + 1 < length; i += 2) {
    dest[i] = src[length - i - 2];
    dest[i + 1] = src[length - i - 1];
  }
  return dest;
}

}  // extern "C"
