// Probe: LDS layout written by buffer_load_dword{,x4} ... lds vs
// global_load_lds_dwordx4 (one wave, lane-linear source), and the M0 base.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;

__global__ void probe(const float *src, float *out, int mode) {
  __shared__ __attribute__((aligned(1024))) float s[2048];
  for (int i = threadIdx.x; i < 2048; i += 64) s[i] = -1.f;
  __syncthreads();
  auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(src), 0, 0x7fffffff, 0x00020000);
  const int lane = threadIdx.x;
#if defined(__HIP_DEVICE_COMPILE__)
  if (mode == 0)
    __builtin_amdgcn_global_load_lds((glob_void_t *)(src + 4 * lane), (lds_void_t *)(s + 256), 16, 0, 0);
  else if (mode == 1)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t *)(s + 256), 16, 16 * lane, 0, 0, 0);
  else if (mode == 2)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t *)(s + 256), 4, 4 * lane, 0, 0, 0);
  else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t *)(s + 256), 16,
                                             lane < 32 ? 16 * lane : 0x80000000u, 0, 0, 0);
#endif
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 64) out[i] = s[i];
}

int main() {
  float *src, *out;
  hipMalloc(&src, 4096 * 4);
  hipMalloc(&out, 2048 * 4);
  float h[4096];
  for (int i = 0; i < 4096; i++) h[i] = i;
  hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  for (int mode = 0; mode < 4; mode++) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out, mode);
    float o[2048];
    hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
    printf("mode %d: s[250..262]:", mode);
    for (int i = 250; i < 262; i++) printf(" %g", o[i]);
    printf(" | s[256+252..256+260]:");
    for (int i = 256 + 252; i < 256 + 260; i++) printf(" %g", o[i]);
    int first = -1, last = -1;
    for (int i = 0; i < 2048; i++)
      if (o[i] != -1.f) { if (first < 0) first = i; last = i; }
    printf(" | written [%d, %d]\n", first, last);
  }
  return 0;
}
