// Memory-pattern ceiling of the fused SWT kernel: the same grid, loads and
// stores (one 4 KB input row read, `levels` 4 KB hi rows and one lo row
// written per signal, non-temporal float4 stores, two signals per
// workgroup), no LDS, no arithmetic, no barriers.  Prints TB/s of the
// bytes the SWT benchmark counts.
// hipcc -O3 --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops \
//   bench/probes/swt_write_pattern.hip -o build/bench/swt_write_pattern
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float native4 __attribute__((ext_vector_type(4)));

// MODE 0: as the SWT kernel.  1: no input read.  2: workgroups walk the
// signals in a grid-stride loop (2048 workgroups).  3: one signal per
// workgroup.  4: lo row stored next to the hi rows (9 contiguous rows).
template <int MODE, int PER = 2, bool NTLOAD = false>
__global__ __launch_bounds__(256) void pattern2(const float *__restrict__ src, float *__restrict__ hi,
                                                float *__restrict__ lo, int levels, int len,
                                                long long batch) {
  const int q = threadIdx.x;
  const int per = MODE == 3 ? 1 : PER;
  for (long long s0 = (long long)blockIdx.x * per; s0 < batch;
       s0 += (MODE == 2 ? (long long)gridDim.x * per : batch)) {
    for (int g = 0; g < per; g++) {
      const long long sig = s0 + g;
      if (sig >= batch) return;
      native4 nv = {1.f, 2.f, 3.f, 4.f};
      if (MODE != 1) {
        if (NTLOAD) {
          nv = __builtin_nontemporal_load(reinterpret_cast<const native4 *>(src + sig * len) + q);
        } else {
          const float4 v = reinterpret_cast<const float4 *>(src + sig * len)[q];
          nv = native4{v.x, v.y, v.z, v.w};
        }
      }
      const long long rows = MODE == 4 ? levels + 1 : levels;
      for (int l = 0; l < levels; l++) {
        __builtin_nontemporal_store(nv, reinterpret_cast<native4 *>(hi + (sig * rows + l) * len) + q);
        nv.x += 1.f;
      }
      if (MODE == 4)
        __builtin_nontemporal_store(nv, reinterpret_cast<native4 *>(hi + (sig * rows + levels) * len) + q);
      else
        reinterpret_cast<native4 *>(lo + sig * len)[q] = nv;
    }
  }
}

template <bool NT, bool LEVEL_SPREAD>
__global__ __launch_bounds__(256) void pattern(const float *__restrict__ src, float *__restrict__ hi,
                                               float *__restrict__ lo, int levels, int len,
                                               long long batch) {
  const int q = threadIdx.x;
  for (int g = 0; g < 2; g++) {
    const long long sig = 2LL * blockIdx.x + g;
    if (sig >= batch) return;
    const float4 v = reinterpret_cast<const float4 *>(src + sig * len)[q];
    native4 nv = {v.x, v.y, v.z, v.w};
    for (int l = 0; l < levels; l++) {
      if (LEVEL_SPREAD) __builtin_amdgcn_s_sleep(20);  // stores spread over the workgroup's life
      native4 *row = reinterpret_cast<native4 *>(hi + (sig * levels + l) * len) + q;
      if (NT) __builtin_nontemporal_store(nv, row);
      else *row = nv;
      nv.x += 1.f;
    }
    reinterpret_cast<native4 *>(lo + sig * len)[q] = nv;
  }
}

int main() {
  const long long batch = 65536;
  const int len = 1024, levels = 8;
  float *src, *hi, *lo;
  hipMalloc(&src, batch * len * 4);
  hipMalloc(&hi, batch * len * 4 * (levels + 1));
  hipMalloc(&lo, batch * len * 4);
  hipMemset(src, 0, batch * len * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = 4.0 * batch * len * (levels + 2);
  for (int arm = 0; arm < 4; arm++) {
    auto launch = [&] {
      const dim3 grid(batch / 2), block(256);
      switch (arm) {
        case 0: hipLaunchKernelGGL((pattern<true, false>), grid, block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 1: hipLaunchKernelGGL((pattern<false, false>), grid, block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 2: hipLaunchKernelGGL((pattern<true, true>), grid, block, 0, 0, src, hi, lo, levels, len, batch); break;
        default: hipLaunchKernelGGL((pattern<false, true>), grid, block, 0, 0, src, hi, lo, levels, len, batch); break;
      }
    };
    for (int i = 0; i < 20; i++) launch();
    hipDeviceSynchronize();
    float best = 1e9f;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(e0);
      for (int i = 0; i < 10; i++) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms / 10 < best) best = ms / 10;
    }
    printf("%s stores%s: %.3f ms, %.2f TB/s\n", arm % 2 == 0 ? "non-temporal" : "plain",
           arm >= 2 ? ", spread by s_sleep" : "", best, bytes / best / 1e9);
  }
  const char *names[] = {"as the SWT kernel", "no input read", "grid-stride over signals, 2048 workgroups",
                         "one signal per workgroup", "lo next to the hi rows",
                         "4 signals per workgroup", "8 signals per workgroup",
                         "4 signals per workgroup, lo next to hi", "non-temporal input load",
                         "non-temporal input load, lo next to hi"};
  for (int mode = 0; mode < 10; mode++) {
    auto launch = [&] {
      const dim3 block(256);
      switch (mode) {
        case 0: hipLaunchKernelGGL(pattern2<0>, dim3(batch / 2), block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 1: hipLaunchKernelGGL(pattern2<1>, dim3(batch / 2), block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 2: hipLaunchKernelGGL(pattern2<2>, dim3(2048), block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 3: hipLaunchKernelGGL(pattern2<3>, dim3(batch), block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 4: hipLaunchKernelGGL(pattern2<4>, dim3(batch / 2), block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 5: hipLaunchKernelGGL((pattern2<0, 4>), dim3(batch / 4), block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 6: hipLaunchKernelGGL((pattern2<0, 8>), dim3(batch / 8), block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 7: hipLaunchKernelGGL((pattern2<4, 4>), dim3(batch / 4), block, 0, 0, src, hi, lo, levels, len, batch); break;
        case 8: hipLaunchKernelGGL((pattern2<0, 2, true>), dim3(batch / 2), block, 0, 0, src, hi, lo, levels, len, batch); break;
        default: hipLaunchKernelGGL((pattern2<4, 2, true>), dim3(batch / 2), block, 0, 0, src, hi, lo, levels, len, batch); break;
      }
    };
    for (int i = 0; i < 20; i++) launch();
    hipDeviceSynchronize();
    float best = 1e9f;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(e0);
      for (int i = 0; i < 10; i++) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms / 10 < best) best = ms / 10;
    }
    printf("%s: %.3f ms, %.2f TB/s\n", names[mode], best, bytes / best / 1e9);
  }
  return 0;
}
