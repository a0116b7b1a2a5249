// LDS-resident Stockham FFT building blocks for CDNA4.
//
// One signal of N = 2^LOGN complex points (N <= 16384) lives in LDS
// (float2, XOR-swizzled within 16-element rows -- see lds_slot -- so the
// power-of-two strides of the exchanges hit distinct banks) while TPS = N/E threads each own E = 16 (32 at
// N = 16384) points in registers.  Each pass is a radix-R Stockham step (R in {2,4,8,16}):
//   butterfly i in [0, N/R), k = i mod P (P = product of earlier radices):
//     u_j = x[i + j N/R] * w^(j k),  w = exp(-+2 pi i / (P R))
//     v   = DFT_R(u)
//     y[(i - k) R + k + j P] = v_j
// so the output is in natural order without a bit-reversal pass.  Inputs of
// the first pass and outputs of the last pass are both "i + j N/R" with
// consecutive i on consecutive lanes, i.e. coalesced global loads/stores, and
// the last forward pass leaves in registers exactly the elements the first
// pass of a reversed-radix inverse transform needs -- the fused convolution
// kernels multiply by the filter spectrum in registers and start the inverse
// FFT without an LDS round trip.
//
// Twiddles come from a per-size table exp(-2 pi i m / N), m < N, computed in
// double precision on the host (csrc/kernels/fft_plan.h).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

namespace vs {
namespace fft {

// Complex helpers written as 2-lane vector arithmetic with lane shuffles so
// each maps onto one or two v_pk_*_f32 with op_sel / neg modifiers (no
// register-pair shuffling between packed and scalar halves).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v to_v(float2 a) { return f2v{a.x, a.y}; }
__device__ __forceinline__ float2 from_v(f2v a) { return make_float2(a.x, a.y); }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return from_v(to_v(a) + to_v(b)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return from_v(to_v(a) - to_v(b)); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  const f2v av = to_v(a), bv = to_v(b);
  return from_v(av.xx * bv + av.yy * (bv.yx * f2v{-1.f, 1.f}));
}
// a * conj(b)
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {
  const f2v av = to_v(a), bv = to_v(b);
  return from_v(av * bv.xx + av.yx * (bv.yy * f2v{1.f, -1.f}));
}
// z * (-i) forward, z * (+i) inverse
template <bool INV>
__device__ __forceinline__ float2 rot90(float2 z) {
  const f2v v = to_v(z).yx;
  return from_v(INV ? v * f2v{-1.f, 1.f} : v * f2v{1.f, -1.f});
}

template <bool INV>
__device__ __forceinline__ void dft2(float2 *v) {
  const float2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}

template <bool INV>
__device__ __forceinline__ void dft4(float2 &a0, float2 &a1, float2 &a2,
                                     float2 &a3) {
  const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
  const float2 t2 = cadd(a1, a3), t3 = rot90<INV>(csub(a1, a3));
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  a1 = cadd(t1, t3);
  a3 = csub(t1, t3);
}

template <bool INV>
__device__ __forceinline__ void dft4(float2 *v) {
  dft4<INV>(v[0], v[1], v[2], v[3]);
}

constexpr float kC8 = 0.70710678118654752440f;   // cos(pi/4)
constexpr float kC16 = 0.92387953251128675613f;  // cos(pi/8)
constexpr float kS16 = 0.38268343236508977173f;  // sin(pi/8)

// z * exp(-+ i pi/4) and z * exp(-+ 3 i pi/4): kC8 (z +- rot90(z))
template <bool INV>
__device__ __forceinline__ float2 w8_1(float2 z) {
  const f2v v = to_v(z), r = to_v(rot90<INV>(z));
  return from_v((v + r) * kC8);
}
template <bool INV>
__device__ __forceinline__ float2 w8_3(float2 z) {
  const f2v v = to_v(z), r = to_v(rot90<INV>(z));
  return from_v((r - v) * kC8);
}

template <bool INV>
__device__ __forceinline__ void dft8(float2 *v) {
  float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
  float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
  dft4<INV>(e0, e1, e2, e3);
  dft4<INV>(o0, o1, o2, o3);
  o1 = w8_1<INV>(o1);
  o2 = rot90<INV>(o2);
  o3 = w8_3<INV>(o3);
  v[0] = cadd(e0, o0);
  v[4] = csub(e0, o0);
  v[1] = cadd(e1, o1);
  v[5] = csub(e1, o1);
  v[2] = cadd(e2, o2);
  v[6] = csub(e2, o2);
  v[3] = cadd(e3, o3);
  v[7] = csub(e3, o3);
}

template <bool INV>
__device__ __forceinline__ void dft16(float2 *v) {
  float2 e[8], o[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    e[j] = v[2 * j];
    o[j] = v[2 * j + 1];
  }
  dft8<INV>(e);
  dft8<INV>(o);
  // o[k] *= exp(-+ 2 pi i k / 16)
  const float sg = INV ? 1.f : -1.f;
  o[1] = cmul(o[1], make_float2(kC16, sg * kS16));
  o[2] = w8_1<INV>(o[2]);
  o[3] = cmul(o[3], make_float2(kS16, sg * kC16));
  o[4] = rot90<INV>(o[4]);
  o[5] = cmul(o[5], make_float2(-kS16, sg * kC16));
  o[6] = w8_3<INV>(o[6]);
  o[7] = cmul(o[7], make_float2(-kC16, sg * kS16));
#pragma unroll
  for (int k = 0; k < 8; k++) {
    v[k] = cadd(e[k], o[k]);
    v[k + 8] = csub(e[k], o[k]);
  }
}

// cos / sin of pi k / 16, k = 0..15 (the 32-point twiddles)
constexpr float kC32[16] = {1.0f, 0.98078528040323044913f, 0.92387953251128675613f,
                            0.83146961230254523708f, 0.70710678118654752440f,
                            0.55557023301960222474f, 0.38268343236508977173f,
                            0.19509032201612826785f, 0.0f, -0.19509032201612826785f,
                            -0.38268343236508977173f, -0.55557023301960222474f,
                            -0.70710678118654752440f, -0.83146961230254523708f,
                            -0.92387953251128675613f, -0.98078528040323044913f};
constexpr float kS32[16] = {0.0f, 0.19509032201612826785f, 0.38268343236508977173f,
                            0.55557023301960222474f, 0.70710678118654752440f,
                            0.83146961230254523708f, 0.92387953251128675613f,
                            0.98078528040323044913f, 1.0f, 0.98078528040323044913f,
                            0.92387953251128675613f, 0.83146961230254523708f,
                            0.70710678118654752440f, 0.55557023301960222474f,
                            0.38268343236508977173f, 0.19509032201612826785f};

// 32-point DFT: two 16-point DFTs (even / odd samples) and one twiddled
// butterfly stage.
template <bool INV>
__device__ __forceinline__ void dft32(float2 *v) {
  float2 e[16], o[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    e[j] = v[2 * j];
    o[j] = v[2 * j + 1];
  }
  dft16<INV>(e);
  dft16<INV>(o);
  const float sg = INV ? 1.f : -1.f;
#pragma unroll
  for (int k = 1; k < 16; k++) {
    if (k == 4) o[k] = w8_1<INV>(o[k]);
    else if (k == 8) o[k] = rot90<INV>(o[k]);
    else if (k == 12) o[k] = w8_3<INV>(o[k]);
    else o[k] = cmul(o[k], make_float2(kC32[k], sg * kS32[k]));
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {
    v[k] = cadd(e[k], o[k]);
    v[k + 16] = csub(e[k], o[k]);
  }
}

template <int R, bool INV>
__device__ __forceinline__ void dft(float2 *v) {
  if constexpr (R == 2) dft2<INV>(v);
  else if constexpr (R == 4) dft4<INV>(v);
  else if constexpr (R == 8) dft8<INV>(v);
  else if constexpr (R == 16) dft16<INV>(v);
  else dft32<INV>(v);
}

// LDS slot of complex element e: bits 0-3 XORed with bits 4-7 ^ 8-11, a
// bijection on every 16-aligned block (no padding).  The exchanges move
// float2 with ds_write_b64 (lane groups of 16, bank = slot mod 16 pairs)
// and ds_read_b64 (groups of 32, bank = slot mod 32 pairs;
// MI355X_MICROARCH.md §LDS).  Reads take 32 consecutive aligned e: the XOR
// permutes within each 16-half and bit 4 keeps the halves apart -> 32
// distinct.  Writes e = (i - k) R + k + j P over 16 consecutive lanes i:
// P >= 16 gives 16 consecutive k with bits >= 4 fixed; P = 1 gives stride R,
// whose lane bits land in e's bits 4-7 (R = 16), or bits 5-8 (R = 32, the
// e >> 8 term separates lanes i and i + 8), or are split between bits 0-3
// and 4-7 (R <= 8): all 16 distinct.  The previous "one pad slot per 16"
// layout put slots 0 and 32 of every 32-element read in one bank (2-way
// conflicts on every read) and 2-way on the radix-32 P = 1 writes.
__device__ __forceinline__ int lds_slot(int e) { return e ^ (((e >> 4) ^ (e >> 8)) & 15); }

// Workgroup barrier that orders LDS only.  __syncthreads() is a full
// workgroup fence: every wave drains vmcnt at every LDS exchange, i.e. waits
// for its prefetches and for the stores of earlier outputs.  The passes only
// exchange data through LDS.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

constexpr int ilog2c(int r) {
  int l = 0;
  while ((1 << l) < r) l++;
  return l;
}

// Twiddle sources for Pass::run.  TableTw reads the per-size table at every
// pass; RegTw holds every twiddle one thread needs for a whole transform in
// registers, loaded once -- a persistent kernel keeps them across its loop,
// so its transforms issue no global loads at all.
struct TableTw {
  const float2 *__restrict__ tw;
  template <class PL, bool REV, int Q>
  __device__ __forceinline__ float2 get(int, int, int idx) const { return tw[idx]; }
};

template <class PL, bool REV>
struct RegTw {
  static constexpr int R(int q) { return REV ? PL::radix_rev(q) : PL::radix(q); }
  // first slot of pass q (pass 0 has no twiddles)
  static constexpr int offset(int q) {
    int o = 0;
    for (int i = 1; i < q; i++) o += (PL::E / R(i)) * ilog2c(R(i));
    return o;
  }
  static constexpr int kCount = offset(PL::NPASS) > 0 ? offset(PL::NPASS) : 1;
  float2 w[kCount];

  template <int Q = 1>
  __device__ __forceinline__ void load(int t, const float2 *__restrict__ tw) {
    if constexpr (Q < PL::NPASS) {
      constexpr int RQ = R(Q), P = PL::stride(Q, REV), S = PL::N / (P * RQ);
      constexpr int LR = ilog2c(RQ);
#pragma unroll
      for (int b = 0; b < PL::E / RQ; b++) {
        const int k = (t + b * PL::TPS) & (P - 1);
#pragma unroll
        for (int q = 0; q < LR; q++) w[offset(Q) + b * LR + q] = tw[(1 << q) * k * S];
      }
      load<Q + 1>(t, tw);
    }
  }
  template <class PL2, bool REV2, int Q>
  __device__ __forceinline__ float2 get(int b, int q, int) const {
    static_assert(REV2 == REV, "twiddle set built for the other radix order");
    return w[offset(Q) + b * ilog2c(R(Q)) + q];
  }
};

// Compile-time pass plan for N = 2^LOGN.  EP = points per thread: 0 picks
// the default (16, or 32 at N = 16384 so the 512-thread workgroup keeps its
// working set in registers -- at 1024 threads the 128-VGPR budget of 4
// waves/SIMD spilled); 32 runs radix-32 passes after one smaller first pass
// (N = 16384: 16 x 32 x 32, N = 8192: 8 x 32 x 32) -- one butterfly of 32
// per thread and a third fewer LDS round trips and barriers than radix 16.
template <int LOGN_, int EP = 0>
struct Plan {
  static constexpr int LOGN = LOGN_;
  static constexpr int N = 1 << LOGN;
  static constexpr int E = EP ? EP : (LOGN >= 14 ? 32 : (LOGN >= 4 ? 16 : N));
  static_assert(E <= N && (E == 32 ? LOGN >= 6 : true), "plan: too few points");
  static constexpr int TPS = N / E;                // threads per signal
  static constexpr int SMALL = LOGN >= 4 ? LOGN % 4 : 0;
  static constexpr bool R32 = E == 32;
  static constexpr int NPASS =
      R32 ? (LOGN + 4) / 5 : (LOGN >= 4 ? LOGN / 4 + (SMALL ? 1 : 0) : 1);
  // LDS layout of the exchanges.  32-point plans pad one element per 32
  // (slot e + e / 32): every element a thread exchanges then sits at its
  // base slot plus a compile-time offset (ds_read / ds_write immediates, no
  // per-access address VALU -- the XOR swizzle cost ~1000 of the 3787 VALU
  // instructions per wave of the M = 8192 conv kernel) and every pass pattern
  // stays bank-conflict-free.  Other plans keep the XOR swizzle (lds_slot).
  // 16-point plans of >= 1024 points pad one element per 16 (the pass
  // patterns of radix-16 butterflies stay conflict-free at that period).
  static constexpr int PADLOG = E == 32 ? 5 : (E == 16 && LOGN >= 10 ? 4 : 0);
  static constexpr bool PAD = PADLOG != 0;
  // per-signal LDS (float2).  Signals narrower than a 32-lane read group
  // (TPS < 32, several per wave) are TPS slots apart so their aligned
  // TPS-slot read blocks land in different banks.
  static constexpr int kLds = PAD ? N + (N >> PADLOG) : N + (TPS < 32 ? TPS : 0);
  // Radix of pass q (forward order: the odd radix first).
  static constexpr int radix(int q) {
    if (R32) return q == 0 ? (1 << (LOGN - 5 * (NPASS - 1))) : 32;
    return LOGN < 4 ? N : ((SMALL && q == 0) ? (1 << SMALL) : 16);
  }
  static constexpr int radix_rev(int q) { return radix(NPASS - 1 - q); }
  static constexpr int stride(int q, bool rev) {
    int p = 1;
    for (int i = 0; i < q; i++) p *= rev ? radix_rev(i) : radix(i);
    return p;
  }
  static constexpr int first_radix(bool rev) { return rev ? radix_rev(0) : radix(0); }
  static constexpr int last_radix(bool rev) {
    return rev ? radix_rev(NPASS - 1) : radix(NPASS - 1);
  }
};

// LDS slot of element e under plan PL's layout.
template <class PL>
__device__ __forceinline__ int slot(int e) {
  if constexpr (PL::PAD) return e + (e >> PL::PADLOG);
  else return lds_slot(e);
}

// Pass Q of a transform (REV: radices in reverse order).  On entry v holds
// this pass's inputs (butterfly b: i = t + b TPS, v[b R + j] = x[i + j N/R]);
// on exit from the last pass v holds the outputs in the same pattern.
template <class PL, bool INV, bool REV, int Q>
struct Pass {
  static constexpr int R = REV ? PL::radix_rev(Q) : PL::radix(Q);
  static constexpr int P = PL::stride(Q, REV);
  static constexpr int NB = PL::E / R;

  // One exchange of the complex values through an N-point LDS image.
  template <class TW, class LT>
  __device__ static void run(float2 (&v)[PL::E], LT *lds, int t, const TW &tw) {
#pragma unroll
    for (int b = 0; b < NB; b++) {
      const int i = t + b * PL::TPS;
      if constexpr (P > 1) {
        // w^j (j < R) as the product of the table entries w, w^2, w^4, ...
        // selected by the bits of j: log2 R gathers instead of R - 1 and
        // only log2 R live twiddles (at most log2 R - 1 products).
        const int k = i & (P - 1);
        constexpr int S = PL::N / (P * R);
        float2 wb[R >= 32 ? 5 : 4];
#pragma unroll
        for (int q = 0; (1 << q) < R; q++)
          wb[q] = tw.template get<PL, REV, Q>(b, q, (1 << q) * k * S);
#pragma unroll
        for (int j = 1; j < R; j++) {
          float2 w = make_float2(1.f, 0.f);
          bool first = true;
#pragma unroll
          for (int q = 0; (1 << q) < R; q++)
            if (j & (1 << q)) {
              w = first ? wb[q] : cmul(w, wb[q]);
              first = false;
            }
          v[b * R + j] = INV ? cmulc(v[b * R + j], w) : cmul(v[b * R + j], w);
        }
      }
      dft<R, INV>(&v[b * R]);
    }
    if constexpr (Q + 1 < PL::NPASS) {
      constexpr int R2 = REV ? PL::radix_rev(Q + 1) : PL::radix(Q + 1);
      // this pass's outputs (one component via `comp`) -> LDS
      const auto put = [&](auto comp) {
#pragma unroll
        for (int b = 0; b < NB; b++) {
          const int i = t + b * PL::TPS;
          const int k = i & (P - 1);
          const int base = (i - k) * R + k;
          if constexpr (PL::PAD) {
            constexpr int G = 1 << PL::PADLOG;
            static_assert(P == 1 || (R * P) % G == 0, "padded layout: carry-free offsets");
            // base % G + (j P) % G < G for every pass (P = 1: base is a multiple
            // of R > j; else R P is a multiple of G, so base % G = k < P and
            // (j P) % G is a multiple of the power of two P), hence
            // slot(base + j P) = slot(base) + j P + (j P) / G
            const int sb = base + (base >> PL::PADLOG);
#pragma unroll
            for (int j = 0; j < R; j++)
              lds[sb + j * P + ((j * P) >> PL::PADLOG)] = comp(v[b * R + j]);
          } else {
#pragma unroll
            for (int j = 0; j < R; j++) lds[lds_slot(base + j * P)] = comp(v[b * R + j]);
          }
        }
      };
      // LDS -> the next pass's inputs, element e of v via `sink(e, value)`
      const auto get = [&](auto sink) {
#pragma unroll
        for (int b = 0; b < PL::E / R2; b++) {
          const int i = t + b * PL::TPS;
          if constexpr (PL::PAD) {
            static_assert((PL::N / R2) % (1 << PL::PADLOG) == 0, "padded layout: read stride");
            constexpr int D = PL::N / R2 + ((PL::N / R2) >> PL::PADLOG);
            const int si = i + (i >> PL::PADLOG);
#pragma unroll
            for (int j = 0; j < R2; j++) sink(b * R2 + j, lds[si + j * D]);
          } else {
#pragma unroll
            for (int j = 0; j < R2; j++) sink(b * R2 + j, lds[lds_slot(i + j * (PL::N / R2))]);
          }
        }
      };
      put([](float2 z) { return z; });
      lds_barrier();
      get([&](int e, float2 z) { v[e] = z; });
      lds_barrier();
      Pass<PL, INV, REV, Q + 1>::run(v, lds, t, tw);
    }
  }
};

// Element index held by v[b R + j] at the input of the first pass (FIRST)
// or at the output of the last pass (R = that pass's radix).
template <class PL, int R>
__device__ __forceinline__ int reg_index(int t, int b, int j) {
  return t + b * PL::TPS + j * (PL::N / R);
}

// Full transform: v (inputs of the first pass, pattern reg_index<first R>)
// -> v (outputs of the last pass, pattern reg_index<last R>).  `tw` is the
// twiddle table (const float2 *) or a preloaded RegTw<PL, REV>.
template <class PL, bool INV, bool REV, class TW, class LT>
__device__ __forceinline__ void transform(float2 (&v)[PL::E], LT *lds, int t,
                                          const TW &tw) {
  if constexpr (std::is_class_v<TW>) Pass<PL, INV, REV, 0>::run(v, lds, t, tw);
  else Pass<PL, INV, REV, 0>::run(v, lds, t, TableTw{tw});
}

}  // namespace fft
}  // namespace vs
