"""veles: namespace package; the MI355X-native library lives in veles.simd_amd."""
