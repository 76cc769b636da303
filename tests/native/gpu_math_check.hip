// GPU check of the kernel's exactness-preserving shortcuts on the device
// itself (v_rsq_f64 exists only there): rtwm::sqrt_rn == __builtin_sqrt and
// rtwm::div_rn == IEEE division, bit for bit, over random bit patterns of
// every exponent (zeros, subnormals, infinities, NaNs included), the
// neighbourhood of sqrt_rn's 2^-767 fast-path threshold, perfect squares and
// their neighbours, and near-all-ones mantissas.  Built by the package
// Makefile (bin/gpu_math_check); run by tests/test_gpu_math.py.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "rtw_math.hpp"

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__global__ void check(uint64_t n, unsigned long long* out) {
  unsigned long long bad_sqrt = 0, bad_div = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t z = mix(0x243F6A8885A308D3ULL + i * 0x9e3779b97f4a7c15ULL), w = mix(z);
    const uint64_t man = z & 0x000FFFFFFFFFFFFFULL;
    double x;
    switch (i & 3) {
      case 0:  // any non-negative bit pattern (zeros, subnormals, inf, NaN)
        x = __longlong_as_double((long long)(z & 0x7FFFFFFFFFFFFFFFULL));
        break;
      case 1:  // [2^-32, 2^32)
        x = __longlong_as_double((long long)(man | ((uint64_t)(0x3FF - 32 + (int)((z >> 52) & 63)) << 52)));
        break;
      case 2: {  // perfect squares and their neighbours
        const double r = __longlong_as_double((long long)(man | (0x3FFULL << 52)));
        const double s = r * r;
        x = __longlong_as_double(__double_as_longlong(s) + (long long)((z >> 60) & 7) - 3);
        break;
      }
      default:  // around the fast-path threshold 2^-767 (biased exponent 256)
        x = __longlong_as_double((long long)(man | ((uint64_t)(252 + ((z >> 52) & 7)) << 52)));
    }
    const double a = rtwm::sqrt_rn(x), r = __builtin_sqrt(x);
    if (__double_as_longlong(a) != __double_as_longlong(r) && !(a != a && r != r)) ++bad_sqrt;
    // division: x / b from y = RN(1 / b), random signs and exponents in +-60
    const double xx = __longlong_as_double((long long)((w & 0x800FFFFFFFFFFFFFULL) |
                                                       ((uint64_t)(0x3FF - 60 + (int)((w >> 52) % 121)) << 52)));
    uint64_t bb = (man | ((uint64_t)(0x3FF - 60 + (int)((z >> 52) % 121)) << 52));
    if ((i & 7) == 0) bb = (bb | 0x000FFFFFFFFFFFFFULL) - ((z >> 61) & 3);  // near all-ones mantissas
    const double b = __longlong_as_double((long long)bb);
    const double y = 1.0 / b;
    if (__double_as_longlong(rtwm::div_rn(xx, b, y)) != __double_as_longlong(xx / b)) ++bad_div;
  }
  atomicAdd(out + 0, bad_sqrt);
  atomicAdd(out + 1, bad_div);
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 28);
  unsigned long long* d = nullptr;
  unsigned long long h[2] = {0, 0};
  if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMemset(d, 0, sizeof(h)) != hipSuccess) return 2;
  hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, n, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  (void)hipFree(d);
  std::printf("tested %llu sqrt_rn mismatches %llu div_rn mismatches %llu\n", (unsigned long long)n, h[0], h[1]);
  return (h[0] || h[1]) ? 1 : 0;
}
