// ubench_valu.hip — issue-rate microbenchmark of the VALU instructions the
// trace kernel's RNG and sphere test are made of (gfx950).  Each thread runs
// 8 independent chains of one instruction (inline asm, so exactly that
// opcode); 16 waves per CU.  Prints lane-ops per clock per CU (clock from
// s_memtime / s_memrealtime inside the kernel).
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_valu.hip -o /tmp/ubench_valu
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHAIN8(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7)

template <int OP>
__global__ void __launch_bounds__(256) kern(uint64_t* out, int iters, uint64_t* clk) {
  uint32_t a[8];
  uint64_t q[8];
  double d[8];
  float f[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = threadIdx.x * 7 + i;
    q[i] = ((uint64_t)a[i] << 32) | (a[i] * 3u + 1u);
    d[i] = 1.0 + a[i] * 1e-9;
    f[i] = 1.0f + a[i] * 1e-7f;
  }
  const uint32_t b = 0x9e3779b9u + blockIdx.x;
  const uint64_t b64 = 0x9e3779b97f4a7c15ull;
  const double bd = 0.999999;
  const float bf = 0.999999f;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#define S_MULLO(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define S_MULHI(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define S_MAD64(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q[i]) : "v"(a[i]), "v"(b) : "vcc");
#define S_ADD32(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define S_XOR32(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define S_SHR64(i) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(q[i]));
#define S_FMA64(i) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(bd));
#define S_ADD64(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(bd));
#define S_FMA32(i) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "v"(bf));
#define S_PKFMA(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(q[i]) : "v"(b64));
#define S_SQRT64(i) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[i]));
#define S_RCP64(i) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[i]));
#define S_RCP32(i) asm volatile("v_rcp_f32 %0, %0" : "+v"(f[i]));
#define S_ADDC64(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(b64));
#define S_CVT(i) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[i]) : "v"(a[i]));
    if constexpr (OP == 0) { CHAIN8(S_MULLO) }
    if constexpr (OP == 1) { CHAIN8(S_MULHI) }
    if constexpr (OP == 2) { CHAIN8(S_MAD64) }
    if constexpr (OP == 3) { CHAIN8(S_ADD32) }
    if constexpr (OP == 4) { CHAIN8(S_XOR32) }
    if constexpr (OP == 5) { CHAIN8(S_SHR64) }
    if constexpr (OP == 6) { CHAIN8(S_FMA64) }
    if constexpr (OP == 7) { CHAIN8(S_ADD64) }
    if constexpr (OP == 8) { CHAIN8(S_FMA32) }
    if constexpr (OP == 9) { CHAIN8(S_PKFMA) }
    if constexpr (OP == 10) { CHAIN8(S_SQRT64) }
    if constexpr (OP == 11) { CHAIN8(S_RCP64) }
    if constexpr (OP == 12) { CHAIN8(S_RCP32) }
    if constexpr (OP == 13) { CHAIN8(S_ADDC64) }
    if constexpr (OP == 14) { CHAIN8(S_CVT) }
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint64_t acc = 0;
  for (int i = 0; i < 8; ++i) acc += a[i] + q[i] + (uint64_t)__double_as_longlong(d[i]) + __float_as_uint(f[i]);
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

static const char* kNames[] = {"v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_add_u32", "v_xor_b32",
                               "v_lshrrev_b64", "v_fma_f64", "v_add_f64", "v_fma_f32", "v_pk_fma_f32",
                               "v_sqrt_f64", "v_rcp_f64", "v_rcp_f32", "v_lshl_add_u64", "v_cvt_f64_u32"};

template <int OP>
static void run(uint64_t* out, uint64_t* clk, int cus) {
  const int blocks = cus * 4, iters = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, out, 64, clk);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  uint64_t h[2];
  hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;  // memrealtime = 100 MHz
  const double lane_ops = (double)blocks * 256 * iters * 8;
  const double per_clk_cu = lane_ops / (ms * 1e-3) / (ghz * 1e9) / cus;
  printf("%-16s %8.3f ms  %7.1f lane-ops/clk/CU  (wave64 instr per SIMD every %.2f clk)  clk %.2f GHz\n", kNames[OP],
         ms, per_clk_cu, 64.0 * 4 / per_clk_cu, ghz);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint64_t *out, *clk;
  hipMalloc(&out, (size_t)cus * 4 * 256 * 8);
  hipMalloc(&clk, 16);
  run<0>(out, clk, cus); run<1>(out, clk, cus); run<2>(out, clk, cus); run<3>(out, clk, cus);
  run<4>(out, clk, cus); run<5>(out, clk, cus); run<6>(out, clk, cus); run<7>(out, clk, cus);
  run<8>(out, clk, cus); run<9>(out, clk, cus); run<10>(out, clk, cus); run<11>(out, clk, cus);
  run<12>(out, clk, cus); run<13>(out, clk, cus); run<14>(out, clk, cus);
  return 0;
}
