// VALU instruction-throughput microbenchmark for gfx950: which multiply
// primitive should carry 254-bit modular products?  Every thread runs 8
// independent dependency chains of one instruction; the grid fills all CUs.
// Prints lane-ops/s for each instruction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHAINS 8
#define ITERS 4096

template <int OP>
__global__ void __launch_bounds__(256) k_rate(uint64_t* out, uint32_t seed) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t a64[CHAINS];
  uint32_t a32[CHAINS];
  double ad[CHAINS];
  const uint32_t x = seed ^ tid, y = seed * 7 + tid;
  const double dx = 1.0000001 + tid * 1e-12, dy = 1e-9;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) {
    a64[c] = tid + c;
    a32[c] = tid * 3 + c;
    ad[c] = c + 1.0;
  }
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) {
      if constexpr (OP == 0) {
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a64[c]) : "v"(x), "v"(y) : "vcc");
      } else if constexpr (OP == 1) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a32[c]) : "v"(x) : "vcc");
      } else if constexpr (OP == 2) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a32[c]) : "v"(x));
      } else if constexpr (OP == 3) {
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a32[c]) : "v"(x));
      } else if constexpr (OP == 4) {
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(ad[c]) : "v"(dx), "v"(dy));
      } else if constexpr (OP == 5) {
        asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a32[c]) : "v"(x), "v"(y));
      } else if constexpr (OP == 6) {
        asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a32[c]) : "v"(x));
      } else if constexpr (OP == 7) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, 0, %2, vcc"
                     : "+v"(a32[c]), "+v"(((uint32_t*)&a64[c])[0]) : "v"(x) : "vcc");
      } else if constexpr (OP == 8) {
        asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(a64[c]) : "v"(a64[(c + 1) % CHAINS]));
      } else if constexpr (OP == 9) {
        asm volatile("v_mul_f64 %0, %0, %1" : "+v"(ad[c]) : "v"(dx));
      } else if constexpr (OP == 10) {
        asm volatile("v_add_f64 %0, %0, %1" : "+v"(ad[c]) : "v"(dy));
      } else if constexpr (OP == 11) {
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a32[c]) : "v"(x), "v"(y));
      } else if constexpr (OP == 12) {
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a32[c]) : "v"(x), "v"(y));
      } else if constexpr (OP == 13) {
        asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(a64[c]));
      } else if constexpr (OP == 14) {
        asm volatile("v_and_b32 %0, %1, %0" : "+v"(a32[c]) : "v"(x));
      } else if constexpr (OP == 15) {
        asm volatile("v_alignbit_b32 %0, %1, %0, 29" : "+v"(a32[c]) : "v"(x));
      } else if constexpr (OP == 16) {
        asm volatile("v_mov_b32 %0, %1" : "=v"(a32[c]) : "v"(a32[(c + 1) % CHAINS]));
      } else if constexpr (OP == 17) {
        asm volatile("v_sub_u32 %0, %1, %0" : "+v"(a32[c]) : "v"(x));
      } else if constexpr (OP == 18) {
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a32[c]) : "v"(x) : "vcc");
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s += a64[c] + a32[c] + (uint64_t)ad[c];
  out[tid] = s;
}

static const char* NAMES[] = {"v_mad_u64_u32",  "v_add_co_u32",   "v_mul_lo_u32",
                              "v_mul_hi_u32",   "v_fma_f64",      "v_mad_u32_u24",
                              "v_mul_hi_u32_u24", "add_co+addc(2)", "v_lshl_add_u64",
                              "v_mul_f64",      "v_add_f64",      "v_fma_f32",
                              "v_add3_u32",     "v_lshrrev_b64",  "v_and_b32",
                              "v_alignbit_b32", "v_mov_b32",      "v_sub_u32",
                              "v_cndmask_b32"};

template <int OP>
static void run(uint64_t* d, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, d, 2u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)blocks * 256 * ITERS * CHAINS;
  // lane-ops per SIMD-cycle at 2.4 GHz on 1024 SIMDs (the engine clock may differ)
  double per_simd_clk = ops / (ms * 1e-3) / (1024 * 2.4e9);
  printf("{\"op\": \"%s\", \"lane_ops_per_s\": %.4e, \"lane_ops_per_simd_clk_at_2.4GHz\": %.2f}\n",
         NAMES[OP], ops / (ms * 1e-3), per_simd_clk);
}

int main() {
  int blocks = 256 * 16;
  uint64_t* d;
  hipMalloc(&d, (size_t)blocks * 256 * 8);
  run<0>(d, blocks);
  run<1>(d, blocks);
  run<2>(d, blocks);
  run<3>(d, blocks);
  run<4>(d, blocks);
  run<5>(d, blocks);
  run<6>(d, blocks);
  run<7>(d, blocks);
  run<8>(d, blocks);
  run<9>(d, blocks);
  run<10>(d, blocks);
  run<11>(d, blocks);
  run<12>(d, blocks);
  run<13>(d, blocks);
  run<14>(d, blocks);
  run<15>(d, blocks);
  run<16>(d, blocks);
  run<17>(d, blocks);
  run<18>(d, blocks);
  hipFree(d);
  return 0;
}
