// Batch-affine bucket additions, the best case: how fast
// can MI355X add pairs of affine points with Montgomery's batch inversion,
// against the XYZZ mixed addition k_msm_accumulate runs, both fed from the
// SAME kind of operand stream?
//
// The operands here are streamed (limb-major, lane-coalesced), not gathered
// from a 27.9 GB table as the MSM must; so each rate is an upper bound for
// its form, and the XYZZ kernel bounds what today's accumulate could reach
// without its gathers (~14.6e9 madds/s with them).
//
//   k_xyzz : per lane B mixed additions acc += (x, y), 1 point read per add
//   k_ba   : per lane B independent pair additions (x1, y1) + (x2, y2):
//            phase 1 forward prefix products of d_k = x2 - x1 (stored to a
//            scratch array: B x 36 B per lane cannot stay on chip), one
//            inversion per lane (Fermat, inv29), phase 2 backward: 1/d_k =
//            inv * pre_k, inv *= d_k, lambda = (y2 - y1) / d_k, x3, y3 —
//            the pair's operands are read twice (the second read cannot
//            come from on-chip memory either: 4 x 36 B x B per lane).
// A checking pass verifies d_k * (1/d_k) == 1 for every pair.  "ba-l2" reads
// its operands from the first 2^16 elements only (cache-resident; timing
// only): the pair additions' compute rate with the operand traffic removed
// (the prefix array still streams).
//
//   hipcc -std=c++17 -O3 --offload-arch=gfx950 micro/ba_bench.hip -o micro/ba_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../csrc/curve.h"
#include "../csrc/curve29.h"
using namespace qg;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

// limb-major field array: limb l of element i at a[l * n + i]
__device__ __forceinline__ Q29 ld29(const uint32_t* __restrict__ a, size_t n, size_t i) {
  Q29 r;
#pragma unroll
  for (int l = 0; l < 9; l++) r.l[l] = __builtin_nontemporal_load(a + l * n + i);
  return r;
}
__device__ __forceinline__ void st29(uint32_t* __restrict__ a, size_t n, size_t i, const Q29& v) {
  // ordinary stores: the prefix array is re-read by the same lane
#pragma unroll
  for (int l = 0; l < 9; l++) a[l * n + i] = v.l[l];
}

// pseudo-random normalized values < 2^253 < p (top limb: bits 232..252)
__global__ void k_fill(uint32_t* a, size_t n, uint64_t seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
  for (int l = 0; l < 9; l++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    a[l * n + i] = (uint32_t)s & (l == 8 ? 0x1fffffu : M29);
  }
}

__global__ void __launch_bounds__(256) k_xyzz(const uint32_t* __restrict__ X, const uint32_t* __restrict__ Y,
                                              size_t n, int B, uint32_t* __restrict__ out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  X29 acc;
  acc.X = ld29(X, n, t);
  acc.Y = ld29(Y, n, t);
  acc.ZZ = Q29::from_l9(F29P<FqP>::ONE);
  acc.ZZZ = acc.ZZ;
  bool inf = false;
  for (int k = 1; k < B; k++) {
    const Q29 ax = ld29(X, n, (size_t)k * T + t), ay = ld29(Y, n, (size_t)k * T + t);
    if (!x29_acc_madd_tp(acc, ax, ay)) x29_acc_madd_exc(acc, ax, ay, &inf);
  }
  uint32_t s = 0;
#pragma unroll
  for (int l = 0; l < 9; l++) s ^= acc.X.l[l] ^ acc.Y.l[l] ^ acc.ZZ.l[l] ^ acc.ZZZ.l[l];
  out[t] = s;
#endif
}

template <bool CHECK, bool SMALL = false>
__global__ void __launch_bounds__(256) k_ba(const uint32_t* __restrict__ X1, const uint32_t* __restrict__ Y1,
                                            const uint32_t* __restrict__ X2, const uint32_t* __restrict__ Y2,
                                            size_t n, int B, uint32_t* __restrict__ pre,
                                            uint32_t* __restrict__ OX, uint32_t* __restrict__ OY,
                                            uint32_t* __restrict__ bad) {
#if defined(__HIP_DEVICE_COMPILE__)
  const size_t T = (size_t)gridDim.x * blockDim.x;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const Q29 one = Q29::from_l9(F29P<FqP>::ONE);
  Q29 acc = one;
  for (int k = 0; k < B; k++) {
    const size_t i = (size_t)k * T + t;
    const size_t o = SMALL ? (i & 0xffffu) : i;  // operand index
    st29(pre, n, i, acc);
    const Q29 d = normfull29(sub29(ld29(X2, n, o), ld29(X1, n, o)));
    acc = mul29t(acc, d);
  }
  Q29 inv = inv29<FqP>(acc);
  uint32_t nbad = 0;
  for (int k = B - 1; k >= 0; k--) {
    const size_t i = (size_t)k * T + t;
    const size_t o = SMALL ? (i & 0xffffu) : i;
    const Q29 x1 = ld29(X1, n, o), y1 = ld29(Y1, n, o), x2 = ld29(X2, n, o), y2 = ld29(Y2, n, o);
    const Q29 d = normfull29(sub29(x2, x1));
    const Q29 pk = ld29(pre, n, i);
    const Q29 invk = mul29t(inv, pk);
    inv = mul29t(inv, d);
    if (CHECK) {
      const Q29 e = canon29(mul29(invk, d));
      bool ok = true;
#pragma unroll
      for (int l = 0; l < 9; l++) ok = ok && e.l[l] == canon29(one).l[l];
      nbad += ok ? 0u : 1u;
    }
    const Q29 lam = mul29t(normfull29(sub29(y2, y1)), invk);
    const Q29 x3 = red16p29(sub29(sub29(sqr29t(lam), x1), x2));
    const Q29 y3 = red6p29(mulsub29t(lam, norm29(sub29(x1, x3)), y1, one));
    st29(OX, n, i, x3);
    st29(OY, n, i, y3);
  }
  if (CHECK && nbad) atomicAdd(bad, nbad);
#endif
}

int main(int argc, char** argv) {
  const int logT = argc > 1 ? atoi(argv[1]) : 18;  // threads (2^18 = 4 waves per SIMD)
  const size_t T = (size_t)1 << logT;
  const int Bs[] = {32, 64, 128, 256};
  const int maxB = 256;
  const size_t n = T * maxB;  // elements per array
  uint32_t *X1, *Y1, *X2, *Y2, *pre, *OX, *OY, *sink, *bad;
  const size_t bytes = n * 9 * sizeof(uint32_t);
  CK(hipMalloc(&X1, bytes));
  CK(hipMalloc(&Y1, bytes));
  CK(hipMalloc(&X2, bytes));
  CK(hipMalloc(&Y2, bytes));
  CK(hipMalloc(&pre, bytes));
  CK(hipMalloc(&OX, bytes));
  CK(hipMalloc(&OY, bytes));
  CK(hipMalloc(&sink, T * sizeof(uint32_t)));
  CK(hipMalloc(&bad, sizeof(uint32_t)));
  CK(hipMemset(bad, 0, sizeof(uint32_t)));
  const unsigned fb = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, 0, X1, n, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, 0, Y1, n, 2ull);
  hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, 0, X2, n, 3ull);
  hipLaunchKernelGGL(k_fill, dim3(fb), dim3(256), 0, 0, Y2, n, 4ull);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const unsigned g = (unsigned)(T / 256);
  // correctness of the batch inversion first (B = 64)
  hipLaunchKernelGGL(k_ba<true>, dim3(g), dim3(256), 0, 0, X1, Y1, X2, Y2, n, 64, pre, OX, OY, bad);
  CK(hipGetLastError());
  uint32_t hbad = 0;
  CK(hipMemcpy(&hbad, bad, sizeof(uint32_t), hipMemcpyDeviceToHost));
  printf("check: %u of %zu pairs with d * (1/d) != 1\n", hbad, T * 64);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  printf("threads %zu (%zu waves per SIMD over 1024 SIMDs)\n", T, T / 64 / 1024);
  for (int B : Bs) {
    for (int form = 0; form < 3; form++) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(a));
        if (form == 0)
          hipLaunchKernelGGL(k_xyzz, dim3(g), dim3(256), 0, 0, X2, Y2, n, B, sink);
        else if (form == 2)
          hipLaunchKernelGGL((k_ba<false, true>), dim3(g), dim3(256), 0, 0, X1, Y1, X2, Y2, n, B, pre, OX, OY, bad);
        else
          hipLaunchKernelGGL(k_ba<false>, dim3(g), dim3(256), 0, 0, X1, Y1, X2, Y2, n, B, pre, OX, OY, bad);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      const double adds = (double)T * (form == 0 ? B - 1 : B);
      // bytes moved: xyzz 72 B per add; ba 144 B (phase 1: x1, x2 + 36 B prefix
      // store) + 144 B operands + 36 B prefix + 72 B result in phase 2
      const double bpa = form == 0 ? 72.0 : form == 1 ? (72.0 + 36.0 + 144.0 + 36.0 + 72.0) : (36.0 + 36.0 + 72.0);
      printf("B %4d %-6s %8.3f ms  %7.2f G additions/s  %6.0f GB/s streamed\n", B,
             form == 0 ? "xyzz" : form == 1 ? "ba" : "ba-l2", best, adds / (best * 1e6), adds * bpa / (best * 1e6));
    }
  }
  return hbad ? 1 : 0;
}
