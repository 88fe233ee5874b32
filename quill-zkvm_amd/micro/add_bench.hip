// XYZZ point-operation latency / throughput on MI355X, for the bucket
// reduction's design (csrc/msm.hip): ns per operation per wave for a chain of
// dependent operations with 1, 2 and 4 waves per SIMD (grid of 64-thread
// blocks = 1024 x w).  Variants: x29_add (latency-form multiplies), the same
// addition with its independent products in interleaved pairs (mul29t2),
// the quad-cooperative x29_add_q4, x29_dbl, x29_dbl_q4.  The cooperative
// results are checked against the single-lane ones (canonical coordinates).
//   hipcc -std=c++17 -O3 --offload-arch=gfx950 micro/add_bench.hip -o micro/add_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../csrc/curve.h"
#include "../csrc/curve29.h"
using namespace qg;

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

#if defined(__HIP_DEVICE_COMPILE__)
template <int S>
__device__ __forceinline__ Q29 q29_quad(const Q29& a) {
  Q29 r;
#pragma unroll
  for (int i = 0; i < 9; i++)
    r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], S * 0x55, 0xf, 0xf, false);
  return r;
}
__device__ __forceinline__ Q29 q29_sel(bool c, const Q29& a, const Q29& b) {
  Q29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}
__device__ __forceinline__ X29 add_q4(const X29& p, const X29& q) {
  if (x29_is_inf(p)) return q;
  if (x29_is_inf(q)) return p;
  const uint32_t r = threadIdx.x & 3u;
  const bool r0 = r == 0, r1 = r == 1, r2 = r == 2, odd = (r & 1u) != 0u;
  const Q29 m0 = mul29(q29_sel(r0, p.X, q29_sel(r1, q.X, q29_sel(r2, p.Y, q.Y))),
                       q29_sel(r0, q.ZZ, q29_sel(r1, p.ZZ, q29_sel(r2, q.ZZZ, p.ZZZ))));
  const Q29 m1 = mul29(q29_sel(odd, p.ZZZ, p.ZZ), q29_sel(odd, q.ZZZ, q.ZZ));
  const Q29 U1 = q29_quad<0>(m0), U2 = q29_quad<1>(m0), S1 = q29_quad<2>(m0), S2 = q29_quad<3>(m0);
  const Q29 ZZ12 = q29_quad<0>(m1), ZZZ12 = q29_quad<1>(m1);
  const Q29 P = normfull29(sub29(U2, U1));
  const Q29 R = normfull29(sub29(S2, S1));
  if (is_zero_mod29_fast<FqP, 8>(P)) return x29_add(p, q);
  const Q29 sq = sqr29(q29_sel(odd, R, P));
  const Q29 PP = q29_quad<0>(sq), RR = q29_quad<1>(sq);
  const Q29 m3 = mul29(q29_sel(r0, P, q29_sel(r1, U1, ZZ12)), PP);
  const Q29 PPP = q29_quad<0>(m3), Q = q29_quad<1>(m3), ZZ3 = q29_quad<2>(m3);
  const Q29 X3 = red16p29(sub29(sub29(sub29(RR, PPP), Q), Q));
  const Q29 z = Q29::zero();
  const Q29 m4 = red6p29(mulsub29(q29_sel(r0, R, ZZZ12), q29_sel(r0, norm29(sub29(Q, X3)), PPP),
                                  q29_sel(r0, S1, z), q29_sel(r0, PPP, z)));
  return {X3, q29_quad<0>(m4), ZZ3, q29_quad<1>(m4)};
}
__device__ __forceinline__ X29 dbl_q4(const X29& p) {
  if (x29_is_inf(p)) return p;
  const uint32_t r = threadIdx.x & 3u;
  const bool r0 = r == 0, r1 = r == 1, r2 = r == 2;
  const Q29 U = normfull29(add29(p.Y, p.Y));
  const Q29 s1 = sqr29(q29_sel((r & 1u) != 0u, p.X, U));
  const Q29 V = q29_quad<0>(s1), X2 = q29_quad<1>(s1);
  const Q29 M = normfull29(add29(add29(X2, X2), X2));
  const Q29 m2 = mul29(q29_sel(r0, U, q29_sel(r1, p.X, q29_sel(r2, p.ZZ, M))), q29_sel(r < 3, V, M));
  const Q29 W = q29_quad<0>(m2), S = q29_quad<1>(m2), ZZ3 = q29_quad<2>(m2), MM = q29_quad<3>(m2);
  const Q29 X3 = red16p29(sub29(sub29(MM, S), S));
  const Q29 z = Q29::zero();
  const Q29 m3 = red6p29(mulsub29(q29_sel(r0, M, W), q29_sel(r0, norm29(sub29(S, X3)), p.ZZZ),
                                  q29_sel(r0, W, z), q29_sel(r0, p.Y, z)));
  return {X3, q29_quad<0>(m3), ZZ3, q29_quad<1>(m3)};
}
// x29_add with the independent products in interleaved pairs
__device__ __forceinline__ X29 add_t2(const X29& p, const X29& q) {
  if (x29_is_inf(p)) return q;
  if (x29_is_inf(q)) return p;
  Q29 U1, U2, S1, S2, Z12, Z123, PP, RR, PPP, Q, ZZ3, ZZZ3;
  mul29t2(p.X, q.ZZ, q.X, p.ZZ, U1, U2);
  mul29t2(p.Y, q.ZZZ, q.Y, p.ZZZ, S1, S2);
  mul29t2(p.ZZ, q.ZZ, p.ZZZ, q.ZZZ, Z12, Z123);
  const Q29 P = normfull29(sub29(U2, U1));
  const Q29 R = normfull29(sub29(S2, S1));
  if (is_zero_mod29_fast<FqP, 8>(P)) return x29_add(p, q);
  sqr29t2(P, R, PP, RR);
  mul29t2(P, PP, U1, PP, PPP, Q);
  const Q29 X3 = red16p29(sub29(sub29(sub29(RR, PPP), Q), Q));
  mul29t2(Z12, PP, Z123, PPP, ZZ3, ZZZ3);
  const Q29 Y3 = red6p29(mulsub29(R, norm29(sub29(Q, X3)), S1, PPP));
  return {X3, Y3, ZZ3, ZZZ3};
}
#endif

__device__ X29 ld(const G1Xyzz* t, uint32_t i) { return x29_load(t[i & 1023]); }

template <int V>
__global__ void __launch_bounds__(64) k_chain(const G1Xyzz* __restrict__ tab, int iters,
                                              G1Xyzz* __restrict__ out) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;
  const uint32_t e = (V == 2 || V == 4) ? t >> 2 : t;  // quad variants: one element per quad
  X29 acc = ld(tab, e), q = ld(tab, e + 7);
  for (int i = 0; i < iters; i++) {
    if (V == 0) acc = x29_add(acc, q);
    if (V == 1) acc = add_t2(acc, q);
    if (V == 2) acc = add_q4(acc, q);
    if (V == 3) acc = x29_dbl(acc);
    if (V == 4) acc = dbl_q4(acc);
  }
  if ((V != 2 && V != 4) || (threadIdx.x & 3u) == 0) out[e] = x29_store(x29_acc_finish(acc));
#endif
}

int main() {
  // pseudo-random XYZZ "points" (limbs < 2^29, values < 2p): the formulas run
  // their main path; the timing does not need curve points
  const int N = 1024;
  G1Xyzz* h = (G1Xyzz*)malloc(N * sizeof(G1Xyzz));
  uint64_t s = 0x5155494c4cull;
  for (int i = 0; i < N; i++) {
    uint32_t* w = reinterpret_cast<uint32_t*>(&h[i]);
    for (int k = 0; k < 32; k++) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      w[k] = (uint32_t)s;
      if (k % 8 == 7) w[k] &= 0x1fffffff;  // top word: value < 2^253 < p
    }
  }
  G1Xyzz *d_tab, *d_out[5];
  CK(hipMalloc(&d_tab, N * sizeof(G1Xyzz)));
  CK(hipMemcpy(d_tab, h, N * sizeof(G1Xyzz), hipMemcpyHostToDevice));
  const int maxb = 1024 * 4;
  for (int v = 0; v < 5; v++) CK(hipMalloc(&d_out[v], (size_t)maxb * 64 * sizeof(G1Xyzz)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[5] = {"x29_add", "add_t2", "add_q4", "x29_dbl", "dbl_q4"};
  const int iters = 64;
  for (int v = 0; v < 5; v++) {
    for (int w = 1; w <= 4; w *= 2) {
      const int nb = 1024 * w;
      for (int rep = 0; rep < 2; rep++) {
        CK(hipEventRecord(a));
        switch (v) {
          case 0: hipLaunchKernelGGL(k_chain<0>, dim3(nb), dim3(64), 0, 0, d_tab, iters, d_out[0]); break;
          case 1: hipLaunchKernelGGL(k_chain<1>, dim3(nb), dim3(64), 0, 0, d_tab, iters, d_out[1]); break;
          case 2: hipLaunchKernelGGL(k_chain<2>, dim3(nb), dim3(64), 0, 0, d_tab, iters, d_out[2]); break;
          case 3: hipLaunchKernelGGL(k_chain<3>, dim3(nb), dim3(64), 0, 0, d_tab, iters, d_out[3]); break;
          case 4: hipLaunchKernelGGL(k_chain<4>, dim3(nb), dim3(64), 0, 0, d_tab, iters, d_out[4]); break;
        }
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep == 1)
          printf("%-8s waves/SIMD %d: %8.3f ms, %7.2f us per op per wave, %8.2f Mops/s (elements)\n",
                 names[v], w, ms, ms * 1e3 / iters,
                 (double)nb * ((v == 2 || v == 4) ? 16 : 64) * iters / (ms * 1e3));
      }
    }
  }
  // cooperative == single-lane (first 1024 elements of the 1-wave runs)
  G1Xyzz* r[5];
  for (int v = 0; v < 5; v++) {
    r[v] = (G1Xyzz*)malloc(1024 * sizeof(G1Xyzz));
    CK(hipMemcpy(r[v], d_out[v], 1024 * sizeof(G1Xyzz), hipMemcpyDeviceToHost));
  }
  // compare in the field: X / ZZ and Y / ZZZ projectively (X1 ZZ2 == X2 ZZ1 etc.)
  int bad = 0;
  for (int i = 0; i < 1024; i++) {
    const int pairs[3][2] = {{0, 1}, {0, 2}, {3, 4}};
    for (auto& pr : pairs) {
      const G1Xyzz& u = r[pr[0]][i];
      const G1Xyzz& v = r[pr[1]][i];
      Fq l1 = to_mont(u.X) * to_mont(v.ZZ), r1 = to_mont(v.X) * to_mont(u.ZZ);
      Fq l2 = to_mont(u.Y) * to_mont(v.ZZZ), r2 = to_mont(v.Y) * to_mont(u.ZZZ);
      if (!(l1 == r1) || !(l2 == r2)) bad++;
    }
  }
  printf("cooperative / paired vs single-lane mismatches: %d of %d\n", bad, 3 * 1024);
  return bad ? 1 : 0;
}
