// Sumcheck prover timed through the C-ABI alone (what a Rust caller of
// qg_sumcheck_prove_dev sees): h = g0 g1 g2 at 2^nv variables, device-resident
// tables.  Prints wall time per call, the kernels' HIP-event time and the
// host/launch remainder.  Build: make -C quill-zkvm_amd micro/sc_capi
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/quill_gpu.h"

#define CK(x)                                                          \
  do {                                                                 \
    int rc_ = (x);                                                     \
    if (rc_) {                                                         \
      fprintf(stderr, "%s -> %d: %s\n", #x, rc_, qg_last_error(ctx)); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t nv = argc > 1 ? (uint32_t)atoi(argv[1]) : 20;
  const int steps = argc > 2 ? atoi(argv[2]) : 50;
  qg_ctx* ctx = nullptr;
  if (qg_ctx_create(0, &ctx)) return 1;
  qg_buf* t[3];
  for (int i = 0; i < 3; i++) {
    CK(qg_buf_create(ctx, (size_t)1 << nv, &t[i]));
    CK(qg_buf_fill_random(t[i], 0x5155494C4CULL + 3 + 7 * i));
  }
  const qg_expr_op prog[5] = {{QG_OP_INPUT, 0}, {QG_OP_INPUT, 1}, {QG_OP_MUL, 0},
                              {QG_OP_INPUT, 2}, {QG_OP_MUL, 0}};
  uint32_t deg = 0;
  CK(qg_expr_degree(prog, 5, &deg));
  const uint32_t w = deg + 1;
  std::vector<uint64_t> coeffs((size_t)nv * w * 4), point((size_t)nv * 4);
  std::vector<uint32_t> lens(nv);
  uint64_t ev[4], claim[4] = {0, 0, 0, 0};
  uint8_t st[32];
  auto call = [&]() {
    memset(st, 7, 32);
    return qg_sumcheck_prove_dev(ctx, nv, 3, t, prog, 5, nullptr, 0, claim, st, coeffs.data(),
                                 lens.data(), point.data(), ev);
  };
  for (int i = 0; i < 5; i++) CK(call());
  CK(qg_ctx_enable_timing(ctx, 1));
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < steps; i++) CK(call());
  const auto t1 = std::chrono::steady_clock::now();
  double rk = 0, tl = 0;
  uint32_t nr = 0, ntl = 0;
  CK(qg_ctx_kernel_time(ctx, "sumcheck_round", &rk, &nr));
  CK(qg_ctx_kernel_time(ctx, "sumcheck_tail", &tl, &ntl));
  CK(qg_ctx_enable_timing(ctx, 0));
  const auto t2 = std::chrono::steady_clock::now();
  for (int i = 0; i < steps; i++) CK(call());
  const auto t3 = std::chrono::steady_clock::now();
  const double ms_t = std::chrono::duration<double, std::milli>(t1 - t0).count() / steps;
  const double ms = std::chrono::duration<double, std::milli>(t3 - t2).count() / steps;
  printf("{\"nv\": %u, \"capi_ms\": %.4f, \"capi_ms_with_timing\": %.4f, \"round_kernels_ms\": %.4f, "
         "\"tail_kernel_ms\": %.4f, \"host_and_gaps_ms\": %.4f, \"digest\": \"%016llx\"}\n",
         nv, ms, ms_t, rk / steps, tl / steps, ms - (rk + tl) / steps,
         (unsigned long long)(coeffs[0] ^ coeffs[4 * w * (nv - 1)] ^ ev[0]));
  for (int i = 0; i < 3; i++) qg_buf_destroy(t[i]);
  qg_ctx_destroy(ctx);
  return 0;
}
