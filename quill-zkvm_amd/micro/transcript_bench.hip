// Latency of the device transcript step used by every sumcheck round:
// absorb (u64 len || 4 coefficients) + draw one Fr, on one wave.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../csrc/blake3.h"
using namespace qg;

struct LdsSrc {
  const uint32_t* p;
  __device__ uint32_t operator()(uint32_t i) const { return p[i]; }
};

__global__ void k_tr(uint32_t* io, int iters, long long* cyc) {
  __shared__ uint32_t msg[8 + 2 + 128], chin[12], ab[20];
  if (threadIdx.x < 8) msg[threadIdx.x] = io[threadIdx.x];
  for (int i = threadIdx.x; i < 128; i += blockDim.x) msg[10 + i] = io[8 + i];
  __syncthreads();
  long long t0 = clock64();
  if (threadIdx.x == 0) {
    Fr acc = Fr::zero();
    for (int it = 0; it < iters; it++) {
      msg[8] = 4;
      msg[9] = 0;
      b3_chunk_words(LdsSrc{msg}, 40 + 32 * 4, chin, 8);
      chin[8] = 0x6c616863u;
      chin[9] = 0x676e656cu;
      chin[10] = 0x65u;
      for (int i = 0; i < 8; i++) ab[i] = chin[i];
      b3_chunk_words(LdsSrc{chin}, 41, ab + 8, 12);
      b3_chunk_words(LdsSrc{ab}, 80, msg, 8);
      Fr lo, hi;
      for (int i = 0; i < 8; i++) lo.v[i] = ab[8 + i];
      for (int i = 0; i < 4; i++) hi.v[i] = ab[16 + i];
      for (int i = 4; i < 8; i++) hi.v[i] = 0;
      acc = acc + lo * Fr::from_raw(FrP::R2) + hi * Fr::from_raw(FrP::R3);
    }
    for (int i = 0; i < 8; i++) io[i] = msg[i] ^ acc.v[i];
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void k_b3only(uint32_t* io, int iters, long long* cyc) {
  __shared__ uint32_t msg[8 + 2 + 128];
  for (int i = threadIdx.x; i < 138; i += blockDim.x) msg[i] = io[i];
  __syncthreads();
  long long t0 = clock64();
  if (threadIdx.x == 0) {
    for (int it = 0; it < iters; it++) b3_chunk_words(LdsSrc{msg}, 64, msg, 8);
    for (int i = 0; i < 8; i++) io[i] = msg[i];
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void k_mul(uint32_t* io, int iters, long long* cyc) {
  Fr a = Fr::from_raw(io), b = Fr::from_raw(io + 8);
  long long t0 = clock64();
  for (int it = 0; it < iters; it++) a = a * b;
  long long t1 = clock64();
  for (int i = 0; i < 8; i++) io[16 + i] = a.v[i];
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

// quad-lane BLAKE3: chained 64-byte hashes
__global__ void k_b3quad(uint32_t* io, int iters, long long* cyc) {
  __shared__ uint32_t msg[16], out[16];
  if (threadIdx.x < 16) msg[threadIdx.x] = io[threadIdx.x];
  __syncthreads();
  long long t0 = clock64();
  if (threadIdx.x < 64) {
    for (int it = 0; it < iters; it++) {
      b3_hash_quad(msg, 64, out, 8);
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
      if (threadIdx.x < 8) msg[threadIdx.x] = out[threadIdx.x];
      __builtin_amdgcn_s_waitcnt(0);
      __builtin_amdgcn_wave_barrier();
    }
    if (threadIdx.x < 8) io[threadIdx.x] = msg[threadIdx.x];
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

// correctness: quad vs single-lane over lengths 0..1024 step 4 (+ 41), XOF 16 words
__global__ void k_b3check(const uint32_t* src, uint32_t* bad) {
  __shared__ uint32_t msg[256 + 16], o1[16], o2[16];
  for (int len = 0; len <= 1024; len += (len == 40 ? 1 : (len == 41 ? 3 : 4))) {
    __syncthreads();
    for (int i = threadIdx.x; i < 272; i += blockDim.x) {
      uint32_t w = src[i];
      int b0 = 4 * i;
      if (b0 >= len) w = 0;
      else if (b0 + 4 > len) w &= (1u << (8 * (len - b0))) - 1;
      msg[i] = w;
    }
    __syncthreads();
    if (threadIdx.x == 0) b3_chunk_words(LdsSrc{msg}, (uint32_t)len, o1, 16);
    __syncthreads();
    if (threadIdx.x < 64) b3_hash_quad(msg, (uint32_t)len, o2, 16);
    __syncthreads();
    if (threadIdx.x < 16 && o1[threadIdx.x] != o2[threadIdx.x]) atomicAdd(bad, 1u);
  }
}

int main() {
  uint32_t* io;
  long long* cyc;
  hipMalloc(&io, 4096);
  hipMalloc(&cyc, 8);
  hipMemset(io, 1, 4096);
  const int iters = 200;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float ms;
  long long c;
  k_tr<<<1, 256>>>(io, 2, cyc);
  hipEventRecord(a);
  k_tr<<<1, 256>>>(io, iters, cyc);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("{\"transcript_step_us\": %.3f, \"cycles\": %.0f}\n", ms * 1e3 / iters, (double)c / iters);
  hipEventRecord(a);
  k_b3only<<<1, 64>>>(io, iters, cyc);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("{\"b3_compress_us\": %.3f, \"cycles\": %.0f}\n", ms * 1e3 / iters, (double)c / iters);
  hipEventRecord(a);
  k_b3quad<<<1, 64>>>(io, iters, cyc);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("{\"b3_quad_compress_us\": %.3f, \"cycles\": %.0f}\n", ms * 1e3 / iters, (double)c / iters);
  {
    uint32_t h[272];
    for (int i = 0; i < 272; i++) h[i] = 0x9E3779B9u * (i + 1) ^ (i << 7);
    uint32_t *dsrc, *dbad, bad = 0;
    hipMalloc(&dsrc, sizeof h);
    hipMalloc(&dbad, 4);
    hipMemcpy(dsrc, h, sizeof h, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 4);
    k_b3check<<<1, 256>>>(dsrc, dbad);
    hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
    printf("{\"b3_quad_vs_scalar_mismatches\": %u}\n", bad);
  }
  hipEventRecord(a);
  k_mul<<<1, 64>>>(io, 2000, cyc);
  hipEventRecord(b);
  hipEventSynchronize(b);
  hipEventElapsedTime(&ms, a, b);
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("{\"dependent_mul_us\": %.4f, \"cycles\": %.0f}\n", ms * 1e3 / 2000, (double)c / 2000);
  return 0;
}
