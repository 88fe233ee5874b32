// Per-XCD speed probe (micro benchmark): the same VALU-only work and the same
// streaming read per block, blocks spread over all XCDs (block b -> XCD b % 8);
// prints per-XCC block durations so a slower half of the chip (clock or memory
// path) shows up.  hipcc --offload-arch=gfx950 -O3 -o micro/xcd_probe micro/xcd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void k_valu(unsigned long long* out, int iters, unsigned seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = a ^ 0x9e3779b9u;
  uint64_t x = a, y = b, z = a ^ b, w = a + b;
  const unsigned long long t0 = wall_clock64();
  for (int i = 0; i < iters; i++) {
    x = (uint64_t)(uint32_t)x * a + y;
    y = (uint64_t)(uint32_t)y * b + z;
    z = (uint64_t)(uint32_t)z * a + w;
    w = (uint64_t)(uint32_t)w * b + x;
  }
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = t1 - t0;
    out[3 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg(6164);
    out[3 * blockIdx.x + 2] = x ^ y ^ z ^ w;
  }
}

__global__ void k_stream(const uint4* __restrict__ src, size_t per, unsigned long long* out) {
  const uint4* p = src + (size_t)blockIdx.x * per;
  uint32_t acc = 0;
  const unsigned long long t0 = wall_clock64();
  for (size_t i = threadIdx.x; i < per; i += blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  __syncthreads();
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[3 * blockIdx.x] = t1 - t0;
    out[3 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg(6164);
  }
  if (acc == 0x12345678u) out[3 * blockIdx.x + 2] = acc;
}

static void report(const char* name, const std::vector<unsigned long long>& h, int nb) {
  std::vector<std::vector<double>> by(16);
  for (int b = 0; b < nb; b++) by[h[3 * b + 1] & 15].push_back(h[3 * b] * 0.01);
  for (int x = 0; x < 16; x++) {
    auto& v = by[x];
    if (v.empty()) continue;
    std::sort(v.begin(), v.end());
    printf("%s XCC %d: blocks=%zu us min/p50/max = %.1f / %.1f / %.1f\n", name, x, v.size(), v[0],
           v[v.size() / 2], v.back());
  }
}

int main() {
  const int nb = 512;
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * 3 * nb);
  std::vector<unsigned long long> h(3 * nb);
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_valu, dim3(nb), dim3(256), 0, 0, d, 20000, 1u);
    hipDeviceSynchronize();
  }
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  report("valu", h, nb);
  const size_t per = (size_t)1 << 18;  // 4 MiB per block
  uint4* src;
  hipMalloc(&src, sizeof(uint4) * per * nb);
  hipMemset(src, 1, sizeof(uint4) * per * nb);
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_stream, dim3(nb), dim3(256), 0, 0, src, per, d);
    hipDeviceSynchronize();
  }
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  report("stream", h, nb);
  return 0;
}
