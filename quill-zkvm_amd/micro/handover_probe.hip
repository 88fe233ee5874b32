// Cross-stream hand-over probe (VERDICT r5 "next" 1): is a producer kernel's
// output, handed to a kernel on another HIP stream by hipEventRecord +
// hipStreamWaitEvent (no host synchronization), always complete and visible
// to the consumer?  Every word is checked, consumers are L1/L2-warm with the
// previous generation, and a third stream can add VALU load.
//
// Patterns (each a ping-pong of two non-blocking streams, like the MSM batch
// side streams and the context stream):
//   raw  : A writes gen g into X, B waits A's event and checks every word,
//          A waits B's event before writing g + 1 (the WAR edge)
//   waw  : A resets X to ~0 (the bucket scan's owner reset), B waits and marks
//          every 5th word with g (the accumulation's flushes), A waits and
//          checks the whole of X (a stale dirty line of the reset written back
//          after B's mark would show as ~0)
//   host : pageable H2D copy on a copy stream, the event recycled right after
//          the wait and re-recorded by the next taker (msm_host's pattern)
// Event policies: held (a fresh event per hand-over, destroyed at the end),
// lifo (one pool, an event pushed back right after its wait and re-recorded
// by the next hand-over: ctx->ev_get()'s order).  d2h: a 16-B D2H copy into
// pinned memory is the producer stream's last command before the record (the
// quotient batch's h_y copy and the bucketing's plan-word copy).
//
// hipcc --offload-arch=gfx950 -O3 -o micro/handover_probe micro/handover_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                    \
    }                                                                             \
  } while (0)

__device__ __forceinline__ uint32_t val(size_t i, uint32_t g) {
  uint32_t h = (uint32_t)i * 0x9e3779b1u ^ g * 0x85ebca6bu;
  h ^= h >> 15;
  return h * 0xc2b2ae35u + g;
}

// producer: `spin` dependent multiplies first (a long kernel, so a consumer
// that starts early sees the previous generation), then the stores
__global__ void k_write(uint32_t* x, size_t n, uint32_t g, int spin) {
  uint32_t a = threadIdx.x + 1;
  for (int k = 0; k < spin; k++) a = a * 0x2545f491u + 7u;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    x[i] = val(i, g) + (a == 0x12345u ? 1u : 0u);
}

__global__ void k_check(const uint32_t* x, size_t n, uint32_t g, unsigned* err) {
  unsigned bad = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    bad += x[i] != val(i, g);
  if (bad) atomicAdd(err, bad);
}

__global__ void k_reset(uint32_t* x, size_t n, int spin) {
  uint32_t a = threadIdx.x + 1;
  for (int k = 0; k < spin; k++) a = a * 0x2545f491u + 7u;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    x[i] = 0xffffffffu - (a == 0x12345u ? 1u : 0u);
}

__global__ void k_mark(uint32_t* x, size_t n, uint32_t g) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    if (i % 5 == 0) x[i] = g;
}

__global__ void k_check_marks(const uint32_t* x, size_t n, uint32_t g, unsigned* err) {
  unsigned bad = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    bad += x[i] != (i % 5 == 0 ? g : 0xffffffffu);
  if (bad) atomicAdd(err, bad);
}

__global__ void k_busy(uint32_t* sink, int iters) {
  uint32_t a = threadIdx.x, b = blockIdx.x | 1;
  for (int k = 0; k < iters; k++) {
    a = a * b + 0x3c6ef372u;
    b = b * 0x2545f491u + a;
  }
  if (a == 0x12345u && b == 7u) sink[0] = a;
}

struct Pool {  // ctx->ev_get() / event_pool order (LIFO)
  std::vector<hipEvent_t> v;
  unsigned flags;
  hipEvent_t get() {
    if (!v.empty()) {
      hipEvent_t e = v.back();
      v.pop_back();
      return e;
    }
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, flags));
    return e;
  }
};

struct Res {
  unsigned long long bad_words = 0;
  int bad_iters = 0;
};

// one hand-over from stream s to stream t: record on s, t waits
static void handover(hipStream_t s, hipStream_t t, Pool& pool, bool lifo, std::vector<hipEvent_t>& held) {
  hipEvent_t e = pool.get();
  CK(hipEventRecord(e, s));
  CK(hipStreamWaitEvent(t, e, 0));
  if (lifo)
    pool.v.push_back(e);
  else
    held.push_back(e);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int spin = argc > 2 ? atoi(argv[2]) : 20000;
  hipStream_t A, B, C;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
  const size_t maxn = (size_t)4 << 20;
  uint32_t *X, *sink;
  unsigned* err;
  CK(hipMalloc(&X, maxn * 4));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&err, 4 * 64));
  uint32_t* pin;
  CK(hipHostMalloc(&pin, 4096, hipHostMallocDefault));
  std::vector<uint32_t> pageable(maxn);
  const char* pats[] = {"raw", "waw"};
  for (const char* pat : pats)
    for (size_t n : {(size_t)1 << 16, maxn})
      for (int lifo = 0; lifo < 2; lifo++)
        for (int d2h = 0; d2h < 2; d2h++)
          for (int load = 0; load < 2; load++)
            for (unsigned fl : {0u, (unsigned)hipEventDisableTiming}) {
              CK(hipDeviceSynchronize());
              CK(hipMemset(err, 0, 4 * 64));
              CK(hipMemset(X, 0, maxn * 4));
              CK(hipDeviceSynchronize());
              Pool pool{{}, fl};
              std::vector<hipEvent_t> held;
              std::vector<unsigned> herr(iters, 0);
              const unsigned grid = (unsigned)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
              for (int it = 0; it < iters; it++) {
                const uint32_t g = (uint32_t)it + 1;
                if (load && it % 8 == 0) hipLaunchKernelGGL(k_busy, dim3(512), dim3(256), 0, C, sink, 200000);
                unsigned* e = err + (it & 63);
                if (pat[0] == 'r') {
                  hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, A, X, n, g, spin);
                  if (d2h) CK(hipMemcpyAsync(pin + 4 * (it & 63), X, 16, hipMemcpyDeviceToHost, A));
                  handover(A, B, pool, lifo, held);
                  hipLaunchKernelGGL(k_check, dim3(grid), dim3(256), 0, B, X, n, g, e);
                  handover(B, A, pool, lifo, held);
                } else {
                  hipLaunchKernelGGL(k_reset, dim3(grid), dim3(256), 0, A, X, n, spin);
                  if (d2h) CK(hipMemcpyAsync(pin + 4 * (it & 63), X, 16, hipMemcpyDeviceToHost, A));
                  handover(A, B, pool, lifo, held);
                  hipLaunchKernelGGL(k_mark, dim3(grid), dim3(256), 0, B, X, n, g);
                  handover(B, A, pool, lifo, held);
                  hipLaunchKernelGGL(k_check_marks, dim3(grid), dim3(256), 0, A, X, n, g, e);
                }
                if (it % 64 == 63) {  // read the 64 error words, every 64 iterations
                  unsigned h[64];
                  CK(hipStreamSynchronize(A));
                  CK(hipStreamSynchronize(B));
                  CK(hipMemcpy(h, err, sizeof(h), hipMemcpyDeviceToHost));
                  CK(hipMemset(err, 0, sizeof(h)));
                  for (int k = 0; k < 64; k++) herr[it - 63 + k] = h[k];
                }
              }
              CK(hipDeviceSynchronize());
              Res r;
              for (int it = 0; it < iters - iters % 64; it++)
                if (herr[it]) {
                  r.bad_iters++;
                  r.bad_words += herr[it];
                }
              printf("pat=%s n=%zu events=%s d2h=%d load=%d flags=%s iters=%d bad_iters=%d bad_words=%llu\n",
                     pat, n, lifo ? "lifo" : "held", d2h, load, fl ? "notiming" : "default",
                     iters - iters % 64, r.bad_iters, r.bad_words);
              fflush(stdout);
              for (hipEvent_t ev : held) CK(hipEventDestroy(ev));
              for (hipEvent_t ev : pool.v) CK(hipEventDestroy(ev));
            }
  // host pattern (msm_host): pageable upload on a copy stream, event recycled
  // right after the wait, the consumer on the other stream
  for (int lifo = 0; lifo < 2; lifo++) {
    CK(hipDeviceSynchronize());
    CK(hipMemset(err, 0, 4 * 64));
    Pool pool{{}, 0};
    std::vector<hipEvent_t> held;
    const size_t n = (size_t)1 << 20;
    unsigned long long bad = 0;
    int bad_it = 0;
    const int hit = iters / 8;
    for (int it = 0; it < hit; it++) {
      const uint32_t g = (uint32_t)it + 1;
      for (size_t i = 0; i < n; i++) {
        uint32_t h = (uint32_t)i * 0x9e3779b1u ^ g * 0x85ebca6bu;
        h ^= h >> 15;
        pageable[i] = h * 0xc2b2ae35u + g;
      }
      handover(B, A, pool, lifo, held);  // uploads after the consumer's previous read
      CK(hipMemcpyAsync(X, pageable.data(), n * 4, hipMemcpyHostToDevice, A));
      handover(A, B, pool, lifo, held);
      hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, B, X, n, g, err);
      // the next taker re-records the recycled event on the consumer stream
      hipEvent_t t = pool.get();
      CK(hipEventRecord(t, B));
      if (lifo)
        pool.v.push_back(t);
      else
        held.push_back(t);
      unsigned h = 0;
      CK(hipStreamSynchronize(B));
      CK(hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost));
      if (h) {
        bad_it++;
        bad += h;
        CK(hipMemset(err, 0, 4));
      }
    }
    printf("pat=host n=%zu events=%s iters=%d bad_iters=%d bad_words=%llu\n", n,
           lifo ? "lifo" : "held", hit, bad_it, bad);
    fflush(stdout);
    for (hipEvent_t ev : held) CK(hipEventDestroy(ev));
    for (hipEvent_t ev : pool.v) CK(hipEventDestroy(ev));
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
