// memset_order_probe.hip -- is a null-stream hipMemset ordered before a
// kernel that a NON-BLOCKING stream launches after hipMemset returns?
//
// The question behind DESIGN.md 5.1 (the round-5 look-back abort): the
// workspace used to zero fresh look-back status words and tickets with a
// synchronous-API hipMemset on the null stream, and the kernels that read
// them run on the caller's stream (torch pool streams are non-blocking).
//
// Probe: a spin kernel keeps the null stream busy for ~300 ms; then
//   (a) hipMemset(buf, 0) on the null stream  -- how long does the host block?
//   (b) a reader kernel on a non-blocking stream copies buf -- does it see 0?
// The same for a freshly hipMalloc'ed buffer (the ensure() growth pattern),
// and for hipMemsetAsync on the reader's own stream (the fix).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

__global__ void spin(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(100);
}

__global__ void reader(const unsigned *buf, unsigned *out) { out[0] = buf[0]; }

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// mode 0: hipMemset (null stream) on an old buffer; 1: hipMalloc + hipMemset;
// 2: hipMalloc + hipMemsetAsync on the reader's stream
static void trial(int mode, hipStream_t rs, unsigned *out, unsigned *pinned) {
  unsigned *buf = nullptr;
  CK(hipMalloc(&buf, 4096));
  CK(hipMemset(buf, 0xab, 4096));
  CK(hipDeviceSynchronize());
  if (mode >= 1) {  // the ensure() pattern: free + malloc (often the same address) + zero
    CK(hipFree(buf));
    CK(hipMalloc(&buf, 4096));
  }
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, nullptr, 30000000ull);  // 300 ms at 100 MHz on the null stream
  const double t0 = now_ms();
  if (mode == 2)
    CK(hipMemsetAsync(buf, 0, 4096, rs));
  else
    CK(hipMemset(buf, 0, 4096));
  const double t1 = now_ms();
  hipLaunchKernelGGL(reader, dim3(1), dim3(1), 0, rs, buf, out);
  CK(hipMemcpyAsync(pinned, out, 4, hipMemcpyDeviceToHost, rs));
  CK(hipStreamSynchronize(rs));
  const double t2 = now_ms();
  CK(hipDeviceSynchronize());
  const char *names[3] = {"hipMemset(null stream), old buffer", "hipMalloc + hipMemset(null stream)",
                          "hipMalloc + hipMemsetAsync(reader stream)"};
  std::printf("{\"mode\": \"%s\", \"host_blocked_ms\": %.3f, \"reader_done_ms\": %.3f, \"reader_saw\": \"0x%08x\", "
              "\"ordered\": %s}\n",
              names[mode], t1 - t0, t2 - t0, pinned[0], pinned[0] == 0u ? "true" : "false");
  CK(hipFree(buf));
}

int main() {
  hipStream_t rs;
  CK(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking));
  unsigned *out = nullptr, *pinned = nullptr;
  CK(hipMalloc(&out, 4));
  CK(hipHostMalloc(reinterpret_cast<void **>(&pinned), 4));
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 3; ++mode) trial(mode, rs, out, pinned);
  CK(hipStreamDestroy(rs));
  return 0;
}
