// queue_map.hip — which HIP streams share a hardware queue (the four-queue layout).
//
// Streams beyond GPU_MAX_HW_QUEUES share hardware queues, and two streams on one queue run one after
// the other.  This creates `n` non-blocking streams in order (after an optional null-stream launch,
// as torch's first use of the device does) and, for every ordered pair (a, b), launches a ~2 ms spin
// kernel on a and then an empty kernel on b: b done long before a means b has a queue of its own.
// Prints the matrix (1 = b waited for a) and the groups of streams that share a queue.
//   hipcc --offload-arch=gfx950 -O2 tools/queue_map.hip -o tools/queue_map
//   GPU_MAX_HW_QUEUES=4 ./tools/queue_map 8 [null]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void spin(unsigned long long cycles, int* sink) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) sink[0] = 1;
}
__global__ void empty(int* sink) {
  if (threadIdx.x == 0) sink[1] = 2;
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 8;
  const bool null_first = argc > 2 && std::strcmp(argv[2], "null") == 0;
  int* sink = nullptr;
  CK(hipMalloc(&sink, 64));
  if (null_first) {  // (torch's first device use: work on the null stream)
    empty<<<1, 64>>>(sink);
    CK(hipDeviceSynchronize());
  }
  std::vector<hipStream_t> s(n);
  for (int i = 0; i < n; ++i) CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0));
  const unsigned long long cycles = static_cast<unsigned long long>(clk_khz) * 2;  // ~2 ms
  hipEvent_t done;
  CK(hipEventCreate(&done));
  std::vector<int> m(n * n, 0);
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b) {
      if (a == b) continue;
      CK(hipDeviceSynchronize());
      spin<<<1, 64, 0, s[a]>>>(cycles, sink);
      empty<<<1, 64, 0, s[b]>>>(sink);
      CK(hipEventRecord(done, s[b]));
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipEventSynchronize(done));
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      m[a * n + b] = ms > 1.0 ? 1 : 0;
    }
  CK(hipDeviceSynchronize());
  std::printf("GPU_MAX_HW_QUEUES=%s null_first=%d streams=%d\n", std::getenv("GPU_MAX_HW_QUEUES") ? std::getenv("GPU_MAX_HW_QUEUES") : "(unset)",
              null_first ? 1 : 0, n);
  for (int a = 0; a < n; ++a) {
    for (int b = 0; b < n; ++b) std::printf("%c", a == b ? '.' : m[a * n + b] ? '1' : '0');
    std::printf("\n");
  }
  std::vector<int> grp(n, -1);
  int ng = 0;
  for (int a = 0; a < n; ++a) {
    if (grp[a] >= 0) continue;
    grp[a] = ng;
    for (int b = a + 1; b < n; ++b)
      if (m[a * n + b] && m[b * n + a]) grp[b] = ng;
    ++ng;
  }
  std::printf("groups:");
  for (int g = 0; g < ng; ++g) {
    std::printf(" {");
    for (int a = 0; a < n; ++a)
      if (grp[a] == g) std::printf(" %d", a);
    std::printf(" }");
  }
  std::printf("\n");
  return 0;
}
