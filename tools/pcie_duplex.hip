// pcie_duplex.hip — PCIe copy rates of one MI355X from page-locked host memory (VERDICT
// r4 next #6): H2D alone, D2H alone and both at once on two streams through hipMemcpyAsync, for
// each hipHostMalloc flavour (the engine's event buffer and the caller's record buffers are
// hipHostMallocDefault), and the same through a kernel that reads / writes mapped host memory
// (16-B lanes).  One JSON line.
// Build: hipcc --offload-arch=gfx950 -O2 tools/pcie_duplex.hip -o tools/pcie_duplex
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

// dst[i] = src[i], 16 B per lane, grid-stride (either side may be host-mapped memory)
__global__ void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x)
    dst[i] = src[i];
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t nb = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 256) << 20;
  const int reps = 5;
  void *d_in, *d_out;
  CK(hipMalloc(&d_in, nb));
  CK(hipMalloc(&d_out, nb));
  CK(hipMemset(d_out, 2, nb));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  auto best = [&](auto fn) {
    double b = 1e9;
    for (int r = 0; r < reps; ++r) {
      CK(hipDeviceSynchronize());
      const double t = now_s();
      fn();
      CK(hipDeviceSynchronize());
      b = std::min(b, now_s() - t);
    }
    return nb / b / 1e9;
  };
  std::string out = "{\"MiB\": " + std::to_string(nb >> 20);
  const struct { const char* name; unsigned flags; } kinds[] = {
      {"default", hipHostMallocDefault}, {"mapped", hipHostMallocMapped},
      {"coherent", hipHostMallocCoherent}, {"noncoherent", hipHostMallocNonCoherent}};
  for (const auto& k : kinds) {
    void *h_in, *h_out;
    CK(hipHostMalloc(&h_in, nb, k.flags));
    CK(hipHostMalloc(&h_out, nb, k.flags));
    std::memset(h_in, 1, nb);
    std::memset(h_out, 0, nb);
    const double h2d = best([&] { CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, s1)); });
    const double d2h = best([&] { CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, s2)); });
    const double both = best([&] {
      CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, s1));
      CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, s2));
    });
    char buf[256];
    std::snprintf(buf, sizeof buf, ", \"%s\": {\"h2d_GBps\": %.2f, \"d2h_GBps\": %.2f, \"both_GBps_each\": %.2f}", k.name,
                  h2d, d2h, both);
    out += buf;
    if (k.flags == hipHostMallocMapped) {
      void *hm_in, *hm_out;
      CK(hipHostGetDevicePointer(&hm_in, h_in, 0));
      CK(hipHostGetDevicePointer(&hm_out, h_out, 0));
      const size_t n16 = nb / 16;
      const double kh2d = best([&] { k_copy16<<<1024, 256, 0, s1>>>((const uint4*)hm_in, (uint4*)d_in, n16); });
      const double kd2h = best([&] { k_copy16<<<1024, 256, 0, s2>>>((const uint4*)d_out, (uint4*)hm_out, n16); });
      const double kboth = best([&] {
        k_copy16<<<1024, 256, 0, s1>>>((const uint4*)hm_in, (uint4*)d_in, n16);
        k_copy16<<<1024, 256, 0, s2>>>((const uint4*)d_out, (uint4*)hm_out, n16);
      });
      std::snprintf(buf, sizeof buf, ", \"kernel_mapped\": {\"h2d_GBps\": %.2f, \"d2h_GBps\": %.2f, \"both_GBps_each\": %.2f}",
                    kh2d, kd2h, kboth);
      out += buf;
    }
    if (k.flags == hipHostMallocDefault) {  // the same buffers, copies of kind hipMemcpyDefault
      const double h2 = best([&] { CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyDefault, s1)); });
      const double d2 = best([&] { CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDefault, s2)); });
      char b2[160];
      std::snprintf(b2, sizeof b2, ", \"default_kind\": {\"h2d_GBps\": %.2f, \"d2h_GBps\": %.2f}", h2, d2);
      out += b2;
    }
    CK(hipHostFree(h_in));
    CK(hipHostFree(h_out));
  }
  {  // malloc'd memory registered with hipHostRegister (how some hosts pin their buffers)
    void *h_in = nullptr, *h_out = nullptr;
    if (posix_memalign(&h_in, 4096, nb) || posix_memalign(&h_out, 4096, nb)) return 1;
    std::memset(h_in, 1, nb);
    std::memset(h_out, 0, nb);
    CK(hipHostRegister(h_in, nb, hipHostRegisterDefault));
    CK(hipHostRegister(h_out, nb, hipHostRegisterDefault));
    const double h2d = best([&] { CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, s1)); });
    const double d2h = best([&] { CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, s2)); });
    const double both = best([&] {
      CK(hipMemcpyAsync(d_in, h_in, nb, hipMemcpyHostToDevice, s1));
      CK(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, s2));
    });
    char buf[200];
    std::snprintf(buf, sizeof buf, ", \"registered\": {\"h2d_GBps\": %.2f, \"d2h_GBps\": %.2f, \"both_GBps_each\": %.2f}",
                  h2d, d2h, both);
    out += buf;
    CK(hipHostUnregister(h_in));
    CK(hipHostUnregister(h_out));
    free(h_in);
    free(h_out);
  }
  std::printf("%s}\n", out.c_str());
  return 0;
}
