// D2H copy rate into host memory of each hipHostMalloc flavour (the fetch path's 10.2 MB of
// strings per metric batch): hipcc --offload-arch=gfx950 -O2 d2h_rate.hip -o d2h_rate
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
int main() {
  const size_t n = 10240000;
  void* d = nullptr;
  if (hipMalloc(&d, n) != hipSuccess) return 1;
  hipMemset(d, 1, n);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  struct F { const char* name; unsigned flags; };
  const F fl[] = {{"default", hipHostMallocDefault}, {"noncoherent", hipHostMallocNonCoherent},
                  {"coherent", hipHostMallocCoherent}};
  for (const F& f : fl) {
    void* h = nullptr;
    if (hipHostMalloc(&h, n, f.flags) != hipSuccess) { std::printf("%s: alloc failed\n", f.name); continue; }
    for (int split = 1; split <= 2; ++split) {
      double best = 1e9;
      for (int it = 0; it < 10; ++it) {
        auto t0 = std::chrono::steady_clock::now();
        for (int q = 0; q < split; ++q)
          hipMemcpyAsync((char*)h + q * (n / split), (char*)d + q * (n / split), n / split, hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt < best) best = dt;
      }
      std::printf("%-12s %d copies: %.3f ms, %.1f GB/s\n", f.name, split, best * 1e3, n / best / 1e9);
    }
    hipHostFree(h);
  }
  std::vector<char> pg(n);
  double best = 1e9;
  for (int it = 0; it < 5; ++it) {
    auto t0 = std::chrono::steady_clock::now();
    hipMemcpy(pg.data(), d, n, hipMemcpyDeviceToHost);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt < best) best = dt;
  }
  std::printf("pageable     1 copy : %.3f ms, %.1f GB/s\n", best * 1e3, n / best / 1e9);
  return 0;
}
