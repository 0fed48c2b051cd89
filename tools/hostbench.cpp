// hostbench.cpp -- host<->device transfer ceilings on the GPU box (not product).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 2; } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
  const size_t n = 1ull << 30;
  std::vector<uint8_t> page(n, 1);
  void *pin, *pin2, *d, *d2;
  CK(hipHostMalloc(&pin, n, 0)); CK(hipHostMalloc(&pin2, n, 0));
  CK(hipMalloc(&d, n)); CK(hipMalloc(&d2, n));
  printf("hw threads %u\n", std::thread::hardware_concurrency());
  for (int th : {1, 2, 4, 8, 16, 32}) {
    double best = 1e9;
    for (int r = 0; r < 3; ++r) {
      double t = now();
      std::vector<std::thread> v;
      size_t per = n / th;
      for (int i = 0; i < th; ++i) v.emplace_back([&, i] { memcpy((uint8_t*)pin + i * per, page.data() + i * per, per); });
      for (auto &x : v) x.join();
      best = std::min(best, now() - t);
    }
    printf("memcpy pageable->pinned %2d threads: %6.1f GB/s\n", th, n / best / 1e9);
  }
  hipStream_t a, b; CK(hipStreamCreate(&a)); CK(hipStreamCreate(&b));
  auto tm = [&](const char *name, auto fn) {
    fn(); CK(hipDeviceSynchronize());
    double t = now(); for (int r = 0; r < 3; ++r) fn(); CK(hipDeviceSynchronize());
    printf("%-28s %6.1f GB/s per direction\n", name, 3.0 * n / (now() - t) / 1e9);
    return 0;
  };
  tm("H2D pinned", [&] { (void)hipMemcpyAsync(d, pin, n, hipMemcpyHostToDevice, a); });
  tm("D2H pinned", [&] { (void)hipMemcpyAsync(pin2, d2, n, hipMemcpyDeviceToHost, a); });
  tm("H2D+D2H concurrent", [&] { (void)hipMemcpyAsync(d, pin, n, hipMemcpyHostToDevice, a); (void)hipMemcpyAsync(pin2, d2, n, hipMemcpyDeviceToHost, b); });
  tm("H2D pageable", [&] { (void)hipMemcpyAsync(d, page.data(), n, hipMemcpyHostToDevice, a); });
  return 0;
}
