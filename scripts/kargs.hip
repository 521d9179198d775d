// kernarg size vs launch cost from an idle queue
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>
#include <algorithm>
struct Big { unsigned long long a[340]; };     // 2720 B
struct Small { unsigned long long a[32]; };    // 256 B
__global__ void kb(Big b, unsigned *o) { if (threadIdx.x == 0 && blockIdx.x == 0 && b.a[5] == 7) o[0] = 1; }
__global__ void ks(Small s, unsigned *o) { if (threadIdx.x == 0 && blockIdx.x == 0 && s.a[5] == 7) o[0] = 1; }
using C = std::chrono::steady_clock;
int main() {
  unsigned *o; hipMalloc(&o, 4);
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t e0, e1; hipEventCreateWithFlags(&e0, hipEventDisableSystemFence); hipEventCreateWithFlags(&e1, hipEventDisableSystemFence);
  Big b{}; Small sm{};
  for (int mode = 0; mode < 4; ++mode) {
    std::vector<double> enq, reg;
    for (int it = 0; it < 200; ++it) {
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      auto t0 = C::now();
      if (mode >= 2) hipEventRecord(e0, s);
      if (mode % 2 == 0) hipLaunchKernelGGL(kb, dim3(4096), dim3(256), 0, s, b, o);
      else hipLaunchKernelGGL(ks, dim3(4096), dim3(256), 0, s, sm, o);
      if (mode >= 2) hipEventRecord(e1, s);
      auto t1 = C::now();
      hipStreamSynchronize(s);
      auto t2 = C::now();
      enq.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      reg.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
    }
    std::sort(enq.begin(), enq.end()); std::sort(reg.begin(), reg.end());
    printf("%s%s: enqueue median %.2f p90 %.2f us; region median %.2f p90 %.2f us\n", mode % 2 ? "small(256B)" : "big(2720B)",
           mode >= 2 ? "+2 markers" : "", enq[100], enq[180], reg[100], reg[180]);
  }
  return 0;
}
