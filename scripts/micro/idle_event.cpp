// Does an event recorded on an idle stream take its timestamp when the host records it, or later?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
#include <thread>
__global__ void k_spin(float *p, int n) {
  float x = p[threadIdx.x];
  for (int i = 0; i < n; ++i) x = x * 1.0000001f + 1e-7f;
  p[threadIdx.x] = x;
}
int main() {
  float *p;
  (void)hipMalloc(&p, 4096);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipEvent_t e0, e1, e2;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); (void)hipEventCreate(&e2);
  k_spin<<<1, 64, 0, s>>>(p, 1000);
  (void)hipStreamSynchronize(s);
  for (int sleep_us : {0, 2000, 5000}) {
    for (int mode = 0; mode < 2; ++mode) {
      (void)hipEventRecord(e0, s);
      std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
      void *q = nullptr;
      if (mode) (void)hipMalloc(&q, 1ull << 31); // 2 GiB between the two records
      (void)hipEventRecord(e1, s);
      k_spin<<<1, 64, 0, s>>>(p, 200000);
      (void)hipEventRecord(e2, s);
      (void)hipEventSynchronize(e2);
      float a, b;
      (void)hipEventElapsedTime(&a, e0, e2);
      (void)hipEventElapsedTime(&b, e1, e2);
      printf("sleep %d us malloc %d: e0->e2 %.3f ms  e1->e2 %.3f ms\n", sleep_us, mode, a, b);
      if (q) (void)hipFree(q);
    }
  }
  return 0;
}
