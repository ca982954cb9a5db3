// Probe (not product): what makes the next kernel start ~6 us after K4 ends?  A producer kernel of each
// kind below, then a one-block consumer that stamps its start; the producer's waves stamp their end
// (atomic max of s_memrealtime, 100 MHz).  gap = consumer start - last producer wave end.
//   hipcc -O3 --offload-arch=gfx950 gap_probe.hip -o gap_probe
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"
#include <cstdio>
#include <cstdint>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void consumer(unsigned long long* t) {  // t[1]: its start
  if (threadIdx.x == 0) t[1] = __builtin_amdgcn_s_memrealtime();
}

// mode 0: nt stores, 1: plain stores, 2: loads only (sum written once per wave), 3: no memory (grid only)
template <int MODE>
__global__ __launch_bounds__(256) void producer(f4* __restrict__ buf, size_t n16, unsigned long long* t, int per_wg) {
  const size_t base = (size_t)blockIdx.x * per_wg * 256 + threadIdx.x;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < per_wg; ++k) {
    const size_t i = base + (size_t)k * 256;
    if (i >= n16) break;
    if constexpr (MODE == 0) __builtin_nontemporal_store(f4{1.f, 2.f, 3.f, (float)k}, &buf[i]);
    if constexpr (MODE == 1) buf[i] = f4{1.f, 2.f, 3.f, (float)k};
    if constexpr (MODE == 2) { const f4 v = __builtin_nontemporal_load(&buf[i]); acc.x += v.x; acc.y += v.y; }
  }
  if constexpr (MODE == 2) if (acc.x == 12345.f) buf[base] = acc;
  __syncthreads();  // every wave of the workgroup done; one plain store per workgroup (no atomic hot spot)
  if (threadIdx.x == 0) t[2 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

int main() {
  const size_t bytes = (size_t)512 << 20;  // 0.5 GB, like K4's dual-output writes at cfg3 fp32
  const size_t n16 = bytes / 16;
  f4* buf;
  unsigned long long* t;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&t, (2 + 32768) * 8) != hipSuccess) return 1;
  unsigned long long* h = new unsigned long long[2 + 32768];
  hipMemset(buf, 0, bytes);
  const char* names[4] = {"nt stores 0.5 GB", "plain stores 0.5 GB", "nt loads 0.5 GB", "no memory"};
  for (int wgs : {2048, 32768}) {
    const int per_wg = (int)((n16 + (size_t)wgs * 256 - 1) / ((size_t)wgs * 256));
    for (int mode = 0; mode < 4; ++mode) {
      double sum = 0, sum_dur = 0;
      const int reps = 20;
      for (int r = 0; r < reps + 2; ++r) {
        hipMemset(t, 0, (2 + 32768) * 8);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL(producer<0>, dim3(wgs), dim3(256), 0, 0, buf, n16, t, per_wg);
        if (mode == 1) hipLaunchKernelGGL(producer<1>, dim3(wgs), dim3(256), 0, 0, buf, n16, t, per_wg);
        if (mode == 2) hipLaunchKernelGGL(producer<2>, dim3(wgs), dim3(256), 0, 0, buf, n16, t, per_wg);
        if (mode == 3) hipLaunchKernelGGL(producer<3>, dim3(wgs), dim3(256), 0, 0, buf, n16, t, per_wg);
        hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, 0, t);
        hipEventRecord(e1);
        hipDeviceSynchronize();
        hipMemcpy(h, t, (2 + wgs) * 8, hipMemcpyDeviceToHost);
        h[0] = 0;
        for (int w = 0; w < wgs; ++w) h[0] = h[2 + w] > h[0] ? h[2 + w] : h[0];
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2) { sum += (double)(long long)(h[1] - h[0]) * 0.01; sum_dur += ms; }
        hipEventDestroy(e0);
        hipEventDestroy(e1);
      }
      printf("%6d WGs  %-22s  gap last-wave-end -> next kernel start %6.2f us   (pair %7.1f us)\n", wgs,
             names[mode], sum / reps, sum_dur / reps * 1e3);
    }
  }
  return 0;
}
