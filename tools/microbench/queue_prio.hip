// Do high-priority streams get hardware queues of their own (beside GPU_MAX_HW_QUEUES normal ones)?  (tooling)
// Four normal streams each run a 1-workgroup kernel that spins ~60 ms; then a short kernel goes to (a) a fifth normal
// stream and (b) a high-priority stream.  A short kernel on a queue shared with a spinning one completes only after it.
//   hipcc --offload-arch=gfx950 -O2 -o tools/microbench/queue_prio tools/microbench/queue_prio.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_spin(long long ticks, int* out) {
  const long long t0 = wall_clock64();
  long long t = t0;
  while (t - t0 < ticks) t = wall_clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = (int)(t - t0);
}
__global__ void k_short(int* out) {
  if (threadIdx.x == 0) out[0] = 1;
}
static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
  int* d;
  if (hipMalloc(&d, 4096) != hipSuccess) return 1;
  int rate_khz = 0;
  (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
  const long long ticks = (long long)rate_khz * 60;  // ~60 ms
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  hipStream_t s[6], sp;
  for (auto& x : s) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
  (void)hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, hi);
  // bind every stream to its queue first (queues are bound at first dispatch)
  for (auto& x : s) hipLaunchKernelGGL(k_short, dim3(1), dim3(64), 0, x, d + 100);
  hipLaunchKernelGGL(k_short, dim3(1), dim3(64), 0, sp, d + 100);
  (void)hipDeviceSynchronize();
  double res[2];
  for (int which = 0; which < 2; ++which) {
    for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[i], ticks, d + 8 * i);
    const double t0 = now_ms();
    hipStream_t tgt = which == 0 ? s[4] : sp;
    hipLaunchKernelGGL(k_short, dim3(1), dim3(64), 0, tgt, d + 64);
    (void)hipStreamSynchronize(tgt);
    res[which] = now_ms() - t0;
    (void)hipDeviceSynchronize();
  }
  printf("{\"priority_range\": [%d, %d], \"wallclock_khz\": %d, \"short_on_5th_normal_ms\": %.2f, "
         "\"short_on_high_priority_ms\": %.2f}\n", lo, hi, rate_khz, res[0], res[1]);
  return 0;
}
