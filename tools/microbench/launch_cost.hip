// Host cost of a kernel launch on this box (tooling): hipLaunchKernel per call on one stream and on 8 streams in
// turn (HIP's 4 hardware queues shared), a kernel with a private segment, a 12-pointer argument list, and one
// hipGraphLaunch of a captured chain of 150 launches.  Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O2 -o tools/microbench/launch_cost tools/microbench/launch_cost.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_nop(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}
__global__ void k_args(int* a, int* b, int* c, int* d, int* e, int* f, int* g, int* h, int* i, int* j, int* k, int* l) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a[0] == 12345) b[1] = c[0] + d[0] + e[0] + f[0] + g[0] + h[0] + i[0] + j[0] + k[0] + l[0];
}
// a private array indexed by a runtime value: the compiler keeps it in scratch (in-bounds: idx < 256)
__global__ void k_scratch(int* p, int idx) {
  if (p[2] == 0 && idx < 0) return;  // (idx < 0: the gated form below, every lane leaves at once)
  volatile int loc[256];
  for (int t = 0; t < 256; ++t) loc[t] = t + threadIdx.x;
  if (p[0] == 12345) p[1] = loc[idx & 255];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int* d;
  if (hipMalloc(&d, 4096) != hipSuccess) return 1;
  (void)hipMemset(d, 0, 4096);
  std::vector<hipStream_t> st(8);
  for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const int N = 2000;
  auto run = [&](int nstreams, int kind) {
    for (int w = 0; w < 50; ++w) hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, st[w % nstreams], d);
    (void)hipDeviceSynchronize();
    const double t0 = now_us();
    for (int i = 0; i < N; ++i) {
      hipStream_t s = st[i % nstreams];
      if (kind == 0) hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s, d);
      if (kind == 1) hipLaunchKernelGGL(k_args, dim3(1), dim3(64), 0, s, d, d, d, d, d, d, d, d, d, d, d, d);
      if (kind == 2) hipLaunchKernelGGL(k_scratch, dim3(1), dim3(64), 0, s, d, i);
      if (kind == 3) hipLaunchKernelGGL(k_nop, dim3(782), dim3(128), 0, s, d);
      // a gated launch with a private segment that finds nothing to do (the isolation's launches on a passed batch)
      if (kind == 4) hipLaunchKernelGGL(k_scratch, dim3(1563), dim3(64), 0, s, d, -1);
      if (kind == 5) {
        if (i & 1) hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s, d);
        else hipLaunchKernelGGL(k_scratch, dim3(1563), dim3(64), 0, s, d, -1);
      }
    }
    const double t1 = now_us();
    (void)hipDeviceSynchronize();
    const double t2 = now_us();
    return std::make_pair((t1 - t0) / N, (t2 - t0) / N);
  };
  printf("{");
  const char* names[] = {"nop", "args12", "scratch", "nop_782wg", "scratch_dead_1563wg", "alt_nop_scratch_dead"};
  for (int kind = 0; kind < 6; ++kind)
    for (int ns : {1, 8}) {
      auto r = run(ns, kind);
      printf("\"%s_%dstreams\": {\"host_us\": %.2f, \"total_us\": %.2f}, ", names[kind], ns, r.first, r.second);
    }
  // graph of 150 launches on one stream
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(st[0], hipStreamCaptureModeRelaxed);
  for (int i = 0; i < 150; ++i) hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, st[0], d);
  (void)hipStreamEndCapture(st[0], &g);
  (void)hipGraphInstantiateWithFlags(&ge, g, 0);
  (void)hipGraphLaunch(ge, st[0]);
  (void)hipDeviceSynchronize();
  const double t0 = now_us();
  for (int i = 0; i < 20; ++i) (void)hipGraphLaunch(ge, st[0]);
  const double t1 = now_us();
  (void)hipDeviceSynchronize();
  const double t2 = now_us();
  printf("\"graph150\": {\"host_us_per_launch\": %.2f, \"total_us_per_launch\": %.2f}", (t1 - t0) / 20, (t2 - t0) / 20);
  printf("}\n");
  return 0;
}
