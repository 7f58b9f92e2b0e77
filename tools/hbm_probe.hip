// hbm_probe.hip — measured HBM ceilings on this MI355X for the access shapes the codec uses.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip ; run: tools/hbm_probe
// read_unit:  one wave streams 4096 contiguous fp32 (16 float4 per lane issued back to back) = k_scan
// write_unit: one wave writes 4096 contiguous fp32 = k_decode's background stores
// copy_gs:    grid-stride float4 copy (reference point, MI355X_MICROARCH.md quotes ~6.3 TB/s)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void read_unit(const float4* __restrict__ in, size_t n4, float* sink) {
  const size_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const unsigned lane = threadIdx.x & 63;
  const size_t base = w * 1024;
  if (base >= n4) return;
  float4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = in[base + i * 64 + lane];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += v[i].x + v[i].y + v[i].z + v[i].w;
  if (s == 12345.678f) sink[0] = s;
}

__global__ __launch_bounds__(256) void read_gs(const float4* __restrict__ in, size_t n4, float* sink) {
  float s = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    float4 v = in[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.678f) sink[0] = s;
}

__global__ __launch_bounds__(256) void write_unit(float4* __restrict__ out, size_t n4) {
  const size_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
  const unsigned lane = threadIdx.x & 63;
  const size_t base = w * 1024;
  if (base >= n4) return;
#pragma unroll
  for (int i = 0; i < 16; ++i) out[base + i * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(256) void copy_gs(const float4* __restrict__ in, float4* __restrict__ out, size_t n4) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) out[i] = in[i];
}

int main() {
  const size_t bytes = (size_t)1 << 31;  // 2 GiB per buffer: far past the 256 MiB Infinity Cache
  const size_t n4 = bytes / 16;
  float4 *a, *b;
  float* sink;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned gu = (unsigned)((n4 / 1024 + 3) / 4);
  auto run = [&](const char* name, double bytes_moved, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"probe\": \"%s\", \"GBps\": %.1f, \"ms\": %.4f}\n", name, bytes_moved * R / (ms * 1e-3) / 1e9, ms / R);
    return 0;
  };
  run("read_unit_16KB_per_wave", (double)bytes, [&] { hipLaunchKernelGGL(read_unit, dim3(gu), dim3(256), 0, 0, a, n4, sink); });
  run("read_gridstride_2048x256", (double)bytes, [&] { hipLaunchKernelGGL(read_gs, dim3(2048), dim3(256), 0, 0, a, n4, sink); });
  run("write_unit_16KB_per_wave", (double)bytes, [&] { hipLaunchKernelGGL(write_unit, dim3(gu), dim3(256), 0, 0, b, n4); });
  run("copy_gridstride_2048x256", 2.0 * bytes, [&] { hipLaunchKernelGGL(copy_gs, dim3(2048), dim3(256), 0, 0, a, b, n4); });
  return 0;
}
