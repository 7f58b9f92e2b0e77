// lds_probe.hip — does an exec-masked ds_read_b128 cost the LDS less than a full-wave one?
// (k_aggregate reads back a per-wave 8 KiB tile per client although only ~20 of its 512 float4 slots hold a
// kept value; if masked reads are cheap, reading only the slots a lane's mask names would cut that traffic.)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/lds_probe tools/lds_probe.hip
// Each wave: ITERS rounds of 8 float4 reads from its own LDS tile; lanes >= ACTIVE are masked off through a
// branch on a runtime value (the compiler cannot speculate the reads). Prints one JSON line per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE>  // 0: all lanes read; 1: lanes with (mask >> lane) & 1 read (branch); 2: no reads (VALU only)
__global__ __launch_bounds__(256) void probe(float4* out, const uint64_t* masks, int iters) {
  __shared__ float4 tile[4][512];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int i = 0; i < 8; ++i) tile[wv][i * 64 + lane] = make_float4(lane, i, wv, 1.0f);
  __builtin_amdgcn_wave_barrier();
  const uint64_t m = masks[blockIdx.x & 255];
  const bool on = (m >> lane) & 1ull;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < iters; ++r) {
    const uint32_t rot = (uint32_t)r & 7u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
      if (MODE == 0 || (MODE == 1 && on)) d = tile[wv][((i + rot) & 7) * 64 + lane];
      acc.x += d.x;
      acc.y += d.y * 1.0001f;
      acc.z += d.z;
      acc.w += d.w;
    }
    __builtin_amdgcn_wave_barrier();
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const int blocks = 256 * 16, iters = 512;
  float4* out;
  uint64_t* masks;
  CK(hipMalloc(&out, sizeof(float4) * blocks * 256));
  CK(hipMalloc(&masks, 8 * 256));
  uint64_t hm[256];
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int active : {64, 16, 4, 1}) {
    for (int i = 0; i < 256; ++i) {  // `active` lanes spread over the wave
      uint64_t m = 0;
      for (int j = 0; j < active; ++j) m |= 1ull << ((j * 64 / active + i) & 63);
      hm[i] = m;
    }
    CK(hipMemcpy(masks, hm, sizeof(hm), hipMemcpyHostToDevice));
    auto run = [&](const char* name, auto launch) {
      launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int k = 0; k < 5; ++k) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double reads = 5.0 * blocks * 4 * iters * 8;  // wave-level ds_read_b128 instructions
      printf("{\"variant\": \"%s\", \"active_lanes\": %d, \"ms\": %.4f, \"ns_per_wave_read_per_CU\": %.3f}\n", name,
             active, ms / 5, ms * 1e6 / (reads / 256.0));
      return 0;
    };
    run("masked", [&] { hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(256), 0, 0, out, masks, iters); });
    if (active == 64) {
      run("full", [&] { hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(256), 0, 0, out, masks, iters); });
      run("valu_only", [&] { hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(256), 0, 0, out, masks, iters); });
    }
  }
  return 0;
}
