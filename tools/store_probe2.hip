// Write-bandwidth probe, round 3: why one 1-KiB store per wave (flat1, 6.9 TB/s) beats a wave writing its
// whole 16-KiB unit (5.4-6.4 TB/s), and whether a decode-shaped wave (dependent metadata loads, then ONE row
// store) keeps flat1's rate. Per buffer size (MiB args), one launch timed over 20 repeats:
//   flat1       one float4 per thread, 256-thread blocks, grid n/4/256 (elementwise style)
//   flat1_nt    the same, non-temporal buffer store
//   flat1_b1024 the same with 1024-thread blocks
//   n2_far      2 stores per wave, the second 64 MiB away (per-wave contiguity vs count of stores)
//   row_dep3    one row (1 KiB) per wave after 3 dependent L2-resident loads (unit record -> bounds ->
//               entry), value merged from the loaded entry: k_decode's work per row, one store per wave
//   row_dep3_x4 the same, 4 rows per wave (the rows of a quarter unit)
//   unit16_x    k_decode's current pattern: one wave per 16 KiB unit, XCD-aware order, NT buffer stores
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__global__ __launch_bounds__(256) void flat1(float4* __restrict__ out, size_t n4, float v) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) out[i] = make_float4(v, v, v, v);
}

__global__ __launch_bounds__(256) void flat1_nt(float4* __restrict__ out, size_t n4, float v) {
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w * 64 >= n4) return;
  const u4v a = {__float_as_uint(v), __float_as_uint(v), __float_as_uint(v), __float_as_uint(v)};
  __builtin_amdgcn_raw_buffer_store_b128(a, rsrc(out + w * 64, 1024), (int)((threadIdx.x & 63) * 16), 0, 2);
}

__global__ __launch_bounds__(1024) void flat1_b1024(float4* __restrict__ out, size_t n4, float v) {
  const size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x;
  if (i < n4) out[i] = make_float4(v, v, v, v);
}

__global__ __launch_bounds__(256) void n2_far(float4* __restrict__ out, size_t n4, float v) {
  const size_t half = n4 / 2;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < half) {
    out[i] = make_float4(v, v, v, v);
    out[i + half] = make_float4(v, v, v, v);
  }
}

struct Unit {
  uint32_t lo, hi, start, pad;
};

// one row of 256 floats per wave (R rows per wave): unit record -> entry range -> its first 64 entries
template <int R>
__global__ __launch_bounds__(256) void row_dep(float4* __restrict__ out, size_t n4, const Unit* __restrict__ units,
                                               const uint32_t* __restrict__ idx, const uint8_t* __restrict__ codes) {
  const uint32_t lane = threadIdx.x & 63;
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // wave -> rows [w*R, w*R + R)
  const size_t row0 = w * R;
  if (row0 * 64 >= n4) return;
  const uint32_t u = (uint32_t)(row0 / 16);  // 16 rows per 16-KiB unit
  const Unit U = units[u];
  const uint32_t e = min(U.lo + lane, U.hi > U.lo ? U.hi - 1 : U.lo);
  const uint32_t pos = idx[e] - U.start;
  const float val = (float)codes[e] * 0.01f;
  const uint32_t cnt = min(U.hi - U.lo, 64u);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t rr = (uint32_t)((row0 + r) % 16);
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    for (uint32_t j = 0; j < cnt; ++j) {
      const uint32_t p = __builtin_amdgcn_readlane(pos, j);
      if ((p >> 8) == rr && ((p >> 2) & 63u) == lane) {
        const float x = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(val), j));
        const uint32_t c = p & 3u;
        b.x = c == 0 ? x : b.x;
        b.y = c == 1 ? x : b.y;
        b.z = c == 2 ? x : b.z;
        b.w = c == 3 ? x : b.w;
      }
    }
    const u4v a = {__float_as_uint(b.x), __float_as_uint(b.y), __float_as_uint(b.z), __float_as_uint(b.w)};
    __builtin_amdgcn_raw_buffer_store_b128(a, rsrc(out + (row0 + r) * 64, 1024), (int)(lane * 16), 0, 2);
  }
}

__device__ __forceinline__ uint32_t xcd_block(uint32_t b) {
  const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8, i = b / 8;
  return x * q + min(x, r) + i;
}

__global__ __launch_bounds__(256) void unit16_x(float4* __restrict__ out, size_t n4, float v) {
  const size_t w = (size_t)xcd_block(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const size_t base = w * 1024;
  if (base >= n4) return;
  const __amdgpu_buffer_rsrc_t r = rsrc(out + base, 16384);
  const u4v a = {__float_as_uint(v), __float_as_uint(v), __float_as_uint(v), __float_as_uint(v)};
#pragma unroll
  for (int i = 0; i < 16; ++i) __builtin_amdgcn_raw_buffer_store_b128(a, r, (int)(((i * 64) + (threadIdx.x & 63)) * 16), 0, 2);
}

int main(int argc, char** argv) {
  for (int a = 1; a < argc; ++a) {
    const size_t bytes = (size_t)atoll(argv[a]) << 20;
    const size_t n4 = bytes / 16;
    const size_t nunits = n4 / 1024;
    float4* out;
    Unit* units;
    uint32_t* idx;
    uint8_t* codes;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&units, nunits * sizeof(Unit)));
    // ~41 kept entries per 4096-element unit (1 %), spread over the unit
    const uint32_t per = 41;
    std::vector<Unit> hu(nunits);
    std::vector<uint32_t> hi(nunits * per);
    for (size_t u = 0; u < nunits; ++u) {
      hu[u] = Unit{(uint32_t)(u * per), (uint32_t)(u * per + per), (uint32_t)(u * 4096), 0};
      for (uint32_t j = 0; j < per; ++j) hi[u * per + j] = (uint32_t)(u * 4096 + j * 99 + 7);
    }
    CK(hipMalloc(&idx, hi.size() * 4));
    CK(hipMalloc(&codes, hi.size()));
    CK(hipMemcpy(units, hu.data(), hu.size() * sizeof(Unit), hipMemcpyHostToDevice));
    CK(hipMemcpy(idx, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(codes, 3, hi.size()));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      const int R = 20;
      CK(hipEventRecord(e0));
      for (int i = 0; i < R; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / R;
      printf("%6zu MiB %-12s %8.1f us %6.2f TB/s\n", bytes >> 20, name, us, bytes / us / 1e6);
    };
    const unsigned g1 = (unsigned)((n4 + 255) / 256);
    run("flat1", [&] { hipLaunchKernelGGL(flat1, dim3(g1), dim3(256), 0, 0, out, n4, 1.0f); });
    run("flat1_nt", [&] { hipLaunchKernelGGL(flat1_nt, dim3(g1), dim3(256), 0, 0, out, n4, 1.0f); });
    run("flat1_b1024", [&] { hipLaunchKernelGGL(flat1_b1024, dim3((unsigned)((n4 + 1023) / 1024)), dim3(1024), 0, 0, out, n4, 1.0f); });
    run("n2_far", [&] { hipLaunchKernelGGL(n2_far, dim3((unsigned)((n4 / 2 + 255) / 256)), dim3(256), 0, 0, out, n4, 1.0f); });
    run("row_dep1", [&] { hipLaunchKernelGGL(row_dep<1>, dim3(g1), dim3(256), 0, 0, out, n4, units, idx, codes); });
    run("row_dep2", [&] { hipLaunchKernelGGL(row_dep<2>, dim3((g1 + 1) / 2), dim3(256), 0, 0, out, n4, units, idx, codes); });
    run("row_dep4", [&] { hipLaunchKernelGGL(row_dep<4>, dim3((g1 + 3) / 4), dim3(256), 0, 0, out, n4, units, idx, codes); });
    run("unit16_x", [&] { hipLaunchKernelGGL(unit16_x, dim3((unsigned)((nunits + 3) / 4)), dim3(256), 0, 0, out, n4, 1.0f); });
    CK(hipFree(out));
    CK(hipFree(units));
    CK(hipFree(idx));
    CK(hipFree(codes));
  }
  return 0;
}
