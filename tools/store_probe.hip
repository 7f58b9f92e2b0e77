// Write-bandwidth probe for k_decode's store pattern (tools/store_probe <MiB> ...): for each buffer size,
// the time of one launch writing it, per store flavour:
//   unit_g    one wave per 16 KiB unit, 16 float4 global stores per lane (stride 1 KiB), plain
//   unit_gnt  the same, non-temporal (__builtin_nontemporal_store)
//   unit_b    buffer stores through a per-unit resource (k_decode's form), cache policy 0
//   unit_bnt  the same, policy 2 (non-temporal: k_decode's default)
//   flat1     one float4 per thread, grid = n/4/256 blocks (elementwise style)
//   gs        grid-stride float4 loop, 8 blocks per CU
// Prints TB/s of bytes written (launch time from hipEvents, mean of 20).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)bytes, 0x00020000);
}

template <int MODE>
__global__ __launch_bounds__(256) void unit_store(float4* __restrict__ out, size_t n4, float v) {
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const unsigned lane = threadIdx.x & 63;
  const size_t base = w * 1024;
  if (base >= n4) return;
  const float4 z = make_float4(v, v, v, v);
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) out[base + i * 64 + lane] = z;
  } else if (MODE == 1) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v zz = {v, v, v, v};
#pragma unroll
    for (int i = 0; i < 16; ++i) __builtin_nontemporal_store(zz, reinterpret_cast<f4v*>(out + base + i * 64 + lane));
  } else {
    const __amdgpu_buffer_rsrc_t r = rsrc(out + base, 16384);
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    const u4v a = {__float_as_uint(v), __float_as_uint(v), __float_as_uint(v), __float_as_uint(v)};
#pragma unroll
    for (int i = 0; i < 16; ++i)
      __builtin_amdgcn_raw_buffer_store_b128(a, r, (int)((i * 64 + lane) * 16), 0, MODE == 2 ? 0 : 2);
  }
}

// N float4 per lane per wave (a wave writes N KiB, strided rows), plain global stores
template <int N>
__global__ __launch_bounds__(256) void unit_n(float4* __restrict__ out, size_t n4, float v) {
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const unsigned lane = threadIdx.x & 63;
  const size_t base = w * 64 * N;
  if (base >= n4) return;
#pragma unroll
  for (int i = 0; i < N; ++i) out[base + i * 64 + lane] = make_float4(v, v, v, v);
}

// a block owns 4 consecutive 16 KiB units; at step j its wave w writes row 4j + w of the 64 KiB (the
// block's stores walk its region in order, 4 KiB per step)
__global__ __launch_bounds__(256) void unit_blk(float4* __restrict__ out, size_t n4, float v) {
  const unsigned wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t base = (size_t)blockIdx.x * 4096;
  if (base >= n4) return;
#pragma unroll
  for (int j = 0; j < 16; ++j) out[base + (j * 4 + wv) * 64 + lane] = make_float4(v, v, v, v);
}

// k_decode's pattern with an XCD-aware block order: workgroups are dispatched round-robin over the 8 XCDs, so
// block b runs on XCD b % 8; remapped, XCD x writes the contiguous x-th eighth of the buffer (MODE 0: plain
// global stores, 1: non-temporal buffer stores)
template <int MODE>
__global__ __launch_bounds__(256) void unit_x(float4* __restrict__ out, size_t n4, float v) {
  const unsigned nb = gridDim.x, per = (nb + 7) / 8;
  const unsigned b = (blockIdx.x % 8) * per + blockIdx.x / 8;
  const size_t w = (size_t)b * 4 + (threadIdx.x >> 6);
  const unsigned lane = threadIdx.x & 63;
  const size_t base = w * 1024;
  if (base >= n4) return;
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) out[base + i * 64 + lane] = make_float4(v, v, v, v);
  } else {
    const __amdgpu_buffer_rsrc_t r = rsrc(out + base, 16384);
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    const u4v a = {__float_as_uint(v), __float_as_uint(v), __float_as_uint(v), __float_as_uint(v)};
#pragma unroll
    for (int i = 0; i < 16; ++i) __builtin_amdgcn_raw_buffer_store_b128(a, r, (int)((i * 64 + lane) * 16), 0, 2);
  }
}

// XCD-aware order in chunks: XCD x takes chunks x, x + 8, x + 16, ... of C blocks (64 KiB each), so every
// XCD streams through C contiguous blocks at a time while all XCDs advance through the buffer together
// (the probe's grids are multiples of 8 * C)
template <int C>
__global__ __launch_bounds__(256) void unit_xc(float4* __restrict__ out, size_t n4, float v) {
  const unsigned x = blockIdx.x % 8, i = blockIdx.x / 8;
  const unsigned b = ((i / C) * 8 + x) * C + i % C;
  const size_t w = (size_t)b * 4 + (threadIdx.x >> 6);
  const unsigned lane = threadIdx.x & 63;
  const size_t base = w * 1024;
  if (base >= n4) return;
  const __amdgpu_buffer_rsrc_t r = rsrc(out + base, 16384);
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const u4v a = {__float_as_uint(v), __float_as_uint(v), __float_as_uint(v), __float_as_uint(v)};
#pragma unroll
  for (int i2 = 0; i2 < 16; ++i2) __builtin_amdgcn_raw_buffer_store_b128(a, r, (int)((i2 * 64 + lane) * 16), 0, 2);
}

// read probes: one wave per 16 KiB unit (k_scan's pattern), in dispatch order or XCD-remapped
template <bool XCD>
__global__ __launch_bounds__(256) void read_u(const float4* __restrict__ in, size_t n4, float* sink) {
  const unsigned nb = gridDim.x, per = (nb + 7) / 8;
  const unsigned b = XCD ? (blockIdx.x % 8) * per + blockIdx.x / 8 : blockIdx.x;
  const size_t w = (size_t)b * 4 + (threadIdx.x >> 6);
  const unsigned lane = threadIdx.x & 63;
  const size_t base = w * 1024;
  if (base >= n4) return;
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v* src = reinterpret_cast<const f4v*>(in);
  f4v x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = __builtin_nontemporal_load(src + base + i * 64 + lane);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += x[i].x + x[i].y + x[i].z + x[i].w;
  if (s == 12345.678f) sink[0] = s;
}

__global__ __launch_bounds__(256) void flat1(float4* __restrict__ out, size_t n4, float v) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) out[i] = make_float4(v, v, v, v);
}

__global__ __launch_bounds__(256) void gs(float4* __restrict__ out, size_t n4, float v) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    out[i] = make_float4(v, v, v, v);
}

int main(int argc, char** argv) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int a = 1; a < argc; ++a) {
    const size_t bytes = (size_t)atoll(argv[a]) << 20;
    const size_t n4 = bytes / 16;
    float4* out;
    float* sink;
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&sink, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned gu = (unsigned)((n4 / 1024 + 3) / 4);
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
      printf("%6zu MiB %-9s %8.1f us %6.2f TB/s\n", bytes >> 20, name, us, bytes / us / 1e6);
    };
    run("unit_g", [&] { hipLaunchKernelGGL(unit_store<0>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_gnt", [&] { hipLaunchKernelGGL(unit_store<1>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_b", [&] { hipLaunchKernelGGL(unit_store<2>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_bnt", [&] { hipLaunchKernelGGL(unit_store<3>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_n4", [&] { hipLaunchKernelGGL(unit_n<4>, dim3((unsigned)((n4 / 256 + 3) / 4)), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_n8", [&] { hipLaunchKernelGGL(unit_n<8>, dim3((unsigned)((n4 / 512 + 3) / 4)), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_n2", [&] { hipLaunchKernelGGL(unit_n<2>, dim3((unsigned)((n4 / 128 + 3) / 4)), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_blk", [&] { hipLaunchKernelGGL(unit_blk, dim3((unsigned)((n4 + 4095) / 4096)), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_xg", [&] { hipLaunchKernelGGL(unit_x<0>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_xbnt", [&] { hipLaunchKernelGGL(unit_x<1>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_xc16", [&] { hipLaunchKernelGGL(unit_xc<16>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_xc64", [&] { hipLaunchKernelGGL(unit_xc<64>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("unit_xc256", [&] { hipLaunchKernelGGL(unit_xc<256>, dim3(gu), dim3(256), 0, 0, out, n4, 1.0f); });
    run("read_u", [&] { hipLaunchKernelGGL(read_u<false>, dim3(gu), dim3(256), 0, 0, out, n4, sink); });
    run("read_ux", [&] { hipLaunchKernelGGL(read_u<true>, dim3(gu), dim3(256), 0, 0, out, n4, sink); });
    run("flat1", [&] { hipLaunchKernelGGL(flat1, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, out, n4, 1.0f); });
    run("gs", [&] { hipLaunchKernelGGL(gs, dim3(cus * 8), dim3(256), 0, 0, out, n4, 1.0f); });
    CK(hipFree(out));
  }
  return 0;
}
