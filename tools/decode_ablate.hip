// decode_ablate.hip — ablation of the decode write stream (coalac.hip k_decode) on synthetic data.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/decode_ablate tools/decode_ablate.hip
// 16 ResNet-50-sized clients of 4096-element units, ~1 % kept entries per unit (sorted positions).
//   0 zero stores only, one wave per unit                         (dispatch + write ceiling of the shape)
//   1 0 + unit metadata load first (dependent chain)
//   2 1 + kept entries loaded, waitcnt, scatter (= coalac k_decode)
//   3 1 + kept entries merged into the registers before the stores (no waitcnt, no second write)
//   4 2 with 4 units per wave (grid / 4)
//   5 3 with 4 units per wave
//   6 zero stores, grid-stride persistent (2048 blocks)           (reference ceiling, like hbm_probe)
//   7 3 with nontemporal stores
//   8 UPW=4 units per wave, every unit's metadata + entries loaded up front (one latency for 4 units)
//   9 8 with UPW=8
//  10 9 with nontemporal stores
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr uint32_t UNIT = 4096;
typedef float f4v __attribute__((ext_vector_type(4)));

struct Unit { uint64_t off; uint32_t lo, hi; };  // element offset, kept-entry range [lo, hi)

template <int V, int UPW>
__global__ __launch_bounds__(256) void dec(float* out, const Unit* units, uint32_t nunits, const int32_t* idx,
                                           const float* vals) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint32_t r = 0; r < UPW; ++r) {
    const uint32_t u = (blockIdx.x * 4 + wv) * UPW + r;
    if (u >= nunits) return;
    uint64_t off = (uint64_t)u * UNIT;
    uint32_t lo = 0, hi = 0;
    if (V >= 1) {
      const Unit U = units[u];
      off = U.off;
      lo = U.lo;
      hi = U.hi;
    }
    float* o = out + off;
    if (V == 0 || V == 1) {
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<float4*>(o + (i * 64 + lane) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    const uint32_t e = lo + lane;
    const uint32_t ec = min(e, hi == lo ? lo : hi - 1);
    const uint32_t p0 = (uint32_t)idx[ec];
    const float v0 = vals[ec];
    const uint32_t pos0 = e < hi ? p0 : 0xFFFFFFFFu;
    if (V == 2) {
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<float4*>(o + (i * 64 + lane) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (pos0 < UNIT) o[pos0] = v0;
      for (uint32_t e2 = lo + 64 + lane; e2 < hi; e2 += 64) o[idx[e2]] = vals[e2];
      continue;
    }
    // V == 3 / 7: merge into registers. Entry j (lane j of the batch) -> row pos >> 8, lane (pos >> 2) & 63.
    float4 b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const uint32_t cnt = hi - lo;
    if (cnt <= 64) {
      // walk the (sorted) entries once; rows are visited in order, so the row index stays static
      uint32_t j = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        while (j < cnt) {
          const uint32_t pos = __builtin_amdgcn_readlane(pos0, j);
          if ((pos >> 8) != (uint32_t)i) break;
          const float v = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v0), j));
          if (((pos >> 2) & 63) == lane) {
            const uint32_t c = pos & 3;
            b[i].x = c == 0 ? v : b[i].x;
            b[i].y = c == 1 ? v : b[i].y;
            b[i].z = c == 2 ? v : b[i].z;
            b[i].w = c == 3 ? v : b[i].w;
          }
          ++j;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (V == 7) {
          f4v t = {b[i].x, b[i].y, b[i].z, b[i].w};
          __builtin_nontemporal_store(t, reinterpret_cast<f4v*>(o + (i * 64 + lane) * 4));
        } else {
          *reinterpret_cast<float4*>(o + (i * 64 + lane) * 4) = b[i];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<float4*>(o + (i * 64 + lane) * 4) = b[i];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (pos0 < UNIT) o[pos0] = v0;
      for (uint32_t e2 = lo + 64 + lane; e2 < hi; e2 += 64) o[idx[e2]] = vals[e2];
    }
  }
}

// merge up to 64 sorted entries (pos in lane j, value v) into the wave's registers b[16] (row = pos >> 8)
__device__ __forceinline__ void merge64(float4 (&b)[16], uint32_t pos0, float v0, uint32_t cnt, uint32_t lane) {
  uint32_t j = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    while (j < cnt) {
      const uint32_t pos = __builtin_amdgcn_readlane(pos0, j);
      if ((pos >> 8) != (uint32_t)i) break;
      const float v = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v0), j));
      if (((pos >> 2) & 63) == lane) {
        const uint32_t c = pos & 3;
        b[i].x = c == 0 ? v : b[i].x;
        b[i].y = c == 1 ? v : b[i].y;
        b[i].z = c == 2 ? v : b[i].z;
        b[i].w = c == 3 ? v : b[i].w;
      }
      ++j;
    }
  }
}

template <int UPW, bool NTS>
__global__ __launch_bounds__(256) void dec_batch(float* out, const Unit* units, uint32_t nunits, const int32_t* idx,
                                                 const float* vals) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t u0 = (blockIdx.x * 4 + wv) * UPW;
  if (u0 >= nunits) return;
  Unit U[UPW];
#pragma unroll
  for (int r = 0; r < UPW; ++r) U[r] = units[min(u0 + r, nunits - 1)];
  uint32_t pos[UPW];
  float v[UPW];
#pragma unroll
  for (int r = 0; r < UPW; ++r) {
    const uint32_t e = U[r].lo + lane;
    const uint32_t ec = min(e, U[r].hi > U[r].lo ? U[r].hi - 1 : U[r].lo);
    pos[r] = (uint32_t)idx[ec];
    v[r] = vals[ec];
  }
#pragma unroll
  for (int r = 0; r < UPW; ++r) {
    if (u0 + r >= nunits) break;
    float4 b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) b[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const uint32_t cnt = min(U[r].hi - U[r].lo, 64u);
    merge64(b, pos[r], v[r], cnt, lane);
    float* o = out + U[r].off;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (NTS) {
        f4v t = {b[i].x, b[i].y, b[i].z, b[i].w};
        __builtin_nontemporal_store(t, reinterpret_cast<f4v*>(o + (i * 64 + lane) * 4));
      } else {
        *reinterpret_cast<float4*>(o + (i * 64 + lane) * 4) = b[i];
      }
    }
  }
}

__global__ __launch_bounds__(256) void persist(float* out, size_t n4) {
  float4* o = reinterpret_cast<float4*>(out);
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    o[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

int main() {
  const uint32_t nunits = 16u * 6252u;
  const size_t n = (size_t)nunits * UNIT;
  std::mt19937 rng(7);
  std::vector<Unit> hu(nunits);
  std::vector<int32_t> hidx;
  std::vector<float> hv;
  for (uint32_t u = 0; u < nunits; ++u) {
    const uint32_t k = 41 + (rng() % 3) - 1;
    std::vector<int32_t> p(UNIT);
    for (uint32_t i = 0; i < UNIT; ++i) p[i] = i;
    std::shuffle(p.begin(), p.end(), rng);
    std::sort(p.begin(), p.begin() + k);
    hu[u] = Unit{(uint64_t)u * UNIT, (uint32_t)hidx.size(), (uint32_t)(hidx.size() + k)};
    for (uint32_t i = 0; i < k; ++i) { hidx.push_back(p[i]); hv.push_back(1.0f + i); }
    // idx are unit-relative here; offsets into the list are global
  }
  float *out, *vals;
  int32_t* idx;
  Unit* units;
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&vals, hv.size() * 4));
  CK(hipMalloc(&idx, hidx.size() * 4));
  CK(hipMalloc(&units, nunits * sizeof(Unit)));
  CK(hipMemcpy(vals, hv.data(), hv.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(idx, hidx.data(), hidx.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(units, hu.data(), nunits * sizeof(Unit), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> check(n);
  auto run = [&](const char* name, auto launch, bool verify) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    int bad = 0;
    if (verify) {
      CK(hipMemcpy(check.data(), out, n * 4, hipMemcpyDeviceToHost));
      size_t nz = 0;
      for (size_t i = 0; i < n; ++i) nz += check[i] != 0.f;
      for (uint32_t u = 0; u < nunits && !bad; ++u)
        for (uint32_t e = hu[u].lo; e < hu[u].hi; ++e)
          if (check[hu[u].off + hidx[e]] != hv[e]) { bad = 1; break; }
      if (nz != hidx.size()) bad |= 2;
    }
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f, \"bad\": %d}\n", name, ms / R,
           n * 4.0 * R / (ms * 1e-3) / 1e9, bad);
    CK(hipMemset(out, 0x7f, n * 4));
    return 0;
  };
  const uint32_t g = (nunits + 3) / 4, g4 = (nunits + 15) / 16;
#define RUN(V, U, G, name, ver) run(name, [&] { hipLaunchKernelGGL((dec<V, U>), dim3(G), dim3(256), 0, 0, out, units, nunits, idx, vals); }, ver)
  RUN(0, 1, g, "0_zero_stores", false);
  RUN(1, 1, g, "1_meta_chain", false);
  RUN(2, 1, g, "2_waitcnt_scatter", true);
  RUN(3, 1, g, "3_register_merge", true);
  RUN(2, 4, g4, "4_scatter_4upw", true);
  RUN(3, 4, g4, "5_merge_4upw", true);
  run("6_persistent_2048", [&] { hipLaunchKernelGGL(persist, dim3(2048), dim3(256), 0, 0, out, n / 4); }, false);
  RUN(7, 1, g, "7_merge_nt_stores", true);
  run("8_hoisted_4upw", [&] { hipLaunchKernelGGL((dec_batch<4, false>), dim3(g4), dim3(256), 0, 0, out, units, nunits, idx, vals); }, true);
  const uint32_t g8 = (nunits + 31) / 32;
  run("9_hoisted_8upw", [&] { hipLaunchKernelGGL((dec_batch<8, false>), dim3(g8), dim3(256), 0, 0, out, units, nunits, idx, vals); }, true);
  run("10_hoisted_8upw_nt", [&] { hipLaunchKernelGGL((dec_batch<8, true>), dim3(g8), dim3(256), 0, 0, out, units, nunits, idx, vals); }, true);
  run("11_hoisted_4upw_nt", [&] { hipLaunchKernelGGL((dec_batch<4, true>), dim3(g4), dim3(256), 0, 0, out, units, nunits, idx, vals); }, true);
  const uint32_t g2 = (nunits + 7) / 8;
  run("12_hoisted_2upw_nt", [&] { hipLaunchKernelGGL((dec_batch<2, true>), dim3(g2), dim3(256), 0, 0, out, units, nunits, idx, vals); }, true);
  RUN(0, 1, g, "0_zero_stores_again", false);
  return 0;
}
