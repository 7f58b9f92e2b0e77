// scan_ablate.hip — ablation of the k_scan streaming pass (coalac.hip scan_unit) on synthetic data.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/scan_ablate tools/scan_ablate.hip
// Each variant streams the same 1.64 GB (16 ResNet-50-sized clients) one 4096-element unit per wave:
//   0 load only                      (ceiling for this access shape)
//   1 + classify + __any skip        (VALU on every element)
//   2 + ballots/mbcnt positions      (kept live, no stores)
//   3 + candidate stores (global, per-lane scattered)   = the real kernel
//   4 = 3 with the unit metadata loaded first (dependent chain as in coalac.hip)
//   5 = 3 with LDS staging of candidates + coalesced flush
//   6 = 3 with nontemporal input loads
//   7 one combined ordered list of 8-byte records {idx | A-flag, value}: one dwordx2 store per candidate
//   8 = 7 staged in LDS (512 records per wave) and flushed with coalesced stores
//   9 = 8 with nontemporal input loads
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <cstring>
typedef float f4v __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr uint32_t UNIT = 4096;

struct Meta { uint64_t off; uint32_t tlo, thi; };

__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int V>
__global__ __launch_bounds__(256) void scan(const float* __restrict__ in, const Meta* meta, uint32_t nunits,
                                            uint32_t tlo0, uint32_t thi0, int32_t* aI, float* aV, int32_t* bI,
                                            float* bV, uint32_t* cnt) {
  __shared__ int32_t stI[4][512];
  __shared__ float stV[4][512];
  __shared__ uint2 stR[V >= 8 ? 4 : 1][V >= 8 ? 512 : 1];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t u = blockIdx.x * 4 + wv;
  if (u >= nunits) return;
  uint64_t off = (uint64_t)u * UNIT;
  uint32_t tlo = tlo0, thi = thi0;
  if (V == 4) {
    const Meta m = meta[u];
    off = m.off;
    tlo = m.tlo;
    thi = m.thi;
  }
  const float4* p = reinterpret_cast<const float4*>(in + off);
  float4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (V == 6 || V == 9) {
      const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p + i * 64 + lane));
      v[i] = make_float4(t.x, t.y, t.z, t.w);
    } else
      v[i] = p[i * 64 + lane];
  }
  if (V == 0) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i].x + v[i].y + v[i].z + v[i].w;
    if (s == 1234.5f) cnt[0] = 1;
    return;
  }
  const uint64_t reg = (uint64_t)u * UNIT;
  uint32_t cA = 0, cB = 0, sink = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t e0 = (i * 64 + lane) * 4;
    const float xs[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
    bool fa[4], fb[4], any = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t key = __float_as_uint(xs[j]) & 0x7FFFFFFFu;
      fa[j] = key > thi;
      fb[j] = !fa[j] && key >= tlo;
      any = any || fa[j] || fb[j];
    }
    if (!__any(any)) continue;
    if (V == 1) {
      sink += any;
      continue;
    }
    if (V >= 7) {
      uint64_t bc[4];
      uint32_t pc = cA;  // combined count
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bc[j] = __ballot(fa[j] || fb[j]);
        pc += mbcnt(bc[j]);
        cB += (uint32_t)__popcll(__ballot(fa[j]));
      }
      uint2* R = reinterpret_cast<uint2*>(aI) + reg;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (fa[j] || fb[j]) {
          const uint2 rec = make_uint2((e0 + j) | (fa[j] ? 0x80000000u : 0u), __float_as_uint(xs[j]));
          if (V == 7) R[pc] = rec;
          else if (pc < 512) stR[wv][pc] = rec;
          else R[pc] = rec;
          ++pc;
        }
        cA += (uint32_t)__popcll(bc[j]);
      }
      continue;
    }
    uint64_t ba[4], bb[4];
    uint32_t pa = cA, pb = cB;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      ba[j] = __ballot(fa[j]);
      bb[j] = __ballot(fb[j]);
      pa += mbcnt(ba[j]);
      pb += mbcnt(bb[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (V == 2) {
        sink += fa[j] ? pa : 0;
        sink += fb[j] ? pb : 0;
      } else if (V == 5) {
        if (fa[j] && pa < 512) { stI[wv][pa] = e0 + j; stV[wv][pa] = xs[j]; }
        if (fb[j] && pb < 512) { bI[reg + pb] = e0 + j; bV[reg + pb] = xs[j]; }
      } else {
        if (fa[j]) { aI[reg + pa] = e0 + j; aV[reg + pa] = xs[j]; }
        if (fb[j]) { bI[reg + pb] = e0 + j; bV[reg + pb] = xs[j]; }
      }
      if (fa[j]) ++pa;
      if (fb[j]) ++pb;
      cA += (uint32_t)__popcll(ba[j]);
      cB += (uint32_t)__popcll(bb[j]);
    }
  }
  if (V >= 8) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint2* R = reinterpret_cast<uint2*>(aI) + reg;
    for (uint32_t i = lane; i < cA && i < 512; i += 64) R[i] = stR[wv][i];
  }
  if (V == 5) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (uint32_t i = lane; i < cA && i < 512; i += 64) { aI[reg + i] = stI[wv][i]; aV[reg + i] = stV[wv][i]; }
  }
  if (lane == 0) { cnt[2 * u] = cA; cnt[2 * u + 1] = cB + sink; }
}

int main() {
  const uint32_t nunits = 16u * 6252u;  // ~ 16 ResNet-50 clients of large units
  const size_t n = (size_t)nunits * UNIT;
  std::vector<float> h(n);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1e-3f);
  for (size_t i = 0; i < n; ++i) h[i] = nd(rng);
  float* in;
  int32_t *aI, *bI;
  float *aV, *bV;
  uint32_t* cnt;
  Meta* meta;
  CK(hipMalloc(&in, n * 4));
  CK(hipMalloc(&aI, n * 8));
  CK(hipMalloc(&aV, n * 4));
  CK(hipMalloc(&bI, n * 4));
  CK(hipMalloc(&bV, n * 4));
  CK(hipMalloc(&cnt, 8 * nunits));
  CK(hipMalloc(&meta, sizeof(Meta) * nunits));
  CK(hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice));
  // |x| rank thresholds for ~0.25 % (A) and ~1.75 % (A+B) of a N(0, 1e-3) sample: 3.02 sigma, 2.38 sigma
  float thi_f = 3.02e-3f, tlo_f = 2.38e-3f;
  uint32_t thi, tlo;
  memcpy(&thi, &thi_f, 4);
  memcpy(&tlo, &tlo_f, 4);
  std::vector<Meta> hm(nunits);
  for (uint32_t u = 0; u < nunits; ++u) hm[u] = Meta{(uint64_t)u * UNIT, tlo, thi};
  CK(hipMemcpy(meta, hm.data(), sizeof(Meta) * nunits, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t g = (nunits + 3) / 4;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int R = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms / R, n * 4.0 * R / (ms * 1e-3) / 1e9);
    return 0;
  };
#define RUN(V, name) run(name, [&] { hipLaunchKernelGGL(scan<V>, dim3(g), dim3(256), 0, 0, in, meta, nunits, tlo, thi, aI, aV, bI, bV, cnt); })
  RUN(0, "0_load_only");
  RUN(1, "1_classify");
  RUN(2, "2_ballot_positions");
  RUN(3, "3_full_stores");
  RUN(4, "4_full_meta_chain");
  RUN(5, "5_lds_staged_A");
  RUN(6, "6_full_nt_loads");
  RUN(7, "7_combined_8B_records");
  RUN(8, "8_combined_lds_staged");
  RUN(9, "9_combined_lds_staged_nt");
  RUN(0, "0_load_only_again");
  return 0;
}
