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

template <int V, int NT = 256>
__global__ __launch_bounds__(NT) void scan(const float* __restrict__ in, const Meta* meta, uint32_t nunits,
                                           uint32_t tlo0, uint32_t thi0, int32_t* aI, float* aV, int32_t* bI,
                                           float* bV, uint32_t* cnt) {
  constexpr int NW = NT / 64;
  __shared__ int32_t stI[V == 5 ? NW : 1][512];
  __shared__ float stV[V == 5 ? NW : 1][512];
  __shared__ uint2 stR[V >= 8 ? NW : 1][V >= 8 ? 512 : 1];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t u = blockIdx.x * NW + wv;
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


__device__ __forceinline__ void load_unit(const float* in, uint32_t u, uint32_t lane, float4 (&v)[16]) {
  const float4* p = reinterpret_cast<const float4*>(in + (uint64_t)u * UNIT);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p + i * 64 + lane));
    v[i] = make_float4(t.x, t.y, t.z, t.w);
  }
}

template <bool WORK>
__device__ __forceinline__ void process_unit(const float4 (&v)[16], uint32_t u, uint32_t lane, uint32_t tlo,
                                             uint32_t thi, uint2* stR, uint2* Rall, uint32_t* cnt) {
  if (!WORK) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += v[i].x + v[i].y + v[i].z + v[i].w;
    if (s == 1234.5f) cnt[0] = 1;
    return;
  }
  const uint64_t reg = (uint64_t)u * UNIT;
  uint32_t cA = 0, cB = 0;
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
    uint64_t bc[4];
    uint32_t pc = cA;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bc[j] = __ballot(fa[j] || fb[j]);
      pc += mbcnt(bc[j]);
      cB += (uint32_t)__popcll(__ballot(fa[j]));
    }
    uint2* R = Rall + reg;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (fa[j] || fb[j]) {
        const uint2 rec = make_uint2((e0 + j) | (fa[j] ? 0x80000000u : 0u), __float_as_uint(xs[j]));
        if (pc < 512) stR[pc] = rec;
        else R[pc] = rec;
        ++pc;
      }
      cA += (uint32_t)__popcll(bc[j]);
    }
  }
  __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory");
  uint2* R = Rall + reg;
  for (uint32_t i = lane; i < cA && i < 512; i += 64) R[i] = stR[i];
  __builtin_amdgcn_wave_barrier(); asm volatile("" ::: "memory");
  if (lane == 0) { cnt[2 * u] = cA; cnt[2 * u + 1] = cB; }
}

template <bool WORK, int PER>
__global__ __launch_bounds__(256, 2) void scan_p(const float* __restrict__ in, uint32_t nunits, uint32_t per,
                                                 uint32_t tlo, uint32_t thi, int32_t* aI, uint32_t* cnt) {
  __shared__ uint2 stR[4][512];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t u0 = (blockIdx.x * 4 + wv) * per;
  if (u0 >= nunits) return;
  const uint32_t u1 = min(u0 + per, nunits);
  uint2* R = reinterpret_cast<uint2*>(aI);
  float4 A[16], B[16];
  if (PER == 0) {
    load_unit(in, u0, lane, A);
    for (uint32_t u = u0; u < u1; u += 2) {
      load_unit(in, min(u + 1, u1 - 1), lane, B);
      process_unit<WORK>(A, u, lane, tlo, thi, stR[wv], R, cnt);
      load_unit(in, min(u + 2, u1 - 1), lane, A);
      if (u + 1 < u1) process_unit<WORK>(B, u + 1, lane, tlo, thi, stR[wv], R, cnt);
    }
  } else {
    // straight-line: PER units, no loop edge for a load to stay in flight across
    load_unit(in, u0, lane, A);
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)PER; k += 2) {
      load_unit(in, min(u0 + k + 1, u1 - 1), lane, B);
      if (u0 + k < u1) process_unit<WORK>(A, u0 + k, lane, tlo, thi, stR[wv], R, cnt);
      if (k + 2 < (uint32_t)PER) load_unit(in, min(u0 + k + 2, u1 - 1), lane, A);
      if (u0 + k + 1 < u1) process_unit<WORK>(B, u0 + k + 1, lane, tlo, thi, stR[wv], R, cnt);
    }
  }
}

// 14: straight-line PER units per wave with the next unit in flight, and NO global store until every unit is
// classified (a store pending beside prefetched loads makes the compiler wait for everything: vmcnt counts
// loads and stores together on gfx9, out of order): records staged per unit in LDS (512 each; more are only
// counted — the real kernel would re-scan such a unit), counts kept in lanes, all flushed at the end.
template <int PER>
__device__ __forceinline__ void classify_unit(const float4 (&v)[16], uint32_t lane, uint32_t tlo, uint32_t thi,
                                              uint2* st, uint32_t& cA, uint32_t& cB) {
  cA = 0;
  cB = 0;
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
    uint64_t bc[4];
    uint32_t pc = cA;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bc[j] = __ballot(fa[j] || fb[j]);
      pc += mbcnt(bc[j]);
      cB += (uint32_t)__popcll(__ballot(fa[j]));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if ((fa[j] || fb[j]) && pc < 512)
        st[pc] = make_uint2((e0 + j) | (fa[j] ? 0x80000000u : 0u), __float_as_uint(xs[j]));
      pc += (fa[j] || fb[j]) ? 1u : 0u;
      cA += (uint32_t)__popcll(bc[j]);
    }
  }
}

template <int PER>
__global__ __launch_bounds__(256, 2) void scan_d(const float* __restrict__ in, uint32_t nunits, uint32_t tlo,
                                                 uint32_t thi, int32_t* aI, uint32_t* cnt) {
  __shared__ uint2 stR[4][PER][512];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t u0 = (blockIdx.x * 4 + wv) * PER;
  if (u0 >= nunits) return;
  const uint32_t u1 = min(u0 + PER, nunits);
  uint2* R = reinterpret_cast<uint2*>(aI);
  float4 A[16], B[16];
  uint32_t ca[PER], cb[PER];
  load_unit(in, u0, lane, A);
#pragma unroll
  for (uint32_t k = 0; k < (uint32_t)PER; k += 2) {
    load_unit(in, min(u0 + k + 1, u1 - 1), lane, B);
    classify_unit<PER>(A, lane, tlo, thi, stR[wv][k], ca[k], cb[k]);
    if (k + 2 < (uint32_t)PER) load_unit(in, min(u0 + k + 2, u1 - 1), lane, A);
    classify_unit<PER>(B, lane, tlo, thi, stR[wv][k + 1], ca[k + 1], cb[k + 1]);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (uint32_t k = 0; k < (uint32_t)PER; ++k) {
    if (u0 + k >= u1) break;
    uint2* Ru = R + (uint64_t)(u0 + k) * UNIT;
    for (uint32_t i = lane; i < ca[k] && i < 512; i += 64) Ru[i] = stR[wv][k][i];
    if (lane == 0) { cnt[2 * (u0 + k)] = ca[k]; cnt[2 * (u0 + k) + 1] = cb[k]; }
  }
}

// 15: half-unit pipeline: PER units per wave as 2*PER halves of 8 float4 per lane, the next half in flight while
// the current one is classified; records staged in LDS (SC per unit; more only counted), stores deferred to
// the end (as 14). Fewer registers than 14: ~5 waves per SIMD.
template <int SC>
__device__ __forceinline__ void classify_half(const float4 (&v)[8], uint32_t hbase, uint32_t lane, uint32_t tlo,
                                              uint32_t thi, uint2* st, uint32_t& cA, uint32_t& cB) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t e0 = hbase + (i * 64 + lane) * 4;
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
    uint64_t bc[4];
    uint32_t pc = cA;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bc[j] = __ballot(fa[j] || fb[j]);
      pc += mbcnt(bc[j]);
      cB += (uint32_t)__popcll(__ballot(fa[j]));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if ((fa[j] || fb[j]) && pc < SC)
        st[pc] = make_uint2((e0 + j) | (fa[j] ? 0x80000000u : 0u), __float_as_uint(xs[j]));
      pc += (fa[j] || fb[j]) ? 1u : 0u;
      cA += (uint32_t)__popcll(bc[j]);
    }
  }
}

__device__ __forceinline__ void load_half(const float* in, uint32_t u, uint32_t half, uint32_t lane, float4 (&v)[8]) {
  const float4* p = reinterpret_cast<const float4*>(in + (uint64_t)u * UNIT + half * (UNIT / 2));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p + i * 64 + lane));
    v[i] = make_float4(t.x, t.y, t.z, t.w);
  }
}

template <int PER, int SC, int OCC>
__global__ __launch_bounds__(256, OCC) void scan_h(const float* __restrict__ in, uint32_t nunits, uint32_t tlo,
                                                   uint32_t thi, int32_t* aI, uint32_t* cnt) {
  __shared__ uint2 stR[4][PER][SC];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t u0 = (blockIdx.x * 4 + wv) * PER;
  if (u0 >= nunits) return;
  const uint32_t u1 = min(u0 + PER, nunits);
  uint2* R = reinterpret_cast<uint2*>(aI);
  float4 A[8], B[8];
  uint32_t ca[PER], cb[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) ca[k] = cb[k] = 0;
  load_half(in, u0, 0, lane, A);
#pragma unroll
  for (uint32_t k = 0; k < (uint32_t)PER; ++k) {
    const uint32_t uk = min(u0 + k, u1 - 1);
    load_half(in, uk, 1, lane, B);
    classify_half<SC>(A, 0, lane, tlo, thi, stR[wv][k], ca[k], cb[k]);
    if (k + 1 < (uint32_t)PER) load_half(in, min(u0 + k + 1, u1 - 1), 0, lane, A);
    classify_half<SC>(B, UNIT / 2, lane, tlo, thi, stR[wv][k], ca[k], cb[k]);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (uint32_t k = 0; k < (uint32_t)PER; ++k) {
    if (u0 + k >= u1) break;
    uint2* Ru = R + (uint64_t)(u0 + k) * UNIT;
    for (uint32_t i = lane; i < ca[k] && i < SC; i += 64) Ru[i] = stR[wv][k][i];
    if (lane == 0) { cnt[2 * (u0 + k)] = ca[k]; cnt[2 * (u0 + k) + 1] = cb[k]; }
  }
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
  for (uint32_t bpc : {2u, 3u}) {
    const uint32_t waves = 256u * bpc * 4u, per = (nunits + waves - 1) / waves, gp = (nunits + per * 4 - 1) / (per * 4);
    char nm[64];
    snprintf(nm, sizeof nm, "11_persistent_load_only_b%u", bpc);
    run(nm, [&] { hipLaunchKernelGGL((scan_p<false, 0>), dim3(gp), dim3(256), 0, 0, in, nunits, per, tlo, thi, aI, cnt); });
    snprintf(nm, sizeof nm, "10_persistent_prefetch_b%u", bpc);
    run(nm, [&] { hipLaunchKernelGGL((scan_p<true, 0>), dim3(gp), dim3(256), 0, 0, in, nunits, per, tlo, thi, aI, cnt); });
  }
#define RUNS(PER) { const uint32_t gp = (nunits + PER * 4 - 1) / (PER * 4); \
    run("12_straight_prefetch_per" #PER, [&] { hipLaunchKernelGGL((scan_p<true, PER>), dim3(gp), dim3(256), 0, 0, in, nunits, PER, tlo, thi, aI, cnt); }); \
    run("13_straight_load_only_per" #PER, [&] { hipLaunchKernelGGL((scan_p<false, PER>), dim3(gp), dim3(256), 0, 0, in, nunits, PER, tlo, thi, aI, cnt); }); }
#define RUND(PER) { const uint32_t gp = (nunits + PER * 4 - 1) / (PER * 4); \
    run("14_deferred_stores_per" #PER, [&] { hipLaunchKernelGGL((scan_d<PER>), dim3(gp), dim3(256), 0, 0, in, nunits, tlo, thi, aI, cnt); }); }
  RUND(2)
#define RUNH(PER, SC, OCC) { const uint32_t gp = (nunits + PER * 4 - 1) / (PER * 4); \
    run("15_half_pipeline_per" #PER "_sc" #SC "_occ" #OCC, [&] { hipLaunchKernelGGL((scan_h<PER, SC, OCC>), dim3(gp), dim3(256), 0, 0, in, nunits, tlo, thi, aI, cnt); }); }
  RUNH(1, 512, 5) RUNH(2, 256, 5) RUNH(2, 256, 6) RUNH(4, 256, 4) RUNH(4, 128, 5) RUNH(8, 128, 4)
  RUN(9, "9_combined_lds_staged_nt_again");
  // block size: a block's slots free only when its slowest wave ends (16: one wave per block)
#define RUNB(V, NT, name) run(name, [&] { hipLaunchKernelGGL((scan<V, NT>), dim3((nunits + NT / 64 - 1) / (NT / 64)), dim3(NT), 0, 0, in, meta, nunits, tlo, thi, aI, aV, bI, bV, cnt); })
  RUNB(0, 64, "16_load_only_nt64");
  RUNB(0, 128, "16_load_only_nt128");
  RUNB(0, 512, "16_load_only_nt512");
  RUNB(9, 64, "16_staged_nt_nt64");
  RUNB(9, 128, "16_staged_nt_nt128");
  RUNB(9, 256, "16_staged_nt_nt256");
  return 0;
}
