// coalac.hip — MI355X (gfx950, CDNA4) model-update codec: CodecSpec v1 (per-segment exact top-k by
// |x| with lower-index tie-break, then b-bit min/max quantisation), behind the C ABI of include/coalac.h.
//
// Reference context: SonyResearch/COALA has no codec (coala/compression/__init__.py is 0 bytes); the
// hooks this replaces are coala/client/base.py:330-332 (encode) and coala/server/base.py:558-560
// (decode), and strategies.federated_averaging on the decoded uploads (aggregate).
// The spec is SURVEY.md §8(a) a3/a4; the CPU oracle restating it is oracle/codec_oracle.py.
//
// Design (DESIGN.md has the full rationale):
//   The path is HBM-bound integer/byte work: no MFMA. Encode must read the input ONCE from HBM, so the
//   exact top-k is found Floyd–Rivest style: per segment a small stratified sample brackets the k-th
//   key between two thresholds [T_lo, T_hi]; one streaming pass classifies every element as
//   A (key > T_hi: surely kept), B (T_lo <= key <= T_hi: maybe) or out, and writes A and B in index
//   order into per-unit candidate lists; a per-segment pass resolves the exact k-th key inside B;
//   a per-unit pass emits the sorted indices and codes. If a sample's bracket misses (count(A) > k or
//   count(A ∪ B) < k) the segment is re-selected exactly inside the same launch sequence (no host
//   round trip), so results are always exact.
//
//   Work unit = 4096 contiguous elements of one segment, owned by ONE wave64: ordered compaction is
//   done with wave ballots + mbcnt (records staged in the wave's LDS slice, flushed coalesced), so the
//   streaming pass has no block barriers. Segments of <= 1024 elements ("small"; COALAC_SMALL_MAX raises the
//   limit up to 4096) are encoded whole by one block in LDS.
//
//   Encode kernels, in stream order:
//     k_presel  the samplers (one block per large segment: stratified sample -> [T_lo, T_hi]) and the small
//               segments side by side (batches; latency-bound plans run k_sample alone and the small
//               segments in k_scan's first blocks)
//     k_scan    one wave per large unit (128-thread blocks in batches): single HBM read, classify A / B,
//               candidate records in index order (u16 position + u32 value bits, 6 B each)
//     k_ghist   one block per 32-unit group: band histogram of the group's B records
//     k_gwin    one block per group: sum the segment's group histograms -> key window of the k-th key
//               (every group block of the segment, redundantly); per-unit counts above the window + the
//               group's in-window entries (latency-bound plans: both sweep their records speculatively)
//     k_select  one block per large segment: exact k-th key + tie quota from the window lists (generic
//               multi-pass select / exact re-select on a bracket miss), per-unit output offsets (= the
//               payload's per-unit starts, wire v2), min / max -> scale, per-unit emit parameters
//     k_emit    one wave per 8 large units (1 in latency-bound plans, one load round): kept records ->
//               ascending idx + codes
//   Decode: k_decode_lds — every output line written once, the unit's kept values placed through a per-wave
//   LDS tile; entry ranges from the payload's per-unit starts (wire v2; a host that received a v1 blob computes
//   them, coala_amd/compression/plan.py).
//   Aggregate (fused decode + FedAvg, server side): k_aggregate — two waves per unit, a per-wave LDS tile
//   holding the unkept x (base + 0), each client's kept values written in and read back in client order.
//   Dense plans (every segment keeps all its elements, ratio 1): k_dense_minmax -> k_dense_seg -> k_dense_quant
//   encode, k_dense_deq decode — the indices implied, never materialised.
//
// Numerics: built with -ffp-contract=off; fp32 sub/div/mul/add are separate IEEE ops, rintf is
// round-half-even — the same op sequence as the oracle, so decoded values are bit-identical.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/coalac.h"

namespace {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
constexpr uint32_t UNIT = 4096;           // elements per wave work unit
constexpr uint32_t UNIT_SHIFT = 12;
constexpr uint32_t UNIT_IT = UNIT / 256;  // float4 loads per lane per unit
constexpr uint32_t SMALL_MAX = 4096;      // segments up to this size can be encoded whole in one block (the
                                          // small-segment LDS arena; COALAC_SMALL_MAX may raise the limit to it)
constexpr uint32_t SMALL_MAX_BATCH = 1024;  // ... and are, by default, in batch plans (4096 until round 3: C2
                                            // 0.296-0.314 -> 0.280-0.285 ms per step, C3 / C4 equal or faster;
                                            // a 4096-element block select takes 14 us, the sampled path streams it)
constexpr uint32_t SMALL_MAX_LATENCY = 1024;  // ... in latency-bound plans (<= LATENCY_PLAN_UNITS units): a
                                              // block's radix select grows with n (64: 5 us, 2048: 9 us,
                                              // 4096: 14 us, alone on a CU) and the slowest small segment set
                                              // the length of k_presel; bigger segments take the sampled path
constexpr uint32_t LATENCY_PLAN_UNITS = 8192;  // ~1.3 ResNet-50 updates
constexpr uint32_t SAMPLE_KEYS = 8192u;
constexpr uint32_t SAMPLE_MAX = SAMPLE_KEYS;  // sampled keys per large segment
constexpr int SEL_NT = 256;               // threads of a k_select block in batches (4 waves: one per SIMD, so
                                          // a block finds room beside a streaming kernel's waves)
constexpr int GWIN_NT_LAT = 512;  // k_gwin block in latency-bound plans (256 or 512: one or two histogram bins per thread)
constexpr int GHIST_NT_LAT = 1024;  // k_ghist block in latency-bound plans (256 / 512 / 1024: 6.5 / 5.7 / 5.3 us on one update)
constexpr int SEL_NT_LAT = 512;           // ... in latency-bound plans, where nothing streams beside it (one
                                          // ResNet-50 update: k_select 11.3 -> 10.2 us; batches measured slower)
constexpr int SCAN_WPE = 5;
constexpr int SCAN_NT = 128;  // batch plans' k_scan block size (launch bounds: SCAN_WPE waves per SIMD; C3 0.584 vs 0.616 ms at 256)
constexpr int SCAN_NT_LAT = 256;  // latency-bound plans' k_scan block size (its first blocks encode the small segments)
constexpr int SCAN_NB = 1;  // load batches per k_scan unit (weights mode): 1 = all 16 float4 per lane in flight
constexpr int SCAN_WPE_LAT = 6;  // latency-bound plans' k_scan: blocks per CU (5 / 1 batch: 24.5 us, 6 / 2: 23.0, 6 / 1
                                 // spills: 31.7, 8 / 4: 24.2 on one update; batches keep SCAN_WPE / SCAN_NB)
constexpr int SCAN_WPE_LAT_1K = 7;  // ... with the default 1024-element small segments (a 16 KB arena): 7 blocks per CU, so
                                    // one ResNet-50 update's ~1,660 blocks fit one round of the chip's block slots
constexpr int SCAN_NB_LAT = 2;  // ... and load batches per unit
constexpr int SAMPLE_NT_LAT = 256;  // latency-bound plans' k_sample block size (1024 threads, 2 load batches each: 0.7 us slower)
constexpr int LOAD_AUX = 2;   // cache policy of the streaming buffer loads (k_scan, the quantise stream): non-temporal
constexpr int STORE_AUX = 2;  // cache policy of the streaming buffer stores (batch k_decode_lds, k_dense_deq): non-temporal
constexpr uint32_t STAGE_CAP = 512;       // candidate records staged in LDS per k_scan wave
constexpr int GU_UNITS = 32;
constexpr int GSWEEP = 4;  // units per record-load batch of a balanced group sweep (batch plans)
constexpr uint32_t GU = GU_UNITS;               // units per select group (k_ghist / k_gwin block)
constexpr uint32_t HB2 = 512;             // bins of the per-group band histograms
constexpr uint32_t GCAP = 256;            // in-window entries a group may hand to k_select
constexpr uint32_t KEY_MAX = 0x7FFFFFFFu;
constexpr uint32_t TIE_FLAG = 0x80000000u;  // in a unit's T_lo: the sampled k-th key K is a heavy tie (tie mode, k_scan)
constexpr int HIST_BINS = 2048;
constexpr uint32_t UCAP = 2048;           // units per k_select chunk (8.4 M elements)
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr int NSTAMP = 32;  // diagnostics slots per segment row (COALAC_FLAG_STAMPS)

struct SegDev {
  uint64_t in_off;
  uint64_t out_off;
  uint32_t n, k;
  uint32_t unit_begin, unit_end;  // range in the all-units table (decode)
  uint32_t lu_begin;              // first large-unit index (large segments)
  uint32_t g_begin;               // first select group (large segments)
};

struct UnitDev {
  uint64_t off;      // element offset of the unit in the flat buffer (= seg.in_off + start)
  uint64_t out_off;  // the segment's out_off
  uint32_t seg, start;
  uint32_t k;        // the segment's k
  uint16_t len;      // elements in this unit (<= UNIT)
  uint16_t last;     // 1 if this is the segment's last unit
};
static_assert(sizeof(UnitDev) == 32, "UnitDev layout");

struct Params {
  // encode / decode operands
  const float* in;
  const float* const* inptr;  // encode from per-segment pointers (coalac_encode_segptr), else null
  const float* base;
  int32_t* idx;
  void* vals;
  float* mn;
  float* scale;
  uint32_t* ustart_out;  // encode: per-unit start of the unit's kept entries (segment-relative), or null
  const int32_t* cidx;
  const void* cvals;
  const float* cmn;
  const float* cscale;
  float* out;
  // plan metadata
  const SegDev* segs;
  const UnitDev* units;   // all units (decode)
  const UnitDev* lunits;  // units of large segments (encode)
  const uint32_t* small_list;
  const uint32_t* large_list;
  const SegDev* lsegs;  // [n_large] the large segments' SegDev, in large_list order (one load round less)
  const SegDev* ssegs;  // [n_small] the small segments' SegDev, in small_list order (likewise)
  uint32_t nseg, n_small, n_large, n_units, n_lunits;
  uint32_t scan_small;  // small segments encoded by k_scan's first blocks (0 when forked to k_small)
  float levels;
  unsigned flags;
  // encode workspace: per segment
  uint32_t *tstar, *rtie, *status;
  // per large unit
  uint32_t *tlo, *thi, *cntA, *cntC, *gtC, *eqC, *eqpre, *outoff;
  uint32_t* cntZ;  // per large unit of a tie-mode segment (T_lo == 0, or flagged): its keys equal to the tie key K
                   // (0, or T_lo & KEY_MAX) — counted, not recorded
  uint32_t* tsgn;  // ... and, for K > 0, the in-unit tie rank of its first positive (bits 0-15) and first negative
                   // (bits 16-31) tie, 0xFFFF = none (a kept +K / -K tie enters mn / scale; a zero's sign does not)
  uint4* uemit;  // per large unit, from k_select: {T*, tie budget | raw-path flag << 31, mn bits, scale bits}
  uint32_t* cval;  // candidate records, ccap slots per large unit, in index order: the value bits ...
  uint16_t* cpos;  // ... and the position inside the unit (the emit reads both; every select sweep the values only)
  uint32_t ccap;  // record slots per large unit (< UNIT: a unit that finds more candidates overflows and its
                  // segment is selected and emitted from the raw data instead)
  // parallel select (groups of GU units of one large segment)
  const uint4* groups;     // {large-segment index, first large unit, units, segment}
  const uint4* gseg;       // per group, its segment: {first large unit, units, k, first group}
  uint32_t n_groups;
  uint32_t* ghist;         // [n_groups][HB2]
  uint32_t* gcnt;          // [n_groups] in-window entries found by the group
  uint2* glist;            // [n_groups][GCAP] {value bits, unit index within the segment}
  float* gmm;              // [n_groups][2] min/max of the group's values above the window
  uint4* sstate;           // [n_large] {wlo, whi, rank inside the window, path: 0 fast / 1 generic}
  uint32_t* shhi;          // [n_large] histogram upper bound: min(T_hi, largest sampled key)

  // decode: first kept entry (segment-relative) of every unit — the payload's (wire v2)
  const uint32_t* ustart;
  // dense plans (every segment keeps all its elements): per unit the NaN-ignoring {min, max} of its values
  float* umm;
  // diagnostics: per-block phase timestamps (COALAC_FLAG_STAMPS), NSTAMP per block, 100 MHz ticks
  uint64_t* stamps;
};

// ------------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------------
#define DEV __device__ __forceinline__

DEV uint32_t fkey(float x) { return __float_as_uint(x) & KEY_MAX; }

// diagnostics only: thread 0 records the 100 MHz real-time counter for phase i of large segment li
#define STAMP(P, li, i)                                                                             \
  do {                                                                                              \
    if ((P).stamps != nullptr && threadIdx.x == 0)                                                  \
      (P).stamps[(uint64_t)(li) * NSTAMP + (i)] = __builtin_amdgcn_s_memrealtime();                \
  } while (0)

// NaN-ignoring min/max (NaN only if both are NaN) = IEEE minNum/maxNum: one v_min_f32 / v_max_f32
// (hipcc quiets signalling NaNs first, so a NaN operand is always ignored). The sign of a zero result is
// canonicalised at the end (+ 0.0f), which makes the reduction order-independent.
DEV float fmin_nan(float a, float b) { return __builtin_fminf(a, b); }
DEV float fmax_nan(float a, float b) { return __builtin_fmaxf(a, b); }
DEV float qnan() { return __int_as_float(0x7FC00000); }

DEV uint32_t lane_id() { return __lane_id(); }

// lane l's value of v (v_readlane: a wave-uniform result)
DEV uint32_t rl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }

// XCD-aware block order: workgroups are dispatched round-robin over the 8 XCDs (block b on XCD b % 8); the
// remapped index gives XCD x the x-th contiguous share of [0, gridDim.x) (a bijection for any grid size), so
// each XCD streams through one region instead of every eighth 64 KiB. NT stores of the unit pattern, 1.5 GiB:
// 5.56 -> 6.38 TB/s (tools/store_probe.hip); reads and ~100 MB buffers gain nothing.
DEV uint32_t xcd_block(uint32_t b) {
  const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8, i = b / 8;
  return x * q + min(x, r) + i;
}

// number of set bits of `m` in lanes below this lane
DEV uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Cross-lane steps by DPP (a VALU operand modifier: a few cycles) — __shfl_* lowers to ds_bpermute_b32, an LDS round
// trip per step (~100+ cycles), and a wave scan is six dependent steps. dpp<CTRL>: lane i reads lane src(i) of v
// (0 where the source lies outside its row or the row is masked off). CTRL: 0x111 + n - 1 row_shr:n, 0x128 row_ror:8,
// 0x140 row_mirror, 0x141 row_half_mirror, 0x142 row_bcast:15, 0x143 row_bcast:31, 0xB1 / 0x4E quad_perm xor 1 / xor 2.
// min(a, b) kept out of the optimiser's reach: next to min(r, x), the tie quota `x >= r ? 0 : min(c, r - x)` was folded
// into a saturating subtract whose clamp the gfx950 build then dropped — min(r, x) came out as x and a unit reserved a
// slot for a tie it did not keep (k_select, round 6: tools/dbg_encode.py, resnet18 ratio 0.1 delta). With qp = this,
// the quota is min(c, r - qp): r - qp never wraps.
DEV uint32_t umin_opaque(uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_min_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int CTRL, int ROWM = 0xF>
DEV uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWM, 0xF, false);
}

// inclusive prefix sum over the 64 lanes (all lanes active)
DEV uint32_t wave_incl_scan(uint32_t v) {
  v += dpp<0x111>(v);  // row_shr:1, 2, 4, 8: each 16-lane row scanned
  v += dpp<0x112>(v);
  v += dpp<0x114>(v);
  v += dpp<0x118>(v);
  v += dpp<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
  v += dpp<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
  return v;
}

// reduction over the 64 lanes, the result in every lane: within each row by quad / half-row / row mirrors, then the
// four rows' values by readlane
template <class OP>
DEV uint32_t wave_reduce(uint32_t v, OP op) {
  v = op(v, dpp<0xB1>(v));
  v = op(v, dpp<0x4E>(v));
  v = op(v, dpp<0x141>(v));
  v = op(v, dpp<0x140>(v));
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return op(op(a, b), op(c, d));
}

DEV float wave_min(float v) {
  return __uint_as_float(wave_reduce(__float_as_uint(v), [](uint32_t a, uint32_t b) {
    return __float_as_uint(fmin_nan(__uint_as_float(a), __uint_as_float(b)));
  }));
}

DEV float wave_max(float v) {
  return __uint_as_float(wave_reduce(__float_as_uint(v), [](uint32_t a, uint32_t b) {
    return __float_as_uint(fmax_nan(__uint_as_float(a), __uint_as_float(b)));
  }));
}

DEV uint32_t wave_min_u32(uint32_t v) {
  return wave_reduce(v, [](uint32_t a, uint32_t b) { return min(a, b); });
}

DEV uint32_t wave_max_u32(uint32_t v) {
  return wave_reduce(v, [](uint32_t a, uint32_t b) { return max(a, b); });
}

DEV uint32_t wave_sum(uint32_t v) {
  return wave_reduce(v, [](uint32_t a, uint32_t b) { return a + b; });
}

// Order one wave's own LDS accesses (a scatter, then reads of the same tile by other lanes): the LDS executes a
// wave's DS instructions in issue order, so only the compiler must not move them across this point. Unlike
// wave_fence (a wavefront-scope seq_cst fence), it emits no s_waitcnt: loads in flight stay in flight.
DEV void lds_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

DEV void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// stores of the select phases' per-group / per-segment results (plain global stores)
DEV void pst(const Params&, uint32_t* p, uint32_t v) { *p = v; }
DEV void pst(const Params&, float* p, float v) { *p = v; }
DEV void pst(const Params&, uint2* p, uint2 v) { *p = v; }

// Block-wide exclusive scan over NT threads. sh needs >= NT/64 words. Returns the exclusive prefix and
// the block total. Contains barriers: call from all threads.
template <int NT>
DEV uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
  constexpr int NW = NT / 64;
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan(v);
  __syncthreads();
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    uint32_t s = sh[i];
    if ((uint32_t)i < w) off += s;
    tot += s;
  }
  total = tot;
  return off + inc - v;
}

// Two block-wide exclusive scans sharing one pair of barriers (sh needs >= 2 * NT/64 words). Call from all threads.
template <int NT>
DEV void block_excl_scan2(uint32_t a, uint32_t b, uint32_t* sh, uint32_t& ea, uint32_t& eb, uint32_t& ta,
                          uint32_t& tb) {
  constexpr int NW = NT / 64;
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  const uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b);
  __syncthreads();
  if (lane == 63) {
    sh[w] = ia;
    sh[NW + w] = ib;
  }
  __syncthreads();
  uint32_t oa = 0, ob = 0, sa = 0, sb = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t x = sh[i], y = sh[NW + i];
    if ((uint32_t)i < w) {
      oa += x;
      ob += y;
    }
    sa += x;
    sb += y;
  }
  ea = oa + ia - a;
  eb = ob + ib - b;
  ta = sa;
  tb = sb;
}

template <int NT>
DEV uint32_t block_sum(uint32_t v, uint32_t* sh) {
  uint32_t t;
  block_excl_scan<NT>(v, sh, t);
  return t;
}

// shf needs >= 2 * NT/64 floats
template <int NT>
DEV void block_minmax(float& mn, float& mx, float* shf) {
  constexpr int NW = NT / 64;
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  mn = wave_min(mn);
  mx = wave_max(mx);
  __syncthreads();
  if (lane == 0) {
    shf[w] = mn;
    shf[NW + w] = mx;
  }
  __syncthreads();
  float a = shf[0], b = shf[NW];
#pragma unroll
  for (int i = 1; i < NW; ++i) {
    a = fmin_nan(a, shf[i]);
    b = fmax_nan(b, shf[NW + i]);
  }
  mn = a;
  mx = b;
}

// Exact selection of the r-th largest key (1-based) among the keys in [lo, hi] that `for_each`
// enumerates (each thread enumerates its own share; the union is the key multiset). Returns T with
// count(key in (T, hi]) < r <= count(key in [T, hi]) and leaves in r the number of keys == T to take
// (r - count(key in (T, hi])). Radix narrowing with 2048-bin LDS histograms: at most 3 passes over the
// keys for a full 31-bit range. Once the bin holding the r-th key has at most RANK_MAX keys, they are
// gathered into LDS (one more enumeration) and ranked against each other instead of further radix passes
// (a small segment's keys crowd a few exponent bins: 3 passes -> 1 pass + gather + rank). sh needs >= 64
// words (broadcast slots sh[36]-sh[41]).
constexpr uint32_t RANK_MAX = 256;

template <int NT, class ForEach>
DEV uint32_t rank_select(ForEach&& for_each, uint32_t lo, uint32_t hi, uint32_t& r, uint32_t* cand, uint32_t* sh) {
  const uint32_t t = threadIdx.x, lane = lane_id();
  if (t == 0) {
    sh[39] = 0;
    sh[36] = lo;
    sh[37] = r;
  }
  __syncthreads();
  for_each([&](uint32_t key) {  // wave-aggregated append of the bin's keys
    const bool in = key >= lo && key <= hi;
    const uint64_t m = __ballot(in);
    if (m) {
      const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1u;
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(&sh[39], (uint32_t)__popcll(m));
      base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
      if (in) cand[base + mbcnt(m)] = key;
    }
  });
  __syncthreads();
  const uint32_t c = sh[39];
  for (uint32_t i = t; i < c; i += NT) {
    const uint32_t ki = cand[i];
    uint32_t g = 0, e = 0;
    for (uint32_t j = 0; j < c; ++j) {  // every thread reads the same word: LDS broadcast
      const uint32_t kj = cand[j];
      g += kj > ki ? 1u : 0u;
      e += kj == ki ? 1u : 0u;
    }
    if (g < r && r <= g + e) {  // the r-th key (every tie of it writes the same two words)
      sh[36] = ki;
      sh[37] = r - g;
    }
  }
  __syncthreads();
  const uint32_t T = sh[36];
  r = sh[37];
  __syncthreads();
  return T;
}

template <int NT, int NB = HIST_BINS, class ForEach>
DEV uint32_t block_select(ForEach&& for_each, uint32_t lo, uint32_t hi, uint32_t& r, uint32_t* hist,
                          uint32_t* sh) {
  constexpr int BPT = NB / NT;  // bins per thread
  constexpr int BITS = NB == 2048 ? 11 : NB == 1024 ? 10 : NB == 512 ? 9 : 8;
  static_assert((1 << BITS) == NB, "power-of-two bins");
  const uint32_t t = threadIdx.x;
  while (lo < hi) {
    const uint32_t w = hi - lo;
    const int bl = 32 - __clz(w);
    const int shift = bl > BITS ? bl - BITS : 0;
    for (uint32_t i = t; i < NB; i += NT) hist[i] = 0;
    __syncthreads();
    const uint32_t l0 = lo, h0 = hi;
    for_each([&](uint32_t key) {
      if (key >= l0 && key <= h0) atomicAdd(&hist[(key - l0) >> shift], 1u);
    });
    __syncthreads();
    uint32_t c[BPT];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      c[j] = hist[t * BPT + j];
      s += c[j];
    }
    uint32_t total;
    const uint32_t ex = block_excl_scan<NT>(s, sh, total);
    const uint32_t above = total - ex - s;  // keys in bins above this thread's bins
    if (t == 0) {
      sh[40] = NONE;
      sh[41] = r;
    }
    __syncthreads();
    if (above < r && r <= above + s) {
      uint32_t acc = above, cb = 0;
      int b = (int)(t * BPT);
#pragma unroll
      for (int j = BPT - 1; j >= 0; --j) {
        if (acc + c[j] >= r) {
          b = (int)(t * BPT) + j;
          cb = c[j];
          break;
        }
        acc += c[j];
      }
      sh[40] = (uint32_t)b;
      sh[41] = r - acc;
      sh[38] = cb;  // keys in the chosen bin
    }
    __syncthreads();
    const uint32_t b = sh[40];
    r = sh[41];
    const uint32_t bc = sh[38];
    __syncthreads();
    if (b == NONE) return lo;  // precondition violated (cannot happen for valid inputs)
    lo = lo + (b << shift);
    const uint32_t nhi = lo + ((1u << shift) - 1u);
    hi = nhi < hi ? nhi : hi;
    if (lo < hi && bc <= RANK_MAX && NB >= (int)RANK_MAX)
      return rank_select<NT>(for_each, lo, hi, r, hist, sh);
  }
  return lo;
}

DEV uint8_t quantize(float v, float mn, float scale, float levels) {
  if (!(scale > 0.0f)) return 0;
  const float t = (v - mn) / scale;
  const float r = rintf(t);
  if (!(r > 0.0f)) return 0;
  return (uint8_t)(r < levels ? r : levels);
}

DEV float dequantize(uint8_t q, float mn, float scale) {
  const float p = (float)q * scale;
  return mn + p;
}

template <bool RAW>
DEV void store_val(const Params& P, uint64_t o, float v, float mn, float scale) {
  if (RAW)
    static_cast<float*>(P.vals)[o] = v;
  else
    static_cast<uint8_t*>(P.vals)[o] = quantize(v, mn, scale, P.levels);
}

template <bool RAW>
DEV float load_val(const Params& P, uint64_t o, float mn, float scale) {
  if (RAW) return static_cast<const float*>(P.cvals)[o];
  return dequantize(static_cast<const uint8_t*>(P.cvals)[o], mn, scale);
}

template <bool RAW>
DEV uint32_t load_code(const Params& P, uint64_t o) {
  if (RAW) return __float_as_uint(static_cast<const float*>(P.cvals)[o]);
  return static_cast<const uint8_t*>(P.cvals)[o];
}

template <bool RAW>
DEV float code_value(uint32_t q, float mn, float scale) {
  return RAW ? __uint_as_float(q) : dequantize((uint8_t)q, mn, scale);
}

template <bool DELTA>
DEV float4 load_x4(const Params& P, uint64_t off) {
  float4 v = *reinterpret_cast<const float4*>(P.in + off);
  if (DELTA) {
    const float4 b = *reinterpret_cast<const float4*>(P.base + off);
    v.x = v.x - b.x;
    v.y = v.y - b.y;
    v.z = v.z - b.z;
    v.w = v.w - b.w;
  }
  return v;
}

typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

// histogram shift of the sampled band [tlo, thi]: HIST_BINS bins of 2^shift keys cover it. k_scan
// (band histogram) and k_select (bin -> key window) must agree, so both use this.
DEV int band_shift(uint32_t tlo, uint32_t thi, int bin_bits = 11) {
  const uint32_t w = thi - tlo;
  if (w == 0) return 0;
  const int bl = 32 - __clz(w);
  return bl > bin_bits ? bl - bin_bits : 0;
}

// Buffer resource over n fp32 elements at p (gfx9 word 3; loads at byte offsets >= 4n return 0).
DEV __amdgpu_buffer_rsrc_t unit_rsrc(const float* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)(n * 4u), 0x00020000);
}

// non-temporal 16-byte buffer load (aux bit 1 = nt on gfx94x/gfx950) of x (or x - base) at byte offset
template <bool DELTA>
DEV float4 unit_load_x4(__amdgpu_buffer_rsrc_t rin, __amdgpu_buffer_rsrc_t rbase, uint32_t boff) {
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const u4v a = __builtin_amdgcn_raw_buffer_load_b128(rin, (int)boff, 0, LOAD_AUX);
  float4 v = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
  if (DELTA) {
    const u4v b = __builtin_amdgcn_raw_buffer_load_b128(rbase, (int)boff, 0, LOAD_AUX);
    v.x = v.x - __uint_as_float(b.x);
    v.y = v.y - __uint_as_float(b.y);
    v.z = v.z - __uint_as_float(b.z);
    v.w = v.w - __uint_as_float(b.w);
  }
  return v;
}

// non-temporal 16-byte buffer store (dropped when it lies past the resource's range)
template <int AUX = STORE_AUX>
DEV void unit_store_x4(__amdgpu_buffer_rsrc_t r, uint32_t boff, float4 v) {
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const u4v a = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(a, r, (int)boff, 0, AUX);
}

// the same 16 bytes as four dword stores: the range check drops exactly the dwords past the end
template <int AUX = STORE_AUX>
DEV void unit_store_x1x4(__amdgpu_buffer_rsrc_t r, uint32_t boff, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.x), r, (int)boff, 0, AUX);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.y), r, (int)boff + 4, 0, AUX);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.z), r, (int)boff + 8, 0, AUX);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.w), r, (int)boff + 12, 0, AUX);
}

// non-temporal (read-once) 16-byte load of x (or x - base)
template <bool DELTA>
DEV float4 load_x4_nt(const Params& P, uint64_t off) {
  const f4v a = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(P.in + off));
  float4 v = make_float4(a.x, a.y, a.z, a.w);
  if (DELTA) {
    const f4v b = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(P.base + off));
    v.x = v.x - b.x;
    v.y = v.y - b.y;
    v.z = v.z - b.z;
    v.w = v.w - b.w;
  }
  return v;
}

template <bool DELTA>
DEV float load_x1(const Params& P, uint64_t off) {
  float v = P.in[off];
  if (DELTA) v = v - P.base[off];
  return v;
}

// Input of segment s: its own pointer (coalac_encode_segptr: the model's parameter storage, no flattening
// copy) or the flat buffer at in_off. The delta base is always the flat buffer.
DEV const float* seg_in(const Params& P, uint32_t s, uint64_t in_off) {
  return P.inptr != nullptr ? P.inptr[s] : P.in + in_off;
}

template <bool DELTA>
DEV float4 load_x4p(const float* x, const float* b) {
  float4 v = *reinterpret_cast<const float4*>(x);
  if (DELTA) {
    const float4 c = *reinterpret_cast<const float4*>(b);
    v.x = v.x - c.x;
    v.y = v.y - c.y;
    v.z = v.z - c.z;
    v.w = v.w - c.w;
  }
  return v;
}

template <bool DELTA>
DEV float load_x1p(const float* x, const float* b) {
  float v = *x;
  if (DELTA) v = v - *b;
  return v;
}

DEV uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// Group-histogram geometry of a segment: bins of 2^shift keys over [tlo, hhi]; keys in (hhi, thi] are
// clamped into the last bin, whose key window therefore ends at thi.
struct Band {
  uint32_t tlo, thi, hhi, last;
  int shift;
  DEV Band(uint32_t lo, uint32_t hi, uint32_t hh) : tlo(lo), thi(hi), hhi(hh) {
    shift = band_shift(lo, hh, 9);
    last = (hh - lo) >> shift;
  }
  DEV uint32_t bin(uint32_t key) const { return key > hhi ? last : (key - tlo) >> shift; }
  DEV uint32_t wlo(uint32_t b) const { return tlo + (b << shift); }
  DEV uint32_t whi(uint32_t b) const { return b == last ? thi : min(thi, wlo(b) + ((1u << shift) - 1u)); }
};

// ------------------------------------------------------------------------------------------------
// streaming classify + ordered compaction of one large unit by one wave (k_scan, exact fallback)
// Candidates (key >= tlo) are written in index order as records {position in the unit, value}: two arrays, the
// u16 positions (cpos) and the value bits (cval) — 6 bytes per record, and the select sweeps, which read values
// only, move 4 (round 3's interleaved 8-byte records: k_scan's writes were 4.4 % of its read traffic). With `stage` (k_scan) the first STAGE_CAP records go to a per-wave
// LDS buffer and leave in coalesced 512-byte stores at the end; scattered per-lane global stores were
// measured 28 % slower (tools/scan_ablate.hip). Input loads are non-temporal: the update is read once.
// The unit is loaded in NB batches of UNIT_IT/NB float4 per lane: NB = 1 for the streaming pass (all
// loads in flight at once), more for the register-lean fallback inside k_select.
// ------------------------------------------------------------------------------------------------
// CHECK: test each element against the unit's length. A full unit never needs it, nor does a partial one when
// tlo > 0 (its loads past len return 0, key 0 < tlo): k_scan picks the lean form then (wave-uniform).
// ZERO = tie mode, for a segment whose k-th key may be one heavily repeated key K: K = 0 when the bracket starts at
// key 0 (tlo == 0: a frozen or pruned tensor, an all-zero delta), or the K the sampler flagged (T_lo = K | TIE_FLAG,
// T_hi = K: its samples around the k-th rank were all K — a sign-SGD or first-Adam-step delta whose |x| are all equal,
// values clipped at a bound, a quantised tensor). Keys equal to K are COUNTED per unit (cntZ), not recorded; the
// candidates are the keys above K (in [K + 1, thi], and above). The select then takes the k-th key as K with a tie
// quota over the K-keys (index order) when the keys above K number fewer than k, and only the units whose K-keys that
// quota reaches re-read their raw data in k_emit — instead of every element becoming a candidate record, every unit
// overflowing its slots and the whole segment taking the one-block raw-data path (one ResNet-50 update of equal-|x|
// values: 9.0 ms per encode + decode on that path, tools/tie_probe.py). For K > 0 the scan also records the in-unit
// rank of the first positive and first negative K-key (tsgn): whether +K / -K is among the kept values.
template <bool DELTA, int NB, bool CHECK = true, bool ZERO = false>
DEV void scan_unit(const Params& P, uint32_t lu, const UnitDev& L, const uint32_t tlo_, const uint32_t thi,
                   uint2* stage) {
  const uint32_t tk = tlo_ & KEY_MAX;     // (ZERO: the tie key K)
  const uint32_t tlo = ZERO ? tk + 1u : tlo_;
  uint32_t cz = 0;                        // K-keys this lane saw (ZERO)
  uint32_t weq = 0, rp = NONE, rn = NONE;  // (ZERO, K > 0: K-keys of the earlier rows; first +K / -K tie rank)
  constexpr uint32_t IT = UNIT_IT / NB;
  const uint32_t lane = lane_id();
  const uint32_t len = L.len;
  const uint64_t off = L.off;
  uint32_t* RV = P.cval + (uint64_t)lu * P.ccap;
  uint16_t* RP = P.cpos + (uint64_t)lu * P.ccap;
  const uint32_t cap = P.ccap;
  uint32_t cC = 0, cA = 0;
  // buffer resources over exactly this unit: one shared lane offset for all loads (constant offsets
  // fold into the instruction), and loads past len return 0 — no separate partial-unit path
  const float* xin = P.inptr != nullptr ? P.inptr[L.seg] + L.start : P.in + off;
  const __amdgpu_buffer_rsrc_t rin = unit_rsrc(xin, len);
  const __amdgpu_buffer_rsrc_t rbase = unit_rsrc(DELTA ? P.base + off : xin, len);
  auto put = [&](uint32_t i, uint2 rec) {
    if (i >= cap) return;  // overflow: counted, not stored (the segment goes to the raw-data path)
    RV[i] = rec.y;
    RP[i] = (uint16_t)rec.x;
  };

  for (uint32_t nb = 0; nb < (uint32_t)NB; ++nb) {
    float4 v[IT];
#pragma unroll
    for (uint32_t i = 0; i < IT; ++i) v[i] = unit_load_x4<DELTA>(rin, rbase, ((nb * IT + i) * 64 + lane) * 16);
#pragma unroll
    for (uint32_t i = 0; i < IT; ++i) {
      const uint32_t e0 = ((nb * IT + i) * 64 + lane) * 4;
      const float xs[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
      bool fc[4], fa[4];
      bool any = false;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t key = fkey(xs[j]);
        fc[j] = (!CHECK || e0 + j < len) && key >= tlo;
        fa[j] = CHECK ? fc[j] && key > thi : key > thi;  // (thi >= tlo or ZERO: key > thi implies a candidate)
        if (ZERO) cz += ((!CHECK || e0 + j < len) && key == tk) ? 1u : 0u;
        any = any || fc[j];
      }
      if (ZERO && tk != 0u) {  // (wave-uniform) the in-unit ranks of this row's K-keys: index order is (lane, j)
        uint64_t tb[4];
        uint32_t pre = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          tb[j] = __ballot((!CHECK || e0 + j < len) && fkey(xs[j]) == tk);
          pre += mbcnt(tb[j]);
        }
        uint32_t mine = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if ((tb[j] >> lane) & 1ull) {
            const uint32_t rank = weq + pre + mine;
            if (__float_as_uint(xs[j]) >> 31)
              rn = min(rn, rank);
            else
              rp = min(rp, rank);
            ++mine;
          }
        }
        weq += (uint32_t)(__popcll(tb[0]) + __popcll(tb[1]) + __popcll(tb[2]) + __popcll(tb[3]));
      }
      const uint32_t c = (uint32_t)fc[0] + (uint32_t)fc[1] + (uint32_t)fc[2] + (uint32_t)fc[3];
      const uint64_t b1 = __ballot(any);
      if (b1 == 0) continue;
      if (__ballot(c >= 2) == 0) {
        // common case (~1.5 % candidates: ~4 per 256-element row): at most one candidate per lane, so its
        // position is one mbcnt instead of four, and each lane writes at most one record
        cA += (uint32_t)__popcll(__ballot(fa[0] || fa[1] || fa[2] || fa[3]));
        if (any) {
          const uint32_t pc = cC + mbcnt(b1);
          const uint32_t j = fc[0] ? 0u : fc[1] ? 1u : fc[2] ? 2u : 3u;
          const float xj = j == 0 ? xs[0] : j == 1 ? xs[1] : j == 2 ? xs[2] : xs[3];
          const uint2 rec = make_uint2(e0 + j, __float_as_uint(xj));
          if (stage != nullptr && pc < STAGE_CAP)
            stage[pc] = rec;
          else
            put(pc, rec);
        }
        cC += (uint32_t)__popcll(b1);
        continue;
      }
      uint64_t bc[4];
      uint32_t pc = cC;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bc[j] = __ballot(fc[j]);
        pc += mbcnt(bc[j]);
        cA += (uint32_t)__popcll(__ballot(fa[j]));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (fc[j]) {
          const uint2 rec = make_uint2(e0 + j, __float_as_uint(xs[j]));
          if (stage != nullptr && pc < STAGE_CAP)
            stage[pc] = rec;
          else
            put(pc, rec);
          ++pc;
        }
        cC += (uint32_t)__popcll(bc[j]);
      }
    }
  }
  if (stage != nullptr) {
    wave_fence();
    for (uint32_t i = lane; i < cC && i < STAGE_CAP; i += 64) put(i, stage[i]);
  }
  if (ZERO) {
    cz = wave_sum(cz);
    if (tk != 0u) {
      rp = wave_min_u32(rp);
      rn = wave_min_u32(rn);
    }
  }
  if (lane == 0) {
    P.cntA[lu] = cA;
    P.cntC[lu] = cC;
    if (ZERO) P.cntZ[lu] = cz;
    if (ZERO && tk != 0u) P.tsgn[lu] = min(rp, 0xFFFFu) | (min(rn, 0xFFFFu) << 16);
  }
}


// Pick the bin of a HIST_BINS histogram (LDS) holding the r-th largest key: returns the bin, leaves in
// r the rank inside that bin. sh needs >= 64 words.
template <int NT, int NB = HIST_BINS>
DEV uint32_t hist_pick(const uint32_t* hist, uint32_t& r, uint32_t* sh) {
  constexpr int BPT = NB / NT;
  const uint32_t t = threadIdx.x;
  uint32_t c[BPT];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    c[j] = hist[t * BPT + j];
    s += c[j];
  }
  uint32_t total;
  const uint32_t ex = block_excl_scan<NT>(s, sh, total);
  const uint32_t above = total - ex - s;
  if (t == 0) {
    sh[40] = NONE;
    sh[41] = r;
  }
  __syncthreads();
  if (above < r && r <= above + s) {
    uint32_t acc = above;
    int b = (int)(t * BPT);
#pragma unroll
    for (int j = BPT - 1; j >= 0; --j) {
      if (acc + c[j] >= r) {
        b = (int)(t * BPT) + j;
        break;
      }
      acc += c[j];
    }
    sh[40] = (uint32_t)b;
    sh[41] = r - acc;
  }
  __syncthreads();
  const uint32_t b = sh[40];
  r = sh[41];
  __syncthreads();
  return b;
}

// hist_pick for two ranks at once (r1, r2; 0 = not wanted): ONE block scan of the bins instead of two.
// Returns the bins in b1 / b2 (NONE when not wanted) and the ranks inside them in q1 / q2. sh needs >= 64 words
// (slots 40-43).
template <int NT, int NB = HIST_BINS>
DEV void hist_pick2(const uint32_t* hist, uint32_t r1, uint32_t r2, uint32_t& b1, uint32_t& b2, uint32_t& q1,
                    uint32_t& q2, uint32_t* sh) {
  constexpr int BPT = NB / NT;
  const uint32_t t = threadIdx.x;
  uint32_t c[BPT];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    c[j] = hist[t * BPT + j];
    s += c[j];
  }
  uint32_t total;
  const uint32_t ex = block_excl_scan<NT>(s, sh, total);
  const uint32_t above = total - ex - s;
  if (t == 0) {
    sh[40] = NONE;
    sh[41] = NONE;
    sh[42] = 0u;
    sh[43] = 0u;
  }
  __syncthreads();
  const uint32_t rr[2] = {r1, r2};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const uint32_t r = rr[q];
    if (r != 0 && above < r && r <= above + s) {
      uint32_t acc = above;
      int b = (int)(t * BPT);
#pragma unroll
      for (int j = BPT - 1; j >= 0; --j) {
        if (acc + c[j] >= r) {
          b = (int)(t * BPT) + j;
          break;
        }
        acc += c[j];
      }
      sh[40 + q] = (uint32_t)b;
      sh[42 + q] = r - acc;
    }
  }
  __syncthreads();
  b1 = sh[40];
  b2 = sh[41];
  q1 = sh[42];
  q2 = sh[43];
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// small segments (n <= SMALL_MAX): one 256-thread block, values in LDS, exact radix select, ordered
// compaction, min/max, codes. Runs as its own kernel (k_small) on the plan's side stream, concurrently
// with k_sample / k_scan, so its latency hides under the HBM streaming.
// ------------------------------------------------------------------------------------------------
template <bool DELTA, bool RAW, int NT = BLOCK>
DEV void small_encode(const Params& P, uint32_t si, float* vals, uint32_t* hist, uint32_t* sh) {
  const uint32_t t = threadIdx.x;
  const uint32_t s = P.small_list[si];
  const SegDev sd = P.ssegs[si];  // (the same load round as s)
  const float* xs = seg_in(P, s, sd.in_off);
  const float* bs = DELTA ? P.base + sd.in_off : xs;
  const uint32_t n = sd.n, k = sd.k;
  STAMP(P, s, 2);  // (slots 2-7: small segments; k_select uses 0, 1, 10-12 of the large segments' rows)
  if (n == 0) {
    if (t == 0) {
      P.mn[s] = 0.0f;
      P.scale[s] = 0.0f;
    }
    return;
  }
  for (uint32_t i = t * 4; i < n; i += NT * 4) {
    if (i + 3 < n) {
      const float4 v = load_x4p<DELTA>(xs + i, bs + i);
      vals[i + 0] = v.x;
      vals[i + 1] = v.y;
      vals[i + 2] = v.z;
      vals[i + 3] = v.w;
    } else {
      for (uint32_t j = i; j < n; ++j) vals[j] = load_x1p<DELTA>(xs + j, bs + j);
    }
  }
  __syncthreads();
  STAMP(P, s, 3);
  uint32_t rt = k;
  const uint32_t T = block_select<NT>(
      [&](auto&& f) {
        for (uint32_t i = t; i < n; i += NT) f(fkey(vals[i]));
      },
      0u, KEY_MAX, rt, hist, sh);
  STAMP(P, s, 4);

  // ordered ownership: thread t owns the contiguous range [b0, b1); the first rt ties are kept
  const uint32_t E = (n + NT - 1) / NT;
  const uint32_t b0 = min(n, t * E), b1 = min(n, b0 + E);
  uint32_t gt = 0, eq = 0;
  for (uint32_t i = b0; i < b1; ++i) {
    const uint32_t key = fkey(vals[i]);
    gt += key > T;
    eq += key == T;
  }
  uint32_t eqtot;
  const uint32_t eqpre = block_excl_scan<NT>(eq, sh, eqtot);
  const uint32_t quota = min(eq, rt - umin_opaque(rt, eqpre));
  uint32_t seltot;
  const uint32_t opre = block_excl_scan<NT>(gt + quota, sh, seltot);
  STAMP(P, s, 5);

  float mn = 0.0f, scale = 0.0f;
  if (!RAW) {
    float a = qnan(), b = qnan();
    uint32_t eqseen = 0;
    for (uint32_t i = b0; i < b1; ++i) {
      const float x = vals[i];
      const uint32_t key = fkey(x);
      const bool sel = key > T || (key == T && eqseen++ < quota);
      if (sel) {
        a = fmin_nan(a, x);
        b = fmax_nan(b, x);
      }
    }
    block_minmax<NT>(a, b, reinterpret_cast<float*>(sh));
    a = a + 0.0f;
    b = b + 0.0f;
    mn = a;
    scale = (b == a) ? 0.0f : (b - a) / P.levels;
  }
  STAMP(P, s, 6);
  if (t == 0) {
    P.mn[s] = mn;
    P.scale[s] = scale;
    if (P.ustart_out != nullptr) P.ustart_out[sd.unit_begin] = 0u;  // (n <= SMALL_MAX < UNIT: one unit)
  }
  uint64_t o = sd.out_off + opre;
  uint32_t eqseen = 0;
  for (uint32_t i = b0; i < b1; ++i) {
    const float x = vals[i];
    const uint32_t key = fkey(x);
    const bool sel = key > T || (key == T && eqseen++ < quota);
    if (sel) {
      P.idx[o] = (int32_t)i;
      store_val<RAW>(P, o, x, mn, scale);
      ++o;
    }
  }
  STAMP(P, s, 7);
}

template <bool DELTA, bool RAW>
__global__ __launch_bounds__(BLOCK) void k_small(Params P) {
  __shared__ __attribute__((aligned(16))) float vals[SMALL_MAX];
  __shared__ uint32_t hist[HIST_BINS];
  __shared__ uint32_t sh[64];
  small_encode<DELTA, RAW>(P, blockIdx.x, vals, hist, sh);
}

// ------------------------------------------------------------------------------------------------
// k_sample: per large segment, sampled thresholds [T_lo, T_hi] for every unit of the segment
// ------------------------------------------------------------------------------------------------
template <bool DELTA, int NT = BLOCK>
DEV void sample_segment(const Params& P, uint32_t li, uint32_t* hist, uint32_t* sh) {
  constexpr uint32_t RPI = NT / 4;                   // runs per load batch (4 threads per 16-element run)
  constexpr uint32_t MAXIT = SAMPLE_MAX / 16 / RPI;  // load batches per thread
  const uint32_t t = threadIdx.x;
  STAMP(P, li, 16);  // (slots 16-19: k_sample, 20-21: k_ghist, 22-24: k_gwin of the segment's last group block)
  const uint32_t s = P.large_list[li];
  const SegDev sd = P.lsegs[li];  // (the same load round as s: no dependent segment-table lookup)
  const float* xs = seg_in(P, s, sd.in_off);
  const float* bs = DELTA ? P.base + sd.in_off : xs;
  const uint32_t n = sd.n, k = sd.k;
  // R runs of 16 contiguous elements, one per stratum of n / R elements, jittered inside it.
  uint32_t R = n / 512;
  R = R < 64 ? 64 : (R > SAMPLE_MAX / 16 ? SAMPLE_MAX / 16 : R);
  R &= ~63u;
  const uint32_t m = R * 16;
  const uint32_t stride = n / R;  // >= 16 because n > small_max >= 1024
  const uint32_t room = stride - 16;
  // The sampled keys stay in registers (4 per batch per thread): all loads in flight at once, and with
  // 8 KB of LDS per block (histogram only) twice as many sample blocks fit a CU as with an LDS key copy.
  uint32_t kk[MAXIT][4];
  uint32_t okm = 0;  // bit it: this thread's batch-it run exists (R is a multiple of 64, not of RPI)
#pragma unroll
  for (uint32_t it = 0; it < MAXIT; ++it) {
    const uint32_t r0 = it * RPI + (t >> 2), q = t & 3;
    okm |= (uint32_t)(r0 < R) << it;
    const uint32_t run = r0 < R ? r0 : R - 1;
    uint32_t start = run * stride + hash32(run * 0x9E3779B9u ^ (s + 1u) * 0x85EBCA6Bu) % (room + 1u);
    start &= ~3u;
    const float4 v = load_x4p<DELTA>(xs + start + q * 4, bs + start + q * 4);
    kk[it][0] = fkey(v.x);
    kk[it][1] = fkey(v.y);
    kk[it][2] = fkey(v.z);
    kk[it][3] = fkey(v.w);
  }
  // Expected sample rank of the k-th key, widened by a margin that assumes partially correlated runs.
  const double p = (double)k / (double)n;
  const double se = p * (double)m;
  const double d = 6.0 * sqrt(se) + 8.0;
  const double rlo = ceil(se + d), rhi = floor(se - d);
  // One histogram pass over the sample's own key range; thresholds are bin EDGES taken outward (lower
  // edge for T_lo, upper edge for T_hi), which only widens the bracket.
  if (t == 0) {
    sh[44] = KEY_MAX;
    sh[45] = 0u;
  }
  for (uint32_t i = t; i < HIST_BINS; i += NT) hist[i] = 0;
  __syncthreads();
  uint32_t kmn = KEY_MAX, kmx = 0;
#pragma unroll
  for (uint32_t it = 0; it < MAXIT; ++it) {
    if ((okm >> it) & 1u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        kmn = min(kmn, kk[it][j]);
        kmx = max(kmx, kk[it][j]);
      }
    }
  }
  kmn = wave_min_u32(kmn);
  kmx = wave_max_u32(kmx);
  if (lane_id() == 0) {
    atomicMin(&sh[44], kmn);
    atomicMax(&sh[45], kmx);
  }
  __syncthreads();
  STAMP(P, li, 17);
  const uint32_t kmin = sh[44], kmax = sh[45];
  const int shift = band_shift(kmin, kmax);
#pragma unroll
  for (uint32_t it = 0; it < MAXIT; ++it) {
    if ((okm >> it) & 1u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(&hist[(kk[it][j] - kmin) >> shift], 1u);
    }
  }
  __syncthreads();
  uint32_t tlo = 0u, thi = KEY_MAX;
  uint32_t blo = 0, bhi = 0, qlo = 0, qhi = 0;  // both bracket bins (and ranks inside) from one scan of the histogram
  // (a sample too small for an upper margin, rhi < 1, leaves T_hi open; the top sample's bin is still picked, for the
  // tie test below)
  hist_pick2<NT>(hist, rlo < (double)m ? (uint32_t)rlo : 0u, rhi >= 1.0 ? (uint32_t)rhi : 1u, blo, bhi, qlo, qhi, sh);
  if (rlo < (double)m) tlo = kmin + (blo << shift);
  if (rhi >= 1.0) {
    const uint64_t edge = (uint64_t)kmin + (((uint64_t)bhi + 1) << shift) - 1;
    thi = (uint32_t)min<uint64_t>(edge, kmax);
  }
  bool tie = false;
  const uint32_t mw = rlo < (double)m ? (uint32_t)rlo - (rhi >= 1.0 ? (uint32_t)rhi : 1u) : 0u;  // margin width (ranks)
  if (rlo < (double)m && (blo == bhi || hist[blo] >= mw)) {
    // The sampled keys are concentrated where the bracket lies: both bracket ranks in ONE bin, or the lower rank's bin
    // holding at least the margin's width of samples (continuous data spreads the margin's ~120 ranks over several
    // bins, each holding a few). Refine inside the bin, 11 bits per pass: while the two ranks share a sub-bin (or for
    // the lower rank alone), down to single keys. Two ranks that part: the bracket is their sub-bins' outward edges.
    // Otherwise the lower rank's key K is exact, and a K repeated in the sample (the margin's quarter, >= 8 samples)
    // is a heavy tie: tie mode (T_lo = K | TIE_FLAG; both ranks on K: T_hi = K too). A K seen fewer times is the
    // lower edge itself.
    const bool two = blo == bhi;
    uint32_t base = kmin + (blo << shift), cK = hist[blo];
    int sft = shift;
    bool split = false;
    __syncthreads();  // (every thread has read hist[blo] before the first refinement clears it)
    while (sft > 0) {
      const int ns = sft > 11 ? sft - 11 : 0;
      const uint32_t top = base + ((1u << sft) - 1u);  // (no wrap: the bin lies inside [kmin, kmax + 2^shift))
      for (uint32_t i = t; i < HIST_BINS; i += NT) hist[i] = 0;
      __syncthreads();
#pragma unroll
      for (uint32_t it = 0; it < MAXIT; ++it) {
        if ((okm >> it) & 1u) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kk[it][j] >= base && kk[it][j] <= top) atomicAdd(&hist[(kk[it][j] - base) >> ns], 1u);
        }
      }
      __syncthreads();
      uint32_t b1, b2;
      hist_pick2<NT>(hist, qlo, two ? qhi : 0u, b1, b2, qlo, qhi, sh);
      if (two && b1 != b2) {
        tlo = base + (b1 << ns);
        if (rhi >= 1.0) thi = min<uint64_t>((uint64_t)base + (((uint64_t)b2 + 1) << ns) - 1, kmax);
        split = true;
        break;
      }
      cK = hist[b1];
      __syncthreads();
      base += b1 << ns;
      sft = ns;
    }
    if (!split) {
      if (base != 0u && (two || cK >= max(8u, mw / 4u))) {
        tie = true;
        tlo = base | TIE_FLAG;
        if (two) thi = base;
      } else {
        tlo = base;  // (base 0: the plain tlo == 0 bracket, tie mode at key 0 already)
        if (two && rhi >= 1.0) thi = base;
      }
    }
  }
  STAMP(P, li, 18);
  const uint32_t nu = sd.unit_end - sd.unit_begin;
  // the band histograms' upper bound (see below)
  const uint32_t hh = tie ? max(tlo & KEY_MAX, min(thi, kmax)) : max(tlo, min(thi, kmax));
  for (uint32_t i = t; i < nu; i += NT) {
    P.tlo[sd.lu_begin + i] = tlo;
    P.thi[sd.lu_begin + i] = thi;
  }
  // The band histograms of the parallel select span [T_lo, min(T_hi, max sampled key)] (keys above go
  // to the last bin): with T_hi = KEY_MAX a full-range histogram would be too coarse.
  if (t == 0) {
    P.shhi[li] = hh;
    P.status[s] = 0;
  }
  STAMP(P, li, 19);
}

template <bool DELTA, bool RAW, int NT>
__global__ __launch_bounds__(NT) void k_sample(Params P) {
  __shared__ uint32_t hist[HIST_BINS];
  __shared__ uint32_t sh[64];
  sample_segment<DELTA, NT>(P, blockIdx.x, hist, sh);
}

// k_presel: the samplers (blocks [0, n_large)) and the small segments (blocks after them) as one launch —
// both latency-bound, they run side by side ahead of k_scan, which then streams large units only (small
// segments inside k_scan held its first blocks and a 25 KB LDS arena: C2 as 2 sub-batches streamed at
// ~2.3 TB/s)
template <bool DELTA, bool RAW>
__global__ __launch_bounds__(BLOCK) void k_presel(Params P) {
  __shared__ __attribute__((aligned(16))) uint8_t arena[(SMALL_MAX + HIST_BINS + 64) * 4];
  uint32_t* hist = reinterpret_cast<uint32_t*>(arena) + SMALL_MAX;
  if (blockIdx.x < P.n_large) {
    sample_segment<DELTA>(P, blockIdx.x, hist, hist + HIST_BINS);
  } else {
    small_encode<DELTA, RAW>(P, blockIdx.x - P.n_large, reinterpret_cast<float*>(arena), hist, hist + HIST_BINS);
  }
}

// k_scan: streams the large units, one wave each. (WITH_SMALL: blocks [0, scan_small) first encode the
// small segments — no longer launched: k_presel runs them beside the samplers.)
// (WPE / NB: launch-bound blocks per CU and load batches; the latency-bound plans' instantiation, the one
// WITH_SMALL, takes its own — nothing streams beside it)
template <bool DELTA, bool RAW, bool WITH_SMALL, int WPE = SCAN_WPE, int NB = SCAN_NB, int NTS = BLOCK,
          uint32_t SCAP = SMALL_MAX>
__global__ __launch_bounds__(NTS, WPE) void k_scan(Params P) {
  // one LDS arena: candidate staging (NTS / 64 x STAGE_CAP records) or a small segment's values + histogram
  // (WITH_SMALL only: without it the block needs 16 KB of LDS instead of 24.8 KB)
  constexpr uint32_t NWS = NTS / 64;
  // (SCAP: the plan's small-segment limit, <= SMALL_MAX — 1024 by default for latency-bound plans, whose
  // arena then leaves room for a seventh block per CU)
  constexpr size_t SMALL_BYTES = WITH_SMALL ? (SCAP + HIST_BINS + 64) * 4 : 0;
  constexpr size_t STAGE_BYTES = NWS * STAGE_CAP * sizeof(uint2);
  __shared__ __attribute__((aligned(16))) uint8_t arena[SMALL_BYTES > STAGE_BYTES ? SMALL_BYTES : STAGE_BYTES];
  if (WITH_SMALL && blockIdx.x < P.scan_small) {
    float* vals = reinterpret_cast<float*>(arena);
    uint32_t* hist = reinterpret_cast<uint32_t*>(arena) + SCAP;
    small_encode<DELTA, RAW, NTS>(P, blockIdx.x, vals, hist, hist + HIST_BINS);
    return;
  }
  uint2* stage = reinterpret_cast<uint2*>(arena);
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t lu = ((!WITH_SMALL ? xcd_block(blockIdx.x) : blockIdx.x) - P.scan_small) * NWS + wv;
  if (lu >= P.n_lunits) return;
  const UnitDev L = P.lunits[lu];
  // delta: 4 load batches (32 float4 in flight spill)
  const uint32_t tlo = P.tlo[lu], thi = P.thi[lu];
  if (tlo == 0 || (tlo & TIE_FLAG)) {  // tie mode (wave-uniform: one bracket per segment)
    if (L.len == UNIT || tlo != 0)  // (K > 0: a partial unit's loads past len read key 0 < K + 1, never counted)
      scan_unit<DELTA, DELTA ? 4 : NB, false, true>(P, lu, L, tlo, thi, stage + wv * STAGE_CAP);
    else
      scan_unit<DELTA, DELTA ? 4 : NB, true, true>(P, lu, L, tlo, thi, stage + wv * STAGE_CAP);
  } else if (L.len == UNIT || tlo > 0)
    scan_unit<DELTA, DELTA ? 4 : NB, false>(P, lu, L, tlo, thi, stage + wv * STAGE_CAP);
  else
    scan_unit<DELTA, DELTA ? 4 : NB, true>(P, lu, L, tlo, thi, stage + wv * STAGE_CAP);
}

// ------------------------------------------------------------------------------------------------
// per-segment select (k_select: one SEL_NT-thread block per large segment)
// ------------------------------------------------------------------------------------------------
// Exclusive prefix of cnt[0..cn) into upre[0..cn] (upre[cn] = total). Barriers inside.
template <int NT>
DEV uint32_t chunk_prefix(const uint32_t* cnt, uint32_t cn, uint32_t cap, uint32_t* upre, uint32_t* sh) {
  const uint32_t t = threadIdx.x;
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < cn; c0 += NT) {
    const uint32_t i = c0 + t;
    const uint32_t v = i < cn ? min(cnt[i], cap) : 0u;  // stored records only
    uint32_t tot;
    const uint32_t ex = block_excl_scan<NT>(v, sh, tot);
    if (i < cn) upre[i] = carry + ex;
    carry += tot;
  }
  if (t == 0) upre[cn] = carry;
  __syncthreads();
  return carry;
}


// The records of a unit past its first two rows (n > 128: plans above ratio ~0.02), TAIL_ROWS rows of 64 per load
// round instead of one dependent round per row (C3 at ratio 0.1: a ~450-record unit took 6 rounds).
constexpr uint32_t TAIL_ROWS = 4;
// (k_emit batches its record rows the same way only in plans above HIGH_RATIO: at ratio 0.01 almost every unit's records
// fit the preloaded first row, and the batched loop measured 1.5 % slower on C3 — 0.600 vs 0.592 ms per step; C3 at
// ratio 0.1: 0.922 vs 0.982 ms with it, profiles/r05_ab.txt)
constexpr double HIGH_RATIO = 0.02;
template <class F>
DEV void tail_rows(const uint32_t* R, uint32_t n, uint32_t u, F&& f, uint32_t from = 128) {
  constexpr uint32_t TR = TAIL_ROWS;
  const uint32_t lane = lane_id();
  for (uint32_t i0 = from; i0 < n; i0 += 64 * TR) {
    uint32_t x[TR];
#pragma unroll
    for (uint32_t b = 0; b < TR; ++b)
      if (i0 + b * 64 < n) x[b] = R[min(i0 + b * 64 + lane, n - 1)];  // (wave-uniform guard)
#pragma unroll
    for (uint32_t b = 0; b < TR; ++b)
      if (i0 + b * 64 < n) f(__uint_as_float(x[b]), i0 + b * 64 + lane < n, u);
  }
}

// Wave w owns the units whose first record index (upre[u]) lies in [w*total/NW, (w+1)*total/NW):
// contiguous unit ranges balanced by record count, so segment order = (wave, unit, lane) order. A wave
// reads one unit at a time from its contiguous region (coalesced, trivial addressing, the unit is
// wave-uniform so per-unit counts are ballot popcounts), G units per batch with 2 records per lane per
// unit in flight. f(x, valid, u) is called by ALL lanes (ballots allowed); fend(u) after each unit.
// RM: record rows per unit in the batch's load round (2; 8 in batch plans above HIGH_RATIO, where a unit holds ~450
// records: all of them in that one round instead of 1 + 2 rounds per unit — C3 at ratio 0.1: 0.908-0.920 vs
// 0.925-0.927 ms; the sweeps there are bound by the HBM traffic the other sub-batch's streams leave them)
template <int NW, int G, int RM = 2, class F, class FE>
DEV void unit_sweep(const uint32_t* cand, uint32_t stride, uint32_t lu0, const uint32_t* upre, uint32_t cn,
                    uint32_t total, F&& f, FE&& fend) {
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  const uint32_t J0 = (uint32_t)((uint64_t)total * w / NW), J1 = (uint32_t)((uint64_t)total * (w + 1) / NW);
  auto lower = [&](uint32_t key) {  // first u in [0, cn] with upre[u] >= key
    uint32_t lo = 0, hi = cn;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (upre[mid] < key)
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo;
  };
  const uint32_t U0 = w == 0 ? 0u : lower(J0);
  const uint32_t U1 = w == NW - 1 ? cn : lower(J1);
  for (uint32_t u = U0; u < U1; u += G) {
    uint32_t x[G][RM], nn[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint32_t uu = min(u + g, U1 - 1);
      const uint32_t n = upre[uu + 1] - upre[uu];
      const uint32_t last = n ? n - 1 : 0u;  // region slot 0 always exists; read it when n == 0
      const uint32_t* R = cand + (uint64_t)(lu0 + uu) * stride;
      nn[g] = n;
#pragma unroll
      for (int r = 0; r < RM; ++r)
        if (r < 2 || 64u * r < n) x[g][r] = R[min(lane + 64u * r, last)];  // (rows past 2: wave-uniform guard)
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (u + g < U1) {
        const uint32_t uu = u + g, n = nn[g];
        f(__uint_as_float(x[g][0]), lane < n, uu);
#pragma unroll
        for (int r = 1; r < RM; ++r)
          if (n > 64u * r) f(__uint_as_float(x[g][r]), lane + 64u * r < n, uu);
        if (n > 64u * RM) tail_rows(cand + (uint64_t)(lu0 + uu) * stride, n, uu, f, 64u * RM);
        fend(uu);
      }
    }
  }
}

// The same prefix from counts already in registers (thread i < cn holds unit i's count, cn <= NT): the
// loads were issued with the caller's other loads of the same round.
template <int NT>
DEV uint32_t reg_prefix(uint32_t c, uint32_t cn, uint32_t* upre, uint32_t* sh) {
  const uint32_t t = threadIdx.x;
  uint32_t tot;
  const uint32_t ex = block_excl_scan<NT>(t < cn ? c : 0u, sh, tot);
  if (t < cn) upre[t] = ex;
  if (t == 0) upre[cn] = tot;
  __syncthreads();
  return tot;
}

// A group's records swept by the block's waves balanced by record count (unit_sweep): the counts and a block
// prefix come first, then the record loads — batch plans, where the select kernels run beside the other
// sub-batch's streaming waves (the speculative sweep below measured slower there: C3 0.617-0.636 vs 0.600-0.604 ms)
template <int NT, int G = GSWEEP, int RM = 2>
struct BalancedSweep {
  uint32_t* upre;
  uint32_t total, cn;
  DEV void load(const Params& P, uint32_t lu0, uint32_t units, uint32_t* upre_, uint32_t* sh) {
    upre = upre_;
    cn = units;
    const uint32_t c = threadIdx.x < units ? min(P.cntC[lu0 + threadIdx.x], P.ccap) : 0u;
    total = reg_prefix<NT>(c, units, upre, sh);  // barriers inside
  }
  template <class F, class FE>
  DEV void run(const Params& P, uint32_t lu0, F&& f, FE&& fend) const {
    unit_sweep<NT / 64, G, RM>(P.cval, P.ccap, lu0, upre, cn, total, f, fend);
  }
};

// A group's records swept by a block WITHOUT waiting for the units' counts first: wave w owns the UPW
// consecutive units [w * UPW, (w + 1) * UPW) of the group (index order = wave order) and loads their counts
// and the first two 64-record rows of every unit in ONE round, speculatively (slots past a unit's count hold
// stale words, never used; ccap >= 128). unit_sweep instead balances the waves by record count, which needs
// the counts and a block prefix before the first record load — one more dependent round on the select chain.
template <uint32_t UPW>
struct SpecSweep {
  uint32_t x0[UPW], x1[UPW], n;  // lane g < UPW: unit g's stored-record count
  uint32_t u0, cn;
  DEV void load(const Params& P, uint32_t lu0, uint32_t units, uint32_t*, uint32_t*) {
    const uint32_t lane = lane_id();
    u0 = (threadIdx.x >> 6) * UPW;
    cn = units;
    const uint32_t uc = min(u0 + min(lane, UPW - 1), units - 1);
    const uint32_t nr = P.cntC[lu0 + uc];
#pragma unroll
    for (uint32_t g = 0; g < UPW; ++g) {
      const uint32_t* R = P.cval + (uint64_t)(lu0 + min(u0 + g, units - 1)) * P.ccap;
      x0[g] = R[lane];
      x1[g] = R[lane + 64];
    }
    n = (lane < UPW && u0 + lane < units) ? min(nr, P.ccap) : 0u;
  }
  // f(x, valid, u) for every lane (ballots allowed), fend(u) after each unit; u = unit index in the group
  template <class F, class FE>
  DEV void run(const Params& P, uint32_t lu0, F&& f, FE&& fend) const {
    const uint32_t lane = lane_id();
#pragma unroll
    for (uint32_t g = 0; g < UPW; ++g) {
      const uint32_t u = u0 + g;
      if (u < cn) {
        const uint32_t nn = (uint32_t)__builtin_amdgcn_readlane((int)n, (int)g);
        f(__uint_as_float(x0[g]), lane < nn, u);
        if (nn > 64) f(__uint_as_float(x1[g]), lane + 64 < nn, u);
        if (nn > 128) tail_rows(P.cval + (uint64_t)(lu0 + u) * P.ccap, nn, u, f);
        fend(u);
      }
    }
  }
};

// LDS scratch of the segment select (k_select, and the SELECT role of the one-launch encode, whose LDS
// must stay <= 32 KB so five streaming blocks still fit a CU): 28.3 KB
constexpr uint32_t WLIST = 1024;  // in-window entries the fast path can hold
constexpr uint32_t SELECT_SPEC = 64u;  // k_select: speculatively gathered slots per group window list (one update: 64 -> 0.0811 ms per
                                       // step, 16 -> 0.0830, 8 -> 0.0838: longer lists otherwise cost a dependent round)
constexpr int SEL_HB = 1024;      // bins of the select's radix histograms
struct SelSmem {
  uint32_t hist[SEL_HB];
  uint32_t upre[UCAP + 1];
  uint32_t ge[UCAP];   // per unit of the chunk: count above T* (bits 0-15) | count equal T* (bits 16-31)
  uint2 lst[WLIST];    // in-window entries {value bits, unit}, all waves concatenated = index order
  uint32_t wcnt[SEL_NT_LAT / 64];
  uint32_t sh[64];
  float shf[2 * (SEL_NT_LAT / 64)];
};
static_assert(sizeof(SelSmem) <= 29 * 1024, "select LDS budget");

// Generic path: radix select over all candidates (1-3 coalesced sweeps) + a counts sweep; handles any
// number of ties and segments of any size (units in chunks of UCAP).
template <int NT>
DEV void select_generic(const Params& P, uint32_t lb, uint32_t nu, uint32_t tlo, uint32_t thi, uint32_t r,
                        SelSmem& S, uint32_t& T_out, uint32_t& rt_out, uint32_t& fp, uint32_t& fn, float& gmn,
                        float& gmx) {
  constexpr int NW = NT / 64;
  const uint32_t t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  uint32_t rt = r;
  auto forC = [&](auto&& f) {
    for (uint32_t c0 = 0; c0 < nu; c0 += UCAP) {
      const uint32_t cn = min(UCAP, nu - c0);
      const uint32_t total = chunk_prefix<NT>(P.cntC + lb + c0, cn, P.ccap, S.upre, S.sh);
      unit_sweep<NW, 4>(
          P.cval, P.ccap, lb + c0, S.upre, cn, total,
          [&](float x, bool valid, uint32_t) {
            if (valid) f(fkey(x));
          },
          [&](uint32_t) {});
      __syncthreads();
    }
  };
  const uint32_t T = rt == 0 ? thi : block_select<NT, SEL_HB>(forC, tlo, thi, rt, S.hist, S.sh);

  // counts sweep: per-unit gt/eq, segment-wide tie rank of the first positive / negative tie, min/max
  // of the values with key > T (all of them are kept).
  float lmn = qnan(), lmx = qnan();
  uint32_t carry_eq = 0;
  if (t == 0) {
    S.sh[42] = NONE;
    S.sh[43] = NONE;
  }
  for (uint32_t c0 = 0; c0 < nu; c0 += UCAP) {
    const uint32_t cn = min(UCAP, nu - c0);
    for (uint32_t i = t; i < cn; i += NT) S.ge[i] = 0;
    const uint32_t total = chunk_prefix<NT>(P.cntC + lb + c0, cn, P.ccap, S.upre, S.sh);
    uint32_t weq = 0, wfp = NONE, wfn = NONE, ug = 0, ue = 0;  // wave-uniform
    unit_sweep<NW, 4>(
        P.cval, P.ccap, lb + c0, S.upre, cn, total,
        [&](float x, bool valid, uint32_t) {
          const uint32_t key = fkey(x);
          const bool g = valid && key > T;
          const bool e = valid && key == T;
          ug += (uint32_t)__popcll(__ballot(g));
          const float xg = g ? x : qnan();
          lmn = fmin_nan(lmn, xg);
          lmx = fmax_nan(lmx, xg);
          const uint64_t eb = __ballot(e);
          if (eb) {
            const bool neg = (__float_as_uint(x) >> 31) != 0;
            const uint64_t pm = __ballot(e && !neg), nm = __ballot(e && neg);
            if (wfp == NONE && pm) wfp = weq + (uint32_t)__popcll(eb & ((1ull << (__ffsll((long long)pm) - 1)) - 1ull));
            if (wfn == NONE && nm) wfn = weq + (uint32_t)__popcll(eb & ((1ull << (__ffsll((long long)nm) - 1)) - 1ull));
            weq += (uint32_t)__popcll(eb);
            ue += (uint32_t)__popcll(eb);
          }
        },
        [&](uint32_t u) {
          if (lane == 0) S.ge[u] = ug | (ue << 16);
          ug = ue = 0;
        });
    if (lane == 0) S.wcnt[wv] = weq;
    __syncthreads();
    uint32_t wpre = carry_eq, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const uint32_t c = S.wcnt[i];
      if ((uint32_t)i < wv) wpre += c;
      tot += c;
    }
    if (lane == 0 && wfp != NONE) atomicMin(&S.sh[42], wpre + wfp);
    if (lane == 0 && wfn != NONE) atomicMin(&S.sh[43], wpre + wfn);
    carry_eq += tot;
    __syncthreads();
    for (uint32_t i = t; i < cn; i += NT) {
      P.gtC[lb + c0 + i] = S.ge[i] & 0xFFFFu;
      P.eqC[lb + c0 + i] = S.ge[i] >> 16;
    }
    __syncthreads();
  }
  T_out = T;
  rt_out = rt;
  fp = S.sh[42];
  fn = S.sh[43];
  gmn = lmn;
  gmx = lmx;
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// parallel select, fast path: groups of GU units of one large segment, one 256-thread block each
// ------------------------------------------------------------------------------------------------
// k_ghist: the group's HB2-bin histogram of the band keys [tlo, thi] -> ghist[group]. (A fused variant in
// which the segment's last-arriving group block ran segment_pick needed an agent-scope release fence in
// every block — an L2 writeback on gfx950 — and was ~100x slower; kernel boundaries are cheaper.)
template <int NT, bool SPEC, bool HR = false>
using GroupSweep = std::conditional_t<SPEC, SpecSweep<(GU + NT / 64 - 1) / (NT / 64)>,
                                      std::conditional_t<HR, BalancedSweep<NT, 2, 8>, BalancedSweep<NT>>>;

template <int NT, bool SPEC, bool HR>
DEV void group_hist(const Params& P, uint32_t gi, uint32_t* hist, uint32_t* upre, uint32_t* sh) {
  const uint4 G = P.groups[gi];  // x: large-segment index, y: first large unit, z: units, w: segment
  const uint32_t t = threadIdx.x;
  STAMP(P, G.x, 20);
  // one load round for everything that depends on G only: the band, and every unit's count and first
  // records (the histogram needs no index order, so no count prefix before the record loads)
  const uint32_t tlo = P.tlo[G.y] & KEY_MAX, thi = P.thi[G.y], hh = P.shhi[G.x];  // (tie mode K: band [K, K], empty)
  GroupSweep<NT, SPEC, HR> sw;
  for (uint32_t i = t; i < HB2; i += NT) hist[i] = 0;
  sw.load(P, G.y, G.z, upre, sh);
  __syncthreads();
  const Band band(tlo, thi, hh);
  sw.run(
      P, G.y,
      [&](float x, bool valid, uint32_t) {
        const uint32_t key = fkey(x);
        if (valid && key >= tlo && key <= thi) atomicAdd(&hist[band.bin(key)], 1u);
      },
      [&](uint32_t) {});
  __syncthreads();
  for (uint32_t i = t; i < HB2; i += NT) pst(P, P.ghist + (uint64_t)gi * HB2 + i, hist[i]);
  STAMP(P, G.x, 21);
}

// NT: 256 threads in batches, GHIST_NT_LAT in latency-bound plans (nothing streams beside the block); SPEC: the
// speculative group sweep (latency-bound plans)
template <int NT, bool SPEC, bool HR = false>  // HR: batch plans above HIGH_RATIO (8 record rows per unit per round)
__global__ __launch_bounds__(NT) void k_ghist(Params P) {
  __shared__ uint32_t hist[HB2];
  __shared__ uint32_t upre[GU + 1];
  __shared__ uint32_t sh[64];
  group_hist<NT, SPEC, HR>(P, blockIdx.x, hist, upre, sh);
}

// segment_pick: per large segment — validate the sampled bracket, sum the group histograms, pick the bin of
// the k-th key: {window lo, window hi, rank inside the window, 0}; {.., 1} routes the segment to the
// generic single-block path (bracket miss, nothing to take from B, huge segment, test flags). Every group
// block of the segment computes it (identically) at the start of k_gwin — cheaper than a launch of its
// own between k_ghist and k_gwin. Returned to every thread.
template <int NT = BLOCK>
DEV uint4 segment_pick(const Params& P, const SegDev& sd, const Band& band, bool tieseg, uint32_t* hist, uint32_t* sh) {
  const uint32_t t = threadIdx.x;
  const uint32_t lb = sd.lu_begin, nu = sd.unit_end - sd.unit_begin, k = sd.k;
  const uint32_t g0 = sd.g_begin, ng = (nu + GU - 1) / GU;
  // one load round: the group histograms (this thread's bins t and t + NT, up to 24 groups' loads in
  // flight) and the per-unit counts (up to 3 per thread) together
  static_assert(HB2 == 2 * NT || HB2 == NT, "one or two histogram bins per thread");
  constexpr bool TWO = HB2 == 2 * NT;
  constexpr uint32_t GB = 24, CB = 3;
  const bool zseg = tieseg;  // the scan counted this segment's keys equal to its tie key (cntZ; tie mode)
  uint32_t h0 = 0, h1 = 0, sa = 0, sc = 0, ov = 0, sz = 0;
  {
    uint32_t v0[GB], v1[GB], ca[CB], cc[CB], cz[CB];
#pragma unroll
    for (uint32_t j = 0; j < GB; ++j) {
      const uint64_t row = (uint64_t)(g0 + min(j, ng - 1)) * HB2;
      v0[j] = P.ghist[row + t];
      v1[j] = TWO ? P.ghist[row + NT + t] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < CB; ++j) {
      const uint32_t i = min(t + j * NT, nu - 1);
      cc[j] = P.cntC[lb + i];
      ca[j] = P.cntA[lb + i];
      cz[j] = P.cntZ[lb + i];  // (unconditional; used for a zero-bracket segment only)
    }
#pragma unroll
    for (uint32_t j = 0; j < GB; ++j) {
      h0 += j < ng ? v0[j] : 0u;
      h1 += j < ng ? v1[j] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < CB; ++j) {
      if (t + j * NT < nu) {
        sa += ca[j];
        sc += cc[j];
        sz += zseg ? cz[j] : 0u;
        ov += cc[j] > P.ccap ? 1u : 0u;
      }
    }
  }
  for (uint32_t g = GB; g < ng; g += 8) {  // segments of more than GB groups
    uint32_t v0[8], v1[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint64_t row = (uint64_t)(g0 + min(g + j, ng - 1)) * HB2;
      v0[j] = P.ghist[row + t];
      v1[j] = TWO ? P.ghist[row + NT + t] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      h0 += g + j < ng ? v0[j] : 0u;
      h1 += g + j < ng ? v1[j] : 0u;
    }
  }
  for (uint32_t i = t + CB * NT; i < nu; i += NT) {
    const uint32_t c = P.cntC[lb + i];
    sa += P.cntA[lb + i];
    sc += c;
    sz += zseg ? P.cntZ[lb + i] : 0u;
    ov += c > P.ccap ? 1u : 0u;
  }
  hist[t] = h0;
  if (TWO) hist[NT + t] = h1;
  sa = block_sum<NT>(sa, sh);  // barriers inside (also publish hist)
  sc = block_sum<NT>(sc, sh);
  ov = block_sum<NT>(ov, sh);
  if (zseg) sz = block_sum<NT>(sz, sh);
  // (a unit that overflowed its record slots sends the segment to the raw-data path in segment_select)
  const bool forced = (P.flags & (COALAC_FLAG_FORCE_EXACT | COALAC_FLAG_GENERIC_SELECT)) || nu > UCAP || ov != 0;
  // the k-th key is the tie key K: every recorded key (all above K) is kept, and the first k - sc K-keys by index. The
  // window [1, 0] is empty: k_gwin counts every record as above it (per-unit kept counts) and takes their min / max
  if (!forced && zseg && sc < k && k - sc <= sz) return make_uint4(1u, 0u, k - sc, 2u);
  const bool generic = forced || !(sa < k && k <= sc);
  if (generic) return make_uint4(0u, 0u, 0u, 1u);
  __syncthreads();
  uint32_t r = k - sa;
  const uint32_t b = hist_pick<NT, HB2>(hist, r, sh);
  if (b == NONE) return make_uint4(0u, 0u, 0u, 1u);
  return make_uint4(band.wlo(b), band.whi(b), r, 0u);
}

// k_gwin: per group — per-unit counts of keys above the window (-> gtC), the group's in-window entries
// in index order (-> glist, count -> gcnt), min/max of the values above the window (-> gmm)
template <int NW = WAVES>
struct GwinSmemT {
  uint32_t upre[GU + 1];
  uint2 slots[NW][GCAP];
  uint32_t wcnt[NW];
  float shf[2 * NW];
};
using GwinSmem = GwinSmemT<WAVES>;

template <int NT, bool DELTA, bool RAW>
DEV void segment_select(const Params& P, uint32_t li, SelSmem& S);

// (sw: the group's counts and first records, loaded by the caller with its other loads)
template <int NT, class SW>
DEV void group_window(const Params& P, uint32_t gi, const uint4 G, const uint4 st, uint32_t lu_begin, const SW& sw,
                      GwinSmemT<NT / 64>& W_, uint32_t* sh) {
  constexpr int NW = NT / 64;
  auto& slots = W_.slots;
  uint32_t* wcnt = W_.wcnt;
  float* shf = W_.shf;
  const uint32_t t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  const uint32_t wlo = st.x, whi = st.y;
  const uint32_t useg0 = G.y - lu_begin;  // unit index (within the segment) of the group's first unit
  uint32_t wc = 0, ug = 0;
  float lmn = qnan(), lmx = qnan();
  sw.run(
      P, G.y,
      [&](float x, bool valid, uint32_t u) {
        const uint32_t key = fkey(x);
        const bool g = valid && key > whi;
        const bool in = valid && key >= wlo && key <= whi;
        ug += (uint32_t)__popcll(__ballot(g));
        const float xg = g ? x : qnan();
        lmn = fmin_nan(lmn, xg);
        lmx = fmax_nan(lmx, xg);
        const uint64_t im = __ballot(in);
        if (im) {
          const uint32_t pos = wc + mbcnt(im);
          if (in && pos < GCAP) slots[wv][pos] = make_uint2(__float_as_uint(x), useg0 + u);
          wc += (uint32_t)__popcll(im);
        }
      },
      [&](uint32_t u) {
        if (lane == 0) {
          pst(P, P.gtC + G.y + u, ug);
          pst(P, P.eqC + G.y + u, 0u);
        }
        ug = 0;
      });
  if (lane == 0) wcnt[wv] = wc;
  __syncthreads();
  uint32_t wpre = 0, W = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t c = wcnt[i];
    if (i < (int)wv) wpre += c;
    W += c;
  }
  for (uint32_t q = lane; q < wc && q < GCAP; q += 64)
    if (wpre + q < GCAP) pst(P, P.glist + (uint64_t)gi * GCAP + wpre + q, slots[wv][q]);
  block_minmax<NT>(lmn, lmx, shf);
  if (t == 0) {
    pst(P, P.gcnt + gi, W);
    pst(P, P.gmm + 2 * gi, lmn);
    pst(P, P.gmm + 2 * gi + 1, lmx);
  }
}

template <int NT, bool SPEC, bool HR>
DEV void group_pick_window(const Params& P, uint32_t gi, GwinSmemT<NT / 64>& W, uint32_t* hist, uint32_t* sh) {
  // round 1: the group and its segment's geometry (gseg: {first large unit, units, k, first group}, so nothing
  // waits for a segment-table lookup); round 2: the band, the group's unit counts and first records
  // (SpecSweep), the segment's group histograms and unit counts — everything the block reads, in one round
  const uint4 G = P.groups[gi];
  const uint4 GS = P.gseg[gi];
  STAMP(P, G.x, 22);
  SegDev sd{};
  sd.lu_begin = GS.x;
  sd.unit_end = GS.y;
  sd.k = GS.z;
  sd.g_begin = GS.w;
  const uint32_t tlo = P.tlo[G.y], thi = P.thi[G.y], hh = P.shhi[G.x];
  GroupSweep<NT, SPEC, HR> sw;
  sw.load(P, G.y, G.z, W.upre, sh);
  const uint4 st = segment_pick<NT>(P, sd, Band(tlo & KEY_MAX, thi, hh), tlo == 0 || (tlo & TIE_FLAG), hist, sh);
  STAMP(P, G.x, 23);
  if (st.w == 0 || st.w == 2) group_window<NT>(P, gi, G, st, GS.x, sw, W, sh);
  if (threadIdx.x == 0 && G.y == GS.x) {  // the segment's first group
    uint2* ss = reinterpret_cast<uint2*>(P.sstate + G.x);
    pst(P, ss, make_uint2(st.x, st.y));
    pst(P, ss + 1, make_uint2(st.z, st.w));
  }
  STAMP(P, G.x, 24);
}

// NT: 256 threads in batches, GWIN_NT_LAT in latency-bound plans (nothing streams beside the block)
template <int NT, bool SPEC, bool HR = false>  // HR: as k_ghist
__global__ __launch_bounds__(NT) void k_gwin(Params P) {
  __shared__ GwinSmemT<NT / 64> W;
  __shared__ uint32_t hist[HB2];
  __shared__ uint32_t sh[64];
  group_pick_window<NT, SPEC, HR>(P, blockIdx.x, W, hist, sh);
}

// ------------------------------------------------------------------------------------------------
// raw-data path of a segment (bracket miss, COALAC_FLAG_FORCE_EXACT, or a unit with more candidates than
// its ccap record slots): T* from the raw keys (segment_select), per-unit counts from the raw data here,
// and the emit re-reads the raw data (emit_raw_unit). No candidate record is used.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t RAW_NB = 2u;  // load rounds per unit of a raw-data pass (round 5: 4 rounds of 4 float4 per lane)
// One wave's pass over a unit's raw data (row by row, index order): per element whether key > T and
// whether key == T, handed to f(row, j, x, gt, tie) for every lane (ballots allowed inside f).
template <bool DELTA, class F>
DEV void raw_unit_rows(const Params& P, const UnitDev& L, F&& f) {
  const uint32_t lane = lane_id();
  const float* xin = P.inptr != nullptr ? P.inptr[L.seg] + L.start : P.in + L.off;
  const __amdgpu_buffer_rsrc_t rin = unit_rsrc(xin, L.len);
  const __amdgpu_buffer_rsrc_t rbase = unit_rsrc(DELTA ? P.base + L.off : xin, L.len);
  for (uint32_t nb = 0; nb < RAW_NB; ++nb) {  // UNIT_IT / RAW_NB float4 per lane in flight
    constexpr uint32_t IT = UNIT_IT / RAW_NB;
    float4 v[IT];
#pragma unroll
    for (uint32_t i = 0; i < IT; ++i) v[i] = unit_load_x4<DELTA>(rin, rbase, ((nb * IT + i) * 64 + lane) * 16);
#pragma unroll
    for (uint32_t i = 0; i < IT; ++i) f(nb * IT + i, v[i]);
  }
}

// Per-unit counts above / equal to T of the raw segment -> gtC / eqC; min / max of the values above T; the
// segment-wide tie rank of the first positive and first negative tie (index order). Waves own contiguous
// unit ranges in order. Block-level: call from all threads.
template <int NT, bool DELTA>
DEV void raw_counts(const Params& P, uint32_t lb, uint32_t nu, uint32_t T, uint32_t* sh, uint32_t* wcnt,
                    uint32_t& fp, uint32_t& fn, float& gmn, float& gmx, uint32_t* ge) {
  constexpr int NW = NT / 64;
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint32_t u0 = (uint32_t)((uint64_t)nu * wv / NW), u1 = (uint32_t)((uint64_t)nu * (wv + 1) / NW);
  uint32_t weq = 0, wfp = NONE, wfn = NONE;
  float lmn = qnan(), lmx = qnan();
  for (uint32_t u = u0; u < u1; ++u) {
    const UnitDev L = P.lunits[lb + u];
    uint32_t ug = 0, ue = 0;
    raw_unit_rows<DELTA>(P, L, [&](uint32_t row, float4 v) {
      const float xs[4] = {v.x, v.y, v.z, v.w};
      const uint32_t e0 = (row * 64 + lane) * 4;
      uint32_t pre = 0, mine = 0;
      uint64_t tb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t key = fkey(xs[j]);
        const bool ok = e0 + j < L.len;
        const bool g = ok && key > T, e = ok && key == T;
        ug += (uint32_t)__popcll(__ballot(g));
        tb[j] = __ballot(e);
        pre += mbcnt(tb[j]);
        const float xg = g ? xs[j] : qnan();
        lmn = fmin_nan(lmn, xg);
        lmx = fmax_nan(lmx, xg);
      }
      // index order inside a row is (lane, j): a tie's rank = ties of lower lanes + earlier ties of its lane
      uint32_t rp = NONE, rn = NONE;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool e = ((tb[j] >> lane) & 1ull) != 0;
        if (e) {
          const bool neg = (__float_as_uint(xs[j]) >> 31) != 0;
          const uint32_t rank = weq + pre + mine;
          if (neg)
            rn = min(rn, rank);
          else
            rp = min(rp, rank);
          ++mine;
        }
      }
      wfp = min(wfp, wave_min_u32(rp));
      wfn = min(wfn, wave_min_u32(rn));
      const uint32_t rowt = (uint32_t)(__popcll(tb[0]) + __popcll(tb[1]) + __popcll(tb[2]) + __popcll(tb[3]));
      weq += rowt;
      ue += rowt;
    });
    if (lane == 0) {
      pst(P, P.gtC + lb + u, ug);
      pst(P, P.eqC + lb + u, ue);
      if (u < UCAP) ge[u] = ug | (ue << 16);  // (select_finish reads LDS: other threads own the unit there)
    }
  }
  // wave prefixes of the tie counts -> segment-wide ranks of the first positive / negative tie
  if (lane == 0) wcnt[wv] = weq;
  if (threadIdx.x == 0) {
    sh[42] = NONE;
    sh[43] = NONE;
  }
  __syncthreads();
  uint32_t wpre = 0;
  for (int i = 0; i < (int)wv; ++i) wpre += wcnt[i];
  if (lane == 0 && wfp != NONE) atomicMin(&sh[42], wpre + wfp);
  if (lane == 0 && wfn != NONE) atomicMin(&sh[43], wpre + wfn);
  __syncthreads();
  fp = sh[42];
  fn = sh[43];
  gmn = lmn;
  gmx = lmx;
  __syncthreads();
}

template <int NT>
DEV void window_resolve(SelSmem& S, uint32_t W, uint4 st, float lmn0, float lmx0, uint32_t& T_out, uint32_t& rt_out,
                        uint32_t& fp, uint32_t& fn, float& gmn, float& gmx);

// Fast-path resolution in k_select: gather the groups' in-window lists (group order = index order),
// find the exact key inside the window, apply the window entries to the per-unit counts. Returns false
// if a group's list overflowed (the caller then runs the generic path from scratch).
template <int NT>
DEV bool select_from_groups(const Params& P, const SegDev& sd, uint32_t lb, uint32_t nu, uint4 st, SelSmem& S,
                            uint32_t& T_out, uint32_t& rt_out, uint32_t& fp, uint32_t& fn, float& gmn, float& gmx) {
  const uint32_t t = threadIdx.x;
  const uint32_t g0 = sd.g_begin, ng = (nu + GU - 1) / GU;  // ng <= UCAP / GU = 64 <= NT
  // one load round: the groups' list lengths, min / max above the window, the first per-unit counts, and —
  // speculatively, before their lengths are known — the first SPEC slots of every group's in-window list (the
  // typical window share of a group fits; a longer list's remainder is loaded after the scan)
  constexpr uint32_t SPEC = SELECT_SPEC, SPT = (UCAP / GU) * SPEC / NT;
  static_assert((UCAP / GU) * SPEC % NT == 0, "speculative gather geometry");
  uint2 sv[SPT];
#pragma unroll
  for (uint32_t j = 0; j < SPT; ++j) {
    const uint32_t i = t + j * NT, g = i / SPEC;
    sv[j] = g < ng ? P.glist[(uint64_t)(g0 + g) * GCAP + i % SPEC] : make_uint2(0u, 0u);
  }
  const uint32_t c = t < ng ? P.gcnt[g0 + t] : 0u;
  const float gmn0 = t < ng ? P.gmm[2 * (g0 + t)] : qnan(), gmx0 = t < ng ? P.gmm[2 * (g0 + t) + 1] : qnan();
  constexpr uint32_t CB = 3;
  uint32_t gtc[CB];
#pragma unroll
  for (uint32_t j = 0; j < CB; ++j) gtc[j] = P.gtC[lb + min(t + j * NT, nu - 1)];
  uint32_t W;
  const uint32_t gpre = block_excl_scan<NT>(c, S.sh, W);
  const uint32_t over = block_sum<NT>(c > GCAP ? 1u : 0u, S.sh);
  if (over || W > WLIST) return false;
  // each group's entries go to its offset in the segment's list (group order = index order)
  if (t < ng) S.upre[t] = gpre;
  if (t == 0) S.upre[ng] = W;
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < SPT; ++j) {
    const uint32_t i = t + j * NT, g = i / SPEC, slot = i % SPEC;
    if (g < ng && S.upre[g] + slot < S.upre[g + 1]) S.lst[S.upre[g] + slot] = sv[j];
  }
  for (uint32_t g = 0; g < ng; ++g) {  // (wave-uniform) lists longer than SPEC: the rest
    const uint32_t a = S.upre[g], n = S.upre[g + 1] - a;
    for (uint32_t slot = SPEC + t; slot < n; slot += NT) S.lst[a + slot] = P.glist[(uint64_t)(g0 + g) * GCAP + slot];
  }
#pragma unroll
  for (uint32_t j = 0; j < CB; ++j)
    if (t + j * NT < nu) S.ge[t + j * NT] = gtc[j];
  for (uint32_t i = t + CB * NT; i < nu; i += NT) S.ge[i] = P.gtC[lb + i];
  __syncthreads();
  window_resolve<NT>(S, W, st, gmn0, gmx0, T_out, rt_out, fp, fn, gmn, gmx);
  return true;
}

// The exact k-th key inside the window [st.x, st.y] from the segment's in-window list S.lst[0, W) (index order), rank
// st.z inside the window; the entries above it and its ties applied to the per-unit counts in S.ge (above | equal << 16);
// the segment-wide tie ranks of the first positive / negative tie; min / max of the kept window entries folded into
// this thread's lmn / lmx (the values above the window). Block-level.
template <int NT>
DEV void window_resolve(SelSmem& S, uint32_t W, uint4 st, float lmn0, float lmx0, uint32_t& T_out, uint32_t& rt_out,
                        uint32_t& fp, uint32_t& fn, float& gmn, float& gmx) {
  const uint32_t t = threadIdx.x;
  uint32_t rt = st.z;
  const uint32_t T = block_select<NT, SEL_HB>(
      [&](auto&& f) {
        for (uint32_t i = t; i < W; i += NT) f(S.lst[i].x & KEY_MAX);
      },
      st.x, st.y, rt, S.hist, S.sh);
  constexpr uint32_t EPT = WLIST / NT;
  const uint32_t q0 = min(W, t * EPT), q1 = min(W, q0 + EPT);
  float lmn = qnan(), lmx = qnan();
  uint32_t leq = 0, lfp = NONE, lfn = NONE;
  for (uint32_t q = q0; q < q1; ++q) {
    const uint32_t vb = S.lst[q].x;
    const uint32_t key = vb & KEY_MAX;
    if (key > T) {
      atomicAdd(&S.ge[S.lst[q].y], 1u);
      lmn = fmin_nan(lmn, __uint_as_float(vb));
      lmx = fmax_nan(lmx, __uint_as_float(vb));
    } else if (key == T) {
      atomicAdd(&S.ge[S.lst[q].y], 1u << 16);
      const bool neg = (vb >> 31) != 0;
      lfp = min(lfp, neg ? NONE : leq);
      lfn = min(lfn, neg ? leq : NONE);
      ++leq;
    }
  }
  lmn = fmin_nan(lmn, lmn0);  // (select_from_groups: thread t < ng holds group t's)
  lmx = fmax_nan(lmx, lmx0);
  uint32_t teq;
  const uint32_t ex = block_excl_scan<NT>(leq, S.sh, teq);
  if (t == 0) {
    S.sh[42] = NONE;
    S.sh[43] = NONE;
  }
  __syncthreads();
  if (lfp != NONE) atomicMin(&S.sh[42], ex + lfp);
  if (lfn != NONE) atomicMin(&S.sh[43], ex + lfn);
  __syncthreads();
  T_out = T;  // per-unit counts stay in S.ge for the caller's in-order scan
  rt_out = rt;
  fp = S.sh[42];
  fn = S.sh[43];
  gmn = lmn;
  gmx = lmx;
  __syncthreads();
}

// Zero-tie ranks (tie mode, the k-th key is the segment's tie key K > 0): the segment-wide ranks of the first +K and
// -K ties, from the units' tie prefixes (S.ge >> 16 = the unit's K-keys) and in-unit ranks (tsgn). Block-level.
template <int NT>
DEV void zero_tie_ranks(const Params& P, uint32_t lb, uint32_t nu, SelSmem& S, uint32_t& fp_rank, uint32_t& fn_rank) {
  const uint32_t t = threadIdx.x;
  uint32_t lp = NONE, ln = NONE, carry = 0;
  for (uint32_t c0 = 0; c0 < nu; c0 += NT) {
    const uint32_t i = c0 + t;
    const uint32_t z = i < nu ? S.ge[i] >> 16 : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<NT>(z, S.sh, tot) + carry;
    carry += tot;
    if (i < nu) {
      const uint32_t sg = P.tsgn[lb + i], fp = sg & 0xFFFFu, fn = sg >> 16;
      if (fp != 0xFFFFu) lp = min(lp, ex + fp);
      if (fn != 0xFFFFu) ln = min(ln, ex + fn);
    }
  }
  if (t == 0) {
    S.sh[42] = NONE;
    S.sh[43] = NONE;
  }
  __syncthreads();
  if (lp != NONE) atomicMin(&S.sh[42], lp);
  if (ln != NONE) atomicMin(&S.sh[43], ln);
  __syncthreads();
  fp_rank = S.sh[42];
  fn_rank = S.sh[43];
  __syncthreads();
}

// The select of a segment that the window path cannot resolve: the generic multi-pass select over the records, or —
// on a bracket miss, a unit that overflowed its record slots, or COALAC_FLAG_FORCE_EXACT — the raw-data path (exact
// k-th key of the whole segment from its input, per-unit counts from the raw data, status 1: k_emit re-reads the input).
// Per-unit counts land in gtC / eqC. Block-level.
template <int NT, bool DELTA>
DEV void select_fallback(const Params& P, uint32_t s, const SegDev& sd, SelSmem& S, uint32_t& T, uint32_t& rt,
                         uint32_t& fp_rank, uint32_t& fn_rank, float& gmn, float& gmx, uint32_t& raw_path) {
  constexpr int NW = NT / 64;
  const uint32_t t = threadIdx.x, wv = t >> 6;
  const float* xs = seg_in(P, s, sd.in_off);
  const float* bs = DELTA ? P.base + sd.in_off : xs;
  const uint32_t lb = sd.lu_begin, nu = sd.unit_end - sd.unit_begin, k = sd.k;
  uint32_t sa = 0, sc = 0;
  for (uint32_t i = t; i < nu; i += NT) {
    sa += P.cntA[lb + i];
    sc += P.cntC[lb + i];
  }
  sa = block_sum<NT>(sa, S.sh);
  sc = block_sum<NT>(sc, S.sh);
  uint32_t mc = 0;  // most candidates any unit found (> ccap: records were dropped)
  for (uint32_t i = t; i < nu; i += NT) mc = max(mc, P.cntC[lb + i]);
  mc = wave_max_u32(mc);
  if (lane_id() == 0) S.wcnt[wv] = mc;
  __syncthreads();
  for (int i = 0; i < NW; ++i) mc = max(mc, S.wcnt[i]);
  __syncthreads();
  const uint32_t tlo = P.tlo[lb] & KEY_MAX, thi = P.thi[lb];  // (tie mode K: records are the keys above K)
  raw_path = 0u;
  if ((P.flags & COALAC_FLAG_FORCE_EXACT) || !(sa <= k && k <= sc) || mc > P.ccap) {
    // raw-data path (rare): the exact k-th key of the whole segment, per-unit counts from the raw data;
    // k_emit re-reads the raw data for this segment (status 1)
    const uint32_t n = sd.n;
    uint32_t rk = k;
    T = block_select<NT, SEL_HB>(
        [&](auto&& f) {
          for (uint32_t i = t; i < n; i += NT) f(fkey(load_x1p<DELTA>(xs + i, bs + i)));
        },
        0u, KEY_MAX, rk, S.hist, S.sh);
    rt = rk;
    raw_counts<NT, DELTA>(P, lb, nu, T, S.sh, S.wcnt, fp_rank, fn_rank, gmn, gmx, S.ge);
    raw_path = 1u;
    if (t == 0) pst(P, P.status + s, 1u);
  } else {
    // rank of the k-th key among candidates with key <= thi (0: none of them)
    select_generic<NT>(P, lb, nu, tlo, thi, k - sa, S, T, rt, fp_rank, fn_rank, gmn, gmx);
  }
}

// The end of every segment select: mn / scale from the kept values' min / max (+ the kept ties' ±T), the segment's
// T*, tie budget, mn, scale, and the in-order scan over its units — global tie prefix, output offsets (= the wire-v2
// starts), each unit's emit parameters (k_emit loads them with the unit's own words, in one round): {T*, tie budget |
// raw-data emit << 31, mn, scale} — raw-data emit for every unit of a raw-path segment, and for the units of a
// zero-tie segment whose K-keys the quota reaches. done: the per-unit counts are in S.ge (above | equal << 16), else
// in gtC / eqC. Block-level.
template <int NT, bool RAW>
DEV void select_finish(const Params& P, uint32_t s, const SegDev& sd, SelSmem& S, bool done, bool zero_tie,
                       uint32_t raw_path, uint32_t T, uint32_t rt, uint32_t fp_rank, uint32_t fn_rank, float gmn,
                       float gmx) {
  const uint32_t t = threadIdx.x;
  const uint32_t lb = sd.lu_begin, nu = sd.unit_end - sd.unit_begin;
  float mn = 0.0f, scale = 0.0f;
  if (!RAW) {
    const float tv = __uint_as_float(T);
    if (t == 0 && fp_rank < rt) {
      gmn = fmin_nan(gmn, tv);
      gmx = fmax_nan(gmx, tv);
    }
    if (t == 0 && fn_rank < rt) {
      gmn = fmin_nan(gmn, -tv);
      gmx = fmax_nan(gmx, -tv);
    }
    block_minmax<NT>(gmn, gmx, S.shf);
    gmn = gmn + 0.0f;
    gmx = gmx + 0.0f;
    mn = gmn;
    scale = (gmx == gmn) ? 0.0f : (gmx - gmn) / P.levels;
  }
  if (t == 0) {
    pst(P, P.tstar + s, T);
    pst(P, P.rtie + s, rt);
    pst(P, P.mn + s, mn);
    pst(P, P.scale + s, scale);
  }
  // thread t takes unit c0 + t of each NT-unit chunk (coalesced loads and stores): ONE paired block scan of the tie and
  // above-T* counts per chunk — the quotas of the units before u sum to min(rt, ties before u), so u's output offset is
  // its above-T* prefix + that. The counts are in LDS (S.ge) whenever nu <= UCAP (every path leaves them there); a
  // segment of more units (the generic path, chunk by chunk) reads gtC / eqC with L1-bypassing loads — this block
  // wrote them, and a plain load may hit a line this CU's L1 cached before (cdna_hip_programming.md §6 G16)
  const bool lds = done || nu <= UCAP;
  uint32_t carry_e = 0, carry_g = 0;
  for (uint32_t c0 = 0; c0 < nu; c0 += NT) {  // (block_excl_scan2 opens with a barrier: S.sh free again)
    const uint32_t i = c0 + t;
    const bool valid = i < nu;
    uint32_t e = 0, g = 0;
    if (valid) {
      if (lds) {
        const uint32_t v = S.ge[i];
        e = v >> 16;
        g = v & 0xFFFFu;
      } else {
        e = __builtin_nontemporal_load(P.eqC + lb + i);
        g = __builtin_nontemporal_load(P.gtC + lb + i);
      }
    }
    uint32_t ex, gx, te, tg;
    block_excl_scan2<NT>(e, g, S.sh, ex, gx, te, tg);
    ex += carry_e;
    gx += carry_g;
    carry_e += te;
    carry_g += tg;
    const uint32_t qp = umin_opaque(rt, ex);  // ties kept before unit i (see umin_opaque)
    const uint32_t quota = min(e, rt - qp);
    const uint32_t so = gx + qp;
    if (valid) {
      pst(P, P.eqpre + lb + i, ex);
      pst(P, P.outoff + lb + i, so);
      if (P.ustart_out != nullptr) pst(P, P.ustart_out + sd.unit_begin + i, so);  // wire v2: the unit's start
      const uint32_t rawu = raw_path | (zero_tie && quota > 0 ? 1u : 0u);
      P.uemit[lb + i] = make_uint4(T, rt | (rawu << 31), __float_as_uint(mn), __float_as_uint(scale));
    }
  }
}

template <int NT, bool DELTA, bool RAW>
DEV void segment_select(const Params& P, uint32_t li, SelSmem& S) {
  const uint32_t t = threadIdx.x;
  const uint32_t s = P.large_list[li];
  const SegDev sd = P.lsegs[li];  // (same load round as s and the select state)
  const uint4 st = P.sstate[li];
  const uint32_t lb = sd.lu_begin, nu = sd.unit_end - sd.unit_begin;
  STAMP(P, li, 0);
  uint32_t T = 0, rt = 0, fp_rank = NONE, fn_rank = NONE;
  float gmn = qnan(), gmx = qnan();
  const bool zero_tie = st.w == 2;  // the k-th key is the segment's tie key K (segment_pick; tie mode)
  bool done;
  if (zero_tie) {
    // every record kept (k_gwin's per-unit counts above the empty window), the first rt K-keys by index. K = 0: a
    // zero's sign does not matter to mn / scale (canonicalised + 0.0f below), so one "positive tie" stands for them;
    // K > 0: the segment-wide ranks of the first +K and -K ties (zero_tie_ranks)
    const uint32_t g0 = sd.g_begin, ng = (nu + GU - 1) / GU;  // ng <= UCAP / GU <= NT
    const uint32_t tk = P.tlo[lb] & KEY_MAX;
    gmn = t < ng ? P.gmm[2 * (g0 + t)] : qnan();
    gmx = t < ng ? P.gmm[2 * (g0 + t) + 1] : qnan();
    for (uint32_t i = t; i < nu; i += NT) S.ge[i] = P.gtC[lb + i] | (P.cntZ[lb + i] << 16);
    __syncthreads();
    T = tk;
    rt = st.z;
    fp_rank = rt > 0 ? 0u : NONE;
    if (tk != 0u) zero_tie_ranks<NT>(P, lb, nu, S, fp_rank, fn_rank);  // (block-uniform)
    done = true;
  } else {
    done = st.w == 0 && select_from_groups<NT>(P, sd, lb, nu, st, S, T, rt, fp_rank, fn_rank, gmn, gmx);
  }
  uint32_t raw_path = 0;
  STAMP(P, li, 1);
  if (!done) select_fallback<NT, DELTA>(P, s, sd, S, T, rt, fp_rank, fn_rank, gmn, gmx, raw_path);
  STAMP(P, li, 10);
  select_finish<NT, RAW>(P, s, sd, S, done, zero_tie, raw_path, T, rt, fp_rank, fn_rank, gmn, gmx);
  STAMP(P, li, 12);
}

template <bool DELTA, bool RAW, int NT = SEL_NT>
__global__ __launch_bounds__(NT) void k_select(Params P) {
  __shared__ SelSmem S;
  segment_select<NT, DELTA, RAW>(P, blockIdx.x, S);
}

// ------------------------------------------------------------------------------------------------
// k_emit: EMIT_UPW consecutive large units per wave — each unit's candidate list is already in index
// order: keep key > T and the ties whose segment-wide tie rank is < rt, compact with ballots, write idx +
// code. No LDS. A unit holds ~1.5 % of its 4096 elements as candidates (about one record per lane), so
// one unit per wave was a chain of dependent loads (count -> unit/segment metadata -> records) per 64
// records: here lane g loads unit g's metadata (two dependent rounds for all units at once) and every
// unit's first 64 records are in flight before the first one is classified.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t EMIT_UPW = 4u;  // large units per k_emit wave in batches (round 6, with the interleaved tile: 4 vs 8
                                   // C3 0.586-0.595 vs 0.608-0.639 ms, C2 0.271 vs 0.275-0.278, C3_signs 1.427-1.436 vs
                                   // 1.471-1.543, C4 2.205 vs 2.155-2.202; 2 units: C3 0.624; profiles/r06_ab_emit_upw.txt)
// ... in latency-bound plans (<= LATENCY_PLAN_UNITS units): a wave's units are handled one after the other,
// so fewer per wave shortens the launch (one ResNet-50 update: 8 per wave 13.1 us, 2 per wave 6.0, 1 per
// wave 5.1)
constexpr uint32_t EMIT_UPW_LAT = 1u;
constexpr uint32_t EMIT_UPW_LATENCY = EMIT_UPW_LAT;

// the raw-data emit of one large unit (its segment took the raw-data path): re-read the unit, keep key > T
// and the ties whose segment-wide rank (eqp + ties before them) is < rt, in index order
template <bool DELTA, bool RAW>
DEV void emit_raw_unit(const Params& P, const UnitDev& L, uint32_t T, uint32_t rt, uint32_t eqp, uint64_t obase,
                       float mn, float scale) {
  const uint32_t lane = lane_id();
  uint32_t eqc = 0, outc = 0;
  raw_unit_rows<DELTA>(P, L, [&](uint32_t row, float4 v) {
    const float xs[4] = {v.x, v.y, v.z, v.w};
    const uint32_t e0 = (row * 64 + lane) * 4;
    bool gt[4], tie[4], sel[4];
    uint32_t tpre = 0, spre = 0, ntie = 0, nsel = 0;
    uint64_t tb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t key = fkey(xs[j]);
      const bool ok = e0 + j < L.len;
      gt[j] = ok && key > T;
      tie[j] = ok && key == T;
      tb[j] = __ballot(tie[j]);
      tpre += mbcnt(tb[j]);
      ntie += (uint32_t)__popcll(tb[j]);
    }
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // rank of a tie: ties of lower lanes, then earlier ties of this lane
      sel[j] = gt[j] || (tie[j] && eqp + eqc + tpre + mine < rt);
      mine += tie[j] ? 1u : 0u;
    }
    uint64_t sb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sb[j] = __ballot(sel[j]);
      spre += mbcnt(sb[j]);
      nsel += (uint32_t)__popcll(sb[j]);
    }
    uint32_t k = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (sel[j]) {
        const uint64_t o = obase + outc + spre + k;
        P.idx[o] = (int32_t)(L.start + e0 + j);
        store_val<RAW>(P, o, xs[j], mn, scale);
        ++k;
      }
    }
    eqc += ntie;
    outc += nsel;
  });
}

// one wave emits the large units lu0 + g * stride, g < UPW, below lu1. Batches: a block takes a tile of WAVES * UPW
// consecutive units and its waves interleave them (stride WAVES), so the units that take the raw-data emit — a tie-mode
// segment's first ones, consecutive — are shared by the block's waves instead of filling one wave with 8 raw passes in
// series, while a wave's metadata loads stay within a few lines. (Striding by the whole grid spread them further but
// scattered every wave's metadata loads over 8 lines per array: C2 +2-10 %, C3 +1-6 % by box, profiles/r06_ab.txt.)
template <bool DELTA, bool RAW, uint32_t UPW, uint32_t TR>
DEV void emit_units(const Params& P, uint32_t lu0, uint32_t lu1, uint32_t stride) {
  const uint32_t lane = lane_id();
  auto unit = [&](uint32_t g) { return lu0 + g * stride; };
  const uint32_t ng = lu0 < lu1 ? min(UPW, (lu1 - lu0 + stride - 1) / stride) : 0u;  // this wave's units
  // lane g < UPW holds unit g's count, offsets and its segment's T*, tie budget, mn, scale (lanes past the wave's
  // units repeat its last one; never used)
  const uint32_t lug = unit(min(lane, ng - 1));
  uint32_t nCg, startg, eqpg, oog, Tg, rtg, stg;
  uint64_t sog;
  float mng, scg;
  uint2 rec0[UPW];  // {position, value bits}: every unit's first 64 records
  if constexpr (UPW == 1) {
    // latency-bound plans — ONE load round: the unit's count, record, offsets and its segment's emit parameters
    // (k_select copies them to every unit), and, before the count is known, the unit's first 64 (128) record
    // slots (ccap >= 128: slots past the count hold stale words, never used)
    const uint32_t nCr = P.cntC[lug];
    startg = P.lunits[lug].start;
    sog = P.lunits[lug].out_off;
    eqpg = P.eqpre[lug];
    oog = P.outoff[lug];
    const uint4 ue = P.uemit[lug];
    const uint64_t r0 = (uint64_t)lu0 * P.ccap;
    rec0[0] = make_uint2(P.cpos[r0 + lane], P.cval[r0 + lane]);
    nCg = min(nCr, P.ccap);  // stored records (a raw-path unit may have dropped some)
    Tg = ue.x;
    rtg = ue.y & 0x7FFFFFFFu;
    stg = ue.y >> 31;  // raw-data emit (a raw-path segment, or a zero-tie unit whose zeros the quota reaches)
    mng = RAW ? 0.0f : __uint_as_float(ue.z);
    scg = RAW ? 0.0f : __uint_as_float(ue.w);
  } else {
    // batches: round 1 — the unit's count, offsets and emit parameters; round 2 — every unit's first rows of
    // records (clamped to the count: the one-round form measured slower beside the other sub-batch's streaming)
    nCg = min(P.cntC[lug], P.ccap);
    startg = P.lunits[lug].start;
    sog = P.lunits[lug].out_off;
    eqpg = P.eqpre[lug];
    oog = P.outoff[lug];
    const uint4 ue = P.uemit[lug];
    Tg = ue.x;
    rtg = ue.y & 0x7FFFFFFFu;
    stg = ue.y >> 31;  // raw-data emit
    mng = RAW ? 0.0f : __uint_as_float(ue.z);
    scg = RAW ? 0.0f : __uint_as_float(ue.w);
#pragma unroll
    for (uint32_t g = 0; g < UPW; ++g) {
      const uint32_t lu = unit(min(g, ng - 1)), nC = rl(nCg, g);
      const uint32_t last = nC ? nC - 1 : 0u;
      const uint64_t r0 = (uint64_t)lu * P.ccap;  // unconditional (clamped) loads
      rec0[g] = make_uint2(P.cpos[r0 + min(lane, last)], P.cval[r0 + min(lane, last)]);
    }
  }
#pragma unroll
  for (uint32_t g = 0; g < UPW; ++g) {
    const uint32_t nC = rl(nCg, g);
    if (g < ng && rl(stg, g) != 0) {
      const uint64_t so = ((uint64_t)rl((uint32_t)(sog >> 32), g) << 32) | rl((uint32_t)sog, g);
      emit_raw_unit<DELTA, RAW>(P, P.lunits[unit(g)], rl(Tg, g), rl(rtg, g), rl(eqpg, g), so + rl(oog, g),
                                __uint_as_float(rl(__float_as_uint(mng), g)), __uint_as_float(rl(__float_as_uint(scg), g)));
    } else if (g < ng && nC != 0) {
      const uint32_t lu = unit(g);
      const uint32_t T = rl(Tg, g), rt = rl(rtg, g), eqp = rl(eqpg, g);
      const float mn = __uint_as_float(rl(__float_as_uint(mng), g));
      const float scale = __uint_as_float(rl(__float_as_uint(scg), g));
      const uint64_t so = ((uint64_t)rl((uint32_t)(sog >> 32), g) << 32) | rl((uint32_t)sog, g);
      const uint64_t obase = so + rl(oog, g);
      const uint32_t start = rl(startg, g);
      const uint64_t r0 = (uint64_t)lu * P.ccap;
      uint32_t eqc = 0, outc = 0;
      auto row = [&](uint32_t i0, uint2 rec) {
        const uint32_t i = i0 + lane;
        const bool valid = i < nC;
        const float x = __uint_as_float(rec.y);
        const uint32_t key = fkey(x);
        const bool e = valid && key == T;
        const uint64_t eb = __ballot(e);
        const uint32_t rank = eqp + eqc + mbcnt(eb);
        eqc += (uint32_t)__popcll(eb);
        const bool sel = valid && (key > T || (e && rank < rt));
        const uint64_t sb = __ballot(sel);
        if (sel) {
          const uint64_t o = obase + outc + mbcnt(sb);
          P.idx[o] = (int32_t)(start + rec.x);
          store_val<RAW>(P, o, x, mn, scale);
        }
        outc += (uint32_t)__popcll(sb);
      };
      row(0, rec0[g]);
      // rows past the first (preloaded) one: TR rows per load round (see tail_rows)
      for (uint32_t i0 = 64; i0 < nC; i0 += 64 * TR) {
        uint2 rb[TR];
#pragma unroll
        for (uint32_t b = 0; b < TR; ++b) {
          const uint32_t ic = min(i0 + b * 64 + lane, nC - 1);
          if (i0 + b * 64 < nC) rb[b] = make_uint2(P.cpos[r0 + ic], P.cval[r0 + ic]);  // (wave-uniform)
        }
#pragma unroll
        for (uint32_t b = 0; b < TR; ++b)
          if (i0 + b * 64 < nC) row(i0 + b * 64, rb[b]);
      }
    }
  }
}

template <bool DELTA, bool RAW, uint32_t UPW, uint32_t TR>  // TR: record rows per load round past the first
__global__ __launch_bounds__(BLOCK) void k_emit(Params P) {
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t t0 = blockIdx.x * WAVES * UPW;  // the block's tile of WAVES * UPW consecutive units
  if (t0 + wv >= P.n_lunits) return;
  const bool st = blockIdx.x < P.nseg;  // diagnostics rows: block index (slots 13-14)
  if (st) STAMP(P, blockIdx.x, 13);
  emit_units<DELTA, RAW, UPW, TR>(P, t0 + wv, min(t0 + WAVES * UPW, P.n_lunits), WAVES);
  if (st) STAMP(P, blockIdx.x, 14);
}

// ------------------------------------------------------------------------------------------------
// decode
// ------------------------------------------------------------------------------------------------
// k_decode_lds: every output line written ONCE (non-temporal float4 stores for batches). WPU waves per unit, each
// owning RPW = 16 / WPU of its 16 rows, in passes of QROWS rows through a per-wave LDS tile: the pass's kept
// values are scattered into the zeroed tile (one ds_write per 64 entries), its rows read back (ds_read_b128, + the
// base in delta mode, whose next pass's rows load while the current one goes through LDS) and stored, and the same
// slots zeroed again. The unit's entry range [lo, hi) comes from the per-unit starts: the payload's own (wire v2,
// written by the encoder) or k_bounds'. Round 2 merged the kept values in registers instead (a wave-uniform walk
// over every entry, ~10 VALU each: as much issue time per unit as its stores); round 3 measured one unit per wave in
// two 8-row passes fastest for batches (C3 0.672 -> 0.622 ms per step, profiles/r03_decode_ab.txt). Entries outside
// the wave's rows (an untrusted list) never match a pass and are dropped.
constexpr int DECODE_LDS_WPE = 5;
constexpr int DECODE_LDS_WPE_BASE = 4;  // delta mode: two passes of base rows in registers (5 per SIMD spilled)
constexpr uint32_t DECODE_QROWS = 8u;  // batches, weights mode: rows per tile pass (8: half a unit, 8 KiB of LDS per wave; 4 rows: C3
                                       // 0.671-0.674 ms per step, 8 rows: 0.621-0.623, profiles/r03_decode_ab.txt)
constexpr uint32_t DECODE_QROWS_BASE = 4u;  // delta mode: rows per tile pass
constexpr int DECODE_NT = 256;  // k_decode_lds block size (its per-wave LDS tile is QROWS KiB)
constexpr uint32_t DECODE_WPU_LAT = 2u;  // latency-bound plans: waves per unit (one update: every wave one 8-row pass)
constexpr int DECODE_SAUX_LAT = 0;  // latency-bound plans: store cache policy (a ~100 MB output: plain stores)

// NCH: 64-entry chunks of the unit's kept entries held in registers across the passes (1 at ratios up to ~1.5 %;
// plans of higher ratios take 8 — up to 512 entries, ratio ~12 % — so the entry lists are loaded once per unit,
// not once per pass and again for the zeroing); chunks past NCH are loaded per pass as before
template <bool RAW, bool HASBASE, uint32_t WPU, uint32_t QROWS, int SAUX, bool XCD, uint32_t NCH = 1>
__global__ __launch_bounds__(DECODE_NT, HASBASE ? DECODE_LDS_WPE_BASE : DECODE_LDS_WPE) void k_decode_lds(Params P) {
  constexpr uint32_t DW = DECODE_NT / 64, RPW = UNIT_IT / WPU, NPASS = RPW / QROWS;
  constexpr uint32_t QSH = QROWS == 2u ? 9u : QROWS == 4u ? 10u : QROWS == 8u ? 11u : 12u, QM = (1u << QSH) - 1u;
  static_assert((QROWS << 8) == (1u << QSH) && RPW % QROWS == 0 && NPASS >= 1, "tile pass geometry");
  __shared__ float4 qtile[DW][QROWS * 64];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint32_t wid = (XCD ? xcd_block(blockIdx.x) : blockIdx.x) * DW + wv;
  const uint32_t u = wid / WPU, pass0 = (wid % WPU) * NPASS;  // this wave's unit and first pass (QROWS rows each)
  if (u >= P.n_units) return;
  float4* tile = qtile[wv];
  float* tf = reinterpret_cast<float*>(tile);
#pragma unroll
  for (uint32_t it = 0; it < QROWS; ++it) tile[it * 64 + lane] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  // round 1: the unit and its entry range (the next unit's start is the end of this one's: a non-last unit is
  // followed by its segment's next unit; the index is clamped for the plan's final unit, which is a last unit)
  const UnitDev U = P.units[u];
  uint32_t lo = P.ustart[u];
  uint32_t hi = P.ustart[min(u + 1, P.n_units - 1)];
  const float mn = RAW ? 0.0f : P.cmn[U.seg], sc = RAW ? 0.0f : P.cscale[U.seg];
  // clamp: the bounds may come from an untrusted payload (k >= 1 for every unit); a valid unit holds at most len
  // kept entries (distinct positions), which also bounds the entry loops below for any corrupt range
  lo = min(lo, U.k);
  hi = max(lo, min(min(U.last ? U.k : hi, U.k), lo + U.len));
  const uint32_t cnt = hi - lo;
  // round 2: the first NCH x 64 entries (+ the base rows of the first pass)
  uint32_t qc[NCH], posc[NCH];
#pragma unroll
  for (uint32_t c = 0; c < NCH; ++c) {
    const uint64_t e1 = U.out_off + min(lo + c * 64 + lane, U.k - 1);
    qc[c] = load_code<RAW>(P, e1);
    posc[c] = (uint32_t)P.cidx[e1] - U.start;
  }
  const uint32_t len = U.len;
  const __amdgpu_buffer_rsrc_t rout = unit_rsrc(P.out + U.off, len);
  const __amdgpu_buffer_rsrc_t rb = unit_rsrc(HASBASE ? P.base + U.off : P.out + U.off, len);
  float4 bq[QROWS], bn[QROWS];
  if (HASBASE) {
#pragma unroll
    for (uint32_t it = 0; it < QROWS; ++it) bn[it] = unit_load_x4<false>(rb, rb, ((pass0 * QROWS + it) * 64 + lane) * 16);
  }
  float valc[NCH];
#pragma unroll
  for (uint32_t c = 0; c < NCH; ++c) valc[c] = code_value<RAW>(qc[c], mn, sc);
  lds_order();
#pragma unroll
  for (uint32_t qi = 0; qi < NPASS; ++qi) {
    const uint32_t qq = pass0 + qi;
    if (HASBASE) {
#pragma unroll
      for (uint32_t it = 0; it < QROWS; ++it) bq[it] = bn[it];
      if (qi + 1 < NPASS) {
#pragma unroll
        for (uint32_t it = 0; it < QROWS; ++it)
          bn[it] = unit_load_x4<false>(rb, rb, (((qq + 1) * QROWS + it) * 64 + lane) * 16);
      }
    }
    // scatter: the first NCH x 64 entries are in registers; more are loaded chunk by chunk
#pragma unroll
    for (uint32_t c = 0; c < NCH; ++c)
      if (c * 64 + lane < cnt && (posc[c] >> QSH) == qq) tf[posc[c] & QM] = valc[c];
    for (uint32_t e0 = lo + NCH * 64; e0 < hi; e0 += 64) {
      const uint64_t e = U.out_off + min(e0 + lane, hi - 1);
      const uint32_t p2 = (uint32_t)P.cidx[e] - U.start;
      if (e0 + lane < hi && (p2 >> QSH) == qq) tf[p2 & QM] = code_value<RAW>(load_code<RAW>(P, e), mn, sc);
    }
    lds_order();
    float4 o[QROWS];
#pragma unroll
    for (uint32_t it = 0; it < QROWS; ++it) {
      const float4 d = tile[it * 64 + lane];
      o[it] = HASBASE ? make_float4(bq[it].x + d.x, bq[it].y + d.y, bq[it].z + d.z, bq[it].w + d.w) : d;
    }
    lds_order();
    if (qi + 1 < NPASS) {  // zero what was written (the same slots), for the next pass
#pragma unroll
      for (uint32_t c = 0; c < NCH; ++c)
        if (c * 64 + lane < cnt && (posc[c] >> QSH) == qq) tf[posc[c] & QM] = 0.0f;
      for (uint32_t e0 = lo + NCH * 64; e0 < hi; e0 += 64) {
        const uint64_t e = U.out_off + min(e0 + lane, hi - 1);
        const uint32_t p2 = (uint32_t)P.cidx[e] - U.start;
        if (e0 + lane < hi && (p2 >> QSH) == qq) tf[p2 & QM] = 0.0f;
      }
    }
    if ((len & 3u) == 0) {  // wave-uniform: one float4 buffer store per slot
#pragma unroll
      for (uint32_t it = 0; it < QROWS; ++it) unit_store_x4<SAUX>(rout, ((qq * QROWS + it) * 64 + lane) * 16, o[it]);
    } else {  // a segment's last unit with n % 4 != 0: dword stores (range-checked per dword)
#pragma unroll
      for (uint32_t it = 0; it < QROWS; ++it) unit_store_x1x4<SAUX>(rout, ((qq * QROWS + it) * 64 + lane) * 16, o[it]);
    }
    lds_order();
  }
}

// ------------------------------------------------------------------------------------------------
// aggregate: fused server-side decode + FedAvg of C client updates of one layout
// ------------------------------------------------------------------------------------------------
constexpr int AGG_WPE = 1;  // k_aggregate launch-bounds blocks per CU (register budget)
constexpr uint32_t AGG_SPLIT = 2u;  // waves per 4096-element unit in k_aggregate (each owns UNIT_IT / AGG_SPLIT rows)
constexpr uint32_t AGG_DEPTH = 16u;  // clients whose entries k_aggregate loads together (16 ResNet-50 clients: 4 -> 73.5 us, 8 -> 70.9 us, 16 -> 69.1 us)

struct AggArgs {
  const uint32_t* ustart;  // [n_units] the clients' per-unit starts (wire v2)
  const float* weights;    // [clients] fp32 weights (float(w_i), as torch converts a Python scalar)
  uint32_t clients, T, U0; // clients, segments per client, units per client
  uint64_t Kc;             // kept entries per client (out_off stride between clients)
  float total, inv_total;  // sum of weights; 1.0f / total (fp32 division)
  const uint8_t* avg_mask; // [T] 1: segment averaged, 0: client 0's value passed through; null: all averaged
};

// k_aggregate: one wave per 4096-element unit of the (client-0) layout. For client i in order (segments
// the avg mask leaves out — the buffers of aggregation_content "parameters" — take client 0's x_0 as is,
// as strategies.weighted_sum_only_params / federated_averaging_only_params leave models[0]'s buffers,
// coala/server/strategies.py:32-54, 93-124):
//   x_i = base + d_i   (d_i = decoded value where client i kept the element, +0.0f elsewhere: exactly
//                       what coalac_decode with a base writes; without a base x_i = d_i)
//   acc = x_0 * w_0, then acc = acc + (x_i * w_i)        (torch: params *= w0; params += s_i * w_i)
//   out = acc / total (mode DIV, torch CPU division) or acc * (1.0f / total) (mode RECIP, torch GPU
//   division by a host scalar)                       — coala/server/strategies.py:6-29, 57-90
//   or out = acc (mode SUM: weighted_sum, strategies.py:57-90, whose result the distributed server hands
//   to reduce_models, coala/distributed/distributed.py:42-57)
// x_i goes through a per-wave LDS tile holding base + 0.0f (= base, checked per wave; zero without a base):
// at the client's kept positions base + d_i is written, every lane reads its rows back with ds_read_b128
// (x_i itself: one multiply and one add per element and client), then the base value is put back.
// Latency: every client's range / mn / scale / weight is fetched lane-parallel in one round (lane j =
// client j of a 64-client chunk); the first 64 kept entries of AGG_DEPTH clients are then loaded in one
// batch and accumulated in client order (a unit where some client keeps more than 64 entries takes the
// unbatched path, one client at a time). Clients are identical copies of one layout, so
// client c's unit / segment / entry offsets are u + c*U0, seg + c*T, out_off + c*Kc (host-validated).
template <bool RAW, bool HASBASE, int MODE>
__global__ __launch_bounds__(BLOCK, AGG_WPE) void k_aggregate(Params P, AggArgs A) {
  // AGG_SPLIT waves per unit, each owning RI of its UNIT_IT rows: a smaller LDS tile and half the registers
  // per wave, so twice the waves are resident
  constexpr uint32_t RI = UNIT_IT / AGG_SPLIT, HE = UNIT / AGG_SPLIT;  // rows / elements per wave
  __shared__ float4 tiles[WAVES][HE / 4];
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint32_t wid = blockIdx.x * WAVES + wv;
  const uint32_t u = __builtin_amdgcn_readfirstlane(wid / AGG_SPLIT), h = __builtin_amdgcn_readfirstlane(wid % AGG_SPLIT);
  if (u >= A.U0) return;
  // round 1: the unit (scalar loads), and the first 64 clients' starts in it (lane j: client j; they need
  // only u), pinned above the first use of either
  const UnitDev U = P.units[u];
  const uint32_t ucl0 = u + min(lane, min(64u, A.clients) - 1) * A.U0;
  uint32_t us0 = A.ustart[ucl0], us1 = A.ustart[min(ucl0 + 1, P.n_units - 1)];
  asm volatile("" : "+v"(us0), "+v"(us1)::"memory");
  const uint32_t len = U.len, kseg = U.k;
  const uint32_t e_lo = h * HE;  // first element (within the unit) of this wave's rows
  if (e_lo >= len) return;
  const uint32_t hlen = min(len - e_lo, HE);
  float4* tile = tiles[wv];
  float* tf = reinterpret_cast<float*>(tile);
  const float* bs = HASBASE ? P.base + U.off + e_lo : nullptr;
  // the body twice: full 2048-element rows (every load and store a float4, no length test, so no control-flow
  // merge drains the loads in flight) and a unit's partial last rows
  auto body = [&](auto full_tag) {
    constexpr bool FULL = decltype(full_tag)::value;
    const uint32_t hl = FULL ? HE : hlen;
    auto load_base = [&](uint32_t it) -> float4 {
      const uint32_t e = (it * 64 + lane) * 4;
      if (FULL) return *reinterpret_cast<const float4*>(bs + e);
      return make_float4(e + 0 < hl ? bs[e + 0] : 0.0f, e + 1 < hl ? bs[e + 1] : 0.0f,
                         e + 2 < hl ? bs[e + 2] : 0.0f, e + 3 < hl ? bs[e + 3] : 0.0f);
    };
    // ---- round 2, every request of it issued before any is used: the avg flag, the clients' mn / scale /
    // weight, the base rows and the first AGG_DEPTH clients' entries (all unconditional: a select after a
    // load, never a branch around it)
    struct Meta {
      uint32_t lo, hi;
      float mn, sc, w;
    };
    // lane j: client c0 + j (clamped to the last client of the chunk)
    auto meta_of = [&](uint32_t c0, uint32_t s0, uint32_t s1) -> Meta {
      const uint32_t cl = c0 + min(lane, min(64u, A.clients - c0) - 1);
      const uint32_t sl = U.seg + cl * A.T;
      Meta m;
      m.lo = min(s0, kseg);
      m.hi = max(m.lo, min(min(U.last ? kseg : s1, kseg), m.lo + len));
      m.mn = RAW ? 0.0f : P.cmn[sl];
      m.sc = RAW ? 0.0f : P.cscale[sl];
      m.w = A.weights[cl];
      return m;
    };
    auto meta = [&](uint32_t c0) -> Meta {
      const uint32_t ucl = u + (c0 + min(lane, min(64u, A.clients - c0) - 1)) * A.U0;
      return meta_of(c0, A.ustart[ucl], A.ustart[min(ucl + 1, P.n_units - 1)]);
    };
    // entries of client c0 + j: the raw loaded words only (any arithmetic on them here would make the wave
    // wait for the loads right away, in-order vmcnt)
    auto fetch = [&](const Meta& M, uint32_t c0, uint32_t j, uint32_t& idx, uint32_t& q) {
      const uint32_t jj = min(j, min(64u, A.clients - c0) - 1);
      const uint32_t lo = __builtin_amdgcn_readlane(M.lo, jj), hi = __builtin_amdgcn_readlane(M.hi, jj);
      const uint64_t oo = U.out_off + (uint64_t)(c0 + jj) * A.Kc;
      const uint32_t e = min(lo + lane, hi > lo ? hi - 1 : lo);  // kseg >= 1: entry lo always exists
      idx = (uint32_t)P.cidx[oo + min(e, kseg - 1)];
      q = load_code<RAW>(P, oo + min(e, kseg - 1));
    };
    float4 bv[RI];
#pragma unroll
    for (uint32_t it = 0; it < RI; ++it) bv[it] = HASBASE ? load_base(it) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    lds_order();  // the requests below stay in this body (common to both, the compiler would hoist them above
                  // the length test, whose branch then drains them)
    const uint8_t* amp = A.avg_mask != nullptr ? A.avg_mask + U.seg : reinterpret_cast<const uint8_t*>(A.weights);
    uint32_t am = *amp;
    Meta M = meta_of(0, us0, us1);
    uint32_t pa[AGG_DEPTH], qa[AGG_DEPTH];
#pragma unroll
    for (uint32_t t = 0; t < AGG_DEPTH; ++t) fetch(M, 0, t, pa[t], qa[t]);
    // pinned: no request above moves below this point (the compiler sinks loads toward their first use,
    // which would put the entries' round behind the base's)
    asm volatile("" : "+v"(M.lo), "+v"(M.hi), "+v"(M.mn), "+v"(M.sc), "+v"(M.w), "+v"(am)::"memory");
    const bool avg = A.avg_mask == nullptr || am != 0;
    const uint32_t nclients = avg ? A.clients : 1u;
    if (!avg) M.w = 1.0f;  // (x_0 * 1.0f == x_0)
    // The tile holds x_i where client i kept nothing: base + 0.0f (HASBASE) or +0.0f. The fast path writes
    // tile + d_i at a client's kept positions, which is base + d_i only where base + 0.0f == base: a wave
    // whose rows hold a -0.0f or a NaN base ("odd") takes the generic path, which adds the base read from
    // global memory
    bool odd = false;
#pragma unroll
    for (uint32_t it = 0; it < RI; ++it) {
      const float v[4] = {bv[it].x, bv[it].y, bv[it].z, bv[it].w};
      if (HASBASE) {
#pragma unroll
        for (int c = 0; c < 4; ++c) odd |= __float_as_uint(v[c]) == 0x80000000u || v[c] != v[c];
      }
      const f2v l = f2v{v[0], v[1]} + f2v{0.0f, 0.0f}, h2 = f2v{v[2], v[3]} + f2v{0.0f, 0.0f};
      tile[it * 64 + lane] = HASBASE ? make_float4(l.x, l.y, h2.x, h2.y) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    odd = HASBASE && __ballot(odd) != 0;
    // acc starts at -0.0f, the exact additive identity (-0 + t == t for every t, signed zeros included): the
    // first client's acc + x_0 * w_0 is torch's x_0 * w_0 bit for bit, and no client is special
    float4 acc[RI];
#pragma unroll
    for (uint32_t it = 0; it < RI; ++it) acc[it] = make_float4(-0.0f, -0.0f, -0.0f, -0.0f);
    // acc = acc + x * w: IEEE fp32 ops in this order, on float2 pairs (v_pk_mul_f32 / v_pk_add_f32), x read
    // from the tile
    auto accumulate = [&](float w) {
      const f2v w2 = {w, w};
#pragma unroll
      for (uint32_t it = 0; it < RI; ++it) {
        const float4 x = tile[it * 64 + lane];
        const f2v tl = f2v{x.x, x.y} * w2, th = f2v{x.z, x.w} * w2;
        const f2v sl2 = f2v{acc[it].x, acc[it].y} + tl, sh2 = f2v{acc[it].z, acc[it].w} + th;
        acc[it] = make_float4(sl2.x, sl2.y, sh2.x, sh2.y);
      }
    };
    auto lanef = [](float v, uint32_t j) { return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), j)); };
    const uint32_t pbase = U.start + e_lo;
    for (uint32_t c0 = 0; c0 < nclients; c0 += 64) {
      if (c0 > 0) {
        M = meta(c0);
#pragma unroll
        for (uint32_t t = 0; t < AGG_DEPTH; ++t) fetch(M, c0, t, pa[t], qa[t]);
      }
      const uint32_t cn = min(64u, nclients - c0);
      // generic path (an odd wave, or any client with more than 64 kept entries in this unit, ratio >~ 1.5 %):
      // every client in turn, its entries loaded chunk by chunk, x_i = base + d_i with the base from global
      // memory, put back as base + 0.0f after the rows are read
      if (odd || __ballot(lane < cn && M.hi - M.lo > 64) != 0) {
        for (uint32_t j = 0; j < cn; ++j) {
          const uint32_t lo = __builtin_amdgcn_readlane(M.lo, j), hi = __builtin_amdgcn_readlane(M.hi, j);
          const float mn = lanef(M.mn, j), sc = lanef(M.sc, j);
          const uint64_t oo = U.out_off + (uint64_t)(c0 + j) * A.Kc;
          for (uint32_t e = lo + lane; e < hi; e += 64) {
            const uint32_t p2 = (uint32_t)P.cidx[oo + e] - pbase;
            const float v2 = load_val<RAW>(P, oo + e, mn, sc);
            if (p2 < hl) tf[p2] = HASBASE ? bs[p2] + v2 : v2;
          }
          lds_order();
          accumulate(lanef(M.w, j));
          lds_order();
          for (uint32_t e = lo + lane; e < hi; e += 64) {
            const uint32_t p2 = (uint32_t)P.cidx[oo + e] - pbase;
            if (p2 < hl) tf[p2] = HASBASE ? bs[p2] + 0.0f : 0.0f;
          }
          lds_order();
        }
        continue;
      }
      // fast path, in client order: x = tile + d written at the client's positions, the rows read and
      // accumulated, the tile's value put back. The tile value under the next client's entries is read right
      // after this client's put-back, so the wave never waits on it
      for (uint32_t j0 = 0; j0 < cn; j0 += AGG_DEPTH) {
        if (j0 > 0) {
#pragma unroll
          for (uint32_t t = 0; t < AGG_DEPTH; ++t) fetch(M, c0, j0 + t, pa[t], qa[t]);
        }
        float tb = HASBASE ? tf[min(pa[0] - pbase, HE - 1)] : 0.0f;
#pragma unroll
        for (uint32_t t = 0; t < AGG_DEPTH; ++t) {
          const uint32_t j = j0 + t;
          if (j >= cn) continue;
          const uint32_t pos = pa[t] - pbase;  // wraps (>= hl) outside this wave's rows
          const uint32_t ne = __builtin_amdgcn_readlane(M.hi, j) - __builtin_amdgcn_readlane(M.lo, j);
          const bool mine = lane < ne && pos < hl;
          const float d = code_value<RAW>(qa[t], lanef(M.mn, j), lanef(M.sc, j));
          if (mine) tf[pos] = HASBASE ? tb + d : d;
          lds_order();
          accumulate(lanef(M.w, j));
          lds_order();
          if (mine) tf[pos] = tb;
          if (HASBASE && t + 1 < AGG_DEPTH) tb = tf[min(pa[t + 1] - pbase, HE - 1)];
          lds_order();
        }
      }
    }
    float* out = P.out + U.off + e_lo;
#pragma unroll
    for (uint32_t it = 0; it < RI; ++it) {
      float4 o;
      if (!avg) {
        o = acc[it];
      } else if (MODE == COALAC_AGG_DIV) {
        o = make_float4(acc[it].x / A.total, acc[it].y / A.total, acc[it].z / A.total, acc[it].w / A.total);
      } else if (MODE == COALAC_AGG_SUM) {
        o = acc[it];
      } else {
        o = make_float4(acc[it].x * A.inv_total, acc[it].y * A.inv_total, acc[it].z * A.inv_total,
                        acc[it].w * A.inv_total);
      }
      const uint32_t e = (it * 64 + lane) * 4;
      if (FULL) {
        *reinterpret_cast<float4*>(out + e) = o;
      } else {
        if (e + 0 < hl) out[e + 0] = o.x;
        if (e + 1 < hl) out[e + 1] = o.y;
        if (e + 2 < hl) out[e + 2] = o.z;
        if (e + 3 < hl) out[e + 3] = o.w;
      }
    }
  };
  if (hlen == HE)
    body(std::true_type{});
  else
    body(std::false_type{});
}

// ------------------------------------------------------------------------------------------------
// dense codec: a plan whose every segment keeps all n elements (ratio 1 — the download direction's default,
// coala/server/base.py:196,397 — or segments too small to drop anything). The index list is implied (0..n-1
// per segment) and never materialised; a caller that passes idx / ustart buffers still gets them written.
//   encode: k_dense_minmax (per unit, NaN-ignoring min / max) -> k_dense_seg (per segment: mn, scale) ->
//           k_dense_quant (per unit: read 4 B, write the 1-B code)         — HBM 4 B + 1 B per element
//           (the min / max pass reads the update once more; an update that fits the 256 MB Infinity Cache
//           is re-read from it)
//   decode: k_dense_deq (per unit: read the 1-B code, write 4 B; + base in delta mode)
// One wave per 4096-element unit, 16 float4 per lane, XCD-aware unit order in batches.
// ------------------------------------------------------------------------------------------------
// cache policies: the min / max pass reads with the default policy (an update that fits the Infinity Cache is still
// there for the quantise pass, which reads non-temporally); the dense decode stores non-temporally (one update's
// download 0.073 vs 0.088 ms per step with plain stores; a reciprocal-multiply quantise measured no faster: these
// streams are memory-bound, profiles/r05_ab.txt)
constexpr int DENSE_MM_AUX = 0;
constexpr int DENSE_Q_AUX = 2;  // the quantise stream's loads (non-temporal)
template <bool DELTA, int AUX>  // (AUX: the loads' cache policy)
DEV void dense_unit_load(const Params& P, const UnitDev& U, float4 (&v)[UNIT_IT]) {
  typedef unsigned int u4v __attribute__((ext_vector_type(4)));
  const uint32_t lane = lane_id();
  const float* xin = P.inptr != nullptr ? P.inptr[U.seg] + U.start : P.in + U.off;
  const __amdgpu_buffer_rsrc_t rin = unit_rsrc(xin, U.len);
  const __amdgpu_buffer_rsrc_t rb = unit_rsrc(DELTA ? P.base + U.off : xin, U.len);
#pragma unroll
  for (uint32_t it = 0; it < UNIT_IT; ++it) {
    const int boff = (int)((it * 64 + lane) * 16);
    const u4v a = __builtin_amdgcn_raw_buffer_load_b128(rin, boff, 0, AUX);
    v[it] = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
    if (DELTA) {
      const u4v b = __builtin_amdgcn_raw_buffer_load_b128(rb, boff, 0, AUX);
      v[it] = make_float4(v[it].x - __uint_as_float(b.x), v[it].y - __uint_as_float(b.y), v[it].z - __uint_as_float(b.z),
                          v[it].w - __uint_as_float(b.w));
    }
  }
}

template <bool DELTA, bool XCD>
__global__ __launch_bounds__(BLOCK) void k_dense_minmax(Params P) {
  const uint32_t u = (XCD ? xcd_block(blockIdx.x) : blockIdx.x) * WAVES + (threadIdx.x >> 6);
  if (u >= P.n_units) return;
  const UnitDev U = P.units[u];
  float4 v[UNIT_IT];
  dense_unit_load<DELTA, DENSE_MM_AUX>(P, U, v);
  const uint32_t lane = lane_id();
  float a = qnan(), b = qnan();
#pragma unroll
  for (uint32_t it = 0; it < UNIT_IT; ++it) {
    const uint32_t e0 = (it * 64 + lane) * 4;
    const float xs[4] = {v[it].x, v[it].y, v[it].z, v[it].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = (U.len == UNIT || e0 + j < U.len) ? xs[j] : qnan();  // (loads past len read 0)
      a = fmin_nan(a, x);
      b = fmax_nan(b, x);
    }
  }
  a = wave_min(a);
  b = wave_max(b);
  if (lane == 0) {
    P.umm[2 * u] = a;
    P.umm[2 * u + 1] = b;
  }
}

// one block per segment: its units' partial min / max -> mn, scale (CodecSpec v1: each + 0.0f; scale 0 when
// they are equal); raw values (bits 32): mn = scale = 0
template <bool RAW>
__global__ __launch_bounds__(BLOCK) void k_dense_seg(Params P) {
  __shared__ float shf[2 * WAVES];
  const uint32_t s = blockIdx.x;
  const SegDev sd = P.segs[s];
  float a = qnan(), b = qnan();
  if (!RAW)
    for (uint32_t u = sd.unit_begin + threadIdx.x; u < sd.unit_end; u += BLOCK) {
      a = fmin_nan(a, P.umm[2 * u]);
      b = fmax_nan(b, P.umm[2 * u + 1]);
    }
  block_minmax<BLOCK>(a, b, shf);
  if (threadIdx.x == 0) {
    float mn = 0.0f, scale = 0.0f;
    if (!RAW && sd.n != 0) {
      a = a + 0.0f;
      b = b + 0.0f;
      mn = a;
      scale = (b == a) ? 0.0f : (b - a) / P.levels;
    }
    P.mn[s] = mn;
    P.scale[s] = scale;
  }
}

// SEGRED: every wave reduces its segment's per-unit min / max itself (k_dense_seg folded in: the unit's loads are in
// flight meanwhile, the ~50 KB of pairs are L2-resident, and one launch boundary goes); the segment's first unit
// writes its mn / scale. Used when every segment has a unit (an empty segment has no wave to write its zeros).
template <bool DELTA, bool RAW, bool XCD, bool SEGRED>
__global__ __launch_bounds__(BLOCK) void k_dense_quant(Params P) {
  const uint32_t u = (XCD ? xcd_block(blockIdx.x) : blockIdx.x) * WAVES + (threadIdx.x >> 6);
  if (u >= P.n_units) return;
  const UnitDev U = P.units[u];
  const uint32_t lane = lane_id();
  // SEGRED: the first SEGRED_PAIRS x 64 units' min / max pairs are loaded ahead of the unit's own loads (straight-line
  // code: the reduce waits for them alone, the unit's loads still in flight); a longer segment's remainder afterwards
  constexpr uint32_t SEGRED_PAIRS = 8;
  SegDev sd{};
  float2 m[SEGRED_PAIRS];
  const float2* umm2 = reinterpret_cast<const float2*>(P.umm);
  if (SEGRED) {
    sd = P.segs[U.seg];
    if (!RAW) {
#pragma unroll
      for (uint32_t j = 0; j < SEGRED_PAIRS; ++j) {
        const uint32_t w = sd.unit_begin + j * 64 + lane;
        m[j] = w < sd.unit_end ? umm2[w] : make_float2(qnan(), qnan());
      }
    }
  }
  float4 v[UNIT_IT];
  dense_unit_load<DELTA, DENSE_Q_AUX>(P, U, v);
  float mn = 0.0f, scale = 0.0f;
  if (SEGRED) {
    if (!RAW) {  // (same NaN-ignoring min / max and + 0.0f as k_dense_seg: order-independent, bit-identical)
      float a = qnan(), b = qnan();
#pragma unroll
      for (uint32_t j = 0; j < SEGRED_PAIRS; ++j) {
        a = fmin_nan(a, m[j].x);
        b = fmax_nan(b, m[j].y);
      }
      for (uint32_t w = sd.unit_begin + SEGRED_PAIRS * 64 + lane; w < sd.unit_end; w += 64) {
        const float2 t = umm2[w];
        a = fmin_nan(a, t.x);
        b = fmax_nan(b, t.y);
      }
      a = wave_min(a) + 0.0f;
      b = wave_max(b) + 0.0f;
      mn = a;
      scale = (b == a) ? 0.0f : (b - a) / P.levels;
    }
    if (u == sd.unit_begin && lane == 0) {
      P.mn[U.seg] = mn;
      P.scale[U.seg] = scale;
    }
  } else if (!RAW) {
    mn = P.mn[U.seg];
    scale = P.scale[U.seg];
  }
  const uint64_t o = U.out_off + U.start;  // the unit's first entry (k == n: entry e is element e)
  // whole-dword stores when the unit's codes start 4-byte aligned (16-byte for raw floats) and end on a dword
  const bool vec = (o & 3u) == 0 && (U.len & 3u) == 0;
  if (RAW) {
    float* dst = static_cast<float*>(P.vals) + o;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)(U.len * 4u), 0x00020000);
#pragma unroll
    for (uint32_t it = 0; it < UNIT_IT; ++it) {
      if (vec)
        unit_store_x4<0>(r, (it * 64 + lane) * 16, v[it]);
      else
        unit_store_x1x4<0>(r, (it * 64 + lane) * 16, v[it]);
    }
  } else {
    uint8_t* dst = static_cast<uint8_t*>(P.vals) + o;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)U.len, 0x00020000);
    // RCP: (x - mn) / scale as q = RN(a * y), y = RN(1 / scale), then q + RN(a - q * scale) * y by two FMAs — the
    // correctly rounded quotient (Markstein) when neither the residual nor the quotient leaves the normal range,
    // which scale in [2^-90, 2^90] ensures wherever the code is not 0 (t >= 0.5 needs a >= 2^-91); below that both
    // round to code 0. The IEEE division sequence it replaces cost 3.5 us of the download step (profiles/r06_ab_dense_segred.txt)
    auto codes = [&](auto rcp_tag) {
      constexpr bool RCP = decltype(rcp_tag)::value;
      const float y = RCP ? 1.0f / scale : 0.0f;
      auto qz = [&](float x) -> uint32_t {
        if (!RCP) return quantize(x, mn, scale, P.levels);
        const float a = x - mn;
        const float q = a * y;
        const float t = __builtin_fmaf(__builtin_fmaf(-q, scale, a), y, q);
        const float rt = rintf(t);
        if (!(rt > 0.0f)) return 0u;
        return (uint32_t)(uint8_t)(rt < P.levels ? rt : P.levels);
      };
#pragma unroll
      for (uint32_t it = 0; it < UNIT_IT; ++it) {
        const uint32_t q0 = qz(v[it].x), q1 = qz(v[it].y), q2 = qz(v[it].z), q3 = qz(v[it].w);
        const uint32_t boff = (it * 64 + lane) * 4;
        if (vec) {
          __builtin_amdgcn_raw_buffer_store_b32(q0 | (q1 << 8) | (q2 << 16) | (q3 << 24), r, (int)boff, 0, 0);
        } else {  // (range-checked per byte: the unit's tail past len is dropped)
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)q0, r, (int)boff, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)q1, r, (int)boff + 1, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)q2, r, (int)boff + 2, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)q3, r, (int)boff + 3, 0, 0);
        }
      }
    };
    if (scale >= 0x1p-90f && scale <= 0x1p90f)  // (uniform per wave; scale 0, NaN, inf or extreme: the division)
      codes(std::true_type{});
    else
      codes(std::false_type{});
  }
  if (P.idx != nullptr) {  // a caller that asked for the (implied) indices
    for (uint32_t e = lane; e < U.len; e += 64) P.idx[o + e] = (int32_t)(U.start + e);
  }
  if (P.ustart_out != nullptr && lane == 0) P.ustart_out[u] = U.start;
}

template <bool RAW, bool HASBASE, bool XCD>
__global__ __launch_bounds__(BLOCK) void k_dense_deq(Params P) {
  const uint32_t u = (XCD ? xcd_block(blockIdx.x) : blockIdx.x) * WAVES + (threadIdx.x >> 6);
  if (u >= P.n_units) return;
  const UnitDev U = P.units[u];
  const uint32_t lane = lane_id();
  const float mn = RAW ? 0.0f : P.cmn[U.seg], scale = RAW ? 0.0f : P.cscale[U.seg];
  const uint64_t o = U.out_off + U.start;
  const bool vec = (o & 3u) == 0 && (U.len & 3u) == 0;
  float4 d[UNIT_IT];
  if (RAW) {
    const float* src = static_cast<const float*>(P.cvals) + o;
    const __amdgpu_buffer_rsrc_t r = unit_rsrc(src, U.len);
#pragma unroll
    for (uint32_t it = 0; it < UNIT_IT; ++it) {
      if (vec) {
        d[it] = unit_load_x4<false>(r, r, (it * 64 + lane) * 16);
      } else {
        const uint32_t b = (it * 64 + lane) * 16;
        d[it] = make_float4(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)b, 0, 0)),
                            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)b + 4, 0, 0)),
                            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)b + 8, 0, 0)),
                            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)b + 12, 0, 0)));
      }
    }
  } else {
    const uint8_t* src = static_cast<const uint8_t*>(P.cvals) + o;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), (short)0, (int)U.len, 0x00020000);
    uint32_t w[UNIT_IT];
#pragma unroll
    for (uint32_t it = 0; it < UNIT_IT; ++it) {
      const uint32_t b = (it * 64 + lane) * 4;
      if (vec) {
        w[it] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)b, 0, 0);
      } else {
        w[it] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)b, 0, 0) |
                ((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)b + 1, 0, 0) << 8) |
                ((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)b + 2, 0, 0) << 16) |
                ((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, (int)b + 3, 0, 0) << 24);
      }
    }
#pragma unroll
    for (uint32_t it = 0; it < UNIT_IT; ++it)
      d[it] = make_float4(dequantize((uint8_t)(w[it] & 0xFFu), mn, scale), dequantize((uint8_t)((w[it] >> 8) & 0xFFu), mn, scale),
                          dequantize((uint8_t)((w[it] >> 16) & 0xFFu), mn, scale), dequantize((uint8_t)(w[it] >> 24), mn, scale));
  }
  const __amdgpu_buffer_rsrc_t rout = unit_rsrc(P.out + U.off, U.len);
  const __amdgpu_buffer_rsrc_t rb = unit_rsrc(HASBASE ? P.base + U.off : P.out + U.off, U.len);
#pragma unroll
  for (uint32_t it = 0; it < UNIT_IT; ++it) {
    float4 x = d[it];
    if (HASBASE) {
      const float4 b = unit_load_x4<false>(rb, rb, (it * 64 + lane) * 16);
      x = make_float4(b.x + x.x, b.y + x.y, b.z + x.z, b.w + x.w);
    }
    if ((U.len & 3u) == 0)
      unit_store_x4<STORE_AUX>(rout, (it * 64 + lane) * 16, x);
    else
      unit_store_x1x4<STORE_AUX>(rout, (it * 64 + lane) * 16, x);
  }
}

// k_gather: n scalars of `bytes` each, from their own storage (one device pointer each), into one contiguous
// buffer — an update's passthrough entries (BatchNorm's int64 num_batches_tracked, one per layer) snapshotted
// in one launch instead of a stack of tensor copies
__global__ __launch_bounds__(BLOCK) void k_gather(const void* const* src, uint32_t n, uint32_t bytes, void* dst) {
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const void* s = src[i];
  uint8_t* d = static_cast<uint8_t*>(dst) + (uint64_t)i * bytes;
  if (bytes == 8)
    *reinterpret_cast<uint64_t*>(d) = *static_cast<const uint64_t*>(s);
  else if (bytes == 4)
    *reinterpret_cast<uint32_t*>(d) = *static_cast<const uint32_t*>(s);
  else if (bytes == 2)
    *reinterpret_cast<uint16_t*>(d) = *static_cast<const uint16_t*>(s);
  else
    *d = *static_cast<const uint8_t*>(s);
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_CHECK(expr)                                                                             \
  do {                                                                                              \
    hipError_t e_ = (expr);                                                                         \
    if (e_ != hipSuccess) return fail(COALAC_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct WsLayout {
  size_t status;
  size_t tstar, rtie;
  size_t tlo, thi, cntA, cntC, cntZ, tsgn, gtC, eqC, eqpre, outoff, uemit;
  size_t cval, cpos, stamps, ghist, gcnt, glist, gmm, sstate, shhi;
  size_t umm;  // dense plans: per-unit min / max
  size_t total;
};

// a dense plan's encode workspace: the per-unit min / max only
WsLayout ws_layout_dense(size_t U) {
  WsLayout L{};
  L.umm = 0;
  L.total = std::max<size_t>(align_up(8 * U, 256), 256);
  return L;
}

WsLayout ws_layout(size_t S, size_t LU, size_t NG, size_t NL, uint32_t CC) {
  WsLayout L{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    size_t r = o;
    o = align_up(o + bytes, 256);
    return r;
  };
  L.status = take(4 * S);
  L.tstar = take(4 * S);
  L.rtie = take(4 * S);
  L.tlo = take(4 * LU);
  L.thi = take(4 * LU);
  L.cntA = take(4 * LU);
  L.cntC = take(4 * LU);
  L.cntZ = take(4 * LU);
  L.tsgn = take(4 * LU);
  L.gtC = take(4 * LU);
  L.eqC = take(4 * LU);
  L.eqpre = take(4 * LU);
  L.outoff = take(4 * LU);
  L.uemit = take(16 * LU);
  L.cval = take(4 * (size_t)CC * LU);
  L.cpos = take(2 * (size_t)CC * LU);
  L.stamps = take(8 * NSTAMP * std::max<size_t>(S, 1));
  L.ghist = take(4 * HB2 * NG);
  L.gcnt = take(4 * NG);
  L.glist = take(sizeof(uint2) * GCAP * NG);
  L.gmm = take(8 * NG);
  L.sstate = take(sizeof(uint4) * NL);
  L.shhi = take(4 * NL);
  L.total = std::max<size_t>(o, 256);
  return L;
}

}  // namespace

struct coalac_plan {
  int device = -1;
  int bits = 8;
  int nseg = 0;
  uint32_t n_small = 0, n_large = 0, n_units = 0, n_lunits = 0;
  uint32_t small_max = SMALL_MAX;  // segments of <= this many elements are "small" (encoded whole by one block)
  uint32_t ccap = UNIT;  // candidate record slots per large unit
  bool dense = false;    // every segment keeps all its elements: the dense codec (indices implied)
  bool dense_empty = false;  // a dense plan with a 0-element segment (keeps the separate k_dense_seg)
  double rmax = 0.0;     // the largest k / n of the plan's segments
  uint64_t span = 0, total_k = 0;
  void* meta = nullptr;
  SegDev* segs = nullptr;
  UnitDev* units = nullptr;
  UnitDev* lunits = nullptr;
  uint32_t* small_list = nullptr;
  uint32_t* large_list = nullptr;
  SegDev* lsegs = nullptr;
  SegDev* ssegs = nullptr;
  uint4* groups = nullptr;
  uint4* gseg = nullptr;
  uint32_t n_groups = 0;
  std::vector<SegDev> hsegs;  // host copy (aggregate validates the client-copy structure)
  // encode fork/join: k_small runs on `side`, concurrently with k_sample / k_scan on the caller's stream
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  std::mutex mu;  // serialises the (asynchronous) enqueue sequences that use side / fork / join
  WsLayout ws{};
};

namespace {

int check_device(coalac_plan_t plan) {
  int dev = -1;
  HIP_CHECK(hipGetDevice(&dev));
  if (dev != plan->device)
    return fail(COALAC_EDEVICE, "current device %d differs from the plan's device %d", dev, plan->device);
  return COALAC_OK;
}

void fill_meta(Params& P, coalac_plan_t plan) {
  P.segs = plan->segs;
  P.units = plan->units;
  P.lunits = plan->lunits;
  P.small_list = plan->small_list;
  P.large_list = plan->large_list;
  P.lsegs = plan->lsegs;
  P.ssegs = plan->ssegs;
  P.groups = plan->groups;
  P.gseg = plan->gseg;
  P.n_groups = plan->n_groups;
  P.nseg = (uint32_t)plan->nseg;
  P.n_small = plan->n_small;
  P.n_large = plan->n_large;
  P.n_units = plan->n_units;
  P.n_lunits = plan->n_lunits;
  P.levels = plan->bits == 32 ? 0.0f : (float)((1u << plan->bits) - 1u);
  P.ccap = plan->ccap;
}

// Timing events of the _ev variants: hipEventRecord(ev[i], stream) at boundary i of a call (NULL array or entries:
// nothing recorded). Encode: [0] before k_sample, [1] after it, [2] after k_scan, [3] after the select kernels,
// [4] after k_emit; decode and aggregate: [0] at the start, [1] before the decode kernel, [2] after it.
struct Marks {
  void* const* ev;
  int n;
  int at(int i, hipStream_t st) const {
    if (ev != nullptr && i < n && ev[i] != nullptr) HIP_CHECK(hipEventRecord(static_cast<hipEvent_t>(ev[i]), st));
    return COALAC_OK;
  }
};

#define MARK(i)                         \
  do {                                  \
    const int rc_ = marks.at((i), st);  \
    if (rc_) return rc_;                \
  } while (0)

// Small segments go beside the large ones' pipeline on a side stream once the batch is big enough for
// the fork / join (~10-20 us) to pay off (>= 16384 large units, ~3 ResNet-50 updates).
constexpr uint32_t FORK_MIN_LUNITS = 16384;

// the dense encode: the min / max pass and the per-segment reduction between marks 0 and 1, the quantise stream
// between 1 and 2 (where k_scan sits in a sparse encode)
template <bool DELTA, bool RAW>
int launch_dense_encode(const Params& P, coalac_plan_t plan, hipStream_t st, const Marks& marks) {
  const dim3 g((plan->n_units + WAVES - 1) / WAVES);
  const bool xcd = plan->n_units > LATENCY_PLAN_UNITS;
  MARK(0);
  if (!RAW) {
    if (xcd)
      hipLaunchKernelGGL((k_dense_minmax<DELTA, true>), g, dim3(BLOCK), 0, st, P);
    else
      hipLaunchKernelGGL((k_dense_minmax<DELTA, false>), g, dim3(BLOCK), 0, st, P);
  }
  if (plan->dense_empty) {  // a segment without units: k_dense_seg writes every segment's mn / scale
    hipLaunchKernelGGL((k_dense_seg<RAW>), dim3(plan->nseg), dim3(BLOCK), 0, st, P);
    MARK(1);
    if (xcd)
      hipLaunchKernelGGL((k_dense_quant<DELTA, RAW, true, false>), g, dim3(BLOCK), 0, st, P);
    else
      hipLaunchKernelGGL((k_dense_quant<DELTA, RAW, false, false>), g, dim3(BLOCK), 0, st, P);
  } else {
    MARK(1);
    if (xcd)
      hipLaunchKernelGGL((k_dense_quant<DELTA, RAW, true, true>), g, dim3(BLOCK), 0, st, P);
    else
      hipLaunchKernelGGL((k_dense_quant<DELTA, RAW, false, true>), g, dim3(BLOCK), 0, st, P);
  }
  MARK(2);
  MARK(3);
  MARK(4);
  return COALAC_OK;
}

template <bool RAW, bool HB>
void launch_dense_decode(const Params& P, coalac_plan_t plan, hipStream_t st) {
  const dim3 g((plan->n_units + WAVES - 1) / WAVES);
  if (plan->n_units > LATENCY_PLAN_UNITS)
    hipLaunchKernelGGL((k_dense_deq<RAW, HB, true>), g, dim3(BLOCK), 0, st, P);
  else
    hipLaunchKernelGGL((k_dense_deq<RAW, HB, false>), g, dim3(BLOCK), 0, st, P);
}

template <bool DELTA, bool RAW>
void launch_emit(const Params& P, coalac_plan_t plan, hipStream_t st) {
  const bool hi = plan->rmax > HIGH_RATIO;
  if (plan->n_lunits <= LATENCY_PLAN_UNITS) {
    constexpr uint32_t U = EMIT_UPW_LATENCY * WAVES;
    const dim3 g((plan->n_lunits + U - 1) / U);
    if (hi)
      hipLaunchKernelGGL((k_emit<DELTA, RAW, EMIT_UPW_LATENCY, 4u>), g, dim3(BLOCK), 0, st, P);
    else
      hipLaunchKernelGGL((k_emit<DELTA, RAW, EMIT_UPW_LATENCY, 1u>), g, dim3(BLOCK), 0, st, P);
  } else {
    constexpr uint32_t U = EMIT_UPW * WAVES;
    const dim3 g((plan->n_lunits + U - 1) / U);
    if (hi)
      hipLaunchKernelGGL((k_emit<DELTA, RAW, EMIT_UPW, 4u>), g, dim3(BLOCK), 0, st, P);
    else
      hipLaunchKernelGGL((k_emit<DELTA, RAW, EMIT_UPW, 1u>), g, dim3(BLOCK), 0, st, P);
  }
}

template <bool DELTA, bool RAW>
int launch_encode(const Params& P, coalac_plan_t plan, hipStream_t st, const Marks& marks) {
  const uint32_t gu = (plan->n_lunits + WAVES - 1) / WAVES;
  // small segments: forked beside k_sample / k_scan on the plan's side stream (big batches), beside the samplers in
  // k_presel (other batches), or in k_scan's first blocks beside the streaming waves (latency-bound plans: k_sample
  // alone ahead of it)
  const bool fork = plan->n_small && plan->n_lunits >= FORK_MIN_LUNITS && !(P.flags & COALAC_FLAG_NO_FORK);
  const bool presel = !fork && plan->n_small;
  const bool small_in_scan = presel && plan->n_lunits <= LATENCY_PLAN_UNITS;
  Params Q = P;
  Q.scan_small = 0u;
  std::unique_lock<std::mutex> lk(plan->mu, std::defer_lock);
  if (fork) {
    lk.lock();
    if (plan->side == nullptr) {  // created on first use: pipelined plans never need it
      if (hipStreamCreateWithFlags(&plan->side, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&plan->fork, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&plan->join, hipEventDisableTiming) != hipSuccess)
        return fail(COALAC_EHIP, "creating the plan's side stream / events failed: %s",
                    hipGetErrorString(hipGetLastError()));
    }
  }
  MARK(0);
  if (fork) {
    HIP_CHECK(hipEventRecord(plan->fork, st));
    HIP_CHECK(hipStreamWaitEvent(plan->side, plan->fork, 0));
    hipLaunchKernelGGL((k_small<DELTA, RAW>), dim3(plan->n_small), dim3(BLOCK), 0, plan->side, P);
    HIP_CHECK(hipEventRecord(plan->join, plan->side));
  }
  if (presel && !small_in_scan)
    hipLaunchKernelGGL((k_presel<DELTA, RAW>), dim3(plan->n_large + plan->n_small), dim3(BLOCK), 0, st, P);
  else if (plan->n_large && plan->n_lunits <= LATENCY_PLAN_UNITS)
    hipLaunchKernelGGL((k_sample<DELTA, RAW, SAMPLE_NT_LAT>), dim3(plan->n_large), dim3(SAMPLE_NT_LAT), 0, st, P);
  else if (plan->n_large)
    hipLaunchKernelGGL((k_sample<DELTA, RAW, BLOCK>), dim3(plan->n_large), dim3(BLOCK), 0, st, P);
  MARK(1);
  if (small_in_scan) {
    Q.scan_small = plan->n_small;
    const dim3 gs((plan->n_lunits + SCAN_NT_LAT / 64 - 1) / (SCAN_NT_LAT / 64) + plan->n_small);
    if (plan->small_max <= SMALL_MAX_LATENCY)
      hipLaunchKernelGGL((k_scan<DELTA, RAW, true, SCAN_WPE_LAT_1K, SCAN_NB_LAT, SCAN_NT_LAT, SMALL_MAX_LATENCY>), gs,
                         dim3(SCAN_NT_LAT), 0, st, Q);
    else
      hipLaunchKernelGGL((k_scan<DELTA, RAW, true, SCAN_WPE_LAT, SCAN_NB_LAT, SCAN_NT_LAT>), gs, dim3(SCAN_NT_LAT), 0, st,
                         Q);
  } else if (gu) {
    hipLaunchKernelGGL((k_scan<DELTA, RAW, false, SCAN_WPE, SCAN_NB, SCAN_NT>),
                       dim3((plan->n_lunits + SCAN_NT / 64 - 1) / (SCAN_NT / 64)), dim3(SCAN_NT), 0, st, Q);
  }
  MARK(2);
  if (plan->n_large) {
    const bool lat = plan->n_lunits <= LATENCY_PLAN_UNITS, hr = plan->rmax > HIGH_RATIO;
    if (lat)
      hipLaunchKernelGGL((k_ghist<GHIST_NT_LAT, true>), dim3(plan->n_groups), dim3(GHIST_NT_LAT), 0, st, P);
    else if (hr)
      hipLaunchKernelGGL((k_ghist<BLOCK, false, true>), dim3(plan->n_groups), dim3(BLOCK), 0, st, P);
    else
      hipLaunchKernelGGL((k_ghist<BLOCK, false>), dim3(plan->n_groups), dim3(BLOCK), 0, st, P);
    if (lat)
      hipLaunchKernelGGL((k_gwin<GWIN_NT_LAT, true>), dim3(plan->n_groups), dim3(GWIN_NT_LAT), 0, st, P);
    else if (hr)
      hipLaunchKernelGGL((k_gwin<BLOCK, false, true>), dim3(plan->n_groups), dim3(BLOCK), 0, st, P);
    else
      hipLaunchKernelGGL((k_gwin<BLOCK, false>), dim3(plan->n_groups), dim3(BLOCK), 0, st, P);
    if (lat)
      hipLaunchKernelGGL((k_select<DELTA, RAW, SEL_NT_LAT>), dim3(plan->n_large), dim3(SEL_NT_LAT), 0, st, P);
    else
      hipLaunchKernelGGL((k_select<DELTA, RAW>), dim3(plan->n_large), dim3(SEL_NT), 0, st, P);
  }
  MARK(3);
  if (plan->n_large) launch_emit<DELTA, RAW>(P, plan, st);
  if (fork) HIP_CHECK(hipStreamWaitEvent(st, plan->join, 0));
  MARK(4);
  return COALAC_OK;
}

}  // namespace

extern "C" {

int coalac_version(void) { return COALAC_ABI_VERSION; }

const char* coalac_last_error(void) { return g_err.c_str(); }

int coalac_plan_create(const coalac_seg_t* h_segs, int nseg, int bits, coalac_plan_t* out) {
  if (!out) return fail(COALAC_EINVAL, "coalac_plan_create: out is NULL");
  *out = nullptr;
  if (nseg < 0 || (nseg > 0 && !h_segs)) return fail(COALAC_EINVAL, "coalac_plan_create: bad segment table");
  if (!((bits >= 1 && bits <= 8) || bits == 32)) return fail(COALAC_EBITS, "unsupported bits=%d (1..8 or 32)", bits);

  std::vector<SegDev> segs(nseg);
  std::vector<UnitDev> units, lunits;
  std::vector<uint4> groups, gseg;
  std::vector<uint32_t> small_list, large_list;
  uint64_t span = 0, total_k = 0;
  std::vector<std::pair<uint64_t, uint64_t>> in_r, out_r;
  uint64_t est_units = 0;
  for (int s = 0; s < nseg; ++s) est_units += (std::min<uint64_t>(h_segs[s].n, 1ull << 31) + UNIT - 1) / UNIT;
  uint32_t small_max = est_units <= LATENCY_PLAN_UNITS ? SMALL_MAX_LATENCY : SMALL_MAX_BATCH;
  if (const char* e = getenv("COALAC_SMALL_MAX")) small_max = std::min<uint32_t>(std::max(atoi(e), 1024), SMALL_MAX);
  for (int s = 0; s < nseg; ++s) {
    const coalac_seg_t& g = h_segs[s];
    if (g.n >= (1ull << 31)) return fail(COALAC_EINVAL, "segment %d: n=%llu >= 2^31", s, (unsigned long long)g.n);
    if (g.in_off % 4)
      return fail(COALAC_EINVAL, "segment %d: in_off=%llu not a multiple of 4", s, (unsigned long long)g.in_off);
    if (g.n == 0 ? g.k != 0 : (g.k < 1 || g.k > g.n))
      return fail(COALAC_EINVAL, "segment %d: k=%llu invalid for n=%llu", s, (unsigned long long)g.k,
                  (unsigned long long)g.n);
    if (g.in_off > (1ull << 46) || g.out_off > (1ull << 46)) return fail(COALAC_EINVAL, "segment %d: offset too large", s);
    SegDev d{};
    d.in_off = g.in_off;
    d.out_off = g.out_off;
    d.n = (uint32_t)g.n;
    d.k = (uint32_t)g.k;
    d.unit_begin = (uint32_t)units.size();
    const bool large = g.n > small_max;
    d.lu_begin = large ? (uint32_t)lunits.size() : 0u;
    for (uint64_t st = 0; st < g.n; st += UNIT) {
      UnitDev u{};
      u.off = g.in_off + st;
      u.out_off = g.out_off;
      u.seg = (uint32_t)s;
      u.start = (uint32_t)st;
      u.k = (uint32_t)g.k;
      u.len = (uint16_t)std::min<uint64_t>(UNIT, g.n - st);
      u.last = st + UNIT >= g.n ? 1 : 0;
      units.push_back(u);
      if (large) lunits.push_back(u);
    }
    d.unit_end = (uint32_t)units.size();
    if (large) {
      d.g_begin = (uint32_t)groups.size();
      const uint32_t nu = d.unit_end - d.unit_begin;
      for (uint32_t g0 = 0; g0 < nu; g0 += GU) {
        groups.push_back(make_uint4((uint32_t)large_list.size(), d.lu_begin + g0, std::min(GU, nu - g0), (uint32_t)s));
        gseg.push_back(make_uint4(d.lu_begin, nu, (uint32_t)g.k, d.g_begin));
      }
    }
    (large ? large_list : small_list).push_back((uint32_t)s);
    segs[s] = d;
    if (g.n) {
      span = std::max<uint64_t>(span, g.in_off + g.n);
      total_k = std::max<uint64_t>(total_k, g.out_off + g.k);
      in_r.push_back({g.in_off, g.in_off + g.n});
      out_r.push_back({g.out_off, g.out_off + g.k});
    }
  }
  if (lunits.size() >= (1ull << 32) / UNIT) return fail(COALAC_EINVAL, "plan too large (%zu large units)", lunits.size());
  auto overlaps = [](std::vector<std::pair<uint64_t, uint64_t>>& r) {
    std::sort(r.begin(), r.end());
    for (size_t i = 1; i < r.size(); ++i)
      if (r[i].first < r[i - 1].second) return true;
    return false;
  };
  if (overlaps(in_r)) return fail(COALAC_EINVAL, "segment input ranges overlap");
  if (overlaps(out_r)) return fail(COALAC_EINVAL, "segment output ranges overlap");

  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  coalac_plan* p = new coalac_plan();
  p->device = dev;
  p->bits = bits;
  p->nseg = nseg;
  p->n_small = (uint32_t)small_list.size();
  p->n_large = (uint32_t)large_list.size();
  p->n_units = (uint32_t)units.size();
  p->n_lunits = (uint32_t)lunits.size();
  p->n_groups = (uint32_t)groups.size();
  p->span = span;
  p->total_k = total_k;
  p->hsegs = segs;
  // record slots per large unit: the candidates a unit can expect at the plan's largest ratio (kept
  // share + the sampled band + margin), so the workspace is ~1 B/element at ratio 0.01 instead of 8
  double rmax = 0.0;
  for (uint32_t s2 : large_list) rmax = std::max(rmax, (double)segs[s2].k / (double)segs[s2].n);
  p->rmax = rmax;
  uint32_t ccap = (uint32_t)align_up((size_t)(UNIT * std::min(1.0, 2.0 * rmax + 0.05) + 256.0), 64);
  if (const char* e = getenv("COALAC_CCAP")) ccap = (uint32_t)atoi(e);  // tests: force overflow
  ccap = std::max<uint32_t>(STAGE_CAP, std::min<uint32_t>(UNIT, ccap));
  p->ccap = ccap;
  p->small_max = small_max;
  p->dense = true;
  for (const SegDev& d : segs) p->dense = p->dense && d.k == d.n;
  for (const SegDev& d : segs) p->dense_empty = p->dense_empty || d.unit_begin == d.unit_end;
  p->ws = p->dense ? ws_layout_dense(units.size())
                   : ws_layout((size_t)nseg, lunits.size(), groups.size(), large_list.size(), ccap);

  const size_t o_segs = 0;
  const size_t o_units = align_up(o_segs + sizeof(SegDev) * segs.size(), 256);
  const size_t o_lunits = align_up(o_units + sizeof(UnitDev) * units.size(), 256);
  const size_t o_small = align_up(o_lunits + sizeof(UnitDev) * lunits.size(), 256);
  const size_t o_large = align_up(o_small + 4 * small_list.size(), 256);
  std::vector<SegDev> lsegs, ssegs;
  for (uint32_t s2 : large_list) lsegs.push_back(segs[s2]);
  for (uint32_t s2 : small_list) ssegs.push_back(segs[s2]);
  const size_t o_lsegs = align_up(o_large + 4 * large_list.size(), 256);
  const size_t o_ssegs = align_up(o_lsegs + sizeof(SegDev) * lsegs.size(), 256);
  const size_t o_grp = align_up(o_ssegs + sizeof(SegDev) * ssegs.size(), 256);
  const size_t o_gseg = align_up(o_grp + sizeof(uint4) * groups.size(), 256);
  const size_t bytes = align_up(o_gseg + sizeof(uint4) * gseg.size(), 256) + 256;
  std::vector<uint8_t> host(bytes, 0);
  if (!segs.empty()) memcpy(host.data() + o_segs, segs.data(), sizeof(SegDev) * segs.size());
  if (!units.empty()) memcpy(host.data() + o_units, units.data(), sizeof(UnitDev) * units.size());
  if (!lunits.empty()) memcpy(host.data() + o_lunits, lunits.data(), sizeof(UnitDev) * lunits.size());
  if (!small_list.empty()) memcpy(host.data() + o_small, small_list.data(), 4 * small_list.size());
  if (!large_list.empty()) memcpy(host.data() + o_large, large_list.data(), 4 * large_list.size());
  if (!lsegs.empty()) memcpy(host.data() + o_lsegs, lsegs.data(), sizeof(SegDev) * lsegs.size());
  if (!ssegs.empty()) memcpy(host.data() + o_ssegs, ssegs.data(), sizeof(SegDev) * ssegs.size());
  if (!groups.empty()) memcpy(host.data() + o_grp, groups.data(), sizeof(uint4) * groups.size());
  if (!gseg.empty()) memcpy(host.data() + o_gseg, gseg.data(), sizeof(uint4) * gseg.size());
  hipError_t e = hipMalloc(&p->meta, bytes);
  if (e != hipSuccess) {
    delete p;
    return fail(COALAC_ENOMEM, "hipMalloc(%zu) for plan metadata failed: %s", bytes, hipGetErrorString(e));
  }
  e = hipMemcpy(p->meta, host.data(), bytes, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(p->meta);
    delete p;
    return fail(COALAC_EHIP, "hipMemcpy of plan metadata failed: %s", hipGetErrorString(e));
  }
  uint8_t* m = static_cast<uint8_t*>(p->meta);
  p->segs = reinterpret_cast<SegDev*>(m + o_segs);
  p->units = reinterpret_cast<UnitDev*>(m + o_units);
  p->lunits = reinterpret_cast<UnitDev*>(m + o_lunits);
  p->small_list = reinterpret_cast<uint32_t*>(m + o_small);
  p->large_list = reinterpret_cast<uint32_t*>(m + o_large);
  p->lsegs = reinterpret_cast<SegDev*>(m + o_lsegs);
  p->ssegs = reinterpret_cast<SegDev*>(m + o_ssegs);
  p->groups = reinterpret_cast<uint4*>(m + o_grp);
  p->gseg = reinterpret_cast<uint4*>(m + o_gseg);
  *out = p;
  return COALAC_OK;
}

int coalac_plan_destroy(coalac_plan_t plan) {
  if (!plan) return COALAC_OK;
  int cur = 0;
  if (hipGetDevice(&cur) == hipSuccess && cur != plan->device) (void)hipSetDevice(plan->device);
  hipError_t e = hipFree(plan->meta);
  if (plan->side) (void)hipStreamDestroy(plan->side);
  if (plan->fork) (void)hipEventDestroy(plan->fork);
  if (plan->join) (void)hipEventDestroy(plan->join);
  if (cur != plan->device) (void)hipSetDevice(cur);
  delete plan;
  if (e != hipSuccess) return fail(COALAC_EHIP, "hipFree failed: %s", hipGetErrorString(e));
  return COALAC_OK;
}

int coalac_plan_query(coalac_plan_t plan, uint64_t* ws_bytes, uint64_t* total_k, uint64_t* span, uint64_t* n_units) {
  if (!plan) return fail(COALAC_EINVAL, "coalac_plan_query: plan is NULL");
  if (ws_bytes) *ws_bytes = plan->ws.total;
  if (total_k) *total_k = plan->total_k;
  if (span) *span = plan->span;
  if (n_units) *n_units = plan->n_units;
  return COALAC_OK;
}

}  // extern "C"

namespace {
int encode_impl(coalac_plan_t plan, const float* d_in, const float* const* d_inptr, const float* d_base,
                int32_t* d_idx, void* d_vals, float* d_mn, float* d_scale, uint32_t* d_ustart, void* d_ws,
                uint64_t ws_bytes, unsigned flags, void* stream, const Marks& marks) {
  if (!plan) return fail(COALAC_EINVAL, "coalac_encode: plan is NULL");
  if (plan->nseg == 0) return COALAC_OK;
  if (!d_mn || !d_scale) return fail(COALAC_EINVAL, "coalac_encode: mn/scale pointers are NULL");
  if (plan->span && !d_in && !d_inptr) return fail(COALAC_EINVAL, "coalac_encode: input pointer is NULL");
  if (plan->total_k && (!(d_idx || plan->dense) || !d_vals))
    return fail(COALAC_EINVAL, "coalac_encode: idx/vals pointers are NULL (idx may be NULL for a dense plan only)");
  if ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_base)) & 15)
    return fail(COALAC_EINVAL, "coalac_encode: input/base must be 16-byte aligned");
  if (reinterpret_cast<uintptr_t>(d_ustart) & 3) return fail(COALAC_EINVAL, "coalac_encode: ustart must be 4-byte aligned");
  if (!d_ws || ws_bytes < plan->ws.total)
    return fail(COALAC_EWORKSPACE, "coalac_encode: workspace %llu < required %llu", (unsigned long long)ws_bytes,
                (unsigned long long)plan->ws.total);
  int rc = check_device(plan);
  if (rc) return rc;
  Params P{};
  fill_meta(P, plan);
  P.in = d_in;
  P.inptr = d_inptr;
  P.base = d_base;
  P.idx = d_idx;
  P.vals = d_vals;
  P.mn = d_mn;
  P.scale = d_scale;
  P.ustart_out = d_ustart;
  P.flags = flags;
  uint8_t* w = static_cast<uint8_t*>(d_ws);
  const WsLayout& L = plan->ws;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool delta = d_base != nullptr, raw = plan->bits == 32;
  if (plan->dense) {
    P.umm = reinterpret_cast<float*>(w + L.umm);
    if (delta && raw)
      rc = launch_dense_encode<true, true>(P, plan, st, marks);
    else if (delta)
      rc = launch_dense_encode<true, false>(P, plan, st, marks);
    else if (raw)
      rc = launch_dense_encode<false, true>(P, plan, st, marks);
    else
      rc = launch_dense_encode<false, false>(P, plan, st, marks);
    if (rc) return rc;
    HIP_CHECK(hipGetLastError());
    return COALAC_OK;
  }
  P.tstar = reinterpret_cast<uint32_t*>(w + L.tstar);
  P.rtie = reinterpret_cast<uint32_t*>(w + L.rtie);
  P.status = reinterpret_cast<uint32_t*>(w + L.status);
  P.tlo = reinterpret_cast<uint32_t*>(w + L.tlo);
  P.thi = reinterpret_cast<uint32_t*>(w + L.thi);
  P.cntA = reinterpret_cast<uint32_t*>(w + L.cntA);
  P.cntC = reinterpret_cast<uint32_t*>(w + L.cntC);
  P.cntZ = reinterpret_cast<uint32_t*>(w + L.cntZ);
  P.tsgn = reinterpret_cast<uint32_t*>(w + L.tsgn);
  P.gtC = reinterpret_cast<uint32_t*>(w + L.gtC);
  P.eqC = reinterpret_cast<uint32_t*>(w + L.eqC);
  P.eqpre = reinterpret_cast<uint32_t*>(w + L.eqpre);
  P.outoff = reinterpret_cast<uint32_t*>(w + L.outoff);
  P.uemit = reinterpret_cast<uint4*>(w + L.uemit);
  P.cval = reinterpret_cast<uint32_t*>(w + L.cval);
  P.cpos = reinterpret_cast<uint16_t*>(w + L.cpos);
  P.stamps = (flags & COALAC_FLAG_STAMPS) ? reinterpret_cast<uint64_t*>(w + L.stamps) : nullptr;
  P.ghist = reinterpret_cast<uint32_t*>(w + L.ghist);
  P.gcnt = reinterpret_cast<uint32_t*>(w + L.gcnt);
  P.glist = reinterpret_cast<uint2*>(w + L.glist);
  P.gmm = reinterpret_cast<float*>(w + L.gmm);
  P.sstate = reinterpret_cast<uint4*>(w + L.sstate);
  P.shhi = reinterpret_cast<uint32_t*>(w + L.shhi);
  if (delta && raw)
    rc = launch_encode<true, true>(P, plan, st, marks);
  else if (delta)
    rc = launch_encode<true, false>(P, plan, st, marks);
  else if (raw)
    rc = launch_encode<false, true>(P, plan, st, marks);
  else
    rc = launch_encode<false, false>(P, plan, st, marks);
  if (rc) return rc;
  HIP_CHECK(hipGetLastError());
  return COALAC_OK;
}
}  // namespace

extern "C" {

int coalac_encode_ev(coalac_plan_t plan, const float* d_in, const float* d_base, int32_t* d_idx,
                     void* d_vals, float* d_mn, float* d_scale, uint32_t* d_ustart, void* d_ws, uint64_t ws_bytes,
                     unsigned flags, void* stream, void* const* events) {
  return encode_impl(plan, d_in, nullptr, d_base, d_idx, d_vals, d_mn, d_scale, d_ustart, d_ws, ws_bytes, flags, stream,
                     Marks{events, 5});
}

int coalac_encode_segptr(coalac_plan_t plan, const float* const* d_seg_in, const float* d_base, int32_t* d_idx,
                         void* d_vals, float* d_mn, float* d_scale, uint32_t* d_ustart, void* d_ws, uint64_t ws_bytes,
                         unsigned flags, void* stream) {
  if (plan && plan->nseg && !d_seg_in) return fail(COALAC_EINVAL, "coalac_encode_segptr: d_seg_in is NULL");
  return encode_impl(plan, nullptr, d_seg_in, d_base, d_idx, d_vals, d_mn, d_scale, d_ustart, d_ws, ws_bytes, flags,
                     stream, Marks{nullptr, 0});
}

int coalac_encode(coalac_plan_t plan, const float* d_in, const float* d_base, int32_t* d_idx, void* d_vals,
                  float* d_mn, float* d_scale, uint32_t* d_ustart, void* d_ws, uint64_t ws_bytes, unsigned flags,
                  void* stream) {
  return coalac_encode_ev(plan, d_in, d_base, d_idx, d_vals, d_mn, d_scale, d_ustart, d_ws, ws_bytes, flags, stream,
                          nullptr);
}

}  // extern "C"

namespace {
// The write-once decode (k_decode_lds) of a whole plan: batches one wave per unit in two 8-row passes (4-row in
// delta mode) with non-temporal stores and the XCD-aware order; latency-bound plans DECODE_WPU_LAT waves per unit
// (one pass each: twice the waves, each with half the work, for a launch of one update's ~6.5 k units).
template <bool RAW, bool HB, uint32_t NCH>
void launch_decode_lds_n(const Params& P, coalac_plan_t plan, hipStream_t st) {
  constexpr uint32_t DW = DECODE_NT / 64;
  if (plan->n_units <= LATENCY_PLAN_UNITS) {
    constexpr uint32_t W = DECODE_WPU_LAT, Q = HB ? DECODE_QROWS_BASE : UNIT_IT / DECODE_WPU_LAT;
    hipLaunchKernelGGL((k_decode_lds<RAW, HB, W, (Q < 8u ? Q : 8u), DECODE_SAUX_LAT, false, NCH>),
                       dim3((plan->n_units * W + DW - 1) / DW), dim3(DECODE_NT), 0, st, P);
  } else {
    hipLaunchKernelGGL((k_decode_lds<RAW, HB, 1u, HB ? DECODE_QROWS_BASE : DECODE_QROWS, STORE_AUX, true, NCH>),
                       dim3((plan->n_units + DW - 1) / DW), dim3(DECODE_NT), 0, st, P);
  }
}

// plans whose segments keep more than ~1.5 % (more than 64 entries in a unit on average) hold 8 entry chunks in
// registers (from ratio 0.02: C3 at ratio 0.1, decode 0.63 -> 0.37 ms)
constexpr double DECODE_NCH_RATIO = HIGH_RATIO;
template <bool RAW, bool HB>
void launch_decode_lds(const Params& P, coalac_plan_t plan, hipStream_t st) {
  if (plan->rmax > DECODE_NCH_RATIO)
    launch_decode_lds_n<RAW, HB, 8u>(P, plan, st);
  else
    launch_decode_lds_n<RAW, HB, 1u>(P, plan, st);
}
}  // namespace

extern "C" {

int coalac_decode_ev(coalac_plan_t plan, const int32_t* d_idx, const void* d_vals, const float* d_mn,
                     const float* d_scale, const uint32_t* d_ustart, const float* d_base, float* d_out, void* stream,
                     void* const* events) {
  if (!plan) return fail(COALAC_EINVAL, "coalac_decode: plan is NULL");
  if (plan->n_units == 0) return COALAC_OK;
  if (!d_out) return fail(COALAC_EINVAL, "coalac_decode: output pointer is NULL");
  // a sparse plan decodes every unit's entry range from the per-unit starts (wire v2; the host computes them for a
  // v1 payload); a dense plan's indices and starts are implied (neither is read)
  if (plan->total_k && (!(plan->dense || (d_idx && d_ustart)) || !d_vals))
    return fail(COALAC_EINVAL, "coalac_decode: idx/vals/ustart pointers are NULL (a sparse plan needs the per-unit "
                "starts of wire v2)");
  if (plan->total_k && plan->bits != 32 && (!d_mn || !d_scale))
    return fail(COALAC_EINVAL, "coalac_decode: mn/scale pointers are NULL");
  if ((reinterpret_cast<uintptr_t>(d_out) | reinterpret_cast<uintptr_t>(d_base)) & 15)
    return fail(COALAC_EINVAL, "coalac_decode: output/base must be 16-byte aligned");
  if (reinterpret_cast<uintptr_t>(d_ustart) & 3) return fail(COALAC_EINVAL, "coalac_decode: ustart must be 4-byte aligned");
  int rc = check_device(plan);
  if (rc) return rc;
  Params P{};
  fill_meta(P, plan);
  P.cidx = d_idx;
  P.cvals = d_vals;
  P.cmn = d_mn;
  P.cscale = d_scale;
  P.base = d_base;
  P.out = d_out;
  P.ustart = d_ustart;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool raw = plan->bits == 32, hb = d_base != nullptr;
  const Marks marks{events, 3};
  MARK(0);
  MARK(1);
#define DISPATCH(F, ...)                                   \
  do {                                                     \
    if (raw && hb) F<true, true>(__VA_ARGS__);             \
    else if (raw) F<true, false>(__VA_ARGS__);             \
    else if (hb) F<false, true>(__VA_ARGS__);              \
    else F<false, false>(__VA_ARGS__);                     \
  } while (0)
  if (plan->dense)
    DISPATCH(launch_dense_decode, P, plan, st);  // every element kept: one positional dequantise stream
  else
    DISPATCH(launch_decode_lds, P, plan, st);
#undef DISPATCH
  MARK(2);
  HIP_CHECK(hipGetLastError());
  return COALAC_OK;
}

int coalac_decode(coalac_plan_t plan, const int32_t* d_idx, const void* d_vals, const float* d_mn,
                  const float* d_scale, const uint32_t* d_ustart, const float* d_base, float* d_out, void* stream) {
  return coalac_decode_ev(plan, d_idx, d_vals, d_mn, d_scale, d_ustart, d_base, d_out, stream, nullptr);
}

int coalac_aggregate_ev(coalac_plan_t plan, int clients, const int32_t* d_idx, const void* d_vals,
                        const float* d_mn, const float* d_scale, const uint32_t* d_ustart, const float* d_weights,
                        float total, int mode,
                        const uint8_t* d_avg_mask, const float* d_base, float* d_out, void* stream,
                        void* const* events) {
  if (!plan) return fail(COALAC_EINVAL, "coalac_aggregate: plan is NULL");
  if (clients < 1 || plan->nseg % clients) return fail(COALAC_EINVAL, "coalac_aggregate: %d segments are not %d copies "
                                                       "of one layout", plan->nseg, clients);
  if (mode != COALAC_AGG_DIV && mode != COALAC_AGG_RECIP && mode != COALAC_AGG_SUM)
    return fail(COALAC_EINVAL, "coalac_aggregate: bad mode %d", mode);
  if (plan->n_units == 0) return COALAC_OK;
  if (!d_out || !d_weights) return fail(COALAC_EINVAL, "coalac_aggregate: output/weights pointer is NULL");
  if (plan->total_k && (!d_idx || !d_vals || !d_ustart))
    return fail(COALAC_EINVAL, "coalac_aggregate: idx/vals/ustart pointers are NULL (the per-unit starts of wire v2; a "
                "dense plan's implied indices and starts must be passed here)");
  if (plan->bits != 32 && (!d_mn || !d_scale)) return fail(COALAC_EINVAL, "coalac_aggregate: mn/scale pointers are NULL");
  if ((reinterpret_cast<uintptr_t>(d_out) | reinterpret_cast<uintptr_t>(d_base)) & 15)
    return fail(COALAC_EINVAL, "coalac_aggregate: output/base must be 16-byte aligned");
  if (reinterpret_cast<uintptr_t>(d_ustart) & 3)
    return fail(COALAC_EINVAL, "coalac_aggregate: ustart must be 4-byte aligned");
  // the table must be `clients` copies of one layout at constant input / output strides
  const uint32_t T = (uint32_t)(plan->nseg / clients);
  const std::vector<SegDev>& H = plan->hsegs;
  const uint32_t U0 = plan->n_units / (uint32_t)clients;
  if (plan->n_units % (uint32_t)clients) return fail(COALAC_EINVAL, "coalac_aggregate: unit count not divisible");
  const uint64_t S = clients > 1 ? H[T].in_off - H[0].in_off : 0, Kc = clients > 1 ? H[T].out_off - H[0].out_off : 0;
  for (uint32_t c = 1; c < (uint32_t)clients; ++c)
    for (uint32_t t = 0; t < T; ++t) {
      const SegDev &a = H[t], &b = H[c * T + t];
      if (b.n != a.n || b.k != a.k || b.in_off != a.in_off + c * S || b.out_off != a.out_off + c * Kc ||
          b.unit_begin != a.unit_begin + c * U0)
        return fail(COALAC_EINVAL, "coalac_aggregate: segment %u of client %u is not a copy of segment %u of client 0",
                    c * T + t, c, t);
    }
  int rc = check_device(plan);
  if (rc) return rc;
  Params P{};
  fill_meta(P, plan);
  P.cidx = d_idx;
  P.cvals = d_vals;
  P.cmn = d_mn;
  P.cscale = d_scale;
  P.base = d_base;
  P.out = d_out;
  AggArgs A{};
  A.ustart = d_ustart;
  A.weights = d_weights;
  A.clients = (uint32_t)clients;
  A.T = T;
  A.U0 = U0;
  A.Kc = Kc;
  A.total = total;
  A.inv_total = 1.0f / total;
  A.avg_mask = d_avg_mask;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const Marks marks{events, 3};
  MARK(0);
  MARK(1);
  const uint32_t g = (U0 * AGG_SPLIT + WAVES - 1) / WAVES;
  const bool raw = plan->bits == 32, hb = d_base != nullptr;
#define AGG(R, H, M) hipLaunchKernelGGL((k_aggregate<R, H, M>), dim3(g), dim3(BLOCK), 0, st, P, A)
#define AGG_MODES(R, H)                     \
  do {                                      \
    if (mode == COALAC_AGG_RECIP)           \
      AGG(R, H, COALAC_AGG_RECIP);          \
    else if (mode == COALAC_AGG_SUM)        \
      AGG(R, H, COALAC_AGG_SUM);            \
    else                                    \
      AGG(R, H, COALAC_AGG_DIV);            \
  } while (0)
  if (raw) {
    if (hb) AGG_MODES(true, true); else AGG_MODES(true, false);
  } else {
    if (hb) AGG_MODES(false, true); else AGG_MODES(false, false);
  }
#undef AGG_MODES
#undef AGG
  MARK(2);
  HIP_CHECK(hipGetLastError());
  return COALAC_OK;
}

int coalac_aggregate(coalac_plan_t plan, int clients, const int32_t* d_idx, const void* d_vals, const float* d_mn,
                     const float* d_scale, const uint32_t* d_ustart, const float* d_weights, float total, int mode,
                     const uint8_t* d_avg_mask, const float* d_base, float* d_out, void* stream) {
  return coalac_aggregate_ev(plan, clients, d_idx, d_vals, d_mn, d_scale, d_ustart, d_weights, total, mode, d_avg_mask,
                             d_base, d_out, stream, nullptr);
}

int coalac_gather(const void* const* d_src, int n, int elem_bytes, void* d_out, void* stream) {
  if (n < 0 || (n > 0 && (!d_src || !d_out))) return fail(COALAC_EINVAL, "coalac_gather: bad arguments");
  if (elem_bytes != 1 && elem_bytes != 2 && elem_bytes != 4 && elem_bytes != 8)
    return fail(COALAC_EINVAL, "coalac_gather: element size %d (1, 2, 4 or 8)", elem_bytes);
  if (reinterpret_cast<uintptr_t>(d_out) % (uintptr_t)elem_bytes)
    return fail(COALAC_EINVAL, "coalac_gather: output not aligned to the element size");
  if (n == 0) return COALAC_OK;
  hipLaunchKernelGGL(k_gather, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, static_cast<hipStream_t>(stream), d_src,
                     (uint32_t)n, (uint32_t)elem_bytes, d_out);
  HIP_CHECK(hipGetLastError());
  return COALAC_OK;
}

int coalac_workspace_fallbacks(coalac_plan_t plan, const void* d_ws, void* stream, int* out) {
  if (!plan || !d_ws || !out) return fail(COALAC_EINVAL, "coalac_workspace_fallbacks: NULL argument");
  *out = 0;
  if (plan->nseg == 0 || plan->dense) return COALAC_OK;
  std::vector<uint32_t> st(plan->nseg);
  std::vector<uint32_t> large(plan->n_large);
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_CHECK(hipMemcpyAsync(st.data(), static_cast<const uint8_t*>(d_ws) + plan->ws.status, 4 * st.size(),
                           hipMemcpyDeviceToHost, s));
  if (plan->n_large)
    HIP_CHECK(hipMemcpyAsync(large.data(), plan->large_list, 4 * large.size(), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  int c = 0;
  for (uint32_t s2 : large) c += st[s2] == 1;
  *out = c;
  return COALAC_OK;
}

int coalac_debug_brackets(coalac_plan_t plan, const void* d_ws, void* stream, uint32_t* host_tlo, uint32_t* host_thi,
                          int n) {
  if (!plan || !d_ws || !host_tlo || !host_thi || n < 0) return fail(COALAC_EINVAL, "coalac_debug_brackets: bad argument");
  if (plan->dense) return 0;
  const size_t cnt = std::min<size_t>((size_t)n, plan->n_lunits);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (cnt) {
    HIP_CHECK(hipMemcpyAsync(host_tlo, static_cast<const uint8_t*>(d_ws) + plan->ws.tlo, 4 * cnt, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(host_thi, static_cast<const uint8_t*>(d_ws) + plan->ws.thi, 4 * cnt, hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(hipStreamSynchronize(s));
  return (int)cnt;
}

int coalac_debug_stamps(coalac_plan_t plan, const void* d_ws, void* stream, uint64_t* host, int n) {
  if (!plan || !d_ws || !host || n < 0) return fail(COALAC_EINVAL, "coalac_debug_stamps: bad argument");
  const size_t cap = (size_t)NSTAMP * std::max<size_t>(plan->nseg, 1);
  const size_t cnt = std::min<size_t>((size_t)n, cap);
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_CHECK(hipMemcpyAsync(host, static_cast<const uint8_t*>(d_ws) + plan->ws.stamps, 8 * cnt,
                           hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return (int)cnt;
}

}  // extern "C"
