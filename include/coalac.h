/*
 * coalac.h — C ABI of the MI355X (gfx950) model-update codec (CodecSpec v1: per-tensor top-k + 8-bit
 * quantise). This is the drop-in boundary for COALA's compression plugin surface.
 *
 * The reference (SonyResearch/COALA) is 100 % Python and has NO codec and NO FFI: coala/compression/
 * __init__.py is 0 bytes. The entry points below replace the work the reference's empty hooks would do:
 *
 *   coalac_encode  <- BaseClient.compression()          /root/reference/coala/client/base.py:330-332
 *                     (called from run_train, base.py:153; its output rides in UploadContent.data via
 *                      codec.marshal, base.py:363 / coala/protocol/codec.py:4-5)
 *                     and BaseServer.compression()        /root/reference/coala/server/base.py:347-349
 *   coalac_decode  <- BaseServer.decompression(model)   /root/reference/coala/server/base.py:558-560
 *                     (called at server/base.py:376 and server/service.py:106,125)
 *                     and BaseClient.decompression()      /root/reference/coala/client/base.py:203-205
 *   coalac_plan_*  <- no counterpart: a tensor layout (segment table) is fixed for a whole FL task, so
 *                     the device-side metadata is built once per layout and reused every round.
 *
 * Conventions
 *   - Every d_* pointer is a DEVICE pointer owned by the caller (e.g. torch tensor storage).
 *   - All work is enqueued on the caller's HIP stream (`stream`, a hipStream_t; NULL = default stream)
 *     and returns immediately. No host synchronisation, no allocation inside encode/decode.
 *   - Re-entrant: no global mutable state. A plan is immutable after creation and may be shared by
 *     threads; each concurrent encode needs its own workspace.
 *   - Errors: return value 0 = OK, negative = error code below; nothing throws across the ABI. The
 *     message of the last failed call on the calling thread is in coalac_last_error().
 */
#ifndef COALAC_H
#define COALAC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define COALAC_ABI_VERSION 5

enum {
  COALAC_OK = 0,
  COALAC_EINVAL = -1,      /* invalid argument (bad segment table, null pointer, misaligned offset) */
  COALAC_EBITS = -2,       /* unsupported bit width (valid: 1..8, or 32 = raw fp32 values) */
  COALAC_EWORKSPACE = -3,  /* workspace smaller than coalac_plan_query() says */
  COALAC_EHIP = -4,        /* a HIP runtime call or kernel launch failed */
  COALAC_EDEVICE = -5,     /* called with a different current device than the plan was created on */
  COALAC_ENOMEM = -6       /* device allocation for the plan failed */
};

enum {
  COALAC_FLAG_FORCE_EXACT = 1,    /* test hook: re-select every large segment exactly (no sampling) */
  COALAC_FLAG_GENERIC_SELECT = 2, /* test hook: resolve the k-th key with the multi-pass select only */
  COALAC_FLAG_STAMPS = 4,         /* diagnostics: record per-block phase timestamps of k_select */
  COALAC_FLAG_NO_FORK = 8         /* encode small segments inside k_scan, never on the plan's side stream
                                     (for callers that run several plans concurrently themselves) */
};
/* (ABI 3 dropped ABI 2's COALAC_FLAG_ONE_LAUNCH / FRONT_LAUNCH / ITEM_STAMPS: the one-launch encode variants
 * measured slower than the kernel sequence, DESIGN.md §6c. ABI 4 added the per-unit starts d_ustart to encode,
 * decode and aggregate: wire v2. ABI 5 makes them required by the sparse decode and the aggregate — a host that
 * receives a version-1 payload computes them (coala_amd/compression/plan.py) — and drops the decode workspace,
 * the k_bounds / k_fill / k_scatter kernels and the staged (_sched) entry points; plans whose every segment keeps
 * all its elements run the dense codec, with the indices implied.) */

/* One fp32 segment (= one flattened tensor of the state_dict). Offsets are in ELEMENTS.
 *   in_off : start of the segment in the flat input / dense output buffer; must be a multiple of 4
 *   n      : element count, 0 <= n < 2^31
 *   k      : kept elements, 0 if n == 0 else 1 <= k <= n (host computes max(1, min(n, ceil(n*ratio))))
 *   out_off: start of this segment's k entries in the idx / vals arrays                              */
typedef struct coalac_seg {
  uint64_t in_off;
  uint64_t n;
  uint64_t k;
  uint64_t out_off;
} coalac_seg_t;

typedef struct coalac_plan* coalac_plan_t;

int coalac_version(void);
const char* coalac_last_error(void);

/* Build the device metadata for a segment table (HOST pointer) on the current device.
 * bits: 1..8 -> uint8 codes (vals is uint8_t[total_k]); 32 -> raw fp32 values (vals is float[total_k]). */
int coalac_plan_create(const coalac_seg_t* h_segs, int nseg, int bits, coalac_plan_t* out);
int coalac_plan_destroy(coalac_plan_t plan);

/* ws_bytes: the workspace coalac_encode needs (decode and aggregate need none);
 * total_k: length of idx/vals;
 * span: max(in_off + n) = the minimum length (elements) of the input/output flat buffers;
 * n_units: 4096-element work units (segment by segment: ceil(n / 4096) each) = the length of the per-unit
 * starts array (ustart). Any output pointer may be NULL. */
int coalac_plan_query(coalac_plan_t plan, uint64_t* ws_bytes, uint64_t* total_k, uint64_t* span, uint64_t* n_units);

/* Encode d_in (fp32[span]) into idx (int32[total_k], segment-relative, ascending per segment),
 * vals (uint8[total_k] codes or fp32[total_k]), mn (fp32[nseg]) and scale (fp32[nseg]).
 * d_ustart (uint32[n_units], or NULL = not written): per 4096-element unit, the index (segment-relative, into
 * the segment's idx list) of its first kept entry — the wire v2 section that lets a decoder find every unit's
 * entries without searching the idx lists (coalac_decode / coalac_aggregate d_ustart).
 * d_base != NULL selects delta mode: the codec encodes (d_in - d_base).
 * A DENSE plan (every segment's k == n: ratio 1, the download direction's default) runs the dense codec: a
 * per-segment min / max pass, then one quantise stream; its indices are implied (0..n-1 per segment) and d_idx /
 * d_ustart may be NULL (given, they are written too). */
int coalac_encode(coalac_plan_t plan, const float* d_in, const float* d_base, int32_t* d_idx,
                  void* d_vals, float* d_mn, float* d_scale, uint32_t* d_ustart, void* d_ws, uint64_t ws_bytes,
                  unsigned flags, void* stream);

/* Encode with every segment read from its OWN device pointer: d_seg_in is a DEVICE array of nseg
 * pointers, d_seg_in[s] -> fp32[n_s], 16-byte aligned (e.g. the data pointers of a model's parameters:
 * the plugin encodes the trained state in place, with no flattening copy — client compression(),
 * coala/client/base.py:330-332). d_base (delta mode) stays a flat buffer indexed by in_off. Outputs,
 * workspace, flags and stream as coalac_encode. */
int coalac_encode_segptr(coalac_plan_t plan, const float* const* d_seg_in, const float* d_base, int32_t* d_idx,
                         void* d_vals, float* d_mn, float* d_scale, uint32_t* d_ustart, void* d_ws, uint64_t ws_bytes,
                         unsigned flags, void* stream);

/* Decode into the dense d_out (fp32[span]); only positions inside segments are written.
 * d_ustart: the encoder's per-unit starts (wire v2; required unless the plan is dense — a host holding a v1
 * payload computes them: for unit u of a segment, the number of the segment's kept indices below u * 4096).
 * d_base != NULL: d_out = d_base + decoded (fused; d_out may alias d_base). The encoded arrays may come from an
 * untrusted blob: out-of-range or unsorted indices, or wrong starts, can mis-decode but never write outside the
 * unit (still, validate blobs on the host; coala_amd/compression/codec.py validate() does). A dense plan decodes
 * positionally (d_idx / d_ustart are not read). */
int coalac_decode(coalac_plan_t plan, const int32_t* d_idx, const void* d_vals, const float* d_mn,
                  const float* d_scale, const uint32_t* d_ustart, const float* d_base, float* d_out, void* stream);

/* Profiling variants: identical work, plus hipEventRecord(events[i], stream) between kernels.
 * encode: [0] before k_sample, [1] after k_sample, [2] after k_scan, [3] after the select kernels
 *         (k_ghist, k_gwin, k_select), [4] after k_emit (recorded even if the plan has no large segment);
 *         dense plans: [1] after the min / max pass, [2] after the quantise stream;
 * decode: [0] at the start, [1] before the decode kernel, [2] after it. NULL array or NULL entries are skipped. */
int coalac_encode_ev(coalac_plan_t plan, const float* d_in, const float* d_base, int32_t* d_idx,
                     void* d_vals, float* d_mn, float* d_scale, uint32_t* d_ustart, void* d_ws, uint64_t ws_bytes,
                     unsigned flags, void* stream, void* const* events);
int coalac_decode_ev(coalac_plan_t plan, const int32_t* d_idx, const void* d_vals, const float* d_mn,
                     const float* d_scale, const uint32_t* d_ustart, const float* d_base, float* d_out, void* stream,
                     void* const* events);

/* Fused server-side decode + FedAvg of the `clients` updates the plan batches.
 * Replaces, on the server, decompression of every upload (coala/server/base.py:558-560, called :376)
 * followed by strategies.federated_averaging (coala/server/strategies.py:6-29, 57-90) on the decoded
 * modules, for the fp32 entries. The plan's table must be `clients` copies of one layout at constant
 * input / output strides (client-major, as a batched encode uses). Per element of client 0's layout:
 *   x_i = d_base + decoded_i   (decoded_i = +0.0f where client i did not keep the element; without a
 *                               base x_i = decoded_i: exactly what coalac_decode writes)
 *   acc = x_0 * w_0;  acc = acc + (x_i * w_i) for i = 1.. in client order (fp32, no FMA)
 *   d_out = acc / total               (mode COALAC_AGG_DIV: torch's CPU division by a scalar)
 *         = acc * (1.0f / total)      (mode COALAC_AGG_RECIP: torch's GPU division by a host scalar)
 *         = acc                       (mode COALAC_AGG_SUM: strategies.weighted_sum, :57-90 — the
 *                                      multi-GPU server's per-rank sum before reduce_models'
 *                                      all_reduce + division, coala/server/base.py:595-598)
 * d_avg_mask: DEVICE uint8[segments per client] or NULL (= every segment averaged). A segment whose byte
 * is 0 is not averaged: d_out = x_0, client 0's decoded value — aggregation_content "parameters"
 * (coala/server/base.py:588-591), where strategies.weighted_sum_only_params / federated_averaging_only_params
 * average the parameters only and keep models[0]'s buffers (coala/server/strategies.py:32-54, 93-124).
 * d_weights: DEVICE fp32[clients] = float(w_i); total: float(sum of the weights). d_out / d_base are
 * indexed like client 0's segments. d_ustart: the clients' per-unit starts, concatenated in client order
 * (uint32[n_units]; required). Events (the _ev variant): [0] at the start, [1] before k_aggregate, [2] after. */
enum { COALAC_AGG_DIV = 0, COALAC_AGG_RECIP = 1, COALAC_AGG_SUM = 2 };
int coalac_aggregate(coalac_plan_t plan, int clients, const int32_t* d_idx, const void* d_vals,
                     const float* d_mn, const float* d_scale, const uint32_t* d_ustart, const float* d_weights,
                     float total, int mode, const uint8_t* d_avg_mask, const float* d_base, float* d_out,
                     void* stream);
int coalac_aggregate_ev(coalac_plan_t plan, int clients, const int32_t* d_idx, const void* d_vals,
                        const float* d_mn, const float* d_scale, const uint32_t* d_ustart, const float* d_weights,
                        float total, int mode, const uint8_t* d_avg_mask, const float* d_base, float* d_out,
                        void* stream, void* const* events);

/* Snapshot n scalars of elem_bytes (1, 2, 4 or 8) each, read through the DEVICE pointer array d_src (each pointer
 * aligned to elem_bytes), into the contiguous d_out, in one launch on `stream`: the passthrough entries of an
 * update — BatchNorm's int64 num_batches_tracked, one per layer — that the carrier takes with the encoded tensors
 * (client compression(), coala/client/base.py:330-332; they travel raw, CodecSpec v1). */
int coalac_gather(const void* const* d_src, int n, int elem_bytes, void* d_out, void* stream);

/* Diagnostics: number of segments whose sampled thresholds were rejected and re-selected exactly in
 * the last encode that used workspace d_ws (synchronises `stream`). */
int coalac_workspace_fallbacks(coalac_plan_t plan, const void* d_ws, void* stream, int* out);

/* Diagnostics: copy up to n phase timestamps (32 per segment row: k_sample, k_ghist, k_gwin, k_select phases, 100 MHz
 * ticks; 0 = phase not reached) of the last COALAC_FLAG_STAMPS encode with d_ws to host (synchronises
 * `stream`). Returns the count copied or a negative error. */
int coalac_debug_stamps(coalac_plan_t plan, const void* d_ws, void* stream, uint64_t* host, int n);

/* Diagnostics: copy the sampled brackets {T_lo, T_hi} of the first n large units (plan order: the large segments'
 * units, segment after segment) of the last encode with d_ws to host (synchronises `stream`). T_lo carries the tie
 * flag (bit 31) of a tie-mode segment. Returns the count copied or a negative error. */
int coalac_debug_brackets(coalac_plan_t plan, const void* d_ws, void* stream, uint32_t* host_tlo, uint32_t* host_thi,
                          int n);

#ifdef __cplusplus
}
#endif

#endif /* COALAC_H */
