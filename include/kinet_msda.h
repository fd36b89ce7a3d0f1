/* kinet_amd C-ABI: multi-scale deformable attention (MSDeformAttn) sampling.
 *
 * Drop-in for the reference extension module `MultiScaleDeformableAttention`
 * (src/trackformer/models/ops/src/vision.cpp:4-7), whose two pybind functions
 *   ms_deform_attn_forward  -> ms_deform_attn.h:10-28  -> ms_deform_attn_cuda.cu:19-86
 *   ms_deform_attn_backward -> ms_deform_attn.h:30-49  -> ms_deform_attn_cuda.cu:89-168
 * are re-exposed by kinet_amd/MultiScaleDeformableAttention.py on top of these symbols.
 *
 * Layouts (all contiguous, row-major, as in ms_deform_attn_cuda.cu:25-27):
 *   value          (N, S, M, D)            value_dtype
 *   spatial_shapes (L, 2) int64 (H, W)     DEVICE memory (as the reference passes it)
 *   sampling_loc   (N, Lq, M, L, P, 2)     loc_dtype, [x, y] in [0,1] (cuh:220-221)
 *   attn_weight    (N, Lq, M, L, P)        loc_dtype
 *   output         (N, Lq, M*D)            value_dtype, channel = m*D + d (cu:83)
 * level_start_index is derived on the device from spatial_shapes (the reference
 * builds it with per-level ATen ops, cu:52-58); a level whose start + H*W exceeds S
 * contributes zero instead of reading out of bounds.
 *
 * dtypes: value in {F32, F64, BF16, F16}; loc_dtype == value_dtype for F32/F64 (the
 * reference's AT_DISPATCH_FLOATING_TYPES, cu:69), loc_dtype == F32 for BF16/F16 (perf
 * mode).  Accumulation is f32 (f64 for F64).
 *
 * im2col_step is accepted for signature parity and validated exactly like the
 * reference (step = min(N, im2col_step); N % step == 0, cu:46-48), but does not
 * change the launch: there is no `columns` staging buffer here.
 */
#ifndef KINET_MSDA_H_
#define KINET_MSDA_H_

#include "kinet_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* replaces ms_deform_attn_cuda_forward (ms_deform_attn_cuda.cu:19-86) */
int kinet_msda_forward(const void* value, const int64_t* spatial_shapes,
                       const void* sampling_loc, const void* attn_weight, void* output,
                       int batch, int spatial_size, int num_heads, int channels,
                       int num_levels, int num_query, int num_point, int im2col_step,
                       int value_dtype, int loc_dtype, kinet_stream_t stream);

/* replaces ms_deform_attn_cuda_backward (ms_deform_attn_cuda.cu:89-168).
 * grad_value (N,S,M,D) value_dtype, grad_loc (N,Lq,M,L,P,2) and grad_attw (N,Lq,M,L,P)
 * loc_dtype; all three are fully overwritten (the reference zero-fills, cu:119-121).
 * For BF16/F16 value, `workspace` must hold N*S*M*D floats (f32 accumulation of
 * grad_value); it may be NULL for F32/F64.  kinet_msda_backward_workspace_bytes()
 * returns the required size. */
int kinet_msda_backward(const void* value, const int64_t* spatial_shapes,
                        const void* sampling_loc, const void* attn_weight,
                        const void* grad_output, void* grad_value, void* grad_loc,
                        void* grad_attw, void* workspace,
                        int batch, int spatial_size, int num_heads, int channels,
                        int num_levels, int num_query, int num_point, int im2col_step,
                        int value_dtype, int loc_dtype, kinet_stream_t stream);

int64_t kinet_msda_backward_workspace_bytes(int batch, int spatial_size, int num_heads,
                                            int channels, int value_dtype);

/* Tuning hook for kinet_msda_backward on the CALLING thread (no reference counterpart).
 * Encoder calls (num_query == spatial_size) sum grad_value on chip: one workgroup per
 * (image, head) walks passes of consecutive queries and adds each value row the pass touches
 * to global memory once.  0 = automatic for every field; mode -1 always selects the
 * one-atomic-per-corner kernel, mode 1 the on-chip-sum kernel for any call, mode 2 the
 * on-chip-sum kernel with queries in index order instead of 8-pixel-wide blocks (A/B, tests),
 * mode 3 the on-chip-sum kernel with four samples' corner loads in flight instead of two;
 * log2_rows = pixel hash size, queries_per_pass (0 = threads / 16). */
void kinet_msda_backward_tune(int mode, int log2_rows, int queries_per_block, int threads,
                              int queries_per_pass);

/* Timing-only phase knobs of the on-chip-sum backward kernel on the CALLING thread (results
 * are wrong while set; tools/msda_bwd_probe.py --phases): 1 = skip the value-corner loads of
 * the location / weight gradients, 2 = skip the per-row global atomics, 4 = skip the row-sum
 * phase, 8 = skip the pixel-hash inserts.  Returns the previous flags. */
int kinet_msda_backward_debug(int flags);

/* Fused module path (MSDeformAttn.forward, ms_deform_attn.py:49-88): computes
 *   attw = softmax over L*P of logits            (ms_deform_attn.py:70-71)
 *   attw = 0 where query_attn_mask               (:73-74, optional, uint8 (N,Lq))
 *   loc  = ref + off / shapes[(H,W)]   (2-d refs, x divided by H: reference quirk :77-79)
 *   loc  = ref_xy + off / P * ref_wh * 0.5       (4-d refs, :80-82)
 * and samples, without materialising loc/attw in HBM.
 *   offsets_logits  (N, Lq, ld_off) f32 rows holding [M*L*P*2 offsets | M*L*P logits]
 *                   (the concatenated sampling_offsets/attention_weights projection)
 *   ref_points      (N, Lq, L, ref_dim) f32, ref_dim in {2, 4}
 *   value element (b, s, m, c) at value[b*value_sb + s*value_ss + m*value_sm + c]
 *                   (elements; all three 0 = row-major (N, S, M, D)).  kinet_amd feeds the
 *                   head-major layout (M, N, S, D) written by kinet_gemm_headmajor, so a
 *                   wave's gathers for neighbouring queries of one head are contiguous.
 * Launch: one head per wave, 64/(D/vec) consecutive queries per wave.
 * Writes output (N, Lq, M*D) in output_dtype and, when loc_out/attw_out are non-NULL, the
 * f32 sampling_loc / attn_weight tensors (needed to run kinet_msda_backward).
 * output_dtype = value_dtype, or KINET_BF16 from KINET_F16 values (f16 values are gathered
 * and accumulated by mixed f16 x f32 FMAs; head_dim 32, L*P in {16, 32} only).
 * offlog_dtype: KINET_F32, or KINET_F16 with 16-bit values (same restrictions).
 * query_tile_order: optional (NULL = natural order) permutation of the ceil(num_query / 16)
 *                 16-query tiles giving the order the specialised kernels process them in
 *                 (outputs unchanged); the encoder passes its tiles sorted by image row across
 *                 levels so the value rows they share are fetched into L2 once.
 * (Encoder-sized calls with their level shapes on the host are faster through
 * kinet_msda_encoder_forward, below.) */
int kinet_msda_fused_forward(const void* value, int64_t value_sb, int64_t value_ss, int64_t value_sm,
                             const int64_t* spatial_shapes,
                             const void* offsets_logits, int ld_off,
                             const float* ref_points, int ref_dim,
                             const uint8_t* query_attn_mask,
                             void* output, float* loc_out, float* attw_out,
                             int batch, int spatial_size, int num_heads, int channels,
                             int num_levels, int num_query, int num_point,
                             int value_dtype, int output_dtype, int offlog_dtype,
                             const int32_t* query_tile_order, kinet_stream_t stream);

/* Encoder-sized fused sampling (the encoder's MSDeformAttn.forward, ms_deform_attn.py:69-87)
 * with the offsets / logits projection in HEAD-MAJOR layout:
 *   offsets_logits_hm  (M, N, Lq, L*P*3) f16: per (head, frame, query) [L*P*2 offsets in
 *                      (l, p, xy) order | L*P logits in (l, p) order] -- the sampling_offsets /
 *                      attention_weights rows of one head interleaved (kinet_amd.msda packs the
 *                      weight rows so kinet_gemm_headmajor_ex writes it directly)
 *   spatial_shapes_host (L, 2) int64 (H, W) in HOST memory (the launch plan -- which levels are
 *                      staged in LDS, how many strips -- is chosen from it; KINET_ERR_ARG when no
 *                      plan fits: use kinet_msda_fused_forward)
 *   value              f16 head-major: (b, s, m, c) at value[b*value_sb + m*value_sm + s*32 + c]
 *   ref_points, query_attn_mask, output, query_tile_order as kinet_msda_fused_forward
 *   (output (N, Lq, M*32) bf16 or f16).
 * Same semantics as kinet_msda_fused_forward (softmax over L*P, the reference's 2-d offset
 * normaliser quirk, 4-d refs, query mask); head_dim 32, L = 4, P = 4.  Each level's 16 taps
 * are summed as f16 pairs before the f32 sum.  One workgroup per CU owns one horizontal strip
 * (a contiguous range of query_tile_order) of one (frame, head) map, with the rows of the
 * coarser levels that strip samples staged in LDS; samples outside the staged rows are
 * gathered from the map (msda_enc.hip).  query_tile_order should be the row-sorted order
 * (any order gives the same output; the sorted one keeps the staged rows hit). */
int kinet_msda_encoder_forward(const void* value, int64_t value_sb, int64_t value_sm,
                               const int64_t* spatial_shapes_host, const void* offsets_logits_hm,
                               const float* ref_points, int ref_dim, const uint8_t* query_attn_mask,
                               void* output, int batch, int spatial_size, int num_heads, int channels,
                               int num_levels, int num_query, int num_point, int output_dtype,
                               const int32_t* query_tile_order, kinet_stream_t stream);

/* The launch plan kinet_msda_encoder_forward would use for these level shapes (host only, no
 * GPU call): plan_out[0] = levels gathered from HBM (the finest ones), [1] = strips per head
 * map, [2] = LDS map pixels used, [3] = workgroups.  KINET_ERR_ARG when no plan fits (the
 * caller then uses kinet_msda_fused_forward). */
int kinet_msda_encoder_plan(const int64_t* spatial_shapes_host, int batch, int num_heads, int num_query,
                            int32_t* plan_out);

/* The encoder call's sampling_offsets | attention_weights projection (ms_deform_attn.py:68-69,
 * one GEMM over query [+ query_add] rows, K = 256) with the rest of the MSDA preparation in its
 * epilogue -- softmax over the head's L*P logits (:70-71), query_attn_mask (:73-74), sampling
 * locations from the reference points (:76-82) and the bilinear setup of
 * ms_deform_im2col_cuda.cuh:227-233 -- written as head-major SAMPLING RECORDS
 * (num_heads, M, 96 bytes) for kinet_msda_encoder_forward_records:
 *   bytes [16 l, 16 l + 16): level l's 4 locations, u32 fixed point
 *       (hl << (16 + fb)) | (round(lh * 2^fb) << 16) | (wl << fb) | round(lw * 2^fb)
 *       of the top-left corner (hl, wl) and the fractions (lh, lw) in level pixels;
 *   bytes [64 + 8 l, 72 + 8 l): level l's 4 attention weights, f16.
 * Corner rows / columns outside the level are folded into the weight (a footprint whose top row
 * is -1 becomes row 0 with weight a*lh and lh = 0, a bottom row H-1 keeps weight a*(1-lh) and
 * lh = 0; the same for columns), a sample outside the level has weight 0.
 * W: (num_heads*48, K) weight rows grouped (head, level, [x0 y0 .. x3 y3 | logit0 .. logit3]);
 * bias likewise (f32).  A (M, K) rows of stride lda, A2 (optional) added at load (query_pos);
 * a2_rows as kinet_gemm_headmajor_ex (0, or A2 of a2_rows rows shared by every frame).
 * ref_points (M, 4, ref_dim) f32, query_attn_mask (M) bytes or NULL, spatial_shapes_host 4 x
 * (H, W) on the host, each <= 2^(16 - frac_bits); frac_bits in [6, 10]; num_heads % 4 == 0.
 * Replaces the offsets / attention-weight nn.Linear + F.softmax + location arithmetic of
 * ms_deform_attn.py:68-82 (the reference's sampling_locations / attention_weights tensors). */
int kinet_msda_sample_records(const void* A, const void* A2, const void* W, const float* bias, int M,
                              int num_heads, int K, int lda, int in_dtype, const float* ref_points,
                              int ref_dim, const uint8_t* query_attn_mask, const int64_t* spatial_shapes_host,
                              int num_levels, int num_point, int frac_bits, void* records, int a2_rows,
                              kinet_stream_t stream);

/* kinet_msda_encoder_forward fed by sampling records (kinet_msda_sample_records) instead of
 * f16 offsets / logits + reference points: the sampling kernel's phase 1 is only the fixed-point
 * unpack, four packed-f16 weight products and the address choice.  records: (num_heads, batch,
 * num_query) x 96 bytes; the other arguments as kinet_msda_encoder_forward. */
int kinet_msda_encoder_forward_records(const void* value, int64_t value_sb, int64_t value_sm,
                                       const int64_t* spatial_shapes_host, const void* records, int frac_bits,
                                       void* output, int batch, int spatial_size, int num_heads, int channels,
                                       int num_levels, int num_query, int num_point, int output_dtype,
                                       const int32_t* query_tile_order, kinet_stream_t stream);

/* Which kernel the calling thread's last kinet_msda_backward launched: 1 = msda_bwd_list_kernel
 * (grad_value rows summed on chip), 0 = msda_bwd_kernel (per-corner atomics), -1 = none (an
 * empty call, or no call yet).  Host-side bookkeeping for the rooflines; no GPU call. */
int kinet_msda_backward_last_kernel(void);

/* Head_dim-36 encoder calls (configs 3-5, d = 288: cfgs/train_multi_frame.yaml:2) on the strip
 * kernel: the value in TWO head-major planes written by kinet_gemm_headmajor_split --
 * value_main (M, N, S, 32) f16 (channels 0-31 of each head; strides as value_sb / value_sm of
 * kinet_msda_encoder_forward) and value_tail (M, N, S, 4) f16 (channels 32-35, 8 bytes per
 * pixel; tail_sb / tail_sm in elements) -- so the 32-channel part runs the D = 32 sampling
 * unchanged and each quad of lanes adds the 4 tail channels (one 8-byte corner read per lane
 * per sample, tail map staged in LDS beside the main map).  channels must be 36; offsets /
 * logits head-major as kinet_msda_encoder_forward; output (N, Lq, M*36).  Same sampling as
 * ms_deform_im2col_cuda.cuh:165-237 for any channel count. */
int kinet_msda_encoder_forward_split(const void* value_main, int64_t main_sb, int64_t main_sm,
                                     const void* value_tail, int64_t tail_sb, int64_t tail_sm,
                                     const int64_t* spatial_shapes_host, const void* offsets_logits_hm,
                                     const float* ref_points, int ref_dim, const uint8_t* query_attn_mask,
                                     void* output, int batch, int spatial_size, int num_heads, int channels,
                                     int num_levels, int num_query, int num_point, int output_dtype,
                                     const int32_t* query_tile_order, kinet_stream_t stream);

/* Strips per head map for the calling thread's encoder launches (0 = the plan's own choice; a
 * count is used when it fits the LDS map, else the plan's choice).  Returns the previous value;
 * KINET_ERR_ARG outside [0, 64].  Tuning / A/B only: any strip count gives the same output. */
int kinet_msda_encoder_set_strips(int strips);

/* kinet_msda_encoder_plan for head_dim `channels` (32, or 36: the split kernel, whose LDS map
 * holds 72 bytes per staged pixel). */
int kinet_msda_encoder_plan_ex(const int64_t* spatial_shapes_host, int batch, int num_heads, int num_query,
                               int channels, int32_t* plan_out);

#ifdef __cplusplus
}
#endif

#endif /* KINET_MSDA_H_ */
