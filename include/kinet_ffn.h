/* kinet_amd C-ABI: fused transformer FFN sub-layer (linear1 -> ReLU -> linear2 -> +residual
 * -> LayerNorm) in ONE launch, the hidden activations never leave the CU.
 *
 * Replaces, on the detection hot path, the post-norm FFN of the deformable encoder and
 * decoder layers:
 *   DeformableTransformerEncoderLayer.forward_ffn  (deformable_transformer.py:284-288)
 *   DeformableTransformerDecoderLayer.forward_ffn  (deformable_transformer.py:361-365)
 *     y = LayerNorm( x + linear2( relu( linear1(x) ) ) )
 * which the reference runs as two cuBLAS GEMMs + elementwise ops with the (M, F) hidden
 * tensor round-tripping through HBM.
 *
 * Weights are packed once (kinet_ffn_pack) from the PyTorch layouts W1 (F, D), W2 (D, F)
 * into a fragment-major stream: for each 32-unit hidden chunk c, 2*(D/32) 1-KiB fragments
 * of W1 rows [32c, 32c+32) followed by D/16 fragments of W2 columns [32c, 32c+32), each
 * fragment laid out exactly as the 64 lanes of a v_mfma_f32_16x16x32 operand read it, so the
 * kernel moves it with LDS-DMA and reads it conflict-free.  packed size = 2*D*F elements.
 *
 * dtype: KINET_BF16 or KINET_F16 for X, the packed weights and Y (f32 accumulation, the
 * hidden activations rounded to dtype exactly where the unfused GEMM would store them).
 * b1 (F), b2 (D) f32; ln_gamma/ln_beta (D) f32 or both NULL (then y = x + FFN(x)).
 * D in {256, 288}, F % 32 == 0, ldx/ldy multiples of 8, 16-byte aligned X, Y, packed.
 */
#ifndef KINET_FFN_H_
#define KINET_FFN_H_

#include "kinet_common.h"

#ifdef __cplusplus
extern "C" {
#endif

int kinet_ffn_pack(const void* W1, const void* W2, void* packed, int D, int F, int dtype,
                   kinet_stream_t stream);

int kinet_ffn_fused(const void* X, int ldx, const void* packed, const float* b1, const float* b2,
                    const float* ln_gamma, const float* ln_beta, float ln_eps, void* Y, int ldy,
                    int M, int D, int F, int dtype, kinet_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* KINET_FFN_H_ */
