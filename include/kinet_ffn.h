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

/* ResNet bottleneck pair (torchvision Bottleneck as the reference instantiates it,
 * backbone.py:94-108): block i's conv3 + FrozenBN + residual + ReLU and the next block's conv1 +
 * FrozenBN + ReLU, both 1x1 stride 1 over NHWC rows, in ONE launch (phase A = conv3, its
 * rounded output chunk is stored to Y and is phase B's operand; phase B = the next conv1):
 *   Y = relu(X (s3 W3)^T + b3 + R)   (M, F)   -- the block output, the next block's residual
 *   T = relu(Y (s1 W1)^T + b1)       (M, DB)  -- the next block's conv1 output
 * kinet_bottleneck_pack: f32 W3 (F, D), W1 (DB, F), FrozenBN scales s3 (F), s1 (DB) -> the FFN
 * fragment stream ((D + DB) * F elements of dtype) with each weight row scaled before rounding.
 * F = 4 D, D in {64, 128, 256}; DB = D (inside a stage) or, at D = 64, DB = 128 (stage 1's last
 * block -> stage 2's first conv1, which is stride 1 in torchvision's v1.5 Bottleneck); X rows of
 * stride ldx; R, Y, T dense rows; b3 (F), b1 (DB) f32; dtype KINET_BF16 / KINET_F16. */
int kinet_bottleneck_pack(const float* W3, const float* W1, const float* s3, const float* s1,
                          void* packed, int D, int F, int DB, int dtype, kinet_stream_t stream);

int kinet_bottleneck_pair(const void* X, int ldx, const void* R, const void* packed, const float* b3,
                          const float* b1, void* Y, void* T, int M, int D, int F, int DB, int dtype,
                          kinet_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* KINET_FFN_H_ */
