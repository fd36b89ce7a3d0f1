/* kinet_amd C-ABI: shared types.
 *
 * Every entry point takes raw device pointers + sizes + a hipStream_t, launches
 * asynchronously on that stream (the caller's current stream, as the reference
 * launcher does with at::cuda::getCurrentCUDAStream(), ms_deform_attn_cuda.cu:70),
 * never allocates, never synchronises, and returns a status code.  A non-zero
 * status leaves a message readable through kinet_last_error() (thread-local); the
 * Python shim raises it as RuntimeError, mirroring AT_ASSERTM -> c10::Error in the
 * reference (ms_deform_attn_cuda.cu:29-34, :48).
 */
#ifndef KINET_COMMON_H_
#define KINET_COMMON_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* kinet_stream_t; /* == hipStream_t */

enum kinet_dtype {
    KINET_F32 = 0,
    KINET_BF16 = 1,
    KINET_F16 = 2,
    KINET_F64 = 3,
    /* f32 storage, products computed as three bf16 MFMA passes (hi*hi + hi*lo + lo*hi of the
     * split x = hi + lo; ~2^-17 relative error per product, f32 accumulation) -- torch's
     * "high" float32 matmul precision.  Accepted as the input dtype of the GEMM / convolution
     * entry points (kinet_gemm.h) and kinet_gemm_tn; outputs are f32. */
    KINET_F32_X3 = 4,
};

enum kinet_status {
    KINET_OK = 0,
    KINET_ERR_ARG = 1,   /* invalid argument / unsupported shape or dtype */
    KINET_ERR_HIP = 2,   /* HIP runtime error at launch */
};

/* Text of the last error raised on this host thread ("" if none). */
const char* kinet_last_error(void);

/* Library build identifier: "kinet_amd <version> gfx950 src <hash>", where <hash> is the
 * sha256 prefix of the kernel sources + headers it was compiled from (kinet_amd/build.py). */
const char* kinet_version(void);

#ifdef __cplusplus
}
#endif

#endif /* KINET_COMMON_H_ */
