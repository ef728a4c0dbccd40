// hpa_internal.h -- shared by the HIP translation units of libpaged_hip.so.
// gfx950 (CDNA4) only: wave64, fp32 MFMA, no CUDA compatibility layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "hip_paged_attn.h"

// Returns a nonzero status after reporting; exits when HPA_FATAL=1
// (cudaCheck convention, reference train_gpt2.cu:27-34).
int hpa_fail(const char* file, int line, const char* what);
hipStream_t hpa_stream();

#define HPA_CHECK(call)                                                          \
    do {                                                                         \
        hipError_t e_ = (call);                                                  \
        if (e_ != hipSuccess) return hpa_fail(__FILE__, __LINE__, hipGetErrorString(e_)); \
    } while (0)

#define HPA_REQUIRE(cond, msg)                                                   \
    do {                                                                         \
        if (!(cond)) return hpa_fail(__FILE__, __LINE__, msg);                   \
    } while (0)

// checks the launch that was just enqueued
#define HPA_LAUNCH_CHECK() HPA_CHECK(hipGetLastError())

namespace hpa {
constexpr int kWave = 64;

// 16-byte write-through (sc1) store / L1-bypassing (sc1) load at
// base + byte_off (base wave-uniform, byte_off per lane, 16-B aligned): the
// hand-off forms of MI355X_MICROARCH.md "Valid forms" row 1 at full width
// (4-byte sc1 stores are one fabric write each, several times slower per byte)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kCpolSc1 = 16;  // gfx940+ cache policy: SC1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void store_wt16(void* base, int byte_off, float4 v) {
    const u32x4 d = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(d, wt_rsrc(base), byte_off, 0, kCpolSc1);
}
__device__ __forceinline__ float4 load_wt16(const void* base, int byte_off) {
    const u32x4 d = __builtin_amdgcn_raw_buffer_load_b128(wt_rsrc(base), byte_off, 0, kCpolSc1);
    return make_float4(__uint_as_float(d.x), __uint_as_float(d.y), __uint_as_float(d.z), __uint_as_float(d.w));
}

// 4-byte forms (one float per lane; a wave's 64 consecutive floats are one
// 256-B write-through burst)
__device__ __forceinline__ void store_wt4(void* base, int byte_off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), wt_rsrc(base), byte_off, 0, kCpolSc1);
}
__device__ __forceinline__ float load_wt4(const void* base, int byte_off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(wt_rsrc(base), byte_off, 0, kCpolSc1));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// "frag" layout of a [rows][K] fp32 matrix (rows padded to 16, K % 16 == 0),
// the operand layout of v_mfma_f32_16x16x4_f32 loaded 16 bytes per lane:
// element (m, k) sits at lane (m%16) + 16*((k%16)/4), float (k%4) of the
// 1 KiB fragment of (16-row block m/16, 16-deep k-step k/16); fragment
// (rb, kb) starts at ((rb * K/16 + kb) * 64) float4s.  A wave loads one
// fragment as one contiguous 1 KiB dwordx4 burst.  Used for streamed weights
// and for every activation that feeds a GEMM.
__device__ __host__ __forceinline__ size_t frag_index(int m, int k, int K) {
    return ((((size_t)(m >> 4) * (size_t)(K >> 4) + (size_t)(k >> 4)) * 64 +
             (size_t)((m & 15) + 16 * ((k >> 2) & 3)))
            << 2) +
           (size_t)(k & 3);
}

// fp32 -> bf16, round to nearest even (finite inputs; the KV pool's storage)
__device__ __host__ __forceinline__ unsigned short f32_to_bf16(float f) {
    unsigned int u;
    __builtin_memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}

// GELU of the reference (paged_infer.c:243-251): 0.5 x (1 + tanh(sqrt(2/pi)(x + 0.044715 x^3)))
__device__ __forceinline__ float gelu_ref(float x) {
    // sqrtf(2.0f / M_PI) as the reference computes it: float(2/pi) then sqrtf
    const float s = __uint_as_float(0x3F4C4229u);  // 0.79788452
    float cube = __fmul_rn(__fmul_rn(__fmul_rn(0.044715f, x), x), x);
    return __fmul_rn(__fmul_rn(0.5f, x), __fadd_rn(1.0f, tanhf(__fmul_rn(s, __fadd_rn(x, cube)))));
}
}  // namespace hpa
