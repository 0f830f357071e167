// flop_count.hip -- how the SQ_INSTS_VALU_*_F32 counters count packed FP32.
//
// Each kernel issues a known number of one FP32 VALU instruction (inline asm,
// so the compiler cannot change the count): per wave, ITERS x 16 of
//   k_pk_fma  v_pk_fma_f32      k_fma  v_fma_f32
//   k_pk_add  v_pk_add_f32      k_add  v_add_f32
//   k_pk_mul  v_pk_mul_f32      k_mul  v_mul_f32
// Run under `rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32
// SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU ...` and divide each counter by the
// printed expected wave-instruction count: a packed instruction counted once
// means the counter-derived flops (64 lanes x (2 FMA + ADD + MUL)) understate
// the packed kernel's executed flops by 2x (bench.py roofline.counters).
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 1024;
typedef float v2f __attribute__((ext_vector_type(2)));

#define REP16(X) X X X X X X X X X X X X X X X X

__global__ void k_pk_fma(float *out, float s) {
    v2f a = {(float)threadIdx.x, s}, b = {s, 0.5f}, c = {0.25f, s};
    for (int i = 0; i < ITERS; ++i) asm volatile(REP16("v_pk_fma_f32 %0, %0, %1, %2\n") : "+v"(a) : "v"(b), "v"(c));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.x + a.y;
}
__global__ void k_pk_add(float *out, float s) {
    v2f a = {(float)threadIdx.x, s}, b = {s, 0.5f};
    for (int i = 0; i < ITERS; ++i) asm volatile(REP16("v_pk_add_f32 %0, %0, %1\n") : "+v"(a) : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.x + a.y;
}
__global__ void k_pk_mul(float *out, float s) {
    v2f a = {(float)threadIdx.x, s}, b = {s, 0.5f};
    for (int i = 0; i < ITERS; ++i) asm volatile(REP16("v_pk_mul_f32 %0, %0, %1\n") : "+v"(a) : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a.x + a.y;
}
__global__ void k_fma(float *out, float s) {
    float a = (float)threadIdx.x, b = s, c = 0.25f;
    for (int i = 0; i < ITERS; ++i) asm volatile(REP16("v_fma_f32 %0, %0, %1, %2\n") : "+v"(a) : "v"(b), "v"(c));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
__global__ void k_add(float *out, float s) {
    float a = (float)threadIdx.x, b = s;
    for (int i = 0; i < ITERS; ++i) asm volatile(REP16("v_add_f32 %0, %0, %1\n") : "+v"(a) : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
__global__ void k_mul(float *out, float s) {
    float a = (float)threadIdx.x, b = s;
    for (int i = 0; i < ITERS; ++i) asm volatile(REP16("v_mul_f32 %0, %0, %1\n") : "+v"(a) : "v"(b));
    out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

int main() {
    const int blocks = 1024, threads = 256;
    float *d = nullptr;
    if (hipMalloc(&d, sizeof(float) * blocks * threads) != hipSuccess) return 1;
    const long long waves = (long long)blocks * threads / 64;
    const long long per = waves * ITERS * 16;
    hipLaunchKernelGGL(k_pk_fma, dim3(blocks), dim3(threads), 0, 0, d, 1.0001f);
    hipLaunchKernelGGL(k_pk_add, dim3(blocks), dim3(threads), 0, 0, d, 1.0001f);
    hipLaunchKernelGGL(k_pk_mul, dim3(blocks), dim3(threads), 0, 0, d, 1.0001f);
    hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, d, 1.0001f);
    hipLaunchKernelGGL(k_add, dim3(blocks), dim3(threads), 0, 0, d, 1.0001f);
    hipLaunchKernelGGL(k_mul, dim3(blocks), dim3(threads), 0, 0, d, 1.0001f);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("expected wave-instructions per kernel: %lld (each kernel issues only its one instruction)\n", per);
    (void)hipFree(d);
    return 0;
}
