#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
__global__ void kpk(float *out, int iters, float s) {
    v2f a[8]; v2f m = {s, s*0.5f}, c = {0.001f, 0.002f};
    for (int i = 0; i < 8; ++i) a[i] = (v2f){(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_elementwise_fma(a[i], m, c);
    }
    v2f t = a[0]; for (int i = 1; i < 8; ++i) t += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;
}
__global__ void ksc(float *out, int iters, float s) {
    float a[16]; float m = s, c = 0.001f;
    for (int i = 0; i < 16; ++i) a[i] = (float)threadIdx.x + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = __builtin_fmaf(a[i], m, c);
    }
    float t = 0; for (int i = 0; i < 16; ++i) t += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}
// complex multiply-accumulate: packed vs scalar
__global__ void kcpk(float *out, int iters, float s) {
    v2f a[8]; v2f w = {s, 0.3f};
    for (int i = 0; i < 8; ++i) a[i] = (v2f){(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            v2f x = a[i];
            v2f r = x.xx * w;
            r = __builtin_elementwise_fma(x.yy, (v2f){-w.y, w.x}, r);
            a[i] = r;
        }
    }
    v2f t = a[0]; for (int i = 1; i < 8; ++i) t += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;
}
__global__ void kcsc(float *out, int iters, float s) {
    float2 a[8]; float2 w = {s, 0.3f};
    for (int i = 0; i < 8; ++i) a[i] = make_float2((float)threadIdx.x + i, (float)i);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float2 x = a[i];
            a[i] = make_float2(__builtin_fmaf(x.x, w.x, -x.y * w.y), __builtin_fmaf(x.x, w.y, x.y * w.x));
        }
    }
    float t = 0; for (int i = 0; i < 8; ++i) t += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__device__ __forceinline__ v2f cmul_pk(v2f x, v2f w) {
    v2f r;
    asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=&v"(r) : "v"(x), "v"(w));
    return r;
}
__global__ void kcasm(float *out, int iters, float s) {
    v2f a[8]; v2f w = {s, 0.3f};
    for (int i = 0; i < 8; ++i) a[i] = (v2f){(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = cmul_pk(a[i], w);
    }
    v2f t = a[0]; for (int i = 1; i < 8; ++i) t += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;
}
__global__ void kcheck(float *out) {
    v2f x = {1.5f, -2.25f}, w = {0.75f, 3.0f};
    v2f r = cmul_pk(x, w);
    if (threadIdx.x == 0) { out[0] = r.x; out[1] = r.y; }
}
int main() {
    float *o; hipMalloc(&o, 4096 * 256 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 20000; const int nb = 4096;
    auto run = [&](const char *nm, void (*k)(float*,int,float), double flop_per_it) {
        hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, o, 100, 1.0001f);
        hipEventRecord(e0); hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, 0, o, iters, 1.0001f); hipEventRecord(e1);
        hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%s %.3f ms  %.1f TFLOP/s\n", nm, ms, flop_per_it * iters * nb * 256.0 / ms / 1e9);
    };
    run("pk_fma", kpk, 32); run("fma", ksc, 32); run("cmul_pk", kcpk, 8*6); run("cmul_scalar", kcsc, 8*6); run("cmul_asm", kcasm, 8*6);
    hipLaunchKernelGGL(kcheck, dim3(1), dim3(64), 0, 0, o); float h[2]; hipMemcpy(h, o, 8, hipMemcpyDeviceToHost);
    printf("check %g %g expect %g %g\n", h[0], h[1], 1.5*0.75 - (-2.25)*3.0, 1.5*3.0 + (-2.25)*0.75);
    return 0;
}
