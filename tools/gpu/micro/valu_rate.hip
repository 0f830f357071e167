// VALU issue-rate microbenchmark: cycles per wave64 instruction per SIMD for
// the operand patterns the FFT code uses (2 or 3 VGPR sources vs SGPR
// sources), at 1, 2, 3 and 4 waves per SIMD (one workgroup per CU, pinned by
// its LDS allocation).  Clock: s_memtime around the timed loop, per wave.
//   hipcc --offload-arch=gfx950 -O3 tools/gpu/micro/valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 16;  // independent chains per lane

template <int KIND>
__global__ void k_rate(float *out, unsigned long long *cyc, int iters, float s0, float s1) {
    extern __shared__ float pin[];  // sized so one block fits per CU
    float a[N], b[N], c[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        a[i] = threadIdx.x * 1e-3f + i;
        b[i] = 1.0f + i * 1e-4f + threadIdx.x * 1e-7f;
        c[i] = 1e-3f * i;
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (KIND == 0) a[i] = __builtin_fmaf(a[i], s0, s1);      // 1 VGPR source
            if (KIND == 1) a[i] = a[i] + b[i];                       // 2 VGPR sources (v_add)
            if (KIND == 2) a[i] = __builtin_fmaf(a[i], b[i], c[i]);  // 3 VGPR sources (v_fma)
            if (KIND == 3) a[i] = a[i] * b[i];                       // 2 VGPR sources (v_mul)
            if (KIND == 4) {                                         // add/sub butterfly pairs
                const float x = a[i], y = b[i];
                a[i] = x + y;
                b[i] = x - y;
            }
        }
        if (KIND == 1 || KIND == 3) {
#pragma unroll
            for (int i = 0; i < N; ++i) asm volatile("" : "+v"(b[i]));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float t = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) t += a[i] + b[i] + c[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
    (void)pin;
}

typedef float v2f __attribute__((ext_vector_type(2)));
// packed FP32: KIND 10 v_pk_add_f32, 11 v_pk_fma_f32, 12 add/sub butterfly pairs, 13 complex multiply
template <int KIND>
__global__ void k_rate_pk(float *out, unsigned long long *cyc, int iters, float s0, float s1) {
    extern __shared__ float pin[];
    v2f a[N], b[N], c[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        a[i] = (v2f){threadIdx.x * 1e-3f + i, 0.5f * i};
        b[i] = (v2f){1.0f + i * 1e-4f, 1.0f - threadIdx.x * 1e-7f};
        c[i] = (v2f){1e-3f * i, 2e-3f};
    }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (KIND == 10) a[i] = a[i] + b[i];
            if (KIND == 11) a[i] = __builtin_elementwise_fma(a[i], b[i], c[i]);
            if (KIND == 12) {
                const v2f x = a[i], y = b[i];
                a[i] = x + y;
                b[i] = x - y;
            }
            if (KIND == 13) {  // a *= b (complex)
                const v2f x = a[i], w = b[i];
                v2f r = x.xx * w;
                a[i] = __builtin_elementwise_fma(x.yy, (v2f){-w.y, w.x}, r);
            }
        }
        if (KIND == 10 || KIND == 13) {
#pragma unroll
            for (int i = 0; i < N; ++i) asm volatile("" : "+v"(b[i]));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    v2f t = a[0];
#pragma unroll
    for (int i = 1; i < N; ++i) t += a[i] + b[i] + c[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y;
    if ((threadIdx.x & 63) == 0) atomicAdd(cyc, t1 - t0);
    (void)pin;
}

template <int KIND>
void run_pk(const char *name, float *out, unsigned long long *cyc, int nt) {
    const int iters = 4096, nblk = 256;
    const int ops = (KIND == 12 || KIND == 13 ? 2 : 1) * N * iters;  // packed instructions
    hipFuncSetAttribute((const void *)k_rate_pk<KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
    hipMemset(cyc, 0, sizeof(unsigned long long));
    hipLaunchKernelGGL(k_rate_pk<KIND>, dim3(nblk), dim3(nt), 100 * 1024, 0, out, cyc, iters, 1.0001f, 1e-4f);
    unsigned long long h = 0;
    hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    const int waves = nblk * nt / 64, wps = nt / 256;
    const double cpw = (double)h / waves;
    printf("%-28s waves/SIMD %d  cycles/pk-instr per wave %6.2f  per SIMD %5.2f  per f32 op %5.2f\n", name, wps,
           cpw / ops, cpw / ops / wps, cpw / ops / wps / 2);
}

template <int KIND>
void run(const char *name, float *out, unsigned long long *cyc, int nt) {
    const int iters = 4096, nblk = 256;
    const int ops = (KIND == 4 ? 2 : 1) * N * iters;
    hipMemset(cyc, 0, sizeof(unsigned long long));
    hipLaunchKernelGGL(k_rate<KIND>, dim3(nblk), dim3(nt), 100 * 1024, 0, out, cyc, iters, 1.0001f, 1e-4f);
    unsigned long long h = 0;
    hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    const int waves = nblk * nt / 64, wps = nt / 256;
    const double cpw = (double)h / waves;  // cycles per wave
    printf("%-28s waves/SIMD %d  cycles/instr per wave %6.2f  per SIMD %5.2f\n", name, wps, cpw / ops,
           cpw / ops / wps);
}

int main() {
    float *out;
    unsigned long long *cyc;
    hipMalloc(&out, 256 * 1024 * sizeof(float));
    hipMalloc(&cyc, sizeof(unsigned long long));
    hipFuncSetAttribute((const void *)k_rate<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
    hipFuncSetAttribute((const void *)k_rate<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
    hipFuncSetAttribute((const void *)k_rate<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
    hipFuncSetAttribute((const void *)k_rate<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
    hipFuncSetAttribute((const void *)k_rate<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024);
    for (int nt : {256, 512, 768, 1024}) {
        run<0>("fma 1 vgpr src", out, cyc, nt);
        run<1>("add 2 vgpr src", out, cyc, nt);
        run<3>("mul 2 vgpr src", out, cyc, nt);
        run<2>("fma 3 vgpr src", out, cyc, nt);
        run<4>("add/sub butterfly", out, cyc, nt);
        run_pk<10>("pk_add", out, cyc, nt);
        run_pk<11>("pk_fma", out, cyc, nt);
        run_pk<12>("pk add/sub butterfly", out, cyc, nt);
        run_pk<13>("pk complex mul", out, cyc, nt);
    }
    return 0;
}
