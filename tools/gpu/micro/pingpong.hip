// Flag ping-pong between two workgroups of the same XCD (blocks k and k+8):
// cycles per round trip for (a) plain store + sc0 (L2) volatile poll and
// (b) agent-scope sc1 store + sc1 poll, alone and beside 240 streaming blocks.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kAux = (int)(1u | (1u << 31));

template <int MODE>
__global__ void k_pp(int *flags, unsigned long long *cyc, int rounds, const float4 *bg, float *sink, size_t nbg) {
    extern __shared__ int pin[];
    const int b = blockIdx.x;
    if (b >= 16) {  // background streamers
        float acc = 0.f;
        for (size_t i = (size_t)(b - 16) * blockDim.x + threadIdx.x; i < nbg; i += (size_t)(gridDim.x - 16) * blockDim.x) {
            const float4 v = bg[i];
            acc += v.x + v.y + v.z + v.w;
        }
        if (acc == 1234.5f) sink[0] = acc;
        return;
    }
    if (b >= 8 + 4 || (b >= 4 && b < 8)) return;  // pairs (0,8) (1,9) (2,10) (3,11)
    const int pair = b & 3, side = b >= 8;
    int *mine = flags + pair * 2 + side, *other = flags + pair * 2 + 1 - side;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(other, 0, 4, 0x00020000);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 1; i <= rounds; ++i) {
        if (side == 0) {
            if (threadIdx.x == 0) {
                if (MODE == 0) __hip_atomic_store(mine, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else __hip_atomic_store(mine, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                while ((MODE == 0 ? (int)__builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, kAux)
                                  : __hip_atomic_load(other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < i)
                    __builtin_amdgcn_s_sleep(1);
            }
        } else {
            if (threadIdx.x == 0) {
                while ((MODE == 0 ? (int)__builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, kAux)
                                  : __hip_atomic_load(other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < i)
                    __builtin_amdgcn_s_sleep(1);
                if (MODE == 0) __hip_atomic_store(mine, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else __hip_atomic_store(mine, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && side == 0) atomicAdd(cyc, __builtin_amdgcn_s_memtime() - t0);
    (void)pin;
}

template <int MODE>
void run(const char *name, int nblk, const float4 *bg, float *sink, size_t nbg) {
    int *flags;
    unsigned long long *cyc;
    hipMalloc(&flags, 64);
    hipMalloc(&cyc, 8);
    hipMemset(flags, 0, 64);
    hipMemset(cyc, 0, 8);
    const int rounds = 2000;
    hipFuncSetAttribute((const void *)k_pp<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024);
    void *args[] = {&flags, &cyc, (void *)&rounds, &bg, &sink, &nbg};
    hipError_t e = hipLaunchCooperativeKernel((const void *)k_pp<MODE>, dim3(nblk), dim3(512), args, 140 * 1024, 0);
    hipDeviceSynchronize();
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-40s %s: %8.0f cycles per round trip\n", name, hipGetErrorString(e), (double)c / 4 / rounds);
    hipFree(flags);
    hipFree(cyc);
}

int main() {
    const size_t nbg = (size_t)1 << 28;  // 4 GiB of float4
    float4 *bg;
    float *sink;
    if (hipMalloc(&bg, nbg * sizeof(float4)) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipMemset(bg, 0, nbg * sizeof(float4));
    run<0>("plain store + sc0 poll, idle chip", 16, bg, sink, nbg);
    run<1>("sc1 store + sc1 poll, idle chip", 16, bg, sink, nbg);
    run<0>("plain store + sc0 poll, 240 streamers", 256, bg, sink, nbg);
    run<1>("sc1 store + sc1 poll, 240 streamers", 256, bg, sink, nbg);
    return 0;
}
