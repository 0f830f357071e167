// Which XCC does each block of a grid land on (s_getreg HW_REG_XCC_ID)?
// Prints the id of blocks 0..31 and the count per id for a 256-block grid,
// for a normal and for a cooperative launch.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_xcc(int *out) {
    int x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    extern __shared__ int pin[];
    if (threadIdx.x == 0) out[blockIdx.x] = x;
    (void)pin;
}

int main() {
    int *d, h[256];
    if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 1;
    for (int coop = 0; coop < 2; ++coop) {
        hipMemset(d, 0xff, 256 * sizeof(int));
        const size_t lds = 140 * 1024;  // one block per CU
        hipFuncSetAttribute((const void *)k_xcc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (coop) {
            void *args[] = {&d};
            hipError_t e = hipLaunchCooperativeKernel((const void *)k_xcc, dim3(256), dim3(512), args, lds, 0);
            printf("cooperative launch: %s\n", hipGetErrorString(e));
        } else {
            hipLaunchKernelGGL(k_xcc, dim3(256), dim3(512), lds, 0, d);
        }
        hipDeviceSynchronize();
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        int cnt[17] = {0};
        for (int i = 0; i < 256; ++i) cnt[(h[i] & 15)]++;
        printf("%s: blocks 0..31:", coop ? "coop" : "normal");
        for (int i = 0; i < 32; ++i) printf(" %d", h[i]);
        printf("\n  per id:");
        for (int i = 0; i < 16; ++i)
            if (cnt[i]) printf(" [%d]=%d", i, cnt[i]);
        int same = 0;
        for (int i = 0; i < 256; ++i)
            if (h[i] == h[(i & ~15) | ((i + 8) & 15)]) ++same;
        printf("\n  blocks k and k^8 (same 16-group) on the same id: %d of 256\n", same);
    }
    return 0;
}
