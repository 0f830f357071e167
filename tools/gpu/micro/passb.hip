// Pass-B microbenchmark of the Np 256 fused kernel (timing only, the data is
// synthetic): the column loop of k_fused_iteration (column IDFT from the six
// half-T slots, amplitude replacement, column DFT, six slots back) for one
// workgroup per CU, with the workgroup size, exchange-tile scheme, twiddle
// placement, measurement prefetch and the number of registers held live
// across the loop (the real kernel's P and F) as template parameters.
// Question answered: how fast does pass B run at 3 or 4 waves per SIMD?
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 \
//       -I fpm-opencv_amd/csrc tools/gpu/micro/passb.hip -o passb && ./passb
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "fused256.hpp"

using namespace fpm;

namespace {
constexpr int SKm[6] = {0, 1, 2, 13, 14, 15};
constexpr int TH = 128, TLD = 129, NROWS = 67, NLED = 16;

__device__ __forceinline__ uint4 ldnt(const uint4 *p) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 v = __builtin_nontemporal_load((const u4 *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

template <int NT, bool HALF>
constexpr size_t lds_bytes() {
    return (size_t)((NT / 16) * (HALF ? 8 * XP : XTILE) + (NROWS + 2) * TLD + 256) * sizeof(float2);
}

template <int NT, bool HALF, bool TWREG, bool PREF, int LIVE, bool MEAS = true>
__global__ void __launch_bounds__(NT, 1) k_passb(const float *__restrict__ meas, float2 *out, int nrep,
                                                 unsigned long long *cyc) {
    constexpr int NG = NT / 16;
    constexpr int XT = HALF ? 8 * XP : XTILE;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2 *scr_all = sm, *th = sm + NG * XT, *tw2 = th + (NROWS + 2) * TLD;
    const int tid = threadIdx.x, g = tid >> 4, t = tid & 15;
    float2 *scr = scr_all + g * XT;
    const int xrd = HALF ? opaque_int((t & 7) * XP) : exch_rbase(t);
    for (int i = tid; i < 256; i += NT) {
        float s, c;
        sincosf(-6.283185307f * (float)(((i >> 4) * (i & 15)) & 255) / 256.f, &s, &c);
        tw2[i] = make_float2(c, s);
    }
    for (int i = tid; i < (NROWS + 2) * TLD; i += NT) th[i] = make_float2(__sinf(i * 0.37f), __cosf(i * 0.11f));
    float2 live[LIVE > 0 ? LIVE : 1];
#pragma unroll
    for (int k = 0; k < LIVE; ++k) live[k] = out[(size_t)(blockIdx.x * NT + tid) * 32 + k];
    int roff[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) roff[s] = ((t + 16 * SKm[s]) % NROWS) * TLD;
    const int zoff = NROWS * TLD;
    __syncthreads();
    float2 v[16], r[16];
    const float epsn = 1e-3f, epsn_im = 1e-3f;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < nrep; ++rep) {
        const float *Ib = meas + ((size_t)(rep % NLED) * gridDim.x + blockIdx.x) * 65536;
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {
            Tw<TWREG> wt;
            wt.load(tw2, t);
            auto ldI = [&](int xl, uint4 (&n)[4]) {
                const uint4 *ip = (const uint4 *)(Ib + ((xl + TH * h) * 16 + t) * 16);
                if (MEAS) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) n[i] = ldnt(ip + i);
                } else {
                    const unsigned u = 0x3f800000u + (unsigned)(xl & 7);
                    for (int i = 0; i < 4; ++i) n[i] = make_uint4(u, u + 1, u + 2, u + 3);
                }
            };
            uint4 nI[4];
            float2 tin[6];
            if (PREF) {
                ldI(g, nI);
#pragma unroll
                for (int s = 0; s < 6; ++s) tin[s] = th[roff[s] + g];
            }
#pragma unroll 1
            for (int xl = g; xl < TH; xl += NG) {
                uint4 cI[4];
                const int xn = xl + NG < TH ? xl + NG : xl;
                if (PREF) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) cI[i] = nI[i];
                    ldI(xn, nI);
                } else {
                    ldI(xl, cI);
#pragma unroll
                    for (int s = 0; s < 6; ++s) tin[s] = th[roff[s] + xl];
                }
#pragma unroll
                for (int k = 0; k < 16; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
                for (int s = 0; s < 6; ++s) v[SKm[s]] = tin[s];
                idft256_in6<HALF>(v, r, scr, wt, t, xrd);
                if (PREF) {
#pragma unroll
                    for (int s = 0; s < 6; ++s) tin[s] = th[roff[s] + xn];
                }
                const unsigned iw[16] = {cI[0].x, cI[0].y, cI[0].z, cI[0].w, cI[1].x, cI[1].y, cI[1].z, cI[1].w,
                                         cI[2].x, cI[2].y, cI[2].z, cI[2].w, cI[3].x, cI[3].y, cI[3].z, cI[3].w};
#pragma unroll
                for (int m2 = 0; m2 < 16; ++m2) {
                    const float invI = __uint_as_float(iw[m2]);
                    const float tre = r[m2].x + epsn, tim = r[m2].y + epsn_im;
                    const float mag2 = __builtin_fmaf(tre, tre, tim * tim);
                    const float sc = __builtin_amdgcn_rsqf(mag2 * invI);
                    v[m2] = make_float2(r[m2].x * sc, r[m2].y * sc);
                }
                float2 o[6];
                dft256_out6<HALF>(v, o, scr, wt, t, xrd);
#pragma unroll
                for (int s = 0; s < 6; ++s) th[roff[s] + (roff[s] == zoff ? TLD : 0) + xl] = o[s];
            }
            __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < LIVE; ++k) live[k] = cadd(live[k], th[(k * 7 + tid) % (NROWS * TLD)]);
    }
    if (tid == 0) atomicAdd(cyc, __builtin_amdgcn_s_memtime() - c0);
    float2 acc = v[0];
#pragma unroll
    for (int k = 0; k < LIVE; ++k) acc = cadd(acc, live[k]);
    out[(size_t)(blockIdx.x * NT + tid) * 32] = acc;
}

template <int NT, bool HALF, bool TWREG, bool PREF, int LIVE, bool MEAS = true>
void run(const char *name, const float *meas, float2 *out, int nblk, int nrep, unsigned long long *cyc) {
    auto fn = k_passb<NT, HALF, TWREG, PREF, LIVE, MEAS>;
    const size_t lds = lds_bytes<NT, HALF>();
    if (hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
        printf("%s: LDS %zu rejected\n", name, lds);
        return;
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(fn, dim3(nblk), dim3(NT), lds, 0, meas, out, 20, cyc);
    hipDeviceSynchronize();
    hipMemset(cyc, 0, 8);
    hipEventRecord(e0);
    hipLaunchKernelGGL(fn, dim3(nblk), dim3(NT), lds, 0, meas, out, nrep, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const hipError_t err = hipGetLastError();
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-36s NT %4d LDS %6zu B  pass B per LED %7.2f us %7.0f cycles  (%s)\n", name, NT, lds, 1e3 * ms / nrep,
           (double)c / nblk / nrep, hipGetErrorString(err));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}
}  // namespace

int main() {
    const int nblk = 256, nrep = 400;
    unsigned long long *cyc;
    hipMalloc(&cyc, 8);
    float *meas;
    float2 *out;
    const size_t nm = (size_t)NLED * nblk * 65536;
    if (hipMalloc(&meas, nm * sizeof(float)) != hipSuccess || hipMalloc(&out, (size_t)nblk * 1024 * 32 * sizeof(float2)) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    std::vector<float> h(1 << 20);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0f / (1.0f + (float)(i % 977));
    for (size_t o = 0; o < nm; o += h.size()) hipMemcpy(meas + o, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice);
    hipMemset(out, 0, (size_t)nblk * 1024 * 32 * sizeof(float2));
    run<512, false, true, false, 24>("warmup", meas, out, nblk, nrep, cyc);
    run<512, false, true, false, 24>("512 full-tile tw-reg live24", meas, out, nblk, nrep, cyc);
    run<512, false, true, false, 24, false>("512 full-tile tw-reg live24 NOMEAS", meas, out, nblk, nrep, cyc);
    run<768, true, false, false, 24, false>("768 half-tile tw-lds live24 NOMEAS", meas, out, nblk, nrep, cyc);
    run<768, true, true, false, 12, false>("768 half-tile tw-reg live12 NOMEAS", meas, out, nblk, nrep, cyc);
    run<1024, true, false, false, 12, false>("1024 half-tile tw-lds live12 NOMEAS", meas, out, nblk, nrep, cyc);
    run<1024, true, false, false, 0, false>("1024 half-tile tw-lds live0 NOMEAS", meas, out, nblk, nrep, cyc);
    run<768, true, true, false, 12>("768 half-tile tw-reg live12", meas, out, nblk, nrep, cyc);
    run<1024, true, false, false, 12>("1024 half-tile tw-lds live12", meas, out, nblk, nrep, cyc);
    hipFree(meas);
    hipFree(out);
    return 0;
}
