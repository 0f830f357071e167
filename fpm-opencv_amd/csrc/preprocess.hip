// preprocess.hip -- loadFPMDataset's per-image preprocessing on the device
// (fpmMain.cpp:124-144), for n_patch patches cut from every full frame.
//
// Per frame (one LED image):
//   k_bg_sums      exact uint64 sums of the two Np x Np background windows of
//                  the undivided frame (cv::mean accumulates in double, which
//                  is exact for these integer sums; so is uint64)
//   k_crop_patches bg = clamp((mean1 + mean2)/2, bgThresh) rounded to int16,
//                  then for each patch pixel: crop, optional darkfield divide
//                  (saturate_cast<ushort>(rint(v / m)), round half to even),
//                  saturating subtract of bg -> meas[led][patch][y][x]
// HBM-bound byte work: 2 B read + 2 B written per patch pixel plus 2 x 2 Np^2 B
// of background windows per frame.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fpm {

namespace {

// sums[w] += window w pixels.  grid (np, 2), block 256: one window row per block
__global__ void __launch_bounds__(256) k_bg_sums(const uint16_t *__restrict__ frame, int width, int np, int bk1x,
                                                 int bk1y, int bk2x, int bk2y, unsigned long long *sums) {
    __shared__ unsigned long long part[4];
    const int w = blockIdx.y, y = blockIdx.x;
    const int x0 = w ? bk2x : bk1x, y0 = w ? bk2y : bk1y;
    const uint16_t *row = frame + (size_t)(y0 + y) * width + x0;
    unsigned long long s = 0;
    for (int x = threadIdx.x; x < np; x += 256) s += row[x];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&sums[w], part[0] + part[1] + part[2] + part[3]);
}

__device__ __forceinline__ int bg_value(const unsigned long long *sums, int np, double bg_threshold) {
    const double n2 = (double)np * (double)np;
    double bg = ((double)sums[1] / n2 + (double)sums[0] / n2) / 2;  // (bk2 + bk1) / 2, fpmMain.cpp:136
    if (bg > bg_threshold) bg = bg_threshold;                       // :137-138
    return (int)(int16_t)round(bg);                                 // :140
}

// grid (np, B), block 256: row y of patch b
__global__ void __launch_bounds__(256) k_crop_patches(const uint16_t *__restrict__ frame, int width, int np,
                                                      const int *__restrict__ px0, const int *__restrict__ py0,
                                                      const unsigned long long *__restrict__ sums,
                                                      double bg_threshold, double dark_mult, int darkfield,
                                                      uint16_t *__restrict__ out, int16_t *bg_out) {
    const int y = blockIdx.x, b = blockIdx.y;
    const int bg = bg_value(sums, np, bg_threshold);
    if (y == 0 && b == 0 && threadIdx.x == 0 && bg_out) *bg_out = (int16_t)bg;
    const uint16_t *src = frame + (size_t)(py0[b] + y) * width + px0[b];
    uint16_t *dst = out + ((size_t)b * np + y) * np;
    for (int x = threadIdx.x; x < np; x += 256) {
        int v = src[x];
        if (darkfield) {  // :128-129, saturate_cast rounds to nearest even
            const double q = rint((double)v / dark_mult);
            v = q < 0.0 ? 0 : (q > 65535.0 ? 65535 : (int)q);
        }
        v -= bg;  // :143-144 saturating
        dst[x] = (uint16_t)(v < 0 ? 0 : (v > 65535 ? 65535 : v));
    }
}

}  // namespace

// One frame -> meas slab [B][np][np].  `sums` is 2 device uint64 (zeroed here).
hipError_t launch_preprocess_frame(const uint16_t *frame, int width, int np, int B, const int *px0_dev,
                                   const int *py0_dev, int bk1x, int bk1y, int bk2x, int bk2y, double bg_threshold,
                                   double dark_mult, bool darkfield, unsigned long long *sums, uint16_t *out,
                                   int16_t *bg_out_dev, hipStream_t s) {
    hipError_t e = hipMemsetAsync(sums, 0, 2 * sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bg_sums, dim3(np, 2), dim3(256), 0, s, frame, width, np, bk1x, bk1y, bk2x, bk2y, sums);
    hipLaunchKernelGGL(k_crop_patches, dim3(np, B), dim3(256), 0, s, frame, width, np, px0_dev, py0_dev,
                       (const unsigned long long *)sums, bg_threshold, dark_mult,
                       (darkfield && dark_mult != 1.0) ? 1 : 0, out, bg_out_dev);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------
// In-place measurement layout of the fused paths.  The fused kernels read one
// image column per 16- (Np 256) or 10-lane (Np 200) group, lane t holding the
// pixels y = t + G m (m = 0 .. R-1, R = Np / G) -- one contiguous 2R-byte run
// per lane when the image is stored column-major in that order:
//     stored[x Np + t R + m] = I[t + G m][x]
// The stack keeps its uint16 values (2 B per pixel, the C-ABI layout's size):
// each block stages one whole image in LDS (Np^2 x 2 B <= 128 KiB), then writes
// it back permuted over itself.  FWD: C-ABI row-major -> fused; !FWD: back.
namespace {
template <int NP, int G, bool FWD>
__global__ void __launch_bounds__(1024) k_meas_layout(uint16_t *meas, size_t nimg) {
    extern __shared__ uint16_t tl[];  // NP x LD
    constexpr int R = NP / G, LD = NP + 2;
    const size_t img = blockIdx.x;
    if (img >= nimg) return;
    uint16_t *p = meas + img * NP * NP;
    for (int i = threadIdx.x; i < NP * NP; i += 1024) {
        const int a = i / NP, b = i - a * NP;  // FWD: (y, x); !FWD: (x, j)
        tl[a * LD + b] = p[i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NP * NP; i += 1024) {
        const int a = i / NP, b = i - a * NP;
        uint16_t v;
        if (FWD) {  // destination (x = a, j = b), j = t R + m
            const int t = b / R, m = b - t * R;
            v = tl[(t + G * m) * LD + a];
        } else {    // destination (y = a, x = b)
            const int t = a % G, m = a / G;
            v = tl[b * LD + t * R + m];
        }
        p[i] = v;
    }
}

template <int NP, int G>
hipError_t launch_layout(uint16_t *meas, size_t nimg, bool fwd, hipStream_t s) {
    const size_t lds = (size_t)NP * (NP + 2) * sizeof(uint16_t);
    const void *fn = fwd ? (const void *)k_meas_layout<NP, G, true> : (const void *)k_meas_layout<NP, G, false>;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (nimg == 0) return hipSuccess;
    if (fwd)
        hipLaunchKernelGGL((k_meas_layout<NP, G, true>), dim3((unsigned)nimg), dim3(1024), lds, s, meas, nimg);
    else
        hipLaunchKernelGGL((k_meas_layout<NP, G, false>), dim3((unsigned)nimg), dim3(1024), lds, s, meas, nimg);
    return hipGetLastError();
}
// g = Np (small-patch fused kernel, any Np <= 128): the plain transpose
// stored[x Np + y] = I[y][x], its own inverse
__global__ void __launch_bounds__(1024) k_meas_transpose(uint16_t *meas, int np, size_t nimg) {
    extern __shared__ uint16_t tl[];  // np x (np + 2)
    const int ld = np + 2, nn = np * np;
    const size_t img = blockIdx.x;
    if (img >= nimg) return;
    uint16_t *p = meas + img * nn;
    for (int i = threadIdx.x; i < nn; i += 1024) {
        const int a = i / np, b = i - a * np;
        tl[a * ld + b] = p[i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nn; i += 1024) {
        const int a = i / np, b = i - a * np;
        p[i] = tl[b * ld + a];
    }
}
// g = Np for large Np (the Np 1024 register kernels, np1024.hip): in-place
// transpose by 64 x 64 tile pairs (ti, tj), ti <= tj, swapped through LDS.
// grid (nt (nt + 1) / 2, nimg), block 256
__global__ void __launch_bounds__(256) k_meas_transpose_tiles(uint16_t *meas, int np, size_t nimg) {
    __shared__ uint16_t ta[64][66], tb[64][66];
    const int nt = np / 64;
    int q = blockIdx.x, ti = 0;
    while (q >= nt - ti) {
        q -= nt - ti;
        ++ti;
    }
    const int tj = ti + q;
    uint16_t *p = meas + (size_t)blockIdx.y * np * np;
    uint16_t *a = p + (size_t)ti * 64 * np + tj * 64, *bb = p + (size_t)tj * 64 * np + ti * 64;
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int y = i >> 6, x = i & 63;
        ta[y][x] = a[(size_t)y * np + x];
        tb[y][x] = bb[(size_t)y * np + x];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 64; i += 256) {
        const int y = i >> 6, x = i & 63;
        bb[(size_t)y * np + x] = ta[x][y];
        a[(size_t)y * np + x] = tb[x][y];
    }
}
}  // namespace

// g = 16 (Np 256 fused kernel), 10 (Np 200 fused kernel) or Np (small-patch
// kernel, Np 1024 register kernels: the plain transpose)
hipError_t meas_layout(uint16_t *meas, int np, int g, size_t nimg, bool fwd, hipStream_t s) {
    if (np == 256 && g == 16) return launch_layout<256, 16>(meas, nimg, fwd, s);
    if (np == 200 && g == 10) return launch_layout<200, 10>(meas, nimg, fwd, s);
    if (np == 90 && g == 9) return launch_layout<90, 9>(meas, nimg, fwd, s);
    if (g == np && np <= 128) {
        if (nimg == 0) return hipSuccess;
        const size_t lds = (size_t)np * (np + 2) * sizeof(uint16_t);
        hipLaunchKernelGGL(k_meas_transpose, dim3((unsigned)nimg), dim3(1024), lds, s, meas, np, nimg);
        return hipGetLastError();
    }
    if (g == np && np % 64 == 0) {
        if (nimg == 0) return hipSuccess;
        const int nt = np / 64;
        hipLaunchKernelGGL(k_meas_transpose_tiles, dim3(nt * (nt + 1) / 2, (unsigned)nimg), dim3(256), 0, s, meas,
                           np, nimg);
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// Out-of-place layout: the device-to-device upload and the permutation in ONE
// pass (fpm_upload_stack_device of the fused Np 256 / Np 200 paths): read the
// caller's C-ABI stack once, write the column layout once -- 4 B of HBM per
// pixel instead of the 8 B of a copy followed by the in-place permutation.
// One block per CW-column strip of one image: the strip (Np rows x CW
// columns) is staged in LDS with 8-byte loads, then every lane writes one
// (x, t) run of R pixels with 8-byte stores (contiguous per wave).  The LDS
// row pitch LD = CW + 4 makes the stride-G column reads conflict-free (rows
// t + G m of 16 lanes land on 16 distinct even dword banks, the x pair on +0/+1).
namespace {
template <int NP, int G, int CW>
__global__ void __launch_bounds__(256) k_meas_layout_copy(const uint16_t *__restrict__ src,
                                                         uint16_t *__restrict__ dst, size_t nimg) {
    constexpr int R = NP / G, LD = CW + 4, NS = NP / CW;
    static_assert(NP % CW == 0 && CW % 4 == 0 && R % 4 == 0, "strip and run widths");
    __shared__ __attribute__((aligned(8))) uint16_t tl[NP * LD];
    const size_t img = blockIdx.x / NS;
    const int x0 = (blockIdx.x % NS) * CW;
    if (img >= nimg) return;
    const uint16_t *p = src + img * NP * NP;
    if constexpr (CW % 8 == 0) {  // 16-byte loads (two 8-byte LDS writes: rows are 8-B aligned)
#pragma unroll 4
        for (int i = threadIdx.x; i < NP * (CW / 8); i += 256) {
            const int y = i / (CW / 8), c = i - y * (CW / 8);
            const uint4 q = *(const uint4 *)&p[y * NP + x0 + 8 * c];
            *(uint2 *)&tl[y * LD + 8 * c] = make_uint2(q.x, q.y);
            *(uint2 *)&tl[y * LD + 8 * c + 4] = make_uint2(q.z, q.w);
        }
    } else {
        for (int i = threadIdx.x; i < NP * (CW / 4); i += 256) {
            const int y = i / (CW / 4), c = i - y * (CW / 4);
            *(uint2 *)&tl[y * LD + 4 * c] = *(const uint2 *)&p[y * NP + x0 + 4 * c];
        }
    }
    __syncthreads();
    uint16_t *q = dst + img * NP * NP + (size_t)x0 * NP;
    for (int i = threadIdx.x; i < CW * G; i += 256) {
        const int xl = i / G, t = i - xl * G;  // run (x0 + xl, t): pixels y = t + G m
        uint16_t v[R];
#pragma unroll
        for (int m = 0; m < R; ++m) v[m] = tl[(t + G * m) * LD + xl];
        auto pk = [&](int m) { return (unsigned)v[m] | ((unsigned)v[m + 1] << 16); };
        if constexpr (R % 8 == 0) {  // 16-byte stores (runs of 32 B are 16-B aligned)
#pragma unroll
            for (int k = 0; k < R / 8; ++k)
                *(uint4 *)&q[xl * NP + t * R + 8 * k] = make_uint4(pk(8 * k), pk(8 * k + 2), pk(8 * k + 4), pk(8 * k + 6));
        } else {
#pragma unroll
            for (int k = 0; k < R / 4; ++k)
                *(uint2 *)&q[xl * NP + t * R + 4 * k] = make_uint2(pk(4 * k), pk(4 * k + 2));
        }
    }
}
}  // namespace

// stack [nimg][Np][Np] (C ABI, device) -> dst in the fused column layout;
// false when (np, g) has no out-of-place kernel (callers copy + permute in place)
bool meas_layout_copy(const uint16_t *src, uint16_t *dst, int np, int g, size_t nimg, hipStream_t s,
                      hipError_t *err) {
    *err = hipSuccess;
    if (nimg == 0) return np == 256 && g == 16;
    if (np == 256 && g == 16) {
        hipLaunchKernelGGL((k_meas_layout_copy<256, 16, 64>), dim3((unsigned)(nimg * 4)), dim3(256), 0, s, src, dst,
                           nimg);
    } else if (np == 200 && g == 10) {
        hipLaunchKernelGGL((k_meas_layout_copy<200, 10, 40>), dim3((unsigned)(nimg * 5)), dim3(256), 0, s, src, dst,
                           nimg);
    } else {
        return false;
    }
    *err = hipGetLastError();
    return true;
}

}  // namespace fpm
