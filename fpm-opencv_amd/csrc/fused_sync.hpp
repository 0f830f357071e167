// fused_sync.hpp -- device-coherent handoffs between the workgroups that
// share one patch (split mode of fpm_fused.hip, the distributed kernel of
// fused_dist.hip), and the streamed measurement load.
#pragma once
#include <hip/hip_runtime.h>

namespace fpm {

// Handoff between the two workgroups of a patch (split mode).  Everything the
// partner reads -- the exchange area, the updated spectrum window, the flags --
// moves with device-coherent (sc1) loads and stores (relaxed agent-scope
// atomics), so no L2 write-back or invalidate is needed; the partner may sit
// on another XCD.  (Agent-scope release/acquire fences instead -- buffer_wbl2 /
// buffer_inv on every handoff -- measured 3.4x slower: they flush and
// invalidate the whole XCD L2 that the other patches' streams use.)
//   publish: every wave waits for its own stores to be acknowledged, then one
//            thread stores the flag.
//   wait:    lane p of the first wave polls part p's flag (one vector load
//            per spin, s_sleep between spins) and gives up after ~1 s,
//            raising abort_flag so the partners leave too.
// Co-located parts (every workgroup reports the same XCC_ID): the XCD's L2
// is the coherence point, so stores stay plain (the L1 writes through and the
// line stays in that L2) and loads bypass the L1 with the sc1 policy: L2
// round trips instead of memory round trips on the critical path.  (An sc0
// load is NOT enough: it hits the CU's L1 like a plain load, and the L1 is
// never refreshed by other CUs' stores -- MI355X_MICROARCH.md, visibility
// row; round 2 used sc0 here and was exposed as stale reads once the
// distributed kernel re-read the same lines every LED.)
// aux: bit 4 = sc1 (L1 bypass, L2-served), bit 31 = volatile (keeps the
// compiler from hoisting a polled load out of its loop or merging it with
// earlier reads)
constexpr int kAuxL2Volatile = (int)(16u | (1u << 31));
__device__ __forceinline__ float2 ld_l2(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, kAuxL2Volatile));
}
__device__ __forceinline__ int ld_l2_i32(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return (int)__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, kAuxL2Volatile);
}
__device__ __forceinline__ int xcc_id() {
    int x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 15;
}
__device__ __forceinline__ void handoff_publish(int *flag, int value, bool local) {
    __builtin_amdgcn_s_waitcnt(0);  // this wave's stores are acknowledged
    __syncthreads();
    if (threadIdx.x == 0) {
        if (local) __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// wait until every other part's flag (flags[0..KS), part `me` excluded) has
// reached `value`.  Lane p < KS of the first wave polls part p's flag and the
// last lane polls the abort word, all in ONE vector load per spin: one L2 round
// trip however many partners (a single polling lane walking the partners in
// turn paid KS - 1 dependent round trips per handoff even when every flag was
// already set).
template <int KS>
__device__ __forceinline__ bool handoff_wait(int *flags, int me, int value, int *abort_flag, int *okslot, bool local,
                                             __amdgpu_buffer_rsrc_t rflag) {
    static_assert(KS < 64, "one polling lane per part");
    if (threadIdx.x < 64) {
        const int l = threadIdx.x;
        const bool poll = l < KS && l != me, watch = l == 63;
        bool done = !poll;  // lanes with nothing to wait for
        int ok = 1;
        for (int spins = 0;; ++spins) {
            int f = 0;
            if (poll && !done)
                f = local ? ld_l2_i32(rflag, l * (int)sizeof(int))
                          : __hip_atomic_load(flags + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else if (watch)
                f = __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (poll) done = done || f >= value;
            const bool aborted = __builtin_amdgcn_readlane(watch ? f : 0, 63) != 0;
            if (__all(done)) break;
            if (aborted) {
                ok = 0;
                break;
            }
            if (spins > (1 << 23)) {
                if (l == 0) __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (l == 0) *okslot = ok;
    }
    __syncthreads();
    return *okslot != 0;
}

// Launch clock probe (the bench line's clock_mhz / kernel_cycles_per_launch,
// MI355X_MICROARCH.md DVFS item 6): block 0's shader cycles (s_memtime) and
// 100 MHz real-time ticks (s_memrealtime) from kernel entry to its last
// phase, summed into clk[0] / clk[1] with clk[2] counting launches.  Read in
// every wave as wave-uniform scalars (no VGPRs held across the kernel);
// thread 0 of block 0 accumulates with vector atomics into the context's own
// probe buffer, which nothing else reads.  Two SMEM reads per wave per launch.
struct ClockProbe {
    unsigned long long c0, r0;
    __device__ __forceinline__ void start() {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ void stop(unsigned long long *clk) const {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (clk && blockIdx.x == 0 && threadIdx.x == 0) {
            atomicAdd(clk, c1 - c0);
            atomicAdd(clk + 1, r1 - r0);
            atomicAdd(clk + 2, 1ull);
        }
    }
};

// measurement stream: read once per LED, so load it non-temporally and keep
// L2 for the spectrum window the next LED re-reads
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_stream(const uint4 *p) {
    const u32x4_t v = __builtin_nontemporal_load((const u32x4_t *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Plain launch of a grid whose workgroups wait on each other (split and
// distributed modes): every block must be resident at once.  The grid is
// checked against the occupancy query -- the check hipLaunchCooperativeKernel
// makes -- and launched plainly: the same residency (MI355X_MICROARCH.md
// "coop-launch") without the cooperative launch's per-launch host cost.
// Two such grids must never run side by side on one device (each could get
// only part of its blocks resident and both would wait for the rest), so
// launch_coresident_raw (api.cpp) orders every co-resident grid of the
// process on a device after the previous one: a per-device mutex, a wait on
// the previous grid's completion event, a new event after the launch -- what
// the cooperative launch's serialisation gave.  Across processes a device is
// single-tenant for these modes.  Every wait in those
// kernels also gives up after ~1 s and raises the sticky abort word, so a grid
// that could not be co-resident fails instead of hanging.
hipError_t launch_coresident_raw(const void *fn, int grid, int block, size_t lds, void **args, hipStream_t s);
template <class Args>
inline hipError_t launch_coresident(const void *fn, int grid, int block, size_t lds, Args *a, hipStream_t s) {
    void *args[] = {a};
    return launch_coresident_raw(fn, grid, block, lds, args, s);
}

}  // namespace fpm
