// fused_common.hpp -- geometry, kernel arguments and host-side tables shared
// by the Np 256 fused LED-update kernels: one workgroup per patch and split
// mode (fpm_fused.hip), and the distributed mode (fused_dist.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "fpm_state.hpp"
#include "fused_sync.hpp"

namespace fpm {

namespace fz {
constexpr int NP = 256;
constexpr int NROWS = 64;           // FFT rows per patch (RPG = NROWS / groups per group)
constexpr int MAXTAIL = 64;         // tail pixels (one owner thread each)
constexpr int MAXTAILROWS = 8;
constexpr int SK[6] = {0, 1, 2, 13, 14, 15};  // registers that can hold |kx| <= 47
constexpr int KYOFF = 48;                     // sigma table covers ky in [-48, 47]
}  // namespace fz

struct FusedArgs {
    DevState st;
    const uint16_t *meas;       // [nS][B][x][t][m2] = I[t + 16 m2][x] (meas_layout, preprocess.hip)
    const int *order, *x0, *y0;
    const float2 *tw;           // exp(-2 pi i k / 256), k < 256
    int n_order;
    int ky_lo, n_fft_rows;      // FFT rows ky_lo .. ky_lo + n_fft_rows - 1 (sigma 0..)
    int n_tail_rows;
    int tail_ky[fz::MAXTAILROWS];  // sigma = 64 + i
    int n_tail_px;
    int2 tail_px[fz::MAXTAIL];  // (ky, kx), sorted by row then kx
    // tail row q holds pixels tail_px[p0 .. p0+np) with kx = kx0, kx0+1, ...
    int tail_row_p0[fz::MAXTAILROWS], tail_row_np[fz::MAXTAILROWS], tail_row_kx0[fz::MAXTAILROWS];
    // tiles of the spectrum's live band (fpm_state.hpp): every other tile is
    // exactly 0 and never changes, so the kernel keeps maxima and dirty bits
    // for these nbt tiles only (band tile k = (bty0 + k / nbx, btx0 + k % nbx));
    // st.tdirty holds the band-indexed bits between launches
    int btx0, bty0, nbx, nbt;
    float rnbx;                 // 1 / nbx
    unsigned long long *dbg;    // diagnostic phase stamps (FPM_STAMPS=1), else null
    // split mode (NT 512, KS = 2 or 4 workgroups per patch, KS * B <= CUs):
    // workgroup p owns column part p (256 / KS columns); handoffs through xch
    // with device-scope flags
    float2 *xch;                // [B][KS parts][2 LED parities][kXchHalf]: F partial | tail F partial
    int *flags;                 // [B][KS]: part p's F partials of LED it published (it + 1);
                                // then the abort flag, then [B][KS] XCC_ID + 1 of each part
    int *abort_flag;            // a handoff timed out: every workgroup leaves.  Sticky: the
                                // per-launch reset does not clear it, fpm_run reports it
    int ledtab_off;             // byte offset of the LED table in dynamic LDS (ledtab.hpp), or -1
    int stall_led;              // fpm_debug_set_stall (tests only): the last part stops
                                // publishing from this LED on, forcing the timeout path; -1 off
    unsigned tag_base;          // distributed mode: LEDs of the context's earlier launches, so
                                // LED it of this launch tags its tile words tag_base + it + 1
                                // (mod 2^31) and a word left by an earlier launch never matches
};

// split-mode exchange area per patch (float2): each part's F partials of the
// 512 lanes (12 slots each, lane-major) and of the <= 64 tail pixels, double
// buffered by LED parity (a part overwrites its LED-i buffer only at LED i+2,
// after every partner has published LED i+1, i.e. has read LED i's partials)
constexpr int kXchTF = 12 * 512, kXchHalf = kXchTF + 64;
constexpr int xch_patch_elems(int ks) { return 2 * ks * kXchHalf; }

// kx of slot s of lane t: t + 16 SK[s] - (s >= 3 ? Np : 0), written without
// the table (SK[s] = s + 10 [s >= 3]) so a run-time s (the spread object
// update) is arithmetic, not a global load whose wait drains every
// outstanding memory operation
__device__ __forceinline__ int slot_kx(int t, int s) { return t + 16 * s - (s >= 3 ? 96 : 0); }
static_assert(fz::SK[3] * 16 - fz::NP == 3 * 16 - 96 && fz::SK[5] * 16 - fz::NP == 5 * 16 - 96, "slot_kx");

// ------------------------------------------------------------------ host side
struct FusedGeom {
    bool ok = false;
    int ky_lo = 0, n_fft_rows = 0, n_tail_rows = 0, tail_ky[fz::MAXTAILROWS] = {0};
    int n_tail_px = 0;
    int2 tail_px[fz::MAXTAIL];
    int nbp = 0;
};

inline FusedGeom fused_geometry(int np, int r) {
    FusedGeom g;
    // the tail tables (8 rows, 64 pixels) hold every box row beyond the 64 FFT
    // rows up to r = 34 (r = 35 has 7 tail rows with more than 64 pixels)
    if (np != fz::NP || r < 1 || r > 34) return g;
    const int nb = 2 * r + 1;
    const int nfft = nb < fz::NROWS ? nb : fz::NROWS;
    const int extra = nb - nfft;
    g.ky_lo = -r + extra / 2;  // the 64 central rows go to the FFT groups
    g.n_fft_rows = nfft;
    for (int ky = -r; ky <= r; ++ky) {
        if (ky >= g.ky_lo && ky < g.ky_lo + nfft) continue;
        if (g.n_tail_rows >= fz::MAXTAILROWS) return g;
        g.tail_ky[g.n_tail_rows++] = ky;
        for (int kx = -r; kx <= r; ++kx)
            if (ky * ky + kx * kx <= r * r) {
                if (g.n_tail_px >= fz::MAXTAIL) return g;
                g.tail_px[g.n_tail_px++] = make_int2(ky, kx);
            }
    }
    g.nbp = ((fz::NROWS + g.n_tail_rows) + 3) / 4 * 4;
    g.ok = true;
    return g;
}

struct Band {
    int bty0, btx0, nbx, nbt;
};
inline Band band_of(const DevState &st) {
    Band b;
    b.bty0 = st.sy0 / kTile;
    b.btx0 = st.sx0 / kTile;
    b.nbx = st.sx1 / kTile - b.btx0 + 1;
    b.nbt = b.nbx * (st.sy1 / kTile - b.bty0 + 1);
    return b;
}

}  // namespace fpm
