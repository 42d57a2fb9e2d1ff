// mrt_psum.h -- per-pixel sums of the tolerance contract ("Pixel sums"):
// draw()'s `color += sample` (main.cpp:151-167) accumulated inside the path kernel instead of
// through a per-path radiance buffer in HBM and a fold kernel.
//
// Under the exact contract the fold adds a pixel's samples in sample order, as draw() does (the
// bits depend on that order); the tolerance contract's bar is per-pixel RMSE against the
// reference, so its sum need not be sequential -- but it should still not depend on which wave
// ran which path, so that a render is reproducible bit for bit.  Each finished path's radiance is
// converted to 64-bit fixed point (2^-20 per unit, rounded to nearest: the f64 "magic number"
// conversion, value + 1.5 * 2^52, whose low 52 bits hold the integer) and integer-added; integer
// sums do not depend on their order.  A wave keeps a few pixels' sums in LDS (direct-mapped by
// local pixel, PSUM_SLOTS slots, see below), so a path costs three LDS adds; a slot is flushed into the pixel's 64-bit HBM accumulator (atomics, 32 B per pixel:
// three sums + the count of non-finite samples) when another pixel takes it and when the wave
// ends.  The launch orders its paths pixel-major (path i = local pixel * chunk samples + sample),
// so a wave's lanes hold samples of one or two pixels at a time.
//
// Every sum carries the conversion's offset once per finite path; the final kernel subtracts
// (samples - non-finite samples) offsets.  Range: |radiance| is clamped to 2^30 per component
// (a path above it makes the pixel's mean exceed any max_luminance clamp at < 2^10 spp), and a
// pixel's sum must stay below 2^43 (2^30 * 8192 spp).
//
// Non-finite samples (main.cpp:162-164: `sample = color`, i.e. the running sum doubles) are
// counted per pixel and listed with their sample index (about one per 10 M paths in the Cornell
// scenes, tools/nonfinite_probe.py); the finite samples ahead of each are traced again
// (mrt_retrace_kernel, phase 1) and the final kernel adds, in sample order, the running colour each
// one doubles (psum_color).
#pragma once
#include "mrt_shade.h"

namespace mrtd {

// A wave's LDS holds PSUM_SLOTS pixel slots (direct-mapped by local pixel); each slot's three 64-bit
// sums are split into PSUM_SUBS sub-sums picked by lane (lane % PSUM_SUBS): the lanes of a wave
// mostly finish samples of the SAME pixel (pixel-major order), and 64-bit LDS atomics of many
// lanes on one address serialise in the LDS pipe (measured with one sum per slot: C2 kernel +10%,
// SQ_LDS_BANK_CONFLICT 2.9e10 cycles against 0, SQ_WAIT_INST_LDS x10).  Layout (u32 words): tags
// [PSUM_SLOTS], then u64 sums [slot][channel][sub].
#define PSUM_SLOTS 4u
#define PSUM_SUBS 16u
#define PSUM_TAGW 4u                                                   // words of the tag block (u64-aligned)
#define PSUM_BYTES (PSUM_TAGW * 4u + PSUM_SLOTS * 3u * PSUM_SUBS * 8u)  // 1552
#define PSUM_WORDS ((PSUM_BYTES + 255u) / 256u)                         // per-lane words of the kernels' LDS layout (7)
#define PSUM_NONE 0xFFFFFFFFu
#define PSUM_SCALE 0x1p20
#define PSUM_MAGIC 0x1.8p52
#define PSUM_C 0x4338000000000000ull       // bits of PSUM_MAGIC: one per finite path in every sum
#define PSUM_CLAMP 0x1p30f

struct PsumOut {
    unsigned long long* __restrict__ acc;  // 4 x u64 per local pixel: r, g, b sums, non-finite count
    uint2* __restrict__ nf;                // non-finite samples: (local pixel, sample index)
    uint32_t* __restrict__ nf_n;           // entries appended (may exceed nf_cap: the rest are unlisted)
    uint32_t nf_cap;
    unsigned long long* __restrict__ nfp;  // per entry: the finite samples ahead of it (3 sums, count)
    // paths whose light sample is rounding-critical (mrt_shade.h light_critical), (local pixel,
    // sample index): ended by the fast kernel without a contribution, traced again by the exact
    // arithmetic (mrt_retrace_kernel); null: no such hand-over (the kernel continues them)
    uint2* __restrict__ rt;
    uint32_t* __restrict__ rt_n;
    uint32_t rt_cap;
    uint32_t* __restrict__ rt_done;        // per-path mode: retrace groups finished (the last one clears rt_n)
};

MRT_DFN uint64_t psum_fx(float x) {
    const float c = __builtin_amdgcn_fmed3f(x, -PSUM_CLAMP, PSUM_CLAMP);
    return (uint64_t)__double_as_longlong(__builtin_fma((double)c, PSUM_SCALE, PSUM_MAGIC));
}

MRT_DFN uint64_t* psum_sums(uint32_t* Ls, uint32_t slot, uint32_t ch) {
    return reinterpret_cast<uint64_t*>(Ls + PSUM_TAGW) + (slot * 3u + ch) * PSUM_SUBS;
}

// the wave's slots to empty; every lane of the wave runs it once
MRT_DFN void psum_init(uint32_t* Ls, uint32_t lane) {
    if (lane < PSUM_TAGW) Ls[lane] = PSUM_NONE;
    uint64_t* z = psum_sums(Ls, 0, 0);
    for (uint32_t i = lane; i < PSUM_SLOTS * 3u * PSUM_SUBS; i += 64u) z[i] = 0ull;
}

// slot's sums (all its sub-sums) into its pixel's HBM accumulator, by ONE lane, and the slot emptied
MRT_DFN void psum_flush_slot(uint32_t* Ls, const PsumOut& O, uint32_t slot) {
    const uint32_t tag = Ls[slot];
    for (uint32_t ch = 0; ch < 3u; ch++) {
        uint64_t* w = psum_sums(Ls, slot, ch);
        uint64_t t = 0;
        for (uint32_t k = 0; k < PSUM_SUBS; k++) {
            t += w[k];
            w[k] = 0ull;
        }
        if (tag != PSUM_NONE) atomicAdd(O.acc + (size_t)tag * 4u + ch, (unsigned long long)t);
    }
}

// Adds the finished paths of the calling lanes (exec mask = lanes whose path ended): lp its local
// pixel, s its sample index, L its radiance.  Wave-uniform control flow inside (ballots over the
// calling lanes).
MRT_DFN void psum_add(uint32_t* Ls, const PsumOut& O, uint32_t lp, uint32_t s, f3 L, uint32_t lane) {
    if (!finite3(L)) {
        atomicAdd(O.acc + (size_t)lp * 4u + 3u, 1ull);
        const uint32_t k = atomicAdd(O.nf_n, 1u);
        if (k < O.nf_cap) O.nf[k] = make_uint2(lp, s);
        return;
    }
    const uint64_t vx = psum_fx(L.x), vy = psum_fx(L.y), vz = psum_fx(L.z);
    const uint32_t slot = lp & (PSUM_SLOTS - 1u);
    const uint64_t miss = __ballot(Ls[slot] != lp);
    bool direct = false;
    if (miss) {  // slots taken by other pixels: flush them to HBM, retag (about once per claim)
        uint64_t todo = miss;
        while (todo) {
            const uint32_t l = (uint32_t)__builtin_ctzll(todo);
            const uint32_t ss = (uint32_t)__builtin_amdgcn_readlane((int)slot, (int)l);
            const uint32_t sp = (uint32_t)__builtin_amdgcn_readlane((int)lp, (int)l);
            if (lane == l) {  // (l is a calling lane)
                psum_flush_slot(Ls, O, ss);
                Ls[ss] = sp;
            }
            todo &= ~__ballot(slot == ss);
        }
        direct = Ls[slot] != lp;  // another pixel of this wave holds the slot now
    }
    if (direct) {
        atomicAdd(O.acc + (size_t)lp * 4u + 0u, (unsigned long long)vx);
        atomicAdd(O.acc + (size_t)lp * 4u + 1u, (unsigned long long)vy);
        atomicAdd(O.acc + (size_t)lp * 4u + 2u, (unsigned long long)vz);
    } else {
        const uint32_t sub = lane & (PSUM_SUBS - 1u);
        __hip_atomic_fetch_add(psum_sums(Ls, slot, 0) + sub, vx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(psum_sums(Ls, slot, 1) + sub, vy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(psum_sums(Ls, slot, 2) + sub, vz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
}

// one path's radiance straight into its pixel's HBM sums (the retrace kernel: a few paths)
MRT_DFN void psum_add_global(const PsumOut& O, uint32_t lp, uint32_t s, f3 L) {
    if (!finite3(L)) {
        atomicAdd(O.acc + (size_t)lp * 4u + 3u, 1ull);
        const uint32_t k = atomicAdd(O.nf_n, 1u);
        if (k < O.nf_cap) O.nf[k] = make_uint2(lp, s);
        return;
    }
    atomicAdd(O.acc + (size_t)lp * 4u + 0u, (unsigned long long)psum_fx(L.x));
    atomicAdd(O.acc + (size_t)lp * 4u + 1u, (unsigned long long)psum_fx(L.y));
    atomicAdd(O.acc + (size_t)lp * 4u + 2u, (unsigned long long)psum_fx(L.z));
}

// the wave's remaining slots to HBM (every lane of the wave, once, at the end)
MRT_DFN void psum_drain(uint32_t* Ls, const PsumOut& O, uint32_t lane) {
    if (lane < PSUM_SLOTS * 3u) {
        const uint32_t slot = lane / 3u, ch = lane - slot * 3u;
        const uint32_t tag = Ls[slot];
        if (tag != PSUM_NONE) {
            const uint64_t* w = psum_sums(Ls, slot, ch);
            uint64_t t = 0;
            for (uint32_t k = 0; k < PSUM_SUBS; k++) t += w[k];
            atomicAdd(O.acc + (size_t)tag * 4u + ch, (unsigned long long)t);
        }
    }
}

// The pixel's colour sum after ns samples (draw()'s color before `/= numSamples`): the fixed-point
// sums minus their offsets, plus, for each non-finite sample j in sample order, the running colour
// it doubles: P_j = (the finite samples before it, traced again by the exact arithmetic:
// nfp[entry] = their three fixed-point sums and their count) + P_0 + ... + P_{j-1}.  A sample the
// list had no room for counts as the middle sample with the pixel's finite mean as its prefix.
MRT_DFN f3 psum_color(const unsigned long long* a, uint32_t lp, uint32_t ns, const uint2* nf, const unsigned long long* nfp, uint32_t nf_n,
                      uint32_t nf_cap) {
    const uint64_t bad = a[3];
    const uint64_t off = (uint64_t)(ns - (uint32_t)bad) * PSUM_C;
    double F[3];
    for (int k = 0; k < 3; k++) F[k] = (double)(int64_t)(a[k] - off) * (1.0 / PSUM_SCALE);
    if (bad) {
        const uint32_t m = (uint32_t)bad;
        const uint32_t nl = nf_n < nf_cap ? nf_n : nf_cap;
        const double nfin = (double)(ns - m);
        double E[3] = {0.0, 0.0, 0.0};  // P_0 + ... + P_{j-1}
        uint32_t prev = 0;
        for (uint32_t j = 0; j < m; j++) {
            uint32_t sj = 0xFFFFFFFFu, ej = 0xFFFFFFFFu;  // the next listed sample above prev
            for (uint32_t i = 0; i < nl; i++)
                if (nf[i].x == lp && nf[i].y < sj && (j == 0 || nf[i].y > prev)) {
                    sj = nf[i].y;
                    ej = i;
                }
            double pre[3];
            if (ej != 0xFFFFFFFFu && nfp) {
                const unsigned long long* q = nfp + (size_t)ej * 4u;
                const uint64_t o2 = q[3] * PSUM_C;
                for (int k = 0; k < 3; k++) pre[k] = (double)(int64_t)(q[k] - o2) * (1.0 / PSUM_SCALE);
            } else {
                if (sj == 0xFFFFFFFFu) sj = ns / 2u;
                const double before = sj > j ? (double)(sj - j) : 0.0;
                for (int k = 0; k < 3; k++) pre[k] = nfin > 0 ? F[k] / nfin * before : 0.0;
            }
            prev = sj;
            for (int k = 0; k < 3; k++) E[k] += pre[k] + E[k];
        }
        for (int k = 0; k < 3; k++) F[k] += E[k];
    }
    return f3{(float)F[0], (float)F[1], (float)F[2]};
}

}  // namespace mrtd
