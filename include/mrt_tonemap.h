/* mrt_tonemap.h -- the image output of the render path: Drago adaptive logarithmic mapping
 * (main.cpp:416-444, L_dmax 230, bias log(0.7)/log(0.5), no gamma) and ARGB32 packing
 * (vec3.h:327-333), written once for the host (mrt_tonemap_argb) and the device tone-map kernel
 * so both produce the same bits; logs and pow are those of the numerics contract (mrt_mathfn.h). */
#ifndef MRT_TONEMAP_H
#define MRT_TONEMAP_H
#include "mrt_mathfn.h"

typedef struct mrt_tonemap_params {
    float scale;   /* L_dmax * 0.01f * invlogmax */
    float invmax;  /* 1 / L_wmax */
    float bias;    /* logf(0.7f) / logf(0.5f) */
} mrt_tonemap_params;

/* relative luminance BT.709 (vec3.h:274-279): (x*cx + y*cy) + z*cz */
MRT_HD float mrt_luminance(const float* c) { return (c[0] * 0.212655f + c[1] * 0.715158f) + c[2] * 0.072187f; }

MRT_HD void mrt_tonemap_setup(float L_wmax, mrt_tonemap_params* tp) {
    const float L_dmax = 230.0f;
    const float invlogmax = 1.0f / mrt_log10f(L_wmax + 1.0f);
    tp->scale = (L_dmax * 0.01f) * invlogmax;
    tp->invmax = 1.0f / L_wmax;
    tp->bias = mrt_logf(0.7f) / mrt_logf(0.5f);
}

/* ARGB32: vmin(v, 1) keeps 1 for NaN (minps), * 255.99, truncation; a negative value (an
 * undefined float->uint32 conversion in the reference) gives 0 */
MRT_HD unsigned int mrt_argb_channel(float v) {
    v = (v < 1.0f ? v : 1.0f) * 255.99f;
    return v > 0.0f ? (unsigned int)v : 0u;
}

MRT_HD unsigned int mrt_tonemap_pixel(const mrt_tonemap_params* tp, const float* c) {
    const float lum = mrt_luminance(c);
    const float loglw = mrt_logf(lum + 1.0f);
    /* logf(2 + powf(..) * 8): one scalar expression, fused as shipped (x86 FMA, main.cpp:437) */
    const float lum_new = tp->scale * (loglw / mrt_logf(fmaf(mrt_powf(lum * tp->invmax, tp->bias), 8.0f, 2.0f)));
    const float d = lum + 0.00001f;
    const unsigned int r = mrt_argb_channel((lum_new * c[0]) / d);
    const unsigned int g = mrt_argb_channel((lum_new * c[1]) / d);
    const unsigned int b = mrt_argb_channel((lum_new * c[2]) / d);
    return (r << 16) | (g << 8) | b;
}

#endif
