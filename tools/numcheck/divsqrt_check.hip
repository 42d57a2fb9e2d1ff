// Validation + timing of exact f32 division / sqrt through f64 (tools/numcheck, GPU only).
//   div:  (float)((double)a * rcp_f64((double)b))  vs  IEEE a / b   (hipcc's correctly rounded f32 division)
//   sqrt: (float)sqrt_f64((double)x)               vs  IEEE sqrtf(x)
// Double rounding is innocuous for / and sqrt when the wide format has >= 2p+2 bits (53 >= 50), so
// the only question is whether the hardware rcp_f64 / sqrt_f64 approximations are close enough;
// this checks every f32 divisor (with K numerators each) and every non-negative f32 radicand.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
#ifndef DIV_VARIANT
#define DIV_VARIANT 1
#endif
__device__ __forceinline__ float fdiv_fast(float a, float b) {
    const double bd = (double)b;
    double r = __builtin_amdgcn_rcp(bd);
#if DIV_VARIANT == 1  // one Newton step on the reciprocal, then one product
    r = __builtin_fma(r, __builtin_fma(-bd, r, 1.0), r);
    return (float)((double)a * r);
#elif DIV_VARIANT == 2  // product, then one residual correction of the quotient
    const double ad = (double)a;
    const double q = ad * r;
    return (float)__builtin_fma(__builtin_fma(-bd, q, ad), r, q);
#else
    return (float)((double)a * r);
#endif
}
__device__ __forceinline__ float fsqrt_fast(float x) { return (float)__builtin_amdgcn_sqrt((double)x); }

__device__ __forceinline__ bool same(float x, float y) {
    if (x != x && y != y) return true;  // NaN payloads are counted separately
    return __float_as_uint(x) == __float_as_uint(y);
}

__global__ void div_check(uint64_t base, uint32_t K, unsigned long long* bad, unsigned long long* nanpay, uint32_t* ex,
                          unsigned long long* cls_cnt) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (1ull << 32)) return;
    const uint32_t bb = (uint32_t)i;
    const float b = __uint_as_float(bb);
    uint32_t nb = 0, np = 0;
    for (uint32_t k = 0; k < K; k++) {
        uint32_t ab = hash32(bb * 0x9E3779B9u + k * 0x85EBCA6Bu + 0x1234567u);
        if (k < 8) {  // numerators spanning exponent ranges near b's
            const uint32_t e = (bb >> 23) & 0xFF;
            ab = (ab & 0x807FFFFFu) | ((uint32_t)((e + (int)(k * 37 % 254)) % 255) << 23);
        }
        const float a = __uint_as_float(ab);
        const float r0 = a / b, r1 = fdiv_fast(a, b);
        (void)0;
        if (!same(r0, r1)) {
            // class: 0 denormal b, 1 denormal a, 2 denormal/zero result, 3 inf result, 4 other
            const uint32_t ea = (ab >> 23) & 0xFF, eb = (bb >> 23) & 0xFF, er = (__float_as_uint(r0) >> 23) & 0xFF;
            const int cls = eb == 0 ? 0 : ea == 0 ? 1 : er == 0 ? 2 : er == 0xFF ? 3 : 4;
            atomicAdd(&cls_cnt[cls], 1ull);
            nb++;
            if (cls >= 2 && ex[0] < 16) { uint32_t s = atomicAdd(&ex[0], 1); if (s < 16) { ex[1 + 2 * s] = ab; ex[2 + 2 * s] = bb; } }
        }
        else if (__float_as_uint(r0) != __float_as_uint(r1)) np++;
    }
    if (nb) atomicAdd(bad, (unsigned long long)nb);
    if (np) atomicAdd(nanpay, (unsigned long long)np);
}

__global__ void sqrt_check(uint64_t base, unsigned long long* bad, unsigned long long* nanpay, uint32_t* ex) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (1ull << 32)) return;
    const float x = __uint_as_float((uint32_t)i);
    const float r0 = __builtin_sqrtf(x), r1 = fsqrt_fast(x);
    if (!same(r0, r1)) {
        atomicAdd(bad, 1ull);
        uint32_t s = atomicAdd(&ex[0], 1);
        if (s < 16) ex[1 + s] = (uint32_t)i;
    } else if (__float_as_uint(r0) != __float_as_uint(r1)) atomicAdd(nanpay, 1ull);
}

// throughput: dependent chains of divisions / square roots per lane
template <int MODE>
__global__ void bench(float* out, int iters) {
    float a = 1.0f + threadIdx.x * 1e-3f, b = 1.5f + blockIdx.x * 1e-4f, c = 0.75f, d = 2.5f;
    for (int i = 0; i < iters; i++) {
        if (MODE == 0) { a = b / a; c = d / c; }
        else if (MODE == 1) { a = fdiv_fast(b, a); c = fdiv_fast(d, c); }
        else if (MODE == 2) { a = __builtin_sqrtf(a) + b; c = __builtin_sqrtf(c) + d; }
        else { a = fsqrt_fast(a) + b; c = fsqrt_fast(c) + d; }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + c;
}

int main(int argc, char** argv) {
    unsigned long long *d_bad, h[2];
    uint32_t *d_ex, ex[40];
    hipMalloc(&d_bad, 16);
    hipMalloc(&d_ex, sizeof(ex));
    unsigned long long* d_cls, hcls[5];
    hipMalloc(&d_cls, sizeof(hcls));
    hipMemset(d_cls, 0, sizeof(hcls));
    // sqrt: every bit pattern
    hipMemset(d_bad, 0, 16); hipMemset(d_ex, 0, sizeof(ex));
    // (a grid of gridDim.x * blockDim.x >= 2^32 threads does not launch: chunks of 2^30)
    for (uint64_t base = 0; base < (1ull << 32); base += (1ull << 30)) {
        sqrt_check<<<(1u << 22), 256>>>(base, d_bad, d_bad + 1, d_ex);
        if (hipGetLastError() != hipSuccess) { printf("launch failed\n"); return 1; }
    }
    hipDeviceSynchronize();
    hipMemcpy(h, d_bad, 16, hipMemcpyDeviceToHost);
    hipMemcpy(ex, d_ex, sizeof(ex), hipMemcpyDeviceToHost);
    printf("sqrt: %llu mismatches over 2^32 inputs (%llu NaN-payload-only)\n", h[0], h[1]);
    for (uint32_t s = 0; s < ex[0] && s < 16; s++) {
        const float x = *(float*)&ex[1 + s];
        printf("  x=0x%08x (%g)\n", ex[1 + s], x);
    }
    // division: every divisor, K numerators each
    const uint32_t K = argc > 1 ? atoi(argv[1]) : 24;
    hipMemset(d_bad, 0, 16); hipMemset(d_ex, 0, sizeof(ex));
    for (uint64_t base = 0; base < (1ull << 32); base += (1ull << 30)) {
        div_check<<<(1u << 22), 256>>>(base, K, d_bad, d_bad + 1, d_ex, d_cls);
        if (hipGetLastError() != hipSuccess) { printf("launch failed\n"); return 1; }
        hipDeviceSynchronize();
        printf("  div: divisors up to 0x%09llx done\n", (unsigned long long)(base + (1ull << 30)));
        fflush(stdout);
    }
    hipMemcpy(h, d_bad, 16, hipMemcpyDeviceToHost);
    hipMemcpy(ex, d_ex, sizeof(ex), hipMemcpyDeviceToHost);
    hipMemcpy(hcls, d_cls, sizeof(hcls), hipMemcpyDeviceToHost);
    printf("div mismatch classes: denormal b %llu, denormal a %llu, denormal/zero result %llu, inf result %llu, other %llu\n",
           hcls[0], hcls[1], hcls[2], hcls[3], hcls[4]);
    printf("div: %llu mismatches over 2^32 divisors x %u numerators (%llu NaN-payload-only)\n", h[0], K, h[1]);
    for (uint32_t s = 0; s < ex[0] && s < 16; s++) printf("  a=0x%08x b=0x%08x\n", ex[1 + 2 * s], ex[2 + 2 * s]);
    // timing
    float* out;
    hipMalloc(&out, 1024 * 256 * 4 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const char* names[4] = {"div IEEE f32", "div f64 rcp", "sqrt IEEE f32", "sqrt f64"};
    for (int m = 0; m < 4; m++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            const int iters = 4096;
            if (m == 0) bench<0><<<1024 * 8, 256>>>(out, iters);
            if (m == 1) bench<1><<<1024 * 8, 256>>>(out, iters);
            if (m == 2) bench<2><<<1024 * 8, 256>>>(out, iters);
            if (m == 3) bench<3><<<1024 * 8, 256>>>(out, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("%-14s %.3f ms  %.1f Gop/s\n", names[m], ms, 2.0 * iters * 1024 * 8 * 256 / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
