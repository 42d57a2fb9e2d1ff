// Exhaustive validation (GPU) of the exact f32 division used by the render kernel (mrt_device.h):
//   y  = RN(1/b)   from v_rcp_f32 + one Newton step  (recip_rn)
//   q  = RN(a*y);  r = fma(-b, q, a);  q' = copysign(fma(r, y, q), q)   (div_y)
// accepted when b and y are normal and either a is zero or q' is normal with |a| >= 2^-100 (so the
// residual r cannot underflow); otherwise the kernel falls back to the IEEE division.  Markstein: with y = RN(1/b) and q within 1 ulp, r is exact and q' = RN(a/b)
// barring over/underflow.  This checks every f32 divisor b against IEEE 1/b, and a/b for K
// numerators per divisor (exponents spread around b's), reporting any ACCEPTED mismatch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ float recip_nr(float b) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y0, 1.0f);
    return __builtin_fmaf(e, y0, y0);
}
__device__ __forceinline__ bool isnorm(float x) { return __builtin_isnormal(x); }

__global__ void rcp_check(uint64_t base, unsigned long long* cnt, uint32_t* ex) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t bb = (uint32_t)i;
    const float b = __uint_as_float(bb);
    if (!isnorm(b)) return;
    const float y = recip_nr(b), ref = 1.0f / b;
    if (!isnorm(ref)) return;
    if (__float_as_uint(y) != __float_as_uint(ref)) {
        atomicAdd(&cnt[0], 1ull);
        if ((bb & 0x7FFFFF) == 0x7FFFFF) atomicAdd(&cnt[1], 1ull);
        uint32_t s = atomicAdd(&ex[0], 1);
        if (s < 16) ex[1 + s] = bb;
    }
}

__global__ void div_check(uint64_t base, uint32_t K, unsigned long long* cnt, uint32_t* ex) {
    const uint64_t i = base + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t bb = (uint32_t)i;
    const float b = __uint_as_float(bb);
    if (!isnorm(b)) return;
    const float y = recip_nr(b);  // == RN(1/b) for normal b with a normal reciprocal (rcp_check)
    if (!isnorm(y)) return;
    uint32_t acc = 0, rej = 0, bad = 0;
    for (uint32_t k = 0; k < K; k++) {
        uint32_t ab = hash32(bb * 0x9E3779B9u + k * 0x85EBCA6Bu + 0x1234567u);
        const uint32_t e = (bb >> 23) & 0xFF;
        if (k < K / 2) ab = (ab & 0x807FFFFFu) | ((uint32_t)((e + (int)(k * 37 % 254)) % 255) << 23);
        if (k == K - 1) ab &= 0x80000000u;  // signed zero numerators
        const float a = __uint_as_float(ab);
        if (!(__builtin_isfinite(a))) continue;
        const float q = a * y;
        const float r = __builtin_fmaf(-b, q, a);
        const float q2 = __builtin_copysignf(__builtin_fmaf(r, y, q), q);
        const bool ok = (isnorm(q2) && __builtin_fabsf(a) >= 0x1p-100f) || a == 0.0f;
        const float ref = a / b;
        if (!ok) { rej++; continue; }
        acc++;
        if (__float_as_uint(q2) != __float_as_uint(ref)) {
            bad++;
            uint32_t s = atomicAdd(&ex[0], 1);
            if (s < 8) { ex[1 + 2 * s] = ab; ex[2 + 2 * s] = bb; }
        }
    }
    atomicAdd(&cnt[0], (unsigned long long)acc);
    atomicAdd(&cnt[1], (unsigned long long)rej);
    if (bad) atomicAdd(&cnt[2], (unsigned long long)bad);
}

int main(int argc, char** argv) {
    const uint32_t K = argc > 1 ? atoi(argv[1]) : 16;
    unsigned long long* d_cnt, h[4];
    uint32_t *d_ex, ex[20];
    (void)hipMalloc(&d_cnt, sizeof(h));
    (void)hipMalloc(&d_ex, sizeof(ex));
    (void)hipMemset(d_cnt, 0, sizeof(h));
    (void)hipMemset(d_ex, 0, sizeof(ex));
    for (uint64_t base = 0; base < (1ull << 32); base += (1ull << 30)) {
        rcp_check<<<(1u << 22), 256>>>(base, d_cnt, d_ex);
        if (hipGetLastError() != hipSuccess) { printf("launch failed\n"); return 1; }
    }
    (void)hipMemcpy(h, d_cnt, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ex, d_ex, sizeof(ex), hipMemcpyDeviceToHost);
    printf("recip_nr: %llu mismatches vs IEEE 1/b over all normal b (%llu with all-ones significand)\n", h[0], h[1]);
    for (uint32_t s = 0; s < ex[0] && s < 16; s++) printf("  b=0x%08x\n", ex[1 + s]);
    (void)hipMemset(d_cnt, 0, sizeof(h));
    (void)hipMemset(d_ex, 0, sizeof(ex));
    for (uint64_t base = 0; base < (1ull << 32); base += (1ull << 30)) {
        div_check<<<(1u << 22), 256>>>(base, K, d_cnt, d_ex);
        if (hipGetLastError() != hipSuccess) { printf("launch failed\n"); return 1; }
        (void)hipDeviceSynchronize();
        printf("  div: divisors < 0x%09llx\n", (unsigned long long)(base + (1ull << 30)));
        fflush(stdout);
    }
    (void)hipMemcpy(h, d_cnt, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipMemcpy(ex, d_ex, sizeof(ex), hipMemcpyDeviceToHost);
    printf("div_rn: %llu accepted, %llu rejected (IEEE fallback), %llu accepted mismatches\n", h[0], h[1], h[2]);
    for (uint32_t s = 0; s < ex[0] && s < 8; s++) printf("  a=0x%08x b=0x%08x\n", ex[1 + 2 * s], ex[2 + 2 * s]);
    return h[2] != 0;
}
