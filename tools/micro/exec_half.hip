// Micro-benchmark: does a wave64 VALU instruction cost less when EXEC has only the low 32 lanes
// set (one SIMD-32 pass) than with 64 lanes or with 32 scattered lanes?  (Informs lane compaction.)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void __launch_bounds__(256) k(float* out, int mode, int iters) {
    const int lane = threadIdx.x & 63;
    bool on = mode == 0 ? true : mode == 1 ? lane < 32 : mode == 2 ? (lane & 1) == 0 : lane < 16;
    float a = lane * 0.001f, b = 1.0001f, c = 0.9999f, d = 0.5f;
    if (on) {
        for (int i = 0; i < iters; i++) {
            a = __builtin_fmaf(a, b, c); d = __builtin_fmaf(d, c, b);
            b = __builtin_fmaf(b, c, a); c = __builtin_fmaf(c, a, d);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
int main() {
    float* o; hipMalloc(&o, 256 * 8192 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const char* names[] = {"64 lanes", "low 32 lanes", "even 32 lanes", "low 16 lanes"};
    for (int rep = 0; rep < 2; rep++)
        for (int m = 0; m < 4; m++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, o, m, 4096);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("%-14s %.3f ms\n", names[m], ms);
        }
    return 0;
}
