// mrt_cpu.h -- the CPU backend (mrt_cpu.hip) as seen from the C-ABI entry points (mrt_render.hip):
// a scene uploaded to MRT_DEVICE_CPU carries one of these instead of device tables.
#pragma once
#include "../../include/mrt.h"

struct mrt_cpu_scene;
mrt_status mrt_cpu_scene_create(const mrt_scene_view* v, mrt_cpu_scene** out);
void mrt_cpu_scene_free(mrt_cpu_scene* c);
uint32_t mrt_cpu_scene_features(const mrt_cpu_scene* c);
mrt_status mrt_cpu_render(mrt_cpu_scene* c, const mrt_render_desc* d, float* rgb_out, uint64_t* rays_out, const volatile int* cancel);
mrt_status mrt_cpu_progress(mrt_cpu_scene* c, float* pct);
mrt_status mrt_cpu_last_ms(mrt_cpu_scene* c, float* ms, uint32_t* threads);
mrt_status mrt_cpu_preview(mrt_cpu_scene* c, float* rgb_out, uint32_t* samples_done);
mrt_status mrt_cpu_set_worker_seeds(mrt_cpu_scene* c, uint32_t n, const uint64_t* initstate, const uint64_t* initseq);
