// Host-side launcher declarations for every dmlab HIP kernel.
// All launchers are allocation-free and sync-free (hipGraph-capturable).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dm {
typedef unsigned short bf16_t;

// optim.hip
void sgd_step(float* p, const float* g, float* mom, bf16_t* pbf, long long n, float lr,
              float momentum, float dampening, float wd, float gscale, bool nesterov,
              bool first, hipStream_t st);
void adam_step(float* p, const float* g, float* m, float* v, bf16_t* pbf, long long n,
               float lr, float b1, float b2, float eps, float wd, float gscale, float bc1,
               float bc2, hipStream_t st);
void cast_f32_bf16(const float* x, bf16_t* y, long long n, hipStream_t st);
void rows_mean(const float* x, float* out, int rows, long long n, float scale,
               hipStream_t st);
void scale_inplace(float* x, long long n, float s, hipStream_t st);

}  // namespace dm
