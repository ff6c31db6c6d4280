// extern "C" launchers exported by the *.hip kernel translation units (raw pointers + stream; no torch types).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

hipError_t dca_adam_step(float* param, const float* grad, float* m, float* v, const int* seg, int64_t n,
                         const float* counts, float* steps, int n_params, float* partials, float* norm_out, float lr,
                         float b1, float b2, float eps, float max_norm, hipStream_t stream);

}  // extern "C"
