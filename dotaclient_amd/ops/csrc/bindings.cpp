// Python bindings for the dotaclient_amd HIP kernels.
//
// Kernels live in *.hip translation units that know nothing about torch (raw pointers + hipStream_t, extern "C"
// launchers); this file only validates tensors, picks the current HIP stream (so every op composes with torch
// streams and hipGraph capture) and forwards. Keeping torch headers out of the device TUs keeps their rebuilds fast.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include "launchers.h"

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

inline void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " must be " #dt)
#define CHECK_F32(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, at::kFloat)
#define CHECK_BF16(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, at::kBFloat16)
#define CHECK_I32(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, at::kInt)
#define CHECK_U8(t) CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, at::kByte)

template <typename T>
inline T* ptr(const torch::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

// ------------------------------------------------------------------------------------------------------------
void adam_step(torch::Tensor param, torch::Tensor grad, torch::Tensor m, torch::Tensor v, torch::Tensor seg,
               torch::Tensor counts, torch::Tensor steps, torch::Tensor norm_out, double lr, double b1, double b2,
               double eps, double max_norm) {
  CHECK_F32(param); CHECK_F32(grad); CHECK_F32(m); CHECK_F32(v); CHECK_I32(seg); CHECK_F32(counts);
  CHECK_F32(steps); CHECK_F32(norm_out);
  const int64_t n = param.numel();
  TORCH_CHECK(n % 4 == 0 && grad.numel() == n && m.numel() == n && v.numel() == n && seg.numel() == n,
              "adam_step: flat buffers must share a length that is a multiple of 4");
  TORCH_CHECK(counts.numel() == steps.numel(), "adam_step: counts/steps length mismatch");
  auto partials = torch::empty({1024}, param.options());
  hip_check(dca_adam_step(ptr<float>(param), ptr<float>(grad), ptr<float>(m), ptr<float>(v), ptr<int>(seg), n,
                          ptr<float>(counts), ptr<float>(steps), (int)counts.numel(), ptr<float>(partials),
                          ptr<float>(norm_out), (float)lr, (float)b1, (float)b2, (float)eps, (float)max_norm,
                          cur_stream()),
            "dca_adam_step");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "dotaclient_amd gfx950 HIP kernels";
  m.def("adam_step", &adam_step, "fused global-norm clip + Adam over a flat fp32 buffer");
}
