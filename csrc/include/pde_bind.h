// Shared helpers of the torch-facing binding layer (csrc/ops_bindings.cpp, csrc/bind_*.cpp).
#pragma once
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <optional>

namespace pde {

using OptT = std::optional<at::Tensor>;

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline void check_cuda(const at::Tensor& t, const char* name, at::ScalarType dt, int64_t min_numel = 0) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() >= min_numel, name, " has ", t.numel(), " elements, needs >= ", min_numel);
}

template <typename T>
inline T* ptr(const at::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

template <typename T>
inline T* optr(const OptT& t, const char* name, at::ScalarType dt, int64_t min_numel = 0) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_cuda(*t, name, dt, min_numel);
  return ptr<T>(*t);
}

inline void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

constexpr auto F32 = at::kFloat;
constexpr auto BF16 = at::kBFloat16;
constexpr auto I32 = at::kInt;
constexpr auto I64 = at::kLong;
constexpr auto U8 = at::kByte;
constexpr auto F64 = at::kDouble;

// registration hooks of the extra binding units (called from PYBIND11_MODULE in ops_bindings.cpp)
void register_transformer(pybind11::module& m);
void register_resnet(pybind11::module& m);

}  // namespace pde
