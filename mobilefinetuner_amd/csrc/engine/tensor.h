// libmft engine: device tensor with strided views (no torch).
//
// Replaces the reference's Tensor / DType / Device (operators/finetune_ops/core/tensor.h:78-235,
// core/dtype.h:8-52, core/device.h:8-92).  MI355X design instead of the reference's CPU arrays:
//   * storage lives in HBM, handed out by the stream-ordered caching allocator (allocator.h), or in
//     (pinned) host memory for staging; a Tensor is a view {storage, element offset, shape, strides}
//     so reshape / view / slice / narrow / transpose / permute never copy (the reference copies on
//     reshape, core/tensor.cpp:274-294, and materialises transposes, :302-369);
//   * dtypes add bf16 (the compute dtype) next to fp32 / fp16 / int32 / int64 / uint8 / bool;
//   * autograd metadata (grad, grad_fn, hooks, retain_grad) hangs off the impl (autograd.h), grads
//     ACCUMULATE (reference overwrites, core/autograd_engine.cpp:243).
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <functional>
#include <initializer_list>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace mft {
namespace eng {

#define MFT_CHECK(cond, ...)                                                              \
  do {                                                                                    \
    if (!(cond)) ::mft::eng::fail(__FILE__, __LINE__, #cond, ::mft::eng::strcat_(__VA_ARGS__)); \
  } while (0)

[[noreturn]] void fail(const char* file, int line, const char* cond, const std::string& msg);

inline std::string strcat_() { return {}; }
template <typename T>
std::string to_s(const T& v) {
  if constexpr (std::is_convertible_v<T, std::string>) return std::string(v);
  else return std::to_string(v);
}
template <typename T, typename... R>
std::string strcat_(const T& a, const R&... r) {
  return to_s(a) + strcat_(r...);
}

#define HIP_OK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) ::mft::eng::fail(__FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
  } while (0)

enum class DType : uint8_t { F32, BF16, F16, I32, I64, U8, BOOL };
size_t dtype_size(DType d);
const char* dtype_name(DType d);

struct Device {
  enum Kind : uint8_t { CPU, HIP } kind = HIP;
  int index = 0;
  bool pinned = false;  // CPU only: page-locked (hipHostMalloc) staging memory
  static Device cpu(bool pinned = false) { return Device{CPU, -1, pinned}; }
  // i < 0: the calling thread's current HIP device (LOCAL_RANK's GPU once the communicator has
  // selected it), so one-process-per-GPU ranks allocate on their own card, never on GPU 0
  static Device hip(int i = -1) { return Device{HIP, i < 0 ? current_hip_device() : i, false}; }
  static int current_hip_device();
  bool is_hip() const { return kind == HIP; }
  bool operator==(const Device& o) const { return kind == o.kind && index == o.index; }
};

// Owned allocation (returned to its allocator on destruction) or an external non-owned buffer.
struct Storage {
  void* ptr = nullptr;
  size_t nbytes = 0;
  Device dev;
  std::function<void(void*)> deleter;
  ~Storage() {
    if (deleter && ptr) deleter(ptr);
  }
};

using Shape = std::vector<int64_t>;

struct Node;  // autograd.h
struct AutogradMeta;

struct TensorImpl {
  std::shared_ptr<Storage> storage;
  int64_t offset = 0;  // elements
  Shape shape, strides;
  DType dtype = DType::F32;
  // autograd (autograd.h)
  bool requires_grad = false;
  std::unique_ptr<AutogradMeta> ag;
  std::string name;
  ~TensorImpl();
};

class Tensor {
 public:
  Tensor() = default;
  explicit Tensor(std::shared_ptr<TensorImpl> p) : p_(std::move(p)) {}

  bool defined() const { return (bool)p_; }
  TensorImpl* impl() const { return p_.get(); }
  const std::shared_ptr<TensorImpl>& impl_ptr() const { return p_; }

  // ---- geometry
  const Shape& shape() const { return p_->shape; }
  const Shape& strides() const { return p_->strides; }
  int dim() const { return (int)p_->shape.size(); }
  int64_t size(int d) const;
  int64_t stride(int d) const;
  int64_t numel() const;
  size_t nbytes() const { return (size_t)numel() * dtype_size(dtype()); }
  DType dtype() const { return p_->dtype; }
  Device device() const { return p_->storage->dev; }
  bool is_hip() const { return device().is_hip(); }
  bool is_contiguous() const;
  std::string str() const;  // "bf16[4, 128, 768]"

  // ---- raw access (offset applied)
  void* data_ptr() const { return (char*)p_->storage->ptr + p_->offset * (int64_t)dtype_size(dtype()); }
  template <typename T>
  T* data() const { return reinterpret_cast<T*>(data_ptr()); }

  // ---- zero-copy views
  Tensor view(Shape shape) const;     // requires a compatible (contiguous-dims) layout; -1 inferred
  Tensor reshape(Shape shape) const;  // view when possible, else contiguous() copy
  Tensor slice(int dim, int64_t start, int64_t end) const;  // step 1
  Tensor narrow(int dim, int64_t start, int64_t len) const { return slice(dim, start, start + len); }
  Tensor select(int dim, int64_t i) const;
  Tensor transpose(int a, int b) const;
  Tensor permute(const std::vector<int>& order) const;
  Tensor t() const { return transpose(0, 1); }
  Tensor unsqueeze(int d) const;
  Tensor squeeze(int d) const;
  Tensor flatten() const { return reshape({-1}); }
  Tensor as_strided(Shape shape, Shape strides, int64_t offset) const;
  Tensor alias() const;  // new impl, same view, no autograd metadata (detach)
  Tensor detach() const { return alias(); }

  // ---- data movement (on the current stream; device kernels from engine_kernels.hip)
  Tensor contiguous() const;
  Tensor clone() const;
  Tensor to(Device dev) const;
  Tensor to(DType dt) const;
  Tensor& copy_(const Tensor& src);  // any strides / dtype cast / H2D / D2H
  Tensor& zero_();
  Tensor& fill_(double v);
  std::vector<float> to_vector_f32() const;  // host copy (synchronises the stream)
  double item() const;

  // ---- autograd (autograd.h)
  bool requires_grad() const { return p_ && p_->requires_grad; }
  Tensor& requires_grad_(bool on = true);
  Tensor grad() const;
  void set_grad(const Tensor& g);
  void retain_grad();
  bool is_leaf() const;
  void backward(const Tensor& grad = Tensor()) const;
  const std::string& name() const { return p_->name; }
  Tensor& set_name(const std::string& n) {
    p_->name = n;
    return *this;
  }

 private:
  std::shared_ptr<TensorImpl> p_;
};

Shape contiguous_strides(const Shape& shape);
int64_t shape_numel(const Shape& shape);
std::string shape_str(const Shape& s);

// ---- factories (device tensors come from the caching allocator on the current stream)
Tensor empty(Shape shape, DType dt = DType::F32, Device dev = Device::hip());
Tensor zeros(Shape shape, DType dt = DType::F32, Device dev = Device::hip());
Tensor ones(Shape shape, DType dt = DType::F32, Device dev = Device::hip());
Tensor full(Shape shape, double v, DType dt = DType::F32, Device dev = Device::hip());
Tensor arange(int64_t n, DType dt = DType::I64, Device dev = Device::hip());
// counter-based (Philox-style) normal / uniform init, identical on host and device for a seed
Tensor randn(Shape shape, uint64_t seed, float stdev = 1.f, DType dt = DType::F32, Device dev = Device::hip());
Tensor rand_uniform(Shape shape, uint64_t seed, float lo, float hi, DType dt = DType::F32, Device dev = Device::hip());
Tensor from_blob(void* ptr, Shape shape, DType dt, Device dev);  // non-owning
Tensor from_host(const void* src, Shape shape, DType dt, Device dev = Device::hip());
template <typename T>
Tensor from_vector(const std::vector<T>& v, Shape shape, DType dt, Device dev = Device::hip()) {
  return from_host(v.data(), std::move(shape), dt, dev);
}

// ---- streams: the engine runs on one "current" stream per thread (graph capture target)
hipStream_t current_stream();
void set_current_stream(hipStream_t s);
struct StreamGuard {
  hipStream_t prev;
  explicit StreamGuard(hipStream_t s) : prev(current_stream()) { set_current_stream(s); }
  ~StreamGuard() { set_current_stream(prev); }
};
void synchronize();  // current stream

// host <-> bf16 conversion (RNE), used by loaders / tests
uint16_t f32_to_bf16(float f);
float bf16_to_f32(uint16_t h);
uint16_t f32_to_f16(float f);
float f16_to_f32(uint16_t h);

}  // namespace eng
}  // namespace mft
