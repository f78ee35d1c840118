// libmft engine: Tensor implementation (views, factories, copies, host conversions).
#include "engine/tensor.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <sstream>

#include "engine/allocator.h"
#include "engine/autograd.h"
#include "engine/ops.h"

namespace mft {
namespace eng {

[[noreturn]] void fail(const char* file, int line, const char* cond, const std::string& msg) {
  std::ostringstream os;
  os << "mft engine: " << msg << " [" << cond << " at " << file << ":" << line << "]";
  throw std::runtime_error(os.str());
}

size_t dtype_size(DType d) {
  switch (d) {
    case DType::F32:
    case DType::I32: return 4;
    case DType::I64: return 8;
    case DType::BF16:
    case DType::F16: return 2;
    default: return 1;
  }
}

const char* dtype_name(DType d) {
  switch (d) {
    case DType::F32: return "f32";
    case DType::BF16: return "bf16";
    case DType::F16: return "f16";
    case DType::I32: return "i32";
    case DType::I64: return "i64";
    case DType::U8: return "u8";
    default: return "bool";
  }
}

TensorImpl::~TensorImpl() = default;

// ------------------------------------------------------------------ streams
namespace {
thread_local hipStream_t t_stream = nullptr;
}
hipStream_t current_stream() { return t_stream; }
int Device::current_hip_device() {
  int d = 0;
  HIP_OK(hipGetDevice(&d));
  return d;
}
void set_current_stream(hipStream_t s) { t_stream = s; }
void synchronize() { HIP_OK(hipStreamSynchronize(t_stream)); }

// ------------------------------------------------------------------ geometry helpers
Shape contiguous_strides(const Shape& shape) {
  Shape st(shape.size());
  int64_t s = 1;
  for (int i = (int)shape.size() - 1; i >= 0; --i) {
    st[i] = s;
    s *= std::max<int64_t>(shape[i], 1);
  }
  return st;
}

int64_t shape_numel(const Shape& s) {
  int64_t n = 1;
  for (auto v : s) n *= v;
  return n;
}

std::string shape_str(const Shape& s) {
  std::string o = "[";
  for (size_t i = 0; i < s.size(); ++i) o += (i ? ", " : "") + std::to_string(s[i]);
  return o + "]";
}

static int wrap_dim(int d, int n) {
  if (d < 0) d += n;
  MFT_CHECK(d >= 0 && d < std::max(n, 1), "dim ", d, " out of range for ", n, " dims");
  return d;
}

int64_t Tensor::size(int d) const { return p_->shape[wrap_dim(d, dim())]; }
int64_t Tensor::stride(int d) const { return p_->strides[wrap_dim(d, dim())]; }
int64_t Tensor::numel() const { return shape_numel(p_->shape); }

bool Tensor::is_contiguous() const {
  int64_t s = 1;
  for (int i = dim() - 1; i >= 0; --i) {
    if (p_->shape[i] != 1 && p_->strides[i] != s) return false;
    s *= p_->shape[i];
  }
  return true;
}

std::string Tensor::str() const {
  if (!p_) return "undefined";
  return std::string(dtype_name(dtype())) + shape_str(shape()) + (is_hip() ? "@hip" : "@cpu");
}

static Tensor make_view(const Tensor& base, Shape shape, Shape strides, int64_t offset) {
  auto t = std::make_shared<TensorImpl>();
  t->storage = base.impl()->storage;
  t->offset = offset;
  t->shape = std::move(shape);
  t->strides = std::move(strides);
  t->dtype = base.dtype();
  return Tensor(t);
}

Tensor Tensor::alias() const { return make_view(*this, shape(), strides(), p_->offset); }

Tensor Tensor::as_strided(Shape shape, Shape strides, int64_t offset) const {
  Tensor out = make_view(*this, shape, strides, offset);
  if (needs_grad(*this)) {
    const int64_t off0 = p_->offset;
    record_view(*this, out,
                [shape, strides, offset, off0](const Tensor& t) {
                  return t.as_strided(shape, strides, t.impl()->offset + (offset - off0));
                },
                nullptr, false);
  }
  return out;
}

// view: infer -1, then compute strides for the new shape if the old layout allows it
static bool view_strides(const Shape& old_shape, const Shape& old_st, const Shape& nshape, Shape& out) {
  // merge old dims into contiguous chunks and split them into new dims (PyTorch's computeStride)
  out.assign(nshape.size(), 0);
  if (shape_numel(old_shape) == 0) {
    out = contiguous_strides(nshape);
    return true;
  }
  int view_d = (int)nshape.size() - 1;
  int64_t chunk_base_stride = old_st.empty() ? 1 : old_st.back();
  int64_t tensor_numel = 1, view_numel = 1;
  for (int tensor_d = (int)old_shape.size() - 1; tensor_d >= 0; --tensor_d) {
    tensor_numel *= old_shape[tensor_d];
    if (tensor_d == 0 || (old_shape[tensor_d - 1] != 1 && old_st[tensor_d - 1] != tensor_numel * chunk_base_stride)) {
      while (view_d >= 0 && (view_numel < tensor_numel || nshape[view_d] == 1)) {
        out[view_d] = view_numel * chunk_base_stride;
        view_numel *= nshape[view_d];
        view_d--;
      }
      if (view_numel != tensor_numel) return false;
      if (tensor_d > 0) {
        chunk_base_stride = old_st[tensor_d - 1];
        tensor_numel = 1;
        view_numel = 1;
      }
    }
  }
  return view_d == -1;
}

static Shape infer_shape(Shape s, int64_t n) {
  int neg = -1;
  int64_t prod = 1;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == -1) {
      MFT_CHECK(neg < 0, "view: more than one -1");
      neg = (int)i;
    } else {
      prod *= s[i];
    }
  }
  if (neg >= 0) {
    MFT_CHECK(prod > 0 && n % prod == 0, "view: cannot infer -1 for ", n, " elements");
    s[neg] = n / prod;
  }
  MFT_CHECK(shape_numel(s) == n, "view: shape ", shape_str(s), " does not match ", n, " elements");
  return s;
}

Tensor Tensor::view(Shape shape) const {
  Shape ns = infer_shape(std::move(shape), numel());
  Shape st;
  MFT_CHECK(view_strides(p_->shape, p_->strides, ns, st), "view: incompatible strides for ", str(), " -> ",
            shape_str(ns), " (use reshape)");
  Tensor out = make_view(*this, ns, st, p_->offset);
  if (needs_grad(*this)) {
    Shape in_shape = p_->shape;
    record_view(*this, out, nullptr, [in_shape](const Tensor& g) { return g.reshape(in_shape); }, true);
  }
  return out;
}

Tensor Tensor::reshape(Shape shape) const {
  Shape ns = infer_shape(std::move(shape), numel());
  Shape st;
  if (view_strides(p_->shape, p_->strides, ns, st)) return view(ns);
  return contiguous().view(ns);
}

Tensor Tensor::slice(int d, int64_t start, int64_t end) const {
  d = wrap_dim(d, dim());
  const int64_t n = p_->shape[d];
  if (start < 0) start += n;
  if (end < 0) end += n;
  start = std::max<int64_t>(0, std::min(start, n));
  end = std::max(start, std::min(end, n));
  Shape ns = p_->shape;
  ns[d] = end - start;
  Tensor out = make_view(*this, ns, p_->strides, p_->offset + start * p_->strides[d]);
  if (needs_grad(*this)) {
    record_view(*this, out, [d, start, end](const Tensor& t) { return t.slice(d, start, end); }, nullptr,
                start == 0 && end == n);
  }
  return out;
}

Tensor Tensor::select(int d, int64_t i) const {
  d = wrap_dim(d, dim());
  if (i < 0) i += p_->shape[d];
  MFT_CHECK(i >= 0 && i < p_->shape[d], "select: index out of range");
  Shape ns = p_->shape, st = p_->strides;
  const int64_t off = p_->offset + i * st[d];
  ns.erase(ns.begin() + d);
  st.erase(st.begin() + d);
  Tensor out = make_view(*this, ns, st, off);
  if (needs_grad(*this)) record_view(*this, out, [d, i](const Tensor& t) { return t.select(d, i); }, nullptr, false);
  return out;
}

Tensor Tensor::transpose(int a, int b) const {
  a = wrap_dim(a, dim());
  b = wrap_dim(b, dim());
  Shape ns = p_->shape, st = p_->strides;
  std::swap(ns[a], ns[b]);
  std::swap(st[a], st[b]);
  Tensor out = make_view(*this, ns, st, p_->offset);
  if (needs_grad(*this)) record_view(*this, out, nullptr, [a, b](const Tensor& g) { return g.transpose(a, b); }, true);
  return out;
}

Tensor Tensor::permute(const std::vector<int>& order) const {
  MFT_CHECK((int)order.size() == dim(), "permute: order size");
  Shape ns(dim()), st(dim());
  std::vector<int> inv(dim());
  for (int i = 0; i < dim(); ++i) {
    const int o = wrap_dim(order[i], dim());
    ns[i] = p_->shape[o];
    st[i] = p_->strides[o];
    inv[o] = i;
  }
  Tensor out = make_view(*this, ns, st, p_->offset);
  if (needs_grad(*this)) record_view(*this, out, nullptr, [inv](const Tensor& g) { return g.permute(inv); }, true);
  return out;
}

Tensor Tensor::unsqueeze(int d) const {
  d = d < 0 ? d + dim() + 1 : d;
  MFT_CHECK(d >= 0 && d <= dim(), "unsqueeze: dim");
  Shape ns = p_->shape, st = p_->strides;
  const int64_t s = d < dim() ? st[d] * ns[d] : 1;
  ns.insert(ns.begin() + d, 1);
  st.insert(st.begin() + d, s);
  Tensor out = make_view(*this, ns, st, p_->offset);
  if (needs_grad(*this)) {
    Shape in = p_->shape;
    record_view(*this, out, nullptr, [in](const Tensor& g) { return g.reshape(in); }, true);
  }
  return out;
}

Tensor Tensor::squeeze(int d) const {
  d = wrap_dim(d, dim());
  if (p_->shape[d] != 1) return *this;
  Shape ns = p_->shape, st = p_->strides;
  ns.erase(ns.begin() + d);
  st.erase(st.begin() + d);
  Tensor out = make_view(*this, ns, st, p_->offset);
  if (needs_grad(*this)) {
    Shape in = p_->shape;
    record_view(*this, out, nullptr, [in](const Tensor& g) { return g.reshape(in); }, true);
  }
  return out;
}

// ------------------------------------------------------------------ allocation
static std::shared_ptr<Storage> alloc_storage(size_t nbytes, Device dev) {
  auto s = std::make_shared<Storage>();
  s->nbytes = nbytes;
  s->dev = dev;
  if (dev.is_hip()) {
    auto& a = CachingAllocator::get(dev.index);
    s->ptr = a.allocate(nbytes, current_stream());
    s->deleter = [&a](void* p) { a.release(p); };
  } else if (dev.pinned) {
    s->ptr = PinnedAllocator::get().allocate(nbytes);
    s->deleter = [](void* p) { PinnedAllocator::get().release(p, current_stream()); };
  } else {
    s->ptr = ::operator new(std::max<size_t>(nbytes, 1));
    s->deleter = [](void* p) { ::operator delete(p); };
  }
  return s;
}

Tensor empty(Shape shape, DType dt, Device dev) {
  for (auto v : shape) MFT_CHECK(v >= 0, "empty: negative dim in ", shape_str(shape));
  auto t = std::make_shared<TensorImpl>();
  t->storage = alloc_storage((size_t)shape_numel(shape) * dtype_size(dt), dev);
  t->strides = contiguous_strides(shape);
  t->shape = std::move(shape);
  t->dtype = dt;
  return Tensor(t);
}

Tensor from_blob(void* ptr, Shape shape, DType dt, Device dev) {
  auto t = std::make_shared<TensorImpl>();
  t->storage = std::make_shared<Storage>();
  t->storage->ptr = ptr;
  t->storage->nbytes = (size_t)shape_numel(shape) * dtype_size(dt);
  t->storage->dev = dev;
  t->strides = contiguous_strides(shape);
  t->shape = std::move(shape);
  t->dtype = dt;
  return Tensor(t);
}

Tensor zeros(Shape shape, DType dt, Device dev) {
  Tensor t = empty(std::move(shape), dt, dev);
  t.zero_();
  return t;
}
Tensor ones(Shape shape, DType dt, Device dev) { return full(std::move(shape), 1.0, dt, dev); }
Tensor full(Shape shape, double v, DType dt, Device dev) {
  Tensor t = empty(std::move(shape), dt, dev);
  t.fill_(v);
  return t;
}

Tensor arange(int64_t n, DType dt, Device dev) {
  std::vector<int64_t> h(n);
  for (int64_t i = 0; i < n; ++i) h[i] = i;
  Tensor t = from_host(h.data(), {n}, DType::I64, dev);
  return dt == DType::I64 ? t : t.to(dt);
}

// ---- host RNG identical to the device kernels (engine/tensor_kernels.hip: mix64 / u01)
static uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static float u01(uint64_t h) { return ((h >> 40) + 0.5f) * (1.0f / 16777216.0f); }

Tensor randn(Shape shape, uint64_t seed, float stdev, DType dt, Device dev) {
  Tensor t = empty(std::move(shape), dt, dev);
  if (dev.is_hip()) {
    k::randn(t.data_ptr(), (int)dt, t.numel(), seed, stdev, current_stream());
  } else {
    std::vector<float> h(t.numel());
    for (int64_t i = 0; i < t.numel(); ++i) {
      const float u1 = u01(mix64(seed * 0x2545F4914F6CDD1Dull + 2 * (uint64_t)i));
      const float u2 = u01(mix64(seed * 0x2545F4914F6CDD1Dull + 2 * (uint64_t)i + 1));
      h[i] = stdev * std::sqrt(-2.f * std::log(u1)) * std::cos(6.283185307f * u2);
    }
    t.copy_(from_blob(h.data(), t.shape(), DType::F32, Device::cpu()));
  }
  return t;
}

Tensor rand_uniform(Shape shape, uint64_t seed, float lo, float hi, DType dt, Device dev) {
  Tensor t = empty(std::move(shape), dt, dev);
  if (dev.is_hip()) {
    k::rand_uniform(t.data_ptr(), (int)dt, t.numel(), seed, lo, hi, current_stream());
  } else {
    std::vector<float> h(t.numel());
    for (int64_t i = 0; i < t.numel(); ++i) h[i] = lo + (hi - lo) * u01(mix64(seed * 0x2545F4914F6CDD1Dull + i));
    t.copy_(from_blob(h.data(), t.shape(), DType::F32, Device::cpu()));
  }
  return t;
}

Tensor from_host(const void* src, Shape shape, DType dt, Device dev) {
  Tensor t = empty(shape, dt, dev);
  if (t.numel() == 0) return t;
  if (dev.is_hip()) {
    // stage through pinned memory so the copy is async on the current stream
    void* pin = PinnedAllocator::get().allocate(t.nbytes());
    std::memcpy(pin, src, t.nbytes());
    HIP_OK(hipMemcpyAsync(t.data_ptr(), pin, t.nbytes(), hipMemcpyHostToDevice, current_stream()));
    PinnedAllocator::get().release(pin, current_stream());
  } else {
    std::memcpy(t.data_ptr(), src, t.nbytes());
  }
  return t;
}

// ------------------------------------------------------------------ copies
static k::Desc desc_of(const Tensor& t, const Shape& over) {
  // t viewed over `over` (broadcast: leading dims added, size-1 dims stride 0)
  k::Desc d{};
  d.ptr = t.data_ptr();
  d.dtype = (int)t.dtype();
  d.ndim = (int)over.size();
  MFT_CHECK(d.ndim <= k::kMaxDims, "more than ", k::kMaxDims, " dims");
  const int off = (int)over.size() - t.dim();
  MFT_CHECK(off >= 0, "broadcast: ", t.str(), " has more dims than ", shape_str(over));
  for (int i = 0; i < d.ndim; ++i) {
    d.shape[i] = over[i];
    if (i < off) {
      d.stride[i] = 0;
    } else {
      const int64_t s = t.shape()[i - off];
      MFT_CHECK(s == over[i] || s == 1, "broadcast: ", t.str(), " vs ", shape_str(over));
      d.stride[i] = (s == 1 && over[i] != 1) ? 0 : t.strides()[i - off];
    }
  }
  if (d.ndim == 0) {
    d.ndim = 1;
    d.shape[0] = 1;
    d.stride[0] = 0;
  }
  return d;
}

k::Desc desc(const Tensor& t) { return desc_of(t, t.shape()); }
k::Desc desc_bcast(const Tensor& t, const Shape& over) { return desc_of(t, over); }

Tensor& Tensor::copy_(const Tensor& src) {
  MFT_CHECK(src.numel() == numel() || src.numel() == 1 || src.dim() <= dim(), "copy_: ", src.str(), " -> ", str());
  if (numel() == 0) return *this;
  const bool dh = is_hip(), sh = src.is_hip();
  if (dh && sh) {
    k::copy(desc(*this), desc_bcast(src, shape()), current_stream());
    return *this;
  }
  // host involved: move contiguous bytes of the same dtype, converting on the side that can
  if (!dh && !sh) {
    Tensor s = src;
    if (s.dtype() != dtype() || !s.is_contiguous() || !is_contiguous() || s.numel() != numel()) {
      // host conversion through fp32 / int64
      std::vector<double> tmp(numel());
      Tensor sc = s;
      auto rd = [&](int64_t lin) -> double {
        int64_t off = 0, l = lin;
        const Shape& shp = shape();
        const int o = (int)shp.size() - sc.dim();
        for (int d = (int)shp.size() - 1; d >= 0; --d) {
          const int64_t q = l / shp[d];
          const int64_t idx = l - q * shp[d];
          l = q;
          if (d >= o && sc.shape()[d - o] != 1) off += idx * sc.strides()[d - o];
        }
        const char* p = (const char*)sc.data_ptr();
        switch (sc.dtype()) {
          case DType::F32: return ((const float*)p)[off];
          case DType::BF16: return bf16_to_f32(((const uint16_t*)p)[off]);
          case DType::F16: return f16_to_f32(((const uint16_t*)p)[off]);
          case DType::I32: return ((const int32_t*)p)[off];
          case DType::I64: return (double)((const int64_t*)p)[off];
          default: return ((const uint8_t*)p)[off];
        }
      };
      auto wr = [&](int64_t lin, double v) {
        int64_t off = 0, l = lin;
        for (int d = dim() - 1; d >= 0; --d) {
          const int64_t q = l / shape()[d];
          off += (l - q * shape()[d]) * strides()[d];
          l = q;
        }
        char* p = (char*)data_ptr();
        switch (dtype()) {
          case DType::F32: ((float*)p)[off] = (float)v; break;
          case DType::BF16: ((uint16_t*)p)[off] = f32_to_bf16((float)v); break;
          case DType::F16: ((uint16_t*)p)[off] = f32_to_f16((float)v); break;
          case DType::I32: ((int32_t*)p)[off] = (int32_t)v; break;
          case DType::I64: ((int64_t*)p)[off] = (int64_t)v; break;
          case DType::BOOL: ((uint8_t*)p)[off] = v != 0; break;
          default: ((uint8_t*)p)[off] = (uint8_t)v; break;
        }
      };
      for (int64_t i = 0; i < numel(); ++i) wr(i, rd(i));
      return *this;
    }
    std::memcpy(data_ptr(), src.data_ptr(), nbytes());
    return *this;
  }
  if (dh) {  // H2D: convert / compact on the host, then one async copy, then cast on device
    Tensor hs = src;
    if (!hs.is_contiguous() || hs.numel() != numel()) {
      Tensor c = empty(shape(), hs.dtype(), Device::cpu());
      c.copy_(hs);
      hs = c;
    }
    if (is_contiguous() && hs.dtype() == dtype()) {
      void* pin = PinnedAllocator::get().allocate(nbytes());
      std::memcpy(pin, hs.data_ptr(), nbytes());
      HIP_OK(hipMemcpyAsync(data_ptr(), pin, nbytes(), hipMemcpyHostToDevice, current_stream()));
      PinnedAllocator::get().release(pin, current_stream());
    } else {
      Tensor dev = from_host(hs.data_ptr(), shape(), hs.dtype(), device());
      k::copy(desc(*this), desc(dev), current_stream());
    }
    return *this;
  }
  // D2H: compact + cast on the device, then a synchronous copy
  Tensor ds = src;
  if (!ds.is_contiguous() || ds.dtype() != dtype() || ds.numel() != numel()) {
    Tensor c = empty(shape(), dtype(), src.device());
    c.copy_(ds);
    ds = c;
  }
  if (is_contiguous()) {
    HIP_OK(hipMemcpyAsync(data_ptr(), ds.data_ptr(), nbytes(), hipMemcpyDeviceToHost, current_stream()));
    HIP_OK(hipStreamSynchronize(current_stream()));
  } else {
    Tensor h = empty(shape(), dtype(), Device::cpu());
    HIP_OK(hipMemcpyAsync(h.data_ptr(), ds.data_ptr(), nbytes(), hipMemcpyDeviceToHost, current_stream()));
    HIP_OK(hipStreamSynchronize(current_stream()));
    copy_(h);
  }
  return *this;
}

Tensor Tensor::contiguous() const {
  if (is_contiguous()) return *this;
  Tensor out;
  {
    NoGradGuard ng;
    out = empty(shape(), dtype(), device());
    out.copy_(*this);
  }
  if (needs_grad(*this)) {
    auto node = lambda_node("ContiguousBackward", [](std::vector<Tensor>& g) { return std::vector<Tensor>{g[0]}; });
    connect(node, {*this}, {out});
  }
  return out;
}

Tensor Tensor::clone() const {
  Tensor out;
  {
    NoGradGuard ng;
    out = empty(shape(), dtype(), device());
    out.copy_(*this);
  }
  if (needs_grad(*this)) {
    auto node = lambda_node("CloneBackward", [](std::vector<Tensor>& g) { return std::vector<Tensor>{g[0]}; });
    connect(node, {*this}, {out});
  }
  return out;
}

Tensor Tensor::to(Device dev) const {
  if (device() == dev && (dev.is_hip() || device().pinned == dev.pinned)) return *this;
  Tensor out = empty(shape(), dtype(), dev);
  out.copy_(*this);
  return out;
}

Tensor Tensor::to(DType dt) const {
  if (dtype() == dt) return *this;
  Tensor out;
  {
    NoGradGuard ng;
    out = empty(shape(), dt, device());
    out.copy_(*this);
  }
  if (needs_grad(*this) && (dt == DType::F32 || dt == DType::BF16 || dt == DType::F16)) {
    const DType src_dt = dtype();
    auto node = lambda_node("CastBackward", [src_dt](std::vector<Tensor>& g) {
      return std::vector<Tensor>{g[0].defined() ? g[0].to(src_dt) : Tensor()};
    });
    connect(node, {*this}, {out});
  }
  return out;
}

Tensor& Tensor::zero_() { return fill_(0.0); }

Tensor& Tensor::fill_(double v) {
  if (numel() == 0) return *this;
  if (is_hip()) {
    k::fill(desc(*this), v, current_stream());
  } else {
    Tensor one = empty({1}, DType::F32, Device::cpu());
    *one.data<float>() = (float)v;
    if (dtype() == DType::I64 || dtype() == DType::I32) {
      for (int64_t i = 0; i < numel(); ++i) {
        if (dtype() == DType::I64) data<int64_t>()[i] = (int64_t)v;
        else data<int32_t>()[i] = (int32_t)v;
      }
    } else {
      copy_(one);
    }
  }
  return *this;
}

std::vector<float> Tensor::to_vector_f32() const {
  Tensor h = empty(shape(), DType::F32, Device::cpu());
  h.copy_(*this);
  return std::vector<float>(h.data<float>(), h.data<float>() + h.numel());
}

double Tensor::item() const {
  MFT_CHECK(numel() == 1, "item(): ", str(), " is not a scalar");
  if (dtype() == DType::I64) {
    Tensor h = empty({1}, DType::I64, Device::cpu());
    h.copy_(*this);
    return (double)*h.data<int64_t>();
  }
  return to_vector_f32()[0];
}

// ------------------------------------------------------------------ autograd accessors
Tensor& Tensor::requires_grad_(bool on) {
  MFT_CHECK(!on || dtype() == DType::F32 || dtype() == DType::BF16 || dtype() == DType::F16,
            "requires_grad on a non-float tensor");
  p_->requires_grad = on;
  return *this;
}
Tensor Tensor::grad() const { return p_->ag ? p_->ag->grad : Tensor(); }
void Tensor::set_grad(const Tensor& g) { meta(p_.get()).grad = g; }
void Tensor::retain_grad() { meta(p_.get()).retain_grad = true; }
bool Tensor::is_leaf() const { return !(p_->ag && p_->ag->grad_fn); }
void Tensor::backward(const Tensor& g) const {
  if (g.defined()) eng::backward({*this}, {g});
  else eng::backward({*this}, {});
}

// ------------------------------------------------------------------ host conversions
uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
uint16_t f32_to_f16(float f) {  // IEEE half, round to nearest even
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t mant = x & 0x7fffffu;
  int exp = (int)((x >> 23) & 0xff);
  if (exp == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0u));
  exp = exp - 127 + 15;
  if (exp >= 0x1f) return (uint16_t)(sign | 0x7c00u);
  if (exp <= 0) {
    if (exp < -10) return (uint16_t)sign;
    mant |= 0x800000u;
    const int shift = 14 - exp;
    uint32_t h = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((uint32_t)exp << 10) | (mant >> 13);
  const uint32_t rem = mant & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) ++h;
  return (uint16_t)(sign | h);
}
float f16_to_f32(uint16_t v) {
  const uint32_t sign = (uint32_t)(v & 0x8000u) << 16;
  uint32_t exp = (v >> 10) & 0x1f, mant = v & 0x3ffu, x;
  if (exp == 0) {
    if (mant == 0) {
      x = sign;
    } else {
      exp = 127 - 15 + 1;
      while (!(mant & 0x400u)) {
        mant <<= 1;
        --exp;
      }
      x = sign | (exp << 23) | ((mant & 0x3ffu) << 13);
    }
  } else if (exp == 0x1f) {
    x = sign | 0x7f800000u | (mant << 13);
  } else {
    x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
  }
  float f;
  std::memcpy(&f, &x, 4);
  return f;
}

}  // namespace eng
}  // namespace mft
