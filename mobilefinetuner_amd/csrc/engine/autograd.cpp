// libmft engine: autograd replay (see autograd.h).
#include "engine/autograd.h"

#include <algorithm>
#include <queue>
#include <unordered_map>
#include <unordered_set>

#include "engine/tensor_kernels.h"
#include "engine/ops.h"

namespace mft {
namespace eng {

namespace {
thread_local bool t_grad = true;
uint64_t g_seq = 0;
}  // namespace

bool grad_enabled() { return t_grad; }
void set_grad_enabled(bool on) { t_grad = on; }

AutogradMeta& meta(TensorImpl* t) {
  if (!t->ag) t->ag = std::make_unique<AutogradMeta>();
  return *t->ag;
}

bool needs_grad(const Tensor& t) { return t_grad && t.defined() && t.requires_grad(); }
bool any_needs_grad(const std::vector<Tensor>& ts) {
  if (!t_grad) return false;
  for (auto& t : ts)
    if (t.defined() && t.requires_grad()) return true;
  return false;
}

bool connect(const std::shared_ptr<Node>& node, const std::vector<Tensor>& inputs, const std::vector<Tensor>& outputs,
             bool force) {
  if (!(force ? t_grad : any_needs_grad(inputs))) return false;
  node->seq = ++g_seq;
  node->next.clear();
  for (auto& in : inputs) {
    Edge e;
    if (in.defined() && in.requires_grad()) {
      TensorImpl* ti = in.impl();
      if (ti->ag && ti->ag->grad_fn) {
        e.fn = ti->ag->grad_fn;
        e.output_nr = ti->ag->output_nr;
      } else {
        e.leaf = in.impl_ptr();
      }
    }
    node->next.push_back(e);
  }
  node->n_outputs = (int)outputs.size();
  node->outputs.clear();
  for (int i = 0; i < (int)outputs.size(); ++i) {
    const Tensor& o = outputs[i];
    if (!o.defined()) {
      node->outputs.emplace_back();
      continue;
    }
    o.impl()->requires_grad = true;
    auto& m = meta(o.impl());
    m.grad_fn = node;
    m.output_nr = i;
    node->outputs.push_back(o.impl_ptr());
  }
  return true;
}

std::shared_ptr<LambdaNode> lambda_node(const std::string& name,
                                        std::function<std::vector<Tensor>(std::vector<Tensor>&)> fn) {
  auto n = std::make_shared<LambdaNode>();
  n->name = name;
  n->fn = std::move(fn);
  return n;
}

void add_ready_hook(const Tensor& leaf, std::function<void(TensorImpl*)> fn) {
  meta(leaf.impl()).ready_hooks.push_back(std::move(fn));
}

Tensor grad_buffer(const Tensor& t) {
  auto& m = meta(t.impl());
  if (!m.grad.defined()) {
    NoGradGuard ng;
    m.grad = zeros(t.shape(), t.dtype() == DType::BF16 || t.dtype() == DType::F16 ? DType::F32 : t.dtype(), t.device());
  }
  return m.grad;
}

// sum g into buf (+=): buf may be a strided view (flat-buffer slice); g is broadcast-reduced when
// it carries extra leading dims or size-1 broadcast dims
static void add_into(Tensor& buf, const Tensor& g, float alpha) {
  NoGradGuard ng;
  if (!buf.is_hip()) {  // host tensors (engine_host_selftest: the tape under ASan / UBSan), via fp32
    MFT_CHECK(!g.is_hip() && g.dim() <= buf.dim(), "add_into: host gradient ", g.str(), " into ", buf.str());
    Tensor a = empty(buf.shape(), DType::F32, Device::cpu()), b = empty(buf.shape(), DType::F32, Device::cpu());
    a.copy_(buf);
    b.copy_(g);  // (broadcast over leading / size-1 dims)
    float* pa = a.data<float>();
    const float* pb = b.data<float>();
    for (int64_t i = 0; i < a.numel(); ++i) pa[i] += alpha * pb[i];
    buf.copy_(a);
    return;
  }
  Tensor gg = g;
  if (gg.shape() != buf.shape()) gg = sum_to(gg, buf.shape());
  k::axpy(desc(buf), desc_bcast(gg, buf.shape()), alpha, 1, current_stream());
}

void accumulate_grad(TensorImpl* t, const Tensor& g, float alpha) {
  if (!g.defined()) return;
  auto& m = meta(t);
  if (!m.grad.defined()) {
    NoGradGuard ng;
    Shape shp = t->shape;
    const DType dt = (t->dtype == DType::BF16 || t->dtype == DType::F16) ? DType::F32 : t->dtype;
    m.grad = zeros(shp, dt, g.device());
  }
  add_into(m.grad, g, alpha);
}

void accumulate_grad(const Tensor& t, const Tensor& g, float alpha) { accumulate_grad(t.impl(), g, alpha); }

// ------------------------------------------------------------------ activation checkpointing
std::vector<Tensor> checkpoint(CheckpointFn fn, const std::vector<Tensor>& inputs) {
  if (!t_grad) return fn(inputs);
  std::vector<Tensor> saved;
  std::vector<char> need;
  for (auto& t : inputs) {
    saved.push_back(t.defined() ? t.detach() : Tensor());
    need.push_back(t.defined() && t.requires_grad());
  }
  std::vector<Tensor> outs;
  {
    NoGradGuard ng;
    outs = fn(saved);
  }
  auto n = lambda_node("CheckpointBackward", [fn, saved, need](std::vector<Tensor>& g) {
    std::vector<Tensor> xin;
    for (size_t i = 0; i < saved.size(); ++i) {
      Tensor t = saved[i].defined() ? saved[i].alias() : Tensor();
      if (need[i]) {
        t.requires_grad_(true);
        t.set_grad(zeros(t.shape(), t.dtype(), t.device()));  // same dtype as the forward's tensor
      }
      xin.push_back(t);
    }
    std::vector<Tensor> re;
    {
      const bool prev = grad_enabled();
      set_grad_enabled(true);
      re = fn(xin);
      set_grad_enabled(prev);
    }
    std::vector<Tensor> roots, seeds;
    for (size_t k = 0; k < re.size() && k < g.size(); ++k)
      if (g[k].defined() && re[k].defined() && re[k].requires_grad()) {
        roots.push_back(re[k]);
        seeds.push_back(g[k]);
      }
    if (!roots.empty()) backward(roots, seeds);
    std::vector<Tensor> res;
    for (size_t i = 0; i < xin.size(); ++i) res.push_back(need[i] ? xin[i].grad() : Tensor());
    return res;
  });
  std::vector<Tensor> alias_outs;
  for (auto& o : outs) alias_outs.push_back(o.defined() ? o.alias() : Tensor());
  connect(n, inputs, alias_outs, /*force=*/true);
  return alias_outs;
}

// ------------------------------------------------------------------ views
namespace {
struct ViewNode : Node {
  Shape in_shape;
  DType in_dtype;
  Device dev;
  std::function<Tensor(const Tensor&)> reapply, inverse;
  bool full = false;
  std::vector<Tensor> apply(std::vector<Tensor>& g) override {
    if (!g[0].defined()) return {Tensor()};
    NoGradGuard ng;
    if (inverse) return {inverse(g[0])};
    Tensor gi = zeros(in_shape, g[0].dtype(), dev);
    Tensor region = reapply(gi);
    region.copy_(g[0]);
    return {gi};
  }
};
}  // namespace

void record_view(const Tensor& in, const Tensor& out, std::function<Tensor(const Tensor&)> reapply,
                 std::function<Tensor(const Tensor&)> inverse, bool full) {
  auto n = std::make_shared<ViewNode>();
  n->name = "ViewBackward";
  n->in_shape = in.shape();
  n->in_dtype = in.dtype();
  n->dev = in.device();
  n->reapply = std::move(reapply);
  n->inverse = std::move(inverse);
  n->full = full;
  connect(n, {in}, {out});
}

// ------------------------------------------------------------------ replay
void backward(const std::vector<Tensor>& roots, const std::vector<Tensor>& grads) {
  NoGradGuard ng;  // backward ops are not recorded
  // 1. discover the graph: dependency counts per node, use counts per leaf
  std::unordered_map<Node*, int> deps;
  std::unordered_map<TensorImpl*, int> leaf_uses;
  std::unordered_map<Node*, std::shared_ptr<Node>> keep;
  std::vector<Node*> stack;
  auto visit_root = [&](const std::shared_ptr<Node>& n) {
    if (!n || keep.count(n.get())) return;
    keep[n.get()] = n;
    deps[n.get()];
    stack.push_back(n.get());
  };
  for (auto& r : roots) {
    MFT_CHECK(r.defined() && r.requires_grad(), "backward: root does not require grad");
    if (r.impl()->ag && r.impl()->ag->grad_fn) visit_root(r.impl()->ag->grad_fn);
  }
  while (!stack.empty()) {
    Node* n = stack.back();
    stack.pop_back();
    for (auto& e : n->next) {
      if (e.fn) {
        deps[e.fn.get()]++;
        if (!keep.count(e.fn.get())) {
          keep[e.fn.get()] = e.fn;
          stack.push_back(e.fn.get());
        }
      } else if (e.leaf) {
        leaf_uses[e.leaf.get()]++;
      }
    }
  }
  // 2. seed
  std::unordered_map<Node*, std::vector<Tensor>> inbuf;
  auto add_grad = [&](Node* n, int slot, const Tensor& g) {
    auto& v = inbuf[n];
    if (v.empty()) v.resize(n->n_outputs);
    if (!g.defined()) return;
    if (!v[slot].defined()) {
      v[slot] = g;
    } else {
      // sum (out of place: g may alias a caller's buffer)
      Tensor s = empty(v[slot].shape(), v[slot].dtype(), v[slot].device());
      s.copy_(v[slot]);
      add_into(s, g, 1.f);
      v[slot] = s;
    }
  };
  for (size_t i = 0; i < roots.size(); ++i) {
    const Tensor& r = roots[i];
    Tensor g = i < grads.size() ? grads[i] : Tensor();
    if (!g.defined()) {
      MFT_CHECK(r.numel() == 1, "backward: implicit gradient only for scalar roots (got ", r.str(), ")");
      g = ones(r.shape(), r.dtype(), r.device());
    }
    if (r.impl()->ag && r.impl()->ag->grad_fn) {
      add_grad(r.impl()->ag->grad_fn.get(), r.impl()->ag->output_nr, g);
    } else {
      accumulate_grad(r, g);
    }
  }
  // 3. replay: ready nodes by descending sequence number (reverse tape order)
  auto cmp = [](Node* a, Node* b) { return a->seq < b->seq; };
  std::priority_queue<Node*, std::vector<Node*>, decltype(cmp)> ready(cmp);
  for (auto& r : roots)
    if (r.impl()->ag && r.impl()->ag->grad_fn && deps[r.impl()->ag->grad_fn.get()] == 0)
      ready.push(r.impl()->ag->grad_fn.get());
  std::unordered_set<Node*> queued;
  auto fire_leaf = [&](TensorImpl* leaf) {
    auto it = leaf_uses.find(leaf);
    if (it == leaf_uses.end()) return;
    if (--it->second == 0 && leaf->ag) {
      for (auto& h : leaf->ag->ready_hooks) h(leaf);
    }
  };
  while (!ready.empty()) {
    Node* n = ready.top();
    ready.pop();
    if (queued.count(n)) continue;
    queued.insert(n);
    auto& gin = inbuf[n];
    if (gin.empty()) gin.resize(n->n_outputs);
    // retain_grad on this node's outputs
    for (int i = 0; i < (int)n->outputs.size() && i < (int)gin.size(); ++i) {
      auto o = n->outputs[i].lock();
      if (o && o->ag && o->ag->retain_grad && gin[i].defined()) {
        if (!o->ag->grad.defined()) o->ag->grad = gin[i].clone();
        else add_into(o->ag->grad, gin[i], 1.f);
      }
    }
    std::vector<Tensor> gout = n->apply(gin);
    inbuf.erase(n);
    MFT_CHECK(gout.size() == n->next.size() || gout.empty(), "node ", n->name, " returned ", gout.size(),
              " grads for ", n->next.size(), " inputs");
    for (size_t i = 0; i < n->next.size(); ++i) {
      const Edge& e = n->next[i];
      const Tensor g = i < gout.size() ? gout[i] : Tensor();
      if (e.fn) {
        add_grad(e.fn.get(), e.output_nr, g);
        if (--deps[e.fn.get()] == 0) ready.push(e.fn.get());
      } else if (e.leaf) {
        if (g.defined()) accumulate_grad(e.leaf.get(), g);
        fire_leaf(e.leaf.get());
      }
    }
  }
}

}  // namespace eng
}  // namespace mft
