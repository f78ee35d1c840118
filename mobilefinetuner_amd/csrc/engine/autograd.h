// libmft engine: reverse-mode autograd (tape of Nodes, dependency-counted replay).
//
// Replaces the reference's global Engine (operators/finetune_ops/core/autograd_engine.h:36-143,
// autograd_engine.cpp:15-268) and its BackwardFunction catalog base (core/backward_functions.h).
// Kept: a node per differentiable op, topological replay from a scalar root seeded with ones,
// set_enabled(false)-style no-grad (NoGradGuard).  Changed by design:
//   * leaf gradients ACCUMULATE (+=) across backward calls / micro-batches; the reference
//     overwrites them with set_grad (autograd_engine.cpp:243), which breaks accumulation;
//   * edges only to inputs that require grad (the reference links every input, :57-59);
//   * nodes replay in reverse creation order among the ready set (sequence numbers), so the
//     backward kernel order mirrors the forward tape and saved activations die as early as possible;
//   * grad-ready hooks fire once a leaf's gradient is final for this backward (all of its consumer
//     nodes ran): the data-parallel bucketed all-reduce and ZeRO reduce-scatter hang off these;
//   * a fused op may accumulate straight into a leaf's gradient buffer (accumulate_grad) and
//     return no tensor for it -- the flat fp32 grad buffers of the optimizer are written in place by
//     the GEMM / LoRA kernels instead of materialising per-op gradients.
#pragma once
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "engine/tensor.h"

namespace mft {
namespace eng {

struct Node;

struct Edge {
  std::shared_ptr<Node> fn;          // producer of a non-leaf input
  int output_nr = 0;                 // which output of fn
  std::shared_ptr<TensorImpl> leaf;  // leaf input (requires_grad, no grad_fn)
  bool valid() const { return fn || leaf; }
};

struct Node : std::enable_shared_from_this<Node> {
  std::string name;
  uint64_t seq = 0;
  int n_outputs = 1;
  std::vector<Edge> next;                             // one per differentiable input slot
  std::vector<std::weak_ptr<TensorImpl>> outputs;     // for retain_grad only
  // grads of this node's outputs (undefined = zero) -> grads of its inputs (undefined = none,
  // or already accumulated into the leaf by the op itself)
  virtual std::vector<Tensor> apply(std::vector<Tensor>& grad_outputs) = 0;
  virtual ~Node() = default;
};

struct AutogradMeta {
  Tensor grad;                      // accumulated gradient (leaves, retain_grad tensors)
  std::shared_ptr<Node> grad_fn;    // producer (non-leaf)
  int output_nr = 0;
  bool retain_grad = false;
  std::vector<std::function<void(TensorImpl*)>> ready_hooks;  // leaves: grad final for this backward
};

// ---- grad mode
bool grad_enabled();
void set_grad_enabled(bool on);
struct NoGradGuard {
  bool prev;
  NoGradGuard() : prev(grad_enabled()) { set_grad_enabled(false); }
  ~NoGradGuard() { set_grad_enabled(prev); }
};

AutogradMeta& meta(TensorImpl* t);
bool needs_grad(const Tensor& t);  // grad mode on and t requires grad
bool any_needs_grad(const std::vector<Tensor>& ts);

// Wire `node` to the differentiable `inputs` (one edge slot per input, in order) and make every
// output require grad with this node as grad_fn.  Returns false (node dropped) when no input needs
// a gradient or grad mode is off.
bool connect(const std::shared_ptr<Node>& node, const std::vector<Tensor>& inputs, const std::vector<Tensor>& outputs,
             bool force = false);  // force: record the node even when no input needs a gradient

// g accumulated (+=, with dtype cast) into leaf t's gradient, allocated zero-filled on first use
// unless a gradient buffer was installed (set_grad with a view into a flat buffer).
void accumulate_grad(const Tensor& t, const Tensor& g, float alpha = 1.f);
void accumulate_grad(TensorImpl* t, const Tensor& g, float alpha = 1.f);
// a leaf's grad buffer (allocating the fp32 / same-dtype zero buffer if absent)
Tensor grad_buffer(const Tensor& t);

void add_ready_hook(const Tensor& leaf, std::function<void(TensorImpl*)> fn);

// run backward from `roots` (scalar roots may omit their seed gradient)
void backward(const std::vector<Tensor>& roots, const std::vector<Tensor>& grads = {});

// zero-copy view bookkeeping used by Tensor::view / slice / transpose / ...: when `in` needs grad,
// `out` gets a node that maps its gradient back (`inverse` rebuilds the same view on a tensor of
// in's shape; `full` = the view covers every element of `in`, so no zero fill is needed)
void record_view(const Tensor& in, const Tensor& out, std::function<Tensor(const Tensor&)> reapply,
                 std::function<Tensor(const Tensor&)> inverse, bool full);

// Activation checkpointing (the Python models use torch.utils.checkpoint): fn(inputs)
// runs WITHOUT recording and only the inputs are kept; the backward re-runs fn from them with
// recording on and back-propagates the incoming gradients through that recomputed graph (a nested
// backward: the parameters' gradients accumulate and their grad-ready hooks fire there), returning
// the inputs' gradients.  fn must be a pure function of its inputs and state that does not change
// before the backward (weights; the LoRA-dropout counter) -- it is called twice.
using CheckpointFn = std::function<std::vector<Tensor>(const std::vector<Tensor>&)>;
std::vector<Tensor> checkpoint(CheckpointFn fn, const std::vector<Tensor>& inputs);

// Node built from lambdas (for simple ops)
struct LambdaNode : Node {
  std::function<std::vector<Tensor>(std::vector<Tensor>&)> fn;
  std::vector<Tensor> apply(std::vector<Tensor>& g) override { return fn(g); }
};
std::shared_ptr<LambdaNode> lambda_node(const std::string& name,
                                        std::function<std::vector<Tensor>(std::vector<Tensor>&)> fn);

}  // namespace eng
}  // namespace mft
