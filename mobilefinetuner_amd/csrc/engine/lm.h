// libmft engine: the interface the Trainer drives (GPT-2 and Gemma-3 implement it).
//
// Reference: the reference has one trainer per family (gpt2_lora_finetune/main.cpp:561-684 for
// GPT-2, GemmaLoRATrainer optim/gemma_trainer.cpp:18-233 for Gemma); here one Trainer (engine/trainer.h)
// runs either model through this interface: a mean-token-NLL loss with autograd, an eval NLL sum
// without it, the trainable parameters in checkpoint order, the LoRA-dropout step counter.
#pragma once
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "engine/nn.h"

namespace mft {
namespace eng {

class LanguageModel {
 public:
  // (the process-wide LoRA weight-prep registry holds this model's tensors: released with it)
  virtual ~LanguageModel() { lora_prep_reset(); }
  // mean token NLL of one micro-batch (ids / labels [B, S], labels already shifted, -100 ignored);
  // a trainable tied embedding's gradient is produced inside the CE scaled by w_grad_scale
  virtual Tensor loss(const Tensor& ids, const Tensor& labels, float w_grad_scale = 1.f) = 0;
  // (sum of token NLL, number of valid tokens) without gradients -- evaluation
  virtual std::pair<Tensor, Tensor> nll(const Tensor& ids, const Tensor& labels) = 0;
  virtual std::vector<std::pair<std::string, Param*>> trainable() = 0;
  virtual size_t num_parameters() const = 0;
  // final hidden states [B*S, C] (after the last norm) and the tied output embedding [Vpad, C]
  virtual Tensor hidden(const Tensor& ids) = 0;
  virtual Param& output_embedding() = 0;
  virtual int vocab() const = 0;
  bool training = true;
  // false after merge_lora(+1): the adapters live in the base weights, the forward skips them
  bool lora_enabled = true;
  Tensor dropout_ctr;    // device int64 step counter (fresh LoRA-dropout masks per step)
  int64_t ce_chunk = 0;  // LM-head CE rows per fused call (default_ce_chunk)
  // --loss_reduction sum|sum_debug (reference core/lm_loss.cpp:184-192): loss() returns the SUM of
  // the token NLL and its gradient is not divided by the valid-token count
  bool loss_sum = false;
  // --activation_checkpointing: each block's activations are recomputed in the backward
  // (autograd.h checkpoint()) instead of kept -- one more forward for O(blocks) less memory
  bool grad_checkpoint = false;
  // --attn_impl naive: the materialized masked-softmax attention (attention_ref) in place of the flash
  // kernels (--dtype fp32 always takes it)
  bool attn_naive = false;
  // the composite path (--dtype fp32 / --attn_impl naive) reads host values (dropout step, id checks,
  // mask tables) during the step: it runs eagerly, never inside a hipGraph capture
  bool capturable() const { return !attn_naive && compute_dtype() != DType::F32; }
  // alignment harness: hidden() copies the listed layers' MLP outputs (after the post-FF norm)
  std::vector<int> capture_layers;
  std::map<int, Tensor> captured;

 protected:
  // the adapters of one projection as the forward sees them (none while merged)
  std::vector<LoraAdapter>& active(std::vector<LoraAdapter>& ads) { return lora_enabled ? ads : no_adapters_; }
  std::vector<LoraAdapter> no_adapters_;
};

// rows of the fused LM-head CE per call: one [rows, Vpad] bf16 E workspace within a 4 GiB budget
// (MFT_CE_BUDGET_GB; MFT_CE_CHUNK overrides), at most 65536 rows (ops/functional.default_ce_chunk)
int64_t default_ce_chunk(int vocab_padded);

// FNV-1a of an adapter's checkpoint name: its stable LoRA-dropout salt
uint32_t adapter_salt(const std::string& name);
// LoRA adapter over output columns [col0, col0 + n) of a frozen Linear: A [r, in] = A_init (fp32
// master + bf16 shadow), B [r, n] = 0
LoraAdapter make_adapter(int col0, int n, int r, const Tensor& A_init, float dropout, const std::string& name);

}  // namespace eng
}  // namespace mft
