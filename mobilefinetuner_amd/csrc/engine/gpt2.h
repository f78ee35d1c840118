// libmft engine: GPT-2 (small ... XL) with LoRA adapters, on the fused ops of nn.h.
//
// Reference: GPT2Config / GPT2Model (operators/finetune_ops/graph/gpt2_model.h:50-186,
// gpt2_model.cpp:121-861), LoraSpec / LoraInjector (graph/lora_injector.h:19-191,
// lora_injector.cpp:48-148), LoraSaver (graph/lora_saver.cpp:123-452), GPT2KeyMapper
// (graph/safetensors_loader.cpp:294-336).  Same graph as the Python package's models/gpt2.py:
// embedding (+wpe) -> per block [LN1 -> c_attn (LoRA, augmented K) -> flash attention on the
// packed qkv -> c_proj (LoRA) -> residual+LN2 -> fc+GELU -> proj] -> residual+LN_f -> tied LM head
// + vocab-chunked CE.  Weights are [out, in] (HF Conv1D [in, out] transposed once at load).
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "engine/lm.h"
#include "engine/weight_stream.h"

namespace mft {
namespace eng {

struct GPT2Config {
  int vocab_size = 50257, n_positions = 1024, n_embd = 768, n_layer = 12, n_head = 12;
  float eps = 1e-5f, init_range = 0.02f;
  int vocab_padded() const { return (vocab_size + 127) / 128 * 128; }
  int head_dim() const { return n_embd / n_head; }
  static GPT2Config preset(const std::string& name);
  static GPT2Config from_json(const std::string& path);
};

struct LoraSpec {
  int rank = 8;
  float alpha = 16.f, dropout = 0.f;
  bool split_qkv = false;
  std::vector<std::string> targets{"AttnQKV", "AttnProj"};  // + MlpFcIn, MlpFcOut
  std::vector<int> layers;                                  // empty = all
  uint64_t seed = 42;
  float scale() const { return alpha / (float)rank; }
  bool has(const std::string& t) const;
};

struct GPT2Block {
  Param ln1_w, ln1_b, attn_w, attn_b, proj_w, proj_b, ln2_w, ln2_b, fc_w, fc_b, mproj_w, mproj_b;
  std::vector<LoraAdapter> lqkv, lproj, lfc, lfcout;
  std::vector<std::string> names_qkv, names_proj, names_fc, names_fcout;  // checkpoint keys
  Tensor waug_qkv, waug_proj;  // augmented weights of the LoRA'd attention projections
};

class GPT2 : public LanguageModel {
 public:
  explicit GPT2(const GPT2Config& cfg);
  const GPT2Config& cfg() const { return cfg_; }
  // HF init: N(0, 0.02), residual projections N(0, 0.02 / sqrt(2L)), zero biases, wpe N(0, 0.01);
  // counter-based RNG (engine/tensor_kernels.hip) seeded per tensor
  void init_random(uint64_t seed);
  // <dir>/model.safetensors (+ config.json): HF GPT-2 keys (optional "transformer." prefix)
  void load_hf(const std::string& dir);
  void save_hf(const std::string& path);  // full-model writer (gpt2_full_finetune)
  // LoRA: reference init A ~ U(+-sqrt(6/(in+r))) seeded 42+in+out, B = 0
  void inject_lora(const LoraSpec& spec);
  void load_lora(const std::string& path);  // reference checkpoint layout (attach_from_state)
  void save_lora(const std::string& path);  // byte-compatible with graph/lora_saver.cpp
  void set_full_finetune();                 // every parameter trainable (fp32 master + bf16 shadow)
  // trainable parameters in a fixed order (name, param)
  std::vector<std::pair<std::string, Param*>> trainable() override;
  std::vector<std::pair<std::string, Param*>> all_params();
  // mean token NLL of one micro-batch (ids / labels [B, S], labels already shifted, -100 ignored)
  Tensor loss(const Tensor& ids, const Tensor& labels, float w_grad_scale = 1.f) override;
  std::pair<Tensor, Tensor> nll(const Tensor& ids, const Tensor& labels) override;  // (sum, count), no grad
  Tensor hidden(const Tensor& ids) override;
  Param& output_embedding() override { return wte_; }
  int vocab() const override { return cfg_.vocab_size; }
  void merge_lora(float sign);
  const LoraSpec& lora_spec() const { return spec_; }
  size_t num_parameters() const override;
  // --shard_enable: every block's frozen weights into the host tier, streamed through device slots
  // within budget_bytes (weight_stream.h); LoRA projections then take the plain (non-augmented) path
  void enable_weight_streaming(size_t budget_bytes, const DiskTier& disk = {});
  const WeightStreamer* streamer() const { return streamer_.get(); }
  // ZeRO-3 (engine/zero3.h): units[0] = {wte, wpe}, units[1 + i] = block i's bf16-compute
  // weights and biases; rep = the fp32-compute LayerNorm parameters (replicated)
  void zero3_layout(std::vector<std::vector<std::pair<std::string, Param*>>>& units,
                    std::vector<std::pair<std::string, Param*>>& rep);
  // the partitioner that gathers each block's weights before hidden() uses them (not owned)
  void set_block_provider(BlockProvider* p) { provider_ = p; }

 private:
  void alloc();
  // transformer block i: (residual x, normed h) -> (x, h normed for the next block)
  std::pair<Tensor, Tensor> block(int i, const Tensor& x, const Tensor& h, int64_t B, int64_t S);
  // the composite path (--dtype fp32 / --attn_impl naive): final hidden states and the full logits
  Tensor hidden_ref(const Tensor& ids);
  Tensor logits_ref(const Tensor& h);
  GPT2Config cfg_;
  LoraSpec spec_;
  bool lora_ = false, full_ = false;
  Param wte_, wpe_, lnf_w_, lnf_b_;
  std::vector<GPT2Block> blocks_;
  std::unique_ptr<WeightStreamer> streamer_;
  BlockProvider* provider_ = nullptr;
  void make_trainable(Param& p);
};

}  // namespace eng
}  // namespace mft
