// libmft engine: Gemma-3 text models (270M / 1B) with LoRA adapters, on the fused ops of nn.h.
//
// Reference: GemmaTextConfig / GemmaModel (operators/finetune_ops/graph/gemma_model.h:17-178,
// gemma_model.cpp:138-944), GemmaLoraInjector (graph/gemma_lora_injector.h:9-56,
// gemma_lora_injector.cpp:30-216).  Same graph as the Python package's models/gemma3.py:
// embedding x bf16(sqrt(H)) -> per layer [RMSNorm(1+w) -> q|k|v GEMM (LoRA slices) -> fused
// q/k RMSNorm + RoPE (theta 1e6 global with linear scaling, 1e4 on sliding layers) + causal GQA
// flash attention (sliding window 512 on "sliding_attention" layers), scale
// query_pre_attn_scalar^-1/2 -> o_proj -> post-attn norm -> residual + pre-ffn norm -> gate|up GEMM
// -> GeGLU -> down -> post-ffn norm -> residual + next input norm] -> final norm -> LM head tied to
// the (padded) embedding + fused CE: no transposed embedding copy (reference :687-694), no logits.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "engine/lm.h"
#include "engine/weight_stream.h"

namespace mft {
namespace eng {

struct Gemma3Config {
  int vocab_size = 262144, hidden = 640, intermediate = 2048, n_layer = 18, n_head = 4, n_kv = 1, head_dim = 256;
  float eps = 1e-6f, rope_theta = 1e6f, rope_local = 1e4f, rope_scaling = 1.f, query_pre_attn_scalar = 256.f;
  int sliding_window = 512, max_positions = 32768;
  int bos_id = 2, eos_id = 1, pad_id = 0;
  float init_range = 0.02f;
  int act = 0;                // 0 GELU-tanh (gelu_pytorch_tanh), 1 SiLU
  std::vector<bool> sliding;  // per layer: "sliding_attention"
  int vocab_padded() const { return (vocab_size + 127) / 128 * 128; }
  static Gemma3Config preset(const std::string& name);
  static Gemma3Config from_json(const std::string& path);  // HF config.json (text_config nesting ok)
};

// Gemma LoRA targets: q_proj k_proj v_proj o_proj gate_proj up_proj down_proj
struct GemmaLoraSpec {
  int rank = 8;
  float alpha = 32.f, dropout = 0.1f;
  std::vector<std::string> targets{"q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"};
  std::vector<int> layers;  // empty = all
  uint64_t seed = 42;
  float scale() const { return alpha / (float)rank; }
  bool has(const std::string& t) const;
  // preset (full / full_attn_mlp / attn / attention_only / light / attention_light) or a csv of
  // q,k,v,o,gate,up,down (optionally with the _proj suffix)
  static std::vector<std::string> parse_targets(const std::string& csv_or_preset);
};

struct Gemma3Layer {
  Param in_norm, qkv_w, o_w, q_norm, k_norm, post_attn_norm, pre_ff_norm, gu_w, down_w, post_ff_norm;
  std::vector<LoraAdapter> lqkv, lo, lgu, ldown;
  std::vector<std::string> names_qkv, names_o, names_gu, names_down;  // checkpoint stems
  Tensor waug_qkv, waug_o, waug_gu, waug_down;                       // augmented weights (LoRA'd)
  bool sliding = false;
};

class Gemma3 : public LanguageModel {
 public:
  explicit Gemma3(const Gemma3Config& cfg);
  const Gemma3Config& cfg() const { return cfg_; }
  void init_random(uint64_t seed);  // N(0, 0.02) matrices, zero norm weights (offset 1), zero pad rows
  // <dir>/model.safetensors (or a .safetensors path): HF Gemma3ForCausalLM / Gemma3TextModel keys
  void load_hf(const std::string& dir);
  void inject_lora(const GemmaLoraSpec& spec);
  void load_lora(const std::string& path);  // reference key layout, A [r, in], B [out, r]
  void save_lora(const std::string& path);  // byte-compatible with io/lora_checkpoint.save_lora
  std::vector<std::pair<std::string, Param*>> trainable() override;
  Tensor loss(const Tensor& ids, const Tensor& labels, float w_grad_scale = 1.f) override;
  std::pair<Tensor, Tensor> nll(const Tensor& ids, const Tensor& labels) override;
  Tensor hidden(const Tensor& ids) override;
  // the scaled token embeddings the first layer sees ([B, S, H], bf16; no autograd) -- the
  // reference's --dump_embedding tensor (graph/gemma_model.cpp:588-597)
  Tensor embed_tokens(const Tensor& ids);
  Param& output_embedding() override { return embed_; }
  int vocab() const override { return cfg_.vocab_size; }
  void merge_lora(float sign);
  size_t num_parameters() const override;
  const GemmaLoraSpec& lora_spec() const { return spec_; }
  // --shard_enable: the layers' frozen projection weights streamed from pinned host memory through
  // device slots within budget_bytes (weight_stream.h); LoRA projections take the plain path
  void enable_weight_streaming(size_t budget_bytes, const DiskTier& disk = {});
  const WeightStreamer* streamer() const { return streamer_.get(); }
  bool interleaved_rope = false;  // reference RoPE pairing

 private:
  void alloc();
  std::pair<Tensor, Tensor> rope(bool local, int S);
  // decoder layer i: (residual x, normed h) -> (x, h normed for the next layer)
  std::pair<Tensor, Tensor> layer(int i, const Tensor& x, const Tensor& h, int64_t B, int64_t S);
  // the composite path (--dtype fp32): final hidden states and the full logits
  Tensor hidden_ref(const Tensor& ids);
  Tensor logits_ref(const Tensor& h);
  Gemma3Config cfg_;
  GemmaLoraSpec spec_;
  Param embed_, final_norm_;
  std::vector<Gemma3Layer> layers_;
  std::unique_ptr<WeightStreamer> streamer_;
  float embed_scale_ = 1.f;
  std::map<int, std::pair<Tensor, Tensor>> rope_;  // key: local ? 1 : 0 -> (cos, sin) [n, D/2]
  int rope_len_ = 0;
};

}  // namespace eng
}  // namespace mft
