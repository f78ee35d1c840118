// Native CLI `eval_ppl` (GPT-2, or Gemma-3 with --model_type gemma) on the libmft engine: token-weighted perplexity of a WikiText-2
// split with the fused LM head (per-tile softmax statistics in the GEMM epilogue; no logits are
// stored), optional LoRA adapter (merged into the weights by default), data-parallel over RCCL
// ranks (each rank scores its shard; the sums are all-reduced).
//
// Reference: gpt2_lora_finetune/eval_ppl.cpp:67-231 (flags --data_root --split --seq_len --batch_size
// --pretrained_dir --lora_path --lora_merge --out --log_every; non-overlapping seq_len windows, mean
// NLL over the predicted tokens, PPL = exp(NLL)).  Extras: --model P --random_init --synthetic_data
// --synthetic_tokens N --pretokenized_path F --pretokenized_meta F --max_batches N --model_type gpt2|gemma
// (the Python CLI's flag; Gemma reads config.json / model.safetensors / tokenizer.json from
// --pretrained_dir and the reference Gemma adapter layout).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "apps/app_common.h"
#include "engine/autograd.h"
#include "engine/comm.h"
#include "engine/gemma3.h"
#include "engine/gpt2.h"
#include "runtime/dataset.h"
#include "runtime/tokenizer.h"

using namespace mft;
using namespace mft::eng;
using mft::apps::Args;

namespace {

const std::set<std::string> kBool = {"random_init", "synthetic_data", "debug", "help"};
const std::set<std::string> kValued = {"data_root", "split", "seq_len", "batch_size", "pretrained_dir", "lora_path",
                                       "lora_merge", "out", "log_every", "model", "synthetic_tokens",
                                       "pretokenized_path", "pretokenized_meta", "max_batches", "device",
                                       "model_type"};

int run(int argc, char** argv) {
  Args a = mft::apps::parse_args(argc, argv, kBool, kValued);
  if (a.b("help")) {
    std::printf(
        "eval_ppl -- native MI355X engine (libmft)\n"
        "  --data_root D --split train|valid|test --seq_len S --batch_size B --pretrained_dir P\n"
        "  [--lora_path F --lora_merge 0|1] [--out F] [--log_every N]\n"
        "  extras: --model P --random_init --synthetic_data --synthetic_tokens N --pretokenized_path F\n"
        "          --pretokenized_meta F --max_batches N --model_type gpt2|gemma\n");
    return 0;
  }
  const char* fc = std::getenv("MFT_DP_FORCE_COMM");
  std::unique_ptr<Communicator> comm = Communicator::from_env(fc && fc[0] == '1');
  if (!comm) HIP_OK(hipSetDevice(0));
  const bool lead = !comm || comm->rank() == 0;
  hipStream_t stream;
  HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  set_current_stream(stream);

  mft::apps::apply_dtype_flag(a);
  const std::string pdir = a.get("pretrained_dir");
  const bool random_init = a.b("random_init") || pdir.empty();
  const std::string mtype = a.get("model_type", "gpt2");
  if (mtype != "gpt2" && mtype != "gemma") throw std::runtime_error("--model_type must be gpt2 or gemma");
  const bool cfg_file = !random_init && mft::apps::file_exists(pdir + "/config.json");
  std::unique_ptr<LanguageModel> model;
  int vocab = 0, max_pos = 0, eos = 50256;
  const std::string lora = a.get("lora_path");
  const bool merge = a.i("lora_merge", 1) != 0;
  if (mtype == "gpt2") {
    GPT2Config cfg = cfg_file ? GPT2Config::from_json(pdir + "/config.json") : GPT2Config::preset(a.get("model", "gpt2"));
    auto m = std::make_unique<GPT2>(cfg);
    if (random_init) m->init_random(1234);
    else m->load_hf(pdir);
    if (!lora.empty()) {
      m->load_lora(lora);
      if (merge) m->merge_lora(1.f);  // W += s A^T B^T: the adapter costs nothing
    }
    vocab = cfg.vocab_size, max_pos = cfg.n_positions;
    mft::apps::apply_model_flags(a, *m);
    model = std::move(m);
  } else {
    Gemma3Config cfg = cfg_file ? Gemma3Config::from_json(pdir + "/config.json")
                                : Gemma3Config::preset(a.get("model", "gemma3-270m"));
    auto m = std::make_unique<Gemma3>(cfg);
    if (random_init) m->init_random(1234);
    else m->load_hf(pdir);
    if (!lora.empty()) {
      m->load_lora(lora);
      if (merge) m->merge_lora(1.f);
    }
    vocab = cfg.vocab_size, max_pos = cfg.max_positions, eos = cfg.eos_id;
    mft::apps::apply_model_flags(a, *m);
    model = std::move(m);
  }
  model->training = false;
  if (!lora.empty() && lead) std::printf("  LoRA %s %s\n", lora.c_str(), merge ? "(merged)" : "(separate)");
  const int seq = std::min(a.i("seq_len", 1024), max_pos);
  const int B = a.i("batch_size", 1);
  const std::string split = a.get("split", "valid");
  const int sidx = split == "train" ? 0 : split == "valid" ? 1 : split == "test" ? 2 : -1;
  if (sidx < 0) throw std::runtime_error("--split must be train, valid or test");

  DataConfig dc;
  dc.seq_len = seq;
  dc.eos_id = eos;
  dc.drop_last = false;
  dc.shuffle = false;
  if (comm) {
    dc.rank = comm->rank();
    dc.world = comm->world();
  }
  TokenDataset ds(dc);
  const std::string pt = a.get("pretokenized_path"), root = a.get("data_root");
  if (!pt.empty()) {
    std::string meta = a.get("pretokenized_meta");
    if (meta.empty()) meta = pt.substr(0, pt.rfind('/') + 1) + "meta.json";
    ds.set_tokens(read_pretok_split(pt, read_pretok_meta(meta), sidx, 1.f, seq));
  } else if (a.b("synthetic_data") || root.empty()) {
    const int64_t n = a.l("synthetic_tokens", 200000);
    std::vector<int32_t> v(n);
    uint64_t z = 7 + (uint64_t)sidx;
    for (int64_t i = 0; i < n; ++i) {
      z += 0x9E3779B97F4A7C15ull;
      uint64_t x = z;
      x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
      x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
      v[i] = (int32_t)((x ^ (x >> 31)) % (uint64_t)vocab);
    }
    ds.set_tokens(std::move(v));
  } else {
    const std::string base = split == "valid" ? "valid" : split;
    const std::string raw = "wiki." + base + ".raw", tokf = "wiki." + base + ".tokens", txt = base + ".txt";
    const char* names[] = {raw.c_str(), tokf.c_str(), txt.c_str(), nullptr};
    const std::string f = mft::apps::split_file(root, names);
    if (f.empty()) throw std::runtime_error("no " + split + " split under " + root);
    mft::apps::Encoder enc;
    if (mtype == "gpt2") {
      std::shared_ptr<ByteLevelBPE> tok = ByteLevelBPE::from_files(pdir + "/vocab.json", pdir + "/merges.txt");
      enc = [tok](const std::string& s) { return tok->encode(s); };
    } else {
      std::shared_ptr<SentencePieceBPE> tok = SentencePieceBPE::from_tokenizer_json(pdir + "/tokenizer.json");
      enc = [tok](const std::string& s) { return tok->encode(s, false); };
    }
    const int threads = std::max(1u, std::thread::hardware_concurrency());
    ds.set_tokens(pack_lines(read_lines(f, true), enc, dc.eos_id, true, 1.f, seq, threads));
  }
  if (lead) std::printf("eval_ppl: %s split, %zu windows of %d tokens, batch %d\n", split.c_str(), ds.num_sequences(),
                        seq, B);

  std::vector<int64_t> ids((size_t)B * seq), tg((size_t)B * seq);
  std::vector<float> mk((size_t)B * seq);
  double nll = 0.0, cnt = 0.0;
  const int max_batches = a.i("max_batches", 0), log_every = a.i("log_every", 50);
  const auto t0 = std::chrono::steady_clock::now();
  int done = 0;
  {
    NoGradGuard ng;
    while (max_batches <= 0 || done < max_batches) {
      const int got = ds.next_batch(B, false, ids.data(), tg.data(), mk.data(), nullptr);
      if (got == 0) break;
      Tensor di = from_host(ids.data(), {B, seq}, DType::I64);
      Tensor dl = from_host(tg.data(), {B, seq}, DType::I64);
      auto r = model->nll(di, dl);
      nll += r.first.item();
      cnt += r.second.item();
      ++done;
      if (lead && log_every > 0 && done % log_every == 0)
        std::printf("  [%d] running ppl %.3f\n", done, std::exp(nll / std::max(1.0, cnt)));
    }
  }
  if (comm) {
    float h2[2] = {(float)nll, (float)cnt};
    Tensor d = from_host(h2, {2}, DType::F32);
    comm->all_reduce_sum(static_cast<float*>(d.data_ptr()), 2, stream);
    Tensor back = d.to(Device::cpu());
    nll = static_cast<const float*>(back.data_ptr())[0];
    cnt = static_cast<const float*>(back.data_ptr())[1];
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const double mean = nll / std::max(1.0, cnt), ppl = std::exp(std::min(mean, 50.0));
  if (lead) {
    std::printf("[Eval] split=%s tokens=%.0f NLL=%.6f PPL=%.4f (%.1f s, %.0f tokens/s)\n", split.c_str(), cnt, mean,
                ppl, secs, cnt / std::max(secs, 1e-9));
    const std::string out = a.get("out");
    if (!out.empty()) {
      std::ofstream o(out);
      o.precision(9);
      o << "{\"split\": \"" << split << "\", \"tokens\": " << cnt << ", \"nll\": " << mean << ", \"ppl\": " << ppl
        << "}\n";
    }
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  mft::apps::install_crash_report();
  try {
    return run(argc, argv);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "eval_ppl: error: %s\n", e.what());
    return 1;
  }
}
