// Host-side tokenizers (tokenization is not a GPU workload).
//
//  * ByteLevelBPE  — GPT-2 byte-level BPE (vocab.json + merges.txt, or tokenizer.json).  Replaces
//    GPT2BPETokenizer (core/tokenizer_bpe.h:24-142, .cpp:20-456), whose pre-tokenisation regex ran
//    on byte-mapped text with ASCII classes.  Here the HF regex
//    's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+ runs on the raw
//    code points with generated Unicode tables, then bytes are mapped (HF-exact byte table).
//  * SentencePieceBPE — Gemma tokenizer.json (BPE + byte fallback, ' ' -> U+2581 normaliser,
//    added/special tokens).  Replaces GemmaTokenizer (core/tokenizer_gemma.h:12-87, .cpp:109-416),
//    whose merge loop was quadratic over whole lines (Q14).
// Both use an O(n log n) priority-queue merge (lowest rank, then leftmost), matching HF tokenizers.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace mft {

class BPECore {
 public:
  void add_token(const std::string& s, int id);
  int token_id(const std::string& s) const;  // -1 if absent
  const std::string& token_str(int id) const;
  int vocab_size() const { return (int)id_to_tok_.size(); }
  void add_merge(const std::string& a, const std::string& b, int rank);
  // merge a sequence of symbol ids in place (ids must be valid vocab ids)
  void merge(std::vector<int>& syms) const;
  size_t num_merges() const { return merges_.size(); }

 protected:
  std::unordered_map<std::string, int> tok_to_id_;
  std::vector<std::string> id_to_tok_;
  struct MergeInfo {
    int rank;
    int id;
  };
  std::unordered_map<uint64_t, MergeInfo> merges_;
};

class ByteLevelBPE : public BPECore {
 public:
  static std::unique_ptr<ByteLevelBPE> from_files(const std::string& vocab_json, const std::string& merges_txt);
  static std::unique_ptr<ByteLevelBPE> from_tokenizer_json(const std::string& path);
  std::vector<int> encode(const std::string& text) const;
  std::string decode(const std::vector<int>& ids, bool skip_special = false) const;
  std::vector<std::string> pretokenize(const std::string& text) const;
  int eos_id = 50256, bos_id = 50256, pad_id = 50256;
  std::unordered_map<std::string, int> special;  // e.g. <|endoftext|>

 private:
  void init_byte_map();
  std::string byte_to_uni_[256];
  std::unordered_map<uint32_t, uint8_t> uni_to_byte_;
  void encode_word(const std::string& w, std::vector<int>& out) const;
  // identity of this vocabulary for the per-thread word cache: a process-unique serial, NOT the
  // object address (a new tokenizer allocated where a destroyed one lived must not see its cache)
  uint64_t uid_ = next_uid();
  static uint64_t next_uid();
};

class SentencePieceBPE : public BPECore {
 public:
  static std::unique_ptr<SentencePieceBPE> from_tokenizer_json(const std::string& path);
  std::vector<int> encode(const std::string& text, bool add_bos) const;
  std::string decode(const std::vector<int>& ids, bool skip_special = true) const;
  int bos_id = 2, eos_id = 1, pad_id = 0, unk_id = 3;
  bool byte_fallback = true;
  std::string replace_from = " ", replace_to = "\xE2\x96\x81";  // U+2581
  bool add_prefix_space = false;
  std::vector<std::pair<std::string, int>> added;  // added/special tokens matched before BPE
  std::vector<bool> is_special;

 private:
  int byte_tok_[256];
  void encode_chunk(const std::string& s, std::vector<int>& out) const;
};

}  // namespace mft
