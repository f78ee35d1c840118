// Token-stream language-modelling dataset (WikiText-2 and friends), host side.
//
// Replaces WikiText2Dataset (data/wikitext2_dataset.h:19-158, .cpp:125-632).  Kept semantics:
// EOS after every line (blank lines included) when insert_eos_between_lines, a trailing EOS,
// chunks of S tokens starting every `stride` tokens with S+1 tokens available, optional padded
// tail chunk when !drop_last, data_fraction truncation, labels = inputs with the shift done by the
// loss (so a full chunk yields S-1 predictions), pad -> label -100 / mask 0, std::mt19937_64(seed)
// + std::shuffle ordering (same libstdc++ algorithm => same order as the reference for a seed),
// reshuffle at epoch end, pretokenized int32 .bin + meta.json splits.
// Dropped: the streaming mode that re-tokenised the file on every cache miss —
// lines are tokenised ONCE, on all host threads.  Added: DistributedSampler-style disjoint
// per-rank shards (rank::world of the shuffled order, equal length), and resumable state.
#pragma once
#include <cstdint>
#include <functional>
#include <random>
#include <string>
#include <vector>

namespace mft {

struct DataConfig {
  int seq_len = 128;
  int stride = -1;  // <= 0 -> seq_len
  int eos_id = 50256;
  int pad_id = 0;
  bool insert_eos_between_lines = true;
  bool drop_last = true;
  uint64_t seed = 2025;
  bool shuffle = true;
  float data_fraction = 1.0f;
  int rank = 0;
  int world = 1;
};

struct PretokMeta {
  int64_t total_tokens = 0;
  int eos_id = -1, pad_id = -1, bos_id = -1, unk_id = -1, vocab_size = -1;
  bool insert_eos_between_lines = true;
  int64_t off[3] = {-1, -1, -1}, len[3] = {0, 0, 0};  // train, valid, test
};

std::vector<std::string> read_lines(const std::string& path, bool keep_blank);
// tokenise lines with `encode` on `threads` threads, EOS after each line, trailing EOS, fraction cut
std::vector<int32_t> pack_lines(const std::vector<std::string>& lines,
                                const std::function<std::vector<int>(const std::string&)>& encode, int eos_id,
                                bool insert_eos, float data_fraction, int seq_len, int threads);
PretokMeta read_pretok_meta(const std::string& path);
std::vector<int32_t> read_pretok_split(const std::string& bin_path, const PretokMeta& m, int split, float data_fraction,
                                       int seq_len);

class TokenDataset {
 public:
  explicit TokenDataset(const DataConfig& cfg);
  void set_tokens(std::vector<int32_t> ids);
  const std::vector<int32_t>& tokens() const { return ids_; }
  size_t num_sequences() const { return starts_.size(); }   // global chunk count
  size_t num_local() const { return local_.size(); }        // this rank's share per epoch
  void shuffle();
  void reset_cursor() { cursor_ = 0; }
  // Fill one batch (B x S) from this rank's order.  Returns the number of rows filled (0 at epoch
  // end when !need_loop).  Rows past the filled count are padding (mask 0, labels -100).
  int next_batch(int B, bool need_loop, int64_t* input_ids, int64_t* targets, float* mask, int32_t* lengths);
  // Fill from explicit global chunk indices (evaluation / tests)
  void get_batch(const size_t* chunk_idx, int B, int64_t* input_ids, int64_t* targets, float* mask,
                 int32_t* lengths) const;
  int64_t epoch() const { return epoch_; }
  size_t cursor() const { return cursor_; }
  std::string rng_state() const;
  void restore(int64_t epoch, size_t cursor, const std::string& rng_state);
  const DataConfig& config() const { return cfg_; }

 private:
  void build_chunks();
  void build_local();
  DataConfig cfg_;
  std::vector<int32_t> ids_;
  std::vector<size_t> starts_;
  std::vector<size_t> order_;
  std::vector<size_t> local_;
  size_t cursor_ = 0;
  int64_t epoch_ = 0;
  std::mt19937_64 rng_;
};

}  // namespace mft
