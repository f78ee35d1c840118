// SafeTensors reader (mmap, zero-copy views) and writer.
// Replaces SafeTensorsReader (graph/safetensors_loader.h:26-92, .cpp:21-288: regex header parse,
// whole-tensor fread, F16/BF16 promoted to F32) and the hand-rolled writers of LoraSaver
// (graph/lora_saver.cpp:156-280) and the full-FT CLI (gpt2_full_finetune/main.cpp:156-237).
// The writer reproduces the reference LoRA file layout byte for byte when asked to
// (sorted keys, compact header, "__metadata__" last, no header padding).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "json.h"

namespace mft {

struct TensorInfo {
  std::string name;
  std::string dtype;  // F32, F16, BF16, I32, I64, I8, U8, BOOL, F64, I16
  std::vector<int64_t> shape;
  uint64_t begin = 0, end = 0;  // byte offsets within the data section
};

size_t safetensors_dtype_size(const std::string& dt);

class SafeTensorsFile {
 public:
  explicit SafeTensorsFile(const std::string& path);
  ~SafeTensorsFile();
  SafeTensorsFile(const SafeTensorsFile&) = delete;
  SafeTensorsFile& operator=(const SafeTensorsFile&) = delete;

  const std::vector<TensorInfo>& tensors() const { return tensors_; }
  const TensorInfo& info(const std::string& name) const;
  bool has(const std::string& name) const { return index_.count(name) != 0; }
  const void* data(const std::string& name) const;  // pointer into the mmap
  const std::map<std::string, std::string>& metadata() const { return meta_; }
  uint64_t header_len() const { return header_len_; }
  const std::string& path() const { return path_; }

 private:
  std::string path_;
  int fd_ = -1;
  void* map_ = nullptr;
  size_t size_ = 0;
  uint64_t header_len_ = 0;
  const char* base_ = nullptr;  // start of the data section
  std::vector<TensorInfo> tensors_;
  std::map<std::string, size_t> index_;
  std::map<std::string, std::string> meta_;
};

struct TensorBlob {
  std::string name;
  std::string dtype;
  std::vector<int64_t> shape;
  const void* data;
  size_t nbytes;
};

// sort_keys: order entries by name (reference LoraSaver sorts); align8: pad the header with spaces
// to a multiple of 8 bytes (HF convention); metadata is written last ("__metadata__").
void safetensors_save(const std::string& path, std::vector<TensorBlob> blobs,
                      const std::vector<std::pair<std::string, std::string>>& metadata, bool sort_keys, bool align8);

}  // namespace mft
