#include "safetensors.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace mft {

size_t safetensors_dtype_size(const std::string& dt) {
  if (dt == "F32" || dt == "I32" || dt == "U32") return 4;
  if (dt == "F16" || dt == "BF16" || dt == "I16" || dt == "U16") return 2;
  if (dt == "F64" || dt == "I64" || dt == "U64") return 8;
  if (dt == "I8" || dt == "U8" || dt == "BOOL" || dt == "F8_E4M3" || dt == "F8_E5M2") return 1;
  throw std::runtime_error("safetensors: unsupported dtype " + dt);
}

SafeTensorsFile::SafeTensorsFile(const std::string& path) : path_(path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw std::runtime_error("safetensors: cannot open " + path);
  struct stat st;
  if (fstat(fd_, &st) != 0) throw std::runtime_error("safetensors: stat failed " + path);
  size_ = (size_t)st.st_size;
  if (size_ < 8) throw std::runtime_error("safetensors: file too small " + path);
  map_ = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
  if (map_ == MAP_FAILED) {
    map_ = nullptr;
    throw std::runtime_error("safetensors: mmap failed " + path);
  }
  const char* p = static_cast<const char*>(map_);
  std::memcpy(&header_len_, p, 8);  // little-endian u64
  if (header_len_ > size_ - 8) throw std::runtime_error("safetensors: bad header length in " + path);
  json::Value h = json::parse(p + 8, header_len_);
  base_ = p + 8 + header_len_;
  const size_t data_size = size_ - 8 - header_len_;
  for (auto& kv : h.as_object()) {
    if (kv.first == "__metadata__") {
      if (kv.second.is_object())
        for (auto& m : kv.second.as_object())
          meta_[m.first] = m.second.is_string() ? m.second.as_string() : std::string();
      continue;
    }
    TensorInfo ti;
    ti.name = kv.first;
    ti.dtype = kv.second["dtype"].as_string();
    for (auto& d : kv.second["shape"].as_array()) ti.shape.push_back(d.as_int());
    auto& off = kv.second["data_offsets"].as_array();
    ti.begin = (uint64_t)off.at(0).as_int();
    ti.end = (uint64_t)off.at(1).as_int();
    size_t numel = 1;
    for (auto d : ti.shape) numel *= (size_t)d;
    if (ti.end < ti.begin || ti.end > data_size || ti.end - ti.begin != numel * safetensors_dtype_size(ti.dtype))
      throw std::runtime_error("safetensors: inconsistent offsets for " + ti.name);
    index_[ti.name] = tensors_.size();
    tensors_.push_back(std::move(ti));
  }
}

SafeTensorsFile::~SafeTensorsFile() {
  if (map_) ::munmap(map_, size_);
  if (fd_ >= 0) ::close(fd_);
}

const TensorInfo& SafeTensorsFile::info(const std::string& name) const {
  auto it = index_.find(name);
  if (it == index_.end()) throw std::runtime_error("safetensors: no tensor '" + name + "' in " + path_);
  return tensors_[it->second];
}

const void* SafeTensorsFile::data(const std::string& name) const { return base_ + info(name).begin; }

void safetensors_save(const std::string& path, std::vector<TensorBlob> blobs,
                      const std::vector<std::pair<std::string, std::string>>& metadata, bool sort_keys, bool align8) {
  if (sort_keys)
    std::sort(blobs.begin(), blobs.end(), [](const TensorBlob& a, const TensorBlob& b) { return a.name < b.name; });
  std::ostringstream h;
  h << "{";
  uint64_t off = 0;
  for (size_t i = 0; i < blobs.size(); ++i) {
    const auto& b = blobs[i];
    if (i) h << ",";
    h << json::escape(b.name) << ":{\"dtype\":\"" << b.dtype << "\",\"shape\":[";
    for (size_t d = 0; d < b.shape.size(); ++d) h << (d ? "," : "") << b.shape[d];
    h << "],\"data_offsets\":[" << off << "," << (off + b.nbytes) << "]}";
    off += b.nbytes;
  }
  if (!metadata.empty()) {
    h << (blobs.empty() ? "" : ",") << "\"__metadata__\":{";
    for (size_t i = 0; i < metadata.size(); ++i)
      h << (i ? "," : "") << json::escape(metadata[i].first) << ":" << json::escape(metadata[i].second);
    h << "}";
  }
  h << "}";
  std::string hs = h.str();
  if (align8)
    while (hs.size() % 8) hs += ' ';
  std::string tmp = path + ".tmp";
  {
    std::ofstream out(tmp, std::ios::binary | std::ios::trunc);
    if (!out) throw std::runtime_error("safetensors: cannot write " + path);
    uint64_t hl = hs.size();
    out.write(reinterpret_cast<const char*>(&hl), 8);
    out.write(hs.data(), (std::streamsize)hs.size());
    for (const auto& b : blobs) out.write(static_cast<const char*>(b.data), (std::streamsize)b.nbytes);
    if (!out) throw std::runtime_error("safetensors: write failed " + path);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("safetensors: rename failed " + path);
}

}  // namespace mft
