// pybind11 registration of the host-side C++ runtime (tokenizers, safetensors IO, datasets,
// host offload tier, power monitor).  The runtime sources under csrc/runtime/ are plain C++17 +
// HIP runtime API (no torch, no python) so they can also back a standalone binary.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <thread>

#include "runtime/dataset.h"
#include "runtime/offload.h"
#include "runtime/power_monitor.h"
#include "runtime/safetensors.h"
#include "runtime/tokenizer.h"

namespace py = pybind11;
using torch::Tensor;

namespace {

torch::Dtype st_to_torch(const std::string& dt) {
  if (dt == "F32") return torch::kFloat32;
  if (dt == "F16") return torch::kFloat16;
  if (dt == "BF16") return torch::kBFloat16;
  if (dt == "F64") return torch::kFloat64;
  if (dt == "I64") return torch::kInt64;
  if (dt == "I32") return torch::kInt32;
  if (dt == "I16") return torch::kInt16;
  if (dt == "I8") return torch::kInt8;
  if (dt == "U8") return torch::kUInt8;
  if (dt == "BOOL") return torch::kBool;
  throw std::runtime_error("safetensors dtype not supported by torch binding: " + dt);
}

std::string torch_to_st(torch::Dtype t) {
  switch (t) {
    case torch::kFloat32: return "F32";
    case torch::kFloat16: return "F16";
    case torch::kBFloat16: return "BF16";
    case torch::kFloat64: return "F64";
    case torch::kInt64: return "I64";
    case torch::kInt32: return "I32";
    case torch::kInt16: return "I16";
    case torch::kInt8: return "I8";
    case torch::kUInt8: return "U8";
    case torch::kBool: return "BOOL";
    default: throw std::runtime_error("dtype not supported by safetensors writer");
  }
}

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int hw_threads() {
  unsigned n = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(n, 16u));
}

}  // namespace

void register_runtime(py::module_& m) {
  auto rt = m.def_submodule("runtime", "host C++ runtime");

  // ---------------------------------------------------------------- safetensors
  py::class_<mft::SafeTensorsFile, std::shared_ptr<mft::SafeTensorsFile>>(rt, "SafeTensorsFile")
      .def(py::init<const std::string&>())
      .def("keys",
           [](const mft::SafeTensorsFile& f) {
             std::vector<std::string> k;
             for (auto& t : f.tensors()) k.push_back(t.name);
             return k;
           })
      .def("metadata", [](const mft::SafeTensorsFile& f) { return f.metadata(); })
      .def("header_len", &mft::SafeTensorsFile::header_len)
      .def("has", &mft::SafeTensorsFile::has)
      .def("info",
           [](const mft::SafeTensorsFile& f, const std::string& n) {
             auto& i = f.info(n);
             return py::make_tuple(i.dtype, i.shape, i.begin, i.end);
           })
      .def("get",
           [](const mft::SafeTensorsFile& f, const std::string& n) {
             auto& i = f.info(n);
             auto view = torch::from_blob(const_cast<void*>(f.data(n)), i.shape,
                                          torch::TensorOptions().dtype(st_to_torch(i.dtype)));
             return view.clone();  // own the bytes (the mmap goes away with the file object)
           });

  rt.def(
      "save_safetensors",
      [](const std::string& path, const std::vector<std::pair<std::string, Tensor>>& tensors,
         const std::vector<std::pair<std::string, std::string>>& metadata, bool sort_keys, bool align8) {
        std::vector<Tensor> keep;
        std::vector<mft::TensorBlob> blobs;
        for (auto& kv : tensors) {
          Tensor t = kv.second.detach().to(torch::kCPU).contiguous();
          keep.push_back(t);
          blobs.push_back({kv.first, torch_to_st(t.scalar_type()), t.sizes().vec(), t.data_ptr(),
                           (size_t)t.numel() * t.element_size()});
        }
        mft::safetensors_save(path, blobs, metadata, sort_keys, align8);
      },
      py::arg("path"), py::arg("tensors"), py::arg("metadata") = std::vector<std::pair<std::string, std::string>>{},
      py::arg("sort_keys") = true, py::arg("align8") = false);

  // ---------------------------------------------------------------- tokenizers
  py::class_<mft::ByteLevelBPE>(rt, "ByteLevelBPE")
      .def_static("from_files", &mft::ByteLevelBPE::from_files)
      .def_static("from_tokenizer_json", &mft::ByteLevelBPE::from_tokenizer_json)
      .def("encode", &mft::ByteLevelBPE::encode, py::call_guard<py::gil_scoped_release>())
      .def("encode_batch",
           [](const mft::ByteLevelBPE& t, const std::vector<std::string>& texts) {
             std::vector<std::vector<int>> out(texts.size());
             py::gil_scoped_release nogil;
             const int T = std::min<int>(hw_threads(), (int)std::max<size_t>(1, texts.size()));
             std::vector<std::thread> th;
             for (int k = 0; k < T; ++k)
               th.emplace_back([&, k] {
                 for (size_t i = k; i < texts.size(); i += T) out[i] = t.encode(texts[i]);
               });
             for (auto& x : th) x.join();
             return out;
           })
      .def("decode", &mft::ByteLevelBPE::decode, py::arg("ids"), py::arg("skip_special") = false)
      .def("pretokenize", &mft::ByteLevelBPE::pretokenize)
      .def("token_id", &mft::ByteLevelBPE::token_id)
      .def("token_str", &mft::ByteLevelBPE::token_str)
      .def_property_readonly("vocab_size", &mft::ByteLevelBPE::vocab_size)
      .def_readwrite("eos_id", &mft::ByteLevelBPE::eos_id)
      .def_readwrite("bos_id", &mft::ByteLevelBPE::bos_id)
      .def_readwrite("pad_id", &mft::ByteLevelBPE::pad_id);

  py::class_<mft::SentencePieceBPE>(rt, "SentencePieceBPE")
      .def_static("from_tokenizer_json", &mft::SentencePieceBPE::from_tokenizer_json)
      .def("encode", &mft::SentencePieceBPE::encode, py::arg("text"), py::arg("add_bos") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("encode_batch",
           [](const mft::SentencePieceBPE& t, const std::vector<std::string>& texts, bool add_bos) {
             std::vector<std::vector<int>> out(texts.size());
             py::gil_scoped_release nogil;
             const int T = std::min<int>(hw_threads(), (int)std::max<size_t>(1, texts.size()));
             std::vector<std::thread> th;
             for (int k = 0; k < T; ++k)
               th.emplace_back([&, k] {
                 for (size_t i = k; i < texts.size(); i += T) out[i] = t.encode(texts[i], add_bos);
               });
             for (auto& x : th) x.join();
             return out;
           },
           py::arg("texts"), py::arg("add_bos") = false)
      .def("decode", &mft::SentencePieceBPE::decode, py::arg("ids"), py::arg("skip_special") = true)
      .def("token_id", &mft::SentencePieceBPE::token_id)
      .def("token_str", &mft::SentencePieceBPE::token_str)
      .def_property_readonly("vocab_size", &mft::SentencePieceBPE::vocab_size)
      .def_readwrite("eos_id", &mft::SentencePieceBPE::eos_id)
      .def_readwrite("bos_id", &mft::SentencePieceBPE::bos_id)
      .def_readwrite("pad_id", &mft::SentencePieceBPE::pad_id)
      .def_readwrite("unk_id", &mft::SentencePieceBPE::unk_id);

  // ---------------------------------------------------------------- datasets
  rt.def("read_lines", &mft::read_lines, py::arg("path"), py::arg("keep_blank") = true);
  rt.def(
      "pack_lines_bytelevel",
      [](const mft::ByteLevelBPE& tok, const std::vector<std::string>& lines, int eos, bool insert_eos, float frac,
         int seq_len) {
        std::vector<int32_t> ids;
        {
          py::gil_scoped_release nogil;
          ids = mft::pack_lines(lines, [&](const std::string& s) { return tok.encode(s); }, eos, insert_eos, frac,
                                seq_len, hw_threads());
        }
        return torch::from_blob(ids.data(), {(long)ids.size()}, torch::kInt32).clone();
      });
  rt.def(
      "pack_lines_sentencepiece",
      [](const mft::SentencePieceBPE& tok, const std::vector<std::string>& lines, int eos, bool insert_eos, float frac,
         int seq_len) {
        std::vector<int32_t> ids;
        {
          py::gil_scoped_release nogil;
          ids = mft::pack_lines(lines, [&](const std::string& s) { return tok.encode(s, false); }, eos, insert_eos,
                                frac, seq_len, hw_threads());
        }
        return torch::from_blob(ids.data(), {(long)ids.size()}, torch::kInt32).clone();
      });
  rt.def("read_pretok_meta", [](const std::string& p) {
    auto m = mft::read_pretok_meta(p);
    py::dict d;
    d["total_tokens"] = m.total_tokens;
    d["eos_token_id"] = m.eos_id;
    d["pad_token_id"] = m.pad_id;
    d["bos_token_id"] = m.bos_id;
    d["unk_token_id"] = m.unk_id;
    d["vocab_size"] = m.vocab_size;
    d["insert_eos_between_lines"] = m.insert_eos_between_lines;
    d["offsets"] = std::vector<int64_t>(m.off, m.off + 3);
    d["lengths"] = std::vector<int64_t>(m.len, m.len + 3);
    return d;
  });
  rt.def("read_pretok_split", [](const std::string& bin, const std::string& meta, int split, float frac, int seq_len) {
    auto m = mft::read_pretok_meta(meta);
    auto ids = mft::read_pretok_split(bin, m, split, frac, seq_len);
    return torch::from_blob(ids.data(), {(long)ids.size()}, torch::kInt32).clone();
  });

  py::class_<mft::DataConfig>(rt, "DataConfig")
      .def(py::init<>())
      .def_readwrite("seq_len", &mft::DataConfig::seq_len)
      .def_readwrite("stride", &mft::DataConfig::stride)
      .def_readwrite("eos_id", &mft::DataConfig::eos_id)
      .def_readwrite("pad_id", &mft::DataConfig::pad_id)
      .def_readwrite("insert_eos_between_lines", &mft::DataConfig::insert_eos_between_lines)
      .def_readwrite("drop_last", &mft::DataConfig::drop_last)
      .def_readwrite("seed", &mft::DataConfig::seed)
      .def_readwrite("shuffle", &mft::DataConfig::shuffle)
      .def_readwrite("data_fraction", &mft::DataConfig::data_fraction)
      .def_readwrite("rank", &mft::DataConfig::rank)
      .def_readwrite("world", &mft::DataConfig::world);

  py::class_<mft::TokenDataset>(rt, "TokenDataset")
      .def(py::init<const mft::DataConfig&>())
      .def("set_tokens",
           [](mft::TokenDataset& d, Tensor ids) {
             Tensor t = ids.to(torch::kInt32).contiguous().cpu();
             std::vector<int32_t> v(t.data_ptr<int32_t>(), t.data_ptr<int32_t>() + t.numel());
             d.set_tokens(std::move(v));
           })
      .def("tokens",
           [](const mft::TokenDataset& d) {
             auto& v = d.tokens();
             return torch::from_blob(const_cast<int32_t*>(v.data()), {(long)v.size()}, torch::kInt32).clone();
           })
      .def("num_sequences", &mft::TokenDataset::num_sequences)
      .def("num_local", &mft::TokenDataset::num_local)
      .def("shuffle", &mft::TokenDataset::shuffle)
      .def("reset_cursor", &mft::TokenDataset::reset_cursor)
      .def("epoch", &mft::TokenDataset::epoch)
      .def("cursor", &mft::TokenDataset::cursor)
      .def("rng_state", [](const mft::TokenDataset& d) { return py::bytes(d.rng_state()); })
      .def("restore", [](mft::TokenDataset& d, int64_t e, size_t c, py::bytes s) { d.restore(e, c, std::string(s)); })
      .def("next_batch",
           [](mft::TokenDataset& d, int B, bool need_loop) {
             const int S = d.config().seq_len;
             auto ids = torch::empty({B, S}, torch::kInt64);
             auto tg = torch::empty({B, S}, torch::kInt64);
             auto mk = torch::empty({B, S}, torch::kFloat32);
             auto ln = torch::empty({B}, torch::kInt32);
             const int got = d.next_batch(B, need_loop, ids.data_ptr<int64_t>(), tg.data_ptr<int64_t>(),
                                          mk.data_ptr<float>(), ln.data_ptr<int32_t>());
             return py::make_tuple(got, ids, tg, mk, ln);
           })
      .def("get_batch", [](const mft::TokenDataset& d, const std::vector<int64_t>& idx) {
        const int S = d.config().seq_len;
        const int B = (int)idx.size();
        std::vector<size_t> ix(idx.begin(), idx.end());
        for (auto& x : ix)
          if ((int64_t)x < 0) x = (size_t)-1;
        auto ids = torch::empty({B, S}, torch::kInt64);
        auto tg = torch::empty({B, S}, torch::kInt64);
        auto mk = torch::empty({B, S}, torch::kFloat32);
        auto ln = torch::empty({B}, torch::kInt32);
        d.get_batch(ix.data(), B, ids.data_ptr<int64_t>(), tg.data_ptr<int64_t>(), mk.data_ptr<float>(),
                    ln.data_ptr<int32_t>());
        return py::make_tuple(ids, tg, mk, ln);
      });

  // ---------------------------------------------------------------- host offload tier
  py::class_<mft::HostTier>(rt, "HostTier")
      .def(py::init<size_t, const std::string&, size_t>(), py::arg("device_budget_bytes"), py::arg("disk_dir") = "",
           py::arg("host_budget_bytes") = 0)
      .def("add", &mft::HostTier::add)
      .def("has", &mft::HostTier::has)
      .def("offload", [](mft::HostTier& h, const std::string& n, Tensor t) {
        TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "offload needs a contiguous GPU tensor");
        TORCH_CHECK((size_t)(t.numel() * t.element_size()) == h.bytes(n), "offload: size mismatch for ", n);
        h.offload(n, t.data_ptr(), cur_stream());
      })
      .def("fetch", [](mft::HostTier& h, const std::string& n, Tensor t) {
        TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "fetch needs a contiguous GPU tensor");
        TORCH_CHECK((size_t)(t.numel() * t.element_size()) == h.bytes(n), "fetch: size mismatch for ", n);
        h.fetch(n, t.data_ptr(), cur_stream());
      })
      .def("host_tensor",
           [](mft::HostTier& h, const std::string& n, torch::Dtype dt, std::vector<int64_t> shape) {
             return torch::from_blob(h.host_ptr(n), shape, torch::TensorOptions().dtype(dt));
           })
      .def("device_tensor",
           [](mft::HostTier& h, const std::string& n, torch::Dtype dt, std::vector<int64_t> shape) {
             int dev = 0;
             TORCH_CHECK(hipGetDevice(&dev) == hipSuccess, "device_tensor: no HIP device");
             // the pinned host bytes, addressed by kernels over PCIe (zero copy); tensor ops that
             // need only the pointer (the fused AdamW) may use it like device memory
             return torch::from_blob(h.device_ptr(n), shape,
                                     torch::TensorOptions().dtype(dt).device(torch::kCUDA, dev));
           })
      .def("synchronize", &mft::HostTier::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("synchronize_all", &mft::HostTier::synchronize_all, py::call_guard<py::gil_scoped_release>())
      .def("mark_resident", &mft::HostTier::mark_resident)
      .def("touch", &mft::HostTier::touch)
      .def("mark_dirty", &mft::HostTier::mark_dirty)
      .def("dirty", &mft::HostTier::dirty)
      .def("resident", &mft::HostTier::resident)
      .def("victims", &mft::HostTier::victims)
      .def("bytes", &mft::HostTier::bytes)
      .def("spill", &mft::HostTier::spill)
      .def("unspill", &mft::HostTier::unspill)
      .def("on_disk", &mft::HostTier::on_disk)
      .def_property("device_budget", &mft::HostTier::device_budget, &mft::HostTier::set_device_budget)
      .def_property_readonly("resident_bytes", &mft::HostTier::resident_bytes)
      .def_property_readonly("host_bytes", &mft::HostTier::host_bytes)
      .def_property_readonly("h2d_bytes", &mft::HostTier::h2d_bytes)
      .def_property_readonly("d2h_bytes", &mft::HostTier::d2h_bytes);

  // ---------------------------------------------------------------- power monitor
  py::class_<mft::PowerConfig>(rt, "PowerConfig")
      .def(py::init<>())
      .def_readwrite("check_interval_steps", &mft::PowerConfig::check_interval_steps)
      .def_readwrite("battery_threshold", &mft::PowerConfig::battery_threshold)
      .def_readwrite("freq_b_high", &mft::PowerConfig::freq_b_high)
      .def_readwrite("freq_b_low", &mft::PowerConfig::freq_b_low)
      .def_readwrite("enable_battery", &mft::PowerConfig::enable_battery)
      .def_readwrite("temp_threshold", &mft::PowerConfig::temp_threshold)
      .def_readwrite("freq_t_high", &mft::PowerConfig::freq_t_high)
      .def_readwrite("freq_t_low", &mft::PowerConfig::freq_t_low)
      .def_readwrite("enable_temp", &mft::PowerConfig::enable_temp)
      .def_readwrite("use_gpu_telemetry", &mft::PowerConfig::use_gpu_telemetry)
      .def_readwrite("gpu_index", &mft::PowerConfig::gpu_index)
      .def_readwrite("pci_bus", &mft::PowerConfig::pci_bus)
      .def_readwrite("power_cap_w", &mft::PowerConfig::power_cap_w);
  py::class_<mft::PowerMonitor>(rt, "PowerMonitor")
      .def(py::init<const mft::PowerConfig&>())
      .def("set_manual_readings", &mft::PowerMonitor::set_manual_readings)
      .def("set_schedule",
           [](mft::PowerMonitor& p, const std::string& spec) { p.set_step_schedule(mft::PowerMonitor::parse_schedule(spec)); })
      .def_static("parse_schedule",
                  [](const std::string& spec) {
                    std::vector<std::tuple<int64_t, int64_t, int>> out;
                    for (auto& s : mft::PowerMonitor::parse_schedule(spec)) out.emplace_back(s.start_step, s.end_step, s.sleep_ms);
                    return out;
                  })
      .def("suggest_sleep_ms", &mft::PowerMonitor::suggest_sleep_ms)
      .def("note_step_ms", &mft::PowerMonitor::note_step_ms)
      .def("debug_state", &mft::PowerMonitor::debug_state)
      .def_property_readonly("battery", &mft::PowerMonitor::battery)
      .def_property_readonly("temperature", &mft::PowerMonitor::temperature);
  rt.def("power_cap_sleep_ms", &mft::power_cap_sleep_ms);
  rt.def("read_gpu_telemetry_bus", [](const std::string& bus) {
    auto t = mft::read_gpu_telemetry_bus(bus);
    py::dict d;
    d["ok"] = t.ok;
    d["temp_c"] = t.temp_c;
    d["power_w"] = t.power_w;
    d["power_cap_w"] = t.power_cap_w;
    return d;
  });
  rt.def("read_gpu_telemetry", [](int i) {
    auto t = mft::read_gpu_telemetry(i);
    py::dict d;
    d["ok"] = t.ok;
    d["temp_c"] = t.temp_c;
    d["power_w"] = t.power_w;
    d["power_cap_w"] = t.power_cap_w;
    return d;
  });
}
