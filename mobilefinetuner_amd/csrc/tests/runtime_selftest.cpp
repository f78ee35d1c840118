// Standalone self-test of the host runtime (no torch, no GPU): JSON, safetensors writer/reader
// (incl. corrupted-header rejection), byte-level and SentencePiece BPE round trips, the WikiText
// token dataset (chunking, DP sharding, resume determinism) and the PowerMonitor policy.
//
// Built twice by scripts/sanitize_runtime.sh: plain, and with -fsanitize=address,undefined (host
// sanitizers, SURVEY §5.2 -- the reference had none).  tests/test_native_runtime.py runs both.
// Exit code 0 = all checks passed; every failure prints "FAIL <what>".
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <random>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "runtime/dataset.h"
#include "runtime/json.h"
#include "runtime/power_monitor.h"
#include "runtime/safetensors.h"
#include "runtime/tokenizer.h"

using namespace mft;

static int g_fail = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                          \
    }                                                                    \
  } while (0)

static std::string tmpdir() {
  char tpl[] = "/tmp/mft_selftest_XXXXXX";
  const char* d = mkdtemp(tpl);
  if (!d) throw std::runtime_error("mkdtemp failed");
  return d;
}

static void write_file(const std::string& p, const std::string& s) {
  std::ofstream o(p, std::ios::binary);
  o << s;
}

static std::string read_all(const std::string& p) {
  std::ifstream in(p, std::ios::binary);
  std::stringstream ss;
  ss << in.rdbuf();
  return ss.str();
}

// ----------------------------------------------------------------------------- JSON
static void test_json() {
  auto v = json::parse(R"({"a": 1, "b": [true, false, null, -2.5e3], "c": {"d": "x\"y\\z\u00e9\n"}, "e": 9007199254740993})");
  CHECK(v["a"].as_int() == 1);
  CHECK(v["b"].as_array().size() == 4);
  CHECK(v["b"].as_array()[0].b == true);
  CHECK(v["b"].as_array()[2].is_null());
  CHECK(std::fabs(v["b"].as_array()[3].as_double() + 2500.0) < 1e-9);
  CHECK(v["c"]["d"].as_string() == "x\"y\\z\xC3\xA9\n");
  CHECK(v["e"].as_int() == 9007199254740993LL);  // exact int64 (no double round trip)
  // key order is preserved (safetensors headers / vocab.json rely on it)
  auto o = json::parse(R"({"z": 0, "y": 1, "x": 2})");
  CHECK(o.as_object()[0].first == "z" && o.as_object()[2].first == "x");
  // escape -> parse round trip over every control char
  std::string s;
  for (int c = 1; c < 128; ++c) s.push_back((char)c);
  auto back = json::parse(json::escape(s));  // escape() returns the quoted literal
  CHECK(back.as_string() == s);
  // malformed inputs throw instead of crashing
  const char* bad[] = {"{", "[1,", "{\"a\" 1}", "\"abc", "tru", "{\"a\":}", "[1 2]", "\"\\u12\""};
  for (const char* b : bad) {
    bool threw = false;
    try {
      json::parse(b);
    } catch (const std::exception&) {
      threw = true;
    }
    CHECK(threw);
  }
}

// ----------------------------------------------------------------------------- safetensors
static void test_safetensors(const std::string& dir) {
  std::vector<float> a(3 * 5);
  for (size_t i = 0; i < a.size(); ++i) a[i] = 0.25f * (float)i - 1.f;
  std::vector<uint16_t> b(7);
  for (size_t i = 0; i < b.size(); ++i) b[i] = (uint16_t)(0x3f80 + i);
  std::vector<int32_t> c = {1, -2, 3};
  const std::string p = dir + "/t.safetensors";
  safetensors_save(p,
                   {{"layer.1.attn.qkv.lora_B", "F32", {3, 5}, a.data(), a.size() * 4},
                    {"layer.0.attn.qkv.lora_A", "BF16", {7}, b.data(), b.size() * 2},
                    {"ids", "I32", {3}, c.data(), c.size() * 4}},
                   {{"rank", "8"}, {"alpha", "16"}}, /*sort_keys=*/true, /*align8=*/true);
  SafeTensorsFile f(p);
  CHECK(f.tensors().size() == 3);
  CHECK(f.tensors()[0].name == "ids");  // sorted
  CHECK(f.header_len() % 8 == 0);
  CHECK(f.metadata().at("rank") == "8");
  CHECK(f.info("layer.1.attn.qkv.lora_B").shape == std::vector<int64_t>({3, 5}));
  CHECK(std::memcmp(f.data("layer.1.attn.qkv.lora_B"), a.data(), a.size() * 4) == 0);
  CHECK(std::memcmp(f.data("layer.0.attn.qkv.lora_A"), b.data(), b.size() * 2) == 0);
  CHECK(std::memcmp(f.data("ids"), c.data(), c.size() * 4) == 0);
  CHECK(!f.has("nope"));

  // corrupted files must be rejected with an exception (never read out of bounds):
  const std::string good = read_all(p);
  std::mt19937 rng(7);
  int rejected = 0, cases = 0;
  auto try_open = [&](const std::string& bytes) {
    const std::string q = dir + "/bad.safetensors";
    write_file(q, bytes);
    ++cases;
    try {
      SafeTensorsFile g(q);
      // a file that opens must have every tensor inside the data section
      for (auto& t : g.tensors()) (void)g.data(t.name);
    } catch (const std::exception&) {
      ++rejected;
    }
  };
  try_open(good.substr(0, 4));                   // shorter than the length prefix
  try_open(good.substr(0, 8 + 10));              // header cut
  try_open(good.substr(0, good.size() - 5));     // data section cut
  {
    std::string huge = good;
    uint64_t n = ~0ull >> 4;
    std::memcpy(&huge[0], &n, 8);                // absurd header length
    try_open(huge);
  }
  for (int it = 0; it < 200; ++it) {            // random byte flips inside the header
    std::string m = good;
    uint64_t hl;
    std::memcpy(&hl, m.data(), 8);
    const size_t pos = 8 + rng() % hl;
    m[pos] = (char)(rng() & 0xff);
    try_open(m);
  }
  CHECK(rejected >= 4);  // the four structural corruptions at least
  std::printf("safetensors: %d/%d corrupted variants rejected, rest parsed consistently\n", rejected, cases);
}

// ----------------------------------------------------------------------------- tokenizers
static std::string utf8(uint32_t cp) {
  std::string s;
  if (cp < 0x80) {
    s.push_back((char)cp);
  } else if (cp < 0x800) {
    s.push_back((char)(0xC0 | (cp >> 6)));
    s.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    s.push_back((char)(0xE0 | (cp >> 12)));
    s.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    s.push_back((char)(0x80 | (cp & 0x3F)));
  }
  return s;
}

// GPT-2 byte -> printable unicode table (the public bytes_to_unicode construction)
static std::vector<std::string> byte_unicode() {
  std::vector<int> bs;
  for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
  for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
  for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
  std::vector<std::string> out(256);
  std::vector<bool> have(256, false);
  for (int b : bs) {
    out[b] = utf8((uint32_t)b);
    have[b] = true;
  }
  int n = 0;
  for (int b = 0; b < 256; ++b)
    if (!have[b]) out[b] = utf8(256 + n++);
  return out;
}

static void test_byte_bpe(const std::string& dir) {
  auto bu = byte_unicode();
  std::string vocab = "{";
  int id = 0;
  for (int b = 0; b < 256; ++b) vocab += (b ? "," : "") + json::escape(bu[b]) + ":" + std::to_string(id++);
  const std::string G = bu[' '];  // "Ġ"
  const char* merges[][2] = {{"t", "h"}, {"th", "e"}, {G.c_str(), "the"}, {"i", "n"}, {G.c_str(), "in"}};
  std::string mtxt = "#version: 0.2\n";
  for (auto& m : merges) {
    vocab += "," + json::escape(std::string(m[0]) + m[1]) + ":" + std::to_string(id++);
    mtxt += std::string(m[0]) + " " + m[1] + "\n";
  }
  vocab += ",\"<|endoftext|>\":" + std::to_string(id++) + "}";
  write_file(dir + "/vocab.json", vocab);
  write_file(dir + "/merges.txt", mtxt);
  auto tok = ByteLevelBPE::from_files(dir + "/vocab.json", dir + "/merges.txt");
  CHECK(tok->eos_id == id - 1);
  auto ids = tok->encode("the cat in the hat");
  CHECK(tok->decode(ids) == "the cat in the hat");
  CHECK(ids.size() >= 1 && ids[0] == tok->token_id("the"));
  CHECK(tok->token_id(G + "the") >= 0);
  // random byte strings (incl. invalid UTF-8) round trip exactly
  std::mt19937 rng(11);
  for (int it = 0; it < 300; ++it) {
    std::string s;
    const int n = rng() % 40;
    for (int k = 0; k < n; ++k) s.push_back((char)(rng() & 0xff));
    CHECK(tok->decode(tok->encode(s)) == s);
  }
  // multilingual / emoji / contractions / digits
  const std::string multi = "Hello, world! It's 2024 -- caf\xC3\xA9 \xE4\xB8\xAD\xE6\x96\x87 \xF0\x9F\x98\x80  x\n\ny";
  CHECK(tok->decode(tok->encode(multi)) == multi);
  auto pre = tok->pretokenize("I'll go  now");
  CHECK(!pre.empty() && pre[0] == "I" && pre[1] == "'ll");
}

static void test_sp_bpe(const std::string& dir) {
  const std::string W = "\xE2\x96\x81";  // ▁
  std::string vocab = "{\"<pad>\":0,\"<eos>\":1,\"<bos>\":2,\"<unk>\":3";
  int id = 4;
  char buf[16];
  for (int b = 0; b < 256; ++b) {
    std::snprintf(buf, sizeof(buf), "<0x%02X>", b);
    vocab += ",\"" + std::string(buf) + "\":" + std::to_string(id++);
  }
  const std::vector<std::string> pieces = {"a", "b", "c", "h", "e", "l", "o", W, W + "h", "he", W + "he", "ll", W + "hell", W + "hello"};
  for (auto& p : pieces) vocab += "," + json::escape(p) + ":" + std::to_string(id++);
  vocab += "}";
  const std::string merges = "[\"" + W + " h\",\"h e\",\"" + W + "h e\",\"l l\",\"" + W + "he ll\",\"" + W + "hell o\"]";
  const std::string tj = "{\"normalizer\":{\"type\":\"Replace\",\"pattern\":{\"String\":\" \"},\"content\":\"" + W +
                         "\"},\"added_tokens\":[{\"id\":0,\"content\":\"<pad>\",\"special\":true},{\"id\":1,\"content\":\"<eos>\",\"special\":true},"
                         "{\"id\":2,\"content\":\"<bos>\",\"special\":true}],\"model\":{\"type\":\"BPE\",\"byte_fallback\":true,"
                         "\"unk_token\":\"<unk>\",\"vocab\":" + vocab + ",\"merges\":" + merges + "}}";
  write_file(dir + "/tokenizer.json", tj);
  auto tok = SentencePieceBPE::from_tokenizer_json(dir + "/tokenizer.json");
  CHECK(tok->bos_id == 2 && tok->eos_id == 1 && tok->pad_id == 0);
  auto ids = tok->encode(" hello", true);
  CHECK(ids.size() == 2 && ids[0] == 2 && ids[1] == tok->token_id(W + "hello"));
  CHECK(tok->decode(ids) == " hello");
  // byte fallback for out-of-vocab code points round trips
  const std::string s = "hello z\xC3\xA9\xE4\xB8\xAD<eos>";
  auto ids2 = tok->encode(s, false);
  CHECK(tok->decode(ids2, /*skip_special=*/false) == s);
  CHECK(ids2.back() == 1);  // added special token matched before BPE
}

// ----------------------------------------------------------------------------- dataset
static void test_dataset() {
  DataConfig cfg;
  cfg.seq_len = 8;
  cfg.seed = 5;
  std::vector<int32_t> ids(8 * 20 + 1);
  for (size_t i = 0; i < ids.size(); ++i) ids[i] = (int32_t)i;
  TokenDataset ds(cfg);
  ds.set_tokens(ids);
  CHECK(ds.num_sequences() == 20);
  std::vector<int64_t> x(2 * 8), y(2 * 8);
  std::vector<float> m(2 * 8);
  std::vector<int32_t> len(2);
  CHECK(ds.next_batch(2, false, x.data(), y.data(), m.data(), len.data()) == 2);
  for (int r = 0; r < 2; ++r)
    for (int t = 0; t < 7; ++t) CHECK(x[r * 8 + t + 1] == x[r * 8 + t] + 1);  // contiguous chunk
  // resume: saving (epoch, cursor, rng) and restoring replays the same batches
  const auto st = ds.rng_state();
  const int64_t ep = ds.epoch();
  const size_t cur = ds.cursor();
  std::vector<int64_t> a1(2 * 8), a2(2 * 8);
  ds.next_batch(2, true, a1.data(), y.data(), m.data(), len.data());
  TokenDataset ds2(cfg);
  ds2.set_tokens(ids);
  ds2.restore(ep, cur, st);
  ds2.next_batch(2, true, a2.data(), y.data(), m.data(), len.data());
  CHECK(a1 == a2);
  // DP sharding: ranks see disjoint chunks covering the epoch
  std::set<int64_t> seen;
  size_t total = 0;
  for (int r = 0; r < 4; ++r) {
    DataConfig c2 = cfg;
    c2.rank = r;
    c2.world = 4;
    TokenDataset d(c2);
    d.set_tokens(ids);
    total += d.num_local();
    for (size_t k = 0; k < d.num_local(); ++k) {
      d.next_batch(1, false, x.data(), y.data(), m.data(), len.data());
      CHECK(seen.insert(x[0]).second);
    }
  }
  CHECK(total == 20);
  // multi-threaded line packing (tokenizer calls fan out over threads): EOS after every line incl.
  // blank ones, order preserved, identical to the single-threaded result
  std::vector<std::string> lines;
  for (int i = 0; i < 500; ++i) lines.push_back(i % 7 == 0 ? std::string() : std::string(1 + i % 13, (char)('a' + i % 26)));
  auto enc = [](const std::string& l) {
    std::vector<int> o;
    for (char c : l) o.push_back((int)c);
    return o;
  };
  auto p1 = pack_lines(lines, enc, 1, true, 1.0f, 8, 1);
  auto p4 = pack_lines(lines, enc, 1, true, 1.0f, 8, 4);
  CHECK(p1 == p4);
  size_t expect = 0;
  for (auto& l : lines) expect += l.size() + 1;
  CHECK(p1.size() == expect);
  CHECK(!p1.empty() && p1.back() == 1);
}

// ----------------------------------------------------------------------------- power monitor
static void test_power() {
  auto sch = PowerMonitor::parse_schedule("0-9:0,10-19:200,20-:50");
  CHECK(sch.size() == 3);
  PowerConfig pc;
  pc.check_interval_steps = 1;
  PowerMonitor pm(pc);
  pm.set_step_schedule(sch);
  CHECK(pm.suggest_sleep_ms(3) == 0);
  CHECK(pm.suggest_sleep_ms(12) == 200);
  CHECK(pm.suggest_sleep_ms(1000) == 50);
  PowerMonitor p2(pc);
  p2.set_manual_readings(100.f, 30.f);  // healthy: high freq 2 Hz -> 500 ms
  CHECK(p2.suggest_sleep_ms(1) == 500);
  p2.set_manual_readings(10.f, 30.f);   // low battery: 0.5 Hz -> 2000 ms
  CHECK(p2.suggest_sleep_ms(2) == 2000);
  // software power cap: above the cap the sleep grows toward t (P_busy / cap - 1); below it decays
  {
    int sl = 0;
    for (int it = 0; it < 12; ++it) {
      // a GPU drawing 1400 W busy, 100 ms steps: the measured average includes the previous sleep
      const float measured = 1400.f * 100.f / (100.f + (float)sl);
      sl = power_cap_sleep_ms(measured, 1000.f, 100.f, sl);
    }
    CHECK(sl >= 35 && sl <= 45);  // fixed point: 100 (1400 / 1000 - 1) = 40 ms
    int d = 40;
    for (int it = 0; it < 12; ++it) d = power_cap_sleep_ms(500.f, 1000.f, 100.f, d);
    CHECK(d <= 2);
    CHECK(power_cap_sleep_ms(0.f, 1000.f, 100.f, 7) == 7);  // no reading: unchanged
    CHECK(read_gpu_telemetry_bus("0000:ff:1f.7").ok == false);  // no such card
  }
}

int main() {
  const std::string dir = tmpdir();
  const std::pair<const char*, std::function<void()>> tests[] = {
      {"json", test_json},
      {"safetensors", [&] { test_safetensors(dir); }},
      {"byte_bpe", [&] { test_byte_bpe(dir); }},
      {"sp_bpe", [&] { test_sp_bpe(dir); }},
      {"dataset", test_dataset},
      {"power", test_power}};
  for (auto& t : tests) {
    try {
      t.second();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "FAIL %s: uncaught exception: %s\n", t.first, e.what());
      ++g_fail;
    }
  }
  std::string cmd = "rm -rf " + dir;
  if (std::system(cmd.c_str()) != 0) std::fprintf(stderr, "warning: could not remove %s\n", dir.c_str());
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("runtime selftest: all checks passed\n");
  return 0;
}
