// Self-test driver for the native text core, built with host sanitizers
// (tests/test_host_sanitizers.py): ASan + UBSan for memory / undefined
// behaviour on adversarial inputs, TSan for the thread-parallel batch paths
// (race detection / sanitizers on the native code).
//
// Checks, on a fixed-seed random corpus:
//  * Python-repr float formatting round-trips exactly (strtod(repr(v)) == v)
//    for random finite doubles, subnormals, integers and signed zero, and
//    prints the special values like Python;
//  * render_row never reads out of bounds and emits the reference template
//    for NaN / inf / huge values in any column;
//  * the tokenizer survives invalid UTF-8, control bytes, long words and
//    empty strings, and the thread-parallel batch equals the serial encode.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "text_core.h"

using namespace fdtext;

// Sanitizer run-time defaults baked into the binary (no environment needed).
extern "C" const char* __asan_default_options() { return "detect_leaks=1"; }
extern "C" const char* __ubsan_default_options() { return "print_stacktrace=1:halt_on_error=1"; }
extern "C" const char* __tsan_default_options() { return "halt_on_error=1"; }

static int failures = 0;
#define CHECK(cond, ...)                          \
  do {                                            \
    if (!(cond)) {                                \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);          \
      std::fprintf(stderr, "\n");                 \
      ++failures;                                 \
    }                                             \
  } while (0)

static void test_repr(std::mt19937_64& rng) {
  std::uniform_int_distribution<uint64_t> bits;
  for (int i = 0; i < 200000; ++i) {
    double v;
    uint64_t b = bits(rng);
    std::memcpy(&v, &b, sizeof(v));
    if (!std::isfinite(v)) continue;
    std::string s;
    append_py_repr(s, v);
    const double back = std::strtod(s.c_str(), nullptr);
    CHECK(back == v || (v == 0 && back == 0), "repr round trip %s", s.c_str());
  }
  const struct { double v; const char* want; } fixed[] = {
      {0.0, "0.0"}, {-0.0, "-0.0"}, {1.0, "1.0"}, {4000000.0, "4000000.0"}, {666666.6667, "666666.6667"},
      {1e16, "1e+16"}, {1e15, "1000000000000000.0"}, {1e-5, "1e-05"}, {0.0001, "0.0001"},
      {0.1 + 0.2, "0.30000000000000004"}, {NAN, "nan"}, {INFINITY, "inf"}, {-INFINITY, "-inf"},
      {5e-324, "5e-324"}, {1.7976931348623157e308, "1.7976931348623157e+308"}};
  for (auto& f : fixed) {
    std::string s;
    append_py_repr(s, f.v);
    CHECK(s == f.want, "repr(%.17g) = %s, want %s", f.v, s.c_str(), f.want);
  }
}

static void test_render(std::mt19937_64& rng) {
  const size_t n = 4096;
  std::vector<std::vector<double>> cols(10, std::vector<double>(n));
  std::uniform_real_distribution<double> u(-1e6, 1e6);
  std::uniform_int_distribution<int> pick(0, 9);
  const double specials[] = {NAN, INFINITY, -INFINITY, 1e300, -1e300, 0.0, -0.0, 9.3e18, -9.3e18, 1e-320};
  for (auto& c : cols)
    for (size_t i = 0; i < n; ++i) c[i] = pick(rng) == 0 ? specials[pick(rng)] : std::round(u(rng));
  std::vector<const double*> p;
  for (auto& c : cols) p.push_back(c.data());
  std::vector<bool> is_int = {true, true, true, true, true, true, true, true, false, false};
  std::vector<std::string> serial(n), parallel(n);
  for (size_t i = 0; i < n; ++i) serial[i] = render_row(p, is_int, i);
  WordPiece::run_parallel(n, 8, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) parallel[i] = render_row(p, is_int, i);
  });
  for (size_t i = 0; i < n; ++i) {
    CHECK(serial[i] == parallel[i], "render row %zu differs between serial and parallel", i);
    CHECK(serial[i].rfind("Destination port is ", 0) == 0 && serial[i].back() == '.', "template %s",
          serial[i].c_str());
  }
}

static std::string random_text(std::mt19937_64& rng) {
  std::uniform_int_distribution<int> len(0, 300), kind(0, 9), byte(0, 255), letter(0, 25);
  const char* words[] = {"flow", "packets", "bytes", "destination", "port", "per", "second", "unaffable",
                         "microseconds", "ÜBER", "naïve", "日本", "x"};
  std::string s;
  const int n = len(rng);
  for (int i = 0; i < n; ++i) {
    switch (kind(rng)) {
      case 0: s.push_back((char)byte(rng)); break;                 // any byte: invalid UTF-8, controls
      case 1: s += std::string(150, (char)('a' + letter(rng))); break;  // > max_chars word -> [UNK]
      case 2: s += "."; break;
      case 3: s += std::to_string(byte(rng) * 12345); break;
      default: s += words[byte(rng) % 13]; s += ' '; break;
    }
  }
  return s;
}

static void test_tokenizer(std::mt19937_64& rng) {
  std::vector<std::string> vocab = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", ".", ",", "!", "ü", "日"};
  for (char c = 'a'; c <= 'z'; ++c) {
    vocab.push_back(std::string(1, c));
    vocab.push_back("##" + std::string(1, c));
  }
  for (char c = '0'; c <= '9'; ++c) {
    vocab.push_back(std::string(1, c));
    vocab.push_back("##" + std::string(1, c));
  }
  for (const char* w : {"flow", "packet", "##s", "byte", "destination", "port", "per", "second", "un", "##aff",
                        "##able", "micro", "##seconds"})
    vocab.push_back(w);
  WordPiece wp(vocab, true, 100, 1, 2, 3, 0);
  const int max_len = 128;
  std::vector<std::string> texts;
  for (int i = 0; i < 3000; ++i) texts.push_back(random_text(rng));
  texts.push_back("");
  texts.push_back(std::string(1000, ' '));
  std::vector<int32_t> ids(texts.size() * max_len), lens(texts.size());
  wp.encode_batch_into(texts, max_len, 8, ids.data(), lens.data());
  for (size_t i = 0; i < texts.size(); ++i) {
    const std::vector<int> e = wp.encode(texts[i], max_len);
    CHECK((int)e.size() == lens[i] && lens[i] >= 2 && lens[i] <= max_len, "length %zu", i);
    CHECK(e.front() == 2 && e.back() == 3, "[CLS]/[SEP] framing %zu", i);
    for (int j = 0; j < max_len; ++j) {
      const int want = j < (int)e.size() ? e[j] : 0;
      CHECK(ids[i * max_len + j] == want, "batch != serial at %zu,%d", i, j);
      CHECK(ids[i * max_len + j] >= 0 && ids[i * max_len + j] < (int)vocab.size(), "id range");
    }
  }
  bool threw = false;
  try {
    wp.encode("abc", 1);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw, "max_len < 2 must be rejected");
}

int main() {
  std::mt19937_64 rng(20261015);
  test_repr(rng);
  test_render(rng);
  test_tokenizer(rng);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("text core self-test: ok\n");
  return 0;
}
