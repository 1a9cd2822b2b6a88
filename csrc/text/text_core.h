// Core of the native text front end (no Python dependency): CICIDS2017 row
// rendering with Python float repr, and a BERT basic + WordPiece tokenizer.
// Included by the pybind11 module (text_native.cpp) and by the sanitizer
// self-test driver (text_selftest.cpp).
#pragma once
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace fdtext {


// ---------------------------------------------------------------- float formatting
// Python repr(float) ("r" mode, shortest round-trip digits): fixed notation when
// -4 < decpt <= 16, scientific otherwise; ".0" appended to integral fixed values.
inline void append_py_repr(std::string& out, double v) {
  if (std::isnan(v)) { out += "nan"; return; }
  if (std::isinf(v)) { out += v < 0 ? "-inf" : "inf"; return; }
  if (v == 0.0) { out += std::signbit(v) ? "-0.0" : "0.0"; return; }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  std::string_view s(buf, r.ptr - buf);
  bool neg = false;
  if (s[0] == '-') { neg = true; s.remove_prefix(1); }
  size_t epos = s.find('e');
  std::string digits;
  for (size_t i = 0; i < epos; ++i)
    if (s[i] != '.') digits.push_back(s[i]);
  int exp10 = 0;
  std::from_chars(s.data() + epos + 1 + (s[epos + 1] == '+' ? 1 : 0), s.data() + s.size(), exp10);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  int nd = (int)digits.size();
  int decpt = exp10 + 1;
  if (neg) out.push_back('-');
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      out += "0.";
      out.append(-decpt, '0');
      out += digits;
    } else if (decpt < nd) {
      out.append(digits, 0, decpt);
      out.push_back('.');
      out.append(digits, decpt, std::string::npos);
    } else {
      out += digits;
      out.append(decpt - nd, '0');
      out += ".0";
    }
  } else {
    out.push_back(digits[0]);
    if (nd > 1) { out.push_back('.'); out.append(digits, 1, std::string::npos); }
    int e = decpt - 1;
    out.push_back('e');
    out.push_back(e < 0 ? '-' : '+');
    int ae = e < 0 ? -e : e;
    if (ae < 10) out.push_back('0');
    out += std::to_string(ae);
  }
}

inline void append_int(std::string& out, double v) {
  // integer columns: exact int64 text; non-finite / out-of-range values (never produced by
  // the reference's cleaning) fall back to the float repr instead of an undefined cast
  if (!(v >= -9.2e18 && v <= 9.2e18)) { append_py_repr(out, v); return; }
  char buf[32];
  auto r = std::to_chars(buf, buf + sizeof(buf), (long long)v);
  out.append(buf, r.ptr - buf);
}

// client1.py:69-80, split around the 10 values.
inline const char* const kPieces[11] = {
    "Destination port is ",
    ". Flow duration is ",
    " microseconds. Total forward packets are ",
    ". Total backward packets are ",
    ". Total length of forward packets is ",
    " bytes. Total length of backward packets is ",
    " bytes. Maximum forward packet length is ",
    ". Minimum forward packet length is ",
    ". Flow bytes per second is ",
    ". Flow packets per second is ",
    ".",
};

inline std::string render_row(const std::vector<const double*>& cols, const std::vector<bool>& is_int,
                       size_t i) {
  std::string s;
  s.reserve(360);
  for (int j = 0; j < 10; ++j) {
    s += kPieces[j];
    if (is_int[j]) append_int(s, cols[j][i]);
    else append_py_repr(s, cols[j][i]);
  }
  s += kPieces[10];
  return s;
}

// ---------------------------------------------------------------- tokenizer
inline bool is_ws(uint32_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
inline bool is_punct(uint32_t c) {
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) ||
         (c >= 123 && c <= 126);
}
inline bool is_control(uint32_t c) {
  if (c == '\t' || c == '\n' || c == '\r') return false;
  return c < 32 || c == 127 || (c >= 0x80 && c < 0xA0);
}

// Decode UTF-8 into (codepoint, byte_offset, byte_len) triples.
struct CP { uint32_t c; uint32_t off; uint32_t len; };
inline void decode_utf8(std::string_view s, std::vector<CP>& out) {
  out.clear();
  size_t i = 0;
  while (i < s.size()) {
    unsigned char b = s[i];
    uint32_t c; uint32_t n;
    if (b < 0x80) { c = b; n = 1; }
    else if ((b >> 5) == 6 && i + 1 < s.size()) { c = ((b & 0x1F) << 6) | (s[i + 1] & 0x3F); n = 2; }
    else if ((b >> 4) == 14 && i + 2 < s.size()) {
      c = ((b & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F); n = 3;
    } else if ((b >> 3) == 30 && i + 3 < s.size()) {
      c = ((b & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
      n = 4;
    } else { c = 0xFFFD; n = 1; }
    out.push_back({c, (uint32_t)i, n});
    i += n;
  }
}

class WordPiece {
 public:
  WordPiece(const std::vector<std::string>& vocab, bool lower, int max_chars, int unk_id, int cls_id,
            int sep_id, int pad_id)
      : lower_(lower), max_chars_(max_chars), unk_(unk_id), cls_(cls_id), sep_(sep_id), pad_(pad_id) {
    map_.reserve(vocab.size() * 2);
    for (size_t i = 0; i < vocab.size(); ++i) map_.emplace(vocab[i], (int)i);
  }

  // Basic-tokenise + WordPiece one text, appending ids.
  void tokenize(std::string_view text, std::vector<int>& ids) const {
    std::string norm;
    norm.reserve(text.size());
    std::vector<CP> cps;
    decode_utf8(text, cps);
    // Split into words: whitespace separates, punctuation is its own word.
    std::string word;
    auto flush = [&]() {
      if (!word.empty()) { wordpiece(word, ids); word.clear(); }
    };
    for (const CP& cp : cps) {
      uint32_t c = cp.c;
      if (c == 0 || c == 0xFFFD || is_control(c)) continue;
      if (is_ws(c)) { flush(); continue; }
      if (c < 128) {
        char ch = (char)c;
        if (lower_ && ch >= 'A' && ch <= 'Z') ch = ch - 'A' + 'a';
        if (is_punct(c)) { flush(); word.push_back(ch); flush(); continue; }
        word.push_back(ch);
      } else {
        word.append(text.data() + cp.off, cp.len);
      }
    }
    flush();
  }

  std::vector<int> encode(std::string_view text, int max_len) const {
    if (max_len < 2) throw std::invalid_argument("max_len must be >= 2 ([CLS] and [SEP])");
    std::vector<int> ids;
    tokenize(text, ids);
    std::vector<int> out;
    out.reserve(max_len);
    out.push_back(cls_);
    int keep = std::min<int>((int)ids.size(), max_len - 2);
    out.insert(out.end(), ids.begin(), ids.begin() + keep);
    out.push_back(sep_);
    return out;
  }

  // ids: [n][max_len] (padded), lens: [n]; rows are independent -> thread-parallel.
  void encode_batch_into(const std::vector<std::string>& texts, int max_len, int threads, int32_t* ids,
                         int32_t* lens) const {
    run_parallel(texts.size(), threads, [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        std::vector<int> e = encode(texts[i], max_len);
        int32_t* row = ids + i * max_len;
        for (int j = 0; j < max_len; ++j) row[j] = j < (int)e.size() ? e[j] : pad_;
        lens[i] = (int32_t)e.size();
      }
    });
  }

  std::vector<std::string> tokenize_str(std::string_view text) const {
    std::vector<int> ids;
    tokenize(text, ids);
    std::vector<std::string> out;
    inv_lazy();
    for (int i : ids) out.push_back(inv_[i]);
    return out;
  }

  static void run_parallel(size_t n, int threads, const std::function<void(size_t, size_t)>& f) {
    if (threads <= 1 || n < 512) { f(0, n); return; }
    std::vector<std::thread> ts;
    size_t chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
      size_t lo = t * chunk, hi = std::min(n, lo + chunk);
      if (lo >= hi) break;
      ts.emplace_back(f, lo, hi);
    }
    for (auto& t : ts) t.join();
  }

 private:
  void wordpiece(const std::string& word, std::vector<int>& ids) const {
    // Count code points (not bytes) against max_chars, as BERT does.
    size_t ncp = 0;
    for (unsigned char b : word) ncp += ((b & 0xC0) != 0x80);
    if ((int)ncp > max_chars_) { ids.push_back(unk_); return; }
    size_t start = 0;
    const size_t n = word.size();
    std::vector<int> pieces;
    std::string key;
    while (start < n) {
      size_t end = n;
      int found = -1;
      while (start < end) {
        key.clear();
        if (start > 0) key = "##";
        key.append(word, start, end - start);
        auto it = map_.find(key);
        if (it != map_.end()) { found = it->second; break; }
        // step back one UTF-8 code point
        do { --end; } while (end > start && ((unsigned char)word[end] & 0xC0) == 0x80);
      }
      if (found < 0) { ids.push_back(unk_); return; }
      pieces.push_back(found);
      start = end;
    }
    ids.insert(ids.end(), pieces.begin(), pieces.end());
  }

  void inv_lazy() const {
    if (!inv_.empty()) return;
    inv_.resize(map_.size());
    for (auto& kv : map_) if (kv.second < (int)inv_.size()) inv_[kv.second] = kv.first;
  }

  std::unordered_map<std::string, int> map_;
  mutable std::vector<std::string> inv_;
  bool lower_;
  int max_chars_, unk_, cls_, sep_, pad_;
};

}  // namespace fdtext
