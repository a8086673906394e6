#include "tokenizer.h"

#include <fstream>

#include "unicode_tables.h"

namespace lzrt {

static bool is_ascii_punct(uint32_t c) {
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}

template <size_t N>
static bool in_ranges(const uni::CpRange (&r)[N], uint32_t cp) {
  size_t lo = 0, hi = N;
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (cp < r[mid].lo) hi = mid;
    else if (cp > r[mid].hi) lo = mid + 1;
    else return true;
  }
  return false;
}

static const char* mapped(uint32_t cp) {
  size_t lo = 0, hi = sizeof(uni::kMap) / sizeof(uni::kMap[0]);
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (cp < uni::kMap[mid].cp) hi = mid;
    else if (cp > uni::kMap[mid].cp) lo = mid + 1;
    else return uni::kMap[mid].to;
  }
  return nullptr;
}

// next code point of UTF-8 text at i (advances i); malformed bytes -> U+FFFD
static uint32_t next_cp(const std::string& s, size_t& i) {
  const unsigned char c = (unsigned char)s[i++];
  if (c < 0x80) return c;
  int n = (c >= 0xF0 && c < 0xF8) ? 3 : (c >= 0xE0) ? 2 : (c >= 0xC0) ? 1 : -1;
  if (n < 0) return 0xFFFD;
  uint32_t cp = c & (0x3F >> n);
  for (int k = 0; k < n; ++k) {
    if (i >= s.size() || (((unsigned char)s[i]) & 0xC0) != 0x80) return 0xFFFD;
    cp = (cp << 6) | (((unsigned char)s[i++]) & 0x3F);
  }
  return cp;
}

static void put_cp(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out.push_back((char)cp);
  } else if (cp < 0x800) {
    out.push_back((char)(0xC0 | (cp >> 6)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else if (cp < 0x10000) {
    out.push_back((char)(0xE0 | (cp >> 12)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  } else {
    out.push_back((char)(0xF0 | (cp >> 18)));
    out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
    out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
    out.push_back((char)(0x80 | (cp & 0x3F)));
  }
}

// BERT's "Chinese character" blocks (CJK ideographs; not Hangul / kana)
static bool is_cjk(uint32_t c) {
  return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) || (c >= 0x20000 && c <= 0x2A6DF) ||
         (c >= 0x2A700 && c <= 0x2B73F) || (c >= 0x2B740 && c <= 0x2B81F) || (c >= 0x2B820 && c <= 0x2CEAF) ||
         (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}

static bool is_space(uint32_t c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || (c >= 0x80 && in_ranges(uni::kSpace, c));
}

static bool is_other(uint32_t c) {  // removed by the normalizer (\t \n \r are whitespace)
  if (c == '\t' || c == '\n' || c == '\r') return false;
  return in_ranges(uni::kControl, c);
}

static bool is_punct(uint32_t c) { return is_ascii_punct(c) || (c >= 0x80 && in_ranges(uni::kPunct, c)); }

bool Tokenizer::load_vocab(const std::string& path) {
  std::ifstream f(path);
  if (!f) return false;
  vocab_.clear();
  std::string line;
  int32_t id = 0;
  while (std::getline(f, line)) {
    while (!line.empty() && (line.back() == '\r' || line.back() == '\n')) line.pop_back();
    vocab_.emplace(line, id++);
  }
  vocab_size_ = id;
  auto special = [&](const char* tok, int32_t dflt) {
    auto it = vocab_.find(tok);
    return it != vocab_.end() ? it->second : dflt;
  };
  pad_ = special("[PAD]", 0);
  unk_ = special("[UNK]", 100);
  cls_ = special("[CLS]", 101);
  sep_ = special("[SEP]", 102);
  return true;
}

// HF BertNormalizer (clean text, isolate CJK ideographs, NFD + drop marks,
// lower-case) + BertPreTokenizer (split on whitespace, isolate punctuation),
// on UTF-8 code points. Uncased models (lower_ = false) keep accents and case.
void Tokenizer::basic_split(const std::string& text, std::vector<std::string>& out) const {
  std::string cur;
  auto flush = [&]() {
    if (!cur.empty()) { out.push_back(cur); cur.clear(); }
  };
  auto emit = [&](uint32_t c) {  // one normalised code point
    if (is_space(c)) { flush(); return; }
    if (is_punct(c)) { flush(); std::string p; put_cp(p, c); out.push_back(p); return; }
    put_cp(cur, c);
  };
  size_t i = 0;
  while (i < text.size()) {
    const uint32_t c = next_cp(text, i);
    if (c == 0 || c == 0xFFFD || is_other(c)) continue;
    if (is_space(c)) { flush(); continue; }
    if (is_cjk(c)) { flush(); std::string w; put_cp(w, c); out.push_back(w); continue; }
    if (!lower_) { emit(c); continue; }
    if (c < 0x80) { emit((c >= 'A' && c <= 'Z') ? c + 32 : c); continue; }
    if (c >= 0xAC00 && c <= 0xD7A3) {  // Hangul syllable -> L V (T) jamo (NFD)
      const uint32_t s = c - 0xAC00;
      emit(0x1100 + s / 588);
      emit(0x1161 + (s % 588) / 28);
      if (s % 28) emit(0x11A7 + s % 28);
      continue;
    }
    const char* m = mapped(c);
    if (!m) { emit(c); continue; }
    const std::string t(m);
    size_t j = 0;
    while (j < t.size()) emit(next_cp(t, j));
  }
  flush();
}

static uint64_t fnv1a(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) { h ^= c; h *= 1099511628211ull; }
  return h;
}

void Tokenizer::wordpiece(const std::string& w, std::vector<int32_t>& out) const {
  if (vocab_.empty()) {
    int span = vocab_size_ - 1000;
    out.push_back(1000 + (int32_t)(fnv1a(w) % (uint64_t)(span > 0 ? span : 1)));
    return;
  }
  size_t nchar = 0;  // max_input_chars_per_word = 100 code points
  for (unsigned char ch : w) nchar += (ch & 0xC0) != 0x80;
  if (nchar > 100) { out.push_back(unk_); return; }
  size_t start = 0;
  std::vector<int32_t> pieces;
  while (start < w.size()) {
    size_t end = w.size();
    int32_t found = -1;
    while (start < end) {
      std::string sub = w.substr(start, end - start);
      if (start > 0) sub = "##" + sub;
      auto it = vocab_.find(sub);
      if (it != vocab_.end()) { found = it->second; break; }
      do { --end; } while (end > start && (((unsigned char)w[end]) & 0xC0) == 0x80);  // whole code points
    }
    if (found < 0) { out.push_back(unk_); return; }
    pieces.push_back(found);
    start = end;
  }
  out.insert(out.end(), pieces.begin(), pieces.end());
}

std::vector<int32_t> Tokenizer::encode(const std::string& text, int max_len) const {
  std::vector<std::string> words;
  basic_split(text, words);
  std::vector<int32_t> ids;
  ids.push_back(cls_);
  for (auto& w : words) {
    wordpiece(w, ids);
    if ((int)ids.size() >= max_len - 1) break;
  }
  if ((int)ids.size() > max_len - 1) ids.resize(max_len - 1);
  ids.push_back(sep_);
  return ids;
}

int Tokenizer::encode_batch(const std::vector<std::string>& texts, int max_len, std::vector<int32_t>& ids,
                            std::vector<int32_t>& lens) const {
  std::vector<std::vector<int32_t>> all(texts.size());
  int S = 1;
  for (size_t i = 0; i < texts.size(); ++i) {
    all[i] = encode(texts[i], max_len);
    S = std::max<int>(S, (int)all[i].size());
  }
  S = std::min(max_len, (S + 7) / 8 * 8);
  ids.assign(texts.size() * (size_t)S, pad_);
  lens.resize(texts.size());
  for (size_t i = 0; i < texts.size(); ++i) {
    lens[i] = (int32_t)all[i].size();
    std::copy(all[i].begin(), all[i].end(), ids.begin() + i * S);
  }
  return S;
}

// Long inputs (SURVEY.md §5 "Long-context": encoder inputs are chunked at the
// model's max length with overlap and the chunk embeddings averaged): every
// text becomes ceil((n - overlap) / (body - overlap)) windows of at most
// `body = max_len - 2` word pieces, each wrapped in [CLS] ... [SEP];
// owner[w] is the text a window belongs to. Short texts give one window.
int Tokenizer::encode_chunks(const std::vector<std::string>& texts, int max_len, int overlap,
                             std::vector<int32_t>& ids, std::vector<int32_t>& lens,
                             std::vector<int32_t>& owner) const {
  const int body = std::max(1, max_len - 2);
  overlap = std::max(0, std::min(overlap, body - 1));
  const int stride = body - overlap;
  std::vector<std::vector<int32_t>> wins;
  owner.clear();
  for (size_t t = 0; t < texts.size(); ++t) {
    std::vector<std::string> words;
    basic_split(texts[t], words);
    std::vector<int32_t> pieces;
    for (auto& w : words) wordpiece(w, pieces);
    size_t start = 0;
    do {
      const size_t end = std::min(pieces.size(), start + (size_t)body);
      std::vector<int32_t> w;
      w.reserve(end - start + 2);
      w.push_back(cls_);
      w.insert(w.end(), pieces.begin() + start, pieces.begin() + end);
      w.push_back(sep_);
      wins.push_back(std::move(w));
      owner.push_back((int32_t)t);
      if (end >= pieces.size()) break;
      start += stride;
    } while (true);
  }
  int S = 1;
  for (auto& w : wins) S = std::max<int>(S, (int)w.size());
  S = std::min(max_len, (S + 7) / 8 * 8);
  ids.assign(wins.size() * (size_t)S, pad_);
  lens.resize(wins.size());
  for (size_t i = 0; i < wins.size(); ++i) {
    lens[i] = (int32_t)wins[i].size();
    std::copy(wins[i].begin(), wins[i].end(), ids.begin() + i * S);
  }
  return S;
}

}  // namespace lzrt
