#include "tokenizer.h"

#include <fstream>

namespace lzrt {

static const int32_t kPad = 0, kUnk = 100, kCls = 101, kSep = 102;

static bool is_punct(unsigned char c) {
  return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}

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
  return true;
}

void Tokenizer::basic_split(const std::string& text, std::vector<std::string>& out) const {
  std::string cur;
  for (unsigned char c : text) {
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r') {
      if (!cur.empty()) { out.push_back(cur); cur.clear(); }
    } else if (c < 128 && is_punct(c)) {
      if (!cur.empty()) { out.push_back(cur); cur.clear(); }
      out.push_back(std::string(1, (char)c));
    } else {
      cur.push_back((lower_ && c >= 'A' && c <= 'Z') ? (char)(c - 'A' + 'a') : (char)c);
    }
  }
  if (!cur.empty()) out.push_back(cur);
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
  if (w.size() > 100) { out.push_back(kUnk); return; }
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
      --end;
    }
    if (found < 0) { out.push_back(kUnk); return; }
    pieces.push_back(found);
    start = end;
  }
  out.insert(out.end(), pieces.begin(), pieces.end());
}

std::vector<int32_t> Tokenizer::encode(const std::string& text, int max_len) const {
  std::vector<std::string> words;
  basic_split(text, words);
  std::vector<int32_t> ids;
  ids.push_back(kCls);
  for (auto& w : words) {
    wordpiece(w, ids);
    if ((int)ids.size() >= max_len - 1) break;
  }
  if ((int)ids.size() > max_len - 1) ids.resize(max_len - 1);
  ids.push_back(kSep);
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
  ids.assign(texts.size() * (size_t)S, kPad);
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
      w.push_back(kCls);
      w.insert(w.end(), pieces.begin() + start, pieces.begin() + end);
      w.push_back(kSep);
      wins.push_back(std::move(w));
      owner.push_back((int32_t)t);
      if (end >= pieces.size()) break;
      start += stride;
    } while (true);
  }
  int S = 1;
  for (auto& w : wins) S = std::max<int>(S, (int)w.size());
  S = std::min(max_len, (S + 7) / 8 * 8);
  ids.assign(wins.size() * (size_t)S, kPad);
  lens.resize(wins.size());
  for (size_t i = 0; i < wins.size(); ++i) {
    lens[i] = (int32_t)wins[i].size();
    std::copy(wins[i].begin(), wins[i].end(), ids.begin() + i * S);
  }
  return S;
}

}  // namespace lzrt
