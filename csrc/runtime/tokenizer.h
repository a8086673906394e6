// BERT-style tokenizer (host runtime): the BERT basic tokenizer on UTF-8 code
// points (clean text, isolate CJK ideographs, strip accents + lower-case for
// uncased models, split on whitespace and Unicode punctuation; tables in
// unicode_tables.h) then WordPiece greedy longest-match against a vocab.txt
// when one is loaded; without a vocab (no weights ship offline) each word maps
// to a deterministic hashed id in [1000, vocab_size). Output: [CLS] ... [SEP];
// special ids come from the vocab ([PAD]=0, [UNK]=100, [CLS]=101, [SEP]=102
// without one).
#pragma once
#include <algorithm>
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace lzrt {

class Tokenizer {
 public:
  Tokenizer(int vocab_size = 30522, bool lower = true) : vocab_size_(vocab_size), lower_(lower) {}
  bool load_vocab(const std::string& path);
  bool has_vocab() const { return !vocab_.empty(); }
  std::vector<int32_t> encode(const std::string& text, int max_len) const;
  // pads to the longest sequence (rounded up to a multiple of 8); returns S
  int encode_batch(const std::vector<std::string>& texts, int max_len, std::vector<int32_t>& ids,
                   std::vector<int32_t>& lens) const;
  // overlapping max_len windows for texts longer than the model (owner = text index)
  int encode_chunks(const std::vector<std::string>& texts, int max_len, int overlap, std::vector<int32_t>& ids,
                    std::vector<int32_t>& lens, std::vector<int32_t>& owner) const;

 private:
  int vocab_size_;
  bool lower_;
  std::unordered_map<std::string, int32_t> vocab_;
  int32_t pad_ = 0, unk_ = 100, cls_ = 101, sep_ = 102;
  void basic_split(const std::string& text, std::vector<std::string>& out) const;
  void wordpiece(const std::string& w, std::vector<int32_t>& out) const;
};

}  // namespace lzrt
