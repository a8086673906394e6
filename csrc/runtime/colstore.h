// Versioned columnar table store (host runtime, C++17).
//
// Replaces the reference's LanceDB tables (vector_store.py:14-244): each table
// lives in `{root}/{name}.lance/` with
//   _versions/<v>.manifest   text manifest, written to a temp file + rename
//   data/<frag>.lzc          immutable column segments (one per append)
//   _deletions/<frag>-<v>.del sorted uint32 row offsets deleted in a fragment
// Commits take an flock on `<table>/_lock`, so several processes (memory
// system + dashboard) can share a directory; versions are monotone and every
// committed operation bumps the version (like Lance MVCC). Readers always see
// the newest manifest. NOTE: the byte format is this framework's own segment
// format, not Lance v2; Arrow IPC export/import is done in Python (pyarrow).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

namespace lzrt {

enum class ColType : uint8_t { Str = 0, F64 = 1, F32 = 2, I32 = 3, Bool = 4, VecF32 = 5, I64 = 6 };

struct ColSpec {
  std::string name;
  ColType type;
  uint32_t dim = 0;  // VecF32 only (0 = inferred on first append)
};

// A materialised column (host memory). Exactly one payload is used.
struct Column {
  ColType type;
  uint32_t dim = 0;
  std::vector<std::string> s;
  std::vector<double> f64;
  std::vector<float> f32;  // F32 and VecF32 (row-major n*dim)
  std::vector<int32_t> i32;
  std::vector<int64_t> i64;
  std::vector<uint8_t> b;
  size_t size() const;
  void append_from(const Column& o, size_t row);
};

struct Fragment {
  std::string file;
  uint64_t rows = 0;
  std::string delfile;  // "" = none
  std::vector<uint32_t> deleted;  // loaded lazily
  bool del_loaded = false;
};

struct Predicate {
  // conjunction of equalities on string columns + optional IN on one string column
  std::vector<std::pair<std::string, std::string>> eq;
  std::string in_col;
  std::unordered_set<std::string> in_vals;
  bool has_in = false;
};

class Table {
 public:
  Table(std::string dir, std::vector<ColSpec> schema);
  uint64_t latest_version();                          // re-reads disk
  uint64_t append(const std::vector<Column>& cols);   // returns new version
  uint64_t delete_where(const Predicate& p, uint64_t* n_deleted);
  // atomic delete_where(p) + append(cols) in one version
  uint64_t replace_where(const Predicate& p, const std::vector<Column>& cols, uint64_t* n_deleted);
  std::vector<Column> scan(const Predicate& p, const std::vector<std::string>& want);
  uint64_t count_rows();
  // two-phase multi-writer commit: stage() writes a fragment only,
  // commit_staged() publishes any number of staged fragments in ONE version
  std::pair<std::string, uint64_t> stage(const std::vector<Column>& cols);
  uint64_t commit_staged(const std::vector<std::pair<std::string, uint64_t>>& frags, uint32_t vec_dim);
  uint64_t compact();  // rewrite live rows into one fragment (new version)
  const std::vector<ColSpec>& schema() const { return schema_; }
  int col_index(const std::string& name) const;

 private:
  struct Manifest {
    uint64_t version = 0;
    std::vector<ColSpec> schema;
    std::vector<Fragment> frags;
  };
  std::string dir_;
  std::vector<ColSpec> schema_;
  Manifest load_latest();
  uint64_t apply_delete(Manifest& m, const Predicate& p, uint64_t nv);
  void write_manifest(const Manifest& m);
  std::vector<Column> read_fragment(const std::string& file, const std::vector<int>& cols);
  void write_fragment(const std::string& file, const std::vector<Column>& cols);
  void load_deleted(Fragment& f);
  bool matches(const std::vector<Column>& cols, const std::vector<int>& pcols,
               const Predicate& p, size_t r) const;
  int lock_fd_ = -1;
  void lock();
  void unlock();
};

}  // namespace lzrt
