// Versioned columnar table store (host runtime, C++20 + Arrow C++).
//
// Replaces the reference's LanceDB tables (vector_store.py:14-244): each table
// lives in `{root}/{name}.lance/` with
//   _versions/<v>.manifest    text manifest, written to a temp file + rename
//   _latest                   the newest version number (O(1) version polls)
//   data/<frag>.arrow         immutable fragments: Arrow IPC files, one record
//                             batch, the table's schema (vector column =
//                             fixed_size_list<float32>[dim], like LanceDB's);
//                             readable by pyarrow.ipc without this runtime
//   _deletions/<frag>-<v>.arrow  deleted row offsets of a fragment (uint32
//                             column "row", Arrow IPC)
// Commits take an flock on `<table>/_lock`, so several processes (memory
// system + dashboard) share a directory; versions are monotone and every
// committed operation bumps the version (like Lance MVCC).
//
// Keyed writes are O(changed rows): a table opened with key columns (nodes /
// edges: user_id + id, profiles: user_id) keeps an in-memory key -> (fragment,
// row) index, refreshed incrementally from the manifest when another process
// commits, so an upsert / delete by key never scans the table. Other
// predicates scan the memory-mapped fragments.
#pragma once
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
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

// Allocator whose value-less construct() leaves the element uninitialised, so
// resize() before a bulk (parallel) copy does not zero-fill first: a reload
// moves a 30 GB vector column.
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind { using other = DefaultInitAlloc<U>; };
  DefaultInitAlloc() = default;
  template <class U>
  DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept { ::new ((void*)p) U; }
  template <class U, class... A>
  void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};
using FloatVec = std::vector<float, DefaultInitAlloc<float>>;

// A materialised column (host memory). Exactly one payload is used.
struct Column {
  ColType type;
  uint32_t dim = 0;
  std::vector<std::string> s;
  std::vector<double> f64;
  FloatVec f32;  // F32 and VecF32 (row-major n*dim)
  std::vector<int32_t> i32;
  std::vector<int64_t> i64;
  std::vector<uint8_t> b;
  // F32 / VecF32 input columns may borrow the caller's buffer instead of
  // owning a copy (a 10M x 768 commit: 30 GB not copied); the owner keeps it
  // alive for the duration of the call
  const float* ext = nullptr;
  size_t ext_n = 0;
  const float* fdata() const { return ext ? ext : f32.data(); }
  size_t fsize() const { return ext ? ext_n : f32.size(); }
  size_t size() const;
  void append_from(const Column& o, size_t row);
};

// One contiguous run of rows of a vector column returned by a scan without
// copying: a view into a memory-mapped fragment (`keep` holds the mapping),
// or rows gathered out of a partly selected fragment (`own`).
struct VecPiece {
  std::shared_ptr<void> keep;
  const float* data = nullptr;
  uint64_t rows = 0;
  uint32_t dim = 0;
  FloatVec own;
};

// memcpy split over threads (huge pages for large destinations)
void parallel_copy(void* dst, const void* src, size_t bytes);

struct Predicate {
  // conjunction of equalities on string columns + optional IN on one string column
  std::vector<std::pair<std::string, std::string>> eq;
  std::string in_col;
  std::unordered_set<std::string> in_vals;
  bool has_in = false;
};

class Table {
 public:
  Table(std::string dir, std::vector<ColSpec> schema, std::vector<std::string> key_cols = {});
  ~Table();
  uint64_t latest_version();                          // reads `_latest`
  uint64_t append(const std::vector<Column>& cols);   // returns new version
  uint64_t delete_where(const Predicate& p, uint64_t* n_deleted);
  // atomic delete_where(p) + append(cols) in one version
  uint64_t replace_where(const Predicate& p, const std::vector<Column>& cols, uint64_t* n_deleted);
  std::vector<Column> scan(const Predicate& p, const std::vector<std::string>& want,
                           std::vector<VecPiece>* vec_pieces = nullptr);
  uint64_t count_rows();
  // two-phase multi-writer commit: stage() writes a fragment only,
  // commit_staged() publishes any number of staged fragments in ONE version
  std::pair<std::string, uint64_t> stage(const std::vector<Column>& cols);
  uint64_t commit_staged(const std::vector<std::pair<std::string, uint64_t>>& frags, uint32_t vec_dim);
  uint64_t compact();  // rewrite live rows into one fragment (new version)
  const std::vector<ColSpec>& schema() const { return schema_; }
  int col_index(const std::string& name) const;
  std::string fragment_dir() const { return dir_ + "/data"; }

 private:
  struct Frag {
    std::string file;
    uint64_t rows = 0;
    std::string delfile;      // "" = none
    std::vector<uint8_t> dead;  // per row (loaded with the fragment's deletion file)
    uint64_t n_dead = 0;
  };
  std::string dir_;
  std::vector<ColSpec> schema_;
  std::vector<std::string> key_cols_;
  std::vector<int> key_idx_;
  // committed state this process has loaded (== the manifest of cur_version_)
  uint64_t cur_version_ = 0;
  std::vector<Frag> frags_;
  // key -> (frag, row); a multimap: the edge id "{src}_{tgt}" repeats when
  // two shards hold the same pair, and a keyed delete removes every row
  std::unordered_multimap<std::string, std::pair<uint32_t, uint32_t>> index_;
  bool indexed_ = false;
  uint64_t indexed_frags_ = 0;  // fragments [0, indexed_frags_) are in index_
  int lock_fd_ = -1;
  int lock_depth_ = 0;
  std::recursive_mutex mu_;  // threads of this process (the flock is per process)

  void lock();
  void unlock();
  void refresh();  // load the newest manifest (incrementally)
  void read_manifest(uint64_t v, std::vector<Frag>& out, std::vector<ColSpec>* sch);
  void write_manifest(uint64_t v);
  void load_dead(Frag& f);
  void write_dead(Frag& f, uint64_t v);
  void ensure_index();
  void index_fragment(uint32_t fi);
  std::string make_key(const std::vector<Column>& cols, size_t r) const;
  bool keyed(const Predicate& p, std::vector<std::string>* keys) const;
  uint64_t apply_delete(const Predicate& p, uint64_t nv);
  void add_fragment(const std::string& file, uint64_t rows, const std::vector<Column>* cols, uint64_t r0 = 0);
  void write_fragments(const std::vector<Column>& cols, size_t n);
  void fix_dims(const std::vector<Column>& cols);
  std::vector<Column> read_fragment(const std::string& file, const std::vector<int>& want, uint64_t* nrows);
  void write_fragment(const std::string& file, const std::vector<Column>& cols, int64_t r0 = 0, int64_t r1 = -1);
  bool matches(const std::vector<Column>& cols, const std::vector<int>& pcols, const Predicate& p, size_t r) const;
};

}  // namespace lzrt
