// Versioned columnar table store -- implementation. See colstore.h.
#include <thread>
#include <cstdlib>
#include "colstore.h"

#include <arrow/api.h>
#include <arrow/io/api.h>
#include <arrow/ipc/api.h>
#include <dirent.h>
#include <fcntl.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <sstream>
#include <stdexcept>

namespace lzrt {

namespace {

constexpr uint64_t kKeepManifests = 64;  // older manifests are garbage-collected

template <class T>
T ok_or_throw(arrow::Result<T> r, const char* what) {
  if (!r.ok()) throw std::runtime_error(std::string("colstore: ") + what + ": " + r.status().ToString());
  return std::move(r).ValueOrDie();
}

void check(const arrow::Status& s, const char* what) {
  if (!s.ok()) throw std::runtime_error(std::string("colstore: ") + what + ": " + s.ToString());
}

void mkdirs(const std::string& p) {
  std::string cur;
  for (size_t i = 0; i < p.size(); ++i) {
    cur.push_back(p[i]);
    if (p[i] == '/' || i + 1 == p.size()) ::mkdir(cur.c_str(), 0755);
  }
}

std::string uniq_name() {
  static std::atomic<uint64_t> ctr{0};
  std::random_device rd;
  uint64_t t = (uint64_t)std::chrono::high_resolution_clock::now().time_since_epoch().count();
  char buf[64];
  snprintf(buf, sizeof buf, "%016llx%08x%04llx", (unsigned long long)t, (unsigned)rd(),
           (unsigned long long)(ctr++ & 0xffff));
  return buf;
}

std::string manifest_path(const std::string& dir, uint64_t v) {
  char name[64];
  snprintf(name, sizeof name, "/_versions/%020llu.manifest", (unsigned long long)v);
  return dir + name;
}

void atomic_write(const std::string& path, const std::string& text) {
  std::string tmp = path + ".tmp-" + uniq_name();
  {
    std::ofstream f(tmp);
    f << text;
    f.flush();
    if (!f) throw std::runtime_error("colstore: write failed " + tmp);
  }
  if (::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("colstore: rename failed " + path);
}

std::shared_ptr<arrow::DataType> arrow_type(const ColSpec& c) {
  switch (c.type) {
    case ColType::Str: return arrow::utf8();
    case ColType::F64: return arrow::float64();
    case ColType::F32: return arrow::float32();
    case ColType::I32: return arrow::int32();
    case ColType::I64: return arrow::int64();
    case ColType::Bool: return arrow::boolean();
    case ColType::VecF32: return arrow::fixed_size_list(arrow::float32(), (int32_t)c.dim);
  }
  return arrow::null();
}

// Rows [r0, r1) of a column -> Arrow array. Fragments are written as several
// record batches (write_fragment): one Arrow array holds < 2^31 values / string
// bytes, and a 10M x 768 vector column is 7.7G floats.
std::shared_ptr<arrow::Array> to_arrow(const Column& c, int64_t r0, int64_t r1) {
  const int64_t n = r1 - r0;
  switch (c.type) {
    case ColType::Str: {
      arrow::StringBuilder b;
      int64_t bytes = 0;
      for (int64_t r = r0; r < r1; ++r) bytes += (int64_t)c.s[r].size();
      check(b.Reserve(n), "reserve");
      check(b.ReserveData(bytes), "reserve");
      for (int64_t r = r0; r < r1; ++r) b.UnsafeAppend(c.s[r]);
      return ok_or_throw(b.Finish(), "string column");
    }
    case ColType::F64: {
      arrow::DoubleBuilder b;
      check(b.AppendValues(c.f64.data() + r0, n), "f64 column");
      return ok_or_throw(b.Finish(), "f64 column");
    }
    case ColType::F32: {
      arrow::FloatBuilder b;
      check(b.AppendValues(c.fdata() + r0, n), "f32 column");
      return ok_or_throw(b.Finish(), "f32 column");
    }
    case ColType::I32: {
      arrow::Int32Builder b;
      check(b.AppendValues(c.i32.data() + r0, n), "i32 column");
      return ok_or_throw(b.Finish(), "i32 column");
    }
    case ColType::I64: {
      arrow::Int64Builder b;
      check(b.AppendValues(c.i64.data() + r0, n), "i64 column");
      return ok_or_throw(b.Finish(), "i64 column");
    }
    case ColType::Bool: {
      arrow::BooleanBuilder b;
      check(b.AppendValues(c.b.data() + r0, n), "bool column");
      return ok_or_throw(b.Finish(), "bool column");
    }
    case ColType::VecF32: {
      // zero-copy: the Arrow array wraps the column's memory (alive until
      // the fragment is written); no 30 GB builder copy for a 10M-row commit
      const int64_t nv = n * (int64_t)c.dim;
      auto buf = arrow::Buffer::Wrap(c.fdata() + (size_t)r0 * c.dim, (size_t)nv);
      auto values = std::make_shared<arrow::FloatArray>(nv, buf);
      return ok_or_throw(arrow::FixedSizeListArray::FromArrays(values, (int32_t)c.dim), "vector column");
    }
  }
  return nullptr;
}

// memcpy split over threads: one core copies ~10 GB/s, a reload moves the
// whole vector column (30 GB at 10M x 768) out of the mapped fragments
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

// Best-effort madvise over the pages covering [p, p + n) (older kernels
// reject the populate advices: the copy then faults page by page as before).
void advise(const void* p, size_t n, int advice, uintptr_t align = 4096) {
  const uintptr_t a = (uintptr_t)p & ~(align - 1);
  const uintptr_t e = ((uintptr_t)p + n + 4095) & ~uintptr_t(4095);
  if (e > a) (void)madvise((void*)a, e - a, advice);
}

// set in a scan's fragment-parallel workers: their copies stay on the thread
thread_local bool t_serial_copy = false;

void par_copy(void* dst, const void* src, size_t bytes) {
  if (t_serial_copy) { std::memcpy(dst, src, bytes); return; }
  constexpr size_t kMin = size_t(64) << 20;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const size_t nt = std::min<size_t>(hw, std::max<size_t>(1, bytes / kMin));
  if (nt <= 1) { std::memcpy(dst, src, bytes); return; }
  // A page fault per 4 KiB on both sides (the source is a mapped fragment,
  // the destination fresh anonymous memory) held a reload at ~1.4 GB/s:
  // huge pages for the destination, page tables of each thread's chunks
  // populated in one call per chunk, then the copy.
  advise((const char*)dst + (size_t(2) << 20), bytes > (size_t(4) << 20) ? bytes - (size_t(4) << 20) : 0,
         MADV_HUGEPAGE, uintptr_t(2) << 20);
  std::vector<std::thread> ts;
  const size_t per = (bytes + nt - 1) / nt;
  for (size_t t = 0; t < nt; ++t) {
    const size_t o = t * per;
    if (o >= bytes) break;
    ts.emplace_back([=] {
      const size_t len = std::min(per, bytes - o);
      advise((const char*)src + o, len, MADV_POPULATE_READ);
      advise((char*)dst + o, len, MADV_POPULATE_WRITE);
      std::memcpy((char*)dst + o, (const char*)src + o, len);
    });
  }
  for (auto& th : ts) th.join();
}

// Append an Arrow array's nrows rows to a Column of the requested type
// (missing array -> defaults).
void from_arrow(const std::shared_ptr<arrow::Array>& a, Column& c, uint64_t nrows) {
  if (!a) {
    switch (c.type) {
      case ColType::Str: c.s.resize(c.s.size() + nrows); break;
      case ColType::F64: c.f64.resize(c.f64.size() + nrows, 0.0); break;
      case ColType::F32: c.f32.resize(c.f32.size() + nrows, 0.f); break;
      case ColType::I32: c.i32.resize(c.i32.size() + nrows, 0); break;
      case ColType::I64: c.i64.resize(c.i64.size() + nrows, 0); break;
      case ColType::Bool: c.b.resize(c.b.size() + nrows, 0); break;
      case ColType::VecF32: c.f32.resize(c.f32.size() + nrows * c.dim, 0.f); break;
    }
    return;
  }
  switch (c.type) {
    case ColType::Str: {
      auto s = std::static_pointer_cast<arrow::StringArray>(a);
      c.s.reserve(c.s.size() + nrows);
      for (uint64_t r = 0; r < nrows; ++r) c.s.emplace_back(s->GetView((int64_t)r));
      break;
    }
    case ColType::F64: {
      auto x = std::static_pointer_cast<arrow::DoubleArray>(a);
      c.f64.insert(c.f64.end(), x->raw_values(), x->raw_values() + nrows);
      break;
    }
    case ColType::F32: {
      auto x = std::static_pointer_cast<arrow::FloatArray>(a);
      c.f32.insert(c.f32.end(), x->raw_values(), x->raw_values() + nrows);
      break;
    }
    case ColType::I32: {
      auto x = std::static_pointer_cast<arrow::Int32Array>(a);
      c.i32.insert(c.i32.end(), x->raw_values(), x->raw_values() + nrows);
      break;
    }
    case ColType::I64: {
      auto x = std::static_pointer_cast<arrow::Int64Array>(a);
      c.i64.insert(c.i64.end(), x->raw_values(), x->raw_values() + nrows);
      break;
    }
    case ColType::Bool: {
      auto x = std::static_pointer_cast<arrow::BooleanArray>(a);
      c.b.reserve(c.b.size() + nrows);
      for (uint64_t r = 0; r < nrows; ++r) c.b.push_back(x->Value((int64_t)r) ? 1 : 0);
      break;
    }
    case ColType::VecF32: {
      auto l = std::static_pointer_cast<arrow::FixedSizeListArray>(a);
      c.dim = (uint32_t)l->list_type()->list_size();
      auto v = std::static_pointer_cast<arrow::FloatArray>(l->values());
      const float* p = v->raw_values() + l->value_offset(0);
      const size_t cnt = nrows * (size_t)c.dim, at = c.f32.size();
      c.f32.resize(at + cnt);
      par_copy(c.f32.data() + at, p, cnt * sizeof(float));
      break;
    }
  }
}

// Rows [0, nrows) of an Arrow array into rows [at, at + nrows) of a column
// already sized for them (missing array -> defaults).
void from_arrow_at(const std::shared_ptr<arrow::Array>& a, Column& c, uint64_t at, uint64_t nrows) {
  switch (c.type) {
    case ColType::Str: {
      if (!a) { for (uint64_t r = 0; r < nrows; ++r) c.s[at + r].clear(); break; }
      auto x = std::static_pointer_cast<arrow::StringArray>(a);
      for (uint64_t r = 0; r < nrows; ++r) c.s[at + r].assign(x->GetView((int64_t)r));
      break;
    }
    case ColType::F64:
      if (a) std::memcpy(c.f64.data() + at, std::static_pointer_cast<arrow::DoubleArray>(a)->raw_values(), nrows * 8);
      else std::fill(c.f64.begin() + at, c.f64.begin() + at + nrows, 0.0);
      break;
    case ColType::F32:
      if (a) std::memcpy(c.f32.data() + at, std::static_pointer_cast<arrow::FloatArray>(a)->raw_values(), nrows * 4);
      else std::fill(c.f32.begin() + at, c.f32.begin() + at + nrows, 0.f);
      break;
    case ColType::I32:
      if (a) std::memcpy(c.i32.data() + at, std::static_pointer_cast<arrow::Int32Array>(a)->raw_values(), nrows * 4);
      else std::fill(c.i32.begin() + at, c.i32.begin() + at + nrows, 0);
      break;
    case ColType::I64:
      if (a) std::memcpy(c.i64.data() + at, std::static_pointer_cast<arrow::Int64Array>(a)->raw_values(), nrows * 8);
      else std::fill(c.i64.begin() + at, c.i64.begin() + at + nrows, 0);
      break;
    case ColType::Bool: {
      if (!a) { std::fill(c.b.begin() + at, c.b.begin() + at + nrows, 0); break; }
      auto x = std::static_pointer_cast<arrow::BooleanArray>(a);
      for (uint64_t r = 0; r < nrows; ++r) c.b[at + r] = x->Value((int64_t)r) ? 1 : 0;
      break;
    }
    case ColType::VecF32: {
      const size_t d = c.dim;
      if (!a) { std::fill(c.f32.begin() + at * d, c.f32.begin() + (at + nrows) * d, 0.f); break; }
      auto l = std::static_pointer_cast<arrow::FixedSizeListArray>(a);
      if ((size_t)l->list_type()->list_size() != d) throw std::runtime_error("colstore: vector dim mismatch in scan");
      auto v = std::static_pointer_cast<arrow::FloatArray>(l->values());
      par_copy(c.f32.data() + at * d, v->raw_values() + l->value_offset(0), nrows * d * sizeof(float));
      break;
    }
  }
}

// One row of an Arrow array into row `dst` of a sized column.
void row_from_arrow(const std::shared_ptr<arrow::Array>& a, Column& c, uint64_t src, uint64_t dst) {
  if (!a) {  // defaults (FloatVec storage is not zeroed by resize)
    if (c.type == ColType::F32) c.f32[dst] = 0.f;
    if (c.type == ColType::VecF32) std::fill(c.f32.begin() + dst * c.dim, c.f32.begin() + (dst + 1) * c.dim, 0.f);
    return;
  }
  switch (c.type) {
    case ColType::Str: c.s[dst].assign(std::static_pointer_cast<arrow::StringArray>(a)->GetView((int64_t)src)); break;
    case ColType::F64: c.f64[dst] = std::static_pointer_cast<arrow::DoubleArray>(a)->Value((int64_t)src); break;
    case ColType::F32: c.f32[dst] = std::static_pointer_cast<arrow::FloatArray>(a)->Value((int64_t)src); break;
    case ColType::I32: c.i32[dst] = std::static_pointer_cast<arrow::Int32Array>(a)->Value((int64_t)src); break;
    case ColType::I64: c.i64[dst] = std::static_pointer_cast<arrow::Int64Array>(a)->Value((int64_t)src); break;
    case ColType::Bool: c.b[dst] = std::static_pointer_cast<arrow::BooleanArray>(a)->Value((int64_t)src) ? 1 : 0; break;
    case ColType::VecF32: {
      auto l = std::static_pointer_cast<arrow::FixedSizeListArray>(a);
      auto v = std::static_pointer_cast<arrow::FloatArray>(l->values());
      std::memcpy(c.f32.data() + dst * c.dim, v->raw_values() + l->value_offset((int64_t)src), c.dim * sizeof(float));
      break;
    }
  }
}

template <class F>
void par_for(size_t n, size_t max_threads, F&& fn) {
  const size_t nt = std::min(n, max_threads);
  if (nt <= 1) { for (size_t i = 0; i < n; ++i) fn(i); return; }
  std::atomic<size_t> next{0};
  std::vector<std::exception_ptr> err(nt);
  std::vector<std::thread> ts;
  for (size_t t = 0; t < nt; ++t)
    ts.emplace_back([&, t] {
      t_serial_copy = true;
      try {
        for (size_t i; (i = next++) < n;) fn(i);
      } catch (...) {
        err[t] = std::current_exception();
      }
    });
  for (auto& th : ts) th.join();
  for (auto& e : err)
    if (e) std::rethrow_exception(e);
}

}  // namespace

// Staging copies (pinned destination, mapped-file source): split over up to 16
// threads at >= 4 MiB each, no madvise of the destination (pinned pages).
void parallel_copy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kMin = size_t(4) << 20;
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const size_t nt = std::min<size_t>(hw, std::max<size_t>(1, bytes / kMin));
  if (nt <= 1) { std::memcpy(dst, src, bytes); return; }
  std::vector<std::thread> ts;
  const size_t per = ((bytes + nt - 1) / nt + 63) & ~size_t(63);
  for (size_t t = 0; t < nt; ++t) {
    const size_t o = t * per;
    if (o >= bytes) break;
    ts.emplace_back([=] { std::memcpy((char*)dst + o, (const char*)src + o, std::min(per, bytes - o)); });
  }
  for (auto& th : ts) th.join();
}

size_t Column::size() const {
  switch (type) {
    case ColType::Str: return s.size();
    case ColType::F64: return f64.size();
    case ColType::F32: return fsize();
    case ColType::I32: return i32.size();
    case ColType::I64: return i64.size();
    case ColType::Bool: return b.size();
    case ColType::VecF32: return dim ? fsize() / dim : 0;
  }
  return 0;
}

void Column::append_from(const Column& o, size_t r) {
  switch (type) {
    case ColType::Str: s.push_back(o.s[r]); break;
    case ColType::F64: f64.push_back(o.f64[r]); break;
    case ColType::F32: f32.push_back(o.fdata()[r]); break;
    case ColType::I32: i32.push_back(o.i32[r]); break;
    case ColType::I64: i64.push_back(o.i64[r]); break;
    case ColType::Bool: b.push_back(o.b[r]); break;
    case ColType::VecF32:
      f32.insert(f32.end(), o.fdata() + r * o.dim, o.fdata() + (r + 1) * o.dim);
      break;
  }
}

Table::Table(std::string dir, std::vector<ColSpec> schema, std::vector<std::string> key_cols)
    : dir_(std::move(dir)), schema_(std::move(schema)), key_cols_(std::move(key_cols)) {
  mkdirs(dir_ + "/_versions");
  mkdirs(dir_ + "/data");
  mkdirs(dir_ + "/_deletions");
  for (auto& k : key_cols_) {
    int c = col_index(k);
    if (c < 0 || schema_[c].type != ColType::Str) throw std::runtime_error("colstore: bad key column " + k);
    key_idx_.push_back(c);
  }
  lock();
  try {
    uint64_t v = latest_version();
    if (v == 0) {
      cur_version_ = 1;
      write_manifest(1);
    } else {
      refresh();
    }
  } catch (...) { unlock(); throw; }
  unlock();
}

Table::~Table() {
  if (lock_fd_ >= 0) ::close(lock_fd_);
}

void Table::lock() {
  mu_.lock();
  if (lock_depth_++ > 0) return;
  std::string lp = dir_ + "/_lock";
  lock_fd_ = ::open(lp.c_str(), O_CREAT | O_RDWR, 0644);
  if (lock_fd_ < 0) {
    --lock_depth_;
    mu_.unlock();
    throw std::runtime_error("colstore: cannot open lock " + lp);
  }
  ::flock(lock_fd_, LOCK_EX);
}

void Table::unlock() {
  if (lock_depth_ <= 0) return;
  if (--lock_depth_ == 0 && lock_fd_ >= 0) {
    ::flock(lock_fd_, LOCK_UN);
    ::close(lock_fd_);
    lock_fd_ = -1;
  }
  mu_.unlock();
}

int Table::col_index(const std::string& name) const {
  for (size_t i = 0; i < schema_.size(); ++i)
    if (schema_[i].name == name) return (int)i;
  return -1;
}

uint64_t Table::latest_version() {
  FILE* f = fopen((dir_ + "/_latest").c_str(), "r");
  if (f) {
    unsigned long long v = 0;
    int got = fscanf(f, "%llu", &v);
    fclose(f);
    if (got == 1 && v > 0) return v;
  }
  // no pointer file (a table from an older writer): newest manifest on disk
  uint64_t best = 0;
  DIR* d = ::opendir((dir_ + "/_versions").c_str());
  if (!d) return 0;
  while (dirent* e = ::readdir(d)) {
    const char* n = e->d_name;
    size_t L = strlen(n);
    if (L > 9 && strcmp(n + L - 9, ".manifest") == 0) best = std::max<uint64_t>(best, strtoull(n, nullptr, 10));
  }
  ::closedir(d);
  return best;
}

void Table::read_manifest(uint64_t v, std::vector<Frag>& out, std::vector<ColSpec>* sch) {
  std::ifstream f(manifest_path(dir_, v));
  if (!f) throw std::runtime_error("colstore: missing manifest v" + std::to_string(v) + " in " + dir_);
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    std::string tag;
    is >> tag;
    if (tag == "col" && sch) {
      ColSpec c;
      int t;
      is >> c.name >> t >> c.dim;
      c.type = (ColType)t;
      sch->push_back(c);
    } else if (tag == "frag") {
      Frag fr;
      is >> fr.file >> fr.rows >> fr.delfile;
      if (fr.delfile == "-") fr.delfile.clear();
      out.push_back(std::move(fr));
    }
  }
}

void Table::write_manifest(uint64_t v) {
  std::ostringstream o;
  o << "LZMANIFEST 2\nversion " << v << "\n";
  for (auto& c : schema_) o << "col " << c.name << " " << (int)c.type << " " << c.dim << "\n";
  for (auto& fr : frags_) o << "frag " << fr.file << " " << fr.rows << " " << (fr.delfile.empty() ? "-" : fr.delfile) << "\n";
  atomic_write(manifest_path(dir_, v), o.str());
  atomic_write(dir_ + "/_latest", std::to_string(v) + "\n");
  cur_version_ = v;
  if (v > kKeepManifests) ::unlink(manifest_path(dir_, v - kKeepManifests).c_str());
}

void Table::load_dead(Frag& f) {
  f.dead.assign(f.rows, 0);
  f.n_dead = 0;
  if (f.delfile.empty()) return;
  auto file = ok_or_throw(arrow::io::MemoryMappedFile::Open(dir_ + "/_deletions/" + f.delfile, arrow::io::FileMode::READ),
                          "open deletion file");
  auto rd = ok_or_throw(arrow::ipc::RecordBatchFileReader::Open(file), "read deletion file");
  for (int b = 0; b < rd->num_record_batches(); ++b) {
    auto batch = ok_or_throw(rd->ReadRecordBatch(b), "deletion batch");
    auto rows = std::static_pointer_cast<arrow::UInt32Array>(batch->column(0));
    for (int64_t i = 0; i < rows->length(); ++i) {
      uint32_t r = rows->Value(i);
      if (r < f.rows && !f.dead[r]) { f.dead[r] = 1; ++f.n_dead; }
    }
  }
}

void Table::write_dead(Frag& f, uint64_t v) {
  arrow::UInt32Builder b;
  check(b.Reserve((int64_t)f.n_dead), "reserve");
  for (uint64_t r = 0; r < f.rows; ++r)
    if (f.dead[r]) b.UnsafeAppend((uint32_t)r);
  auto arr = ok_or_throw(b.Finish(), "deletion column");
  auto sch = arrow::schema({arrow::field("row", arrow::uint32())});
  std::string stem = f.file.substr(0, f.file.rfind('.'));
  char dn[160];
  snprintf(dn, sizeof dn, "%s-%llu.arrow", stem.c_str(), (unsigned long long)v);
  std::string tmp = dir_ + "/_deletions/.tmp-" + uniq_name();
  {
    auto out = ok_or_throw(arrow::io::FileOutputStream::Open(tmp), "open deletion file");
    auto w = ok_or_throw(arrow::ipc::MakeFileWriter(out, sch), "deletion writer");
    check(w->WriteRecordBatch(*arrow::RecordBatch::Make(sch, arr->length(), {arr})), "write deletions");
    check(w->Close(), "close deletions");
    check(out->Close(), "close deletions");
  }
  if (::rename(tmp.c_str(), (dir_ + "/_deletions/" + dn).c_str()) != 0)
    throw std::runtime_error("colstore: deletion rename failed");
  f.delfile = dn;
}

void Table::refresh() {
  uint64_t v = latest_version();
  if (v == 0 || v == cur_version_) return;
  std::vector<Frag> nf;
  std::vector<ColSpec> sch;
  read_manifest(v, nf, &sch);
  for (auto& c : schema_)  // adopt persisted vector dims
    for (auto& pc : sch)
      if (pc.name == c.name && c.type == ColType::VecF32 && c.dim == 0) c.dim = pc.dim;
  // incremental when the old fragments are an unchanged prefix (pure appends
  // by another writer); anything else rebuilds the state
  bool prefix = nf.size() >= frags_.size();
  for (size_t i = 0; prefix && i < frags_.size(); ++i)
    prefix = nf[i].file == frags_[i].file && nf[i].delfile == frags_[i].delfile;
  size_t from = prefix ? frags_.size() : 0;
  if (!prefix) {
    frags_.clear();
    index_.clear();
    indexed_ = false;
    indexed_frags_ = 0;
  }
  for (size_t i = from; i < nf.size(); ++i) {
    load_dead(nf[i]);
    frags_.push_back(std::move(nf[i]));
  }
  cur_version_ = v;
  if (indexed_)
    for (uint32_t fi = (uint32_t)indexed_frags_; fi < frags_.size(); ++fi) index_fragment(fi);
}

std::string Table::make_key(const std::vector<Column>& cols, size_t r) const {
  std::string k;
  for (size_t i = 0; i < key_idx_.size(); ++i) {
    if (i) k.push_back('\x1f');
    k += cols[key_idx_[i]].s[r];
  }
  return k;
}

void Table::index_fragment(uint32_t fi) {
  Frag& f = frags_[fi];
  uint64_t nrows = 0;
  auto cols = read_fragment(f.file, key_idx_, &nrows);
  for (uint64_t r = 0; r < nrows; ++r)
    if (!f.dead[r]) index_.emplace(make_key(cols, r), std::make_pair(fi, (uint32_t)r));
  indexed_frags_ = std::max<uint64_t>(indexed_frags_, fi + 1);
}

void Table::ensure_index() {
  if (indexed_ || key_idx_.empty()) return;
  index_.clear();
  indexed_frags_ = 0;
  for (uint32_t fi = 0; fi < frags_.size(); ++fi) index_fragment(fi);
  indexed_ = true;
}

// The predicate names exactly the key columns (eq on all but the last, IN on
// the last; or eq on all) -> the keys it selects.
bool Table::keyed(const Predicate& p, std::vector<std::string>* keys) const {
  if (key_cols_.empty()) return false;
  const size_t K = key_cols_.size();
  std::string prefix;
  if (p.has_in) {
    if (p.eq.size() != K - 1 || p.in_col != key_cols_[K - 1]) return false;
  } else if (p.eq.size() != K) {
    return false;
  }
  for (size_t i = 0; i + (p.has_in ? 1 : 0) < K; ++i) {
    if (p.eq[i].first != key_cols_[i]) return false;
    if (i) prefix.push_back('\x1f');
    prefix += p.eq[i].second;
  }
  keys->clear();
  if (!p.has_in) {
    keys->push_back(prefix);
  } else {
    for (auto& v : p.in_vals) keys->push_back(K > 1 ? prefix + '\x1f' + v : v);
  }
  return true;
}

bool Table::matches(const std::vector<Column>& cols, const std::vector<int>& pcols, const Predicate& p,
                    size_t r) const {
  for (size_t i = 0; i < p.eq.size(); ++i) {
    int ci = pcols[i];
    if (ci < 0 || cols[ci].s[r] != p.eq[i].second) return false;
  }
  if (p.has_in) {
    int ci = pcols[p.eq.size()];
    if (ci < 0 || !p.in_vals.count(cols[ci].s[r])) return false;
  }
  return true;
}

// Marks rows matching p as deleted (deletion files tagged with version nv).
// Keyed predicates touch only the selected rows. Caller holds the lock and has
// refreshed.
uint64_t Table::apply_delete(const Predicate& p, uint64_t nv) {
  uint64_t total = 0;
  std::vector<uint8_t> touched(frags_.size(), 0);
  std::vector<std::string> keys;
  if (keyed(p, &keys)) {
    ensure_index();
    for (auto& k : keys) {
      auto range = index_.equal_range(k);
      for (auto it = range.first; it != range.second; ++it) {
        auto [fi, r] = it->second;
        Frag& f = frags_[fi];
        if (!f.dead[r]) { f.dead[r] = 1; ++f.n_dead; ++total; touched[fi] = 1; }
      }
      index_.erase(range.first, range.second);
    }
  } else {
    std::vector<int> pcols;
    for (auto& kv : p.eq) pcols.push_back(col_index(kv.first));
    if (p.has_in) pcols.push_back(col_index(p.in_col));
    std::vector<int> need;
    for (int c : pcols) if (c >= 0 && std::find(need.begin(), need.end(), c) == need.end()) need.push_back(c);
    for (auto& k : key_idx_) if (std::find(need.begin(), need.end(), k) == need.end()) need.push_back(k);
    for (uint32_t fi = 0; fi < frags_.size(); ++fi) {
      Frag& f = frags_[fi];
      if (f.n_dead == f.rows) continue;
      uint64_t nrows = 0;
      auto cols = read_fragment(f.file, need, &nrows);
      for (uint64_t r = 0; r < nrows; ++r) {
        if (f.dead[r] || !matches(cols, pcols, p, r)) continue;
        f.dead[r] = 1;
        ++f.n_dead;
        ++total;
        touched[fi] = 1;
        if (indexed_) {
          auto range = index_.equal_range(make_key(cols, r));
          for (auto it = range.first; it != range.second; ++it)
            if (it->second == std::make_pair(fi, (uint32_t)r)) { index_.erase(it); break; }
        }
      }
    }
  }
  for (uint32_t fi = 0; fi < frags_.size(); ++fi)
    if (touched[fi]) write_dead(frags_[fi], nv);
  return total;
}

void Table::fix_dims(const std::vector<Column>& cols) {
  for (size_t i = 0; i < schema_.size(); ++i) {
    if (schema_[i].type != ColType::VecF32 || cols[i].size() == 0) continue;
    if (schema_[i].dim == 0) schema_[i].dim = cols[i].dim;
    if (schema_[i].dim != cols[i].dim) throw std::runtime_error("colstore: vector dim mismatch");
  }
}

void Table::add_fragment(const std::string& file, uint64_t rows, const std::vector<Column>* cols, uint64_t r0) {
  Frag f;
  f.file = file;
  f.rows = rows;
  f.dead.assign(rows, 0);
  frags_.push_back(std::move(f));
  const uint32_t fi = (uint32_t)frags_.size() - 1;
  if (!indexed_) return;
  if (cols) {
    for (uint64_t r = 0; r < rows; ++r) index_.emplace(make_key(*cols, r0 + r), std::make_pair(fi, (uint32_t)r));
    indexed_frags_ = fi + 1;
  } else {
    index_fragment(fi);
  }
}

// Rows [0, n) of cols as one fragment, or -- past LZK_COLSTORE_PAR_ROWS rows
// (default 2^20) -- as up to 16 fragments of consecutive row ranges encoded
// and written by one thread each (a 10M x 768 commit is 31 GB of Arrow IPC:
// one writer thread held it at ~0.7 GB/s). Caller holds the lock; the
// fragments join the table in row order, in the caller's one version.
void Table::write_fragments(const std::vector<Column>& cols, size_t n) {
  static const size_t kPar = [] {
    const char* e = getenv("LZK_COLSTORE_PAR_ROWS");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (size_t)v : (size_t(1) << 20);
  }();
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const size_t nt = std::min<size_t>(hw, std::max<size_t>(1, n / kPar));
  std::vector<std::string> files(nt);
  std::vector<size_t> lo(nt + 1);
  for (size_t t = 0; t <= nt; ++t) lo[t] = n * t / nt;
  for (auto& f : files) f = uniq_name() + ".arrow";
  if (nt == 1) {
    write_fragment(files[0], cols, 0, (int64_t)n);
  } else {
    std::vector<std::exception_ptr> err(nt);
    std::vector<std::thread> ts;
    for (size_t t = 0; t < nt; ++t)
      ts.emplace_back([&, t] {
        try {
          write_fragment(files[t], cols, (int64_t)lo[t], (int64_t)lo[t + 1]);
        } catch (...) {
          err[t] = std::current_exception();
        }
      });
    for (auto& th : ts) th.join();
    for (auto& e : err)
      if (e) std::rethrow_exception(e);
  }
  for (size_t t = 0; t < nt; ++t) add_fragment(files[t], lo[t + 1] - lo[t], &cols, lo[t]);
}

void Table::write_fragment(const std::string& file, const std::vector<Column>& cols, int64_t r_begin,
                           int64_t r_end) {
  arrow::FieldVector fields;
  std::vector<std::shared_ptr<arrow::Array>> arrays;
  int64_t width = 1;  // values per row of the widest column
  for (size_t i = 0; i < cols.size(); ++i) {
    ColSpec spec = schema_[i];
    if (spec.type == ColType::VecF32) spec.dim = cols[i].dim ? cols[i].dim : spec.dim;
    if (spec.type == ColType::VecF32) width = std::max<int64_t>(width, spec.dim);
    fields.push_back(arrow::field(spec.name, arrow_type(spec), false));
  }
  auto sch = arrow::schema(fields);
  const int64_t n = r_end >= 0 ? r_end : (cols.empty() ? 0 : (int64_t)cols[0].size());
  // record batches of <= 2^30 values per array and <= 2^30 string bytes
  // (LZK_COLSTORE_BATCH_VALUES lowers the cap: tests exercise multi-batch files)
  static const int64_t kMaxVals = [] {
    const char* e = getenv("LZK_COLSTORE_BATCH_VALUES");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (int64_t)v : (int64_t(1) << 30);
  }();
  std::string tmp = dir_ + "/data/.tmp-" + uniq_name();
  {
    auto out = ok_or_throw(arrow::io::FileOutputStream::Open(tmp), "open fragment");
    auto w = ok_or_throw(arrow::ipc::MakeFileWriter(out, sch), "fragment writer");
    int64_t r0 = r_begin;
    do {
      int64_t r1 = std::min<int64_t>(n, r0 + std::max<int64_t>(1, kMaxVals / width));
      for (size_t i = 0; i < cols.size(); ++i) {
        if (cols[i].type != ColType::Str) continue;
        int64_t bytes = 0;
        for (int64_t r = r0; r < r1; ++r) {
          bytes += (int64_t)cols[i].s[r].size();
          if (bytes > kMaxVals) { r1 = std::max<int64_t>(r0 + 1, r); break; }
        }
      }
      arrays.clear();
      for (size_t i = 0; i < cols.size(); ++i) arrays.push_back(to_arrow(cols[i], r0, r1));
      check(w->WriteRecordBatch(*arrow::RecordBatch::Make(sch, r1 - r0, arrays)), "write fragment");
      r0 = r1;
    } while (r0 < n);
    check(w->Close(), "close fragment");
    check(out->Close(), "close fragment");
  }
  if (::rename(tmp.c_str(), (dir_ + "/data/" + file).c_str()) != 0)
    throw std::runtime_error("colstore: fragment rename failed");
}

std::vector<Column> Table::read_fragment(const std::string& file, const std::vector<int>& want, uint64_t* nrows) {
  auto mm = ok_or_throw(arrow::io::MemoryMappedFile::Open(dir_ + "/data/" + file, arrow::io::FileMode::READ),
                        "open fragment");
  auto rd = ok_or_throw(arrow::ipc::RecordBatchFileReader::Open(mm), "read fragment");
  std::vector<Column> out(schema_.size());
  for (size_t i = 0; i < schema_.size(); ++i) { out[i].type = schema_[i].type; out[i].dim = schema_[i].dim; }
  // batches are zero-copy views of the mapping; size every output column
  // once, so a multi-batch fragment (> 2^30 values) is never re-allocated
  // and copied batch by batch (a 10M x 768 vector column is 8 batches)
  std::vector<std::shared_ptr<arrow::RecordBatch>> batches;
  uint64_t n = 0;
  for (int bi = 0; bi < rd->num_record_batches(); ++bi) {
    batches.push_back(ok_or_throw(rd->ReadRecordBatch(bi), "fragment batch"));
    n += (uint64_t)batches.back()->num_rows();
  }
  for (int ci : want) {
    Column& c = out[ci];
    switch (c.type) {
      case ColType::Str: c.s.reserve(n); break;
      case ColType::F64: c.f64.reserve(n); break;
      case ColType::F32: c.f32.reserve(n); break;
      case ColType::I32: c.i32.reserve(n); break;
      case ColType::I64: c.i64.reserve(n); break;
      case ColType::Bool: c.b.reserve(n); break;
      case ColType::VecF32: {
        uint32_t d = c.dim;
        if (!batches.empty()) {
          auto a = batches[0]->GetColumnByName(schema_[ci].name);
          if (a) d = (uint32_t)std::static_pointer_cast<arrow::FixedSizeListArray>(a)->list_type()->list_size();
        }
        c.f32.reserve(n * (size_t)d);
        break;
      }
    }
  }
  for (auto& batch : batches) {
    const uint64_t m = (uint64_t)batch->num_rows();
    for (int ci : want) from_arrow(batch->GetColumnByName(schema_[ci].name), out[ci], m);
  }
  *nrows = n;
  return out;
}

uint64_t Table::append(const std::vector<Column>& cols_in) {
  Predicate none;
  return replace_where(none, cols_in, nullptr);
}

uint64_t Table::delete_where(const Predicate& p, uint64_t* n_deleted) {
  lock();
  uint64_t total = 0;
  try {
    refresh();
    const uint64_t nv = cur_version_ + 1;
    total = apply_delete(p, nv);
    if (total > 0) write_manifest(nv);
  } catch (...) { unlock(); throw; }
  unlock();
  if (n_deleted) *n_deleted = total;
  return cur_version_;
}

// Delete every row matching p AND append cols in ONE committed version: a
// reader (or a crash) sees either the old rows or the new ones, never a
// table with the tenant's rows deleted but not yet re-added.
uint64_t Table::replace_where(const Predicate& p, const std::vector<Column>& cols_in, uint64_t* n_deleted) {
  if (cols_in.size() != schema_.size()) throw std::runtime_error("colstore: column count mismatch");
  const size_t n = cols_in.empty() ? 0 : cols_in[0].size();
  for (auto& c : cols_in) if (c.size() != n) throw std::runtime_error("colstore: ragged columns");
  const bool has_pred = !p.eq.empty() || p.has_in;
  lock();
  uint64_t total = 0;
  try {
    refresh();
    if (n > 0) fix_dims(cols_in);
    const uint64_t nv = cur_version_ + 1;
    if (has_pred) total = apply_delete(p, nv);
    if (n > 0) write_fragments(cols_in, n);
    if (n > 0 || total > 0 || has_pred) write_manifest(nv);
  } catch (...) { unlock(); throw; }
  unlock();
  if (n_deleted) *n_deleted = total;
  return cur_version_;
}

// Rows matching p, every wanted column. Each fragment is memory-mapped once;
// rows are selected on zero-copy views of the predicate columns, the output
// columns are sized once, and the fragments decode straight into their row
// range -- in parallel over fragments when there are several (a parallel
// commit leaves ~10 per 10M-row tenant), else with a multi-threaded copy of
// the vector column. No fragment is materialised and then copied again.
std::vector<Column> Table::scan(const Predicate& p, const std::vector<std::string>& want_names,
                                std::vector<VecPiece>* vec_pieces) {
  lock();  // a consistent fragment list (writers append under the same lock)
  std::vector<Frag> frags;
  try {
    refresh();
    frags = frags_;
  } catch (...) { unlock(); throw; }
  unlock();
  std::vector<int> pcols;
  for (auto& kv : p.eq) pcols.push_back(col_index(kv.first));
  if (p.has_in) pcols.push_back(col_index(p.in_col));
  const bool bad_pred = std::find(pcols.begin(), pcols.end(), -1) != pcols.end();
  std::vector<int> want;
  if (want_names.empty()) {
    for (size_t i = 0; i < schema_.size(); ++i) want.push_back((int)i);
  } else {
    for (auto& n : want_names) { int c = col_index(n); if (c >= 0) want.push_back(c); }
  }
  std::vector<Column> out(schema_.size());
  for (size_t i = 0; i < schema_.size(); ++i) { out[i].type = schema_[i].type; out[i].dim = schema_[i].dim; }
  if (bad_pred) return out;
  struct FR {
    std::vector<std::shared_ptr<arrow::RecordBatch>> batches;
    std::vector<uint64_t> base;  // first row of each batch
    uint64_t n = 0;
    std::vector<uint32_t> sel;
    bool all = false;
  };
  const size_t F = frags.size();
  std::vector<FR> fr(F);
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const size_t fthreads = F >= 4 ? hw : 1;
  par_for(F, fthreads, [&](size_t i) {
    const Frag& meta = frags[i];
    FR& f = fr[i];
    if (meta.n_dead == meta.rows) return;
    auto mm = ok_or_throw(arrow::io::MemoryMappedFile::Open(dir_ + "/data/" + meta.file, arrow::io::FileMode::READ),
                          "open fragment");
    auto rd = ok_or_throw(arrow::ipc::RecordBatchFileReader::Open(mm), "read fragment");
    for (int bi = 0; bi < rd->num_record_batches(); ++bi) {
      f.batches.push_back(ok_or_throw(rd->ReadRecordBatch(bi), "fragment batch"));
      f.base.push_back(f.n);
      f.n += (uint64_t)f.batches.back()->num_rows();
    }
    f.sel.reserve(f.n);
    for (size_t bi = 0; bi < f.batches.size(); ++bi) {
      auto& b = f.batches[bi];
      std::vector<std::shared_ptr<arrow::StringArray>> pa;
      bool missing = false;
      for (int ci : pcols) {
        auto arr = b->GetColumnByName(schema_[ci].name);
        if (!arr) missing = true;
        pa.push_back(std::static_pointer_cast<arrow::StringArray>(arr));
      }
      const uint64_t m = (uint64_t)b->num_rows();
      for (uint64_t r = 0; r < m; ++r) {
        const uint64_t R = f.base[bi] + r;
        if (R < meta.dead.size() && meta.dead[R]) continue;
        if (!pcols.empty()) {
          if (missing) continue;
          bool ok = true;
          for (size_t k = 0; k < p.eq.size() && ok; ++k) ok = pa[k]->GetView((int64_t)r) == p.eq[k].second;
          if (ok && p.has_in) ok = p.in_vals.count(std::string(pa.back()->GetView((int64_t)r))) > 0;
          if (!ok) continue;
        }
        f.sel.push_back((uint32_t)R);
      }
    }
    f.all = f.sel.size() == f.n;
    if (f.all) std::vector<uint32_t>().swap(f.sel);
  });
  std::vector<uint64_t> off(F + 1, 0);
  for (size_t i = 0; i < F; ++i) off[i + 1] = off[i] + (fr[i].all ? fr[i].n : fr[i].sel.size());
  const uint64_t total = off[F];
  // with vec_pieces the (first) vector column is returned as pieces, not copied
  int vcol = -1;
  if (vec_pieces)
    for (int c : want)
      if (out[c].type == ColType::VecF32) { vcol = c; break; }
  for (int c : want) {
    Column& o = out[c];
    if (o.type == ColType::VecF32 && o.dim == 0)
      for (auto& f : fr)
        if (!f.batches.empty()) {
          auto a = f.batches[0]->GetColumnByName(schema_[c].name);
          if (a) { o.dim = (uint32_t)std::static_pointer_cast<arrow::FixedSizeListArray>(a)->list_type()->list_size(); break; }
        }
    switch (o.type) {
      case ColType::Str: o.s.resize(total); break;
      case ColType::F64: o.f64.resize(total); break;
      case ColType::F32: o.f32.resize(total); break;
      case ColType::I32: o.i32.resize(total); break;
      case ColType::I64: o.i64.resize(total); break;
      case ColType::Bool: o.b.resize(total); break;
      case ColType::VecF32: if (c != vcol) o.f32.resize(total * (size_t)o.dim); break;
    }
  }
  // vector pieces, in row order: one per batch of a fully selected fragment
  // (a view of the mapping), one gathered run per partly selected fragment
  std::vector<std::vector<VecPiece>> fpieces(vcol >= 0 ? F : 0);
  const uint32_t vdim = vcol >= 0 ? out[vcol].dim : 0;
  par_for(F, fthreads, [&](size_t i) {
    FR& f = fr[i];
    if (off[i + 1] == off[i]) return;
    if (f.all) {
      for (size_t bi = 0; bi < f.batches.size(); ++bi) {
        const uint64_t m = (uint64_t)f.batches[bi]->num_rows();
        for (int c : want) {
          if (c == vcol) {
            auto a = f.batches[bi]->GetColumnByName(schema_[c].name);
            VecPiece pc;
            pc.rows = m;
            pc.dim = vdim;
            if (a) {
              auto l = std::static_pointer_cast<arrow::FixedSizeListArray>(a);
              if ((uint32_t)l->list_type()->list_size() != vdim) throw std::runtime_error("colstore: vector dim mismatch in scan");
              auto v = std::static_pointer_cast<arrow::FloatArray>(l->values());
              pc.data = v->raw_values() + l->value_offset(0);
              pc.keep = f.batches[bi];
            } else {
              pc.own.assign((size_t)m * vdim, 0.f);
              pc.data = pc.own.data();
            }
            fpieces[i].push_back(std::move(pc));
            continue;
          }
          from_arrow_at(f.batches[bi]->GetColumnByName(schema_[c].name), out[c], off[i] + f.base[bi], m);
        }
      }
      return;
    }
    if (vcol >= 0) {
      VecPiece pc;
      pc.rows = f.sel.size();
      pc.dim = vdim;
      pc.own.resize(pc.rows * (size_t)vdim);
      Column tmp;
      tmp.type = ColType::VecF32;
      tmp.dim = vdim;
      size_t b2 = 0;
      std::shared_ptr<arrow::Array> va = f.batches[0]->GetColumnByName(schema_[vcol].name);
      for (size_t j = 0; j < f.sel.size(); ++j) {
        const uint64_t R = f.sel[j];
        while (b2 + 1 < f.batches.size() && R >= f.base[b2 + 1]) va = f.batches[++b2]->GetColumnByName(schema_[vcol].name);
        if (!va) { std::fill(pc.own.begin() + j * vdim, pc.own.begin() + (j + 1) * vdim, 0.f); continue; }
        auto l = std::static_pointer_cast<arrow::FixedSizeListArray>(va);
        auto v = std::static_pointer_cast<arrow::FloatArray>(l->values());
        std::memcpy(pc.own.data() + j * vdim, v->raw_values() + l->value_offset((int64_t)(R - f.base[b2])),
                    vdim * sizeof(float));
      }
      pc.data = pc.own.data();
      fpieces[i].push_back(std::move(pc));
    }
    size_t bi = 0;
    std::vector<std::shared_ptr<arrow::Array>> arrs(schema_.size());
    auto load = [&](size_t b) { for (int c : want) arrs[c] = f.batches[b]->GetColumnByName(schema_[c].name); };
    load(0);
    for (size_t j = 0; j < f.sel.size(); ++j) {
      const uint64_t R = f.sel[j];
      while (bi + 1 < f.batches.size() && R >= f.base[bi + 1]) load(++bi);
      for (int c : want)
        if (c != vcol) row_from_arrow(arrs[c], out[c], R - f.base[bi], off[i] + j);
    }
  });
  if (vcol >= 0)
    for (auto& v : fpieces)
      for (auto& pc : v) vec_pieces->push_back(std::move(pc));
  return out;
}

uint64_t Table::count_rows() {
  lock();
  uint64_t n = 0;
  try {
    refresh();
    for (auto& fr : frags_) n += fr.rows - fr.n_dead;
  } catch (...) { unlock(); throw; }
  unlock();
  return n;
}

uint64_t Table::compact() {
  lock();
  try {
    refresh();
    bool clean = frags_.size() <= 1 && (frags_.empty() || frags_[0].n_dead == 0);
    if (clean) { unlock(); return cur_version_; }
    std::vector<int> all;
    for (size_t i = 0; i < schema_.size(); ++i) all.push_back((int)i);
    std::vector<Column> out(schema_.size());
    for (size_t i = 0; i < schema_.size(); ++i) { out[i].type = schema_[i].type; out[i].dim = schema_[i].dim; }
    for (auto& fr : frags_) {
      uint64_t nrows = 0;
      auto cols = read_fragment(fr.file, all, &nrows);
      for (uint64_t r = 0; r < nrows; ++r)
        if (!fr.dead[r])
          for (size_t c = 0; c < schema_.size(); ++c) {
            if (out[c].type == ColType::VecF32 && out[c].dim == 0) out[c].dim = cols[c].dim;
            out[c].append_from(cols[c], r);
          }
    }
    frags_.clear();
    index_.clear();
    indexed_ = false;
    indexed_frags_ = 0;
    if (!out.empty() && out[0].size() > 0) {
      std::string file = uniq_name() + ".arrow";
      write_fragment(file, out);
      add_fragment(file, out[0].size(), nullptr);
    }
    write_manifest(cur_version_ + 1);
  } catch (...) { unlock(); throw; }
  unlock();
  return cur_version_;
}

// Two-phase multi-writer commit: every rank writes its
// rows as an immutable fragment WITHOUT touching the manifest (stage), the
// fragments are gathered, and one process publishes them all in a single new
// version (commit_staged). Readers never observe a partial multi-rank update;
// a staged fragment that is never committed is unreachable garbage.
std::pair<std::string, uint64_t> Table::stage(const std::vector<Column>& cols_in) {
  if (cols_in.size() != schema_.size()) throw std::runtime_error("colstore: column count mismatch");
  const size_t n = cols_in.empty() ? 0 : cols_in[0].size();
  for (auto& c : cols_in) if (c.size() != n) throw std::runtime_error("colstore: ragged columns");
  if (n == 0) return {"", 0};
  std::string file = uniq_name() + ".arrow";
  write_fragment(file, cols_in);
  return {file, n};
}

uint64_t Table::commit_staged(const std::vector<std::pair<std::string, uint64_t>>& frags, uint32_t vec_dim) {
  lock();
  try {
    refresh();
    for (auto& sc : schema_)
      if (sc.type == ColType::VecF32) {
        if (sc.dim == 0) sc.dim = vec_dim;
        if (vec_dim && sc.dim != vec_dim) throw std::runtime_error("colstore: vector dim mismatch");
      }
    bool any = false;
    for (auto& f : frags) {
      if (f.first.empty() || f.second == 0) continue;
      add_fragment(f.first, f.second, nullptr);
      any = true;
    }
    if (any) write_manifest(cur_version_ + 1);
  } catch (...) { unlock(); throw; }
  unlock();
  return cur_version_;
}

}  // namespace lzrt
