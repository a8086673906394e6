// Versioned columnar table store -- implementation. See colstore.h.
#include "colstore.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/file.h>
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

static const char kMagic[4] = {'L', 'Z', 'C', '1'};

size_t Column::size() const {
  switch (type) {
    case ColType::Str: return s.size();
    case ColType::F64: return f64.size();
    case ColType::F32: return f32.size();
    case ColType::I32: return i32.size();
    case ColType::I64: return i64.size();
    case ColType::Bool: return b.size();
    case ColType::VecF32: return dim ? f32.size() / dim : 0;
  }
  return 0;
}

void Column::append_from(const Column& o, size_t r) {
  switch (type) {
    case ColType::Str: s.push_back(o.s[r]); break;
    case ColType::F64: f64.push_back(o.f64[r]); break;
    case ColType::F32: f32.push_back(o.f32[r]); break;
    case ColType::I32: i32.push_back(o.i32[r]); break;
    case ColType::I64: i64.push_back(o.i64[r]); break;
    case ColType::Bool: b.push_back(o.b[r]); break;
    case ColType::VecF32:
      f32.insert(f32.end(), o.f32.begin() + r * o.dim, o.f32.begin() + (r + 1) * o.dim);
      break;
  }
}

static void mkdirs(const std::string& p) {
  std::string cur;
  for (size_t i = 0; i < p.size(); ++i) {
    cur.push_back(p[i]);
    if (p[i] == '/' || i + 1 == p.size()) ::mkdir(cur.c_str(), 0755);
  }
}

static std::string uniq_name() {
  static std::atomic<uint64_t> ctr{0};
  std::random_device rd;
  uint64_t t = (uint64_t)std::chrono::high_resolution_clock::now().time_since_epoch().count();
  char buf[64];
  snprintf(buf, sizeof buf, "%016llx%08x%04llx", (unsigned long long)t, (unsigned)rd(),
           (unsigned long long)(ctr++ & 0xffff));
  return buf;
}

Table::Table(std::string dir, std::vector<ColSpec> schema) : dir_(std::move(dir)), schema_(std::move(schema)) {
  mkdirs(dir_ + "/_versions");
  mkdirs(dir_ + "/data");
  mkdirs(dir_ + "/_deletions");
  lock();
  Manifest m = load_latest();
  if (m.version == 0) {
    m.version = 1;
    m.schema = schema_;
    write_manifest(m);
  } else {
    // adopt persisted dims for vector columns
    for (auto& c : schema_)
      for (auto& pc : m.schema)
        if (pc.name == c.name && c.type == ColType::VecF32 && c.dim == 0) c.dim = pc.dim;
  }
  unlock();
}

void Table::lock() {
  if (lock_fd_ >= 0) return;
  std::string lp = dir_ + "/_lock";
  lock_fd_ = ::open(lp.c_str(), O_CREAT | O_RDWR, 0644);
  if (lock_fd_ < 0) throw std::runtime_error("colstore: cannot open lock " + lp);
  ::flock(lock_fd_, LOCK_EX);
}

void Table::unlock() {
  if (lock_fd_ < 0) return;
  ::flock(lock_fd_, LOCK_UN);
  ::close(lock_fd_);
  lock_fd_ = -1;
}

int Table::col_index(const std::string& name) const {
  for (size_t i = 0; i < schema_.size(); ++i)
    if (schema_[i].name == name) return (int)i;
  return -1;
}

uint64_t Table::latest_version() {
  uint64_t best = 0;
  DIR* d = ::opendir((dir_ + "/_versions").c_str());
  if (!d) return 0;
  while (dirent* e = ::readdir(d)) {
    const char* n = e->d_name;
    size_t L = strlen(n);
    if (L > 9 && strcmp(n + L - 9, ".manifest") == 0) {
      uint64_t v = strtoull(n, nullptr, 10);
      best = std::max(best, v);
    }
  }
  ::closedir(d);
  return best;
}

Table::Manifest Table::load_latest() {
  Manifest m;
  uint64_t v = latest_version();
  if (v == 0) return m;
  char name[64];
  snprintf(name, sizeof name, "/_versions/%020llu.manifest", (unsigned long long)v);
  std::ifstream f(dir_ + name);
  if (!f) return m;
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    std::string tag;
    is >> tag;
    if (tag == "version") {
      is >> m.version;
    } else if (tag == "col") {
      ColSpec c;
      int t;
      is >> c.name >> t >> c.dim;
      c.type = (ColType)t;
      m.schema.push_back(c);
    } else if (tag == "frag") {
      Fragment fr;
      is >> fr.file >> fr.rows >> fr.delfile;
      if (fr.delfile == "-") fr.delfile.clear();
      m.frags.push_back(fr);
    }
  }
  if (m.version == 0) m.version = v;
  return m;
}

void Table::write_manifest(const Manifest& m) {
  char name[64];
  snprintf(name, sizeof name, "/_versions/%020llu.manifest", (unsigned long long)m.version);
  std::string tmp = dir_ + "/_versions/.tmp-" + uniq_name();
  {
    std::ofstream f(tmp);
    f << "LZMANIFEST 1\n";
    f << "version " << m.version << "\n";
    for (auto& c : schema_) f << "col " << c.name << " " << (int)c.type << " " << c.dim << "\n";
    for (auto& fr : m.frags)
      f << "frag " << fr.file << " " << fr.rows << " " << (fr.delfile.empty() ? "-" : fr.delfile) << "\n";
    f.flush();
    if (!f) throw std::runtime_error("colstore: manifest write failed");
  }
  if (::rename(tmp.c_str(), (dir_ + name).c_str()) != 0)
    throw std::runtime_error("colstore: manifest rename failed");
}

static size_t payload_bytes(const Column& c) {
  size_t n = c.size();
  switch (c.type) {
    case ColType::Str: {
      size_t tot = 0;
      for (auto& x : c.s) tot += x.size();
      return 8 * (n + 1) + tot;
    }
    case ColType::F64: case ColType::I64: return 8 * n;
    case ColType::F32: case ColType::I32: return 4 * n;
    case ColType::Bool: return n;
    case ColType::VecF32: return 4 * n * (size_t)c.dim;
  }
  return 0;
}

void Table::write_fragment(const std::string& file, const std::vector<Column>& cols) {
  std::string tmp = dir_ + "/data/.tmp-" + uniq_name();
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) throw std::runtime_error("colstore: cannot write " + tmp);
  uint32_t nc = (uint32_t)cols.size();
  uint64_t nrows = cols.empty() ? 0 : cols[0].size();
  fwrite(kMagic, 1, 4, f);
  fwrite(&nc, 4, 1, f);
  fwrite(&nrows, 8, 1, f);
  uint64_t hdr = 4 + 4 + 8;
  for (size_t i = 0; i < cols.size(); ++i) hdr += 4 + schema_[i].name.size() + 1 + 4 + 8 + 8;
  uint64_t off = hdr;
  for (size_t i = 0; i < cols.size(); ++i) {
    uint32_t L = (uint32_t)schema_[i].name.size();
    fwrite(&L, 4, 1, f);
    fwrite(schema_[i].name.data(), 1, L, f);
    uint8_t t = (uint8_t)cols[i].type;
    fwrite(&t, 1, 1, f);
    uint32_t dim = cols[i].dim;
    fwrite(&dim, 4, 1, f);
    uint64_t nb = payload_bytes(cols[i]);
    fwrite(&off, 8, 1, f);
    fwrite(&nb, 8, 1, f);
    off += nb;
  }
  for (auto& c : cols) {
    switch (c.type) {
      case ColType::Str: {
        uint64_t o = 0;
        fwrite(&o, 8, 1, f);
        for (auto& x : c.s) { o += x.size(); fwrite(&o, 8, 1, f); }
        for (auto& x : c.s) fwrite(x.data(), 1, x.size(), f);
        break;
      }
      case ColType::F64: fwrite(c.f64.data(), 8, c.f64.size(), f); break;
      case ColType::I64: fwrite(c.i64.data(), 8, c.i64.size(), f); break;
      case ColType::F32: case ColType::VecF32: fwrite(c.f32.data(), 4, c.f32.size(), f); break;
      case ColType::I32: fwrite(c.i32.data(), 4, c.i32.size(), f); break;
      case ColType::Bool: fwrite(c.b.data(), 1, c.b.size(), f); break;
    }
  }
  if (fflush(f) != 0 || fclose(f) != 0) throw std::runtime_error("colstore: write failed");
  if (::rename(tmp.c_str(), (dir_ + "/data/" + file).c_str()) != 0)
    throw std::runtime_error("colstore: fragment rename failed");
}

std::vector<Column> Table::read_fragment(const std::string& file, const std::vector<int>& want) {
  std::string p = dir_ + "/data/" + file;
  FILE* f = fopen(p.c_str(), "rb");
  if (!f) throw std::runtime_error("colstore: missing fragment " + p);
  char mg[4];
  uint32_t nc;
  uint64_t nrows;
  if (fread(mg, 1, 4, f) != 4 || memcmp(mg, kMagic, 4) != 0) { fclose(f); throw std::runtime_error("colstore: bad magic " + p); }
  if (fread(&nc, 4, 1, f) != 1 || fread(&nrows, 8, 1, f) != 1) { fclose(f); throw std::runtime_error("colstore: bad header"); }
  struct Ent { std::string name; ColType t; uint32_t dim; uint64_t off, nb; };
  std::vector<Ent> ents(nc);
  for (auto& e : ents) {
    uint32_t L;
    if (fread(&L, 4, 1, f) != 1) break;
    e.name.resize(L);
    if (L && fread(&e.name[0], 1, L, f) != L) break;
    uint8_t t;
    if (fread(&t, 1, 1, f) != 1) break;
    e.t = (ColType)t;
    if (fread(&e.dim, 4, 1, f) != 1 || fread(&e.off, 8, 1, f) != 1 || fread(&e.nb, 8, 1, f) != 1) break;
  }
  std::vector<Column> out(schema_.size());
  for (size_t i = 0; i < schema_.size(); ++i) { out[i].type = schema_[i].type; out[i].dim = schema_[i].dim; }
  for (int ci : want) {
    const std::string& nm = schema_[ci].name;
    const Ent* e = nullptr;
    for (auto& x : ents) if (x.name == nm) { e = &x; break; }
    Column& c = out[ci];
    if (!e) {  // column added after this fragment was written: defaults
      switch (c.type) {
        case ColType::Str: c.s.assign(nrows, ""); break;
        case ColType::F64: c.f64.assign(nrows, 0.0); break;
        case ColType::F32: c.f32.assign(nrows, 0.f); break;
        case ColType::I32: c.i32.assign(nrows, 0); break;
        case ColType::I64: c.i64.assign(nrows, 0); break;
        case ColType::Bool: c.b.assign(nrows, 0); break;
        case ColType::VecF32: c.f32.assign(nrows * c.dim, 0.f); break;
      }
      continue;
    }
    c.dim = e->dim;
    fseek(f, (long)e->off, SEEK_SET);
    switch (c.type) {
      case ColType::Str: {
        std::vector<uint64_t> offs(nrows + 1);
        fread(offs.data(), 8, nrows + 1, f);
        std::string blob(offs[nrows], '\0');
        if (!blob.empty()) fread(&blob[0], 1, blob.size(), f);
        c.s.resize(nrows);
        for (uint64_t r = 0; r < nrows; ++r) c.s[r] = blob.substr(offs[r], offs[r + 1] - offs[r]);
        break;
      }
      case ColType::F64: c.f64.resize(nrows); fread(c.f64.data(), 8, nrows, f); break;
      case ColType::I64: c.i64.resize(nrows); fread(c.i64.data(), 8, nrows, f); break;
      case ColType::F32: c.f32.resize(nrows); fread(c.f32.data(), 4, nrows, f); break;
      case ColType::I32: c.i32.resize(nrows); fread(c.i32.data(), 4, nrows, f); break;
      case ColType::Bool: c.b.resize(nrows); fread(c.b.data(), 1, nrows, f); break;
      case ColType::VecF32: c.f32.resize(nrows * (size_t)e->dim); fread(c.f32.data(), 4, c.f32.size(), f); break;
    }
  }
  fclose(f);
  return out;
}

void Table::load_deleted(Fragment& fr) {
  if (fr.del_loaded) return;
  fr.del_loaded = true;
  fr.deleted.clear();
  if (fr.delfile.empty()) return;
  FILE* f = fopen((dir_ + "/_deletions/" + fr.delfile).c_str(), "rb");
  if (!f) return;
  uint64_t n = 0;
  fread(&n, 8, 1, f);
  fr.deleted.resize(n);
  fread(fr.deleted.data(), 4, n, f);
  fclose(f);
}

bool Table::matches(const std::vector<Column>& cols, const std::vector<int>& pcols,
                    const Predicate& p, size_t r) const {
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

uint64_t Table::append(const std::vector<Column>& cols_in) {
  if (cols_in.size() != schema_.size()) throw std::runtime_error("colstore: column count mismatch");
  size_t n = cols_in.empty() ? 0 : cols_in[0].size();
  for (auto& c : cols_in) if (c.size() != n) throw std::runtime_error("colstore: ragged columns");
  lock();
  Manifest m = load_latest();
  if (n == 0) { unlock(); return m.version; }
  for (size_t i = 0; i < schema_.size(); ++i) {
    if (schema_[i].type == ColType::VecF32) {
      uint32_t d = cols_in[i].dim;
      for (auto& pc : m.schema) if (pc.name == schema_[i].name && pc.dim) schema_[i].dim = pc.dim;
      if (schema_[i].dim == 0) schema_[i].dim = d;
      if (schema_[i].dim != d) { unlock(); throw std::runtime_error("colstore: vector dim mismatch"); }
    }
  }
  std::string file = uniq_name() + ".lzc";
  try {
    write_fragment(file, cols_in);
    Fragment fr;
    fr.file = file;
    fr.rows = n;
    m.frags.push_back(fr);
    m.version += 1;
    write_manifest(m);
  } catch (...) { unlock(); throw; }
  unlock();
  return m.version;
}

// Marks rows matching p as deleted in m (new deletion files tagged with
// version nv); fully deleted fragments leave the manifest. Caller holds the lock.
uint64_t Table::apply_delete(Manifest& m, const Predicate& p, uint64_t nv) {
  std::vector<int> pcols;
  for (auto& kv : p.eq) pcols.push_back(col_index(kv.first));
  if (p.has_in) pcols.push_back(col_index(p.in_col));
  uint64_t total = 0;
  std::vector<Fragment> keep;
  for (auto& fr : m.frags) {
    load_deleted(fr);
    std::vector<int> need;
    for (int c : pcols) if (c >= 0) need.push_back(c);
    auto cols = read_fragment(fr.file, need);
    std::vector<uint32_t> del = fr.deleted;
    std::vector<char> dead(fr.rows, 0);
    for (auto d : del) if (d < fr.rows) dead[d] = 1;
    uint64_t added = 0;
    for (uint64_t r = 0; r < fr.rows; ++r) {
      if (dead[r]) continue;
      if (matches(cols, pcols, p, r)) { dead[r] = 1; ++added; }
    }
    if (added == 0) { keep.push_back(fr); continue; }
    total += added;
    uint64_t live = 0;
    del.clear();
    for (uint64_t r = 0; r < fr.rows; ++r) { if (dead[r]) del.push_back((uint32_t)r); else ++live; }
    if (live == 0) continue;  // fragment fully deleted: drop from this version
    std::string stem = fr.file.substr(0, fr.file.size() - 4);
    char dn[128];
    snprintf(dn, sizeof dn, "%s-%llu.del", stem.c_str(), (unsigned long long)nv);
    FILE* f = fopen((dir_ + "/_deletions/" + dn).c_str(), "wb");
    if (!f) throw std::runtime_error("colstore: cannot write deletion file");
    uint64_t nd = del.size();
    bool ok = fwrite(&nd, 8, 1, f) == 1 && fwrite(del.data(), 4, nd, f) == nd;
    ok = (fclose(f) == 0) && ok;
    if (!ok) throw std::runtime_error("colstore: short write of deletion file");
    Fragment nf = fr;
    nf.delfile = dn;
    nf.deleted = del;
    keep.push_back(nf);
  }
  m.frags = keep;
  return total;
}

uint64_t Table::delete_where(const Predicate& p, uint64_t* n_deleted) {
  lock();
  Manifest m;
  uint64_t total = 0;
  try {
    m = load_latest();
    const uint64_t nv = m.version + 1;
    total = apply_delete(m, p, nv);
    if (total > 0) {
      m.version = nv;
      write_manifest(m);
    }
  } catch (...) { unlock(); throw; }
  unlock();
  if (n_deleted) *n_deleted = total;
  return m.version;
}

// Delete every row matching p AND append cols in ONE committed version: a
// reader (or a crash) sees either the old rows or the new ones, never a
// table with the tenant's rows deleted but not yet re-added.
uint64_t Table::replace_where(const Predicate& p, const std::vector<Column>& cols_in, uint64_t* n_deleted) {
  if (cols_in.size() != schema_.size()) throw std::runtime_error("colstore: column count mismatch");
  const size_t n = cols_in.empty() ? 0 : cols_in[0].size();
  for (auto& c : cols_in) if (c.size() != n) throw std::runtime_error("colstore: ragged columns");
  lock();
  Manifest m;
  uint64_t total = 0;
  try {
    m = load_latest();
    for (size_t i = 0; i < schema_.size(); ++i) {
      if (schema_[i].type == ColType::VecF32 && n > 0) {
        uint32_t d = cols_in[i].dim;
        for (auto& pc : m.schema) if (pc.name == schema_[i].name && pc.dim) schema_[i].dim = pc.dim;
        if (schema_[i].dim == 0) schema_[i].dim = d;
        if (schema_[i].dim != d) throw std::runtime_error("colstore: vector dim mismatch");
      }
    }
    const uint64_t nv = m.version + 1;
    total = apply_delete(m, p, nv);
    if (n > 0) {
      std::string file = uniq_name() + ".lzc";
      write_fragment(file, cols_in);
      Fragment fr;
      fr.file = file;
      fr.rows = n;
      m.frags.push_back(fr);
    }
    m.version = nv;
    write_manifest(m);
  } catch (...) { unlock(); throw; }
  unlock();
  if (n_deleted) *n_deleted = total;
  return m.version;
}

std::vector<Column> Table::scan(const Predicate& p, const std::vector<std::string>& want_names) {
  Manifest m = load_latest();
  for (auto& c : schema_)
    for (auto& pc : m.schema)
      if (pc.name == c.name && c.type == ColType::VecF32 && c.dim == 0) c.dim = pc.dim;
  std::vector<int> pcols;
  for (auto& kv : p.eq) pcols.push_back(col_index(kv.first));
  if (p.has_in) pcols.push_back(col_index(p.in_col));
  std::vector<int> want;
  if (want_names.empty()) {
    for (size_t i = 0; i < schema_.size(); ++i) want.push_back((int)i);
  } else {
    for (auto& n : want_names) { int c = col_index(n); if (c >= 0) want.push_back(c); }
  }
  std::vector<int> need = want;
  for (int c : pcols) if (c >= 0 && std::find(need.begin(), need.end(), c) == need.end()) need.push_back(c);
  std::vector<Column> out(schema_.size());
  for (size_t i = 0; i < schema_.size(); ++i) { out[i].type = schema_[i].type; out[i].dim = schema_[i].dim; }
  for (auto& fr : m.frags) {
    load_deleted(fr);
    auto cols = read_fragment(fr.file, need);
    std::vector<char> dead(fr.rows, 0);
    for (auto d : fr.deleted) if (d < fr.rows) dead[d] = 1;
    for (uint64_t r = 0; r < fr.rows; ++r) {
      if (dead[r] || !matches(cols, pcols, p, r)) continue;
      for (int c : want) {
        if (out[c].type == ColType::VecF32 && out[c].dim == 0) out[c].dim = cols[c].dim;
        out[c].append_from(cols[c], r);
      }
    }
  }
  return out;
}

uint64_t Table::count_rows() {
  Manifest m = load_latest();
  uint64_t n = 0;
  for (auto& fr : m.frags) { load_deleted(fr); n += fr.rows - fr.deleted.size(); }
  return n;
}

uint64_t Table::compact() {
  lock();
  Manifest m = load_latest();
  if (m.frags.size() <= 1) {
    bool clean = m.frags.empty() || m.frags[0].delfile.empty();
    if (clean) { unlock(); return m.version; }
  }
  std::vector<int> all;
  for (size_t i = 0; i < schema_.size(); ++i) all.push_back((int)i);
  std::vector<Column> out(schema_.size());
  for (size_t i = 0; i < schema_.size(); ++i) { out[i].type = schema_[i].type; out[i].dim = schema_[i].dim; }
  for (auto& fr : m.frags) {
    load_deleted(fr);
    auto cols = read_fragment(fr.file, all);
    std::vector<char> dead(fr.rows, 0);
    for (auto d : fr.deleted) if (d < fr.rows) dead[d] = 1;
    for (uint64_t r = 0; r < fr.rows; ++r)
      if (!dead[r])
        for (size_t c = 0; c < schema_.size(); ++c) {
          if (out[c].type == ColType::VecF32 && out[c].dim == 0) out[c].dim = cols[c].dim;
          out[c].append_from(cols[c], r);
        }
  }
  m.frags.clear();
  if (!out.empty() && out[0].size() > 0) {
    std::string file = uniq_name() + ".lzc";
    write_fragment(file, out);
    Fragment fr;
    fr.file = file;
    fr.rows = out[0].size();
    m.frags.push_back(fr);
  }
  m.version += 1;
  write_manifest(m);
  unlock();
  return m.version;
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
  std::string file = uniq_name() + ".lzc";
  write_fragment(file, cols_in);
  return {file, n};
}

uint64_t Table::commit_staged(const std::vector<std::pair<std::string, uint64_t>>& frags, uint32_t vec_dim) {
  lock();
  Manifest m;
  try {
    m = load_latest();
    for (auto& sc : schema_)
      if (sc.type == ColType::VecF32) {
        for (auto& pc : m.schema) if (pc.name == sc.name && pc.dim) sc.dim = pc.dim;
        if (sc.dim == 0) sc.dim = vec_dim;
        if (vec_dim && sc.dim != vec_dim) throw std::runtime_error("colstore: vector dim mismatch");
      }
    bool any = false;
    for (auto& f : frags) {
      if (f.first.empty() || f.second == 0) continue;
      Fragment fr;
      fr.file = f.first;
      fr.rows = f.second;
      m.frags.push_back(fr);
      any = true;
    }
    if (any) {
      m.version += 1;
      write_manifest(m);
    }
  } catch (...) { unlock(); throw; }
  unlock();
  return m.version;
}

}  // namespace lzrt
