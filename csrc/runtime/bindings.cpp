// pybind11 bindings for the host runtime (module `lazzaro_amd._lib._lzrt`).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <string_view>
#include <unordered_map>

#include "colstore.h"
#include "tokenizer.h"
#include "graph_host.h"
#include "batch_plan.h"

namespace py = pybind11;
using namespace lzrt;

namespace lzrt {
int add_strcol(PyObject* m);  // strcol.cpp
}

namespace {

// Python column -> Column. String lists are read through the CPython API
// (the UTF-8 of a compact str is cached in the object: no encode) and a run of
// the same object (["{}"] * n, a constant user_id) copies the previous value;
// fp32 arrays are BORROWED (Column::ext) -- `keep` holds them until the call
// that uses the columns returns.
Column to_column(const ColSpec& spec, py::handle obj, std::vector<py::object>& keep) {
  Column c;
  c.type = spec.type;
  c.dim = spec.dim;
  switch (spec.type) {
    case ColType::Str: {
      PyObject* seq = PySequence_Fast(obj.ptr(), "string column must be a sequence");
      if (!seq) throw py::error_already_set();
      const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
      PyObject** items = PySequence_Fast_ITEMS(seq);
      c.s.resize((size_t)n);
      PyObject* prev = nullptr;
      for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* o = items[i];
        if (o == prev) { c.s[i] = c.s[i - 1]; continue; }
        if (PyUnicode_Check(o)) {
          Py_ssize_t len = 0;
          const char* p = PyUnicode_AsUTF8AndSize(o, &len);
          if (!p) { Py_DECREF(seq); throw py::error_already_set(); }
          c.s[i].assign(p, (size_t)len);
        } else {
          c.s[i] = py::cast<std::string>(py::handle(o));
        }
        prev = o;
      }
      Py_DECREF(seq);
      break;
    }
    case ColType::F64: {
      auto a = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(obj);
      c.f64.assign(a.data(), a.data() + a.size());
      break;
    }
    case ColType::F32: {
      auto a = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(obj);
      c.ext = a.data();
      c.ext_n = (size_t)a.size();
      keep.push_back(a);
      break;
    }
    case ColType::I32: {
      auto a = py::array_t<int32_t, py::array::c_style | py::array::forcecast>::ensure(obj);
      c.i32.assign(a.data(), a.data() + a.size());
      break;
    }
    case ColType::I64: {
      auto a = py::array_t<int64_t, py::array::c_style | py::array::forcecast>::ensure(obj);
      c.i64.assign(a.data(), a.data() + a.size());
      break;
    }
    case ColType::Bool: {
      auto a = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>::ensure(obj);
      c.b.assign(a.data(), a.data() + a.size());
      break;
    }
    case ColType::VecF32: {
      auto a = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(obj);
      if (a.ndim() != 2) throw std::runtime_error("vector column must be 2-D");
      c.dim = (uint32_t)a.shape(1);
      c.ext = a.data();
      c.ext_n = (size_t)a.size();
      keep.push_back(a);
      break;
    }
  }
  return c;
}

// numpy array that takes ownership of the vector's buffer (no copy: a
// 10M x 768 vector column is 30 GB)
template <class V>
py::array_t<typename V::value_type> adopt(V&& v, std::vector<py::ssize_t> shape) {
  auto* heap = new V(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<V*>(p); });
  return py::array_t<typename V::value_type>(shape, heap->data(), owner);
}

py::object from_column(Column& c) {
  switch (c.type) {
    case ColType::Str: {
      // CPython API directly (a 10M-row column is 10M objects), and values
      // that repeat (type, shard_key, parent_id, "[]", "{}") share one str
      // object -- a bounded intern cache, so unique columns (id, content)
      // only pay for its lookups until it fills
      const size_t n = c.s.size();
      PyObject* l = PyList_New((Py_ssize_t)n);
      if (!l) throw py::error_already_set();
      std::unordered_map<std::string_view, PyObject*> cache;
      constexpr size_t kCacheMax = 4096;
      size_t misses = 0;
      for (size_t i = 0; i < n; ++i) {
        const std::string& v = c.s[i];
        PyObject* o = nullptr;
        if (misses < 4 * kCacheMax) {
          auto it = cache.find(std::string_view(v));
          if (it != cache.end()) {
            o = it->second;
            Py_INCREF(o);
          } else {
            ++misses;
          }
        }
        if (!o) {
          o = PyUnicode_DecodeUTF8(v.data(), (Py_ssize_t)v.size(), "replace");
          if (!o) { Py_DECREF(l); throw py::error_already_set(); }
          if (cache.size() < kCacheMax && misses < 4 * kCacheMax) {
            Py_INCREF(o);
            cache.emplace(std::string_view(v), o);
          }
        }
        PyList_SET_ITEM(l, (Py_ssize_t)i, o);
      }
      for (auto& kv : cache) Py_DECREF(kv.second);
      return py::reinterpret_steal<py::object>(l);
    }
    case ColType::F64: { auto n = (py::ssize_t)c.f64.size(); return adopt(std::move(c.f64), {n}); }
    case ColType::F32: { auto n = (py::ssize_t)c.f32.size(); return adopt(std::move(c.f32), {n}); }
    case ColType::I32: { auto n = (py::ssize_t)c.i32.size(); return adopt(std::move(c.i32), {n}); }
    case ColType::I64: { auto n = (py::ssize_t)c.i64.size(); return adopt(std::move(c.i64), {n}); }
    case ColType::Bool: { auto n = (py::ssize_t)c.b.size(); return adopt(std::move(c.b), {n}); }
    case ColType::VecF32: {
      auto n = (py::ssize_t)c.size();
      return adopt(std::move(c.f32), {n, (py::ssize_t)c.dim});
    }
  }
  return py::none();
}

Predicate make_pred(const std::vector<std::pair<std::string, std::string>>& eq,
                    const std::string& in_col, const py::object& in_vals) {
  Predicate p;
  p.eq = eq;
  if (!in_col.empty() && !in_vals.is_none()) {
    p.has_in = true;
    p.in_col = in_col;
    for (auto v : in_vals) p.in_vals.insert(py::cast<std::string>(v));
  }
  return p;
}

}  // namespace

PYBIND11_MODULE(_lzrt, m) {
  m.doc() = "lazzaro_amd host runtime: columnar store, tokenizer, graph utilities";

  py::class_<Table>(m, "Table")
      .def(py::init([](const std::string& dir, const std::vector<std::tuple<std::string, int, int>>& sch,
                       const std::vector<std::string>& keys) {
             std::vector<ColSpec> s;
             for (auto& t : sch) s.push_back({std::get<0>(t), (ColType)std::get<1>(t), (uint32_t)std::get<2>(t)});
             py::gil_scoped_release r;
             return new Table(dir, s, keys);
           }),
           py::arg("dir"), py::arg("schema"), py::arg("key_cols") = std::vector<std::string>{})
      .def("latest_version", [](Table& t) { py::gil_scoped_release r; return t.latest_version(); })
      .def("count_rows", [](Table& t) { py::gil_scoped_release r; return t.count_rows(); })
      .def("compact", [](Table& t) { py::gil_scoped_release r; return t.compact(); })
      .def("append", [](Table& t, py::dict cols) {
        std::vector<Column> cs;
        std::vector<py::object> keep;
        for (auto& spec : t.schema()) {
          if (!cols.contains(spec.name.c_str())) throw std::runtime_error("missing column " + spec.name);
          cs.push_back(to_column(spec, cols[spec.name.c_str()], keep));
        }
        py::gil_scoped_release r;
        return t.append(cs);
      })
      .def("delete_where",
           [](Table& t, const std::vector<std::pair<std::string, std::string>>& eq, const std::string& in_col,
              py::object in_vals) {
             Predicate p = make_pred(eq, in_col, in_vals);
             uint64_t n = 0, v;
             {
               py::gil_scoped_release r;
               v = t.delete_where(p, &n);
             }
             return py::make_tuple(n, v);
           },
           py::arg("eq"), py::arg("in_col") = "", py::arg("in_vals") = py::none())
      .def("stage",
           [](Table& t, py::dict cols) {
             std::vector<Column> cs;
             std::vector<py::object> keep;
             uint32_t dim = 0;
             for (auto& spec : t.schema()) {
               if (!cols.contains(spec.name.c_str())) throw std::runtime_error("missing column " + spec.name);
               cs.push_back(to_column(spec, cols[spec.name.c_str()], keep));
               if (spec.type == ColType::VecF32) dim = cs.back().dim;
             }
             std::pair<std::string, uint64_t> r;
             {
               py::gil_scoped_release g;
               r = t.stage(cs);
             }
             return py::make_tuple(r.first, r.second, dim);
           })
      .def("commit_staged",
           [](Table& t, const std::vector<std::pair<std::string, uint64_t>>& frags, uint32_t dim) {
             py::gil_scoped_release g;
             return t.commit_staged(frags, dim);
           },
           py::arg("frags"), py::arg("vec_dim") = 0)
      .def("replace_where",
           [](Table& t, const std::vector<std::pair<std::string, std::string>>& eq, const std::string& in_col,
              py::object in_vals, py::dict cols) {
             Predicate p = make_pred(eq, in_col, in_vals);
             std::vector<Column> cs;
             std::vector<py::object> keep;
             for (auto& spec : t.schema()) {
               if (!cols.contains(spec.name.c_str())) throw std::runtime_error("missing column " + spec.name);
               cs.push_back(to_column(spec, cols[spec.name.c_str()], keep));
             }
             uint64_t n = 0, v;
             {
               py::gil_scoped_release r;
               v = t.replace_where(p, cs, &n);
             }
             return py::make_tuple(n, v);
           },
           py::arg("eq"), py::arg("in_col"), py::arg("in_vals"), py::arg("cols"))
      .def("scan",
           [](Table& t, const std::vector<std::pair<std::string, std::string>>& eq, const std::string& in_col,
              py::object in_vals, const std::vector<std::string>& want, bool vec_pieces) {
             Predicate p = make_pred(eq, in_col, in_vals);
             std::vector<Column> cols;
             std::vector<VecPiece> pieces;
             {
               py::gil_scoped_release r;
               cols = t.scan(p, want, vec_pieces ? &pieces : nullptr);
             }
             py::dict d;
             const auto& sch = t.schema();
             bool vec_done = false;
             for (size_t i = 0; i < sch.size(); ++i) {
               bool w = want.empty();
               for (auto& n : want) if (n == sch[i].name) w = true;
               if (!w) continue;
               if (vec_pieces && !vec_done && sch[i].type == ColType::VecF32) {
                 // list of [rows, dim] arrays in row order: views of the mapped
                 // fragments (kept alive by the arrays) or gathered copies
                 py::list l;
                 for (auto& pc : pieces) {
                   const py::ssize_t rows = (py::ssize_t)pc.rows, dim = (py::ssize_t)pc.dim;
                   if (pc.keep) {
                     auto* hold = new std::shared_ptr<void>(pc.keep);
                     py::capsule cap(hold, [](void* q) { delete reinterpret_cast<std::shared_ptr<void>*>(q); });
                     l.append(py::array_t<float>({rows, dim}, pc.data, cap));
                   } else {
                     l.append(adopt(std::move(pc.own), {rows, dim}));
                   }
                 }
                 d[sch[i].name.c_str()] = l;
                 vec_done = true;
                 continue;
               }
               d[sch[i].name.c_str()] = from_column(cols[i]);
             }
             return d;
           },
           py::arg("eq") = std::vector<std::pair<std::string, std::string>>{}, py::arg("in_col") = "",
           py::arg("in_vals") = py::none(), py::arg("want") = std::vector<std::string>{},
           py::arg("vec_pieces") = false);

  // ---- tokenizer ----
  py::class_<Tokenizer>(m, "Tokenizer")
      .def(py::init<int, bool>(), py::arg("vocab_size") = 30522, py::arg("lower") = true)
      .def("load_vocab", &Tokenizer::load_vocab)
      .def("has_vocab", &Tokenizer::has_vocab)
      .def("encode", [](Tokenizer& t, const std::string& s, int max_len) { return t.encode(s, max_len); },
           py::arg("text"), py::arg("max_len") = 512)
      .def("encode_batch",
           [](Tokenizer& t, const std::vector<std::string>& texts, int max_len) {
             std::vector<int32_t> ids, lens;
             int S = 0;
             {
               py::gil_scoped_release r;
               S = t.encode_batch(texts, max_len, ids, lens);
             }
             py::array_t<int32_t> a({(py::ssize_t)texts.size(), (py::ssize_t)S});
             if (!ids.empty()) std::memcpy(a.mutable_data(), ids.data(), ids.size() * 4);
             py::array_t<int32_t> l(lens.size(), lens.data());
             return py::make_tuple(a, l);
           },
           py::arg("texts"), py::arg("max_len") = 512)
      .def("encode_chunks",
           [](Tokenizer& t, const std::vector<std::string>& texts, int max_len, int overlap) {
             std::vector<int32_t> ids, lens, owner;
             int S = 0;
             {
               py::gil_scoped_release r;
               S = t.encode_chunks(texts, max_len, overlap, ids, lens, owner);
             }
             py::array_t<int32_t> a({(py::ssize_t)lens.size(), (py::ssize_t)S});
             if (!ids.empty()) std::memcpy(a.mutable_data(), ids.data(), ids.size() * 4);
             return py::make_tuple(a, py::array_t<int32_t>(lens.size(), lens.data()),
                                   py::array_t<int32_t>(owner.size(), owner.data()));
           },
           py::arg("texts"), py::arg("max_len") = 512, py::arg("overlap") = 64);

  // ---- graph host utilities ----
  m.def("build_csr",
        [](py::array_t<int32_t, py::array::c_style | py::array::forcecast> src,
           py::array_t<int32_t, py::array::c_style | py::array::forcecast> dst, int n, bool undirected) {
          std::vector<int64_t> off;
          std::vector<int32_t> adj, eid;
          build_csr(src.data(), dst.data(), (int64_t)src.size(), n, undirected, off, adj, eid);
          return py::make_tuple(py::array_t<int64_t>(off.size(), off.data()),
                                py::array_t<int32_t>(adj.size(), adj.data()),
                                py::array_t<int32_t>(eid.size(), eid.data()));
        });
  m.def("par_copy",
        [](uintptr_t dst, uintptr_t src, size_t bytes) {
          // multi-threaded host memcpy with the GIL released (staging copies)
          py::gil_scoped_release r;
          lzrt::parallel_copy(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), bytes);
        },
        py::arg("dst"), py::arg("src"), py::arg("bytes"));
  m.def("max_node_num",
        [](py::object ids_any) {
          // largest n of "node_<n>" ids (the reference's id scheme), 0 if none;
          // any sequence of str (a list, a StrColumn)
          PyObject* seq = PySequence_Fast(ids_any.ptr(), "max_node_num needs a sequence");
          if (!seq) throw py::error_already_set();
          py::list ids = py::reinterpret_steal<py::list>(PySequence_List(seq));
          Py_DECREF(seq);
          if (!ids) throw py::error_already_set();
          long long mx = 0;
          for (auto h : ids) {
            PyObject* o = h.ptr();
            if (!PyUnicode_Check(o)) continue;
            Py_ssize_t len = 0;
            const char* p = PyUnicode_AsUTF8AndSize(o, &len);
            if (!p || len <= 5 || len > 5 + 18 || std::memcmp(p, "node_", 5) != 0) continue;
            long long v = 0;
            bool ok = true;
            for (Py_ssize_t i = 5; i < len; ++i) {
              if (p[i] < '0' || p[i] > '9') { ok = false; break; }
              v = v * 10 + (p[i] - '0');
            }
            if (ok && v > mx) mx = v;
          }
          PyErr_Clear();
          return mx;
        },
        py::arg("ids"));
  m.def("union_find_components",
        [](py::array_t<int32_t, py::array::c_style | py::array::forcecast> src,
           py::array_t<int32_t, py::array::c_style | py::array::forcecast> dst, int n) {
          std::vector<int32_t> lab;
          union_find(src.data(), dst.data(), (int64_t)src.size(), n, lab);
          return py::array_t<int32_t>(lab.size(), lab.data());
        });
  m.def("tenant_rank_among", &tenant_rank_among, py::arg("tenant"), py::arg("ranks"),
        "rendezvous-hash owner of a tenant among an explicit set of rank ids");
  m.def("tenant_rank", &tenant_rank, py::arg("tenant"), py::arg("world"),
        "consistent-hash placement of a tenant id onto one of `world` ranks");
  register_batch_plan(m);
  if (lzrt::add_strcol(m.ptr()) < 0) throw py::error_already_set();
}
