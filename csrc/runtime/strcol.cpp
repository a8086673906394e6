// StrColumn: a tenant's per-row host strings (node ids, contents, types) in
// one native array of references that the cyclic garbage collector never
// traverses.
//
// Why: a 10M-row tenant held three Python lists of 10M references each. The
// collector's full passes visit every reference of every tracked container,
// and CPython's trigger (long-lived *objects* pending) counts a 10M-entry
// list as one object, so full passes ran every few serving steps at ~5-7 ms
// each (profiles/r4/headline_host_profile_gc_stalls.txt). The round-4 fix
// froze the whole interpreter heap (gc.freeze) from inside the library. The
// strings themselves are immutable atoms that can be part of no reference
// cycle, so a container of them needs no traversal: this type is not
// GC-tracked (no Py_TPFLAGS_HAVE_GC) and gc.freeze is gone.
//
// Python surface (what TenantGraph and the views use of a list): len, [i]
// (negative i too), [i] = s, [a:b] -> list, iteration, append, extend,
// take(rows) -> list (None for a negative row), tolist(). The item access
// goes through the sequence / mapping slots directly (no argument parsing),
// so g.ids[r] costs what a list index costs.
#include <Python.h>

#include <cstdlib>
#include <cstring>

namespace {

struct StrCol {
  PyObject_HEAD
  PyObject** items;
  Py_ssize_t n;
  Py_ssize_t cap;
};

int reserve(StrCol* self, Py_ssize_t need) {
  if (need <= self->cap) return 0;
  Py_ssize_t cap = self->cap ? self->cap : 16;
  while (cap < need) cap = cap + cap / 2 + 16;
  PyObject** p = static_cast<PyObject**>(std::realloc(self->items, (size_t)cap * sizeof(PyObject*)));
  if (!p) {
    PyErr_NoMemory();
    return -1;
  }
  self->items = p;
  self->cap = cap;
  return 0;
}

void sc_dealloc(StrCol* self) {
  // a heap type (PyType_FromSpec): every instance holds a reference to it
  PyTypeObject* tp = Py_TYPE(self);
  for (Py_ssize_t i = 0; i < self->n; ++i) Py_XDECREF(self->items[i]);
  std::free(self->items);
  tp->tp_free(reinterpret_cast<PyObject*>(self));
  Py_DECREF(tp);
}

// Items are str or None only: the type is not GC-tracked, so an item that
// could refer back to the column would make a cycle the collector never frees.
int check_item(PyObject* v) {
  if (v == Py_None || PyUnicode_Check(v)) return 0;
  PyErr_Format(PyExc_TypeError, "StrColumn holds str or None, not %.100s", Py_TYPE(v)->tp_name);
  return -1;
}

int extend_from(StrCol* self, PyObject* it) {
  PyObject* seq = PySequence_Fast(it, "StrColumn.extend needs an iterable");
  if (!seq) return -1;
  const Py_ssize_t m = PySequence_Fast_GET_SIZE(seq);
  if (reserve(self, self->n + m) < 0) {
    Py_DECREF(seq);
    return -1;
  }
  PyObject** src = PySequence_Fast_ITEMS(seq);
  for (Py_ssize_t i = 0; i < m; ++i) {
    if (check_item(src[i]) < 0) {
      Py_DECREF(seq);
      return -1;
    }
  }
  for (Py_ssize_t i = 0; i < m; ++i) {
    Py_INCREF(src[i]);
    self->items[self->n + i] = src[i];
  }
  self->n += m;
  Py_DECREF(seq);
  return 0;
}

int sc_init(StrCol* self, PyObject* args, PyObject* kwds) {
  PyObject* it = nullptr;
  static const char* kw[] = {"iterable", nullptr};
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|O", const_cast<char**>(kw), &it)) return -1;
  for (Py_ssize_t i = 0; i < self->n; ++i) Py_XDECREF(self->items[i]);
  self->n = 0;
  if (it && it != Py_None) return extend_from(self, it);
  return 0;
}

Py_ssize_t sc_len(StrCol* self) { return self->n; }

PyObject* sc_item(StrCol* self, Py_ssize_t i) {
  if (i < 0 || i >= self->n) {
    PyErr_SetString(PyExc_IndexError, "StrColumn index out of range");
    return nullptr;
  }
  PyObject* o = self->items[i];
  Py_INCREF(o);
  return o;
}

int sc_ass_item(StrCol* self, Py_ssize_t i, PyObject* v) {
  if (!v) {
    PyErr_SetString(PyExc_TypeError, "StrColumn does not support item deletion");
    return -1;
  }
  if (i < 0 || i >= self->n) {
    PyErr_SetString(PyExc_IndexError, "StrColumn assignment index out of range");
    return -1;
  }
  if (check_item(v) < 0) return -1;
  Py_INCREF(v);
  PyObject* old = self->items[i];
  self->items[i] = v;
  Py_XDECREF(old);
  return 0;
}

PyObject* slice_list(StrCol* self, Py_ssize_t a, Py_ssize_t step, Py_ssize_t len) {
  PyObject* out = PyList_New(len);
  if (!out) return nullptr;
  for (Py_ssize_t k = 0; k < len; ++k) {
    PyObject* o = self->items[a + k * step];
    Py_INCREF(o);
    PyList_SET_ITEM(out, k, o);
  }
  return out;
}

PyObject* sc_subscript(StrCol* self, PyObject* key) {
  if (PyIndex_Check(key)) {
    Py_ssize_t i = PyNumber_AsSsize_t(key, PyExc_IndexError);
    if (i == -1 && PyErr_Occurred()) return nullptr;
    if (i < 0) i += self->n;
    return sc_item(self, i);
  }
  if (PySlice_Check(key)) {
    Py_ssize_t a, b, step;
    if (PySlice_Unpack(key, &a, &b, &step) < 0) return nullptr;
    const Py_ssize_t len = PySlice_AdjustIndices(self->n, &a, &b, step);
    return slice_list(self, a, step, len);
  }
  PyErr_SetString(PyExc_TypeError, "StrColumn indices must be integers or slices");
  return nullptr;
}

int sc_ass_subscript(StrCol* self, PyObject* key, PyObject* v) {
  if (!PyIndex_Check(key)) {
    PyErr_SetString(PyExc_TypeError, "StrColumn assignment index must be an integer");
    return -1;
  }
  Py_ssize_t i = PyNumber_AsSsize_t(key, PyExc_IndexError);
  if (i == -1 && PyErr_Occurred()) return -1;
  if (i < 0) i += self->n;
  return sc_ass_item(self, i, v);
}

PyObject* sc_tolist(StrCol* self, PyObject*) { return slice_list(self, 0, 1, self->n); }

PyObject* sc_iter(StrCol* self) {
  // a snapshot list's iterator: appends during the iteration are not seen
  PyObject* l = sc_tolist(self, nullptr);
  if (!l) return nullptr;
  PyObject* it = PyObject_GetIter(l);
  Py_DECREF(l);
  return it;
}

PyObject* sc_append(StrCol* self, PyObject* v) {
  if (check_item(v) < 0 || reserve(self, self->n + 1) < 0) return nullptr;
  Py_INCREF(v);
  self->items[self->n++] = v;
  Py_RETURN_NONE;
}

PyObject* sc_extend(StrCol* self, PyObject* it) {
  if (extend_from(self, it) < 0) return nullptr;
  Py_RETURN_NONE;
}

// take(rows): [self[r] for r in rows] with None for r < 0 (rows: any
// sequence of ints, e.g. a list from a tensor's tolist())
PyObject* sc_take(StrCol* self, PyObject* rows) {
  PyObject* seq = PySequence_Fast(rows, "StrColumn.take needs a sequence of ints");
  if (!seq) return nullptr;
  const Py_ssize_t m = PySequence_Fast_GET_SIZE(seq);
  PyObject** src = PySequence_Fast_ITEMS(seq);
  PyObject* out = PyList_New(m);
  if (!out) {
    Py_DECREF(seq);
    return nullptr;
  }
  for (Py_ssize_t k = 0; k < m; ++k) {
    const Py_ssize_t r = PyNumber_AsSsize_t(src[k], PyExc_IndexError);
    if (r == -1 && PyErr_Occurred()) {
      Py_DECREF(out);
      Py_DECREF(seq);
      return nullptr;
    }
    PyObject* o;
    if (r < 0) {
      o = Py_None;
    } else if (r >= self->n) {
      PyErr_SetString(PyExc_IndexError, "StrColumn.take row out of range");
      Py_DECREF(out);
      Py_DECREF(seq);
      return nullptr;
    } else {
      o = self->items[r];
    }
    Py_INCREF(o);
    PyList_SET_ITEM(out, k, o);
  }
  Py_DECREF(seq);
  return out;
}

PyObject* sc_reduce(StrCol* self, PyObject*) {
  PyObject* l = sc_tolist(self, nullptr);
  if (!l) return nullptr;
  return Py_BuildValue("(O(N))", reinterpret_cast<PyObject*>(Py_TYPE(self)), l);
}

PyMethodDef sc_methods[] = {
    {"append", reinterpret_cast<PyCFunction>(sc_append), METH_O, "append one string"},
    {"extend", reinterpret_cast<PyCFunction>(sc_extend), METH_O, "append the strings of an iterable"},
    {"take", reinterpret_cast<PyCFunction>(sc_take), METH_O, "[self[r] for r in rows], None for r < 0"},
    {"tolist", reinterpret_cast<PyCFunction>(sc_tolist), METH_NOARGS, "a list copy"},
    {"__reduce__", reinterpret_cast<PyCFunction>(sc_reduce), METH_NOARGS, nullptr},
    {nullptr, nullptr, 0, nullptr}};

PyType_Slot sc_slots[] = {
    {Py_tp_dealloc, reinterpret_cast<void*>(sc_dealloc)},
    {Py_tp_init, reinterpret_cast<void*>(sc_init)},
    {Py_tp_new, reinterpret_cast<void*>(PyType_GenericNew)},
    {Py_tp_iter, reinterpret_cast<void*>(sc_iter)},
    {Py_tp_methods, sc_methods},
    {Py_sq_length, reinterpret_cast<void*>(sc_len)},
    {Py_sq_item, reinterpret_cast<void*>(sc_item)},
    {Py_sq_ass_item, reinterpret_cast<void*>(sc_ass_item)},
    {Py_mp_length, reinterpret_cast<void*>(sc_len)},
    {Py_mp_subscript, reinterpret_cast<void*>(sc_subscript)},
    {Py_mp_ass_subscript, reinterpret_cast<void*>(sc_ass_subscript)},
    {Py_tp_doc, const_cast<char*>("Per-row host strings of a tenant, outside the cyclic collector")},
    {0, nullptr}};

PyType_Spec sc_spec = {"lazzaro_amd._lib._lzrt.StrColumn", sizeof(StrCol), 0, Py_TPFLAGS_DEFAULT, sc_slots};

}  // namespace

namespace lzrt {
// Adds StrColumn to module `m` (called from the pybind11 module init).
int add_strcol(PyObject* m) {
  PyObject* t = PyType_FromSpec(&sc_spec);
  if (!t) return -1;
  if (PyModule_AddObject(m, "StrColumn", t) < 0) {
    Py_DECREF(t);
    return -1;
  }
  return 0;
}
}  // namespace lzrt
