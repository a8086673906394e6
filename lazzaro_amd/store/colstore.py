"""Python face of the native versioned columnar store (``csrc/runtime/colstore.*``).

Table layout mirrors the reference's LanceDB database
(``{db_dir}/lancedb/{nodes,edges,profiles}``, reference vector_store.py:16-85):
same table names, column names and logical types. Each
table is a ``<name>.lance/`` directory holding versioned manifests, immutable
fragments and deletion files written by the C++ runtime. Fragments and
deletion files are Arrow IPC files (``data/*.arrow``, ``_deletions/*.arrow``)
that pyarrow reads directly (:func:`read_fragments`); ``to_arrow`` gives the
table's live rows as one ``pyarrow.Table`` for moving into a real LanceDB
(``lance.write_dataset``) on a networked machine. The byte format of the
Lance v2 file itself is not reproduced.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..utils.faults import fault_point

STR, F64, F32, I32, BOOL, VEC, I64 = 0, 1, 2, 3, 4, 5, 6


def _rt():
    try:
        from .._lib import _lzrt  # type: ignore
        return _lzrt
    except ImportError:
        from .. import _build
        _build.build_runtime(verbose=True)
        from .._lib import _lzrt  # type: ignore
        return _lzrt


NODE_SCHEMA: List[Tuple[str, int, int]] = [
    ("id", STR, 0), ("user_id", STR, 0), ("content", STR, 0), ("vector", VEC, 0),
    ("type", STR, 0), ("timestamp", F64, 0), ("access_count", I32, 0),
    ("last_accessed", F64, 0), ("salience", F32, 0), ("is_super_node", BOOL, 0),
    ("child_ids", STR, 0), ("parent_id", STR, 0), ("shard_key", STR, 0), ("metadata", STR, 0),
    ("decay_clock", F64, 0),
]
EDGE_SCHEMA: List[Tuple[str, int, int]] = [
    ("id", STR, 0), ("user_id", STR, 0), ("source_id", STR, 0), ("target_id", STR, 0),
    ("weight", F32, 0), ("edge_type", STR, 0), ("co_occurrence", I32, 0),
    ("last_updated", F64, 0), ("metadata", STR, 0), ("decay_clock", F64, 0),
]
PROFILE_SCHEMA: List[Tuple[str, int, int]] = [
    ("user_id", STR, 0), ("data", STR, 0), ("updated_at", F64, 0),
]

_NP = {F64: np.float64, F32: np.float32, I32: np.int32, BOOL: np.uint8, I64: np.int64}


# key columns of the reference's tables: a row is identified by (user_id, id)
# (nodes, edges) or user_id (profiles); keyed upserts / deletes are O(rows
# changed) through the runtime's in-memory key index
KEYS = {"nodes": ["user_id", "id"], "edges": ["user_id", "id"], "profiles": ["user_id"]}


class ColumnarTable:
    def __init__(self, root: str, name: str, schema: List[Tuple[str, int, int]], dim: int = 0,
                 key_cols: Optional[Sequence[str]] = None):
        self.name = name
        self.path = os.path.join(root, name + ".lance")
        sch = [(n, t, (dim if t == VEC else d)) for n, t, d in schema]
        self.schema = sch
        keys = list(key_cols) if key_cols is not None else KEYS.get(name, [])
        self._t = _rt().Table(self.path, sch, keys)

    @property
    def version(self) -> int:
        return int(self._t.latest_version())

    def _columns(self, rows: Sequence[Dict]) -> Dict:
        cols = {}
        for n, t, d in self.schema:
            dflt = 0.0 if t in (F64, F32) else (0 if t in (I32, I64, BOOL) else ("{}" if n == "metadata" else ""))
            vals = [r.get(n, dflt) for r in rows]
            if t == STR:
                cols[n] = [("" if v is None else str(v)) for v in vals]
            elif t == VEC:
                cols[n] = (np.asarray(vals, dtype=np.float32).reshape(len(rows), -1) if rows
                           else np.zeros((0, d or 0), dtype=np.float32))
            else:
                cols[n] = np.asarray(vals, dtype=_NP[t])
        return cols

    def add_rows(self, rows: Sequence[Dict]) -> int:
        if not rows:
            return self.version
        fault_point("store.commit")
        return int(self._t.append(self._columns(rows)))

    def stage_rows(self, rows: Sequence[Dict]):
        """Write rows as an unpublished fragment -> (file, rows, vector dim)."""
        fault_point("store.commit")
        f, n, d = self._t.stage(self._columns(rows))
        return str(f), int(n), int(d)

    def commit_staged(self, staged: Sequence[Tuple[str, int, int]]) -> int:
        """Publish staged fragments (from any number of writers) in one version."""
        fault_point("store.commit")
        dims = {int(d) for _, n, d in staged if n}
        if len(dims) > 1:
            raise ValueError("staged fragments with different vector dims")
        return int(self._t.commit_staged([(f, int(n)) for f, n, _ in staged], dims.pop() if dims else 0))

    def replace_rows(self, eq: Sequence[Tuple[str, str]], rows: Sequence[Dict]) -> Tuple[int, int]:
        """Atomically delete the rows matching ``eq`` and append ``rows`` (one
        committed version). Returns (rows deleted, new version)."""
        fault_point("store.commit")
        n, v = self._t.replace_where(list(eq), "", None, self._columns(rows))
        return int(n), int(v)

    def fill_columns(self, cols: Dict, n: int, const: Dict) -> Dict:
        """Complete a column dict for ``n`` rows: ``const`` gives values for
        columns held constant (e.g. user_id), missing ones get defaults."""
        out = {}
        for name, t, d in self.schema:
            if name in const:
                v = const[name]
                out[name] = [v] * n if t == STR else np.full(n, v, dtype=_NP[t])
            elif name in cols:
                out[name] = cols[name]
            elif t == STR:
                out[name] = ["{}" if name == "metadata" else ""] * n
            elif t == VEC:
                out[name] = np.zeros((n, d or 0), dtype=np.float32)
            else:
                out[name] = np.zeros(n, dtype=_NP[t])
        return out

    def upsert_columns(self, eq: Sequence[Tuple[str, str]], key: str, keys: Sequence[str], cols: Dict
                       ) -> Tuple[int, int]:
        """One committed version that deletes the rows matching ``eq`` whose
        ``key`` is in ``keys`` and appends ``cols`` (upsert + delete)."""
        fault_point("store.commit")
        fault_point("store.commit." + self.name)
        n, v = self._t.replace_where(list(eq), key, list(keys), cols)
        return int(n), int(v)

    def add_columns(self, cols: Dict) -> int:
        fault_point("store.commit")
        fault_point("store.commit." + self.name)
        return int(self._t.append(cols))

    def delete(self, eq: Sequence[Tuple[str, str]], in_col: str = "", in_vals=None) -> Tuple[int, int]:
        fault_point("store.commit")
        n, v = self._t.delete_where(list(eq), in_col, None if in_vals is None else list(in_vals))
        return int(n), int(v)

    def scan_columns(self, eq: Sequence[Tuple[str, str]] = (), in_col: str = "", in_vals=None,
                     want: Optional[Sequence[str]] = None, vec_pieces: bool = False) -> Dict:
        """Matching rows' columns. ``vec_pieces``: the vector column comes back
        as a list of [rows, dim] float32 arrays in row order -- zero-copy
        views of the memory-mapped fragments where a fragment is wholly
        selected -- instead of one array copied out of them (a tenant load
        streams those pieces to the device)."""
        return self._t.scan(list(eq), in_col, None if in_vals is None else list(in_vals), list(want or []),
                            bool(vec_pieces))

    def scan(self, eq: Sequence[Tuple[str, str]] = (), in_col: str = "", in_vals=None,
             want: Optional[Sequence[str]] = None) -> List[Dict]:
        cols = self.scan_columns(eq, in_col, in_vals, want)
        if not cols:
            return []
        names = list(cols.keys())
        n = len(cols[names[0]])
        out = []
        conv = {}
        for k in names:
            c = cols[k]
            t = next(tt for nn, tt, _ in self.schema if nn == k)
            if t == VEC:
                conv[k] = [row.tolist() for row in c]
            elif t == BOOL:
                conv[k] = [bool(x) for x in c]
            elif t in (I32, I64):
                conv[k] = [int(x) for x in c]
            elif t in (F32, F64):
                conv[k] = [float(x) for x in c]
            else:
                conv[k] = c
        for i in range(n):
            out.append({k: conv[k][i] for k in names})
        return out

    def fragment_files(self) -> List[str]:
        """Arrow IPC files of the fragments and deletion files on disk."""
        out = []
        for sub in ("data", "_deletions"):
            d = os.path.join(self.path, sub)
            out += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".arrow"))
        return out

    def count(self) -> int:
        return int(self._t.count_rows())

    def compact(self) -> int:
        return int(self._t.compact())

    # ---- Arrow interchange --------------------------------------------------
    def to_arrow(self):
        import pyarrow as pa

        cols = self.scan_columns()
        arrays, fields = [], []
        for n, t, _ in self.schema:
            c = cols[n]
            if t == VEC:
                dim = c.shape[1] if c.ndim == 2 else 0
                flat = pa.array(c.reshape(-1), type=pa.float32())
                arrays.append(pa.FixedSizeListArray.from_arrays(flat, dim))
                fields.append(pa.field(n, pa.list_(pa.float32(), dim)))
            elif t == STR:
                arrays.append(pa.array(c, type=pa.string()))
                fields.append(pa.field(n, pa.string()))
            elif t == BOOL:
                arrays.append(pa.array(c.astype(bool)))
                fields.append(pa.field(n, pa.bool_()))
            else:
                typ = {F64: pa.float64(), F32: pa.float32(), I32: pa.int32(), I64: pa.int64()}[t]
                arrays.append(pa.array(c, type=typ))
                fields.append(pa.field(n, typ))
        return pa.Table.from_arrays(arrays, schema=pa.schema(fields))

    def from_arrow(self, table) -> int:
        cols = {}
        for n, t, _ in self.schema:
            col = table.column(n)
            if t == VEC:
                cols[n] = np.asarray(col.to_pylist(), dtype=np.float32)
            elif t == STR:
                cols[n] = [("" if v is None else v) for v in col.to_pylist()]
            else:
                cols[n] = np.asarray(col.to_pylist(), dtype=_NP[t])
        return self.add_columns(cols)


def read_fragments(table_dir: str):
    """The live rows of a table directory read with pyarrow alone (no
    ``_lzrt``): the newest manifest's fragments minus their deletion files."""
    import pyarrow as pa
    import pyarrow.ipc as ipc

    with open(os.path.join(table_dir, "_latest")) as f:
        v = int(f.read().strip())
    frags = []
    with open(os.path.join(table_dir, "_versions", "%020d.manifest" % v)) as f:
        for line in f:
            p = line.split()
            if p and p[0] == "frag":
                frags.append((p[1], None if p[3] == "-" else p[3]))
    parts = []
    for fn, dl in frags:
        t = ipc.open_file(os.path.join(table_dir, "data", fn)).read_all()
        if dl:
            dead = ipc.open_file(os.path.join(table_dir, "_deletions", dl)).read_all().column("row").to_numpy()
            keep = np.ones(t.num_rows, dtype=bool)
            keep[dead] = False
            t = t.filter(pa.array(keep))
        parts.append(t)
    return pa.concat_tables(parts) if parts else None
