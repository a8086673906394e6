"""Legacy (pre-v0.3 reference) API shims so older lazzaro code keeps working.

* :class:`LanceDBVectorStore` -- the old ``add/search/delete`` vector store
  (reference tests/test_vector_store.py), backed by :class:`HBMStore`.
* :class:`PersistenceManager` -- pickle snapshot file with ``.bak`` rotation
  (reference tests/test_persistence.py). Only files this framework wrote are
  ever unpickled.
"""
from .legacy import LanceDBVectorStore, PersistenceManager  # noqa: F401
