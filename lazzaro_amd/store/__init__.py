"""Persistence: the native versioned columnar store (LanceDB-schema tables)."""
from .colstore import EDGE_SCHEMA, NODE_SCHEMA, PROFILE_SCHEMA, ColumnarTable  # noqa: F401
