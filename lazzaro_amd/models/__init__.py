"""Models: the memory-graph data model and the on-device sentence encoders."""
from .graph import Edge, Node  # noqa: F401

__all__ = ["Node", "Edge"]
