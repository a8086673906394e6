"""Device-resident memory engine under ``MemorySystem``.

:class:`TenantGraph` holds one tenant's memory graph as HBM columns and runs
every graph step as a HIP kernel / batched tensor op; :mod:`.views` exposes it
through the reference's ``Node``/``Edge``/``MemoryShard``/``BufferGraph``
shapes.
"""
from .tenant_graph import FREE, GHOST, NODE, TenantGraph  # noqa: F401
