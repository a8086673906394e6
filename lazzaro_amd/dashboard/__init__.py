"""FastAPI dashboard (same routes as the reference, offline-capable page)."""
