"""Web dashboard (reference ``src/lazzaro/dashboard/api.py:12-139``).

Same FastAPI routes and JSON shapes: ``GET /``, ``/api/stats``, ``/api/users``,
``POST /api/users/switch``, ``/api/insights``, ``/api/export``, ``/api/graph``,
``/api/profile``, ``POST /api/consolidate``; served on port 5299. The page is
self-contained (no CDN scripts, renders offline) and polls every 30 s.
Extra: ``GET /api/search?q=&limit=`` (on-device vector search) and
``GET /api/engine`` (device / kernel-library status).
"""
from __future__ import annotations

import os
from typing import Optional

from fastapi import FastAPI, Request
from fastapi.responses import HTMLResponse

app = FastAPI(title="Lazzaro MI355X Memory Dashboard")
_ms = None
_HERE = os.path.dirname(os.path.abspath(__file__))


def set_memory_system(ms) -> None:
    global _ms
    _ms = ms


@app.get("/", response_class=HTMLResponse)
async def get_dashboard(request: Request):
    with open(os.path.join(_HERE, "templates", "index.html"), encoding="utf-8") as f:
        return HTMLResponse(f.read())


@app.get("/api/stats")
async def get_stats():
    if not _ms:
        return {"error": "Memory system not initialized"}
    _ms.check_for_updates()
    s = _ms.get_stats()
    s["user_id"] = _ms.user_id
    return s


@app.get("/api/users")
async def get_users():
    return _ms.get_all_users() if _ms else []


@app.post("/api/users/switch")
async def switch_user(request: Request):
    if not _ms:
        return {"error": "Memory system not initialized"}
    data = await request.json()
    uid = data.get("user_id")
    if not uid:
        return {"error": "User ID required"}
    _ms.switch_user(uid)
    return {"status": "success", "user_id": _ms.user_id}


@app.get("/api/insights")
async def get_insights():
    if not _ms:
        return {"error": "Memory system not initialized"}
    return {"insights": _ms.get_insights()}


@app.get("/api/export")
async def export_observations(format: str = "markdown"):
    if not _ms:
        return {"error": "Memory system not initialized"}
    return {"content": _ms.export_observations(format=format)}


@app.get("/api/graph")
async def get_graph():
    if not _ms:
        return {"nodes": [], "links": []}
    _ms.check_for_updates()
    return _ms.graph_json()


@app.get("/api/profile")
async def get_profile():
    if not _ms:
        return {}
    _ms.check_for_updates()
    with _ms._graph_lock:
        return _ms.profile.to_dict()


@app.post("/api/consolidate")
async def consolidate():
    if not _ms:
        return {"error": "Memory system not initialized"}
    return {"status": _ms.run_consolidation()}


@app.get("/api/search")
async def search(q: str, limit: int = 5):
    if not _ms:
        return []
    return [{"id": n.id, "content": n.content, "salience": n.salience, "shard": n.shard_key}
            for n in _ms.search_memories(q, limit=limit)]


@app.get("/api/engine")
async def engine():
    import torch

    from ..ops import _lib

    dev = str(getattr(_ms, "_device", None)) if _ms else None
    return {"device": dev, "hip_available": torch.cuda.is_available(), "kernel_library": _lib.available(),
            "store": type(_ms.store).__name__ if _ms else None}


def entry_point(host: str = "0.0.0.0", port: int = 5299, ms: Optional[object] = None) -> None:
    import uvicorn

    if ms is None:
        from ..core.memory_system import MemorySystem

        ms = MemorySystem(load_from_disk=True)
    set_memory_system(ms)
    print(f"🚀 Starting Lazzaro MI355X Dashboard on http://localhost:{port}")
    uvicorn.run(app, host=host, port=port)


if __name__ == "__main__":
    entry_point()
