"""Elastic recovery on CPU (gloo, 3 ranks): rank 2 dies after persisting its
tenants; the survivors detect it by heartbeat, re-form a 2-rank group, re-place
only the dead rank's tenants (rendezvous hashing over the surviving ids) and
serve them from the shared columnar store."""
import os
import socket
import tempfile
import time

import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LZK_DEVICE="cpu")
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from lazzaro_amd.core.vector_store import HBMStore
        from lazzaro_amd.parallel import Communicator
        from lazzaro_amd.parallel.elastic import ElasticPlacement, Heartbeat, detect_failed, reform_group

        hb = Heartbeat(dist.FileStore(os.path.join(tmp, "hb"), world), rank, world, interval=0.1).start()
        tenants = [f"user{i}" for i in range(30)]
        place = ElasticPlacement(world)
        store = HBMStore(db_dir=os.path.join(tmp, "db"), device="cpu")
        mine = [t for t in tenants if place.owner(t) == rank]
        for t in mine:
            v = [0.0] * 8
            v[hash(t) % 8] = 1.0
            store.add_nodes([{"id": f"{t}_n0", "content": f"fact of {t}", "embedding": v}], user_id=t)
        Communicator().barrier()
        if rank == 2:
            hb.stop()
            q.put((rank, sorted(mine)))
            q.close()
            q.join_thread()  # flush the result before the simulated crash
            os._exit(0)  # simulated crash: no group teardown
        # let rank 2's last beat land before the window opens, and give the
        # survivors' heartbeat threads slack on a loaded host
        time.sleep(0.5)
        dead = detect_failed(hb, window=2.0)
        survivors = [r for r in range(world) if r not in dead]
        reform_group(lambda g, n: dist.FileStore(os.path.join(tmp, f"pg_gen{g}"), n), survivors, rank)
        comm = Communicator()
        after = place.remove(dead)
        now_mine = [t for t in tenants if after.owner(t) == rank]
        moved_in = [t for t in now_mine if place.owner(t) != rank]
        ok = True
        for t in moved_in:  # reload from the shared store
            v = [0.0] * 8
            v[hash(t) % 8] = 1.0
            ok = ok and store.search_nodes(v, user_id=t, limit=1) == [f"{t}_n0"]
        owned = comm.all_gather_object(sorted(now_mine))
        hb.stop()
        q.put((rank, {"dead": dead, "new_rank": comm.rank, "world": comm.world, "moved_in": moved_in,
                      "reload_ok": ok, "union": sorted(t for part in owned for t in part),
                      "kept": all(after.owner(t) == place.owner(t) for t in tenants if place.owner(t) != 2)}))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


def test_rank_failure_detect_reform_replace():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    with tempfile.TemporaryDirectory() as tmp:
        ps = [ctx.Process(target=_worker, args=(r, 3, port, tmp, q)) for r in range(3)]
        for p in ps:
            p.start()
        out = dict(q.get(timeout=180) for _ in range(3))
        for p in ps:
            p.join(timeout=60)
    for r, v in out.items():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    dead_tenants = out[2]
    for r in (0, 1):
        o = out[r]
        assert o["dead"] == [2] and o["world"] == 2 and o["new_rank"] == r and o["reload_ok"] and o["kept"]
        assert o["union"] == sorted(f"user{i}" for i in range(30))
    assert sorted(out[0]["moved_in"] + out[1]["moved_in"]) == dead_tenants


def _svc_factory(db, user):
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    return MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=32), enable_async=False,
                        db_dir=db, user_id=user, device="cpu", max_buffer_size=50)


def _svc_worker(rank, world, port, tmp, q):
    """DistributedMemoryService through a failure: tenants converse on their
    owners, rank 2 dies, the survivors re-form, the service re-places the dead
    rank's tenants and serves their searches from the shared store."""
    import functools
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LZK_DEVICE="cpu")
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from lazzaro_amd.parallel import Communicator
        from lazzaro_amd.parallel.elastic import ElasticPlacement, Heartbeat, detect_failed, reform_group
        from lazzaro_amd.parallel.service import DistributedMemoryService
        hb = Heartbeat(dist.FileStore(os.path.join(tmp, "hb"), world), rank, world, interval=0.1).start()
        place = ElasticPlacement(world)
        svc = DistributedMemoryService(Communicator(), functools.partial(_svc_factory, os.path.join(tmp, "db")),
                                       placement=place)
        tenants = [f"user{i}" for i in range(9)]
        mine = [t for t in tenants if svc.is_local(t)]
        for step in (("start_conversation",), ("chat", "My hobby is sailing and my sister lives in Porto."),
                     ("chat", "I am preparing a robotics demo for Friday."), ("end_conversation",)):
            svc.serve([(t,) + step for t in mine])
        before = {t: r for t, r in zip(mine, svc.serve([(t, "search_memories", "sailing hobby", 3) for t in mine]))}
        Communicator().barrier()
        if rank == 2:
            hb.stop()
            q.put((rank, {"mine": sorted(mine), "before": before}))
            q.close()
            q.join_thread()
            os._exit(0)
        # let rank 2's last beat land before the window opens, and give the
        # survivors' heartbeat threads slack on a loaded host
        time.sleep(0.5)
        dead = detect_failed(hb, window=2.0)
        survivors = [r for r in range(world) if r not in dead]
        reform_group(lambda g, n: dist.FileStore(os.path.join(tmp, f"svc_gen{g}"), n), survivors, rank)
        released = svc.reform(Communicator(), place.remove(dead))
        # every survivor asks for every tenant: remote ones route to the new owners
        reqs = [(t, "search_memories", "sailing hobby", 3) for t in tenants] if rank == 0 else []
        out = svc.serve(reqs)
        res = dict(zip(tenants, out)) if rank == 0 else {}
        resident = sorted(svc.systems)
        allres = svc.comm.all_gather_object(resident)
        hb.stop()
        svc.close()
        q.put((rank, {"before": before, "after": res, "released": released, "resident": allres}))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))


def test_service_survives_rank_failure():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    with tempfile.TemporaryDirectory() as tmp:
        ps = [ctx.Process(target=_svc_worker, args=(r, 3, port, tmp, q)) for r in range(3)]
        for p in ps:
            p.start()
        out = dict(q.get(timeout=240) for _ in range(3))
        for p in ps:
            p.join(timeout=60)
    for r, v in out.items():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    before = {**out[0]["before"], **out[1]["before"], **out[2]["before"]}
    after = out[0]["after"]
    assert sorted(after) == sorted(before) and len(after) == 9
    for t in after:  # the dead rank's tenants answer from the store exactly as before the failure
        assert [n["id"] for n in after[t]] == [n["id"] for n in before[t]], t
        assert after[t], t
    resident = sorted(u for part in out[0]["resident"] for u in part)
    assert resident == sorted(after)  # every tenant now resident on exactly one survivor
    assert set(out[2]["mine"]) <= set(resident)
    assert out[0]["released"] == [] and out[1]["released"] == []  # survivors keep their own tenants
