"""Columnar search routing (lazzaro_amd/parallel/routing.py) on CPU with gloo:
``search_routed`` (queries embedded by the front end, routed to the tenants'
owners in one all-to-all, (score, row) hits back in one more), ``resolve``
and ``search_global_batch`` (all-gather of queries + one all-to-all of
candidates back to their origin) against single-process truth."""
import functools
import json

import numpy as np
import pytest
import torch

from tests.distributed.test_dist_gloo import spawn

USERS = [f"tenant{i}" for i in range(9)]
D = 32


def _rows(user):
    rng = np.random.default_rng(int(user[6:]) + 11)
    n = 30 + 17 * int(user[6:])
    return n, rng.standard_normal((n, D)).astype(np.float32)


def _factory(db, user, load_from_disk=False):
    from lazzaro_amd.core.memory_system import MemorySystem
    from lazzaro_amd.core.providers import HashEmbedder, LocalLLM
    return MemorySystem(llm_provider=LocalLLM(), embedding_provider=HashEmbedder(dim=D), enable_async=False,
                        db_dir=db, user_id=user, device="cpu", load_from_disk=load_from_disk, max_buffer_size=10 ** 6)


def _fill(ms, user):
    n, V = _rows(user)
    g = ms.graph
    g.add_nodes([f"{user}_m{i}" for i in range(n)], [f"memory {i} of {user}" for i in range(n)],
                torch.from_numpy(V), shard=g.shard_id("work"), stored=True)


def _queries(rank, n=13):
    return [f"rank {rank} question {q} about memories" for q in range(n)]


def _workload(comm, db, force=False, device_dir=False):
    from lazzaro_amd.core.providers import HashEmbedder
    from lazzaro_amd.parallel import routing
    from lazzaro_amd.parallel.service import DistributedMemoryService
    svc = DistributedMemoryService(comm, functools.partial(_factory, db), embedder=HashEmbedder(dim=D),
                                   force_collectives=force)
    if device_dir:  # every owned tenant counts as "large": owners match tenant keys on the device
        routing.BIG_ROWS = 1
        svc.DEVICE_ROUTE_MAX_TENANTS = len(USERS)
    for u in USERS:
        if svc.is_local(u):
            _fill(svc.system(u), u)
    rng = np.random.default_rng(comm.rank)
    qs = _queries(comm.rank)
    users = [USERS[int(rng.integers(len(USERS)))] for _ in qs]
    limits = [int(x) for x in rng.integers(1, 6, len(qs))]
    hits = svc.search_routed(users, qs, limits)
    nodes = svc.resolve(hits)
    again = svc.search_routed(users, qs, limits)  # names already announced: tensor-only round
    same = bool(torch.equal(again.rows, hits.rows))
    third = svc.search_routed(users, qs, limits)  # every owner knows its senders' view of its directory
    same = same and bool(torch.equal(third.rows, hits.rows)) and bool(torch.equal(third.scores, hits.scores))
    stats3 = dict(svc.route_stats)  # (the three calls above)
    # the pipelined form (search_routed_stream): the same hits, batch by batch
    streamed = list(svc.search_routed_stream([(users, qs), (users[:5], qs[:5]), (users, qs)], limits[0]))
    ref5 = svc.search_routed(users[:5], qs[:5], limits[0])
    refa = svc.search_routed(users, qs, limits[0])
    same = same and len(streamed) == 3 and bool(torch.equal(streamed[1].rows, ref5.rows)) \
        and bool(torch.equal(streamed[0].rows, refa.rows)) and bool(torch.equal(streamed[2].scores, refa.scores))
    glob = svc.search_global_batch(qs[:5], limit=4)
    rk, slot, row = glob.split()
    svc.get_all_users()  # names every tenant key
    gusers = glob.users(svc)
    table = svc.tenant_table()
    names = {int(s): n for n, s in table.slot.items()}
    svc.close()
    return json.dumps({"users": users, "limits": limits, "ids": [[n["id"] for n in r] for r in nodes],
                       "scores": hits.scores.tolist(), "same": same,
                       "global": [[[int(a), int(b), int(c)] for a, b, c in zip(x, y, z)]
                                  for x, y, z in zip(rk.tolist(), slot.tolist(), row.tolist())],
                       "gscores": glob.scores.tolist(), "names": names, "rank": comm.rank,
                       "route_stats": stats3, "force": svc.force_collectives, "gusers": gusers})


def _truth(qs, users, limits):
    from lazzaro_amd.core.providers import HashEmbedder
    E = np.asarray(HashEmbedder(dim=D).batch_embed(qs), np.float32)
    out = []
    for q, (u, k) in enumerate(zip(users, limits)):
        n, V = _rows(u)
        d = ((E[q][None, :] - V) ** 2).sum(1)
        out.append([f"{u}_m{i}" for i in np.argsort(d, kind="stable")[:k]])
    return out


def _global_truth(qs, k):
    from lazzaro_amd.core.providers import HashEmbedder
    E = np.asarray(HashEmbedder(dim=D).batch_embed(qs), np.float32)
    res = []
    for q in range(len(qs)):
        c = []
        for u in USERS:
            n, V = _rows(u)
            d = ((E[q][None, :] - V) ** 2).sum(1)
            c += [(float(d[i]), u, i) for i in range(n)]
        c.sort()
        res.append([(u, i) for _, u, i in c[:k]])
    return res


@pytest.mark.parametrize("world", [1, 2, 4])
def test_routed_and_global_search(world, tmp_path):
    fn = functools.partial(_workload, db=str(tmp_path / f"r{world}"))
    if world == 1:
        from lazzaro_amd.parallel import Communicator
        outs = {0: fn(Communicator.local())}
    else:
        outs = spawn(world, fn)
    d = {r: json.loads(v) for r, v in outs.items()}
    names = {r: {int(s): n for s, n in x["names"].items()} for r, x in d.items()}
    for r, x in d.items():
        qs = _queries(r)
        assert x["same"]
        assert x["ids"] == _truth(qs, x["users"], x["limits"]), r
        # scores are exact -|q - x|^2, sorted, -inf past each limit
        for sc, k in zip(x["scores"], x["limits"]):
            assert all(s > float("-inf") for s in sc[:k]) and sc[:k] == sorted(sc[:k], reverse=True)
        got = [[(names[rk][sl], row) for rk, sl, row in qq] for qq in x["global"]]
        assert got == _global_truth(qs[:5], 4), r
        assert [[u for u, _ in qq] for qq in got] == x["gusers"]


@pytest.mark.parametrize("world,device_dir", [(1, False), (1, True), (2, True), (3, True)])
def test_routed_forced_collectives_and_device_directory(world, device_dir, tmp_path):
    """A 1-rank process group with ``force_collectives`` runs every exchange
    of the N-rank job (the form ``bench.py`` uses under a 1-rank
    torch.distributed.run on one GPU); with the device directory the owners
    serve the steady-state rounds by matching tenant keys on the device (no
    read-back of the received rows) -- results identical to the truth."""
    fn = functools.partial(_workload, db=str(tmp_path / f"f{world}{device_dir}"), force=True, device_dir=device_dir)
    outs = spawn(world, fn)
    d = {r: json.loads(v) for r, v in outs.items()}
    names = {r: {int(s): n for s, n in x["names"].items()} for r, x in d.items()}
    for r, x in d.items():
        qs = _queries(r)
        assert x["force"] is True
        assert x["same"]
        assert x["ids"] == _truth(qs, x["users"], x["limits"]), r
        got = [[(names[rk][sl], row) for rk, sl, row in qq] for qq in x["global"]]
        assert got == _global_truth(qs[:5], 4), r
        st = x["route_stats"]
        assert st["device"] + st["host"] == 3
        if device_dir:
            assert st["device"] >= 1, st  # the third round at the latest
        else:
            assert st["device"] == 0
