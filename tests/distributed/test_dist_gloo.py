"""Multi-process tests of the distributed layer on CPU (gloo, world 2 and 4):
placement, cross-shard search merge (C1), all-to-all re-shard (C3),
distributed k-means (C4) and distributed components (C5)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LZK_DEVICE="cpu")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lazzaro_amd.parallel import Communicator
        q.put((rank, fn(Communicator())))
    except Exception as e:  # surface worker failures in the parent
        import traceback
        q.put((rank, "ERR " + traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def spawn(world, fn):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_run, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r, v in out.items():
        assert not (isinstance(v, str) and v.startswith("ERR")), v
    return out


def _sharded_search(comm):
    from lazzaro_amd.ops.search import _ref_topk
    from lazzaro_amd.parallel import ShardedIndex
    g = torch.Generator().manual_seed(0)
    X = torch.randn(1003, 32, generator=g)
    Q = torch.randn(9, 32, generator=g)
    idx = ShardedIndex.partition(comm, X)
    s, i = idx.search(Q, 7)
    rs, ri = _ref_topk(X, Q, 7)
    return bool(torch.allclose(s, rs, atol=1e-5) and torch.equal(i, ri))


def _reshard(comm):
    n = 50 + comm.rank * 7
    ids = torch.arange(n) + 1000 * comm.rank
    dest = ids % comm.world
    vec = ids.float()[:, None].repeat(1, 3)
    rid, rvec = comm.reshard(dest, ids, vec)
    ok = bool((rid % comm.world == comm.rank).all()) and torch.equal(rvec[:, 0], rid.float())
    tot = torch.tensor([rid.numel()])
    comm.all_reduce(tot)
    expect = sum(50 + r * 7 for r in range(comm.world))
    return ok and int(tot) == expect


def _placement(comm):
    from lazzaro_amd.parallel import TenantDirectory, tenant_rank
    d = TenantDirectory(comm)
    users = [f"user_{i}" for i in range(200)]
    for u in users:
        if d.is_local(u):
            d.register(u, 1)
    allu = d.all_tenants()
    owners = [tenant_rank(u, comm.world) for u in users]
    return allu == sorted(users) and len(set(owners)) == comm.world


def _kmeans(comm):
    from lazzaro_amd.index.kmeans import kmeans
    torch.manual_seed(5)
    centers = torch.nn.functional.normalize(torch.randn(4, 16), dim=1)
    g = torch.Generator().manual_seed(10 + comm.rank)
    X = torch.cat([torch.nn.functional.normalize(c + 0.05 * torch.randn(50, 16, generator=g), dim=1)
                   for c in centers])
    c32, _, lab = kmeans(X, 4, iters=6, comm=comm)
    allc = comm.all_gather_rows(c32.contiguous())
    same = torch.allclose(allc[:4], allc[-4:], atol=1e-6)
    pure = all(len(set(lab[j * 50:(j + 1) * 50].tolist())) == 1 for j in range(4))
    return bool(same and pure)


def _full_labels(comm, n, verts, lab):
    full = torch.arange(n, dtype=torch.int64)
    for v, l in comm.all_gather_object((verts.tolist(), lab.tolist())):
        full[torch.tensor(v, dtype=torch.long)] = torch.tensor(l, dtype=torch.int64)
    return full


def _components(comm):
    from lazzaro_amd.ops import graph_ops as G
    from lazzaro_amd.parallel import distributed_components
    n = 300
    g = torch.Generator().manual_seed(3)
    src = torch.randint(0, n, (240,), generator=g, dtype=torch.int32)
    dst = torch.randint(0, n, (240,), generator=g, dtype=torch.int32)
    ref = G.connected_components(src, dst, n).to(torch.int64)
    mine = torch.arange(240) % comm.world == comm.rank
    verts, lab = distributed_components(comm, src[mine], dst[mine], n)
    return bool(torch.equal(_full_labels(comm, n, verts, lab), ref))


def _components_local(comm):
    """Each rank's edges stay in its own id block except a chain of bridges:
    after the subscription round only the bridge vertices travel, and the
    labels are the single-process ones."""
    from lazzaro_amd.ops import graph_ops as G
    from lazzaro_amd.parallel import distributed_components
    W, per = comm.world, 5000
    n = W * per
    g = torch.Generator().manual_seed(7)
    srcs, dsts = [], []
    for r in range(W):  # a long path inside each block (deep local structure) + random chords
        base = r * per
        p = torch.arange(base, base + per - 1)
        srcs += [p, base + torch.randint(0, per, (2000,), generator=g)]
        dsts += [p + 1, base + torch.randint(0, per, (2000,), generator=g)]
    src, dst = torch.cat(srcs), torch.cat(dsts)
    owner = src // per
    # bridges: the last vertex of block r to the first of block r+1, held by rank r
    bs = torch.arange(W - 1) * per + per - 1
    src, dst, owner = torch.cat([src, bs]), torch.cat([dst, bs + 1]), torch.cat([owner, torch.arange(W - 1)])
    ref = G.connected_components(src.int(), dst.int(), n).to(torch.int64)
    mine = owner == comm.rank
    st = {}
    verts, lab = distributed_components(comm, src[mine].int(), dst[mine].int(), n, stats=st)
    ok = bool(torch.equal(_full_labels(comm, n, verts, lab), ref)) and bool((ref == 0).all())
    # after subscription, traffic is per boundary vertex, not per vertex
    return ok and st["rows_sent"] <= 2 * W and st["rounds"] <= W + 1


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_components(world):
    assert all(spawn(world, _components).values())


@pytest.mark.parametrize("world", [2, 8])
def test_distributed_components_boundary_traffic(world):
    assert all(spawn(world, _components_local).values())


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_search(world):
    assert all(spawn(world, _sharded_search).values())


@pytest.mark.parametrize("world", [2, 3])
def test_all_to_all_reshard(world):
    assert all(spawn(world, _reshard).values())


def test_tenant_placement():
    assert all(spawn(2, _placement).values())


def test_distributed_kmeans():
    assert all(spawn(2, _kmeans).values())


def _commit(comm):
    import os
    import tempfile

    from lazzaro_amd.parallel.commit import distributed_commit
    from lazzaro_amd.store.colstore import NODE_SCHEMA, ColumnarTable
    root = os.environ["LZK_TEST_ROOT"]
    t = ColumnarTable(root, "nodes", NODE_SCHEMA)
    comm.barrier()
    v0 = t.version
    comm.barrier()
    rows = [dict(id=f"r{comm.rank}_{i}", user_id=f"u{comm.rank}", content="c", vector=[float(comm.rank)] * 4,
                 type="semantic", timestamp=0.0, access_count=0, last_accessed=0.0, salience=0.5,
                 is_super_node=False, child_ids="[]", parent_id="", shard_key="default", metadata="{}")
            for i in range(comm.rank + 2)]
    v = distributed_commit(comm, t, rows)
    return (v0, v, t.count(), sorted({r["user_id"] for r in t.scan()}))


def test_distributed_commit_is_one_version(tmp_path, monkeypatch):
    monkeypatch.setenv("LZK_TEST_ROOT", str(tmp_path))
    out = spawn(3, _commit)
    v0 = {o[0] for o in out.values()}
    vs = {o[1] for o in out.values()}
    assert len(vs) == 1 and vs.pop() == v0.pop() + 1
    for o in out.values():
        assert o[2] == 2 + 3 + 4 and o[3] == ["u0", "u1", "u2"]


def _eight_rank_pipeline(comm):
    """The 8-GPU node's collective pattern on 8 CPU ranks: tenant placement,
    all-to-all re-shard, cross-shard search merge and a multi-rank commit."""
    from lazzaro_amd.ops.search import _ref_topk
    from lazzaro_amd.parallel import ShardedIndex
    from lazzaro_amd.parallel.placement import TenantDirectory
    assert comm.world == 8
    g = torch.Generator().manual_seed(11)
    X = torch.randn(4001, 32, generator=g)
    Q = torch.randn(13, 32, generator=g)
    idx = ShardedIndex.partition(comm, X)
    s, i = idx.search(Q, 5)
    rs, ri = _ref_topk(X, Q, 5)
    ok = bool(torch.allclose(s, rs, atol=1e-5) and torch.equal(i, ri))
    # re-shard 100 rows per rank to pseudo-random owners
    rows = torch.arange(100) + 1000 * comm.rank
    dest = (rows * 7919) % comm.world
    (got,) = comm.reshard(dest, rows.float())
    ok = ok and bool(((got.long() * 7919) % comm.world == comm.rank).all())
    total = comm.all_reduce(torch.tensor([got.numel()], dtype=torch.float64))
    ok = ok and int(total.item()) == 800
    d = TenantDirectory(comm)
    for t in (f"user{i}" for i in range(200)):
        if d.is_local(t):
            d.register(t, 1)
    ok = ok and len(d.all_tenants()) == 200
    return ok


def test_eight_ranks_gloo():
    assert all(spawn(8, _eight_rank_pipeline).values())
