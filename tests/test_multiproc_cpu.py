"""The N>1 path of bench.py / batch drivers (gsnapdp.shard, gsnapdp.gather) on
CPU: ranks under the gloo backend split ONE batch per read
(shard.balanced_ranges), align their slices with the CPU restatement (the GPU
step's stand-in here), build the payload the GPU path builds (result records +
compact variable-length streams), gather it to rank 0 with the same
shard.gather_to_root call bench.py makes, and rank 0 reassembles the batch.
The reassembled batch must be byte-identical to a single-rank run of the whole
batch; timing uses the same barrier + max-over-ranks code as the benchmark."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from gsnapdp import shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, outdir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import oracle as O
    from gsnapdp import shard as S
    from gsnapdp import workload as W

    r = S.init_from_env("gloo")
    genome = W.synthetic_genome(300_000, seed=1)
    blocks = W.pack_genome(genome)
    batch = W.c2_windows(genome, n=300, seed=S.shard_seed(2, r.rank))
    O.setup(blocks)
    out = {}

    def step():
        res, _, _, _ = O.run_batch(batch.windows, batch.query, batch.query_uc, nthreads=1)
        out["score_sum"] = int(res["finalscore"].astype(np.int64).sum())

    elapsed = S.timed_steps(r, step, 2, lambda: None)
    rate = S.aggregate_rate(len(batch), r, 2, elapsed)
    # every rank must see the same (max) time; shards must differ
    t = torch.tensor([elapsed], dtype=torch.float64)
    ts = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    r.dist.all_gather(ts, t)
    first = torch.tensor([int(batch.windows["chrpos"][0])], dtype=torch.int64)
    firsts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    r.dist.all_gather(firsts, first)
    total = torch.tensor([len(batch)], dtype=torch.int64)
    r.dist.all_reduce(total)
    json.dump({"elapsed": [float(x) for x in ts], "firsts": [int(x) for x in firsts],
               "total": int(total), "rate": rate, "score_sum": out["score_sum"]},
              open(os.path.join(outdir, "rank%d.json" % r.rank), "w"))
    S.finish(r)


def _batch():
    from gsnapdp import workload as W
    g = W.c3_genome(seed=3, scale=0.002)
    return g, W.c3_windows(g, n=1203, seed=33)


def _payload_of(res, pairs, poff, npairs):
    """The payload's variable-length stream on CPU: each window's pair records
    (6 words each) stand in for its op stream, so `nops` = 6 x npairs and the
    capacity offsets are the pair offsets x 6."""
    from gsnapdp import gather as G
    r = res.copy()
    r["nops"] = 6 * npairs
    words = pairs.view(np.uint32)
    comp = G.compact_ops(r, words, 6 * poff)
    return r, comp


def _gather_main(rank, world, port, outdir):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import oracle as O
    from gsnapdp import gather as G
    from gsnapdp import shard as S
    from gsnapdp.records import PAIR

    r = S.init_from_env("gloo")
    g, batch = _batch()
    cells = np.full(len(batch), 4410) + (np.arange(len(batch)) % 7)  # uneven weights
    spans = S.balanced_ranges(cells, world)
    sizes = [b - a for a, b in spans]
    lo, hi = spans[r.rank]
    O.setup(g.blocks)
    res, pairs, poff, npairs = O.run_batch(batch.windows[lo:hi], batch.query, batch.query_uc, nthreads=1)
    rr, comp = _payload_of(res, pairs, poff, npairs)
    lay = G.Layout(max(sizes), 6 * 200 * max(sizes))
    mine = torch.from_numpy(G.pack(lay, rr, comp))
    recv = [torch.zeros(lay.nbytes, dtype=torch.uint8) for _ in range(world)] if r.rank == 0 else None
    S.gather_to_root(r, mine, recv)
    if r.rank == 0:
        allres, allops, alloff = G.reassemble(lay, [t.numpy() for t in recv], sizes)
        np.save(os.path.join(outdir, "res.npy"), allres)
        np.save(os.path.join(outdir, "ops.npy"), allops)
        np.save(os.path.join(outdir, "off.npy"), alloff)
        json.dump({"spans": spans}, open(os.path.join(outdir, "spans.json"), "w"))
    S.finish(r)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gather_equals_single_rank(tmp_path, world):
    """One batch split per read over `world` gloo ranks, gathered to rank 0:
    byte-identical to the single-rank results and streams."""
    mp.spawn(_gather_main, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    import oracle as O
    from gsnapdp import gather as G
    from gsnapdp.records import RESULT
    g, batch = _batch()
    O.setup(g.blocks)
    res, pairs, poff, npairs = O.run_batch(batch.windows, batch.query, batch.query_uc, nthreads=4)
    rr, comp = _payload_of(res, pairs, poff, npairs)
    got_res = np.load(os.path.join(str(tmp_path), "res.npy"), allow_pickle=False)
    got_ops = np.load(os.path.join(str(tmp_path), "ops.npy"), allow_pickle=False)
    got_off = np.load(os.path.join(str(tmp_path), "off.npy"), allow_pickle=False)
    spans = json.load(open(os.path.join(str(tmp_path), "spans.json")))["spans"]
    assert spans[0][0] == 0 and spans[-1][1] == len(batch)
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert all(b - a > 0 for a, b in spans)
    assert got_res.dtype == RESULT and got_res.tobytes() == rr.tobytes()
    assert got_ops.tobytes() == comp.tobytes()
    assert np.array_equal(got_off, G.offsets_from_nops(rr))


def test_payload_round_trip_and_overflow():
    from gsnapdp import gather as G
    from gsnapdp.records import RESULT
    rng = np.random.default_rng(1)
    n = 300
    res = np.zeros(n, dtype=RESULT)
    cap = rng.integers(1, 12, size=n)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(cap, out=off[1:])
    res["nops"] = rng.integers(0, 12, size=n)
    res["nops"] = np.minimum(res["nops"], cap)
    res["finalscore"] = rng.integers(-100, 450, size=n)
    ops = rng.integers(0, 1 << 32, size=int(off[-1]), dtype=np.uint32)
    comp = G.compact_ops(res, ops, off)
    assert comp.size == int(res["nops"].sum())
    lay = G.Layout(n, comp.size)
    r2, o2, f2 = G.unpack(lay, G.pack(lay, res, comp), n)
    assert r2.tobytes() == res.tobytes() and o2.tobytes() == comp.tobytes()
    for i in range(n):
        assert np.array_equal(o2[f2[i]:f2[i + 1]], ops[off[i]:off[i] + res["nops"][i]])
    small = G.Layout(n, comp.size - 1)
    with pytest.raises(RuntimeError):
        G.unpack(small, G.pack(small, res, comp), n)


def test_balanced_ranges():
    w = np.array([1, 1, 1, 1, 10, 1, 1, 1], dtype=float)
    spans = shard.balanced_ranges(w, 2)
    assert spans[0][0] == 0 and spans[1][1] == 8 and spans[0][1] == spans[1][0]
    for n in (0, 1, 5, 1000):
        for world in (1, 2, 3, 8):
            spans = shard.balanced_ranges(np.ones(n), world)
            assert [i for a, b in spans for i in range(a, b)] == list(range(n))
            if n >= world:
                sz = [b - a for a, b in spans]
                assert max(sz) - min(sz) <= 1


def test_shard_range_covers_batch_exactly():
    for n in (0, 1, 7, 100, 101):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, world) for r in range(world)]
            covered = [i for lo, hi in spans for i in range(lo, hi)]
            assert covered == list(range(n))


def test_single_rank_needs_no_process_group(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    r = shard.init_from_env("gloo")
    assert (r.rank, r.world, r.dist) == (0, 1, None)
    assert shard.timed_steps(r, lambda: None, 3, lambda: None) >= 0.0
    assert shard.aggregate_rate(100, r, 2, 0.5) == 400.0


@pytest.mark.timeout(300)
def test_two_ranks_gloo(tmp_path):
    world = 2
    mp.spawn(_rank_main, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(os.path.join(str(tmp_path), "rank%d.json" % r))) for r in range(world)]
    # max-over-ranks timing: identical on every rank
    assert res[0]["elapsed"] == res[1]["elapsed"]
    assert max(res[0]["elapsed"]) == min(res[0]["elapsed"])
    # disjoint shards (different seeds), whole-job unit count and rate
    assert res[0]["firsts"][0] != res[0]["firsts"][1]
    assert res[0]["total"] == 600
    el = res[0]["elapsed"][0]
    assert abs(res[0]["rate"] - 600 * 2 / el) < 1e-6 * res[0]["rate"]
    assert res[0]["score_sum"] != res[1]["score_sum"]


def _bench_path_main(rank, world, port, outdir, cache):
    """bench.py's own N>1 path on CPU: the node-level C3 cache (every rank maps
    what local rank 0 wrote), bench.shard_slice, the payload layout with a
    deliberately short op budget grown by bench.payload_budget (all-reduced),
    the gather to rank 0 and gather.reassemble."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "gmap-gsnap_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import bench
    import oracle as O
    from gsnapdp import gather as G
    from gsnapdp import shard as S
    from gsnapdp import workload as W

    r = S.init_from_env("gloo")
    g, batch = W.c3_cached(1603, r.local, scale=0.002, cache_dir=cache)
    cells = bench.cells_per_window(batch.windows)
    wl, ql, sizes, lo, hi = bench.shard_slice(batch, cells, world, r.rank)
    O.setup(np.ascontiguousarray(g.blocks))
    res, pairs, poff, npairs = O.run_batch(wl, ql, ql, nthreads=1)  # the GPU step's stand-in
    rr, comp = _payload_of(res, pairs, poff, npairs)
    lay = G.Layout(max(sizes), 64)  # far too small: 6 words per pair
    mine = G.pack(lay, rr, comp)
    grow = bench.payload_budget(r, mine[:G.HEADER], lay)
    assert grow > 0
    lay = G.Layout(max(sizes), grow)
    mine = torch.from_numpy(G.pack(lay, rr, comp))
    recv = [torch.zeros(lay.nbytes, dtype=torch.uint8) for _ in range(world)] if r.rank == 0 else None
    S.gather_to_root(r, mine, recv)
    if r.rank == 0:
        allres, allops, alloff = G.reassemble(lay, [t.numpy() for t in recv], sizes)
        np.save(os.path.join(outdir, "res.npy"), allres)
        np.save(os.path.join(outdir, "ops.npy"), allops)
        json.dump({"sizes": sizes, "budget": lay.budget}, open(os.path.join(outdir, "meta.json"), "w"))
    S.finish(r)


@pytest.mark.timeout(600)
def test_bench_path_world8_equals_single_rank(tmp_path):
    """World 8 (the scaling target's width) through bench.py's functions: one
    batch, eight slices, one gather, byte-identical to one rank."""
    world = 8
    cache = str(tmp_path / "c3cache")
    mp.spawn(_bench_path_main, args=(world, free_port(), str(tmp_path), cache), nprocs=world, join=True)
    import oracle as O
    from gsnapdp import workload as W
    g, batch = W.c3_cached(1603, 0, scale=0.002, cache_dir=cache)
    O.setup(np.ascontiguousarray(g.blocks))
    res, pairs, poff, npairs = O.run_batch(batch.windows, batch.query, batch.query_uc, nthreads=4)
    rr, comp = _payload_of(res, pairs, poff, npairs)
    got_res = np.load(os.path.join(str(tmp_path), "res.npy"), allow_pickle=False)
    got_ops = np.load(os.path.join(str(tmp_path), "ops.npy"), allow_pickle=False)
    meta = json.load(open(os.path.join(str(tmp_path), "meta.json")))
    assert len(meta["sizes"]) == 8 and sum(meta["sizes"]) == len(batch) and min(meta["sizes"]) > 0
    assert got_res.tobytes() == rr.tobytes() and got_ops.tobytes() == comp.tobytes()
